"""Per-kernel SQ/GRBM counter summary from rocprofv3 --pmc passes (each pass its own output dir).

    python tools/pmc_sq.py <pass_dir> [<pass_dir> ...] [-o profiles/rNN_pmc_sq.json] [--top 25]

Counters are averaged per dispatch and keyed by the athd profile labels (tools/knames.py).  Derived columns
(MI355X_MICROARCH.md §rocprofv3 PMC slots and § Per-instruction cycle constants):
  wait     = SQ_WAIT_ANY / SQ_WAVE_CYCLES        waves parked on s_waitcnt / barrier
  stall    = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   issue stalls (dependency / pipe busy)
  active   = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (the three are disjoint and sum to ~1)
  valu     = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  mfma     = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs): the fraction of SIMD-cycles of the
             dispatch the MFMA pipes were busy (MFMA_BUSY counts cycles, GRBM_GUI_ACTIVE sums the 8 XCDs' cycles)
  lds_conf = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from knames import short_name  # noqa: E402

SIMDS = 256 * 4


def load(dirs):
    """{kernel: {counter: [sum, dispatches]}}"""
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: [0.0, set()]))
    for d in dirs:
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            raise SystemExit(f"no *counter_collection.csv under {d}")
        for f in files:
            for r in csv.DictReader(open(f)):
                k = short_name(r["Kernel_Name"])
                a = acc[k][r["Counter_Name"]]
                a[0] += float(r["Counter_Value"])
                a[1].add((d, f, r.get("Dispatch_Id", r.get("Correlation_Id"))))
    return {k: {c: v[0] / max(1, len(v[1])) for c, v in cs.items()} | {"dispatches": max(len(v[1]) for v in cs.values())}
            for k, cs in acc.items()}


def derive(c):
    out = {}
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for name, key in (("wait", "SQ_WAIT_ANY"), ("stall", "SQ_WAIT_INST_ANY"), ("active", "SQ_ACTIVE_INST_ANY"),
                          ("valu", "SQ_ACTIVE_INST_VALU")):
            if key in c:
                out[name] = c[key] / wc
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
        out["mfma"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * SIMDS)
    if c.get("SQ_ACTIVE_INST_LDS") and "SQ_LDS_BANK_CONFLICT" in c:
        out["lds_conf"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_ACTIVE_INST_LDS"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("-o", default=None)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    ks = load(a.dirs)
    res = {k: {"counters": c, "derived": derive(c)} for k, c in ks.items()}
    if a.o:
        os.makedirs(os.path.dirname(os.path.abspath(a.o)), exist_ok=True)
        json.dump(res, open(a.o, "w"), indent=1)
    order = sorted(res, key=lambda k: -res[k]["counters"].get("GRBM_GUI_ACTIVE", 0) * res[k]["counters"]["dispatches"])
    print(f"{'gui_active/8 (cyc)':>18} {'n':>4} {'wait':>6} {'stall':>6} {'active':>6} {'valu':>6} {'mfma':>6} "
          f"{'ldsconf':>7}  kernel")
    for k in order[:a.top]:
        c, d = res[k]["counters"], res[k]["derived"]
        f = lambda x: f"{d[x]:6.3f}" if x in d else f"{'-':>6}"  # noqa: E731
        print(f"{c.get('GRBM_GUI_ACTIVE', 0) / 8:18.0f} {c['dispatches']:4d} {f('wait')} {f('stall')} {f('active')} "
              f"{f('valu')} {f('mfma')} {d.get('lds_conf', float('nan')):7.3f}  {k}")


if __name__ == "__main__":
    main()
