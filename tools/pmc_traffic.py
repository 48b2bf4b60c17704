"""HBM traffic per kernel launch from two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on
gfx950: MI355X_MICROARCH.md §rocprofv3 PMC slots).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE (KiB) reports exactly
half the bytes of a wide coalesced streaming read (16 B per lane) on gfx950 and is uncalibrated for other widths.

Width correction.  With --calib (profiles/pmc_calib.json: the counter's factor per bytes-per-lane, measured by
tools/pmc_calib.hip on a known byte count) and --widths (profiles/load_widths.json: each kernel's static share of
load bytes per width, tools/load_widths.py), a kernel's fetch correction is sum_w share_w / factor_w, i.e. every
width class of its loads divided by that width's measured factor (a kernel whose loads are all 16 B/lane gets
1 / 0.5 = 2).  Without them, the round-2 rule: x2 for the kernels in WIDE_READS, else 1.  Raw and corrected bytes
are both recorded.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> --batch B --dtype bf16 [--calib C] [--widths W]
                                [--kernels bench_kernels.json] [-o profiles/pmc_traffic.json]
--kernels (bench.py --dump-kernels output): also record each kernel's algorithmic bytes per launch and the ratio
corrected / algorithmic (below ~0.95 flags an accounting problem: cold reads cannot undercut the algorithmic bytes).

Writes {"batch", "dtype", "correction", "kernels": {label: {"launches", "fetch_kib", "write_kib",
"hbm_bytes_per_launch"}}} keyed by the athd profile labels bench.py uses (tools/knames.py)."""
import argparse
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from knames import short_name  # noqa: E402


WIDE_READS = ("gemm", "attn", "istft_ola")


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {d}")
    acc = collections.defaultdict(lambda: [0, 0.0])
    seen = set()
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            key = (f, r.get("Dispatch_Id", r.get("Correlation_Id")))
            if key in seen:
                acc[short_name(r["Kernel_Name"])][1] += float(r["Counter_Value"])
                continue
            seen.add(key)
            a = acc[short_name(r["Kernel_Name"])]
            a[0] += 1
            a[1] += float(r["Counter_Value"])
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--dtype", required=True)
    ap.add_argument("--calib", default=None)
    ap.add_argument("--widths", default=None)
    ap.add_argument("--kernels", default=None)
    ap.add_argument("-o", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fe = per_kernel(a.fetch_dir, "FETCH_SIZE")
    wr = per_kernel(a.write_dir, "WRITE_SIZE")
    calib = json.load(open(a.calib)) if a.calib else None
    widths = json.load(open(a.widths))["kernels"] if a.widths else None
    algo = {}
    if a.kernels:
        for r in json.load(open(a.kernels)):
            if r.get("launches"):
                algo[r["kernel"]] = r["bytes"] / r["launches"]
    if calib and widths:
        rule = ("hbm_bytes = (c * FETCH_SIZE + WRITE_SIZE / w16) * 1024 per launch, c = sum_w share_w / fetch_factor_w "
                "(load-width shares: " + a.widths + "; factors measured by tools/pmc_calib.hip: " + a.calib + ")")
    elif calib:
        rule = ("hbm_bytes = (c * FETCH_SIZE + WRITE_SIZE / w16) * 1024 per launch, c = 1 / the FETCH_SIZE factor "
                "measured by tools/pmc_calib.hip (" + a.calib + "), the same at every access width")
    else:
        rule = ("hbm_bytes = (c * FETCH_SIZE + WRITE_SIZE) * 1024 per launch; c = 2 for 16-B/lane read streams "
                "(gfx950 FETCH_SIZE halving, kernels " + ", ".join(WIDE_READS) + "), else 1")
    out = {"batch": a.batch, "dtype": a.dtype, "correction": rule, "calibration": calib and
           {"fetch": calib["fetch"], "write": calib["write"]}, "kernels": {}}

    uniform = calib and len(set(calib["fetch"].values())) == 1

    def fetch_corr(k):
        if calib and widths:
            base = k if k in widths else k.split("<", 1)[0]
            wk = widths.get(base) or next((v for n, v in widths.items() if n.split("<", 1)[0] == base), None)
            if wk:
                return sum(sh / calib["fetch"].get(w, 1.0) for w, sh in wk["byte_share"].items()), "calibrated"
        if uniform:        # the measured factor is the same at every width: no per-kernel width mix needed
            return 1.0 / next(iter(calib["fetch"].values())), "calibrated (same factor at 2/4/8/16 B per lane)"
        return (2 if k.startswith(WIDE_READS) else 1), "round-2 rule"
    wf = calib["write"].get("16", 1.0) if calib else 1.0
    for k in sorted(set(fe) | set(wr)):
        nf, f = fe.get(k, [0, 0.0])
        nw, w = wr.get(k, [0, 0.0])
        fk = f / nf if nf else 0.0
        wk = w / nw if nw else 0.0
        c, how = fetch_corr(k)
        rec = {"launches": max(nf, nw), "fetch_kib": fk, "write_kib": wk, "fetch_correction": round(c, 4),
               "correction_basis": how, "hbm_bytes_raw": (fk + wk) * 1024,
               "hbm_bytes_per_launch": (c * fk + wk / wf) * 1024}
        if k in algo or k.split("<", 1)[0] in algo:
            ab = algo.get(k, algo.get(k.split("<", 1)[0]))
            rec["algorithmic_bytes_per_launch"] = ab
            rec["traffic_over_algorithmic"] = round(rec["hbm_bytes_per_launch"] / ab, 3) if ab else None
        out["kernels"][k] = rec
    os.makedirs(os.path.dirname(a.o), exist_ok=True)
    json.dump(out, open(a.o, "w"), indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"])[:15]:
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch x{v['launches']:>4}  {k}")


if __name__ == "__main__":
    main()
