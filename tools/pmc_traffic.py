"""HBM traffic per kernel launch from two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on
gfx950: MI355X_MICROARCH.md §rocprofv3 PMC slots).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE (KiB) reports exactly
half the bytes of a wide coalesced streaming read (16 B per lane) on gfx950 and is uncalibrated for other widths.
So the x2 correction is applied only to the kernels whose HBM reads are 16-B-per-lane streams (WIDE_READS: the GEMM
and attention tile loads, the fused iSTFT's spectrum loads); for the others hbm_bytes_per_launch is the raw
(FETCH_SIZE + WRITE_SIZE) * 1024 and `fetch_correction` says 1 (uncalibrated width).  Both figures are recorded.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> --batch B --dtype bf16 [-o profiles/pmc_traffic.json]

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
    ap.add_argument("-o", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    fe = per_kernel(a.fetch_dir, "FETCH_SIZE")
    wr = per_kernel(a.write_dir, "WRITE_SIZE")
    out = {"batch": a.batch, "dtype": a.dtype,
           "correction": "hbm_bytes = (c * FETCH_SIZE + WRITE_SIZE) * 1024 per launch; c = 2 for 16-B/lane read "
                         "streams (gfx950 FETCH_SIZE halving, kernels " + ", ".join(WIDE_READS) + "), else 1",
           "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        nf, f = fe.get(k, [0, 0.0])
        nw, w = wr.get(k, [0, 0.0])
        fk = f / nf if nf else 0.0
        wk = w / nw if nw else 0.0
        c = 2 if k.startswith(WIDE_READS) else 1
        out["kernels"][k] = {"launches": max(nf, nw), "fetch_kib": fk, "write_kib": wk, "fetch_correction": c,
                             "hbm_bytes_raw": (fk + wk) * 1024, "hbm_bytes_per_launch": (c * fk + wk) * 1024}
    os.makedirs(os.path.dirname(a.o), exist_ok=True)
    json.dump(out, open(a.o, "w"), indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["launches"])[:15]:
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch x{v['launches']:>4}  {k}")


if __name__ == "__main__":
    main()
