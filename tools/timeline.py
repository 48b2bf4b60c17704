"""Concurrency of the two HIP streams in a rocprofv3 --kernel-trace run of bench.py (production mode, both streams).

    python tools/timeline.py <kernel_trace_dir> [--last-steps K]

Takes the last K forwards (a forward = the span from a stft_kernel start to the next stft_kernel start) and reports
per step: wall time, time with >= 1 kernel running, time with >= 2 kernels running (the two branches overlapping),
and the idle gaps (no kernel running), plus the kernels that run alone longest (the critical path candidates)."""
import argparse
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from knames import short_name  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--last-steps", type=int, default=2)
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short_name(r["Kernel_Name"]))
            for r in csv.DictReader(open(f))]
    rows.sort()
    starts = [s for s, _, k in rows if k.startswith("stft_kernel")]
    if len(starts) < a.last_steps + 1:
        raise SystemExit("not enough forwards in the trace")
    t0, t1 = starts[-a.last_steps - 1], starts[-1]
    ev = [(s, e, k) for s, e, k in rows if t0 <= s < t1]
    # sweep
    pts = sorted([(s, 1, k) for s, e, k in ev] + [(e, -1, k) for s, e, k in ev])
    active = collections.Counter()
    n = 0
    last = t0
    busy1 = busy2 = 0
    alone = collections.Counter()
    for t, d, k in pts:
        dt = t - last
        if n >= 1:
            busy1 += dt
        if n >= 2:
            busy2 += dt
        if n == 1:
            (only,) = [x for x, c in active.items() if c > 0]
            alone[only] += dt
        n += d
        active[k] += d
        last = t
    wall = t1 - t0
    steps = a.last_steps
    print(f"per forward: wall {wall / steps / 1e6:.3f} ms, >=1 kernel {busy1 / steps / 1e6:.3f} ms, "
          f">=2 kernels {busy2 / steps / 1e6:.3f} ms, idle {(wall - busy1) / steps / 1e6:.3f} ms")
    print("kernels running alone longest (ms per forward):")
    for k, v in alone.most_common(15):
        print(f"  {v / steps / 1e6:8.3f}  {k}")


if __name__ == "__main__":
    main()
