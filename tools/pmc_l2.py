"""Per-kernel L2 hit rate from a rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum pass (tools/gpu_l2.sh).

    python tools/pmc_l2.py <pass_dir> [--top 30]

hit = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum) (MI355X_MICROARCH.md §L2); requests are 128-B L2 accesses summed
over the 8 XCDs, averaged per dispatch."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_sq import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    d = load(a.dirs)
    rows = []
    for k, c in d.items():
        h, m = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        if h + m <= 0:
            continue
        rows.append((h + m, k, h / (h + m), c["dispatches"]))
    rows.sort(reverse=True)
    print("%12s %6s %5s  %s" % ("L2 req/disp", "hit", "n", "kernel"))
    for req, k, hit, n in rows[:a.top]:
        print("%12.0f %6.3f %5d  %s" % (req, hit, n, k))


if __name__ == "__main__":
    main()
