"""Compare two per-call-site kernel time dumps (bench.py --dump-kernels X.json -> X_sites.json).

    python tools/sites_diff.py OLD_sites.json NEW_sites.json [-n 20]
"""
import argparse
import json


def load(p):
    return {r["kernel"]: r["ms"] for r in json.load(open(p))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("old")
    ap.add_argument("new")
    ap.add_argument("-n", type=int, default=20)
    a = ap.parse_args()
    fa, fb = load(a.old), load(a.new)
    print(f"total {sum(fa.values()):.3f} -> {sum(fb.values()):.3f} ms")
    keys = sorted(set(fa) | set(fb), key=lambda k: -abs(fb.get(k, 0) - fa.get(k, 0)))
    for k in keys[:a.n]:
        print(f"{k:72s} {fa.get(k, 0):8.3f} {fb.get(k, 0):8.3f}")


if __name__ == "__main__":
    main()
