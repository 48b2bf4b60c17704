"""Per-call-site kernel times of two bench.py --dump-kernels runs (the warm-up forward, every launch evented, branches
serialised): python tools/sites_diff.py A_sites.json B_sites.json [--top N]"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--top", type=int, default=20)
    x = ap.parse_args()
    A = {r["kernel"]: r["ms"] for r in json.load(open(x.a))}
    B = {r["kernel"]: r["ms"] for r in json.load(open(x.b))}
    keys = set(A) | set(B)
    print(f"total: {sum(A.values()):.3f} ms -> {sum(B.values()):.3f} ms")
    rows = sorted(keys, key=lambda k: -abs(B.get(k, 0.0) - A.get(k, 0.0)))
    for k in rows[:x.top]:
        a, b = A.get(k, 0.0), B.get(k, 0.0)
        print(f"{a:8.3f} {b:8.3f} {b - a:+8.3f}  {k}")


if __name__ == "__main__":
    main()
