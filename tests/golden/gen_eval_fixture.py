"""Extract the reference's published evaluation results into a small numpy fixture (data only).

Source: /root/reference/eval_results/results_{full,v2,v3}/evaluation_results.json, written by the reference's
`save_results` (benchmark.py:853-888) from `TrackResult`s (:618-634) and `aggregate_results` (:784-804).  Per run:
  <run>_tracks     (n,)   track names in file order
  <run>_sdr        (n, 5) per-track SDR   [drums, bass, other, vocals, average]
  <run>_sisdr      (n, 5) per-track SI-SDR, same columns
  <run>_agg_sdr    (5,)   the file's aggregate SDR, same columns
  <run>_agg_sisdr  (5,)   the file's aggregate SI-SDR
  model_name       ()     the single model key of every file
Run here (the reference is not on the GPU box):  python tests/golden/gen_eval_fixture.py
"""
import json
import os

import numpy as np

SRC = "/root/reference/eval_results"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "eval_results.npz")
COLS = ["drums", "bass", "other", "vocals", "average"]


def main():
    arrs = {}
    names = set()
    for run in ("full", "v2", "v3"):
        d = json.load(open(os.path.join(SRC, f"results_{run}", "evaluation_results.json")))
        (model, body), = d.items()
        names.add(model)
        pt = body["per_track"]
        arrs[f"{run}_tracks"] = np.array([p["track"] for p in pt])
        for m in ("sdr", "sisdr"):
            arrs[f"{run}_{m}"] = np.array([[p[m][c] for c in COLS] for p in pt], dtype=np.float64)
            arrs[f"{run}_agg_{m}"] = np.array([body["aggregate"][m][c] for c in COLS], dtype=np.float64)
    assert len(names) == 1, names
    arrs["model_name"] = np.array(names.pop())
    np.savez_compressed(OUT, **arrs)
    print("wrote", OUT, {k: v.shape for k, v in arrs.items()})


if __name__ == "__main__":
    main()
