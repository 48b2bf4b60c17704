"""The benchmark.py result bookkeeping pinned by the reference's own published results (CPU).

`tests/golden/eval_results.npz` holds the per-track and aggregate SDR / SI-SDR of the reference's three published
runs (eval_results/results_{full,v2,v3}/evaluation_results.json, 50 MUSDB18 test tracks each; extracted by
tests/golden/gen_eval_fixture.py).  Those files were written by the reference's `save_results` from
`aggregate_results` (benchmark.py:784-888) over `TrackResult`s whose averages are `sum(scores) / len(scores)`
(:673-674).  Rebuilding the TrackResults from the per-track rows, the build's `athd.benchmark` must reproduce:
  * every per-track average (track_result, the averaging of evaluate_model_on_track) to 1e-12;
  * every aggregate (aggregate_results) to 1e-12;
  * the JSON layout and values of save_results, read back.
"""
import json

import numpy as np
import pytest

from conftest import GOLDEN

RUNS = ("full", "v2", "v3")
COLS = ["drums", "bass", "other", "vocals", "average"]


@pytest.fixture(scope="module")
def fixture():
    return dict(np.load(GOLDEN + "/eval_results.npz"))


def _results(fx, run):
    from athd.benchmark import TrackResult
    name = str(fx["model_name"])
    out = []
    for t, s, si in zip(fx[f"{run}_tracks"], fx[f"{run}_sdr"], fx[f"{run}_sisdr"]):
        out.append(TrackResult(str(t), name, *map(float, s[:4]), float(s[4]), *map(float, si[:4]), float(si[4])))
    return out


@pytest.mark.parametrize("run", RUNS)
def test_track_averages_match_published(fixture, run):
    """track_result (the per-stem metrics -> TrackResult step of evaluate_model_on_track / separate_dataset) fed the
    published per-stem scores gives the published per-track averages."""
    import torch
    from athd.benchmark import track_result
    from athd.weights import STEMS
    for t, s, si in zip(fixture[f"{run}_tracks"], fixture[f"{run}_sdr"], fixture[f"{run}_sisdr"]):
        scores = {stem: (float(s[j]), float(si[j])) for j, stem in enumerate(STEMS)}
        est = {stem: torch.full((2, 4), float(j)) for j, stem in enumerate(STEMS)}
        lookup = {float(j): scores[stem] for j, stem in enumerate(STEMS)}
        r = track_result(str(t), "m", est, {stem: torch.zeros(2, 4) for stem in STEMS},
                         metric_fn=lambda e, ref: lookup[float(e[0, 0])])
        assert abs(r.sdr_avg - s[4]) <= 1e-12 and abs(r.sisdr_avg - si[4]) <= 1e-12, (run, str(t))


@pytest.mark.parametrize("run", RUNS)
def test_aggregate_results_match_published(fixture, run):
    from athd.benchmark import aggregate_results
    agg = aggregate_results(_results(fixture, run))
    for m in ("sdr", "sisdr"):
        want = fixture[f"{run}_agg_{m}"]
        for j, c in enumerate(COLS):
            assert abs(agg[m][c] - want[j]) <= 1e-12, (run, m, c, agg[m][c], want[j])


@pytest.mark.parametrize("run", RUNS)
def test_save_results_layout(fixture, run, tmp_path):
    from athd.benchmark import save_results
    res = _results(fixture, run)
    name = str(fixture["model_name"])
    path = save_results({name: res}, tmp_path)
    assert path.name == "evaluation_results.json"
    d = json.load(open(path))
    assert list(d) == [name] and list(d[name]) == ["per_track", "aggregate"]
    pt = d[name]["per_track"]
    assert [p["track"] for p in pt] == [str(t) for t in fixture[f"{run}_tracks"]]
    for p, s, si in zip(pt, fixture[f"{run}_sdr"], fixture[f"{run}_sisdr"]):
        assert list(p) == ["track", "sdr", "sisdr"] and list(p["sdr"]) == COLS and list(p["sisdr"]) == COLS
        assert [p["sdr"][c] for c in COLS] == list(s) and [p["sisdr"][c] for c in COLS] == list(si)
    agg = d[name]["aggregate"]
    assert list(agg) == ["sdr", "sisdr"] and list(agg["sdr"]) == COLS
    for m in ("sdr", "sisdr"):
        assert np.abs(np.array([agg[m][c] for c in COLS]) - fixture[f"{run}_agg_{m}"]).max() <= 1e-12
