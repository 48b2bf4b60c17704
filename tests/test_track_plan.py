"""Window plan of the test_inference.py:92-141 loop: host mirror (athd/inference.py) vs the oracle restatement and
the library's analytic window count (CPU only; no kernel launches)."""
import numpy as np
import pytest

from oracle.athtdemucs_ref import chunk_plan


def _plan(L, **kw):
    from athd.inference import window_plan
    return [(w.start, w.end, w.fade_in, w.fade_out) for w in window_plan(L, **kw)]


@pytest.mark.parametrize("L", [1, 4410, 44100, 260190, 264600, 264600 + 4410, 260190 + 264600, 44100 * 300,
                               2 * 260190 + 264600, 44100 * 60 + 17])
def test_plan_matches_oracle(L):
    assert _plan(L) == chunk_plan(L)


def test_plan_random_lengths():
    rng = np.random.default_rng(0)
    n = 0
    for L in rng.integers(1, 44100 * 400, 300):
        L = int(L)
        ref = chunk_plan(L)
        if any(e - s < max(fi, fo) for s, e, fi, fo in ref):
            with pytest.raises(RuntimeError):
                _plan(L)
        else:
            assert _plan(L) == ref
            n += 1
    assert n > 250


def test_plan_short_tail_raises_like_reference():
    # second window [260190, 264599) has 4409 samples < its 4410-sample fade-in: torchaudio's Fade fails in the
    # reference loop (any length with 0 < (L - k*hop) < overlap for the last window)
    L = 264599
    ref = chunk_plan(L)
    assert ref[-1][1] - ref[-1][0] < ref[-1][2]
    with pytest.raises(RuntimeError):
        _plan(L)


def test_plan_other_rates():
    for sr, seg, ov in [(16000, 4.0, 0.25), (44100, 7.8, 0.1), (22050, 6.0, 0.0)]:
        for L in (1000, sr * 10, sr * 33 + 5):
            ref = chunk_plan(L, sr, seg, ov)
            if any(e - s < max(fi, fo) for s, e, fi, fo in ref):
                continue
            assert _plan(L, sample_rate=sr, segment_seconds=seg, overlap=ov) == ref
