"""MUSDB18 track loading and the dataset segment index (athd/musdb.py) against `src/dataloader.py` semantics.
MUSDB18 itself is not available offline: the tracks here are synthetic, written in the decoded forms the loader
reads (MUSDB18-HQ wav directories and (5, T, 2) .stem.npy arrays)."""
import math

import numpy as np
import pytest

from athd import musdb


def test_prompt_tables_match_reference():
    # dataloader.py:21-34
    assert musdb.STEM_PROMPTS["other"] == ["other instruments", "accompaniment", "instruments"]
    assert musdb.PROMPT_TO_STEM["bass line"] == "bass" and musdb.PROMPT_TO_STEM["voice"] == "vocals"
    assert musdb.STEM_NAME_TO_INDEX == {"drums": 0, "bass": 1, "other": 2, "vocals": 3}


def test_segment_index_matches_reference_rule():
    S = 264600
    lengths = [S, S + 1, 3 * S - 7, 1]
    idx = musdb.segment_index(lengths, S)
    assert len(idx) == 4 * sum(math.ceil(n / S) for n in lengths)
    assert idx[:4] == [(0, 0, 0), (0, 1, 0), (0, 2, 0), (0, 3, 0)]
    assert idx[4:8] == [(1, 0, 0), (1, 0, 1), (1, 1, 0), (1, 1, 1)]
    assert idx[-1] == (3, 3, 0)


def test_extract_segment_zero_pads_the_last():
    st = np.arange(5 * 10 * 2, dtype=np.float32).reshape(5, 10, 2)
    a = musdb.extract_segment(st, 0, 4)
    assert np.array_equal(a, st[:, :4])
    c = musdb.extract_segment(st, 2, 4)
    assert c.shape == (5, 4, 2) and np.array_equal(c[:, :2], st[:, 8:]) and not c[:, 2:].any()


@pytest.mark.parametrize("subtype", ["PCM_16", "FLOAT"])
def test_wav_roundtrip(tmp_path, subtype):
    x = np.random.default_rng(0).uniform(-0.9, 0.9, size=(1234, 2)).astype(np.float32)
    musdb.write_wav(tmp_path / "a.wav", x, 44100, subtype)
    y, rate = musdb.read_wav(tmp_path / "a.wav")
    assert rate == 44100 and y.shape == x.shape
    assert np.abs(y - x).max() <= (1 / 16384 if subtype == "PCM_16" else 0.0)     # x 32767 in, / 32768 out


def test_tracks_from_hq_dirs_and_npy(tmp_path):
    rng = np.random.default_rng(1)
    lens = {"Artist - A": 50000, "Artist - B": 30001}
    for name, n in lens.items():
        d = tmp_path / name
        d.mkdir()
        for f in musdb.HQ_FILES:
            musdb.write_wav(d / f"{f}.wav", rng.uniform(-0.5, 0.5, size=(n, 2)), 44100, "FLOAT")
    npy = rng.uniform(-0.5, 0.5, size=(5, 20000, 2)).astype(np.float32)
    np.save(tmp_path / "Artist - C.stem.npy", npy)
    tr = musdb.MusDBTracks(tmp_path)
    assert len(tr) == 3 and [tr.name(i) for i in range(3)] == ["Artist - A", "Artist - B", "Artist - C"]
    name, mix, refs = tr.track(2)
    assert name == "Artist - C" and mix.shape == (2, 20000)
    assert np.array_equal(mix.numpy(), npy[0].T) and np.array_equal(refs["vocals"].numpy(), npy[4].T)
    segs, keys = tr.mixture_segments(16000)
    assert keys == [(0, 0), (0, 1), (0, 2), (0, 3), (1, 0), (1, 1), (2, 0), (2, 1)]
    assert segs.shape == (8, 2, 16000)
    assert np.array_equal(segs[7, :, :4000].numpy(), npy[0, 16000:].T) and not segs[7, :, 4000:].any()


def test_empty_dir_raises(tmp_path):
    with pytest.raises(ValueError):
        musdb.MusDBTracks(tmp_path)
