"""BASELINE configs[3] / [4] on the GPU through the sharded runner (athd/dist.py) with a real RCCL process group
(backend "nccl", world size 1 on the lease's single GPU; the world-2 exchange logic is covered with gloo in
tests/test_dist_gloo.py), plus checkpoint ingestion (test_inference.py:21-40).

  * separate_segments (64 segments x 6 s x 4 prompts)        == forward_prompts of the same batch
  * configs[3] at one rank's size: 750 segments x 4 stems     == forward_prompts (sample) and >= 70 dB vs the
    (f32; also bf16 with the bench's decode chunk)               oracle (3 segments, f32)
  * separate_dataset on a 3-track MUSDB18-HQ directory       == OurModel.separate_all + evaluate_model per track
                                                                 (estimates, SDR / SI-SDR, evaluation_results.json)
  * separate_track_sharded, 300 s track x 4 stems            == separate_track (test_inference protocol) and
                                                                 == OurModel (benchmark protocol);
    a sample of its windows (first, middle, last)            >= 70 dB (f32) against the oracle forward
  * torch.save({"model_state_dict": ...}) -> load_model      -> forward >= 70 dB (f32) against the oracle
"Equal" is up to run-to-run noise: the GroupNorm statistics are fp64 atomics whose order varies between two runs
of the same batch, which can flip a last bit of an fp32 (f32 mode: >= 120 dB) or a bf16 rounding of an intermediate
(bf16 mode: >= 40 dB, as tests/test_gpu_parity.py::test_forward_prompts_matches_forward).  The span recombination
itself is bit-exact on fixed window outputs (tests/test_gpu_track.py, tests/test_dist_gloo.py).
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SEG = 264600


def _sdr(ref, out):
    ref = np.asarray(ref, np.float64)
    out = np.asarray(out, np.float64)
    return float(10 * np.log10(np.sum(ref ** 2) / max(np.sum((ref - out) ** 2), 1e-300)))


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def model_f32(state_dict, text_table):
    from athd.model import AudioTextHTDemucs
    from athd.weights import STEMS
    m = AudioTextHTDemucs(dtype="f32", text_table={s: text_table[i] for i, s in enumerate(STEMS)})
    m.load_state_dict(state_dict)
    return m.to("cuda").eval()


def test_separate_segments_nccl_equals_forward_prompts(pg, state_dict, text_table):
    from athd.dist import separate_segments
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_batch
    from athd.weights import STEMS
    m = AudioTextHTDemucs(dtype="bf16", text_table={s: text_table[i] for i, s in enumerate(STEMS)},
                          decode_items=256)
    m.load_state_dict(state_dict)
    m = m.to("cuda").eval()
    segs = torch.as_tensor(synthetic_batch(64, SEG, seed0=2024))            # host tensor, read block by block
    got = separate_segments(m, segs, STEMS, max_batch=32)
    ref = m.forward_prompts(segs.cuda(), STEMS)
    assert got.shape == (64, 4, 2, SEG)
    worst = min(_sdr(ref[i, p].cpu().numpy(), got[i, p].cpu().numpy()) for i in (0, 31, 32, 63) for p in range(4))
    assert worst >= 40.0, worst
    del got, ref
    torch.cuda.empty_cache()


def _distinct_segments(n, seed0=7000, n_base=12, gain=1.0):
    """n distinct 6 s segments on the device, cheaply: segment i is synthetic base (i % n_base) rolled by a per-i
    offset and scaled by a per-i gain (synthesising 750 tone mixtures on the host would take minutes)."""
    from athd.synth import synthetic_batch
    base = torch.as_tensor(synthetic_batch(n_base, SEG, seed0=seed0)).cuda()
    out = torch.empty((n, 2, SEG), dtype=torch.float32, device="cuda")
    for i in range(n):
        out[i] = torch.roll(base[i % n_base], shifts=(i * 7919) % SEG, dims=-1) * (gain * (0.5 + (i % 17) / 16.0))
    return out


def test_config3_per_rank_750_segments(pg, model_f32, oracle_model, text_table):
    """BASELINE configs[3] at one rank's size: ~6k MUSDB18 test-set segments over 8 GPUs = 750 per rank.  750
    distinct segments x 4 stems through separate_segments with the rank's block already resident (n_total) and a
    preallocated (750, 4, 2, T) output, as each rank of the 8-GPU job runs it; batches of 64 (the last 46).  Checked:
    a sample of rows against forward_prompts of the same segments (>= 120 dB, f32 run-to-run noise only) and 3
    segments against the oracle forward (>= 70 dB, gated away from the mask singularity like the 300 s test)."""
    from athd.dist import separate_segments
    from athd.weights import STEMS
    from test_gpu_parity import PHASE_COND_MIN, _phase_cond, _report
    n = 750
    # x100 level: keeps the spectra away from the reference mask's absolute singular point (see the 300 s test)
    segs = _distinct_segments(n, gain=100.0)
    out = torch.empty((n, 4, 2, SEG), dtype=torch.float32, device="cuda")
    got = separate_segments(model_f32, segs, STEMS, max_batch=64, n_total=n, out=out)
    assert got is out
    for rows in ([0, 63], [64, 400], [703, 749]):
        ref = model_f32.forward_prompts(segs[rows].contiguous(), STEMS)
        for j, i in enumerate(rows):
            for p in range(4):
                assert _sdr(ref[j, p].cpu().numpy(), got[i, p].cpu().numpy()) >= 120.0, (i, p)
    res, cond = {}, {}
    for i in (5, 377, 748, 100, 611, 250, 42):
        if sum(1 for c in cond.values() if c >= PHASE_COND_MIN) >= 3:
            break
        seg = segs[i:i + 1].cpu()
        cond[i] = _phase_cond(oracle_model.prepare(seg)[0])
        if cond[i] < PHASE_COND_MIN:
            continue
        o = oracle_model.forward_prompts(seg, torch.as_tensor(text_table))[0]
        res[i] = min(_sdr(o[p].numpy(), got[i, p].cpu().numpy()) for p in range(4))
    _report("config3_750_segments_f32", {str(i): {"sdr_db_min_over_stems": res.get(i), "phase_cond": cond[i]}
                                         for i in cond})
    assert len(res) >= 3, cond
    assert min(res.values()) >= 70.0, (res, cond)
    del out, got, segs
    torch.cuda.empty_cache()


def test_config3_750_segments_bf16(pg, state_dict, text_table):
    """The same 750-segment per-rank pass in the bench dtype with the bench's decode chunk (256 items): a sample
    equals forward_prompts of the same segments (>= 40 dB: bf16 run-to-run noise of the fp64-atomic statistics)."""
    from athd.dist import separate_segments
    from athd.model import AudioTextHTDemucs
    from athd.weights import STEMS
    m = AudioTextHTDemucs(dtype="bf16", text_table={s: text_table[i] for i, s in enumerate(STEMS)},
                          decode_items=256)
    m.load_state_dict(state_dict)
    m = m.to("cuda").eval()
    n = 750
    segs = _distinct_segments(n, seed0=7100)
    got = separate_segments(m, segs, STEMS, max_batch=64, n_total=n)
    assert got.shape == (n, 4, 2, SEG) and bool(torch.isfinite(got).all())
    rows = [0, 64, 500, 749]
    ref = m.forward_prompts(segs[rows].contiguous(), STEMS)
    worst = min(_sdr(ref[j, p].cpu().numpy(), got[i, p].cpu().numpy()) for j, i in enumerate(rows) for p in range(4))
    assert worst >= 40.0, worst
    del got, segs, m
    torch.cuda.empty_cache()


def test_separate_dataset_musdb_hq_split(pg, model_f32, tmp_path):
    """§8(f)3 end to end: a 3-track MUSDB18-HQ split directory -> MusDBTracks -> separate_dataset (every window of
    every track one unit of separate_segments, tracks reassembled from the gathered rows, SDR / SI-SDR,
    evaluation_results.json) == the reference's per-track loop, OurModel.separate_all + evaluate_model
    (benchmark.py:742-781).  Same estimates (f32 run-to-run noise only, >= 120 dB) and the same metrics (1e-3 dB)."""
    import json
    from athd.benchmark import OurModel, evaluate_model
    from athd.dist import separate_dataset
    from athd.musdb import HQ_FILES, MusDBTracks, write_wav
    from athd.synth import synthetic_mixture
    from athd.weights import STEMS
    lengths = [44100 * 20 + 1234, 44100 * 9, 264600]
    for t, L in enumerate(lengths):
        d = tmp_path / "test" / f"Artist {t} - Song"
        d.mkdir(parents=True)
        parts = [synthetic_mixture(L, seed=900 + 10 * t + j) for j in range(4)]
        for f, x in zip(HQ_FILES, [sum(parts)] + parts):
            write_wav(d / f"{f}.wav", x, 44100, "FLOAT")
    tracks = MusDBTracks(tmp_path / "test")
    results, est = separate_dataset(model_f32, tracks, STEMS, max_batch=4, output_dir=tmp_path / "out",
                                    keep_estimates=True, log=None)
    ref = evaluate_model(OurModel(model_f32), tracks.tracks(), log=None)
    assert [r.track_name for r in results] == [r.track_name for r in ref]
    for r, q in zip(results, ref):
        for f in ("sdr", "sisdr"):
            for s in STEMS + ["avg"]:
                assert abs(getattr(r, f"{f}_{s}") - getattr(q, f"{f}_{s}")) < 1e-3, (r.track_name, f, s)
    for i in range(len(tracks)):
        name, mix, _ = tracks.track(i)
        want = OurModel(model_f32).separate_stems(mix.cuda(), STEMS)
        assert est[name].shape == (4, 2, lengths[i])
        assert min(_sdr(want[s].cpu().numpy(), est[name][s].cpu().numpy()) for s in range(4)) >= 120.0
    saved = json.load(open(tmp_path / "out" / "evaluation_results.json"))
    body = saved["AudioTextHTDemucs (Ours)"]
    assert [p["track"] for p in body["per_track"]] == [r.track_name for r in results]
    assert abs(body["aggregate"]["sdr"]["average"] - np.mean([r.sdr_avg for r in results])) < 1e-12


def test_separate_track_sharded_300s(pg, model_f32, oracle_model, text_table):
    """300 s x 4 stems (BASELINE configs[4]): 51 windows per stem, the last one 220500 samples."""
    from athd.dist import separate_track_sharded
    from athd.inference import run_windows, separate_track, window_plan
    from athd.synth import synthetic_mixture
    from athd.weights import STEMS
    L = 300 * 44100
    # x100 amplitude: the reference mask's singular point (Re z_L = -1e-8, _phase_cond) is absolute, so a louder track
    # keeps the ~1M spectrum values of each 6 s window away from it (at RMS 0.1 nearly every window has a bin within
    # 5e-8 of it, where fp32 parity is not defined); the encoder normalises the level away
    mix = (torch.as_tensor(synthetic_mixture(L, seed=300)) * 100.0).cuda()
    plan = window_plan(L)
    assert len(plan) == 51 and plan[-1].end - plan[-1].start == 220500
    got = separate_track_sharded(model_f32, mix, STEMS)
    ref = separate_track(model_f32, mix, STEMS)
    assert got.shape == (4, 2, L)
    assert torch.equal(got, ref) or _sdr(ref.cpu().numpy(), got.cpu().numpy()) >= 120.0
    # sample windows against the oracle forward (encode once, decode 4x on the CPU).  Windows whose spectrum has a
    # bin near the reference mask's singularity (Re z_L ~ -1e-8, tests/test_gpu_parity.py::_phase_cond) are
    # reported but not gated: there the output depends on the last bits of that STFT bin.
    from test_gpu_parity import PHASE_COND_MIN, _phase_cond, _report
    res, cond = {}, {}
    for k in [0, 25, 50, 12, 37, 49, 1]:
        if sum(1 for kk in cond if cond[kk] >= PHASE_COND_MIN) >= 3:
            break
        w = plan[k]
        seg = mix[:, w.start:w.end].cpu()[None]
        cond[k] = _phase_cond(oracle_model.prepare(seg)[0])
        win = run_windows(model_f32, mix, plan, STEMS, SEG, k, k + 1).cpu()[0]     # (4, 2, SEG)
        o = oracle_model.forward_prompts(seg, torch.as_tensor(text_table))[0]
        res[k] = min(_sdr(o[si].numpy(), win[si, :, :w.end - w.start].numpy()) for si in range(4))
    _report("track300s_windows_f32", {str(k): {"sdr_db_min_over_stems": res[k], "phase_cond": cond[k]} for k in res})
    gated = [k for k in res if cond[k] >= PHASE_COND_MIN]
    assert len(gated) >= 3, cond
    assert min(res[k] for k in gated) >= 70.0, (res, cond)
    del got, ref
    torch.cuda.empty_cache()


def test_separate_track_sharded_benchmark_protocol(pg, model_f32):
    from athd.benchmark import OurModel
    from athd.dist import separate_track_sharded
    from athd.synth import synthetic_mixture
    from athd.weights import STEMS
    L = 61 * 44100 + 777
    mix = torch.as_tensor(synthetic_mixture(L, seed=61)).cuda()
    got = separate_track_sharded(model_f32, mix, STEMS, overlap=1.5, protocol="benchmark")
    ref = OurModel(model_f32).separate_stems(mix, STEMS)
    assert got.shape == ref.shape
    assert torch.equal(got, ref) or _sdr(ref.cpu().numpy(), got.cpu().numpy()) >= 120.0


def test_checkpoint_load_model_forward(tmp_path, state_dict, text_table, oracle_model):
    """test_inference.py:21-40: a {"model_state_dict", "epoch", ...} checkpoint (src/train.py:218-224) with keys the
    hot path does not use (clap.*, htdemucs.decoder.*) read by load_model (torch.load weights_only=True)."""
    from athd.inference import load_model
    from athd.synth import synthetic_batch
    from athd.weights import STEMS
    sd = {k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}
    sd["clap.text_model.embeddings.word_embeddings.weight"] = torch.zeros(8, 4)
    sd["htdemucs.decoder.0.conv_tr.weight"] = torch.zeros(4, 4, 8, 1)
    path = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": sd, "epoch": 7, "optimizer_state_dict": {}, "val_loss": -4.2}, path)
    table = {s: text_table[i] for i, s in enumerate(STEMS)}
    m = load_model(str(path), "cuda", dtype="f32", text_table=table)
    wav = torch.as_tensor(synthetic_batch(1, 44100 * 2, seed0=321))
    out = m(wav.cuda(), "drums").cpu().numpy()
    ref = oracle_model.forward(wav, torch.as_tensor(text_table[0:1])).numpy()
    assert _sdr(ref, out) >= 70.0, _sdr(ref, out)
