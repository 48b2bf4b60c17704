"""BASELINE configs[3] / [4] on the GPU through the sharded runner (athd/dist.py) with a real RCCL process group
(backend "nccl", world size 1 on the lease's single GPU; the world-2 exchange logic is covered with gloo in
tests/test_dist_gloo.py), plus checkpoint ingestion (test_inference.py:21-40).

  * separate_segments (64 segments x 6 s x 4 prompts)        == forward_prompts of the same batch
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
