"""Parity of the HIP path (through the C-ABI) against the oracle and the reference's golden fixtures.

Tolerances (stated per north_star's "stated fp32 tolerance (SDR delta reported)"), each within ~10-15 dB of the
value measured on MI355X (profiles/r02_parity_report.json), so that a regression of that size fails:
  * f32 mode (exact-f32 MFMA everywhere): max|err| <= F32_MAXREL * RMS(ref) (1e-4) and SDR >= 110 dB
    wherever the input's spectrum keeps away from the reference mask's singularity (_phase_cond); on the reference
    fixtures, whose spectra do not, per-fixture SDR gates F32_FIXTURE_DB (measured 80 / 98 / 127 dB);
  * bf16 mode (bf16 MFMA operands, fp32 accumulation and norms): SDR >= BF16_SDR_DB = 40 dB (measured 49-54 dB);
  * stage-by-stage (f32): SDR >= F32_STAGE_DB = 90 dB per intermediate (measured 103-135 dB).
SDR here is 10 log10(sum ref^2 / sum (ref - out)^2) over the whole output (`src/loss.py:9-30` without clamp).
"""
import json
import os
import tempfile

import numpy as np
import pytest
import torch

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu

F32_SDR_DB = 110.0          # f32, inputs away from the mask singularity (measured 124-127 dB)
F32_MAXREL = 1e-4
F32_FIXTURE_DB = {"b1_t44100_vocals": 70.0, "b2_t30000_drums_bass": 85.0, "b1_t1500_other": 110.0}
F32_6S_DB = {"oracle": 85.0, "fixture": 75.0}   # measured 98.6 / 89.4 dB (phase-singular bins in the fixture)
F32_STAGE_DB = 90.0
BF16_SDR_DB = 40.0

REPORT = os.path.join(REPO, "gpurun_out", "parity_report.json")


def _report(key, val):
    os.makedirs(os.path.dirname(REPORT), exist_ok=True)
    d = {}
    if os.path.exists(REPORT):
        try:
            d = json.load(open(REPORT))
        except Exception:
            d = {}
    d[key] = val
    json.dump(d, open(REPORT, "w"), indent=1)


def sdr_db(ref, out):
    ref = np.asarray(ref, np.float64)
    out = np.asarray(out, np.float64)
    return float(10 * np.log10(np.sum(ref ** 2) / max(np.sum((ref - out) ** 2), 1e-300)))


@pytest.fixture(scope="module")
def models(state_dict, text_table):
    from athd.model import AudioTextHTDemucs
    from athd.weights import STEMS
    table = {s: text_table[i] for i, s in enumerate(STEMS)}
    ms = {}
    for dt in ("f32", "bf16"):
        m = AudioTextHTDemucs(dtype=dt, text_table=table)
        m.load_state_dict(state_dict)
        ms[dt] = m.to("cuda").eval()
    return ms


def _golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz")))


@pytest.mark.parametrize("name", ["b1_t44100_vocals", "b2_t30000_drums_bass", "b1_t1500_other"])
@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_golden_fixture(models, name, dt):
    from athd.weights import STEMS
    g = _golden(name)
    wav = torch.as_tensor(g["wav"]).cuda()
    prompts = [STEMS[i] for i in g["prompt_idx"]]
    out = models[dt](wav, prompts[0] if len(prompts) == 1 else prompts)
    torch.cuda.synchronize()
    out = out.cpu().numpy()
    ref = g["out"]
    assert out.shape == ref.shape
    assert np.isfinite(out).all()
    s = sdr_db(ref, out)
    rel = float(np.abs(out - ref).max() / np.sqrt(np.mean(ref ** 2)))
    _report(f"{name}/{dt}", {"sdr_db": s, "maxabs_over_rms": rel})
    if dt == "f32":
        assert s >= F32_FIXTURE_DB[name], (s, rel)
        if F32_FIXTURE_DB[name] >= F32_SDR_DB:        # the fixture whose spectrum is away from the singularity
            assert rel <= F32_MAXREL, rel
    else:
        assert s >= BF16_SDR_DB, s


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_full_segment_6s(models, oracle_model, text_table, dt):
    """Full 6 s segment (T = 264600, the BASELINE config), reference fixture subsample + oracle full output."""
    g = _golden("b1_t264600_vocals")
    wav = torch.as_tensor(g["wav"])
    out = models[dt](wav.cuda(), "vocals").cpu().numpy()
    sub = out[..., ::97]
    s_fix = sdr_db(g["out_stride97"], sub)
    ref = oracle_model.forward(wav, torch.as_tensor(text_table[3:4])).numpy()
    s = sdr_db(ref, out)
    _report(f"6s/{dt}", {"sdr_db_vs_oracle": s, "sdr_db_vs_fixture_stride97": s_fix})
    if dt == "f32":
        assert s >= F32_6S_DB["oracle"] and s_fix >= F32_6S_DB["fixture"], (s, s_fix)
    else:
        assert s >= BF16_SDR_DB and s_fix >= BF16_SDR_DB, (s, s_fix)


PHASE_COND_MIN = 5e-8


def _phase_cond(z):
    """min |m + 1e-8| over the nonzero CaC magnitudes the reference divides by (`phase = z / (mag + 1e-8)`,
    ATHTDemucs_v2.py:308; mag[:, :2] = Re, Im of the left channel).  Where a bin has m close to -1e-8 the mask
    formula is singular: its output depends on the last bits of that STFT bin, which no two FFTs share (a bin
    with |m + 1e-8| = 4e-9 costs ~50 dB of whole-output SDR).  Parity inputs are chosen away from that set."""
    zl = z[:, 0].numpy()
    m = np.stack([zl.real, zl.imag])
    return float(np.abs(m + 1e-8)[m != 0].min())


@pytest.mark.parametrize("T", [30001, 44102, 9999, 33297])
def test_ragged_length(models, oracle_model, text_table, T):
    """T % 4 != 0: the time encoder's right pad and the time decoder's last ConvT output (4 L1 samples) linearly
    resized to T (ATHTDemucs_v2.py:128-131), the general branch of tdec_last (dec_last.hip).  T = 33297 (Tspec = 33):
    the fused iSTFT splits the frames over 2 workgroups of 17 | 16 (spectral.hip istft_ola_split; a fixed 32-frame
    split would leave a 1-frame last workgroup whose head and tail blocks coincide)."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(1, T, seed0=6))
    cap = {}
    ref = oracle_model.forward(wav, torch.as_tensor(text_table[1:2]), capture=cap).numpy()
    assert _phase_cond(cap["z"]) >= PHASE_COND_MIN
    for dt in ("f32", "bf16"):
        out = models[dt](wav.cuda(), "bass").cpu().numpy()
        assert out.shape == ref.shape
        s = sdr_db(ref, out)
        rel = float(np.abs(out - ref).max() / np.sqrt(np.mean(ref.astype(np.float64) ** 2)))
        _report(f"ragged_T{T}/{dt}", {"sdr_db_vs_oracle": s, "maxabs_over_rms": rel})
        if dt == "f32":
            assert s >= F32_SDR_DB and rel <= F32_MAXREL, (s, rel)
        else:
            assert s >= BF16_SDR_DB, s


@pytest.mark.parametrize("T,B", [(300000, 1), (4096, 2)])
def test_prompts_long_and_short(models, oracle_model, text_table, T, B):
    """forward_prompts (4 prompts) at the two ends of the supported lengths, both dtypes, against the oracle:
      * T = 300000 (Tspec = 293 > 272): the frequency levels 0-1 take the unfused implicit-GEMM path (fenc_row.hip
        holds at most 272 frames per row), the main.py:277-290 "variable lengths" case beyond one 6 s window;
      * T = 4096 (Tspec = 4), B = 2: 8 decode items whose level-2 ConvT rows per item (Tspec^2 = 16 freq, L = 16
        time) are fewer than a convt4 unit's 32, so a unit would straddle 3+ items: the tiled four-residue GEMM
        runs instead (convt4_supported)."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(B, T, seed0=T % 1000 + 11))
    cap = {}
    oracle_model.forward(wav[:1], torch.as_tensor(text_table[:1]), capture=cap)
    cond = _phase_cond(cap["z"])
    ref = oracle_model.forward_prompts(wav, torch.as_tensor(text_table)).numpy()
    for dt in ("f32", "bf16"):
        out = models[dt].forward_prompts(wav.cuda(), ["drums", "bass", "other", "vocals"]).cpu().numpy()
        assert out.shape == ref.shape and np.isfinite(out).all()
        s = min(sdr_db(ref[b, p], out[b, p]) for b in range(B) for p in range(4))
        _report(f"prompts_T{T}_B{B}/{dt}", {"sdr_db_min_vs_oracle": s, "phase_cond": cond})
        if dt == "bf16":
            assert s >= BF16_SDR_DB, s
        elif cond >= PHASE_COND_MIN:
            assert s >= F32_SDR_DB, s
        else:
            assert s >= F32_FIXTURE_DB["b1_t44100_vocals"], (s, cond)


def test_forward_prompts_matches_forward(models):
    """Encode-once/decode-P path == P separate forwards.  f32 model: equal to fp32 rounding (GroupNorm statistics
    are fp64 atomics whose order varies); bf16 model: the two paths agree to >= 40 dB (order-dependent statistics
    can flip individual bf16 roundings of intermediates)."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(3, 50000)).cuda()
    prompts = ["drums", "bass", "other", "vocals"]
    for dt in ("f32", "bf16"):
        m = models[dt]
        multi = m.forward_prompts(wav, prompts)
        for p, name in enumerate(prompts):
            single = m(wav, name)
            if dt == "f32":
                assert torch.allclose(multi[:, p], single, atol=1e-5, rtol=1e-4), name
            else:
                assert sdr_db(single.cpu().numpy(), multi[:, p].cpu().numpy()) >= 40.0, name


@pytest.mark.parametrize("T", [264600, 33297, 50000])
def test_fdec1_fused_matches_unfused(models, monkeypatch, T):
    """The level-1 frequency decoder's GroupNorm statistics as quadratic forms of per-item Gram matrices of Z
    (fdec1f.hip: Z tiles computed on the matrix cores into LDS, never stored; the merge pass reads a 4-tap Z) ==
    the unfused path (8-tap Z stored by a GEMM, fdec_lr_stats3_kernel's sweep; ATHD_FDEC1_FUSED=0), bf16 model,
    3 segments x 4 prompts (segment / prompt item mapping of the skip-projection rows).  T = 264600: Tspec = 259,
    the bench shape (33 w blocks of 8, the last one 3 columns wide); 33297: Tspec = 33, the smallest Tspec the
    Gram pass takes; 50000: Tspec = 49.  The two differ in the MFMA accumulation order of Z (a bf16 rounding of Z
    may flip) and in how {sum, sumsq} are accumulated (fp32 Gram blocks vs fp32 row sums, both folded in fp64)."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(3, T, seed0=31)).cuda()
    prompts = ["drums", "bass", "other", "vocals"]
    m = models["bf16"]
    monkeypatch.setenv("ATHD_FDEC1_FUSED", "0")
    ref = m.forward_prompts(wav, prompts).cpu().numpy()
    monkeypatch.setenv("ATHD_FDEC1_FUSED", "1")
    out = m.forward_prompts(wav, prompts).cpu().numpy()
    assert np.isfinite(out).all()
    s = min(sdr_db(ref[b, p], out[b, p]) for b in range(3) for p in range(4))
    _report(f"fdec1_fused_T{T}", {"sdr_db_min_vs_unfused": s})
    assert s >= 60.0, s


def test_rowln_off_matches_default(models, oracle_model, text_table, monkeypatch):
    """ATHD_ROWLN=0 (bf16: out_proj on gemm5's residual epilogue + the FFN's LayerNorm as its own pass, round 4's
    form) == the default out_proj + LayerNorm in one full-row pass (rowln.hip), and both match the oracle: every
    kernel path left in libathd.so is reached by a test.  Both paths round H to bf16 from the
    same f32 rows, so they differ only in the f32 summation order of out_proj's K loop."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(2, 264600, seed0=41))
    prompts = ["drums", "vocals"]
    m = models["bf16"]
    monkeypatch.setenv("ATHD_ROWLN", "0")
    off = m.forward_prompts(wav.cuda(), prompts).cpu().numpy()
    monkeypatch.setenv("ATHD_ROWLN", "1")
    on = m.forward_prompts(wav.cuda(), prompts).cpu().numpy()
    ref = oracle_model.forward_prompts(wav, torch.as_tensor(text_table[[0, 3]])).numpy()
    s_on_off = min(sdr_db(on[b, p], off[b, p]) for b in range(2) for p in range(2))
    s_off = min(sdr_db(ref[b, p], off[b, p]) for b in range(2) for p in range(2))
    _report("rowln_off", {"sdr_db_min_on_vs_off": s_on_off, "sdr_db_min_off_vs_oracle": s_off})
    assert s_on_off >= 50.0 and s_off >= BF16_SDR_DB, (s_on_off, s_off)


def test_text_mlp2_ln_forms_match(models, oracle_model, text_table, monkeypatch):
    """The text cross-attention's mlp2 + norm_out (ATHTDemucs_v2.py:47-49, bf16): rowln.hip's text form (weights L2 ->
    VGPR, A staged in LDS; the default) against the gemm3 row-LayerNorm form (ATHD_RLT=0), and both against the
    oracle - every kernel path left in libathd.so is reached by a test.  The two differ only in the f32 summation
    order of the K loop (and the text form's per-wave row partial sums)."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(2, 264600, seed0=43))
    prompts = ["bass", "other"]
    m = models["bf16"]
    monkeypatch.setenv("ATHD_RLT", "0")
    off = m.forward_prompts(wav.cuda(), prompts).cpu().numpy()
    monkeypatch.setenv("ATHD_RLT", "1")
    on = m.forward_prompts(wav.cuda(), prompts).cpu().numpy()
    ref = oracle_model.forward_prompts(wav, torch.as_tensor(text_table[[1, 2]])).numpy()
    s_on_off = min(sdr_db(on[b, p], off[b, p]) for b in range(2) for p in range(2))
    s_on = min(sdr_db(ref[b, p], on[b, p]) for b in range(2) for p in range(2))
    s_off = min(sdr_db(ref[b, p], off[b, p]) for b in range(2) for p in range(2))
    _report("text_mlp2_ln_forms", {"sdr_db_min_on_vs_off": s_on_off, "sdr_db_min_on_vs_oracle": s_on,
                                   "sdr_db_min_off_vs_oracle": s_off})
    assert s_on_off >= 50.0 and s_on >= BF16_SDR_DB and s_off >= BF16_SDR_DB, (s_on_off, s_on, s_off)


def test_fdec1_gram_large_mean(state_dict, text_table, monkeypatch):
    """VERDICT r04 weak #1 caveat 2: the level-1 Gram statistics in the cancellation regime.  The level-0 frequency
    decoder's GroupNorm shift (`freq_decoder.layers.0.1.bias`) is set to +30, so the level-1 ConvT input is
    GELU(30 + O(1)) ~ 30 + O(1): mean / std >= 30, and the fp32 Gram blocks sum_{w,c} x x^T are dominated by the DC
    part whose square the variance then subtracts.  bf16 fused (fdec1f.hip) and unfused (ATHD_FDEC1_FUSED=0, fp32 row
    sums) against the fp32 oracle on the same weights: fused within 3 dB of unfused."""
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_batch
    from athd.weights import STEMS
    from oracle.athtdemucs_ref import AudioTextHTDemucsRef
    sd = dict(state_dict)
    sd["freq_decoder.layers.0.1.bias"] = np.full_like(np.asarray(sd["freq_decoder.layers.0.1.bias"]), 30.0)
    wav = torch.as_tensor(synthetic_batch(2, 264600, seed0=41))
    oracle = AudioTextHTDemucsRef(sd)
    cap = {}
    oracle.forward(wav[:1], torch.as_tensor(text_table[:1]), capture=cap)
    ref = oracle.forward_prompts(wav, torch.as_tensor(text_table)).numpy()
    m = AudioTextHTDemucs(dtype="bf16", text_table={s: text_table[i] for i, s in enumerate(STEMS)})
    m.load_state_dict(sd)
    m = m.to("cuda").eval()
    res = {}
    for fused in ("0", "1"):
        monkeypatch.setenv("ATHD_FDEC1_FUSED", fused)
        out = m.forward_prompts(wav.cuda(), list(STEMS)).cpu().numpy()
        assert np.isfinite(out).all()
        res[fused] = min(sdr_db(ref[b, p], out[b, p]) for b in range(2) for p in range(4))
    _report("fdec1_gram_large_mean", {"sdr_db_min_fused": res["1"], "sdr_db_min_unfused": res["0"],
                                      "phase_cond": _phase_cond(cap["z"])})
    assert res["1"] >= res["0"] - 3.0, res
    assert res["1"] >= BF16_SDR_DB - 10.0, res


def test_bf16_forward_reproducible(models):
    """Two bf16 forwards of the same inputs (bench shape: 6 s segments x 4 prompts) are bit-identical (round 5):
    the level-1 frequency decoder's Gram statistics are summed from per-(workgroup, item) partial slots in a fixed
    order (fdec1f.hip fdec1_gram_reduce_kernel; round 4's fp32 atomics made two forwards differ at ~121 dB), and
    tdec_tail_kernel carries its 48-state pad (dec_last.hip; without it ~100 outputs per forward differed when the
    frequency branch ran beside it - round 6's probes show the pad is not covering an MFMA -> store hazard, DESIGN
    §4, so this test is what guards it).
    Residual risk, bounded: the GEMM epilogues' fp64 statistics atomics still add in arrival order; their last-bit
    differences are rounded away in the fp32 (mean, rstd) they feed, which has held in every comparison so far
    (DESIGN §4).  If this assert ever fails with a handful of differing outputs, compare with ATHD_SERIAL=1 first."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(4, 264600, seed0=57)).cuda()
    prompts = ["drums", "bass", "other", "vocals"]
    m = models["bf16"]
    a = m.forward_prompts(wav, prompts)
    diffs = []
    for _ in range(3):
        b = m.forward_prompts(wav, prompts)
        diffs.append(int((a != b).sum().item()))
    _report("bf16_reproducible", {"differing_outputs": diffs, "outputs": a.numel()})
    assert diffs == [0, 0, 0], diffs


def test_batch_independence(models):
    """Each segment of a batch is computed independently (per-sample normalisation, no cross-sample state)."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(3, 40000, seed0=99)).cuda()
    m = models["f32"]
    full = m(wav, ["vocals", "drums", "bass"])
    one = m(wav[1:2], "drums")
    assert torch.allclose(full[1:2], one, atol=1e-5, rtol=1e-5)


def test_decode_chunks_match_one_chunk(models):
    """Several decode chunks (each chunk's iSTFT on the second stream, overlapping the next chunk's decoder, the freq
    output double-buffered) == one chunk, f32 to fp32 rounding."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(3, 40000, seed0=77)).cuda()
    prompts = ["drums", "bass", "other", "vocals"]
    m = models["f32"]
    one = m.forward_prompts(wav, prompts)           # 12 items: one chunk at the default 64
    m.set_decode_items(4)                           # 3 chunks of one segment x 4 prompts
    try:
        many = m.forward_prompts(wav, prompts)
    finally:
        m.set_decode_items(None)
    assert torch.allclose(many, one, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_decode_chunks_per_item_prompts(models, dt):
    """athd_forward with a DIFFERENT prompt per segment over 5 decode chunks of one item each: every chunk rewrites
    the prompt row vectors (text_vec_kernel) and every other chunk the freq output buffer, while the previous
    chunk's time branch and iSTFT may still run on the second stream (forward.cpp decode_chunk orders both with
    ev_t).  Equals one chunk (f32: fp32 rounding; bf16: >= 40 dB, order-dependent statistics)."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(5, 40000, seed0=78)).cuda()
    prompts = ["drums", "vocals", "bass", "other", "vocals"]
    m = models[dt]
    one = m(wav, prompts)                           # 5 items: one chunk at the default 64
    m.set_decode_items(1)                           # 5 chunks of one (segment, prompt) item
    try:
        many = m(wav, prompts)
        torch.cuda.synchronize()
    finally:
        m.set_decode_items(None)
    if dt == "f32":
        assert torch.allclose(many, one, atol=1e-5, rtol=1e-4)
    else:
        for i in range(5):
            assert sdr_db(one[i].cpu().numpy(), many[i].cpu().numpy()) >= 40.0, i


def test_bench_batch_one_chunk(models, oracle_model, text_table):
    """The bench configuration exactly as timed: B=64 x 6 s x 4 prompts = 256 items in one decode chunk (the
    largest buffers and launch grids of the path), captured as a HIP graph and REPLAYED (bench.py at N=1).  Rows 0
    and 63 of the replayed output against the fp32 oracle's forward_prompts (bf16 gate BF16_SDR_DB), and against
    the same segments run as a 2-segment eager batch."""
    from athd.synth import synthetic_batch
    prompts = ["drums", "bass", "other", "vocals"]
    base = synthetic_batch(8, 264600, seed0=4242)
    wav = torch.as_tensor(np.concatenate([base] * 8)).cuda()          # (64, 2, 264600)
    m = models["bf16"]
    m.set_decode_items(256)                     # the bench's setting: all 256 items in one decode chunk
    try:
        g, full = m.capture_prompts(wav, prompts)
        full.zero_()
        g.replay()
        torch.cuda.synchronize()
    finally:
        m.set_decode_items(None)
    pick = [0, 63]
    few = m.forward_prompts(wav[pick], prompts)
    ref = oracle_model.forward_prompts(wav[pick].cpu(), torch.as_tensor(text_table)).numpy()
    res = {}
    for i, j in enumerate(pick):
        for p in range(len(prompts)):
            got = full[j, p].cpu().numpy()
            s_or = sdr_db(ref[i, p], got)
            res[f"{j}/{prompts[p]}"] = s_or
            assert s_or >= BF16_SDR_DB, (j, prompts[p], s_or)
            assert sdr_db(few[i, p].cpu().numpy(), got) >= 40.0, (j, prompts[p])
    _report("bench_config_graph_replay_vs_oracle/bf16", res)
    del g, full, few
    torch.cuda.empty_cache()


def test_splitk_tail_matches_unsplit(models, oracle_model, text_table, monkeypatch):
    """linear2 (K = 2048) with its last partial round of 256 x 256 tiles split along K (gemm5.hip: the pieces leave
    f32 partial tiles, gemm5_sk_reduce_kernel adds them in piece order and runs the residual / statistics epilogue)
    == the unsplit launch (ATHD_SK=0).  B = 34: freq 552 tiles (tail 40, 6 pieces each), time 276 tiles (tail 20, 8
    pieces each) on 256 CUs.  The two differ only in the fp32 summation order of those tiles' K loops; the split is
    bit-reproducible run to run."""
    from athd.synth import synthetic_batch
    base = synthetic_batch(17, 264600, seed0=77)
    wav = torch.as_tensor(np.concatenate([base, base[::-1]])).cuda()       # (34, 2, 264600)
    prompts = ["drums", "vocals"]
    m = models["bf16"]
    monkeypatch.setenv("ATHD_SK", "0")
    off = m.forward_prompts(wav, prompts).cpu().numpy()
    monkeypatch.setenv("ATHD_SK", "1")
    on = m.forward_prompts(wav, prompts).cpu().numpy()
    again = m.forward_prompts(wav, prompts).cpu().numpy()
    pick = [0, 33]
    ref = oracle_model.forward_prompts(wav[pick].cpu(), torch.as_tensor(text_table[[0, 3]])).numpy()
    s_on_off = min(sdr_db(off[b, p], on[b, p]) for b in range(34) for p in range(2))
    s_ref = min(sdr_db(ref[i, p], on[j, p]) for i, j in enumerate(pick) for p in range(2))
    _report("splitk_tail", {"sdr_db_min_split_vs_unsplit": s_on_off, "sdr_db_min_vs_oracle": s_ref,
                            "split_reproducible": bool(np.array_equal(on, again))})
    assert np.array_equal(on, again)            # the pieces are added in a fixed order
    # (a different fp32 summation order of linear2's K loop moves some bf16 roundings downstream: measured 55.6 dB,
    # the same as out_proj's two accumulation orders in test_rowln_off_matches_default)
    assert s_on_off >= 50.0 and s_ref >= BF16_SDR_DB, (s_on_off, s_ref)


@pytest.mark.parametrize("T", [30000, 30001])
def test_intermediates_f32(models, oracle_model, text_table, T):
    """Stage-by-stage parity (f32) via the ATHD_DUMP debug dump: localises any divergence.  T = 30001 runs the
    ragged-length paths (time encoder right pad, last time level resized 4 L1 -> T)."""
    from athd.synth import synthetic_batch
    B = 2
    wav = torch.as_tensor(synthetic_batch(B, T, seed0=5 if T == 30000 else 6))
    te = torch.as_tensor(text_table[[0, 3]])
    with tempfile.TemporaryDirectory() as tmp:
        os.environ["ATHD_DUMP"] = tmp
        try:
            out = models["f32"](wav.cuda(), ["drums", "vocals"]).cpu().numpy()
            torch.cuda.synchronize()
        finally:
            del os.environ["ATHD_DUMP"]
        dump = {}
        for line in open(os.path.join(tmp, "index.txt")):
            name, n, _ = line.split()
            dump[name] = np.fromfile(os.path.join(tmp, name + ".f32"), dtype=np.float32, count=int(n))
    cap = {}
    ref_out = oracle_model.forward(wav, te, capture=cap).numpy()
    Ts = cap["z"].shape[-1]
    if T != 30000:
        assert _phase_cond(cap["z"]) >= PHASE_COND_MIN
    res = {}

    def cmp(name, ref, got):
        ref = np.asarray(ref, np.float32).reshape(-1)
        got = got.reshape(-1)
        res[name] = {"sdr_db": sdr_db(ref, got), "maxabs": float(np.abs(ref - got).max()),
                     "ref_rms": float(np.sqrt(np.mean(ref.astype(np.float64) ** 2)))}

    z = cap["z"]
    spec = torch.view_as_real(z).permute(0, 2, 3, 1, 4).reshape(B, 2048, Ts, 4).numpy()
    cmp("specT", spec.transpose(0, 2, 1, 3), dump["specT"])
    for i in range(4):
        cmp(f"saved{i}", cap["saved"][i].permute(0, 2, 3, 1).numpy(), dump[f"saved{i}"])
        cmp(f"saved_t{i}", cap["saved_t"][i].permute(0, 2, 1).numpy(), dump[f"saved_t{i}"])
    cmp("x_enc", cap["x_enc"].permute(0, 2, 3, 1).numpy(), dump["x_enc"])
    cmp("xt_enc", cap["xt_enc"].permute(0, 2, 1).numpy(), dump["xt_enc"])
    cmp("x_cond", cap["x_cond"].permute(0, 2, 3, 1).numpy(), dump["x_cond"])
    cmp("xt_cond", cap["xt_cond"].permute(0, 2, 1).numpy(), dump["xt_cond"])
    cmp("FO", cap["x_fo"].permute(0, 3, 2, 1).numpy(), dump["FO"])          # FO^T [item][t][row][2]
    cmp("XT2", cap["xt_out"].permute(0, 2, 1).numpy(), dump["XT2"])      # time_out(time decoder) [item][n][2]
    cmp("freq_wav", cap["freq_wav"].numpy(), out - cap["xt_dec"].numpy())
    cmp("out", ref_out, out)
    _report(f"intermediates_f32_T{T}", res)
    bad = {k: v for k, v in res.items() if v["sdr_db"] < F32_STAGE_DB}
    assert not bad, bad


def _bf16_dump(path, shape):
    raw = np.fromfile(path, dtype=np.uint16)
    return (raw.astype(np.uint32) << 16).view(np.float32).reshape(shape)


@pytest.mark.parametrize("T,B", [(44100, 2), (264600, 1)])
def test_encoder_levels_bf16_stage(models, oracle_model, text_table, monkeypatch, T, B):
    """The bf16 encoder levels (ATHD_DUMP's raw saved{i} / saved_t{i}) against the fp32 oracle's captures, and the
    fused narrow frequency levels (fenc_row.hip: fenc_row0_kernel as 8-wave workgroups, fenc_row1_kernel) against the
    unfused implicit-GEMM + DConv path (ATHD_FENC_ROW=0) at the same inputs.  Tspec = 44 and 259 (the bench rows)."""
    from athd.synth import synthetic_batch
    wav = torch.as_tensor(synthetic_batch(B, T, seed0=23))
    te = torch.as_tensor(text_table[:B])
    cap = {}
    oracle_model.forward(wav, te, capture=cap)
    prompts = ["drums", "bass"][:B]
    dumps = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("ATHD_FENC_ROW", fused)
        with tempfile.TemporaryDirectory() as tmp:
            monkeypatch.setenv("ATHD_DUMP", tmp)
            models["bf16"](wav.cuda(), prompts)
            torch.cuda.synchronize()
            monkeypatch.delenv("ATHD_DUMP")
            d = {}
            for i in range(4):
                ref = cap["saved"][i].permute(0, 2, 3, 1).numpy()        # [B][F][Ts][C]
                d[f"saved{i}"] = _bf16_dump(os.path.join(tmp, f"saved{i}.bf16"), ref.shape)
                reft = cap["saved_t"][i].permute(0, 2, 1).numpy()       # [B][L][C]
                d[f"saved_t{i}"] = _bf16_dump(os.path.join(tmp, f"saved_t{i}.bf16"), reft.shape)
            dumps[fused] = d
    res = {}
    for i in range(4):
        res[f"saved{i}"] = sdr_db(cap["saved"][i].permute(0, 2, 3, 1).numpy(), dumps["1"][f"saved{i}"])
        res[f"saved_t{i}"] = sdr_db(cap["saved_t"][i].permute(0, 2, 1).numpy(), dumps["1"][f"saved_t{i}"])
    for i in (0, 1):
        res[f"saved{i}_fused_vs_unfused"] = sdr_db(dumps["0"][f"saved{i}"], dumps["1"][f"saved{i}"])
    _report(f"encoder_levels_bf16_T{T}", res)
    # (measured round 6: 44.5-51.5 dB vs the oracle, fused vs unfused 46.3-51.6 dB: two bf16 roundings apart)
    bad = {k: v for k, v in res.items() if v < (42.0 if "unfused" in k else BF16_SDR_DB)}
    assert not bad, (bad, res)


def test_reference_decoders_stage_f32(models, state_dict):
    """The reference-owned decoders pinned at their own stage on REFERENCE-made data.

    tests/golden/b1_t44100_vocals.npz holds the reference's own FreqDecoder / TimeDecoder outputs (`x_fdec`,
    `xt_tdec`, captured by oracle/gen_golden.py at ATHTDemucs_v2.py:293 / :313).  The HIP f32 path's dumps after the
    1x1 projections (`FO` = freq_out(freq_decoder), `XT2` = time_out(time_decoder), ATHTDemucs_v2.py:294 / :314)
    are compared with the same projections applied here (float64) to the reference's captures.  These stages sit
    upstream of the mask's phase singularity (`:304-309`), so SURVEY.md §8(c)'s f32 tolerance applies as stated:
    max|err| <= 1e-4 * RMS."""
    from athd.weights import STEMS
    g = _golden("b1_t44100_vocals")
    wav = torch.as_tensor(g["wav"]).cuda()
    prompt = STEMS[int(g["prompt_idx"][0])]
    with tempfile.TemporaryDirectory() as tmp:
        os.environ["ATHD_DUMP"] = tmp
        try:
            models["f32"](wav, prompt)
            torch.cuda.synchronize()
        finally:
            del os.environ["ATHD_DUMP"]
        dump = {}
        for line in open(os.path.join(tmp, "index.txt")):
            name, n, _ = line.split()
            dump[name] = np.fromfile(os.path.join(tmp, name + ".f32"), dtype=np.float32, count=int(n))
    wf = np.asarray(state_dict["freq_out.weight"], np.float64).reshape(2, 4)
    bf = np.asarray(state_dict["freq_out.bias"], np.float64)
    wt = np.asarray(state_dict["time_out.weight"], np.float64).reshape(2, 4)
    bt = np.asarray(state_dict["time_out.bias"], np.float64)
    fo_ref = np.einsum("oc,bchw->bohw", wf, g["x_fdec"].astype(np.float64)) + bf[None, :, None, None]
    xt_ref = np.einsum("oc,bcn->bon", wt, g["xt_tdec"].astype(np.float64)) + bt[None, :, None]
    res = {}
    for name, ref, got in (("FO", fo_ref.transpose(0, 3, 2, 1), dump["FO"]),      # FO^T [item][t][row][2]
                           ("XT2", xt_ref.transpose(0, 2, 1), dump["XT2"])):        # [item][n][2]
        ref = ref.reshape(-1)
        assert got.size == ref.size, (name, got.size, ref.size)
        rms = float(np.sqrt(np.mean(ref ** 2)))
        res[name] = {"maxabs_over_rms": float(np.abs(got - ref).max() / rms), "sdr_db": sdr_db(ref, got)}
    _report("reference_decoders_stage_f32", res)
    for name, v in res.items():
        assert v["maxabs_over_rms"] <= F32_MAXREL, (name, v)


SHARP_SCALE = 6.0          # Q and K in-projection rows x6: logits x36, mean max softmax prob ~0.1-0.3 (vs ~0.005)
SHARP_BF16_SDR_DB = 35.0   # bf16 logit rounding is amplified by the sharpening (measured 47.6-48.2 dB)


def test_sharp_attention_encoder(state_dict, text_table):
    """With the synthetic weights every attention row is nearly uniform (max prob ~ 1/Nk), so a kernel that pairs
    P with the wrong V rows inside a key tile would still pass the model-level tests.  Sharpen all ten transformer
    attentions (scale W_q, W_k) and compare the transformer output x_enc / xt_enc with the oracle."""
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_batch
    from athd.weights import STEMS
    from oracle.athtdemucs_ref import AudioTextHTDemucsRef
    sd = dict(state_dict)
    for k in sd:
        if "crosstransformer" in k and k.endswith("in_proj_weight"):
            w = np.array(sd[k], dtype=np.float32, copy=True)
            w[:1024] *= SHARP_SCALE
            sd[k] = w
    wav = torch.as_tensor(synthetic_batch(2, 30000, seed0=11))
    te = torch.as_tensor(text_table[[1, 2]])
    cap = {}
    AudioTextHTDemucsRef(sd).forward(wav, te, capture=cap)
    ref = {"x_enc": cap["x_enc"].permute(0, 2, 3, 1).numpy(), "xt_enc": cap["xt_enc"].permute(0, 2, 1).numpy()}
    table = {s: text_table[i] for i, s in enumerate(STEMS)}
    res = {}
    for dt in ("f32", "bf16"):
        m = AudioTextHTDemucs(dtype=dt, text_table=table)
        m.load_state_dict(sd)
        m = m.to("cuda").eval()
        with tempfile.TemporaryDirectory() as tmp:
            os.environ["ATHD_DUMP"] = tmp
            try:
                m(wav.cuda(), ["bass", "other"])
                torch.cuda.synchronize()
            finally:
                del os.environ["ATHD_DUMP"]
            for name in ("x_enc", "xt_enc"):
                got = np.fromfile(os.path.join(tmp, name + ".f32"), dtype=np.float32)
                res[f"{dt}/{name}"] = sdr_db(ref[name].reshape(-1), got)
    _report("sharp_attention", res)
    for key, v in res.items():
        assert v >= (F32_STAGE_DB if key.startswith("f32") else SHARP_BF16_SDR_DB), res


def test_attn_pingpong_bit_identical(models, state_dict, text_table):
    """attn_pp_kernel (ATHD_ATTN_PP=1: two wave groups per SIMD alternating MFMA and softmax sections, attn.hip) does
    attn32_kernel's arithmetic in the same order, so the bf16 forward is bit-identical with either kernel: on the
    bench shape (6 s segments x 4 prompts: full and tail key tiles) and with sharpened attentions on a short input
    (Nq / Nk below one 256-query block; the defer-max rescale branch taken)."""
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_batch
    from athd.weights import STEMS

    def both(fn):
        outs = []
        for pp in ("0", os.environ.get("ATHD_PP_TEST_MODE", "1")):
            os.environ["ATHD_ATTN_PP"] = pp
            try:
                outs.append(fn())
            finally:
                del os.environ["ATHD_ATTN_PP"]
        return outs

    wav = torch.as_tensor(synthetic_batch(4, 264600, seed0=57)).cuda()
    m = models["bf16"]
    a, b = both(lambda: m.forward_prompts(wav, ["drums", "bass", "other", "vocals"]).cpu())
    n_full = int((a != b).sum().item())
    sd = dict(state_dict)
    for k in sd:
        if "crosstransformer" in k and k.endswith("in_proj_weight"):
            w = np.array(sd[k], dtype=np.float32, copy=True)
            w[:1024] *= SHARP_SCALE
            sd[k] = w
    ms = AudioTextHTDemucs(dtype="bf16", text_table={s: text_table[i] for i, s in enumerate(STEMS)})
    ms.load_state_dict(sd)
    ms = ms.to("cuda").eval()
    wav2 = torch.as_tensor(synthetic_batch(2, 30000, seed0=11)).cuda()
    c, e = both(lambda: ms(wav2, ["bass", "other"]).cpu())
    n_sharp = int((c != e).sum().item())
    _report("attn_pingpong", {"differing_full": n_full, "differing_sharp": n_sharp, "outputs": a.numel() + c.numel()})
    assert n_full == 0 and n_sharp == 0, (n_full, n_sharp)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_graph_replay_matches_eager(models, dt):
    """capture_prompts: one forward_prompts captured into a HIP graph (both branch streams, event fork/joins,
    statistics memset) and replayed equals the eager call, also after the input is rewritten in place (the graph
    reads the buffer, not a snapshot).  f32: fp32 rounding (order-dependent fp64 statistics atomics); bf16: >= 40 dB."""
    from athd.synth import synthetic_batch
    prompts = ["drums", "bass", "other", "vocals"]
    m = models[dt]
    wav = torch.as_tensor(synthetic_batch(2, 50000, seed0=321)).cuda()
    g, out = m.capture_prompts(wav, prompts)
    for seed in (321, 555):
        wav.copy_(torch.as_tensor(synthetic_batch(2, 50000, seed0=seed)))
        g.replay()
        torch.cuda.synchronize()
        ref = m.forward_prompts(wav, prompts)
        if dt == "f32":
            assert torch.allclose(out, ref, atol=1e-5, rtol=1e-4), seed
        else:
            assert sdr_db(ref.cpu().numpy(), out.cpu().numpy()) >= 40.0, seed
    del g
