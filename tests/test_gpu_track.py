"""A15 on the GPU: fade + overlap-add (athd_overlap_add), sdr_loss (athd_sdr) and whole-track separation
(athd.inference.separate_track) against the oracle restatement of test_inference.py:92-155 / src/loss.py:9-30.
Tolerances: overlap-add max|err| <= 1e-6 * max|x| (torch.linspace's own CPU/GPU formulas differ by <= 1 ulp);
sharded spans recombine bit-exactly; SDR within 1e-4 dB; f32 track separation >= 70 dB SDR vs the oracle loop."""
import numpy as np
import pytest
import torch

from oracle.athtdemucs_ref import chunk_plan, linear_fade, sdr_db

pytestmark = pytest.mark.gpu


def _sdr(ref, out):
    """Unclamped SDR (dB) for parity; the oracle's sdr_db keeps the reference metric's +-30 dB clamp."""
    ref = ref.double()
    return float(10 * torch.log10((ref ** 2).sum() / ((ref - out.double()) ** 2).sum().clamp_min(1e-300)))


def _oracle_ola(win, L, sr=44100, seg=6.0, ov=0.1):
    S = win.shape[1]
    final = torch.zeros((S, 2, L), dtype=torch.float32)
    for k, (s, e, fi, fo) in enumerate(chunk_plan(L, sr, seg, ov)):
        final[:, :, s:e] += linear_fade(win[k, :, :, :e - s], fi, fo)
    return final


@pytest.mark.parametrize("L", [44100 * 20, 264600, 100000, 2 * 260190 + 264600, 44100 * 61 + 12345])
def test_overlap_add_matches_oracle(L):
    from athd.inference import overlap_add, window_plan
    plan = window_plan(L)
    g = torch.Generator().manual_seed(L)
    win = torch.randn((len(plan), 3, 2, 264600), generator=g)
    ref = _oracle_ola(win, L)
    got = overlap_add(win.cuda(), L, 264600, 4410).cpu()
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() <= 1e-6 * win.abs().max().item()


def test_overlap_add_sharded_spans_recombine_exactly():
    """Window ranges [0, a) and [a, n) summed into a track by rank order == the single-range result, bit-exactly
    (0.0f + x = x, and each seam sample adds window k-1 before window k as the reference loop does)."""
    from athd.inference import overlap_add, window_plan
    L = 44100 * 45
    plan = window_plan(L)
    n = len(plan)
    win = torch.randn((n, 2, 2, 264600), generator=torch.Generator().manual_seed(3)).cuda()
    full = overlap_add(win, L, 264600, 4410)
    for a in (1, n // 2, n - 1):
        track = torch.zeros_like(full)
        for k0, k1 in ((0, a), (a, n)):
            span = overlap_add(win[k0:k1].contiguous(), L, 264600, 4410, k0, k1)
            s0 = plan[k0].start
            track[:, :, s0:s0 + span.shape[-1]] += span
        assert torch.equal(track, full), a


def test_sdr_loss_matches_reference_formula():
    from athd.inference import sdr_loss
    g = torch.Generator().manual_seed(1)
    tgt = torch.randn(2, 300000, generator=g)
    for scale in (0.0, 1e-3, 0.1, 1.0, 3.0):
        est = tgt + scale * torch.randn(2, 300000, generator=g)
        got = -sdr_loss(est.cuda(), tgt.cuda()).item()
        assert abs(got - sdr_db(est, tgt)) < 1e-4, scale
    assert abs(-sdr_loss(torch.zeros(2, 1000).cuda(), tgt[:, :1000].cuda()).item() - 0.0) < 1e-4
    # batch rows: (4, 2, T) estimates reshape to 4 rows like the reference
    est = torch.randn(4, 2, 5000, generator=g)
    t4 = torch.randn(4, 2, 5000, generator=g)
    assert abs(-sdr_loss(est.cuda(), t4.cuda()).item() - sdr_db(est, t4)) < 1e-4


def test_loss_known_answers_main_py():
    """The reference's own known-answer loss checks, `main.py:65-140` (test_losses), on athd_sdr / athd_sisdr with
    (4, 2, 44100) batches: perfect reconstruction clamps both at +30 dB; a random estimate is negative; a 2x gain
    gives SDR 10 log10(|s|^2 / |s|^2) = 0 dB and SI-SDR +30 (clamp); target + noise at SNR 20 / 10 / 5 / 0 / -5 dB
    gives SDR ~ SNR (decreasing); 0.8 target + 0.2 interference gives 10 log10(1 / 0.08) = 10.97 dB (the comment
    at main.py:136 says "~13-14 dB"; the arithmetic says 11.0).  Every value also equals the oracle's fp64 restatement
    of src/loss.py to 1e-4 dB (1e-3 for SI-SDR, computed in fp32 torch ops by the reference)."""
    from athd.inference import sdr_loss, sisdr_loss
    from oracle.athtdemucs_ref import sisdr_db
    g = torch.Generator().manual_seed(65)

    def both(est, tgt):
        s = -sdr_loss(est.cuda(), tgt.cuda()).item()
        si = -sisdr_loss(est.cuda(), tgt.cuda()).item()
        assert abs(s - sdr_db(est, tgt)) < 1e-4 and abs(si - sisdr_db(est, tgt)) < 1e-3, (s, si)
        return s, si

    tgt = torch.randn(4, 2, 44100, generator=g)
    assert both(tgt.clone(), tgt) == (30.0, 30.0)                                   # Test 1
    s, si = both(torch.randn(4, 2, 44100, generator=g), torch.randn(4, 2, 44100, generator=g))
    assert s < 0 and si < 0                                                          # Test 2
    s, si = both(2.0 * tgt, tgt)                                                     # Test 3
    assert abs(s) < 1e-5 and si == 30.0
    prev = None
    for snr_db in (20, 10, 5, 0, -5):                                                # Test 4
        noise = torch.randn(4, 2, 44100, generator=g) * torch.sqrt((tgt ** 2).mean() / 10 ** (snr_db / 10))
        s, _ = both(tgt + noise, tgt)
        assert abs(s - snr_db) < 0.2, (snr_db, s)
        assert prev is None or s < prev
        prev = s
    s, _ = both(0.8 * tgt + 0.2 * torch.randn(4, 2, 44100, generator=g), tgt)     # Test 5
    assert abs(s - 10 * np.log10(1 / 0.08)) < 0.2, s


def test_separate_track_matches_oracle_loop(state_dict, text_table, oracle_model):
    """12.1 s track, 3 windows (2 full + a 10k-sample tail), 2 stems, f32 model vs the oracle running the
    reference loop window by window (B=1, one stem at a time)."""
    from athd.inference import separate_and_score, separate_track
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_mixture
    from athd.weights import STEMS
    L = 520380 + 10000
    mix = torch.as_tensor(synthetic_mixture(L, seed=77))
    stems = ["drums", "vocals"]
    table = {s: text_table[i] for i, s in enumerate(STEMS)}
    m = AudioTextHTDemucs(dtype="f32", text_table=table)
    m.load_state_dict(state_dict)
    m = m.to("cuda").eval()
    got = separate_track(m, mix.cuda(), stems).cpu()
    ref = torch.zeros((2, 2, L))
    for si, s in enumerate(stems):
        te = torch.as_tensor(text_table[STEMS.index(s)][None])
        for st, en, fi, fo in chunk_plan(L):
            out = oracle_model.forward(mix[:, st:en][None], te)
            ref[si, :, st:en] += linear_fade(out, fi, fo)[0]
    for si in range(2):
        assert _sdr(ref[si], got[si]) >= 70.0, (stems[si], _sdr(ref[si], got[si]))
    final, scores = separate_and_score(m, mix.cuda(), ref.cuda(), stems)
    assert all(v >= 29.99 for v in scores.values()), scores      # clamped at +30 dB like sdr_loss


def test_test_inference_reference_signature(tmp_path, state_dict, text_table, oracle_model):
    """`test_inference.py:43-205` through the reference's own signature: a torch.save checkpoint and a one-track
    MUSDB18-HQ directory in, the per-stem SDR dict out, `<output_dir>/<cleaned name>/extracted_{stem}.wav` and
    `mixture.wav` written (`:157-175`).  f32 estimates vs the oracle running the reference loop window by window
    (>= 70 dB per stem), the returned SDRs == the oracle's sdr_loss of the device estimates, and the WAVs read back
    equal to the 16-bit PCM image of `final`."""
    from athd.inference import test_inference as run_test_inference
    from athd.musdb import HQ_FILES, read_wav, write_wav
    from athd.synth import synthetic_mixture
    from athd.weights import STEMS
    L = 520380 + 10000                                   # 3 windows: 2 full + a 10000-sample tail
    data = tmp_path / "quick_test"
    d = data / "Art's Band - A Song"
    d.mkdir(parents=True)
    # the mixture of test_separate_track_matches_oracle_loop (its spectrum keeps away from the mask's singular bins,
    # test_gpu_parity._phase_cond); the true stems are independent signals (only the SDR arithmetic reads them)
    parts = [synthetic_mixture(L, seed=77)] + [0.5 * synthetic_mixture(L, seed=500 + j) for j in range(4)]
    for f, x in zip(HQ_FILES, parts):
        write_wav(d / f"{f}.wav", x, 44100, "FLOAT")
    sd = {k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}
    ckpt = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": sd, "epoch": 3}, ckpt)
    table = {s: text_table[i] for i, s in enumerate(STEMS)}
    scores, final = run_test_inference(str(ckpt), str(data), str(tmp_path / "results"), 44100, 6.0, 0.1, "cuda",
                                       text_table=table, dtype="f32", return_final=True)
    assert list(scores) == STEMS
    mix = torch.as_tensor(read_wav(d / "mixture.wav")[0].T.copy())
    for si, s in enumerate(STEMS):
        te = torch.as_tensor(text_table[si][None])
        ref = torch.zeros((2, L))
        for st, en, fi, fo in chunk_plan(L):
            ref[:, st:en] += linear_fade(oracle_model.forward(mix[:, st:en][None], te), fi, fo)[0]
        got = final[si].cpu()
        assert _sdr(ref, got) >= 70.0, (s, _sdr(ref, got))
        truth = torch.as_tensor(read_wav(d / f"{s}.wav")[0].T.copy())
        want = sdr_db(got, truth)
        assert abs(scores[s] - want) < 1e-4, (s, scores[s], want)
    out = tmp_path / "results" / "Arts_Band__A_Song"           # test_inference.py:159-163 name cleaning
    for i, s in enumerate(STEMS):
        back = read_wav(out / f"extracted_{s}.wav")[0]
        img = np.clip(np.rint(final[i].cpu().numpy().T * 32767.0), -32768, 32767) / 32768.0
        assert np.array_equal(back, img.astype(np.float32)), s
    back = read_wav(out / "mixture.wav")[0]
    assert np.array_equal(back, (np.clip(np.rint(mix.numpy().T * 32767.0), -32768, 32767) / 32768.0).astype(np.float32))


def test_test_inference_default_clap(tmp_path, monkeypatch, state_dict):
    """VERDICT r04 #1 on the device: `test_inference(checkpoint_path, data_dir)` with no keyword arguments (the
    reference's own call, bf16 default) builds CLAP from the local cache (from_pretrained stubbed with a tiny offline
    CLAP: no pretrained files exist here), loads the checkpoint's clap.* keys and runs the whole track; its scores
    equal the same call given the checkpoint CLAP's get_text_features rows as an explicit text_table."""
    pytest.importorskip("transformers")
    import torch.nn.functional as F
    from test_text import FakeTokenizer, _clap_model, _patch_from_pretrained
    from athd.inference import test_inference as run_test_inference
    from athd.musdb import HQ_FILES, write_wav
    from athd.synth import synthetic_mixture
    from athd.weights import STEMS
    clap, trained = _clap_model(), _clap_model()
    with torch.no_grad():
        trained.text_projection.linear1.weight.mul_(-2.0)
    seen = []
    _patch_from_pretrained(monkeypatch, clap, seen)
    L = 264600 + 40000
    data = tmp_path / "quick_train"
    d = data / "A - B"
    d.mkdir(parents=True)
    parts = [synthetic_mixture(L, seed=77)] + [0.5 * synthetic_mixture(L, seed=500 + j) for j in range(4)]
    for f, x in zip(HQ_FILES, parts):
        write_wav(d / f"{f}.wav", x, 44100, "FLOAT")
    sd = {k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}
    sd.update({"clap." + k: v.clone() for k, v in trained.state_dict().items()})
    ckpt = tmp_path / "best_model.pt"
    torch.save({"model_state_dict": sd, "epoch": 1}, ckpt)
    monkeypatch.chdir(tmp_path)
    scores, final = run_test_inference(str(ckpt), str(data), return_final=True)
    assert [s[:2] for s in seen] == [("clap", "laion/clap-htsat-unfused"), ("tok", "laion/clap-htsat-unfused")]
    with torch.no_grad():
        rows = F.normalize(trained.text_projection(trained.text_model(**FakeTokenizer()(list(STEMS))).pooler_output),
                           dim=-1)
    table = {s: rows[i].numpy() for i, s in enumerate(STEMS)}
    scores2, final2 = run_test_inference(str(ckpt), str(data), "results2", text_table=table, return_final=True)
    assert list(scores) == list(STEMS)
    for s in STEMS:
        assert abs(scores[s] - scores2[s]) < 1e-3, (s, scores[s], scores2[s])
    assert _sdr(final2.cpu(), final.cpu()) > 80.0
    assert (tmp_path / "results" / "A__B" / "extracted_vocals.wav").exists()
