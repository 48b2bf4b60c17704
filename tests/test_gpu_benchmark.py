"""benchmark.py protocol twin on the GPU (athd/benchmark.py) against the oracle restatement of
`OurModel._chunked_inference` (benchmark.py:155-204) and `compute_sdr` / `compute_sisdr` (:555-588).

Tolerances: weighted overlap-add max|err| <= 1e-6 * max|x| (torch.linspace's CPU and GPU formulas differ by
<= 1 ulp); partial spans + normalise == the one-range result bit for bit; SDR / SI-SDR within 1e-3 dB; a 60 s track
separated with the f32 model >= 70 dB SDR against the oracle loop (one forward per window and stem)."""
import numpy as np
import pytest
import torch

from oracle.athtdemucs_ref import benchmark_chunked_inference, sdr_db, sisdr_db

pytestmark = pytest.mark.gpu

CH, OV = 264600, 66150


def _oracle_weighted(win, L):
    """Oracle loop with the window outputs given: window k's model output = win[k]."""
    outs = []
    for si in range(win.shape[1]):
        ks = iter(range(win.shape[0]))
        outs.append(benchmark_chunked_inference(lambda chunk: win[next(ks), si][None], torch.zeros(2, L)))
    return torch.stack(outs)


@pytest.mark.parametrize("L", [CH, CH + 1, 2 * 198450 + 5, 44100 * 60 + 4321, 100000, 3])
def test_weighted_overlap_add_matches_oracle(L):
    from athd.benchmark import num_windows, overlap_add_weighted
    n = num_windows(L, CH, OV)
    win = torch.randn((n, 2, 2, CH), generator=torch.Generator().manual_seed(L))
    ref = _oracle_weighted(win, L)
    got = overlap_add_weighted(win.cuda(), L, CH, OV).cpu()
    assert got.shape == ref.shape == (2, 2, L)
    assert (got - ref).abs().max().item() <= 1e-6 * win.abs().max().item()


def test_weighted_partial_spans_recombine_exactly():
    from athd.benchmark import num_windows, ola_normalize, overlap_add_weighted
    L = 44100 * 40 + 17
    n = num_windows(L, CH, OV)
    win = torch.randn((n, 2, 2, CH), generator=torch.Generator().manual_seed(9)).cuda()
    full = overlap_add_weighted(win, L, CH, OV)
    hop = CH - OV
    for cut in (1, n // 2, n - 1):
        acc = torch.zeros_like(full)
        wsum = torch.zeros(L, device="cuda")
        for k0, k1 in ((0, cut), (cut, n)):
            sp, ws = overlap_add_weighted(win[k0:k1].contiguous(), L, CH, OV, k0, k1, partial=True)
            acc[:, :, k0 * hop:k0 * hop + sp.shape[-1]] += sp
            wsum[k0 * hop:k0 * hop + ws.shape[0]] += ws
        assert torch.equal(ola_normalize(acc, wsum), full), cut


def test_compute_sdr_sisdr_match_reference_formulas():
    from athd.benchmark import compute_sdr, compute_sisdr
    g = torch.Generator().manual_seed(5)
    ref = torch.randn(2, 400000, generator=g) * 0.1
    for scale, gain in ((0.0, 1.0), (1e-3, 0.7), (0.05, 1.3), (0.3, 1.0), (3.0, 0.2)):
        est = gain * ref + scale * torch.randn(2, 400000, generator=g) + 0.01
        assert abs(compute_sdr(est.cuda(), ref.cuda()) - sdr_db(est[None], ref[None])) < 1e-3, scale
        assert abs(compute_sisdr(est.cuda(), ref.cuda()) - sisdr_db(est[None], ref[None])) < 1e-3, scale


def test_our_model_60s_track_matches_oracle(state_dict, text_table, oracle_model):
    """60 s synthetic track, 14 windows (the last zero-padded), 2 stems, f32 model vs the oracle loop."""
    from athd.benchmark import OurModel, evaluate_model_on_track
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_mixture
    from athd.weights import STEMS
    L = 44100 * 60
    mix = torch.as_tensor(synthetic_mixture(L, seed=60))
    m = AudioTextHTDemucs(dtype="f32", text_table={s: text_table[i] for i, s in enumerate(STEMS)})
    m.load_state_dict(state_dict)
    om = OurModel(m.to("cuda").eval())
    got = om.separate_stems(mix.cuda(), ["bass", "vocals"]).cpu()
    for j, stem in enumerate(["bass", "vocals"]):
        te = torch.as_tensor(text_table[STEMS.index(stem)][None])
        ref = benchmark_chunked_inference(lambda c: oracle_model.forward(c, te), mix)
        s = 10 * np.log10((ref.double() ** 2).sum().item() / ((ref.double() - got[j].double()) ** 2).sum().item())
        assert s >= 70.0, (stem, s)
    # per-track metrics of the reference's evaluation (benchmark.py:637-689) on the separated stems
    refs = {s: torch.as_tensor(synthetic_mixture(L, seed=100 + i)) * 0.5 for i, s in enumerate(STEMS)}
    res, est = evaluate_model_on_track(om, mix.cuda(), refs, "synthetic-60s")
    for s in STEMS:
        e = est[s].cpu()
        assert abs(getattr(res, f"sdr_{s}") - sdr_db(e[None], refs[s][None])) < 1e-3
        assert abs(getattr(res, f"sisdr_{s}") - sisdr_db(e[None], refs[s][None])) < 1e-3
    assert abs(res.sdr_avg - np.mean([getattr(res, f"sdr_{s}") for s in STEMS])) < 1e-9
