"""Structural pins of the oracle's HTDemucs restatement against the reference's own dumps (the only offline
pins for demucs internals).  Numbers are copied from
/root/reference/src/models/stem_separation/HTDemucs_Fwd_Pass.txt (line numbers cited) and
AudioTextHTDemucs_Full.txt."""
import torch

from oracle.htdemucs_ref import DConv, HTDemucsHot, MyTransformerEncoderLayer, CrossTransformerEncoderLayer


def _n(m):
    return sum(p.numel() for p in m.parameters())


def test_total_param_count():
    # HTDemucs_Fwd_Pass.txt:147  Total params: 41,984,456
    assert _n(HTDemucsHot(with_unused_decoder=True)) == 41_984_456


def test_layer_param_counts():
    m = HTDemucsHot()
    # HTDemucs_Fwd_Pass.txt:8-12,14-18 (tenc0 conv 816, dconv 3588, rewrite 4704; enc0 conv 1584)
    assert _n(m.tencoder[0].conv) == 816 and _n(m.tencoder[0].dconv) == 3588 and _n(m.tencoder[0].rewrite) == 4704
    assert _n(m.encoder[0].conv) == 1584
    # :21-24 (enc1/tenc1 conv 36960, dconv 12936, rewrite 18624), :56-59 (level 3: 590208, 189984, 295680)
    assert _n(m.encoder[1].conv) == 36960 and _n(m.encoder[1].dconv) == 12936 and _n(m.encoder[1].rewrite) == 18624
    assert _n(m.encoder[3].conv) == 590208 and _n(m.encoder[3].dconv) == 189984 and _n(m.encoder[3].rewrite) == 295680
    # :62-63 channel up-samplers 197120; :86-87 down-samplers 196992; :17 freq emb 24576
    assert _n(m.channel_upsampler) == 197120 and _n(m.channel_downsampler_t) == 196992
    assert _n(m.freq_emb) == 24576
    # :67,71 MyTransformerEncoderLayer 3,154,432; CrossTransformerEncoderLayer 3,155,456
    assert _n(MyTransformerEncoderLayer()) == 3_154_432
    assert _n(CrossTransformerEncoderLayer()) == 3_155_456
    assert _n(DConv(48)) == 3588


def test_reference_owned_param_count(state_dict):
    # 2,983,804 trainable parameters of the reference-owned modules
    n = sum(v.size for k, v in state_dict.items() if not k.startswith("htdemucs."))
    assert n == 2_983_804
    # hot htdemucs subset (A14): 35,212,376
    n = sum(v.size for k, v in state_dict.items() if k.startswith("htdemucs."))
    assert n == 35_212_376


def test_encoder_shapes_at_7p8s(state_dict):
    """HTDemucs_Fwd_Pass.txt shapes for the 7.8 s training segment (343980 samples): tenc 85995 -> 21499 ->
    5375 -> 1344 (proves the right pad to a multiple of 4), freq 512/128/32/8 rows x 336 frames, DConv on
    (B*Fr, C, T) (:16 '[512, 48, 336]'), 2688 = 8 x 336 freq tokens (:66)."""
    from oracle.htdemucs_ref import load_hot
    h = load_hot(state_dict)
    T = 343980
    x = torch.randn(1, 2, T) * 0.1
    z = h._spec(x)
    assert tuple(z.shape) == (1, 2, 2048, 336)
    mag = h._magnitude(z)
    xt, xf = x, mag
    exp_t = [85995, 21499, 5375, 1344]
    exp_f = [512, 128, 32, 8]
    with torch.no_grad():
        for i in range(4):
            xt = h.tencoder[i](xt)
            xf = h.encoder[i](xf)
            assert xt.shape[-1] == exp_t[i]
            assert tuple(xf.shape[-2:]) == (exp_f[i], 336)
    assert xf.shape[-2] * xf.shape[-1] == 2688
