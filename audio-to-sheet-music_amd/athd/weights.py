"""Weight contract for the hot path.

The reference model is `AudioTextHTDemucs` (`ATHTDemucs_v2.py:151-188`) wrapping demucs 4.0.1 `HTDemucs`.
A checkpoint's `model_state_dict` (`test_inference.py:34-35`, `src/train.py:218-224`) holds three key families:

* ``htdemucs.*``  - the frozen HTDemucs; only the encoder side, the 1x1 channel up/down samplers, the
  frequency embedding and the cross-transformer are executed (`ATHTDemucs_v2.py:190-236`). Its own
  ``decoder``/``tdecoder`` are loaded but never run, so they are not part of this contract.
* ``clap.*``      - the frozen CLAP text tower; it is off the per-segment path once prompt embeddings are
  cached (`ATHTDemucs_v2.py:238-248`), so it is not part of this contract either.
* reference-owned trainables: ``text_attn.*``, ``freq_decoder.*``, ``time_decoder.*``, ``freq_out.*``,
  ``time_out.*`` (`ATHTDemucs_v2.py:178-188`).

`hot_path_spec()` lists every key the native path consumes, with its shape.  `synthetic_state_dict()`
builds a seeded, deterministic set of weights of exactly that architecture (there is no network, so no
pretrained checkpoint can be fetched).
"""
from __future__ import annotations

import zlib
from collections import OrderedDict

import numpy as np

# HTDemucs hyper-parameters of the pretrained 'htdemucs' model (AudioTextHTDemucs_Full.txt:4-117,232-345,460-628)
ENC_CH = [48, 96, 192, 384]          # channels=48, growth=2, depth=4
FREQ_IN = 4                          # CaC: 2 audio channels x (re, im)
TIME_IN = 2
DCONV_COMP = 8                       # hidden = C / 8
DCONV_DEPTH = 2
BOTTOM = 512                         # bottom_channels
T_LAYERS = 5
T_HIDDEN = 2048
FREQ_EMB_ROWS = 512
MODEL_DIM = 384                      # config.yaml:15
TEXT_DIM = 512                       # config.yaml:16
DEC_CH = [384, 192, 96, 48, 4]       # ATHTDemucs_v2.py:183-184


def _dconv_keys(prefix: str, c: int):
    h = c // DCONV_COMP
    out = []
    for d in range(DCONV_DEPTH):
        p = f"{prefix}.dconv.layers.{d}"
        out += [
            (f"{p}.0.weight", (h, c, 3), "conv"), (f"{p}.0.bias", (h,), "bias"),
            (f"{p}.1.weight", (h,), "gn_w"), (f"{p}.1.bias", (h,), "gn_b"),
            (f"{p}.3.weight", (2 * c, h, 1), "conv"), (f"{p}.3.bias", (2 * c,), "bias"),
            (f"{p}.4.weight", (2 * c,), "gn_w"), (f"{p}.4.bias", (2 * c,), "gn_b"),
            (f"{p}.6.scale", (c,), "dconv_scale"),
        ]
    return out


def _tlayer_keys(prefix: str, cross: bool):
    a = "cross_attn" if cross else "self_attn"
    d = BOTTOM
    out = [
        (f"{prefix}.{a}.in_proj_weight", (3 * d, d), "lin"), (f"{prefix}.{a}.in_proj_bias", (3 * d,), "bias"),
        (f"{prefix}.{a}.out_proj.weight", (d, d), "lin"), (f"{prefix}.{a}.out_proj.bias", (d,), "bias"),
        (f"{prefix}.linear1.weight", (T_HIDDEN, d), "lin"), (f"{prefix}.linear1.bias", (T_HIDDEN,), "bias"),
        (f"{prefix}.linear2.weight", (d, T_HIDDEN), "lin"), (f"{prefix}.linear2.bias", (d,), "bias"),
        (f"{prefix}.norm1.weight", (d,), "gn_w"), (f"{prefix}.norm1.bias", (d,), "gn_b"),
        (f"{prefix}.norm2.weight", (d,), "gn_w"), (f"{prefix}.norm2.bias", (d,), "gn_b"),
    ]
    if cross:
        out += [(f"{prefix}.norm3.weight", (d,), "gn_w"), (f"{prefix}.norm3.bias", (d,), "gn_b")]
    out += [
        (f"{prefix}.norm_out.weight", (d,), "gn_w"), (f"{prefix}.norm_out.bias", (d,), "gn_b"),
        (f"{prefix}.gamma_1.scale", (d,), "t_scale"), (f"{prefix}.gamma_2.scale", (d,), "t_scale"),
    ]
    return out


def hot_path_spec():
    """[(key, shape, kind)] for every tensor the hot path reads, reference key names."""
    spec = []
    cin_f, cin_t = FREQ_IN, TIME_IN
    for i, c in enumerate(ENC_CH):
        p = f"htdemucs.encoder.{i}"
        spec += [(f"{p}.conv.weight", (c, cin_f, 8, 1), "conv"), (f"{p}.conv.bias", (c,), "bias")]
        spec += _dconv_keys(p, c)
        spec += [(f"{p}.rewrite.weight", (2 * c, c, 1, 1), "conv"), (f"{p}.rewrite.bias", (2 * c,), "bias")]
        p = f"htdemucs.tencoder.{i}"
        spec += [(f"{p}.conv.weight", (c, cin_t, 8), "conv"), (f"{p}.conv.bias", (c,), "bias")]
        spec += _dconv_keys(p, c)
        spec += [(f"{p}.rewrite.weight", (2 * c, c, 1), "conv"), (f"{p}.rewrite.bias", (2 * c,), "bias")]
        cin_f = cin_t = c
    spec += [("htdemucs.freq_emb.embedding.weight", (FREQ_EMB_ROWS, ENC_CH[0]), "freq_emb")]
    for s in ("", "_t"):
        spec += [(f"htdemucs.channel_upsampler{s}.weight", (BOTTOM, ENC_CH[-1], 1), "conv"),
                 (f"htdemucs.channel_upsampler{s}.bias", (BOTTOM,), "bias"),
                 (f"htdemucs.channel_downsampler{s}.weight", (ENC_CH[-1], BOTTOM, 1), "conv"),
                 (f"htdemucs.channel_downsampler{s}.bias", (ENC_CH[-1],), "bias")]
    ct = "htdemucs.crosstransformer"
    spec += [(f"{ct}.norm_in.weight", (BOTTOM,), "gn_w"), (f"{ct}.norm_in.bias", (BOTTOM,), "gn_b"),
             (f"{ct}.norm_in_t.weight", (BOTTOM,), "gn_w"), (f"{ct}.norm_in_t.bias", (BOTTOM,), "gn_b")]
    for idx in range(T_LAYERS):
        cross = idx % 2 == 1      # cross_first=False -> layers 1,3 are cross (AudioTextHTDemucs_Full.txt:471-547)
        spec += _tlayer_keys(f"{ct}.layers.{idx}", cross)
        spec += _tlayer_keys(f"{ct}.layers_t.{idx}", cross)
    # reference-owned trainables (ATHTDemucs_v2.py:21-58, :61-139, :178-188)
    D, TD = MODEL_DIM, TEXT_DIM
    ta = "text_attn"
    spec += [(f"{ta}.q_proj.weight", (D, D), "lin"), (f"{ta}.q_proj.bias", (D,), "bias"),
             (f"{ta}.k_proj.weight", (D, TD), "lin"), (f"{ta}.k_proj.bias", (D,), "bias"),
             (f"{ta}.v_proj.weight", (D, TD), "lin"), (f"{ta}.v_proj.bias", (D,), "bias"),
             (f"{ta}.attn.in_proj_weight", (3 * D, D), "lin"), (f"{ta}.attn.in_proj_bias", (3 * D,), "bias"),
             (f"{ta}.attn.out_proj.weight", (D, D), "lin"), (f"{ta}.attn.out_proj.bias", (D,), "bias"),
             (f"{ta}.out_mlp.0.weight", (D, D), "lin"), (f"{ta}.out_mlp.0.bias", (D,), "bias"),
             (f"{ta}.out_mlp.2.weight", (D, D), "lin"), (f"{ta}.out_mlp.2.bias", (D,), "bias"),
             (f"{ta}.norm_q.weight", (D,), "gn_w"), (f"{ta}.norm_q.bias", (D,), "gn_b"),
             (f"{ta}.norm_out.weight", (D,), "gn_w"), (f"{ta}.norm_out.bias", (D,), "gn_b")]
    for name, kdims in (("freq_decoder", (8, 1)), ("time_decoder", (8,))):
        for i in range(len(DEC_CH) - 1):
            ci, co = DEC_CH[i], DEC_CH[i + 1]
            spec += [(f"{name}.layers.{i}.0.weight", (ci, co) + kdims, "convT"),
                     (f"{name}.layers.{i}.0.bias", (co,), "bias")]
            if i < len(DEC_CH) - 2:
                spec += [(f"{name}.layers.{i}.1.weight", (co,), "gn_w"), (f"{name}.layers.{i}.1.bias", (co,), "gn_b")]
    spec += [("freq_out.weight", (2, 4, 1, 1), "conv"), ("freq_out.bias", (2,), "bias"),
             ("time_out.weight", (2, 4, 1), "conv"), ("time_out.bias", (2,), "bias")]
    return spec


def _fan_in(shape, kind):
    if kind == "convT":          # ConvTranspose weight is (Cin, Cout, k...): PyTorch uses dim 1 * prod(k) as fan_in
        return int(shape[1] * np.prod(shape[2:]))
    return int(np.prod(shape[1:]))


def synthetic_state_dict(seed: int = 0, dtype=np.float32) -> "OrderedDict[str, np.ndarray]":
    """Seeded weights of the hot-path architecture.

    Generator: numpy PCG64 seeded with ``seed`` xor crc32(key) per key, so every tensor is independent of the
    iteration order.  Linear/conv weights ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (the PyTorch default bound),
    biases ~ U(-b, b) with the same bound, GroupNorm/LayerNorm weight 1 + 0.1 N(0,1) and bias 0.1 N(0,1),
    LayerScales U(0.05, 0.3) (larger than demucs' 1e-3/1e-4 inits so the residual branches are exercised by
    parity tests), and the frequency embedding with ScaledEmbedding's smooth init (cumsum of N(0,1) over rows,
    / sqrt(row+1), / scale 10).
    """
    sd = OrderedDict()
    spec = hot_path_spec()
    fan = {}
    for key, shape, kind in spec:
        if kind in ("conv", "convT", "lin"):
            fan[key.rsplit(".", 1)[0]] = _fan_in(shape, kind)
    for key, shape, kind in spec:
        rng = np.random.Generator(np.random.PCG64((seed ^ zlib.crc32(key.encode())) & 0xFFFFFFFF))
        if kind in ("conv", "convT", "lin"):
            b = 1.0 / np.sqrt(_fan_in(shape, kind))
            w = rng.uniform(-b, b, size=shape)
        elif kind == "bias":
            stem = key.rsplit(".", 1)[0]
            if key.endswith("in_proj_bias"):
                stem = key[: -len("in_proj_bias")] + "in_proj"
                b = 1.0 / np.sqrt(shape[0] // 3)
            else:
                b = 1.0 / np.sqrt(fan.get(stem, shape[0]))
            w = rng.uniform(-b, b, size=shape)
        elif kind == "gn_w":
            w = 1.0 + 0.1 * rng.standard_normal(size=shape)
        elif kind == "gn_b":
            w = 0.1 * rng.standard_normal(size=shape)
        elif kind in ("dconv_scale", "t_scale"):
            w = rng.uniform(0.05, 0.3, size=shape)
        elif kind == "freq_emb":
            w = rng.standard_normal(size=shape)
            w = np.cumsum(w, axis=0) / np.sqrt(np.arange(1, shape[0] + 1))[:, None]
            w = w / 10.0
        else:
            raise ValueError(kind)
        sd[key] = np.ascontiguousarray(w.astype(dtype))
    return sd


def synthetic_text_table(n: int = 4, seed: int = 7, dim: int = TEXT_DIM) -> np.ndarray:
    """(n, 512) seeded, L2-normalised prompt embeddings (mimics ClapModel.get_text_features, which
    L2-normalises; CLAP_Text_Model_Fwd_Pass.txt:1)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    t = rng.standard_normal(size=(n, dim))
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    return t.astype(np.float32)


STEMS = ["drums", "bass", "other", "vocals"]          # test_inference.py:18


def weights_checksum(sd) -> float:
    return float(sum(float(np.abs(v).astype(np.float64).sum()) for v in sd.values()))
