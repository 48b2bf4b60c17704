"""ORACLE (test infrastructure only) - CPU restatement of the demucs==4.0.1 HTDemucs pieces on the hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the product
path (audio-to-sheet-music_amd/) never does.

demucs 4.0.1 (`requirements.txt:1`) is NOT installed in this image and its source is not under
/root/reference, so this file restates its published algorithm from scratch.  Module
and parameter names follow demucs so that reference checkpoint keys (``htdemucs.*``) load unchanged.
Call sites in the reference: `src/models/stem_separation/ATHTDemucs_v2.py:197-236` (encoders, freq emb,
up/down samplers, cross-transformer), `:261-262` (`_spec`, `_magnitude`), `:310` (`_ispec`).

Parity of this file against demucs itself is UNPINNED (no demucs source, tests or fixtures exist offline).
What pins it: the structural dumps in the reference (per-layer parameter counts and output shapes in
`HTDemucs_Fwd_Pass.txt:4-150` and module hyper-parameters/eps in `AudioTextHTDemucs_Full.txt`), checked by
tests/test_oracle_structure.py.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


# ---------------------------------------------------------------------------------------------------------
# demucs.spec / HTDemucs._spec / _ispec / _magnitude  (call sites ATHTDemucs_v2.py:261-262,310)
# ---------------------------------------------------------------------------------------------------------
def pad1d(x: torch.Tensor, paddings, mode: str = "constant", value: float = 0.0):
    """demucs.hdemucs.pad1d: reflect padding that tolerates inputs shorter than the pad by first zero-extending
    on the right (then left) so that the reflection is defined."""
    length = x.shape[-1]
    padding_left, padding_right = paddings
    if mode == "reflect":
        max_pad = max(padding_left, padding_right)
        if length <= max_pad:
            extra_pad = max_pad - length + 1
            extra_pad_right = min(padding_right, extra_pad)
            extra_pad_left = extra_pad - extra_pad_right
            paddings = (padding_left - extra_pad_left, padding_right - extra_pad_right)
            x = F.pad(x, (extra_pad_left, extra_pad_right))
    out = F.pad(x, paddings, mode, value)
    assert out.shape[-1] == length + padding_left + padding_right
    return out


def spectro(x, n_fft=512, hop_length=None):
    *other, length = x.shape
    x = x.reshape(-1, length)
    z = torch.stft(x, n_fft, hop_length or n_fft // 4, window=torch.hann_window(n_fft).to(x),
                   win_length=n_fft, normalized=True, center=True, return_complex=True, pad_mode="reflect")
    _, freqs, frame = z.shape
    return z.view(*other, freqs, frame)


def ispectro(z, hop_length=None, length=None):
    *other, freqs, frames = z.shape
    n_fft = 2 * freqs - 2
    z = z.view(-1, freqs, frames)
    x = torch.istft(z, n_fft, hop_length, window=torch.hann_window(n_fft).to(z.real), win_length=n_fft,
                    normalized=True, length=length, center=True)
    _, length = x.shape
    return x.view(*other, length)


# ---------------------------------------------------------------------------------------------------------
# Encoder layers (demucs.hdemucs.HEncLayer, demucs.demucs.DConv / LayerScale, hdemucs.ScaledEmbedding)
# ---------------------------------------------------------------------------------------------------------
class LayerScale(nn.Module):
    """Per-channel rescale of a residual branch; `channel_last` selects (.., C) vs (C, T) broadcasting."""

    def __init__(self, channels: int, init: float = 0.0, channel_last: bool = False):
        super().__init__()
        self.channel_last = channel_last
        self.scale = nn.Parameter(torch.full((channels,), float(init)))

    def forward(self, x):
        if self.channel_last:
            return self.scale * x
        return self.scale[:, None] * x


class DConv(nn.Module):
    """Residual dilated 1-D conv stack: for d in 0..depth-1, x = x + LS(GLU(GN(conv1x1(GELU(GN(conv3_d(x)))))))."""

    def __init__(self, channels: int, compress: float = 8, depth: int = 2, init: float = 1e-3):
        super().__init__()
        hidden = int(channels / compress)
        self.layers = nn.ModuleList()
        for d in range(depth):
            dilation = 2 ** d
            self.layers.append(nn.Sequential(
                nn.Conv1d(channels, hidden, 3, dilation=dilation, padding=dilation),
                nn.GroupNorm(1, hidden), nn.GELU(),
                nn.Conv1d(hidden, 2 * channels, 1),
                nn.GroupNorm(1, 2 * channels), nn.GLU(1),
                LayerScale(channels, init)))

    def forward(self, x):
        for layer in self.layers:
            x = x + layer(x)
        return x


class HEncLayer(nn.Module):
    """One encoder level: conv (kernel 8 stride 4 pad 2, along freq for the spectral branch) -> GELU -> DConv
    (run along time; for the freq branch on (B*Fr, C, T)) -> 1x1 rewrite -> GLU.  norm1/norm2 are Identity for
    the pretrained model (norm_starts=4, AudioTextHTDemucs_Full.txt:7,9)."""

    def __init__(self, chin, chout, freq=True, kernel_size=8, stride=4):
        super().__init__()
        self.freq = freq
        self.stride = stride
        self.empty = False
        pad = kernel_size // 4
        if freq:
            self.conv = nn.Conv2d(chin, chout, (kernel_size, 1), (stride, 1), (pad, 0))
            self.rewrite = nn.Conv2d(chout, 2 * chout, 1)
        else:
            self.conv = nn.Conv1d(chin, chout, kernel_size, stride, pad)
            self.rewrite = nn.Conv1d(chout, 2 * chout, 1)
        self.norm1 = nn.Identity()
        self.norm2 = nn.Identity()
        self.dconv = DConv(chout)

    def forward(self, x, inject=None):
        if not self.freq:
            le = x.shape[-1]
            if le % self.stride != 0:          # right zero-pad to a multiple of the stride (85995->21499->...)
                x = F.pad(x, (0, self.stride - (le % self.stride)))
        y = self.conv(x)
        if inject is not None:
            y = y + inject
        y = F.gelu(self.norm1(y))
        if self.freq:
            B, C, Fr, T = y.shape
            y = y.permute(0, 2, 1, 3).reshape(-1, C, T)
        y = self.dconv(y)
        if self.freq:
            y = y.view(B, Fr, C, T).permute(0, 2, 1, 3)
        z = self.norm2(self.rewrite(y))
        return F.glu(z, dim=1)


class ScaledEmbedding(nn.Module):
    def __init__(self, num_embeddings, embedding_dim, scale=10.0):
        super().__init__()
        self.embedding = nn.Embedding(num_embeddings, embedding_dim)
        self.scale = scale

    def forward(self, x):
        return self.embedding(x) * self.scale


# ---------------------------------------------------------------------------------------------------------
# Cross-domain transformer (demucs.transformer)
# ---------------------------------------------------------------------------------------------------------
def create_sin_embedding(length: int, dim: int, shift: int = 0, max_period: float = 10000):
    pos = shift + torch.arange(length).view(-1, 1, 1)
    half_dim = dim // 2
    adim = torch.arange(dim // 2).view(1, 1, -1)
    phase = pos / (max_period ** (adim / (half_dim - 1)))
    return torch.cat([torch.cos(phase), torch.sin(phase)], dim=-1)      # (T, 1, C)


def create_2d_sin_embedding(d_model, height, width, max_period=10000):
    pe = torch.zeros(d_model, height, width)
    d_model = int(d_model / 2)
    div_term = torch.exp(torch.arange(0.0, d_model, 2) * -(math.log(max_period) / d_model))
    pos_w = torch.arange(0.0, width).unsqueeze(1)
    pos_h = torch.arange(0.0, height).unsqueeze(1)
    pe[0:d_model:2, :, :] = torch.sin(pos_w * div_term).transpose(0, 1).unsqueeze(1).repeat(1, height, 1)
    pe[1:d_model:2, :, :] = torch.cos(pos_w * div_term).transpose(0, 1).unsqueeze(1).repeat(1, height, 1)
    pe[d_model::2, :, :] = torch.sin(pos_h * div_term).transpose(0, 1).unsqueeze(2).repeat(1, 1, width)
    pe[d_model + 1::2, :, :] = torch.cos(pos_h * div_term).transpose(0, 1).unsqueeze(2).repeat(1, 1, width)
    return pe[None, :]                                                    # (1, C, H, W)


class MyGroupNorm(nn.GroupNorm):
    """GroupNorm over (tokens, channels) of a (B, T, C) tensor: one group => per-sample statistics over T*C."""

    def forward(self, x):
        return super().forward(x.transpose(1, 2)).transpose(1, 2)


class MyTransformerEncoderLayer(nn.Module):
    """norm_first self-attention layer with LayerScale and a GroupNorm(1) output norm (eval: no dropout)."""

    def __init__(self, d_model=512, nhead=8, dim_feedforward=2048, init_values=1e-4):
        super().__init__()
        self.self_attn = nn.MultiheadAttention(d_model, nhead, batch_first=True)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.norm_out = MyGroupNorm(1, d_model)
        self.gamma_1 = LayerScale(d_model, init_values, True)
        self.gamma_2 = LayerScale(d_model, init_values, True)

    def forward(self, x):
        h = self.norm1(x)
        x = x + self.gamma_1(self.self_attn(h, h, h, need_weights=False)[0])
        x = x + self.gamma_2(self.linear2(F.gelu(self.linear1(self.norm2(x)))))
        return self.norm_out(x)


class CrossTransformerEncoderLayer(nn.Module):
    def __init__(self, d_model=512, nhead=8, dim_feedforward=2048, init_values=1e-4):
        super().__init__()
        self.cross_attn = nn.MultiheadAttention(d_model, nhead, batch_first=True)
        self.linear1 = nn.Linear(d_model, dim_feedforward)
        self.linear2 = nn.Linear(dim_feedforward, d_model)
        self.norm1 = nn.LayerNorm(d_model)
        self.norm2 = nn.LayerNorm(d_model)
        self.norm3 = nn.LayerNorm(d_model)
        self.norm_out = MyGroupNorm(1, d_model)
        self.gamma_1 = LayerScale(d_model, init_values, True)
        self.gamma_2 = LayerScale(d_model, init_values, True)

    def forward(self, q, k):
        kk = self.norm2(k)
        x = q + self.gamma_1(self.cross_attn(self.norm1(q), kk, kk, need_weights=False)[0])
        x = x + self.gamma_2(self.linear2(F.gelu(self.linear1(self.norm3(x)))))
        return self.norm_out(x)


class CrossTransformerEncoder(nn.Module):
    """5 layers x {freq, time}; even layers self-attention, odd layers cross-attention (cross_first=False).
    Freq tokens are ordered (t1 fr), time tokens t2; sinusoidal 2-D / 1-D position embeddings (weight 1.0)."""

    def __init__(self, dim=512, num_layers=5, max_period=10000.0):
        super().__init__()
        self.max_period = max_period
        self.num_layers = num_layers
        self.norm_in = nn.LayerNorm(dim)
        self.norm_in_t = nn.LayerNorm(dim)
        self.layers = nn.ModuleList()
        self.layers_t = nn.ModuleList()
        for idx in range(num_layers):
            if idx % 2 == 0:
                self.layers.append(MyTransformerEncoderLayer(dim))
                self.layers_t.append(MyTransformerEncoderLayer(dim))
            else:
                self.layers.append(CrossTransformerEncoderLayer(dim))
                self.layers_t.append(CrossTransformerEncoderLayer(dim))

    def forward(self, x, xt):
        B, C, Fr, T1 = x.shape
        pos_emb_2d = create_2d_sin_embedding(C, Fr, T1, self.max_period)
        pos_emb_2d = pos_emb_2d.permute(0, 3, 2, 1).reshape(1, T1 * Fr, C)        # b c fr t1 -> b (t1 fr) c
        x = x.permute(0, 3, 2, 1).reshape(B, T1 * Fr, C)
        x = self.norm_in(x) + pos_emb_2d
        B, C, T2 = xt.shape
        xt = xt.permute(0, 2, 1)
        pos_emb = create_sin_embedding(T2, C, 0, self.max_period).permute(1, 0, 2)  # t2 b c -> b t2 c
        xt = self.norm_in_t(xt) + pos_emb
        for idx in range(self.num_layers):
            if idx % 2 == 0:
                x = self.layers[idx](x)
                xt = self.layers_t[idx](xt)
            else:
                old_x = x
                x = self.layers[idx](x, xt)
                xt = self.layers_t[idx](xt, old_x)
        x = x.reshape(B, T1, Fr, C).permute(0, 3, 2, 1)
        xt = xt.permute(0, 2, 1)
        return x, xt


# ---------------------------------------------------------------------------------------------------------
# The HTDemucs stand-in: the encoder half the reference executes (ATHTDemucs_v2.py:190-236) + spec helpers.
# ---------------------------------------------------------------------------------------------------------
class HTDemucsHot(nn.Module):
    """Hot-path subset of the pretrained 'htdemucs' (channels 48, depth 4, nfft 4096, cac, bottom 512).

    With ``with_unused_decoder`` the never-executed decoder/tdecoder parameter holders are also created so
    the total parameter count can be checked against the reference dump (HTDemucs_Fwd_Pass.txt:147)."""

    def __init__(self, with_unused_decoder: bool = False):
        super().__init__()
        self.nfft = 4096
        self.hop_length = 1024
        self.cac = True
        self.freq_emb_scale = 0.2
        self.bottom_channels = 512
        chs = [48, 96, 192, 384]
        self.encoder = nn.ModuleList()
        self.tencoder = nn.ModuleList()
        cin_f, cin_t = 4, 2
        for c in chs:
            self.encoder.append(HEncLayer(cin_f, c, freq=True))
            self.tencoder.append(HEncLayer(cin_t, c, freq=False))
            cin_f = cin_t = c
        self.freq_emb = ScaledEmbedding(512, chs[0], scale=10.0)
        self.channel_upsampler = nn.Conv1d(384, 512, 1)
        self.channel_downsampler = nn.Conv1d(512, 384, 1)
        self.channel_upsampler_t = nn.Conv1d(384, 512, 1)
        self.channel_downsampler_t = nn.Conv1d(512, 384, 1)
        self.crosstransformer = CrossTransformerEncoder(512, 5)
        if with_unused_decoder:
            self.decoder = nn.ModuleList()
            self.tdecoder = nn.ModuleList()
            for chin, cf, ct in ((384, 192, 192), (192, 96, 96), (96, 48, 48), (48, 16, 8)):
                dec = nn.Module()
                dec.conv_tr = nn.ConvTranspose2d(chin, cf, (8, 1), (4, 1))
                dec.rewrite = nn.Conv2d(chin, 2 * chin, 3, 1, 1)
                dec.dconv = DConv(chin)
                self.decoder.append(dec)
                tdec = nn.Module()
                tdec.conv_tr = nn.ConvTranspose1d(chin, ct, 8, 4)
                tdec.rewrite = nn.Conv1d(chin, 2 * chin, 3, 1, 1)
                tdec.dconv = DConv(chin)
                self.tdecoder.append(tdec)

    def _spec(self, x):
        hl = self.hop_length
        le = int(math.ceil(x.shape[-1] / hl))
        pad = hl // 2 * 3
        x = pad1d(x, (pad, pad + le * hl - x.shape[-1]), mode="reflect")
        z = spectro(x, self.nfft, hl)[..., :-1, :]
        assert z.shape[-1] == le + 4, (z.shape, x.shape, le)
        return z[..., 2: 2 + le]

    def _ispec(self, z, length=None):
        hl = self.hop_length
        z = F.pad(z, (0, 0, 0, 1))
        z = F.pad(z, (2, 2))
        pad = hl // 2 * 3
        le = hl * int(math.ceil(length / hl)) + 2 * pad
        x = ispectro(z, hl, length=le)
        return x[..., pad: pad + length]

    def _magnitude(self, z):
        B, C, Fr, T = z.shape
        m = torch.view_as_real(z).permute(0, 1, 4, 2, 3)
        return m.reshape(B, C * 2, Fr, T)


def load_hot(state_dict, with_unused_decoder=False) -> HTDemucsHot:
    """Build the stand-in and load the ``htdemucs.*`` keys of a (numpy or torch) state dict."""
    m = HTDemucsHot(with_unused_decoder)
    sd = {k[len("htdemucs."):]: torch.as_tensor(v) for k, v in state_dict.items() if k.startswith("htdemucs.")}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not (k.startswith("decoder.") or k.startswith("tdecoder."))]
    assert not missing and not unexpected, (missing, unexpected)
    return m.eval()
