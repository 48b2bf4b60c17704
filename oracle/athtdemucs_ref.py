"""ORACLE (test infrastructure only) - CPU restatement of `AudioTextHTDemucs.forward`
(`/root/reference/src/models/stem_separation/ATHTDemucs_v2.py:250-326`), of the reference's metrics
(`src/loss.py:9-68`: SDR, SI-SDR) and of its two chunk loops (`test_inference.py:92-141`; `benchmark.py:155-204`).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

The reference-owned arithmetic (TextCrossAttention `:21-58`, FreqDecoder `:61-104`, TimeDecoder `:107-139`,
the 1x1 output convs `:187-188`, normalisation `:267-275`, masking `:300-309`, branch sum `:324`) is restated
literally here and PINNED against fixtures produced by running the reference module itself
(tests/golden/*, made by oracle/gen_golden.py; checked by tests/test_oracle_golden.py).  The HTDemucs pieces
come from oracle/htdemucs_ref.py (parity with demucs itself unpinned, structure pinned).
"""
from __future__ import annotations

import math
from typing import List

import numpy as np
import torch
import torch.nn.functional as F

from .htdemucs_ref import HTDemucsHot, load_hot


def _t(sd, k):
    return torch.as_tensor(sd[k])


class TextCrossAttentionRef:
    """`ATHTDemucs_v2.py:21-58`: queries attend to ONE text token (text_emb.unsqueeze(1), :40-41)."""

    def __init__(self, sd, prefix="text_attn", n_heads=8):
        self.sd = {k[len(prefix) + 1:]: _t(sd, k) for k in sd if k.startswith(prefix + ".")}
        self.n_heads = n_heads

    def forward_attend(self, queries, text_emb):                               # :38-48
        s = self.sd
        D = queries.shape[-1]
        q = F.layer_norm(queries, (D,), s["norm_q.weight"], s["norm_q.bias"], 1e-5)
        if text_emb.dim() == 2:
            text_emb = text_emb.unsqueeze(1)
        k = F.linear(text_emb, s["k_proj.weight"], s["k_proj.bias"])
        v = F.linear(text_emb, s["v_proj.weight"], s["v_proj.bias"])
        q_proj = F.linear(q, s["q_proj.weight"], s["q_proj.bias"])
        attn_out, _ = F.multi_head_attention_forward(
            q_proj.transpose(0, 1), k.transpose(0, 1), v.transpose(0, 1), D, self.n_heads,
            s["attn.in_proj_weight"], s["attn.in_proj_bias"], None, None, False, 0.0,
            s["attn.out_proj.weight"], s["attn.out_proj.bias"], training=False, need_weights=False)
        out = queries + attn_out.transpose(0, 1)
        h = F.linear(F.gelu(F.linear(out, s["out_mlp.0.weight"], s["out_mlp.0.bias"])),
                     s["out_mlp.2.weight"], s["out_mlp.2.bias"])
        out = out + h
        return F.layer_norm(out, (D,), s["norm_out.weight"], s["norm_out.bias"], 1e-5)

    def __call__(self, x, xt, text_emb):                                     # :50-58
        B, C, Fq, T = x.shape
        x_seq = x.permute(0, 2, 3, 1).reshape(B, Fq * T, C)                     # b c f t -> b (f t) c
        xt_seq = xt.permute(0, 2, 1)
        x_seq = self.forward_attend(x_seq, text_emb)
        xt_seq = self.forward_attend(xt_seq, text_emb)
        x = x_seq.reshape(B, Fq, T, C).permute(0, 3, 1, 2)
        xt = xt_seq.permute(0, 2, 1)
        return x, xt


class _DecoderRef:
    """FreqDecoder (`:61-104`) / TimeDecoder (`:107-139`): ConvT(k8,s4,p2) [+GN(1)+GELU except last]; resize to
    target length; skip truncated to Cout channels, resized, added x0.1."""

    def __init__(self, sd, prefix, freq: bool, channels=(384, 192, 96, 48, 4)):
        self.freq = freq
        self.layers = []
        n = len(channels) - 1
        for i in range(n):
            w = _t(sd, f"{prefix}.layers.{i}.0.weight")
            b = _t(sd, f"{prefix}.layers.{i}.0.bias")
            gn = None
            if i < n - 1:
                gn = (_t(sd, f"{prefix}.layers.{i}.1.weight"), _t(sd, f"{prefix}.layers.{i}.1.bias"))
            self.layers.append((w, b, gn))

    def __call__(self, x, skips: List[torch.Tensor], target_lengths: List[int]):
        for i, (w, b, gn) in enumerate(self.layers):
            if self.freq:
                x = F.conv_transpose2d(x, w, b, stride=(4, 1), padding=(2, 0))
            else:
                x = F.conv_transpose1d(x, w, b, stride=4, padding=2)
            if gn is not None:
                x = F.gelu(F.group_norm(x, 1, gn[0], gn[1], 1e-5))
            if i < len(target_lengths):
                tl = target_lengths[i]
                if x.shape[2] != tl:
                    if self.freq:
                        x = F.interpolate(x, size=(tl, x.shape[3]), mode="bilinear", align_corners=False)
                    else:
                        x = F.interpolate(x, size=tl, mode="linear", align_corners=False)
            if i < len(skips):
                skip = skips[i]
                if skip.shape[1] != x.shape[1]:
                    skip = skip[:, :x.shape[1]]
                if skip.shape[2:] != x.shape[2:]:
                    if self.freq:
                        skip = F.interpolate(skip, size=x.shape[2:], mode="bilinear", align_corners=False)
                    else:
                        skip = F.interpolate(skip, size=x.shape[2], mode="linear", align_corners=False)
                x = x + skip * 0.1
        return x


class AudioTextHTDemucsRef:
    """Restatement of the reference forward with injected text embeddings (the CLAP call `:282` is replaced by a
    table lookup)."""

    def __init__(self, state_dict, htdemucs: HTDemucsHot = None):
        self.sd = state_dict
        self.htdemucs = htdemucs if htdemucs is not None else load_hot(state_dict)
        self.text_attn = TextCrossAttentionRef(state_dict)
        self.freq_decoder = _DecoderRef(state_dict, "freq_decoder", True)
        self.time_decoder = _DecoderRef(state_dict, "time_decoder", False)
        self.freq_out = (_t(state_dict, "freq_out.weight"), _t(state_dict, "freq_out.bias"))
        self.time_out = (_t(state_dict, "time_out.weight"), _t(state_dict, "time_out.bias"))

    # `ATHTDemucs_v2.py:190-236`
    def encode(self, x, xt):
        h = self.htdemucs
        saved, saved_t, lengths, lengths_t = [], [], [], []
        for idx, encode in enumerate(h.encoder):
            lengths.append(x.shape[-1])
            lengths_t.append(xt.shape[-1])
            xt = h.tencoder[idx](xt)
            saved_t.append(xt)
            x = encode(x, None)
            if idx == 0:
                frs = torch.arange(x.shape[-2])
                emb = h.freq_emb(frs).t()[None, :, :, None].expand_as(x)
                x = x + h.freq_emb_scale * emb
            saved.append(x)
        b, c, f, t = x.shape
        x = h.channel_upsampler(x.reshape(b, c, f * t)).reshape(b, -1, f, t)
        xt = h.channel_upsampler_t(xt)
        x, xt = h.crosstransformer(x, xt)
        x = h.channel_downsampler(x.reshape(b, -1, f * t)).reshape(b, -1, f, t)
        xt = h.channel_downsampler_t(xt)
        return x, xt, saved, saved_t, lengths, lengths_t

    def prepare(self, wav):
        """STFT, CaC and the two per-sample normalisations (`:261-275`)."""
        z = self.htdemucs._spec(wav)
        mag = self.htdemucs._magnitude(z)
        mean = mag.mean(dim=(1, 2, 3), keepdim=True)
        std = mag.std(dim=(1, 2, 3), keepdim=True)
        x = (mag - mean) / (1e-5 + std)
        meant = wav.mean(dim=(1, 2), keepdim=True)
        stdt = wav.std(dim=(1, 2), keepdim=True)
        xt = (wav - meant) / (1e-5 + stdt)
        return z, mag, x, xt, meant, stdt

    def decode(self, z, mag, enc, text_emb, meant, stdt, original_length, capture=None):
        """Per-prompt half of the forward (`:282-324`)."""
        x_enc, xt_enc, saved, saved_t, lengths, lengths_t = enc
        Fq, T_spec = mag.shape[2], mag.shape[3]
        x_cond, xt_cond = self.text_attn(x_enc, xt_enc, text_emb)
        x_dec = self.freq_decoder(x_cond, saved[::-1], lengths[::-1])
        if capture is not None:
            capture["x_fdec"] = x_dec        # FreqDecoder output, before freq_out (`:293`)
        x_dec = F.conv2d(x_dec, *self.freq_out)
        if capture is not None:
            capture["x_fo"] = x_dec
        x_dec = F.interpolate(x_dec, size=(Fq, T_spec), mode="bilinear", align_corners=False)
        mask = torch.sigmoid(x_dec)
        mag_stereo = mag[:, :2]
        masked_spec = mag_stereo * mask
        phase = z[:, :2] / (mag_stereo + 1e-8)
        masked_z = masked_spec * phase
        freq_wav = self.htdemucs._ispec(masked_z, original_length)
        xt_dec = self.time_decoder(xt_cond, saved_t[::-1], lengths_t[::-1])
        if capture is not None:
            capture["xt_dec3"] = xt_dec
        xt_dec = F.conv1d(xt_dec, *self.time_out)
        if xt_dec.shape[-1] != original_length:
            xt_dec = F.interpolate(xt_dec, size=original_length, mode="linear", align_corners=False)
        if capture is not None:
            capture["xt_out"] = xt_dec
        xt_dec = xt_dec * stdt + meant
        if capture is not None:
            capture.update(x_cond=x_cond, xt_cond=xt_cond, mask=mask, freq_wav=freq_wav, xt_dec=xt_dec)
        return freq_wav + xt_dec

    @torch.no_grad()
    def forward(self, wav: torch.Tensor, text_emb: torch.Tensor, capture=None):
        """wav (B,2,T) f32, text_emb (B,512) f32 -> (B,2,T) f32."""
        z, mag, x, xt, meant, stdt = self.prepare(wav)
        enc = self.encode(x, xt)
        if capture is not None:
            capture.update(z=z, x_norm=x, xt_norm=xt, x_enc=enc[0], xt_enc=enc[1],
                           saved=list(enc[2]), saved_t=list(enc[3]))
        return self.decode(z, mag, enc, text_emb, meant, stdt, wav.shape[-1], capture)

    @torch.no_grad()
    def forward_prompts(self, wav: torch.Tensor, text_table: torch.Tensor):
        """Encode once, decode once per prompt row: (B,2,T) x (P,512) -> (B,P,2,T).  Equal to P calls of
        `forward` because the encoder does not see the prompt (`:278-283`)."""
        z, mag, x, xt, meant, stdt = self.prepare(wav)
        enc = self.encode(x, xt)
        B, P = wav.shape[0], text_table.shape[0]
        outs = []
        for p in range(P):
            te = text_table[p:p + 1].expand(B, -1)
            outs.append(self.decode(z, mag, enc, te, meant, stdt, wav.shape[-1]))
        return torch.stack(outs, dim=1)


# ------------------------------------------------------------------------------------------------------------
# Metric and chunk loop
# ------------------------------------------------------------------------------------------------------------
def sdr_db(estimated: torch.Tensor, target: torch.Tensor) -> float:
    """`src/loss.py:9-30` with the sign flipped: mean over rows of clamp(10 log10((|s|^2+d)/(|s-e|^2+d)), +-30)."""
    est = estimated.reshape(estimated.shape[0], -1).double()
    tgt = target.reshape(target.shape[0], -1).double()
    num = (tgt ** 2).sum(-1)
    den = ((tgt - est) ** 2).sum(-1)
    sdr = 10 * torch.log10((num + 1e-8) / (den + 1e-8))
    return float(sdr.clamp(-30, 30).mean())


def chunk_plan(length: int, sample_rate: int = 44100, segment_seconds: float = 6.0, overlap: float = 0.1):
    """Windows of `test_inference.py:92-141`: [(start, end, fade_in, fade_out)]."""
    chunk_len = int(sample_rate * segment_seconds)
    overlap_frames = int(overlap * sample_rate)
    out = []
    start = 0
    while start < length:
        end = min(start + chunk_len, length)
        out.append((start, end, 0 if start == 0 else overlap_frames, overlap_frames if end < length else 0))
        start += chunk_len - overlap_frames
    return out


def linear_fade(x: torch.Tensor, fade_in: int, fade_out: int) -> torch.Tensor:
    """torchaudio.transforms.Fade(fade_shape='linear') on the last axis (`test_inference.py:126-132`).
    torchaudio is not installed; its published formula is restated: fade_in = cat(linspace(0,1,n_in), ones),
    fade_out = cat(ones, 1 - linspace(0,1,n_out)), both clamped to [0,1]; result = fade_in * fade_out * x."""
    L = x.shape[-1]
    fi = torch.cat((torch.linspace(0, 1, fade_in, dtype=x.dtype), torch.ones(L - fade_in, dtype=x.dtype))).clamp_(0, 1)
    fo = torch.cat((torch.ones(L - fade_out, dtype=x.dtype), -torch.linspace(0, 1, fade_out, dtype=x.dtype) + 1)).clamp_(0, 1)
    return fi * fo * x


def sisdr_db(estimated: torch.Tensor, target: torch.Tensor) -> float:
    """`src/loss.py:33-68` with the sign flipped (benchmark.py:573-588), literally in fp32 torch ops."""
    est_flat = estimated.reshape(estimated.shape[0], -1).float()
    tgt_flat = target.reshape(target.shape[0], -1).float()
    est_flat = est_flat - est_flat.mean(dim=-1, keepdim=True)
    tgt_flat = tgt_flat - tgt_flat.mean(dim=-1, keepdim=True)
    dot = torch.sum(est_flat * tgt_flat, dim=-1, keepdim=True)
    s_target_norm_sq = torch.sum(tgt_flat ** 2, dim=-1, keepdim=True)
    s_target = (dot / (s_target_norm_sq + 1e-8)) * tgt_flat
    e_noise = est_flat - s_target
    sisdr = 10 * torch.log10((torch.sum(s_target ** 2, dim=-1) + 1e-8) / (torch.sum(e_noise ** 2, dim=-1) + 1e-8))
    return float(torch.clamp(sisdr, min=-30, max=30).mean())


def benchmark_chunked_inference(model_fn, mixture: torch.Tensor, sample_rate: int = 44100,
                                segment_seconds: float = 6.0, overlap: float = 1.5) -> torch.Tensor:
    """`benchmark.py:155-204` (OurModel._chunked_inference) restated: model_fn((1, C, chunk_len)) -> (1, C, chunk_len).
    Windows of chunk_len every chunk_len - overlap_frames samples; the last one zero-padded to chunk_len; linspace
    fades of min(overlap_frames, len // 2) samples; weighted overlap-add normalised by the summed weights."""
    C, T = mixture.shape
    chunk_len = int(sample_rate * segment_seconds)
    overlap_frames = int(overlap * sample_rate)
    output = torch.zeros(C, T)
    weight = torch.zeros(T)
    start = 0
    while start < T:
        end = min(start + chunk_len, T)
        chunk = mixture[:, start:end].unsqueeze(0)
        if chunk.shape[-1] < chunk_len:
            chunk = F.pad(chunk, (0, chunk_len - chunk.shape[-1]))
        out = model_fn(chunk).squeeze(0)
        actual_len = end - start
        out = out[:, :actual_len]
        fade_len = min(overlap_frames, actual_len // 2)
        chunk_weight = torch.ones(actual_len)
        if start > 0 and fade_len > 0:
            chunk_weight[:fade_len] = torch.linspace(0, 1, fade_len)
        if end < T and fade_len > 0:
            chunk_weight[-fade_len:] = torch.linspace(1, 0, fade_len)
        output[:, start:end] += out * chunk_weight
        weight[start:end] += chunk_weight
        start += chunk_len - overlap_frames
    weight = weight.clamp(min=1e-8)
    return output / weight
