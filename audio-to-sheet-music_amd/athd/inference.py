"""Track-level surface of the reference around the hot path.

Mirrors `test_inference.py`:
  * `load_model`       <- `test_inference.py:21-40`
  * `window_plan`      <- the window arithmetic of `test_inference.py:96-141`
  * `separate_track`   <- the per-stem chunk loop `test_inference.py:92-141`, batched: all full windows of the track
                          go through `forward_prompts` (encode once, decode once per stem), the fades and the
                          additive overlap-add run in `athd_overlap_add` (same fp32 additions, same order)
  * `sdr_loss`         <- `src/loss.py:9-30` (device reduction, fp64 sums); `test_inference.py:153` uses -sdr_loss
  * `separate_and_score` <- `test_inference.py:91-155` on an in-memory track
  * `test_inference`   <- `test_inference.py:43-205` (same signature and defaults: checkpoint, first track of
                          data_dir, per-stem SDR dict, extracted_{stem}.wav + mixture.wav; no plots)
  * `load_config`, `main` <- `utils.py:18-23`, `test_inference.py:208-218`
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import native
from .model import AudioTextHTDemucs
from .text import load_clap
from .weights import STEMS


def load_model(checkpoint_path: str, device: str = "cuda", dtype: str = "bf16",
               text_table: Optional[Dict[str, np.ndarray]] = None, clap=None, tokenizer=None) -> AudioTextHTDemucs:
    """`test_inference.py:21-40`.  The checkpoint is read with `torch.load(weights_only=True)` (no unpickling of
    code); `checkpoint["model_state_dict"]` is loaded non-strictly.  The pretrained htdemucs object of the reference
    is not needed: every `htdemucs.*` key the hot path uses is in the checkpoint, as the reference's own
    `load_state_dict` overwrites the pretrained values with them.  Prompt embeddings: `text_table` or `clap`/`tokenizer`
    (see athd/text.py).  With neither given, CLAP and its tokenizer are built from `laion/clap-htsat-unfused` in the
    local Hugging Face cache as the reference does (`:26-28`, `text.load_clap`, `local_files_only=True`), the
    checkpoint's `clap.*` keys are loaded into it (`:34-35`), and the embeddings of the 4 stem prompts are computed
    once and cached (the CLAP tower is frozen: its output depends on the prompt string only)."""
    if text_table is None and (clap is None) != (tokenizer is None):
        # the reference builds the two together (`:26-28`); a lone tokenizer must not be silently replaced by the
        # cached one, nor a lone model be left without one
        raise ValueError("load_model: pass both clap= and tokenizer=, or neither (then both come from the local "
                         "Hugging Face cache), or text_table=")
    default_clap = text_table is None and clap is None
    if default_clap:
        clap, tokenizer = load_clap()
    ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    sd = ckpt["model_state_dict"] if isinstance(ckpt, dict) and "model_state_dict" in ckpt else ckpt
    model = AudioTextHTDemucs(None, clap, tokenizer, dtype=dtype, text_table=text_table)
    model.load_state_dict(sd, strict=False)
    if default_clap:
        model.embedder.rows(list(STEMS), len(STEMS))     # the 4 stem embeddings, cached in the prompt table
    model = model.to(device)
    model.eval()
    return model


@dataclass(frozen=True)
class Window:
    start: int
    end: int
    fade_in: int
    fade_out: int


def window_plan(length: int, sample_rate: int = 44100, segment_seconds: float = 6.0,
                overlap: float = 0.1) -> List[Window]:
    """Windows of `test_inference.py:96-141` in loop order.  Raises like the reference when a window is shorter
    than its fade (torchaudio's Fade then asks for a negative-size `torch.ones`)."""
    chunk_len = int(sample_rate * segment_seconds)
    overlap_frames = int(overlap * sample_rate)
    if chunk_len <= overlap_frames:
        raise ValueError("segment must be longer than the overlap")
    plan = []
    start = 0
    while start < length:
        end = min(start + chunk_len, length)
        fade_in = 0 if start == 0 else overlap_frames
        fade_out = overlap_frames if end < length else 0
        if end - start < max(fade_in, fade_out):
            raise RuntimeError(f"window [{start}, {end}) is shorter than its fade ({max(fade_in, fade_out)} samples):"
                               f" the reference's torchaudio Fade fails here (negative dimension)")
        plan.append(Window(start, end, fade_in, fade_out))
        start += chunk_len - overlap_frames
    n_native = native.lib.athd_num_windows(length, chunk_len, overlap_frames)
    if n_native != len(plan):
        raise AssertionError(f"window count mismatch: host {len(plan)}, library {n_native}")
    return plan


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def overlap_add(windows: torch.Tensor, length: int, chunk_len: int, overlap_frames: int, k0: int = 0,
                k1: Optional[int] = None) -> torch.Tensor:
    """Fade + additive overlap-add of window outputs `windows` (k1-k0, S, 2, chunk_len) into the track span of
    windows [k0, k1) (the whole track by default) -> (S, 2, span) on the same device (athd_overlap_add)."""
    n = native.lib.athd_num_windows(length, chunk_len, overlap_frames)
    k1 = n if k1 is None else k1
    S = windows.shape[1]
    if windows.dim() != 4 or windows.shape[0] != k1 - k0 or windows.shape[2] != 2 or windows.shape[3] != chunk_len:
        raise ValueError(f"windows must be ({k1 - k0}, S, 2, {chunk_len}), got {tuple(windows.shape)}")
    if windows.dtype != torch.float32 or not windows.is_contiguous() or windows.device.type != "cuda":
        raise ValueError("windows must be a contiguous float32 device tensor")
    hop = chunk_len - overlap_frames
    span = min((k1 - 1) * hop + chunk_len, length) - k0 * hop
    out = torch.empty((S, 2, span), dtype=torch.float32, device=windows.device)
    rc = native.lib.athd_overlap_add(windows.data_ptr(), length, chunk_len, overlap_frames, S, k0, k1, out.data_ptr(),
                                     _stream(windows.device))
    if rc != 0:
        raise native.AthdError(f"athd_overlap_add failed ({rc})")
    return out


@torch.no_grad()
def run_windows(model: AudioTextHTDemucs, mixture: torch.Tensor, plan: Sequence[Window], stems: Sequence[str],
                chunk_len: int, k0: int = 0, k1: Optional[int] = None, max_batch: int = 64) -> torch.Tensor:
    """Model outputs of windows [k0, k1) of `plan` for every stem -> (k1-k0, S, 2, chunk_len); full windows are
    batched `max_batch` at a time (encode once, decode once per stem), a short last window runs on its own."""
    k1 = len(plan) if k1 is None else k1
    dev = mixture.device
    S = len(stems)
    win = torch.zeros((k1 - k0, S, 2, chunk_len), dtype=torch.float32, device=dev)
    full = [k for k in range(k0, k1) if plan[k].end - plan[k].start == chunk_len]
    if full and full != list(range(k0, k0 + len(full))):
        raise AssertionError("full windows must form a prefix of the plan")
    for b0 in range(0, len(full), max_batch):
        ks = full[b0:b0 + max_batch]
        batch = torch.stack([mixture[:, plan[k].start:plan[k].end] for k in ks]).contiguous()
        model.forward_prompts(batch, list(stems), out=win[ks[0] - k0:ks[-1] - k0 + 1])
    for k in range(k0 + len(full), k1):
        w = plan[k]
        o = model.forward_prompts(mixture[:, w.start:w.end].unsqueeze(0).contiguous(), list(stems))
        win[k - k0, :, :, :w.end - w.start] = o[0]
    return win


@torch.no_grad()
def separate_track(model: AudioTextHTDemucs, mixture: torch.Tensor, stems: Sequence[str] = STEMS,
                   sample_rate: int = 44100, segment_seconds: float = 6.0, overlap: float = 0.1,
                   max_batch: int = 64) -> torch.Tensor:
    """`test_inference.py:91-141`: mixture (2, L) (or (1, 2, L)) on the model's device -> final (S, 2, L)."""
    if mixture.dim() == 3:
        mixture = mixture[0]
    if mixture.dim() != 2 or mixture.shape[0] != 2:
        raise ValueError(f"expected a (2, L) stereo mixture, got {tuple(mixture.shape)}")
    mixture = mixture.float().contiguous()
    length = mixture.shape[-1]
    chunk_len = int(sample_rate * segment_seconds)
    overlap_frames = int(overlap * sample_rate)
    plan = window_plan(length, sample_rate, segment_seconds, overlap)
    win = run_windows(model, mixture, plan, stems, chunk_len, max_batch=max_batch)
    return overlap_add(win, length, chunk_len, overlap_frames)


def sdr_loss(estimated: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """`src/loss.py:9-30`: -mean over rows (dim 0) of clamp(10 log10((|t|^2 + 1e-8) / (|t - e|^2 + 1e-8)), -30, 30);
    a device scalar.  Sums are accumulated in fp64 on the device (athd_sdr)."""
    if estimated.shape[0] != target.shape[0] or estimated.numel() != target.numel():
        raise ValueError("estimated and target must have the same rows and size")
    rows = estimated.shape[0]
    est = estimated.reshape(rows, -1).float().contiguous()
    tgt = target.reshape(rows, -1).float().contiguous()
    scratch = torch.empty(2 * rows, dtype=torch.float64, device=est.device)
    out = torch.empty(1, dtype=torch.float32, device=est.device)
    rc = native.lib.athd_sdr(est.data_ptr(), tgt.data_ptr(), rows, est.shape[1], scratch.data_ptr(), out.data_ptr(),
                             _stream(est.device))
    if rc != 0:
        raise native.AthdError(f"athd_sdr failed ({rc})")
    return -out[0]


def sisdr_loss(estimated: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """`src/loss.py:33-68`: -mean over rows of the clamped SI-SDR of the zero-meaned rows; a device scalar (fp64
    sums on the device, athd_sisdr)."""
    if estimated.shape[0] != target.shape[0] or estimated.numel() != target.numel():
        raise ValueError("estimated and target must have the same rows and size")
    rows = estimated.shape[0]
    est = estimated.reshape(rows, -1).float().contiguous()
    tgt = target.reshape(rows, -1).float().contiguous()
    scratch = torch.empty(5 * rows, dtype=torch.float64, device=est.device)
    out = torch.empty(1, dtype=torch.float32, device=est.device)
    rc = native.lib.athd_sisdr(est.data_ptr(), tgt.data_ptr(), rows, est.shape[1], scratch.data_ptr(),
                               out.data_ptr(), _stream(est.device))
    if rc != 0:
        raise native.AthdError(f"athd_sisdr failed ({rc})")
    return -out[0]


@torch.no_grad()
def separate_and_score(model: AudioTextHTDemucs, mixture: torch.Tensor, references: Optional[torch.Tensor] = None,
                       stems: Sequence[str] = STEMS, sample_rate: int = 44100, segment_seconds: float = 6.0,
                       overlap: float = 0.1):
    """The body of `test_inference.py:91-155` on an in-memory track: mixture (2, L); references (S, 2, L) true stems
    (optional).  Returns (final (S, 2, L), {stem: SDR dB}) with SDR = -sdr_loss(estimate, reference) per stem for the
    first min(S, 4) stems (`:147-155`), -30.0 for the others and when no references are given."""
    final = separate_track(model, mixture, stems, sample_rate, segment_seconds, overlap)
    scores = {s: -30.0 for s in stems}
    if references is not None:
        for i, s in enumerate(list(stems)[:4]):
            scores[s] = float(-sdr_loss(final[i], references[i]).item())
    return final, scores


def cleaned_track_name(filename) -> str:
    """The output directory name of `test_inference.py:159-162`: `Path(filename).stem` without ".stem", "-" and
    "'", spaces as "_"."""
    name = Path(filename).stem.replace(".stem", "")
    return name.replace("-", "").replace("'", "").replace(" ", "_")


@torch.no_grad()
def test_inference(checkpoint_path: str = "checkpoints/best_model.pt", data_dir: str = "data/quick_train",
                   output_dir: str = "results", sample_rate: int = 44100, segment_seconds: float = 6.0,
                   overlap: float = 0.1, device: Optional[str] = None, *,
                   text_table: Optional[Dict[str, np.ndarray]] = None, clap=None, tokenizer=None,
                   dtype: str = "bf16", stems: Sequence[str] = STEMS, return_final: bool = False):
    """`test_inference.py:43-205` with the same positional signature and defaults (`:44-52`).

    Loads the checkpoint (`load_model`, `:71`), takes the first track of `data_dir` (`dataset.files[0]`, `:85-90`;
    MUSDB18-HQ directories / `.stem.npy` here, see athd/musdb.py), separates every stem with the 6 s window loop
    (`:92-141`, batched through `forward_prompts`), scores stems 0..3 against the true stems with -sdr_loss (`:147-155`)
    and writes `<output_dir>/<cleaned name>/extracted_{stem}.wav` for every stem and `mixture.wav` (`:157-175`, 16-bit
    PCM like soundfile's WAV default).  Returns the `{stem: SDR dB}` dict (`:205`); with `return_final=True`
    (sdr_scores, final (S, 2, L) on the device).  The keyword-only arguments are this build's: the prompt embeddings
    (`text_table` or a local CLAP `clap`/`tokenizer`, athd/text.py: the reference's `from_pretrained` at `:27-28` is
    not reachable offline) and the compute dtype.  The spectrogram plots of `:177-185` are not drawn (no display)."""
    from .musdb import MusDBTracks, write_wav
    if device is None:
        device = "cuda"
        if not torch.cuda.is_available():
            raise RuntimeError("athd runs on a HIP device only (there is no CPU path)")
    model = load_model(checkpoint_path, device, dtype=dtype, text_table=text_table, clap=clap, tokenizer=tokenizer)
    tracks = MusDBTracks(data_dir, sample_rate=sample_rate)
    all_stems = torch.from_numpy(tracks.load_stems(0)).permute(0, 2, 1).float().to(model.device)   # (5, C, T)
    full_mixture = all_stems[0]
    final, sdr_scores = separate_and_score(model, full_mixture, all_stems[1:], stems, sample_rate, segment_seconds,
                                           overlap)
    for i in range(min(len(stems), 4)):
        print(f"{stems[i]:8s} | SDR: {sdr_scores[stems[i]]:6.2f} dB")
    if output_dir:
        f0 = tracks.files[0]       # an HQ directory stands for the reference's "<name>.stem.mp4"
        full_dir = Path(output_dir) / cleaned_track_name(f0.name + ".stem.mp4" if f0.is_dir() else f0)
        full_dir.mkdir(parents=True, exist_ok=True)
        for i, s in enumerate(stems):
            write_wav(full_dir / f"extracted_{s}.wav", final[i].cpu().numpy().T, sample_rate)
        write_wav(full_dir / "mixture.wav", full_mixture.cpu().numpy().T, sample_rate)
    return (sdr_scores, final) if return_final else sdr_scores


def load_config(file_path) -> dict:
    """`utils.py:18-23`: a YAML file through `yaml.safe_load`."""
    import yaml
    with open(file_path, "r") as f:
        return yaml.safe_load(f)


def main(config_path: str = "config.yaml", **kw):
    """`test_inference.py:208-218`: the checkpoint, data and output paths and the audio constants from config.yaml."""
    cfg = load_config(config_path)
    return test_inference(checkpoint_path=str(Path(cfg["wandb"]["checkpoint_dir"]) / "best_model.pt"),
                          data_dir=cfg["data"]["test_dir"], output_dir=cfg["wandb"]["output_dir"],
                          sample_rate=cfg["data"]["sample_rate"], segment_seconds=cfg["data"]["segment_seconds"], **kw)
