"""`benchmark.py` protocol twin: the evaluation path that produced the reference's published
`eval_results/*/evaluation_results.json`, on the native hot path.

Mirrors, name for name:
  * `OurModel`                      <- `benchmark.py:122-215`: 6 s windows with a 1.5 s overlap, the last window
                                       zero-padded to 6 s, linspace fades of min(overlap, len // 2) samples, weighted
                                       overlap-add normalised by the summed weights (`_chunked_inference`, :155-204).
                                       All windows of a track are full 6 s forwards, so they are batched
                                       (`forward_prompts`: encode once, decode once per stem) and the weighted
                                       overlap-add runs in `athd_overlap_add_weighted` (same fp32 products, sums and
                                       order as the reference loop).
  * `compute_sdr` / `compute_sisdr` <- `benchmark.py:555-588`: one SDR / SI-SDR per stem over the (1, C*T) flatten
                                       (`athd_sdr` / `athd_sisdr`, fp64 sums on the device).
  * `TrackResult`, `evaluate_model_on_track`, `evaluate_model`, `aggregate_results`, `save_results`
                                    <- `benchmark.py:618-888` (same JSON layout), minus plotting / wandb.
The MUSDB18 `.stem.mp4` decode (`load_track_stems`, :591-615) needs stempeg/ffmpeg, which are absent here; tracks
come from `athd.musdb` (pre-decoded arrays) or from memory.
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass
from pathlib import Path
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import native
from .weights import STEMS

SAMPLE_RATE = 44100


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def num_windows(length: int, chunk_len: int, overlap_frames: int) -> int:
    """Windows of `while start < T: ...; start += chunk_len - overlap_frames` (benchmark.py:164-198)."""
    return int(native.lib.athd_num_windows(length, chunk_len, overlap_frames))


def window_batch(mixture: torch.Tensor, chunk_len: int, overlap_frames: int, k0: int = 0,
                 k1: Optional[int] = None) -> torch.Tensor:
    """Model inputs of windows [k0, k1): (k1-k0, C, chunk_len), the last window zero-padded (benchmark.py:167-172)."""
    C, L = mixture.shape
    hop = chunk_len - overlap_frames
    n = num_windows(L, chunk_len, overlap_frames)
    k1 = n if k1 is None else k1
    out = torch.zeros((k1 - k0, C, chunk_len), dtype=torch.float32, device=mixture.device)
    for k in range(k0, k1):
        s = k * hop
        e = min(s + chunk_len, L)
        out[k - k0, :, :e - s] = mixture[:, s:e]
    return out


def overlap_add_weighted(windows: torch.Tensor, length: int, chunk_len: int, overlap_frames: int, k0: int = 0,
                         k1: Optional[int] = None, partial: bool = False):
    """windows (k1-k0, S, 2, chunk_len) -> normalised (S, 2, span) track span; partial=True -> (sum w x, sum w) of the
    span for sharded runs (finish with `ola_normalize` after adding the spans in window order)."""
    n = num_windows(length, chunk_len, overlap_frames)
    k1 = n if k1 is None else k1
    S = windows.shape[1]
    if windows.dim() != 4 or windows.shape[0] != k1 - k0 or windows.shape[2] != 2 or windows.shape[3] != chunk_len:
        raise ValueError(f"windows must be ({k1 - k0}, S, 2, {chunk_len}), got {tuple(windows.shape)}")
    if windows.dtype != torch.float32 or not windows.is_contiguous() or windows.device.type != "cuda":
        raise ValueError("windows must be a contiguous float32 device tensor")
    hop = chunk_len - overlap_frames
    span = min((k1 - 1) * hop + chunk_len, length) - k0 * hop
    out = torch.empty((S, 2, span), dtype=torch.float32, device=windows.device)
    wsum = torch.empty(span, dtype=torch.float32, device=windows.device) if partial else None
    rc = native.lib.athd_overlap_add_weighted(windows.data_ptr(), length, chunk_len, overlap_frames, S, k0, k1,
                                              out.data_ptr(), wsum.data_ptr() if partial else None,
                                              _stream(windows.device))
    if rc != 0:
        raise native.AthdError(f"athd_overlap_add_weighted failed ({rc})")
    return (out, wsum) if partial else out


def ola_normalize(out: torch.Tensor, wsum: torch.Tensor) -> torch.Tensor:
    """out (..., n) /= max(wsum (n), 1e-8) in place (benchmark.py:201-202)."""
    n = out.shape[-1]
    if wsum.shape != (n,) or not out.is_contiguous() or not wsum.is_contiguous():
        raise ValueError("out (..., n) and wsum (n,) must be contiguous")
    rc = native.lib.athd_ola_normalize(out.data_ptr(), wsum.data_ptr(), out.numel() // n, n, _stream(out.device))
    if rc != 0:
        raise native.AthdError(f"athd_ola_normalize failed ({rc})")
    return out


def _metric(fn, estimate: torch.Tensor, reference: torch.Tensor) -> torch.Tensor:
    est = estimate.reshape(1, -1).float().contiguous()
    ref = reference.reshape(1, -1).float().contiguous()
    if est.shape != ref.shape:
        raise ValueError("estimate and reference must have the same size")
    scratch = torch.empty(5, dtype=torch.float64, device=est.device)
    out = torch.empty(1, dtype=torch.float32, device=est.device)
    rc = fn(est.data_ptr(), ref.data_ptr(), 1, est.shape[1], scratch.data_ptr(), out.data_ptr(), _stream(est.device))
    if rc != 0:
        raise native.AthdError(f"metric kernel failed ({rc})")
    return out[0]


def compute_sdr(estimate: torch.Tensor, reference: torch.Tensor) -> float:
    """`benchmark.py:555-570`: -sdr_loss on (1, C, T), i.e. one SDR over both channels flattened."""
    return float(_metric(native.lib.athd_sdr, estimate, reference).item())


def compute_sisdr(estimate: torch.Tensor, reference: torch.Tensor) -> float:
    """`benchmark.py:573-588`: -sisdr_loss on (1, C, T)."""
    return float(_metric(native.lib.athd_sisdr, estimate, reference).item())


class OurModel:
    """`benchmark.py:122-215` around an already-loaded `athd.model.AudioTextHTDemucs` (construct it with
    `athd.inference.load_model(checkpoint)`; the reference's remote htdemucs / CLAP downloads are not needed)."""

    def __init__(self, model, device: Optional[str] = None, segment_seconds: float = 6.0, overlap: float = 1.5,
                 max_batch: int = 64):
        self.model = model
        self.device = torch.device(device) if device is not None else model.device
        self.segment_seconds = segment_seconds
        self.overlap = overlap
        self.max_batch = max_batch

    @property
    def name(self) -> str:
        return "AudioTextHTDemucs (Ours)"

    @property
    def chunk_len(self) -> int:
        return int(SAMPLE_RATE * self.segment_seconds)

    @property
    def overlap_frames(self) -> int:
        return int(self.overlap * SAMPLE_RATE)

    @torch.no_grad()
    def run_windows(self, mixture: torch.Tensor, stems: Sequence[str], k0: int = 0,
                    k1: Optional[int] = None) -> torch.Tensor:
        """Model outputs of windows [k0, k1) for every stem: (k1-k0, S, C, chunk_len)."""
        C, L = mixture.shape
        n = num_windows(L, self.chunk_len, self.overlap_frames)
        k1 = n if k1 is None else k1
        win = torch.empty((k1 - k0, len(stems), C, self.chunk_len), dtype=torch.float32, device=self.device)
        for b0 in range(k0, k1, self.max_batch):
            b1 = min(k1, b0 + self.max_batch)
            batch = window_batch(mixture, self.chunk_len, self.overlap_frames, b0, b1)
            self.model.forward_prompts(batch, list(stems), out=win[b0 - k0:b1 - k0])
        return win

    @torch.no_grad()
    def _chunked_inference(self, mixture: torch.Tensor, prompt: str) -> torch.Tensor:
        """`benchmark.py:155-204`: one stem -> (C, T)."""
        return self.separate_stems(mixture, [prompt])[0]

    @torch.no_grad()
    def separate_stems(self, mixture: torch.Tensor, stems: Sequence[str]) -> torch.Tensor:
        mixture = mixture.to(self.device).float().contiguous()
        if mixture.dim() != 2 or mixture.shape[0] != 2:
            raise ValueError(f"expected a (2, T) stereo mixture, got {tuple(mixture.shape)}")
        win = self.run_windows(mixture, stems)
        return overlap_add_weighted(win, mixture.shape[-1], self.chunk_len, self.overlap_frames)

    def separate(self, mixture: torch.Tensor, stem_name: str) -> torch.Tensor:
        return self._chunked_inference(mixture, stem_name)

    def separate_all(self, mixture: torch.Tensor) -> Dict[str, torch.Tensor]:
        """`benchmark.py:210-215`; all stems share each window's encoder pass."""
        out = self.separate_stems(mixture, STEMS)
        return {s: out[i] for i, s in enumerate(STEMS)}


@dataclass
class TrackResult:
    """`benchmark.py:618-634`."""
    track_name: str
    model_name: str
    sdr_drums: float
    sdr_bass: float
    sdr_other: float
    sdr_vocals: float
    sdr_avg: float
    sisdr_drums: float
    sisdr_bass: float
    sisdr_other: float
    sisdr_vocals: float
    sisdr_avg: float


def track_result(track_name: str, model_name: str, estimates: Dict[str, torch.Tensor],
                 reference_stems: Dict[str, torch.Tensor],
                 metric_fn: Optional[Callable] = None) -> TrackResult:
    """Per stem SDR / SI-SDR on the common length and their averages (`benchmark.py:655-688`).  metric_fn(est,
    ref) -> (sdr, sisdr) defaults to the native kernels (compute_sdr / compute_sisdr)."""
    sdr, sisdr = {}, {}
    for stem in STEMS:
        e = estimates[stem]
        r = torch.as_tensor(reference_stems[stem]).to(e.device)
        n = min(e.shape[-1], r.shape[-1])
        e, r = e[:, :n].contiguous(), r[:, :n].contiguous()
        if metric_fn is None:
            sdr[stem], sisdr[stem] = compute_sdr(e, r), compute_sisdr(e, r)
        else:
            sdr[stem], sisdr[stem] = metric_fn(e, r)
    return TrackResult(track_name, model_name, sdr["drums"], sdr["bass"], sdr["other"], sdr["vocals"],
                       sum(sdr.values()) / len(sdr), sisdr["drums"], sisdr["bass"], sisdr["other"],
                       sisdr["vocals"], sum(sisdr.values()) / len(sisdr))


def evaluate_model_on_track(model: OurModel, mixture: torch.Tensor, reference_stems: Dict[str, torch.Tensor],
                            track_name: str) -> Tuple[TrackResult, Dict[str, torch.Tensor]]:
    """`benchmark.py:637-739` without plotting: per stem SDR / SI-SDR on the common length."""
    est = model.separate_all(mixture)
    return track_result(track_name, model.name, est, reference_stems), est


def log_track(r: TrackResult, log: Callable[[str], None] = print) -> None:
    """The per-track lines of `benchmark.py:766-773`."""
    log(f"  {r.track_name}:\n    SDR:   avg={r.sdr_avg:.2f} dB (D={r.sdr_drums:.1f}, B={r.sdr_bass:.1f}, "
        f"O={r.sdr_other:.1f}, V={r.sdr_vocals:.1f})\n    SISDR: avg={r.sisdr_avg:.2f} dB "
        f"(D={r.sisdr_drums:.1f}, B={r.sisdr_bass:.1f}, O={r.sisdr_other:.1f}, V={r.sisdr_vocals:.1f})")


def evaluate_model(model: OurModel, tracks: Iterable[Tuple[str, torch.Tensor, Dict[str, torch.Tensor]]],
                   log: Optional[Callable[[str], None]] = print) -> List[TrackResult]:
    """`benchmark.py:742-781`: tracks = (name, mixture (2, T), {stem: (2, T)}); a failing track is reported and
    skipped like the reference's try/except."""
    results = []
    for name, mixture, refs in tracks:
        try:
            r, _ = evaluate_model_on_track(model, mixture, refs, name)
        except Exception as e:          # noqa: BLE001 - the reference skips a failing track (:777-779)
            if log:
                log(f"  Error processing {name}: {e}")
            continue
        results.append(r)
        if log:
            log_track(r, log)
    return results


def aggregate_results(results: List[TrackResult]) -> Dict[str, Dict[str, float]]:
    """`benchmark.py:784-804`."""
    if not results:
        return {}
    agg = {}
    for metric in ("sdr", "sisdr"):
        agg[metric] = {s: float(np.mean([getattr(r, f"{metric}_{s}") for r in results])) for s in STEMS}
        agg[metric]["average"] = float(np.mean([getattr(r, f"{metric}_avg") for r in results]))
    return agg


def save_results(all_results: Dict[str, List[TrackResult]], output_dir) -> Path:
    """`benchmark.py:853-888`: <output_dir>/evaluation_results.json in the reference's layout."""
    output_dir = Path(output_dir)
    output_dir.mkdir(parents=True, exist_ok=True)
    out = {}
    for model_name, results in all_results.items():
        out[model_name] = {
            "per_track": [{"track": r.track_name,
                           "sdr": {**{s: getattr(r, f"sdr_{s}") for s in STEMS}, "average": r.sdr_avg},
                           "sisdr": {**{s: getattr(r, f"sisdr_{s}") for s in STEMS}, "average": r.sisdr_avg}}
                          for r in results],
            "aggregate": aggregate_results(results),
        }
    path = output_dir / "evaluation_results.json"
    with open(path, "w") as f:
        json.dump(out, f, indent=2)
    return path


def track_result_dict(r: TrackResult) -> dict:
    return asdict(r)
