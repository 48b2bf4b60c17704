"""Multi-GPU runner for the hot path: one process per GPU under torchrun, `torch.distributed`
with backend "nccl" (RCCL over xGMI on MI355X).

Units are independent, so sharding needs no data-path collective; the single exchange is north_star's gather of
results to rank 0:
  * `separate_segments`: N segments -> contiguous blocks of ceil(N/W) per rank; each rank runs
    `forward_prompts` on its block (encode once, decode P times) and rank `dst` gathers (B_r, P, 2, T) from all
    ranks with one `gather` per call.
  * `separate_track_sharded`: the windows of one track (test_inference.py:92-141) -> contiguous window ranges per
    rank; each rank overlap-adds its windows into a partial track span (athd_overlap_add with [k0, k1)); rank
    `dst` gathers the spans and adds them in rank order.  Seams get window k-1 then window k, as in the
    reference loop, and 0.0f + x = x elsewhere, so the result equals the single-GPU track bit-exactly.
Span and block sizes follow from the plan, so no size exchange is needed; ragged blocks are padded for the
gather and cut on rank `dst`.

`window_fn` / `ola_fn` default to the native path (athd.inference.run_windows / overlap_add); tests substitute
CPU stand-ins to exercise the sharding and gather logic with the gloo backend.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .weights import STEMS


def shard_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of ceil(n / world) units for `rank` (the last blocks may be short or empty)."""
    per = -(-n // world) if n else 0
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def _world(group) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def _gather_padded(t: torch.Tensor, sizes: List[int], dst: int, group) -> Optional[List[torch.Tensor]]:
    """Gather tensors whose dim 0 is sizes[r] on rank r (padded to max(sizes)) -> list on dst, None elsewhere."""
    world, rank = _world(group)
    if world == 1:
        return [t]
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if t.shape[0]:
        pad[:t.shape[0]] = t
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return [b[:s] for b, s in zip(bufs, sizes)]


@torch.no_grad()
def separate_segments(model, segments: torch.Tensor, prompts: Sequence[str] = STEMS, dst: int = 0, group=None,
                      max_batch: int = 64, forward_fn: Optional[Callable] = None) -> Optional[torch.Tensor]:
    """segments: (N, 2, T), the full list (every rank passes the same tensor, or a lazy view); rank r computes
    block shard_range(N) -> returns (N, P, 2, T) on rank dst, None on the others."""
    world, rank = _world(group)
    N, P = segments.shape[0], len(prompts)
    lo, hi = shard_range(N, world, rank)
    fwd = forward_fn or (lambda wav: model.forward_prompts(wav, list(prompts)))
    dev = model.device if forward_fn is None else segments.device
    parts = []
    for b0 in range(lo, hi, max_batch):
        wav = segments[b0:min(hi, b0 + max_batch)].to(dev, non_blocking=True).contiguous()
        parts.append(fwd(wav))
    T = segments.shape[-1]
    mine = torch.cat(parts) if parts else torch.empty((0, P, 2, T), dtype=torch.float32, device=dev)
    sizes = [shard_range(N, world, r)[1] - shard_range(N, world, r)[0] for r in range(world)]
    got = _gather_padded(mine, sizes, dst, group)
    return torch.cat(got) if got is not None else None


@torch.no_grad()
def separate_track_sharded(model, mixture: torch.Tensor, stems: Sequence[str] = STEMS, sample_rate: int = 44100,
                           segment_seconds: float = 6.0, overlap: float = 0.1, dst: int = 0, group=None,
                           max_batch: int = 64, window_fn: Optional[Callable] = None,
                           ola_fn: Optional[Callable] = None) -> Optional[torch.Tensor]:
    """One track split by window ranges across ranks -> (S, 2, L) on rank dst (None elsewhere)."""
    from .inference import overlap_add, run_windows, window_plan
    world, rank = _world(group)
    if mixture.dim() == 3:
        mixture = mixture[0]
    L = mixture.shape[-1]
    chunk_len = int(sample_rate * segment_seconds)
    ov = int(overlap * sample_rate)
    hop = chunk_len - ov
    plan = window_plan(L, sample_rate, segment_seconds, overlap)
    n, S = len(plan), len(stems)
    ranges = [shard_range(n, world, r) for r in range(world)]

    def span_len(k0, k1):
        return 0 if k1 <= k0 else min((k1 - 1) * hop + chunk_len, L) - k0 * hop

    k0, k1 = ranges[rank]
    wfn = window_fn or (lambda a, b: run_windows(model, mixture, plan, stems, chunk_len, a, b, max_batch))
    ofn = ola_fn or (lambda win, a, b: overlap_add(win, L, chunk_len, ov, a, b))
    if k1 > k0:
        span = ofn(wfn(k0, k1), k0, k1)
    else:
        span = torch.empty((S, 2, 0), dtype=torch.float32, device=mixture.device)
    # gather along the sample axis: move it to dim 0 for the padded gather
    sizes = [span_len(a, b) for a, b in ranges]
    got = _gather_padded(span.permute(2, 0, 1).contiguous(), sizes, dst, group)
    if got is None:
        return None
    final = torch.zeros((S, 2, L), dtype=torch.float32, device=span.device)
    for (a, b), part in zip(ranges, got):          # rank order = window order
        if b > a:
            s0 = a * hop
            final[:, :, s0:s0 + part.shape[0]] += part.permute(1, 2, 0)
    return final
