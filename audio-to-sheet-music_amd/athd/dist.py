"""Multi-GPU runner for the hot path: one process per GPU under torchrun, `torch.distributed`
with backend "nccl" (RCCL over xGMI on MI355X).

Units are independent, so sharding needs no data-path collective; the one exchange is north_star's gather of the
separated waveforms to rank `dst`:
  * `separate_segments`: N segments -> contiguous blocks of ceil(N/W) per rank.  Each rank runs `forward_prompts`
    (encode once, decode P times) on batches of its block.  As soon as a batch is computed its (b, P, 2, T) result
    is sent point-to-point to `dst`, which receives it straight into its slice of the preallocated (N, P, 2, T)
    output (the block of rank r is rows [lo_r, hi_r), so every batch lands in one contiguous slice: no padding,
    no `torch.cat`).  The sends run on RCCL's stream while the next batch computes on the compute stream; at most
    two batches are in flight per rank.  xGMI is point to point, so a gather to one GPU is one direct link per
    peer, never a ring.
  * `separate_track_sharded`: the windows of one track -> contiguous window ranges per rank; each rank overlap-adds
    its windows into a partial track span and sends it to `dst`, which adds the spans in rank order.  Protocols:
      - "test_inference" (test_inference.py:92-141, Fade + additive OLA, athd_overlap_add): seams get window k-1
        then window k as in the reference loop and 0.0f + x = x elsewhere, so the result equals the single-GPU
        track bit for bit;
      - "benchmark" (benchmark.py:155-204, weighted OLA, athd_overlap_add_weighted): the partial spans carry the
        unnormalised sum and the weight sum, added in rank order the same way, then normalised once on `dst`.
  * `separate_dataset`: a whole MUSDB18 split (athd.musdb.MusDBTracks) in track-aligned groups of a bounded number
    of windows: every window of a group is a unit of `separate_segments`; `dst` gathers the group into one reused
    buffer, reassembles each track from its rows (weighted overlap-add), scores it against the reference stems and
    writes evaluation_results.json (benchmark.py:742-781, :853-888).
Block, batch and span sizes follow from (N, W) or the window plan, so no size exchange is needed.  Before its first
exchange each runner makes one barrier per process group, so a lazily created NCCL communicator (no `device_id`
in init_process_group) exists on every rank even when some rank's block is empty.

`forward_fn` / `window_fn` / `ola_fn` default to the native path; tests substitute CPU stand-ins to exercise the
sharding and exchange logic with the gloo backend.
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


def _global(group, r: int) -> int:
    return dist.get_global_rank(group, r) if group is not None else r


_READY: List = []          # process-group objects whose communicator is known to exist


def _ensure_comm(group, world: int) -> None:
    """Initialise the group's communicator with one collective before its first point-to-point exchange.  With a
    lazily created NCCL communicator (init_process_group without device_id) the first batch_isend_irecv must be
    made by every rank of the group, but a rank whose block is empty makes none; one barrier per group (every rank
    calls the runner) creates the communicator on all of them."""
    if world <= 1:
        return
    pg = group if group is not None else dist.group.WORLD
    if not any(g is pg for g in _READY):
        dist.barrier(group)
        _READY.append(pg)


class PendingSends:
    """Point-to-point transfers in flight; `limit` bounds how many are outstanding (the oldest is waited on, which
    only makes the current stream wait for it on NCCL - no host synchronisation)."""

    def __init__(self, limit: Optional[int] = 2):
        self.limit = limit
        self.works: List = []

    def add(self, works, keep=None):
        """works: the list batch_isend_irecv returned; keep: tensors that must stay alive until they complete."""
        self.works.append((works, keep))
        while self.limit is not None and len(self.works) > self.limit:
            for w in self.works.pop(0)[0]:
                w.wait()

    def wait(self):
        for ws, _ in self.works:
            for w in ws:
                w.wait()
        self.works = []


@torch.no_grad()
def separate_segments(model, segments: torch.Tensor, prompts: Sequence[str] = STEMS, dst: int = 0, group=None,
                      max_batch: int = 64, forward_fn: Optional[Callable] = None, n_total: Optional[int] = None,
                      out: Optional[torch.Tensor] = None, pending: Optional[PendingSends] = None
                      ) -> Optional[torch.Tensor]:
    """Separate N segments into P stems across the ranks of `group` -> (N, P, 2, T) on rank `dst`, None elsewhere.

    segments: (N, 2, T), the full list on every rank (a host tensor or a lazy view is fine: only this rank's block
    is read), or - with `n_total=N` - only this rank's block [lo, hi) of shard_range(N, W, rank), e.g. already
    resident on the device.  `out`: optional preallocated (N, P, 2, T) result on `dst`.  `pending`: a PendingSends
    to leave the transfers in flight in (the caller waits on it later, e.g. across bench steps); by default they
    are completed before returning."""
    world, rank = _world(group)
    N = n_total if n_total is not None else segments.shape[0]
    P, T = len(prompts), segments.shape[-1]
    lo, hi = shard_range(N, world, rank)
    if n_total is not None and segments.shape[0] != hi - lo:
        raise ValueError(f"rank {rank}: expected its block of {hi - lo} segments, got {segments.shape[0]}")
    base = 0 if n_total is None else lo          # segment index of row 0 of `segments`
    fwd = forward_fn or (lambda wav, o: model.forward_prompts(wav, list(prompts), out=o))
    dev = model.device if forward_fn is None else segments.device
    if rank == dst:
        if out is None:
            out = torch.empty((N, P, 2, T), dtype=torch.float32, device=dev)
        elif tuple(out.shape) != (N, P, 2, T) or not out.is_contiguous():
            raise ValueError(f"out must be a contiguous {(N, P, 2, T)} tensor")
    _ensure_comm(group, world)
    own = pending is None
    pend = pending if pending is not None else PendingSends()
    per = -(-N // world) if N else 0
    for j in range(-(-per // max_batch) if per else 0):          # same batch count on every rank
        recvs = []
        if rank == dst:
            for r in range(world):
                a, b = shard_range(N, world, r)
                b0, b1 = min(b, a + j * max_batch), min(b, a + (j + 1) * max_batch)
                if r != dst and b1 > b0:
                    recvs.append(dist.P2POp(dist.irecv, out[b0:b1], _global(group, r), group))
        b0, b1 = min(hi, lo + j * max_batch), min(hi, lo + (j + 1) * max_batch)
        if b1 > b0:
            wav = segments[b0 - base:b1 - base].to(dev, non_blocking=True).contiguous()
            if rank == dst:
                res = fwd(wav, out[b0:b1])
                # forward_fn(wav, o) fills `o` (and may return it); a new result tensor is copied in
                if res is not None and res.data_ptr() != out[b0:b1].data_ptr():
                    if tuple(res.shape) != (b1 - b0, P, 2, T):
                        raise ValueError(f"forward_fn returned {tuple(res.shape)}, expected {(b1 - b0, P, 2, T)}")
                    out[b0:b1].copy_(res)
            else:
                res = fwd(wav, None).contiguous()
                pend.add(dist.batch_isend_irecv([dist.P2POp(dist.isend, res, _global(group, dst), group)]), res)
        if recvs:
            pend.add(dist.batch_isend_irecv(recvs), out)
    if own:
        pend.wait()
    return out if rank == dst else None


def dataset_plan(lengths: Sequence[int], chunk_len: int, overlap_frames: int) -> List[Tuple[int, int]]:
    """Units of a whole split: (track index, window index) in track order.  Track i has ceil(L_i / hop) windows
    starting at k * hop, hop = chunk_len - overlap_frames (the `while start < T` loop of benchmark.py:164-198; with
    overlap 0 these are the dataloader's deterministic segments, dataloader.py:67,104-121)."""
    hop = chunk_len - overlap_frames
    if hop <= 0:
        raise ValueError("overlap must be shorter than the window")
    return [(ti, k) for ti, L in enumerate(lengths) for k in range(-(-int(L) // hop))]


def dataset_windows(tracks, units: Sequence[Tuple[int, int]], chunk_len: int, overlap_frames: int) -> torch.Tensor:
    """Model inputs of `units` (consecutive entries of dataset_plan): (n, 2, chunk_len), each window zero-padded
    past the end of its track (benchmark.py:167-172).  Only the tracks the units touch are read (mixture only)."""
    hop = chunk_len - overlap_frames
    out = torch.zeros((len(units), 2, chunk_len), dtype=torch.float32)
    cur, mix = None, None
    for j, (ti, k) in enumerate(units):
        if ti != cur:
            cur, mix = ti, tracks.mixture(ti)
        s = k * hop
        e = min(s + chunk_len, mix.shape[-1])
        out[j, :, :e - s] = mix[:, s:e]
    return out.pin_memory() if torch.cuda.is_available() else out


def dataset_groups(lengths: Sequence[int], chunk_len: int, overlap_frames: int, cap: int) -> List[Tuple[int, int]]:
    """Track-aligned gather groups of a split: consecutive track ranges [t0, t1) whose windows total <= cap (a track
    with more than `cap` windows forms a group of its own).  Every rank derives the same list from the lengths."""
    hop = chunk_len - overlap_frames
    groups, t0, n = [], 0, 0
    for ti, L in enumerate(lengths):
        w = -(-int(L) // hop)
        if ti > t0 and n + w > cap:
            groups.append((t0, ti))
            t0, n = ti, 0
        n += w
    if len(lengths) > t0:
        groups.append((t0, len(lengths)))
    return groups


@torch.no_grad()
def separate_dataset(model, tracks, stems: Sequence[str] = STEMS, segment_seconds: float = 6.0,
                     overlap: float = 1.5, sample_rate: int = 44100, dst: int = 0, group=None, max_batch: int = 64,
                     output_dir=None, forward_fn: Optional[Callable] = None, ola_fn: Optional[Callable] = None,
                     metric_fn: Optional[Callable] = None, model_name: str = "AudioTextHTDemucs (Ours)",
                     keep_estimates: bool = False, log: Optional[Callable[[str], None]] = print,
                     group_windows: Optional[int] = None, stats: Optional[dict] = None):
    """A whole MUSDB18 split through the sharded runner -> per-track stems and metrics on rank `dst`.

    The reference evaluates a split track by track, one 6 s window and one stem at a time
    (test_inference.py:75-88 -> dataloader.py:56-84 -> benchmark.py:742-781, OurModel._chunked_inference
    :155-204).  Here the split is cut into track-aligned groups of at most `group_windows` windows (dataset_groups;
    default 4 x world x max_batch, at least the longest track's windows).  Per group, every window is one unit of
    `separate_segments`: the units are sharded in contiguous blocks over the ranks (each rank reads only the tracks
    its block touches), each rank separates its block into all stems (encode once, decode len(stems) times, batches
    of `max_batch` windows spanning tracks) and the separated windows are gathered point to point into ONE reused
    (group_windows, S, 2, chunk) buffer on `dst`.  `dst` then reassembles every track of the group from its rows with
    the weighted overlap-add of benchmark.py:177-202 (athd_overlap_add_weighted), computes SDR / SI-SDR per stem
    against the track's reference stems (benchmark.py:655-688) before the buffer is reused, and, with `output_dir`,
    writes `evaluation_results.json` (save_results, benchmark.py:853-888).  So the gather buffer on `dst` (8.47 MB
    per window at 4 stems x 6 s) and each rank's pinned host block are bounded by `group_windows`, whatever the
    split's size (configs[3]: ~6k windows would otherwise be ~51 GB on dst).

    overlap=1.5 is benchmark.py's protocol (OurModel's default, the one behind eval_results/*.json); overlap=0
    separates the dataloader's non-overlapping segments (dataloader.py:67,104-121) and concatenates them.
    Returns (results, estimates) on dst - estimates {track name: (S, 2, L)} only with keep_estimates - and None
    elsewhere.  forward_fn / ola_fn(win, L, chunk, ov) / metric_fn(est, ref) -> (sdr, sisdr) default to the native
    path; tests substitute CPU stand-ins to run the exchange on gloo.  `stats` (optional dict) receives
    {"groups", "buffer_rows"}."""
    from .benchmark import track_result, log_track, save_results
    if sorted(stems) != sorted(STEMS):
        raise ValueError(f"the evaluation needs every stem of {STEMS}, got {list(stems)}")
    world, rank = _world(group)
    chunk_len = int(sample_rate * segment_seconds)
    ov = int(overlap * sample_rate)
    hop = chunk_len - ov
    lengths = tracks.lengths()
    longest = max((-(-int(L) // hop) for L in lengths), default=0)
    cap = max(group_windows if group_windows is not None else 4 * world * max_batch, longest)
    groups = dataset_groups(lengths, chunk_len, ov, cap)
    if ola_fn is None and rank == dst:
        from .benchmark import overlap_add_weighted
        ola_fn = lambda win, L, c, o: overlap_add_weighted(win, L, c, o)      # noqa: E731
    buf = None
    results, estimates = [], {}
    for t0, t1 in groups:
        units = dataset_plan(lengths[t0:t1], chunk_len, ov)
        units = [(t0 + ti, k) for ti, k in units]
        N = len(units)
        lo, hi = shard_range(N, world, rank)
        block = dataset_windows(tracks, units[lo:hi], chunk_len, ov)
        out = None
        if rank == dst:
            if buf is None:
                dev = model.device if forward_fn is None else block.device
                rows = min(cap, sum(-(-int(L) // hop) for L in lengths))
                buf = torch.empty((rows, len(stems), 2, chunk_len), dtype=torch.float32, device=dev)
            out = buf[:N]
        out = separate_segments(model, block, stems, dst=dst, group=group, max_batch=max_batch,
                                forward_fn=forward_fn, n_total=N, out=out)
        del block
        if rank != dst:
            continue
        row = 0
        for ti in range(t0, t1):
            L = int(lengths[ti])
            n = -(-L // hop)                                                    # this track's rows of the group
            est = ola_fn(out[row:row + n], L, chunk_len, ov)                    # (S, 2, L)
            row += n
            name, _, refs = tracks.track(ti)
            r = track_result(name, model_name, {s: est[i] for i, s in enumerate(stems)}, refs, metric_fn)
            results.append(r)
            if keep_estimates:
                estimates[name] = est
            if log:
                log_track(r, log)
    if stats is not None:
        stats.update(groups=len(groups), buffer_rows=0 if buf is None else buf.shape[0])
    if rank != dst:
        return None
    if output_dir is not None:
        save_results({model_name: results}, output_dir)
    return results, estimates


@torch.no_grad()
def separate_track_sharded(model, mixture: torch.Tensor, stems: Sequence[str] = STEMS, sample_rate: int = 44100,
                           segment_seconds: float = 6.0, overlap: float = 0.1, dst: int = 0, group=None,
                           max_batch: int = 64, window_fn: Optional[Callable] = None,
                           ola_fn: Optional[Callable] = None, protocol: str = "test_inference"
                           ) -> Optional[torch.Tensor]:
    """One track split by window ranges across ranks -> (S, 2, L) on rank dst (None elsewhere).

    protocol "test_inference": test_inference.py:92-141 (overlap default 0.1 s); "benchmark": benchmark.py:155-204
    (pass overlap=1.5 for its default).  window_fn(k0, k1) -> (k1-k0, S, 2, chunk) model outputs; ola_fn(win, k0, k1)
    -> span (test_inference) or (span, weight sums) (benchmark)."""
    if protocol not in ("test_inference", "benchmark"):
        raise ValueError(f"unknown protocol {protocol!r}")
    world, rank = _world(group)
    if mixture.dim() == 3:
        mixture = mixture[0]
    L = mixture.shape[-1]
    chunk_len = int(sample_rate * segment_seconds)
    ov = int(overlap * sample_rate)
    hop = chunk_len - ov
    n = -(-L // hop)
    S = len(stems)
    ranges = [shard_range(n, world, r) for r in range(world)]
    k0, k1 = ranges[rank]
    bench = protocol == "benchmark"
    if window_fn is None or ola_fn is None:
        if bench:
            from .benchmark import OurModel, overlap_add_weighted
            om = OurModel(model, segment_seconds=segment_seconds, overlap=overlap, max_batch=max_batch)
            wfn = lambda a, b: om.run_windows(mixture, stems, a, b)                         # noqa: E731
            ofn = lambda win, a, b: overlap_add_weighted(win, L, chunk_len, ov, a, b, partial=True)  # noqa: E731
        else:
            from .inference import overlap_add, run_windows, window_plan
            plan = window_plan(L, sample_rate, segment_seconds, overlap)
            wfn = lambda a, b: run_windows(model, mixture, plan, stems, chunk_len, a, b, max_batch)  # noqa: E731
            ofn = lambda win, a, b: overlap_add(win, L, chunk_len, ov, a, b)                 # noqa: E731
        window_fn = window_fn or wfn
        ola_fn = ola_fn or ofn

    def span_len(a, b):
        return 0 if b <= a else min((b - 1) * hop + chunk_len, L) - a * hop

    dev = mixture.device
    if k1 > k0:
        res = ola_fn(window_fn(k0, k1), k0, k1)
        span, wsum = res if bench else (res, None)
    else:
        span = torch.empty((S, 2, 0), dtype=torch.float32, device=dev)
        wsum = torch.empty(0, dtype=torch.float32, device=dev)
    # exchange: every non-empty span goes to dst point to point (sizes follow from the plan)
    _ensure_comm(group, world)
    parts = {rank: (span, wsum)}
    ops = []
    for r, (a, b) in enumerate(ranges):
        m = span_len(a, b)
        if r == rank or m == 0 or world == 1:
            continue
        if rank == dst:
            pr = (torch.empty((S, 2, m), dtype=torch.float32, device=dev),
                  torch.empty(m, dtype=torch.float32, device=dev) if bench else None)
            parts[r] = pr
            ops.append(dist.P2POp(dist.irecv, pr[0], _global(group, r), group))
            if bench:
                ops.append(dist.P2POp(dist.irecv, pr[1], _global(group, r), group))
    if rank != dst and world > 1 and k1 > k0:
        ops.append(dist.P2POp(dist.isend, span.contiguous(), _global(group, dst), group))
        if bench:
            ops.append(dist.P2POp(dist.isend, wsum.contiguous(), _global(group, dst), group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if rank != dst:
        return None
    final = torch.zeros((S, 2, L), dtype=torch.float32, device=dev)
    weight = torch.zeros(L, dtype=torch.float32, device=dev) if bench else None
    for r, (a, b) in enumerate(ranges):                       # rank order = window order
        if b <= a:
            continue
        sp, ws = parts[r]
        s0 = a * hop
        final[:, :, s0:s0 + sp.shape[-1]] += sp
        if bench:
            weight[s0:s0 + ws.shape[0]] += ws
    if bench:
        if weight.device.type == "cuda":
            from .benchmark import ola_normalize
            ola_normalize(final, weight)
        else:                                                  # CPU stand-in runs (tests)
            final /= weight.clamp(min=1e-8)
    return final
