"""Multi-process (world_size 2, gloo, CPU) tests of the sharded runner athd/dist.py: segment sharding + gather to
rank 0, and track-window sharding whose partial overlap-add spans recombine on rank 0 bit-exactly.  The per-rank
compute is a CPU stand-in (deterministic per-window transform + the oracle's fade/OLA); the native kernels are
covered by the -m gpu tests."""
import multiprocessing as mp
import os
import socket
import traceback

import pytest
import torch

from oracle.athtdemucs_ref import benchmark_chunked_inference, chunk_plan, linear_fade

SR, SEG, OV = 1000, 6.0, 0.1          # chunk 6000, overlap 100, hop 5900 (small CPU-sized analogue of 44.1 kHz)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_model_windows(mix, plan, stems, chunk, k0, k1):
    win = torch.zeros((k1 - k0, len(stems), 2, chunk))
    for k in range(k0, k1):
        s, e = plan[k].start, plan[k].end
        for si in range(len(stems)):
            win[k - k0, si, :, :e - s] = torch.tanh(mix[:, s:e] * (si + 1)) + 0.01 * si
    return win


def _oracle_span(win, k0, k1, L):
    cp = chunk_plan(L, SR, SEG, OV)
    s0 = cp[k0][0]
    span = torch.zeros((win.shape[1], 2, cp[k1 - 1][1] - s0))
    for k in range(k0, k1):
        s, e, fi, fo = cp[k]
        span[:, :, s - s0:e - s0] += linear_fade(win[k - k0, :, :, :e - s], fi, fo)
    return span


def _fake_stem(chunk, si):
    return torch.tanh(chunk * (si + 1)) + 0.01 * si


BCH, BOV = int(SR * SEG), int(1.5 * SR)        # benchmark protocol analogue: chunk 6000, overlap 1500


def _bench_windows(mix, stems, k0, k1):
    """Model outputs of the zero-padded windows [k0, k1) (benchmark.py:167-175)."""
    L = mix.shape[-1]
    win = torch.zeros((k1 - k0, len(stems), 2, BCH))
    for k in range(k0, k1):
        s = k * (BCH - BOV)
        e = min(s + BCH, L)
        chunk = torch.zeros(2, BCH)
        chunk[:, :e - s] = mix[:, s:e]
        for si in range(len(stems)):
            win[k - k0, si] = _fake_stem(chunk, si)
    return win


def _bench_partial(win, k0, k1, L):
    """Unnormalised weighted sum and weight sum of windows [k0, k1) (benchmark.py:177-198 without :200-202)."""
    hop = BCH - BOV
    s0 = k0 * hop
    n = min((k1 - 1) * hop + BCH, L) - s0
    out, wsum = torch.zeros((win.shape[1], 2, n)), torch.zeros(n)
    for k in range(k0, k1):
        s = k * hop
        e = min(s + BCH, L)
        a = e - s
        fl = min(BOV, a // 2)
        w = torch.ones(a)
        if s > 0 and fl > 0:
            w[:fl] = torch.linspace(0, 1, fl)
        if e < L and fl > 0:
            w[-fl:] = torch.linspace(1, 0, fl)
        out[:, :, s - s0:e - s0] += win[k - k0, :, :, :a] * w
        wsum[s - s0:e - s0] += w
    return out, wsum


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from athd.dist import separate_segments, separate_track_sharded
        from athd.inference import window_plan
        torch.manual_seed(0)
        # --- segments: N=5 over 2 ranks (3 + 2), P=3 prompts
        segs = torch.randn(5, 2, 700)
        ref = torch.stack([segs * (p + 1) - p for p in range(3)], dim=1)

        def fwd(wav, o):
            r = torch.stack([wav * (p + 1) - p for p in range(3)], dim=1)
            return r if o is None else o.copy_(r)

        for mb in (1, 2, 3, 8):
            out = separate_segments(None, segs, ["a", "b", "c"], forward_fn=fwd, max_batch=mb)
            if rank == 0:
                assert out is not None and torch.equal(out, ref), ("segments", mb)
            else:
                assert out is None
        # block-local input (n_total): each rank passes only its own segments; transfers left pending across calls
        from athd.dist import PendingSends, shard_range
        lo, hi = shard_range(5, world, rank)
        pend = PendingSends(limit=None)
        res = torch.full((5, 3, 2, 700), float("nan")) if rank == 0 else None
        for _ in range(2):
            out = separate_segments(None, segs[lo:hi], ["a", "b", "c"], forward_fn=fwd, max_batch=2, n_total=5,
                                    out=res, pending=pend)
        pend.wait()
        if rank == 0:
            assert out is res and torch.equal(out, ref), "segments n_total"
        # N smaller than the world: empty blocks on the last ranks
        out = separate_segments(None, segs[:1], ["a", "b", "c"], forward_fn=fwd, max_batch=2)
        if rank == 0:
            assert torch.equal(out, ref[:1]), "segments N=1"
        # --- one track, windows sharded over ranks
        L = 25000
        mix = torch.randn(2, L)
        stems = ["drums", "vocals"]
        plan = window_plan(L, SR, SEG, OV)
        chunk = int(SR * SEG)
        got = separate_track_sharded(
            None, mix, stems, SR, SEG, OV,
            window_fn=lambda a, b: _fake_model_windows(mix, plan, stems, chunk, a, b),
            ola_fn=lambda win, a, b: _oracle_span(win, a, b, L))
        if rank == 0:
            n = len(plan)
            ref = torch.zeros((2, 2, L)) + _oracle_span(_fake_model_windows(mix, plan, stems, chunk, 0, n), 0, n, L)
            assert torch.equal(got, ref), (got - ref).abs().max()
        # --- the benchmark.py protocol (1.5 s overlap analogue, zero-padded last window, weighted OLA)
        for Lb in (25000, 6000 * 3 + 17, 4000):
            mixb = torch.randn(2, Lb, generator=torch.Generator().manual_seed(Lb))
            got = separate_track_sharded(None, mixb, stems, SR, SEG, 1.5, protocol="benchmark",
                                         window_fn=lambda a, b: _bench_windows(mixb, stems, a, b),
                                         ola_fn=lambda win, a, b: _bench_partial(win, a, b, Lb))
            if rank == 0:
                for si in range(len(stems)):
                    refb = benchmark_chunked_inference(lambda c: _fake_stem(c, si), mixb, SR, SEG, 1.5)
                    assert torch.equal(got[si], refb), (Lb, si, (got[si] - refb).abs().max())
            else:
                assert got is None
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))


def test_shard_range():
    from athd.dist import shard_range
    assert [shard_range(5, 2, r) for r in range(2)] == [(0, 3), (3, 5)]
    assert [shard_range(3, 8, r) for r in range(8)][3:] == [(3, 3)] * 5
    for n in range(0, 40):
        for w in (1, 2, 3, 8):
            blocks = [shard_range(n, w, r) for r in range(w)]
            assert sum(b - a for a, b in blocks) == n and all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))


def test_world2_gloo():
    # spawn, not fork: a child forked after the parent used torch's CPU thread pool can deadlock
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in ps:
            r, msg = q.get(timeout=240)
            res[r] = msg
    finally:
        for p in ps:
            p.join(timeout=20)
            if p.is_alive():
                p.kill()
                p.join(timeout=5)
    assert res == {0: "ok", 1: "ok"}, res
