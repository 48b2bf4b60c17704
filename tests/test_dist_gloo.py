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


def _fake_forward(wav, o, n_stems=4):
    """(b, 2, T) windows -> (b, S, 2, T) stand-in stems; returns a NEW tensor (never fills `o`), the forward_fn
    contract separate_segments must also accept on dst."""
    return torch.stack([_fake_stem(wav, si) for si in range(n_stems)], dim=1)


def _write_split(root, lengths, sr):
    """A synthetic MUSDB18-HQ split: one directory per track with mixture/drums/bass/other/vocals.wav (float)."""
    from athd.musdb import HQ_FILES, write_wav
    g = torch.Generator().manual_seed(5)
    for i, L in enumerate(lengths):
        d = os.path.join(root, f"track {i:02d}")
        os.makedirs(d, exist_ok=True)
        for f in HQ_FILES:
            write_wav(os.path.join(d, f + ".wav"), (0.3 * torch.randn(2, L, generator=g)).numpy(), sr, "FLOAT")


def _dataset_checks(rank, world, split_dir, out_dir):
    """separate_dataset over a 3-track split (benchmark protocol and the dataloader's non-overlapping segments)
    == per-track benchmark_chunked_inference + oracle metrics, and save_results' layout."""
    import json
    from athd.dist import separate_dataset
    from athd.musdb import MusDBTracks
    from athd.weights import STEMS
    from oracle.athtdemucs_ref import sdr_db, sisdr_db
    tracks = MusDBTracks(split_dir, sample_rate=SR)
    metric = lambda e, r: (sdr_db(e[None], r[None]), sisdr_db(e[None], r[None]))          # noqa: E731

    def ola(win, L, chunk, ov):
        hop = chunk - ov
        out, wsum = torch.zeros((win.shape[1], 2, L)), torch.zeros(L)
        for k in range(win.shape[0]):
            s, e = k * hop, min(k * hop + chunk, L)
            a = e - s
            fl = min(ov, a // 2)
            w = torch.ones(a)
            if s > 0 and fl > 0:
                w[:fl] = torch.linspace(0, 1, fl)
            if e < L and fl > 0:
                w[-fl:] = torch.linspace(1, 0, fl)
            out[:, :, s:e] += win[k, :, :, :a] * w
            wsum[s:e] += w
        return out / wsum.clamp(min=1e-8)

    hop = lambda ovs: int(SEG * SR) - int(ovs * SR)                                         # noqa: E731
    for ovs, gw in ((1.5, None), (0.0, None), (1.5, 1), (0.0, 1)):
        st = {}
        res = separate_dataset(None, tracks, STEMS, segment_seconds=SEG, overlap=ovs, sample_rate=SR, max_batch=2,
                               forward_fn=_fake_forward, ola_fn=ola, metric_fn=metric, keep_estimates=True,
                               output_dir=out_dir if (rank == 0 and ovs and gw is None) else None, log=None,
                               group_windows=gw, stats=st)
        wins = [-(-L // hop(ovs)) for L in tracks.lengths()]
        if gw == 1:
            # several track-aligned gather groups; dst's buffer holds the longest track's windows (the
            # smallest cap), not the split's
            assert st["groups"] > 1, st
            assert st["buffer_rows"] == (max(wins) if rank == 0 else 0), (st, wins)
            assert max(wins) < sum(wins)
        else:
            assert st["buffer_rows"] == (min(sum(wins), max(4 * world * 2, max(wins))) if rank == 0 else 0), st
        if rank != 0:
            assert res is None
            continue
        results, est = res
        assert [r.track_name for r in results] == [tracks.name(i) for i in range(len(tracks))]
        for i, r in enumerate(results):
            name, mix, refs = tracks.track(i)
            for si, s in enumerate(STEMS):
                want = benchmark_chunked_inference(lambda c: _fake_stem(c, si), mix, SR, SEG, ovs)
                assert torch.equal(est[name][si], want), (ovs, name, s)
                sd, ss = metric(want, refs[s])
                assert getattr(r, f"sdr_{s}") == sd and getattr(r, f"sisdr_{s}") == ss, (ovs, name, s)
    if rank == 0:
        saved = json.load(open(os.path.join(out_dir, "evaluation_results.json")))
        (mname, body), = saved.items()
        assert mname == "AudioTextHTDemucs (Ours)" and set(body) == {"per_track", "aggregate"}
        assert [p["track"] for p in body["per_track"]] == [tracks.name(i) for i in range(len(tracks))]
        assert set(body["per_track"][0]["sdr"]) == set(STEMS) | {"average"}
        assert set(body["aggregate"]) == {"sdr", "sisdr"}


def _worker(rank, world, port, q, split_dir=None, out_dir=None):
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
        # bench.py's N>1 call pattern: block-local input, `out` slices on rank 0, transfers left pending across
        # 3 steps of >= 3 batches per rank with at most 2 in flight (PendingSends(limit=2)); forward_fn returns a
        # new tensor (copied into `out` on rank 0)
        lo, hi = shard_range(14, world, rank)
        segs14 = torch.randn(14, 2, 300, generator=torch.Generator().manual_seed(14))
        ref14 = torch.stack([_fake_stem(segs14, si) for si in range(4)], dim=1)
        pend = PendingSends(limit=2)
        res = torch.full((14, 4, 2, 300), float("nan")) if rank == 0 else None
        peak = 0
        for _ in range(3):
            out = separate_segments(None, segs14[lo:hi], ["a", "b", "c", "d"], forward_fn=_fake_forward,
                                    max_batch=2, n_total=14, out=res, pending=pend)
            peak = max(peak, len(pend.works))
        pend.wait()
        assert peak <= 2, peak
        if rank == 0:
            assert out is res and torch.equal(out, ref14), "bench pattern"
        # bench.py's graph-replayed N>1 pattern: one batch per rank and step; rank 0's forward writes its own rows of
        # the gathered output in place (the graph is captured on out[0:B]); the other ranks alternate two send
        # buffers with PendingSends(limit=1), so a step never rewrites a buffer whose send may be in flight
        B = 3
        lo, hi = shard_range(B * world, world, rank)
        blk = torch.randn(B, 2, 200, generator=torch.Generator().manual_seed(100 + rank))
        res = torch.full((B * world, 4, 2, 200), float("nan")) if rank == 0 else None
        bufs = [res[0:B]] if rank == 0 else [torch.empty(B, 4, 2, 200) for _ in range(2)]
        pend = PendingSends(limit=1 if rank else 2)
        calls = [0]

        def ping_pong(wav, o, scale):
            k = calls[0] % len(bufs)
            calls[0] += 1
            bufs[k].copy_(torch.stack([_fake_stem(wav * scale, si) for si in range(4)], dim=1))
            return bufs[k]

        for step in range(4):
            out = separate_segments(None, blk, ["a", "b", "c", "d"], forward_fn=lambda w, o: ping_pong(w, o, step + 1),
                                    max_batch=B, n_total=B * world, out=res, pending=pend)
            assert len(pend.works) <= (1 if rank else 2)
        pend.wait()
        if rank == 0:
            want = torch.cat([torch.randn(B, 2, 200, generator=torch.Generator().manual_seed(100 + r))
                              for r in range(world)])
            want = torch.stack([_fake_stem(want * 4, si) for si in range(4)], dim=1)
            assert out is res and torch.equal(res, want), "graph ping-pong pattern"
            assert calls[0] == 4
        else:
            assert calls[0] == 4
        if split_dir is not None:
            _dataset_checks(rank, world, split_dir, out_dir)
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


def test_world2_gloo(tmp_path):
    split = tmp_path / "test"
    _write_split(str(split), [25000, 6000 * 2 + 17, 4000], SR)
    # spawn, not fork: a child forked after the parent used torch's CPU thread pool can deadlock
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, str(split), str(tmp_path / "results")))
          for r in range(2)]
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
