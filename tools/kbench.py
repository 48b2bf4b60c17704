"""Time GEMM / attention kernel variants vs torch (hipBLASLt / SDPA) on the GPU box (tooling, not a test)."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
VARIANTS = (33, 40)
lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("KB_LIB", "libkbench.so")))
vp = ctypes.c_void_p


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def gemm_case(M, N, K, act=0):
    dev = "cuda"
    A = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    Kp = (K + 63) // 64 * 64
    W = torch.zeros(N, Kp, device=dev, dtype=torch.bfloat16)
    W[:, :K] = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=dev) * 0.1
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    ref = (A.float() @ W[:, :K].float().t() + bias)
    if act == 1:
        ref = torch.nn.functional.gelu(ref)
    flops = 2.0 * M * N * K
    res = {}
    for v in VARIANTS:
        f = lambda: lib.kb_gemm(v, vp(A.data_ptr()), 1, vp(W.data_ptr()), vp(bias.data_ptr()), vp(C.data_ptr()), 1,
                                M, N, K, Kp, act, vp(st))
        us = timeit(f)
        err = (C.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-9)
        res[f"v{v}"] = (us, flops / us / 1e6, err)
    Wt = W[:, :K].t().contiguous()
    us = timeit(lambda: torch.addmm(bias.to(torch.bfloat16), A, W[:, :K].t()))
    res["torch"] = (us, flops / us / 1e6, 0.0)
    print(f"GEMM M={M} N={N} K={K} act={act}: " + "  ".join(f"{k}: {v[0]:8.1f}us {v[1]:7.1f}TF err={v[2]:.1e}" for k, v in res.items()), flush=True)


def res_case(M, N, K, stats=False, variants=(50, 31, 131, 32, 132, 37, 137)):
    """transformer residual GEMM (out_proj: K = 512; linear2: K = 2048 with GroupNorm statistics), C f32 in place"""
    dev = "cuda"
    A = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    Kp = (K + 63) // 64 * 64
    W = torch.zeros(N, Kp, device=dev, dtype=torch.bfloat16)
    W[:, :K] = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=dev) * 0.1
    scale = torch.rand(N, device=dev) * 0.2
    R = torch.randn(M, N, device=dev)
    C = R.clone()
    st_buf = torch.zeros(2, device=dev, dtype=torch.float64) if stats else None
    s = torch.cuda.current_stream().cuda_stream
    ref = R + scale * (A.float() @ W[:, :K].float().t() + bias)
    flops = 2.0 * M * N * K
    hbm = M * K * 2 + 2 * M * N * 4
    res = {}
    for v in variants:
        C.copy_(R)
        rc = lib.kb_gemm_res(v, vp(A.data_ptr()), vp(W.data_ptr()), vp(bias.data_ptr()), vp(C.data_ptr()),
                             vp(scale.data_ptr()), vp(st_buf.data_ptr() if stats else 0), M, N, K, Kp, vp(s))
        if rc != 0:
            continue
        torch.cuda.synchronize()
        err = (C - ref).abs().max().item() / (ref.abs().max().item() + 1e-9)
        f = lambda: lib.kb_gemm_res(v, vp(A.data_ptr()), vp(W.data_ptr()), vp(bias.data_ptr()), vp(C.data_ptr()),
                                    vp(scale.data_ptr()), vp(st_buf.data_ptr() if stats else 0), M, N, K, Kp, vp(s))
        us = timeit(f)
        res[f"v{v}"] = (us, flops / us / 1e6, hbm / us / 1e3, err)
    print(f"RES GEMM M={M} N={N} K={K} stats={stats}: " + "  ".join(
        f"{k}: {v[0]:7.1f}us {v[1]:6.1f}TF {v[2]:6.0f}GB/s err={v[3]:.1e}" for k, v in res.items()), flush=True)


def convt_case(nb, H, Wd, Cin, Cout, variants):
    dev = "cuda"
    A = (torch.randn(nb, H, Wd, Cin, device=dev) * 0.5).to(torch.bfloat16)
    K = 2 * Cin
    Kp = (K + 63) // 64 * 64
    W = torch.zeros(2 * Cout, Kp, device=dev, dtype=torch.bfloat16)
    W[:, :K] = (torch.randn(2 * Cout, K, device=dev) * 0.05).to(torch.bfloat16)
    bias = torch.randn(2 * Cout, device=dev) * 0.1
    C = torch.zeros(nb, 2 * H, Wd, Cout, device=dev, dtype=torch.bfloat16)
    st = torch.zeros(2 * nb, device=dev, dtype=torch.float64)
    s = torch.cuda.current_stream().cuda_stream
    flops = 2.0 * nb * H * Wd * 2 * Cout * K
    # reference for row-slot 2u: columns >= Cout of [A[u-1] | A[u]] @ W^T + b
    Ap = torch.cat([torch.zeros_like(A[:, :1]), A], dim=1)                    # row -1 = 0
    X = torch.cat([Ap[:, :-1], Ap[:, 1:]], dim=-1).float()                    # (nb, H, Wd, 2Cin)
    ref = (X @ W[:, :K].float().t() + bias)[..., Cout:]
    out = []
    for v in variants:
        f = lambda: lib.kb_convt(v, vp(A.data_ptr()), vp(W.data_ptr()), vp(bias.data_ptr()), vp(C.data_ptr()),
                                 vp(st.data_ptr()), nb, H, Wd, Cin, Cout, Kp, vp(s))
        us = timeit(f)
        err = (C[:, 0::2].float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-9)
        out.append(f"v{v}: {us:8.1f}us {flops / us / 1e6:6.1f}TF err={err:.1e}")
    print(f"CONVT nb={nb} H={H} W={Wd} Cin={Cin} Cout={Cout}: " + "  ".join(out), flush=True)


def quad_case(nb, H, Wd, Cin, Cout, variants):
    dev = "cuda"
    A = (torch.randn(nb, H, Wd, Cin, device=dev) * 0.5).to(torch.bfloat16)
    K = 3 * Cin
    Kp = (K + 63) // 64 * 64
    W = torch.zeros(4 * Cout, Kp, device=dev, dtype=torch.bfloat16)
    W[:, :K] = (torch.randn(4 * Cout, K, device=dev) * 0.05).to(torch.bfloat16)
    W[:2 * Cout, 2 * Cin:K] = 0          # residues 0/1 never read row u+1, 2/3 never row u-1
    W[2 * Cout:, :Cin] = 0
    bias = torch.randn(4 * Cout, device=dev) * 0.1
    C = torch.zeros(nb, 2 * H, Wd, Cout, device=dev, dtype=torch.bfloat16)
    st = torch.zeros(2 * nb, device=dev, dtype=torch.float64)
    s = torch.cuda.current_stream().cuda_stream
    flops = 2.0 * nb * H * Wd * 4 * Cout * K
    z = torch.zeros_like(A[:, :1])
    X = torch.cat([torch.cat([z, A[:, :-1]], 1), A, torch.cat([A[:, 1:], z], 1)], dim=-1).float()
    ref = X @ W[:, :K].float().t() + bias                                     # (nb, H, Wd, 4 Cout)
    r1, r2 = ref[..., Cout:2 * Cout], ref[..., 2 * Cout:3 * Cout]
    rs = torch.stack([ref[..., i * Cout:(i + 1) * Cout] for i in range(4)]).double()
    out = []
    for v, ksk in variants:
        st.zero_()
        f = lambda: lib.kb_convt_quad(v, ksk, vp(A.data_ptr()), vp(W.data_ptr()), vp(bias.data_ptr()),
                                      vp(C.data_ptr()), vp(st.data_ptr()), nb, H, Wd, Cin, Cout, Kp, vp(s))
        st.zero_(); f(); torch.cuda.synchronize()
        sref = rs.sum(dim=(0, 2, 3, 4)).cpu()
        serr = ((st.view(nb, 2)[:, 0].cpu() - sref).abs().max() / sref.abs().max()).item()
        us = timeit(f)
        err = max((C[:, 0::2].float() - r1).abs().max().item(), (C[:, 1::2].float() - r2).abs().max().item())
        err /= ref.abs().max().item()
        out.append(f"v{v}{'s' if ksk else ''}: {us:8.1f}us {flops / us / 1e6:6.1f}TF err={err:.1e} serr={serr:.1e}")
    print(f"QUAD nb={nb} H={H} W={Wd} Cin={Cin} Cout={Cout}: " + "  ".join(out), flush=True)


def attn_case(B, N, variants=(1, 0, 2, 3)):
    qkv = (torch.randn(B, N, 1536, device="cuda")).to(torch.bfloat16)
    qkvp = qkv.clone()
    qkvp[..., :512] = (qkv[..., :512].float() * (0.125 * 1.4426950408889634)).to(torch.bfloat16)
    out = torch.empty(B, N, 512, device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    flops = 4.0 * B * 8 * N * N * 64
    q, k, v = qkv.view(B, N, 3, 8, 64).permute(2, 0, 3, 1, 4)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v)
    res = []
    for var in variants:
        for pre, src in ((0, qkv), (1, qkvp)):
            if var != 1 and not pre:
                continue
            if var == 1 and pre:
                continue
            f = lambda: lib.kb_attn(var, pre, vp(src.data_ptr()), B, N, vp(out.data_ptr()), vp(st))
            out.zero_()
            us = timeit(f)
            err = (out.view(B, N, 8, 64).permute(0, 2, 1, 3).float() - ref.float()).abs().max().item()
            res.append(f"v{var}: {us:8.1f}us {flops / us / 1e6:7.1f}TF err={err:.1e}")
    ust = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v))
    print(f"ATTN B={B} N={N}: " + " | ".join(res) + f" | torch sdpa {ust:8.1f}us {flops / ust / 1e6:7.1f}TF", flush=True)


def attn_acc(B, N, scales=(1.0, 4.0, 6.0), ramp=(0.0, 8.0)):
    """Accuracy of the product attention kernel (v0) against torch SDPA in fp32 on bf16 inputs whose logit range forces
    the rescale path: Q and K scaled (logits x scale^2) and a per-key ramp added along the key axis through an extra
    channel pair (later keys score higher, so later tiles exceed the first tile's max)."""
    st = torch.cuda.current_stream().cuda_stream
    for sc in scales:
        for rp in ramp:
            g = torch.Generator(device="cuda").manual_seed(int(sc * 10 + rp))
            qkv = torch.randn(B, N, 1536, device="cuda", generator=g)
            qkv[..., :1024] *= sc
            if rp:
                # head dim 63 of q = 1, of k = ramp * key / N  (adds ramp * key / N to every logit of the key)
                qkv.view(B, N, 3, 8, 64)[:, :, 0, :, 63] = 1.0
                qkv.view(B, N, 3, 8, 64)[:, :, 1, :, 63] = (rp * 8.0 * torch.arange(N, device="cuda") / N)[None, :, None]
            qkv = qkv.to(torch.bfloat16)
            qkvp = qkv.clone()
            qkvp[..., :512] = (qkv[..., :512].float() * (0.125 * 1.4426950408889634)).to(torch.bfloat16)
            q, k, v = qkv.float().view(B, N, 3, 8, 64).permute(2, 0, 3, 1, 4)
            ref = torch.nn.functional.scaled_dot_product_attention(q, k, v)
            out = torch.zeros(B, N, 512, device="cuda", dtype=torch.bfloat16)
            lib.kb_attn(0, 1, vp(qkvp.data_ptr()), B, N, vp(out.data_ptr()), vp(st))
            torch.cuda.synchronize()
            o = out.view(B, N, 8, 64).permute(0, 2, 1, 3).float()
            err = (o - ref).abs().max().item()
            sdr = 10 * torch.log10((ref ** 2).sum() / ((o - ref) ** 2).sum()).item()
            print(f"ATTNACC B={B} N={N} scale={sc} ramp={rp}: maxerr={err:.2e} sdr={sdr:.2f} dB finite={bool(torch.isfinite(o).all())}",
                  flush=True)


def tr_probe():
    out = torch.zeros(64, 4, dtype=torch.int16, device="cuda")
    lib.kb_tr(vp(out.data_ptr()))
    o = out.cpu().numpy().astype(int)
    for lane in range(0, 64, 5):
        print(f"TR lane {lane:2d}: " + " ".join(f"({v // 256},{v % 256})" for v in o[lane]), flush=True)


def g4_stamps(M, N, K, act=0):
    """Per-block s_memtime stamps of one gemm4 launch: where a 256x256 tile's time goes."""
    import numpy as np
    dev = "cuda"
    A = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    Kp = (K + 63) // 64 * 64
    W = (torch.randn(N, Kp, device=dev) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=dev) * 0.1
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    buf = torch.zeros(tiles * 24, dtype=torch.int64, device=dev)
    run = lambda: lib.kb_gemm(int(os.environ.get("G4V", "40")), vp(A.data_ptr()), 1, vp(W.data_ptr()), vp(bias.data_ptr()), vp(C.data_ptr()), 1,
                              M, N, K, Kp, act, vp(st))
    run()
    lib.athd_g4_stamp_set(vp(buf.data_ptr()))
    run()
    torch.cuda.synchronize()
    lib.athd_g4_stamp_set(vp(0))
    s = buf.view(tiles, 24).cpu().numpy()
    n = int(s[0, 23])
    t0 = s[:, 0].min()
    rel = s[:, :n] - t0
    names = ["start", "issued", "kt0", "kt1", "ktlast", "epi", "epi_iss", "end"][:n]
    d = np.diff(s[:, :n], axis=1)
    print(f"G4STAMP M={M} N={N} K={K}: tiles={tiles} stamps={n} span={(s[:, n-1].max() - t0)} (s_memtime ticks)")
    for i in range(n - 1):
        print(f"  {names[i]:>7s}->{names[i+1]:<7s} median {np.median(d[:, i]):9.0f}  p10 {np.percentile(d[:, i], 10):9.0f}  p90 {np.percentile(d[:, i], 90):9.0f}")
    e = s[:, 12:16].astype(np.int64)
    ep = s[:, 5].astype(np.int64)
    print("  epilogue marks rel. to 'epi' (bias loaded, rows start, row 1, rows done):",
          [int(np.median(e[:, k] - ep)) for k in range(4)])
    # per CU: blocks in start order; busy = sum(start -> epilogue issued), gap = next start - this block's end
    hw = s[:, 21] & 0xFFFFFFFF
    xcc = s[:, 22] & 0xF
    cu_key = xcc * 100000 + ((hw >> 13) & 7) * 1000 + ((hw >> 12) & 1) * 100 + ((hw >> 8) & 15)
    gaps, busy_frac, inflight = [], [], []
    for key in np.unique(cu_key):
        idx = np.where(cu_key == key)[0]
        st = s[idx, 0]
        o = np.argsort(st)
        st = st[o]
        ei = s[idx, 6][o]
        en = s[idx, 7][o]
        span = en.max() - st.min()
        busy_frac.append((ei - st).sum() / max(span, 1))
        gaps.extend(list(st[1:] - en[:-1]))
        inflight.append(len(idx))
    gaps = np.array(gaps)
    print(f"  CUs={len(busy_frac)} blocks/CU median {np.median(inflight):.0f}; per-CU sum(start->epi issued)/span median {np.median(busy_frac):.2f}")
    print(f"  gap next-start minus prev-end: median {np.median(gaps):.0f} p10 {np.percentile(gaps, 10):.0f} p90 {np.percentile(gaps, 90):.0f}")


if __name__ == "__main__":
    torch.manual_seed(0)
    if "stamp" in sys.argv[1:]:
        g4_stamps(64 * 2072, 1536, 512)
        g4_stamps(64 * 2072, 512, 2048)
        g4_stamps(64 * 2072, 2048, 512, act=1)
        sys.exit(0)
    if "tr" in sys.argv[1:]:
        tr_probe()
    if "quad" in sys.argv[1:]:
        vs = [(3, 1), (103, 1), (7, 1), (107, 1), (3, 3), (103, 3)]
        quad_case(64, 259, 259, 96, 48, vs)
        quad_case(64, 16538, 1, 96, 48, vs)
        if "contention" in sys.argv[1:]:    # same rows, statistics groups of 1 / 64 / 2368 batches
            quad_case(1, 64 * 259, 259, 96, 48, [(3, 1), (3, 3)])
            quad_case(2368, 7, 259, 96, 48, [(3, 1), (3, 3)])
        sys.exit(0)
    if "convt" in sys.argv[1:]:
        convt_case(64, 259, 259, 192, 96, (2, 33, 34, 35))
        convt_case(64, 259, 259, 96, 48, (2, 34, 35, 36))
        convt_case(64, 1034, 1, 384, 192, (2, 33, 34, 35))
        sys.exit(0)
    if "attn1" in sys.argv[1:]:          # one shape, for PMC passes
        vs = tuple(int(v) for v in os.environ.get("ATTN_VARIANTS", "1,0,2").split(","))
        attn_case(64, 2072, vs)
        sys.exit(0)
    if "attn" in sys.argv[1:]:
        av = tuple(int(x) for x in os.environ.get("ATTN_VARIANTS", "1,0,2,3").split(","))
        attn_case(4, 200, av)
        attn_case(2, 67, av)
        attn_case(64, 2072, av)
        attn_case(64, 1034, av)
        sys.exit(0)
    M = 64 * 2072
    if "persist" in sys.argv[1:]:
        VARIANTS = (33, 133, 37, 137)
        gemm_case(M, 1536, 512)
        gemm_case(M, 512, 2048)
        gemm_case(M, 512, 512)
        gemm_case(64 * 259 * 259, 192, 384)
        gemm_case(64 * 259 * 259, 96, 192)
        sys.exit(0)
    if "nostore" in sys.argv[1:]:
        VARIANTS = (40, 41, 42)
        gemm_case(M, 1536, 512)
        gemm_case(M, 2048, 512, act=1)
        gemm_case(M, 512, 2048)
        gemm_case(M, 512, 512)
        sys.exit(0)
    if "zgemm" in sys.argv[1:]:           # the decoder's level-1 tap GEMM (fdec1.z): M = 256 items x 32 x 259, K = 192
        VARIANTS = (40, 38, 108, 37, 137, 33, 133)
        gemm_case(256 * 32 * 259, 768, 192)
        gemm_case(M, 1536, 512)
        sys.exit(0)
    if "g5var" in sys.argv[1:]:               # gemm5 schedule variants: 55 no sleep, 56 early + no sleep, 57 early
        VARIANTS = (40, 50, 55, 56, 57)
        for _ in range(2):
            gemm_case(4096, 4096, 4096)
            gemm_case(M, 512, 2048)
            gemm_case(M, 1536, 512)
            gemm_case(M, 2048, 512, act=1)
            gemm_case(M, 512, 512)
        sys.exit(0)
    if "quant" in sys.argv[1:]:               # tile quantisation: 1024 vs 1036 256x256 tiles (N 512), time branch 518
        VARIANTS = (50,)
        for _ in range(2):
            for m in (131072, M, 64 * 1034, 65536):
                gemm_case(m, 512, 2048)
                gemm_case(m, 512, 512)
        sys.exit(0)
    if "g5probe" in sys.argv[1:]:             # gemm5 ablations: 51 no staging, 52 no fragment reads, 53 no MFMA, 54 no barriers
        VARIANTS = (40, 50, 51, 52, 53, 54)
        gemm_case(4096, 4096, 4096)
        gemm_case(M, 512, 2048)
        gemm_case(M, 1536, 512)
        sys.exit(0)
    if "res" in sys.argv[1:]:                 # residual-epilogue GEMMs: gemm5 vs gemm3 tiles (+100: persistent)
        for _ in range(2):
            res_case(M, 512, 512)
            res_case(M, 512, 2048, stats=True)
            res_case(64 * 259, 512, 512)
        sys.exit(0)
    if "g5" in sys.argv[1:]:
        VARIANTS = (40, 50)
        for _ in range(2):
            gemm_case(M, 1536, 512)
            gemm_case(M, 2048, 512, act=1)
            gemm_case(M, 512, 2048)
            gemm_case(M, 512, 512)
            gemm_case(4096, 4096, 4096)
            gemm_case(256 * 32 * 259, 768, 192)
        sys.exit(0)
    if "attnacc" in sys.argv[1:]:
        attn_acc(8, 2072)
        attn_acc(8, 1034)
        sys.exit(0)
    if "g4" in sys.argv[1:]:
        gemm_case(M, 1536, 512)
        gemm_case(M, 2048, 512, act=1)
        gemm_case(M, 512, 2048)
        gemm_case(M, 512, 512)
        gemm_case(4096, 4096, 4096)
        gemm_case(M, 1536, 512)
        sys.exit(0)
    gemm_case(M, 1536, 512)
    gemm_case(M, 2048, 512, act=1)
    gemm_case(M, 512, 2048)
    gemm_case(M, 512, 512)
    gemm_case(64 * 259 * 259, 192, 384)
    gemm_case(64 * 259 * 259, 96, 192)
    attn_case(64, 2072)
    attn_case(64, 1034)
