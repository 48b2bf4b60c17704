"""Library GEMM reference points for the transformer shapes (torch.matmul -> hipBLASLt/rocBLAS), for DESIGN's
comparison of the hand-written gemm5 against the vendor library.  Not part of the product path."""
import torch, json
torch.manual_seed(0)
dev = "cuda"
res = []
for name, M, K, N in [("linear1.freq", 132608, 512, 2048), ("linear1.time", 66176, 512, 2048),
                      ("linear2.freq", 132608, 2048, 512), ("qkv.freq", 132608, 512, 1536)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=dev, dtype=torch.bfloat16)
    for mode in ("plain", "bias"):
        f = (lambda: torch.matmul(a, w.t())) if mode == "plain" else (lambda: torch.nn.functional.linear(a, w, b))
        for _ in range(3): f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n): f()
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        res.append({"gemm": name, "mode": mode, "M": M, "K": K, "N": N, "ms": round(ms, 4),
                    "tflops": round(2 * M * K * N / ms / 1e9, 1)})
        print(json.dumps(res[-1]), flush=True)
