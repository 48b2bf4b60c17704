"""Throughput bench of the MI355X-native AudioTextHTDemucs hot path.

Workload (BASELINE.json configs[2]): per GPU a batch of B=64 synthetic 6 s 44.1 kHz stereo segments, each
separated into all 4 stems (drums/bass/other/vocals) - encode once, decode 4x (athd_forward_prompts).  A "step"
is one such batch.  `value` = segments/s over all ranks (each segment fully separated into 4 stems).
Multi-GPU: one process per GPU (torchrun), segments sharded across ranks (weak scaling), no data-path
collective; timing = barrier + sync around K steps, max over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--dtype bf16|f32] [--no-cpu-baseline]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "audio-to-sheet-music_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

SEG = 264600
STEMS = ["drums", "bass", "other", "vocals"]
# Essential FLOPs: encode 87.03 GMAC + per-prompt 10.31 GMAC
ENC_GMAC, DEC_GMAC = 87.03, 10.31
BF16_PEAK_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md chip table)
F32_PEAK_TFLOPS = 157.3
HBM_PEAK_GBS = 8000.0
MFMA_KERNELS = ("gemm", "attn")   # kernel-name prefixes priced against the MFMA peak; the rest against HBM
ROOF_STEPS = 2
PMC_FILE = os.environ.get("ATHD_PMC_TRAFFIC", os.path.join(REPO, "profiles", "pmc_traffic.json"))


def pmc_traffic(kernel, batch, dtype):
    """HBM bytes per launch of `kernel` measured by tools/pmc_traffic.py (rocprofv3 FETCH_SIZE / WRITE_SIZE in
    separate passes, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM) for this build and workload, else None."""
    try:
        d = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None, None
    if d.get("batch") != batch or d.get("dtype") != dtype:
        return None, None
    k = d.get("kernels", {}).get(kernel)
    return (k["hbm_bytes_per_launch"], os.path.relpath(PMC_FILE, REPO)) if k else (None, None)


def cpu_baseline(sd, table, budget_s=15.0):
    """Oracle (PyTorch-CPU restatement of the reference forward) on the host cores, reference protocol:
    one forward per (segment, prompt)."""
    from oracle.athtdemucs_ref import AudioTextHTDemucsRef
    from athd.synth import synthetic_batch
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    m = AudioTextHTDemucsRef(sd)
    wav = torch.as_tensor(synthetic_batch(1, SEG, seed0=4242))
    te = torch.as_tensor(table[3:4])
    m.forward(wav, te)                       # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        m.forward(wav, te)
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= 20:
            break
    per_fwd = el / n
    return {"value": 1.0 / (4 * per_fwd), "unit": "6s-segments/s (4 stems each)", "cores": threads,
            "kind": "port", "sample": f"{n} x forward(B=1, T=264600, 1 prompt) = {n} (segment,prompt) pairs, "
                                      f"{per_fwd * 1e3:.0f} ms each; 4 forwards per segment"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dump-kernels", default=None, help="write the warmup step's per-kernel profile (JSON)")
    ap.add_argument("--kernel", default=None, help="roofline kernel (default: largest summed time in warmup)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_batch
    from athd.weights import synthetic_state_dict, synthetic_text_table

    sd = synthetic_state_dict(seed=0)
    table = synthetic_text_table(4, seed=7)
    model = AudioTextHTDemucs(dtype=args.dtype, text_table={s: table[i] for i, s in enumerate(STEMS)})
    model.load_state_dict(sd)
    model = model.to(dev).eval()
    B = args.batch
    # distinct synthetic segments per rank (weak scaling: each rank owns its shard of segments)
    base = synthetic_batch(min(B, 8), SEG, seed0=1000 + 64 * rank)
    wav = torch.as_tensor(np.concatenate([base] * ((B + len(base) - 1) // len(base)))[:B]).to(dev)

    def step():
        return model.forward_prompts(wav, STEMS)

    # warmup; the last warmup step times every kernel (HIP events) to find the dominant one
    for i in range(args.warmup):
        if i == args.warmup - 1:
            model.profile_start(None)
        step()
    torch.cuda.synchronize()
    dominant = args.kernel
    if args.warmup > 0:
        allk = model.profile_stop()
        if args.dump_kernels and rank == 0:
            for r in allk:
                r["tflops"] = r["flops"] / (r["ms"] * 1e-3) / 1e12 if r["ms"] else 0.0
                r["gbs"] = r["bytes"] / (r["ms"] * 1e-3) / 1e9 if r["ms"] else 0.0
            json.dump(sorted(allk, key=lambda r: -r["ms"]), open(args.dump_kernels, "w"), indent=1)
        if dominant is None:
            dominant = max(allk, key=lambda r: r["ms"])["kernel"]
    if dominant is None:
        dominant = "gemm3_kernel<256,192,4,2,2,200>"

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    # roofline kernel: every launch of it bracketed with HIP events on its launch stream, over ROOF_STEPS further
    # steps outside the timed region (with a profile open the library runs the freq / time branches serially on one
    # stream, so the events time the kernel alone rather than sharing the chip with the other branch)
    model.profile_start(dominant)
    for _ in range(ROOF_STEPS):
        step()
    torch.cuda.synchronize()
    prof = model.profile_stop()
    if world > 1:
        t = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    ms = el / args.steps * 1e3
    value = B * world * args.steps / el
    flops_step = 2e9 * (ENC_GMAC + 4 * DEC_GMAC) * B
    step_tf = flops_step / (ms * 1e-3) / 1e12
    kp = next((r for r in prof if r["kernel"] == dominant), None)
    if kp is None or kp["launches"] == 0:
        raise RuntimeError(f"roofline kernel {dominant!r} was not launched in the timed region")
    per_launch_ms = kp["ms"] / kp["launches"]
    roof_step_ms = ms
    if dominant.startswith(MFMA_KERNELS):
        peak = BF16_PEAK_TFLOPS if args.dtype == "bf16" else F32_PEAK_TFLOPS
        ach = kp["flops"] / (kp["ms"] * 1e-3) / 1e12
        bound, unit = "mfma", "TFLOP/s"
    else:
        peak, bound, unit = HBM_PEAK_GBS, "hbm", "GB/s"
        ach = kp["bytes"] / (kp["ms"] * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(dominant, B, args.dtype)
    roofline = {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
                "traffic": traffic, "kernel": dominant, "launches_per_step": kp["launches"] / ROOF_STEPS,
                "avg_launch_us": round(per_launch_ms * 1e3, 2),
                "share_of_step": round(kp["ms"] / ROOF_STEPS / roof_step_ms, 4),
                "algorithmic_per_launch": {"flops": kp["flops"] / kp["launches"],
                                           "bytes": kp["bytes"] / kp["launches"]},
                "timing": f"HIP events on the launch stream around every launch of the kernel, {ROOF_STEPS} steps after the timed region (branches serialised on one stream)"}
    if traffic_src:
        roofline["traffic_source"] = traffic_src
    rec = {
        "metric": "6s-segments/sec (each separated into 4 stems; encode once, decode 4x)",
        "value": round(value, 3),
        "unit": "segments/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (seeded tones+noise 6 s stereo, seeded random weights of the htdemucs/AudioTextHTDemucs architecture)",
        "config": {"workload": "BASELINE configs[2]: B=64 x 6 s segments x 4 prompts per GPU", "global_batch": B * world,
                   "seq_len": SEG, "prompts": 4, "parallelism": f"segment-sharded dp{world}"},
        "stems_per_s": round(4 * value, 3),
        "roofline": roofline,
        "step_essential_tflops": round(step_tf, 2),
        "workspace_gb": round(model._ws.numel() / 1e9, 2) if model._ws is not None else None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(sd, table)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    del out


if __name__ == "__main__":
    main()
