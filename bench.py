"""Throughput bench of the MI355X-native AudioTextHTDemucs hot path.

Workload (BASELINE.json configs[2]): per GPU a batch of B=64 distinct synthetic 6 s 44.1 kHz stereo segments, each
separated into all 4 stems (drums/bass/other/vocals) - encode once, decode 4x (athd_forward_prompts).  A "step" is
one such batch per GPU.  `value` = segments/s over all ranks (each segment fully separated into 4 stems).
Multi-GPU (configs[3] shape): one process per GPU (torchrun), segments sharded across ranks (weak scaling); every
step runs athd.dist.separate_segments, so the point-to-point RCCL gather of all separated waveforms to rank 0
(xGMI) is inside the timed region, overlapped with the next step's compute.  Timing = barrier + sync around K steps,
max over ranks.

Beside the headline (all outside the timed region, rank 0): the roofline of the dominant kernel (HIP events) and of
each forward section, the whole-step MFMA fraction, the bf16 output's SDR against the fp32 oracle, an f32-mode
(parity mode) throughput line, and the CPU baseline (the oracle on the host's cores).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--dtype bf16|f32] [--no-cpu-baseline]
"""
import argparse
import json
import os
import statistics
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
MFMA_KERNELS = ("gemm", "attn", "fenc_row")   # kernel-name prefixes priced against the MFMA peak; the rest HBM
ROOF_STEPS = 2
PMC_FILE = os.environ.get("ATHD_PMC_TRAFFIC", os.path.join(REPO, "profiles", "pmc_traffic.json"))


def pmc_traffic(kernel, batch, dtype):
    """HBM bytes per launch of `kernel` measured by tools/pmc_traffic.py (rocprofv3 FETCH_SIZE / WRITE_SIZE in
    separate passes, corrected per MI355X_MICROARCH.md §HBM) for this build and workload, else None."""
    try:
        d = json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None, None
    if d.get("batch") != batch or d.get("dtype") != dtype:
        return None, None
    ks = d.get("kernels", {})
    k = ks.get(kernel)
    if k is None:
        # the library labels some kernels without their template arguments (attn32_kernel); rocprofv3 names the
        # instantiation: accept the one instantiation of that name
        inst = [v for n, v in ks.items() if n.split("<", 1)[0] == kernel]
        k = inst[0] if len(inst) == 1 else None
    return (k["hbm_bytes_per_launch"], os.path.relpath(PMC_FILE, REPO)) if k else (None, None)


def cpu_info():
    """(threads usable by this process, host logical CPUs, CPU model).  Usable = the process's CPU affinity,
    capped by the cgroup CPU quota (the GPU box grants each job a share of the host: os.cpu_count() there counts the
    whole machine, and running that many threads on the share would oversubscribe it)."""
    host = os.cpu_count() or 1
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else host
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            usable = min(usable, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, host, model


def cpu_baseline(sd, table):
    """The oracle (PyTorch-CPU restatement of the reference forward, same torch ops) on the host cores with the
    reference protocol (one forward per (segment, prompt)), SURVEY.md §8(d): median of 5 timed forwards after 1
    warm-up, at B=1 (test_inference's batch) and B=8."""
    from oracle.athtdemucs_ref import AudioTextHTDemucsRef
    from athd.synth import synthetic_batch
    threads, host, model = cpu_info()
    torch.set_num_threads(threads)
    m = AudioTextHTDemucsRef(sd)
    res = {}
    for B in (1, 8):
        wav = torch.as_tensor(synthetic_batch(B, SEG, seed0=4242))
        te = torch.as_tensor(table[3:4]).expand(B, -1).contiguous()
        m.forward(wav, te)                                  # warm-up
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            m.forward(wav, te)
            ts.append(time.perf_counter() - t0)
        res[B] = statistics.median(ts)
    per1, per8 = res[1], res[8] / 8
    return {"value": round(1.0 / (4 * per1), 4), "unit": "6s-segments/s (4 stems each: 4 forwards per segment)",
            "cores": threads, "host_cores": host, "cpu_model": model, "kind": "port",
            "b8": {"value": round(1.0 / (4 * per8), 4), "ms_per_forward": round(res[8] * 1e3, 1)},
            "sample": f"median of 5 (after 1 warm-up) forward(B=1, T=264600, 1 prompt) = {per1 * 1e3:.0f} ms; "
                      f"forward(B=8) = {res[8] * 1e3:.0f} ms; {threads} torch threads"}


def sdr_vs_oracle(model, sd, table, wav0):
    """SDR (dB) of this model's output for one segment x 4 prompts against the fp32 oracle forward (north_star:
    'SDR delta reported'); min and mean over the prompts."""
    from oracle.athtdemucs_ref import AudioTextHTDemucsRef
    got = model.forward_prompts(wav0, STEMS).cpu().double()[0]
    ref = AudioTextHTDemucsRef(sd).forward_prompts(wav0.cpu(), torch.as_tensor(table)).double()[0]
    s = [float(10 * torch.log10((ref[p] ** 2).sum() / ((ref[p] - got[p]) ** 2).sum())) for p in range(4)]
    return {"min": round(min(s), 2), "mean": round(sum(s) / 4, 2), "per_prompt": [round(x, 2) for x in s],
            "what": "SDR of the bench dtype's output vs the fp32 oracle, segment 0 x 4 prompts (unclamped)"}


def f32_line(sd, table, wav, steps=3):
    """Throughput of the f32 parity mode (fp32 MFMA everywhere) on the same batch, outside the headline."""
    from athd.model import AudioTextHTDemucs
    m = AudioTextHTDemucs(dtype="f32", text_table={s: table[i] for i, s in enumerate(STEMS)})
    m.load_state_dict(sd)
    m = m.to(wav.device).eval()
    m.forward_prompts(wav, STEMS)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        m.forward_prompts(wav, STEMS)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms = el / steps * 1e3
    tf = 2e9 * (ENC_GMAC + 4 * DEC_GMAC) * wav.shape[0] / (ms * 1e-3) / 1e12
    out = {"value": round(wav.shape[0] * steps / el, 3), "unit": "segments/s", "ms_per_step": round(ms, 3),
           "steps": steps, "warmup": 1, "step_essential_tflops": round(tf, 2),
           "frac_of_f32_mfma_peak": round(tf / F32_PEAK_TFLOPS, 4)}
    del m
    torch.cuda.empty_cache()
    return out


def dataset_pass(model, wav, n, batch, world, rank, dev):
    """BASELINE configs[3]: n segments sharded over the ranks in contiguous blocks (each rank's block resident in
    HBM: distinct segments derived from its bench batch by a per-segment roll and gain), each separated into 4 stems
    in batches of `batch` by athd.dist.separate_segments, every result gathered point to point into one
    preallocated (n, 4, 2, T) tensor on rank 0.  Timed: barrier + sync on both sides of the whole pass, max over
    ranks (one pass after one untimed warm-up pass)."""
    from athd.dist import separate_segments, shard_range
    lo, hi = shard_range(n, world, rank)
    blk = torch.empty((hi - lo, 2, SEG), dtype=torch.float32, device=dev)
    for j, i in enumerate(range(lo, hi)):
        blk[j] = torch.roll(wav[i % wav.shape[0]], shifts=(i * 7919) % SEG, dims=-1) * (0.5 + (i % 17) / 16.0)
    out = torch.empty((n, len(STEMS), 2, SEG), dtype=torch.float32, device=dev) if rank == 0 else None

    def run():
        separate_segments(model, blk, STEMS, max_batch=batch, n_total=n, out=out)

    run()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    return {"metric": "dataset pass: 6s-segments/sec (each separated into 4 stems), gather to rank 0 included",
            "value": round(n / el, 3), "unit": "segments/s", "n_gpus": world, "segments": n,
            "segments_per_rank": -(-n // world), "seconds": round(el, 4), "higher_is_better": True,
            "dtype": model.dtype, "data": "synthetic (rolled / scaled bench segments)",
            "config": {"workload": "BASELINE configs[3]: dataset of N segments batch-sharded over the GPUs, RCCL "
                                   "point-to-point gather of every separated waveform to rank 0",
                       "batch": batch, "prompts": 4, "parallelism": f"segment-sharded dp{world}"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the SDR, f32 and section measurements")
    ap.add_argument("--dump-kernels", default=None, help="write the warmup step's per-kernel profile (JSON)")
    ap.add_argument("--kernel", default=None, help="roofline kernel (default: largest summed time in warmup)")
    ap.add_argument("--pipelines", type=int, default=1,
                    help="N = 1: run the steps as this many concurrent forward pipelines (each its own context, "
                         "workspace, input batch, stream and graph), step i on pipeline i %% n")
    ap.add_argument("--eager", action="store_true",
                    help="launch every step's kernels from the host instead of replaying the captured HIP graph")
    ap.add_argument("--segments", type=int, default=0,
                    help="also time one dataset pass of N segments over all ranks (BASELINE configs[3]: ~6k MUSDB18 "
                         "test-set segments) through athd.dist.separate_segments; printed as a second JSON line")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from athd.dist import PendingSends, separate_segments
    from athd.model import AudioTextHTDemucs
    from athd.synth import synthetic_batch
    from athd.weights import synthetic_state_dict, synthetic_text_table

    sd = synthetic_state_dict(seed=0)
    table = synthetic_text_table(4, seed=7)
    B = args.batch
    # the whole per-GPU batch in one decode chunk (B x 4 items): fewer, larger decoder launches (≈49 GB: athd_workspace_bytes, reported as workspace_gb)
    model = AudioTextHTDemucs(dtype=args.dtype, text_table={s: table[i] for i, s in enumerate(STEMS)},
                              decode_items=B * len(STEMS))
    model.load_state_dict(sd)
    model = model.to(dev).eval()
    # B distinct synthetic segments per rank, resident in HBM before timing (weak scaling: each rank owns its block)
    wav = torch.as_tensor(synthetic_batch(B, SEG, seed0=1000 + B * rank)).to(dev)
    N = B * world
    out = torch.empty((N, len(STEMS), 2, SEG), dtype=torch.float32, device=dev) if rank == 0 else None
    pending = PendingSends(limit=2)          # at most two batches in flight per rank (bounded send buffers)

    # N = 1: one athd_forward_prompts captured into a HIP graph (both branch streams and their event joins), replayed
    # per step: the same kernels on the same buffers, without the host launch gaps between them
    graph = None
    if world == 1 and not args.eager:
        graph, _ = model.capture_prompts(wav, STEMS, out=out)
    # further pipelines (N = 1, --pipelines > 1): own model context, batch, output, stream and graph each
    pipes = []
    if world == 1 and graph is not None and args.pipelines > 1:
        for k in range(1, args.pipelines):
            mk = AudioTextHTDemucs(dtype=args.dtype, text_table={s: table[i] for i, s in enumerate(STEMS)},
                                   decode_items=B * len(STEMS))
            mk.load_state_dict(sd)
            mk = mk.to(dev).eval()
            wk = torch.as_tensor(synthetic_batch(B, SEG, seed0=1000 + B * (world + k))).to(dev)
            gk, _ = mk.capture_prompts(wk, STEMS)
            pipes.append((torch.cuda.Stream(dev), gk, mk, wk))
    nstep = [0]

    def step():
        if pipes:
            k = nstep[0] % (len(pipes) + 1)
            nstep[0] += 1
            if k > 0:
                with torch.cuda.stream(pipes[k - 1][0]):
                    return pipes[k - 1][1].replay()
            return graph.replay()
        if graph is not None:
            return graph.replay()
        if world == 1:
            return model.forward_prompts(wav, STEMS, out=out)
        # shard + point-to-point gather of the separated waveforms to rank 0, transfers left in flight
        return separate_segments(model, wav, STEMS, max_batch=B, n_total=N, out=out, pending=pending)

    def fwd_only():
        return model.forward_prompts(wav, STEMS)

    # warmup; the last warmup step times every kernel per call site (HIP events) to find the dominant call site
    for i in range(args.warmup):
        if i == args.warmup - 1:
            model.profile_start("@sites")        # (events around eager launches: the graph's launches are baked)
            fwd_only() if graph is not None else step()
        else:
            step()
    pending.wait()
    torch.cuda.synchronize()
    dominant = args.kernel
    sites = []
    if args.warmup > 0:
        sites = model.profile_stop()
        if args.dump_kernels and rank == 0:
            per_kernel = {}
            for r in sites:
                a = per_kernel.setdefault(r["kernel"].split("@", 1)[0],
                                          {"kernel": r["kernel"].split("@", 1)[0], "launches": 0, "ms": 0.0,
                                           "flops": 0.0, "bytes": 0.0})
                for f in ("launches", "ms", "flops", "bytes"):
                    a[f] += r[f]
            allk = list(per_kernel.values())
            for r in allk + sites:
                r["tflops"] = r["flops"] / (r["ms"] * 1e-3) / 1e12 if r["ms"] else 0.0
                r["gbs"] = r["bytes"] / (r["ms"] * 1e-3) / 1e9 if r["ms"] else 0.0
            json.dump(sorted(allk, key=lambda r: -r["ms"]), open(args.dump_kernels, "w"), indent=1)
            json.dump(sorted(sites, key=lambda r: -r["ms"]), open(args.dump_kernels.replace(".json", "_sites.json"),
                                                                   "w"), indent=1)
        if dominant is None:
            dominant = max(sites, key=lambda r: r["ms"])["kernel"]
    if dominant is None:
        dominant = "attn32_kernel@transformer"

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    barrier()
    torch.cuda.synchronize()
    nstep[0] = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    pending.wait()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    # roofline kernel: every launch of it bracketed with HIP events on its launch stream, over ROOF_STEPS further
    # forwards outside the timed region (with a profile open the library runs the freq / time branches serially on
    # one stream, so the events time the kernel alone rather than sharing the chip with the other branch)
    model.profile_start(dominant)
    for _ in range(ROOF_STEPS):
        fwd_only()
    torch.cuda.synchronize()
    prof = model.profile_stop()
    sections = None
    if not args.no_extras:
        model.profile_start("@section")
        fwd_only()
        torch.cuda.synchronize()
        sections = model.profile_stop()
    if world > 1:
        t = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    ms = el / args.steps * 1e3
    value = B * world * args.steps / el
    peak_mfma = BF16_PEAK_TFLOPS if args.dtype == "bf16" else F32_PEAK_TFLOPS
    flops_step = 2e9 * (ENC_GMAC + 4 * DEC_GMAC) * B
    step_tf = flops_step / (ms * 1e-3) / 1e12
    kp = next((r for r in prof if r["kernel"] == dominant), None)
    if kp is None or kp["launches"] == 0:
        raise RuntimeError(f"roofline kernel {dominant!r} was not launched in the timed region")
    per_launch_ms = kp["ms"] / kp["launches"]
    kernel_sym = dominant.split("@", 1)[0]
    # the call site's bound is the larger of its two floors: algorithmic flops at the MFMA peak, algorithmic bytes at
    # the HBM peak (e.g. the decoder's K = 288 ConvT GEMM moves 6.2 GB for 1.2 TFLOP: HBM-bound)
    t_mfma = kp["flops"] / (peak_mfma * 1e12) if kernel_sym.startswith(MFMA_KERNELS) else 0.0
    t_hbm = kp["bytes"] / (HBM_PEAK_GBS * 1e9)
    if t_mfma >= t_hbm:
        peak = peak_mfma
        ach = kp["flops"] / (kp["ms"] * 1e-3) / 1e12
        bound, unit = "mfma", "TFLOP/s"
    else:
        peak, bound, unit = HBM_PEAK_GBS, "hbm", "GB/s"
        ach = kp["bytes"] / (kp["ms"] * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(kernel_sym, B, args.dtype)
    # the same kernel over ALL its call sites (warm-up profile): what rocprofv3's per-symbol average reports
    same = [r for r in sites if r["kernel"].split("@", 1)[0] == kernel_sym]
    all_sites = None
    if same:
        n_all = sum(r["launches"] for r in same)
        all_sites = {"kernel": kernel_sym, "launches_per_step": n_all, "sites": len(same),
                     "avg_launch_us": round(sum(r["ms"] for r in same) / n_all * 1e3, 2),
                     "timing": "warm-up step, every launch evented, branches serialised"}
    roofline = {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
                "traffic": traffic, "kernel": kernel_sym, "call_site": dominant,
                "kernel_all_sites": all_sites,
                "traffic_note": "PMC bytes per launch of the kernel symbol (all call sites; rocprofv3 cannot split "
                                "them)" if all_sites and all_sites["sites"] > 1 else "PMC bytes per launch",
                "launches_per_step": kp["launches"] / ROOF_STEPS,
                "avg_launch_us": round(per_launch_ms * 1e3, 2),
                "share_of_step": round(kp["ms"] / ROOF_STEPS / ms, 4),
                "algorithmic_per_launch": {"flops": kp["flops"] / kp["launches"],
                                           "bytes": kp["bytes"] / kp["launches"]},
                "floors_ms_per_launch": {"mfma": round(t_mfma * 1e3 / kp["launches"], 4),
                                         "hbm": round(t_hbm * 1e3 / kp["launches"], 4)},
                "timing": f"HIP events on the launch stream around every launch of the call site, {ROOF_STEPS} "
                          "forwards after the timed region (branches serialised on one stream)",
                "step": {"achieved_tflops": round(step_tf, 2), "peak": peak_mfma, "frac": round(step_tf / peak_mfma, 4),
                         "basis": "essential FLOPs per step (SURVEY.md §8(d): 256.5 GFLOP per segment x 4 stems) / "
                                  "timed ms per step"}}
    if traffic_src:
        roofline["traffic_source"] = traffic_src
    if sections:
        sec = {}
        for r in sections:
            if not r["ms"]:
                continue
            tf = r["flops"] / (r["ms"] * 1e-3) / 1e12
            sec[r["kernel"]] = {"ms": round(r["ms"], 3), "tflops": round(tf, 1), "frac_mfma": round(tf / peak_mfma, 4),
                                "hbm_gbs": round(r["bytes"] / (r["ms"] * 1e-3) / 1e9, 1)}
        roofline["sections"] = sec
        roofline["sections_timing"] = ("one forward after the timed region, every kernel bracketed by HIP events "
                                       "(branches serialised), summed per section; flops / bytes = the kernels' "
                                       "algorithmic work")
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
        "data": "synthetic (64 distinct seeded tones+noise 6 s stereo segments per GPU, seeded random weights of the "
                "htdemucs/AudioTextHTDemucs architecture)",
        "config": {"workload": "BASELINE configs[2]: B=64 x 6 s segments x 4 prompts per GPU"
                               + ("; configs[3] shape: segments sharded over the GPUs, RCCL gather to rank 0 timed"
                                  if world > 1 else ""),
                   "global_batch": N, "seq_len": SEG, "prompts": 4, "parallelism": f"segment-sharded dp{world}",
                   "gather_timed": world > 1,
                   "launch": "hipGraph replay of one athd_forward_prompts" if graph is not None else "eager",
                   "pipelines": len(pipes) + 1},
        "stems_per_s": round(4 * value, 3),
        "roofline": roofline,
        "step_essential_tflops": round(step_tf, 2),
        "workspace_gb": round(model._ws.numel() / 1e9, 2) if model._ws is not None else None,
    }
    if rank == 0 and not args.no_extras:
        rec["sdr_db_vs_oracle"] = sdr_vs_oracle(model, sd, table, wav[:1].contiguous())
        if world == 1 and args.dtype == "bf16":
            rec["f32"] = f32_line(sd, table, wav)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(sd, table)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if args.segments > 0:
        rec2 = dataset_pass(model, wav, args.segments, B, world, rank, dev)
        if rank == 0:
            print(json.dumps(rec2), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
