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


def sdr_vs_oracle(out, sd, table, wav, rows=(0, 63)):
    """SDR (dB) of the TIMED output - rows `rows` of the last step's (B, 4, 2, T) result, written by the replayed
    graph (N = 1) or the eager launches - against the fp32 oracle's forward_prompts on the same segments (north_star:
    'SDR delta reported'); min and mean over rows x prompts."""
    from oracle.athtdemucs_ref import AudioTextHTDemucsRef
    rows = [r for r in rows if r < wav.shape[0]]
    got = out[rows].cpu().double()
    ref = AudioTextHTDemucsRef(sd).forward_prompts(wav[rows].cpu(), torch.as_tensor(table)).double()
    s = [[float(10 * torch.log10((ref[i, p] ** 2).sum() / ((ref[i, p] - got[i, p]) ** 2).sum())) for p in range(4)]
         for i in range(len(rows))]
    flat = [x for r in s for x in r]
    return {"min": round(min(flat), 2), "mean": round(sum(flat) / len(flat), 2),
            "per_row_prompt": {str(r): [round(x, 2) for x in s[i]] for i, r in enumerate(rows)},
            "what": f"SDR of the timed bench output (rows {rows} of the last timed step, prompts {STEMS}) vs the fp32 "
                    "oracle forward_prompts (unclamped)"}


def roofline_of(model, fwd, dominant, peak_mfma, ms_step, sites, steps=ROOF_STEPS, sections=True):
    """Roofline of call site `dominant`: every launch of it bracketed with HIP events on its launch stream over
    `steps` forwards (with a profile open the library runs the freq / time branches serially on one stream, so the
    events time the kernel alone), priced against the larger of its two floors (algorithmic flops at the MFMA peak,
    algorithmic bytes at the HBM peak); plus the per-section sums of one more fully evented forward."""
    model.profile_start(dominant)
    for _ in range(steps):
        fwd()
    torch.cuda.synchronize()
    prof = model.profile_stop()
    kp = next((r for r in prof if r["kernel"] == dominant), None)
    if kp is None or kp["launches"] == 0:
        raise RuntimeError(f"roofline kernel {dominant!r} was not launched")
    per_launch_ms = kp["ms"] / kp["launches"]
    kernel_sym = dominant.split("@", 1)[0]
    t_mfma = kp["flops"] / (peak_mfma * 1e12) if kernel_sym.startswith(MFMA_KERNELS) else 0.0
    t_hbm = kp["bytes"] / (HBM_PEAK_GBS * 1e9)
    if t_mfma >= t_hbm:
        peak, bound, unit = peak_mfma, "mfma", "TFLOP/s"
        ach = kp["flops"] / (kp["ms"] * 1e-3) / 1e12
    else:
        peak, bound, unit = HBM_PEAK_GBS, "hbm", "GB/s"
        ach = kp["bytes"] / (kp["ms"] * 1e-3) / 1e9
    same = [r for r in sites if r["kernel"].split("@", 1)[0] == kernel_sym]
    all_sites = None
    if same:
        n_all = sum(r["launches"] for r in same)
        all_sites = {"kernel": kernel_sym, "launches_per_step": n_all, "sites": len(same),
                     "avg_launch_us": round(sum(r["ms"] for r in same) / n_all * 1e3, 2),
                     "timing": "warm-up step, every launch evented, branches serialised"}
    roof = {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
            "kernel": kernel_sym, "call_site": dominant, "kernel_all_sites": all_sites,
            "launches_per_step": kp["launches"] / steps, "avg_launch_us": round(per_launch_ms * 1e3, 2),
            "share_of_step": round(kp["ms"] / steps / ms_step, 4),
            "algorithmic_per_launch": {"flops": kp["flops"] / kp["launches"], "bytes": kp["bytes"] / kp["launches"]},
            "floors_ms_per_launch": {"mfma": round(t_mfma * 1e3 / kp["launches"], 4),
                                     "hbm": round(t_hbm * 1e3 / kp["launches"], 4)},
            "timing": f"HIP events on the launch stream around every launch of the call site, {steps} forwards after "
                      "the timed region (branches serialised on one stream)"}
    if sections:
        model.profile_start("@section")
        fwd()
        torch.cuda.synchronize()
        sec = {}
        for r in model.profile_stop():
            if not r["ms"]:
                continue
            tf = r["flops"] / (r["ms"] * 1e-3) / 1e12
            sec[r["kernel"]] = {"ms": round(r["ms"], 3), "tflops": round(tf, 1), "frac_mfma": round(tf / peak_mfma, 4),
                                "hbm_gbs": round(r["bytes"] / (r["ms"] * 1e-3) / 1e9, 1)}
        roof["sections"] = sec
        roof["sections_timing"] = ("one forward after the timed region, every kernel bracketed by HIP events "
                                   "(branches serialised), summed per section; flops / bytes = the kernels' "
                                   "algorithmic work")
    return roof


def site_profile(model, fwd):
    """Every launch of one forward evented, keyed by call site (kernel@stage.site)."""
    model.profile_start("@sites")
    fwd()
    torch.cuda.synchronize()
    return model.profile_stop()


def f32_line(m32, wav, steps=3):
    """Throughput of the f32 parity mode (fp32 MFMA everywhere) on the same batch, outside the headline, with its
    own roofline call site (the largest summed time of one evented forward) and per-section sums."""
    fwd = lambda: m32.forward_prompts(wav, STEMS)          # noqa: E731
    fwd()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fwd()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms = el / steps * 1e3
    tf = 2e9 * (ENC_GMAC + 4 * DEC_GMAC) * wav.shape[0] / (ms * 1e-3) / 1e12
    sites = site_profile(m32, fwd)
    dom = max(sites, key=lambda r: r["ms"])["kernel"]
    return {"value": round(wav.shape[0] * steps / el, 3), "unit": "segments/s", "ms_per_step": round(ms, 3),
            "steps": steps, "warmup": 1, "step_essential_tflops": round(tf, 2),
            "frac_of_f32_mfma_peak": round(tf / F32_PEAK_TFLOPS, 4),
            "roofline": roofline_of(m32, fwd, dom, F32_PEAK_TFLOPS, ms, sites, steps=1)}


def sdr_delta_split(m_bf16, m_f32, n_tracks=2):
    """north_star's 'SDR delta' under the benchmark.py protocol (its offline proxy: no MUSDB18, no trained weights):
    a synthetic MUSDB18-HQ split (n_tracks tracks of 4 seeded tone+noise stems, mixture = their sum) through
    athd.dist.separate_dataset (6 s windows, 1.5 s overlap, weighted overlap-add, per-stem SDR / SI-SDR as
    benchmark.py:655-688) with the bf16 (bench) and the f32 (parity) model: the aggregate metric of each, their
    difference, and the SDR of the bf16 estimates against the f32 ones."""
    import tempfile
    from athd.benchmark import aggregate_results
    from athd.dist import separate_dataset
    from athd.musdb import HQ_FILES, MusDBTracks, write_wav
    from athd.synth import synthetic_mixture
    with tempfile.TemporaryDirectory() as tmp:
        lens = [44100 * 20 + 777, 44100 * 13 + 5][:n_tracks]
        for t, L in enumerate(lens):
            d = os.path.join(tmp, f"Synthetic {t} - Track")
            os.makedirs(d)
            parts = [0.25 * synthetic_mixture(L, seed=3000 + 10 * t + j) for j in range(4)]
            for f, x in zip(HQ_FILES, [sum(parts)] + parts):
                write_wav(os.path.join(d, f + ".wav"), x, 44100, "FLOAT")
        tracks = MusDBTracks(tmp)
        out = {}
        for name, m in (("bf16", m_bf16), ("f32", m_f32)):
            results, est = separate_dataset(m, tracks, STEMS, max_batch=16, keep_estimates=True, log=None)
            out[name] = (aggregate_results(results), est)
    agg = {k: {f: {s: round(x, 4) for s, x in v[0][f].items()} for f in v[0]} for k, v in out.items()}
    delta = {f: {s: round(agg["bf16"][f][s] - agg["f32"][f][s], 4) for s in agg["f32"][f]} for f in agg["f32"]}
    est_sdr = []
    for name in out["f32"][1]:
        a, b = out["f32"][1][name].double(), out["bf16"][1][name].double()
        est_sdr.append(float(10 * torch.log10((a ** 2).sum() / ((a - b) ** 2).sum())))
    return {"protocol": "benchmark.py:155-204 (6 s windows, 1.5 s overlap, weighted OLA) via athd.dist.separate_dataset",
           "data": f"{len(lens)} synthetic MUSDB18-HQ-layout tracks ({[round(L / 44100, 1) for L in lens]} s), seeded "
                   "random weights", "aggregate": agg, "delta_bf16_minus_f32": delta,
           "sdr_bf16_estimates_vs_f32_db": [round(x, 2) for x in est_sdr]}


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
    ap.add_argument("--decode-items", type=int, default=0,
                    help="(segment, prompt) items per decode chunk (default: the whole batch, B x 4, in one chunk)")
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
    tt = {s: table[i] for i, s in enumerate(STEMS)}
    # the whole per-GPU batch in one decode chunk (B x 4 items): fewer, larger decoder launches (≈49 GB: athd_workspace_bytes, reported as workspace_gb)
    dec_items = args.decode_items or B * len(STEMS)
    model = AudioTextHTDemucs(dtype=args.dtype, text_table=tt, decode_items=dec_items)
    model.load_state_dict(sd)
    model = model.to(dev).eval()
    # B distinct synthetic segments per rank, resident in HBM before timing (weak scaling: each rank owns its block)
    wav = torch.as_tensor(synthetic_batch(B, SEG, seed0=1000 + B * rank)).to(dev)
    N = B * world
    out = torch.empty((N, len(STEMS), 2, SEG), dtype=torch.float32, device=dev) if rank == 0 else None
    ws_bytes = model._ensure_ctx().workspace_bytes(B, SEG, len(STEMS))

    # Every step is one athd_forward_prompts captured into a HIP graph (both branch streams and their event joins)
    # and replayed: the same kernels on the same buffers, without the host launch gaps between them.
    #  * N = 1: the graph writes the bench output directly.
    #  * N > 1: the same graph replay is the forward_fn of athd.dist.separate_segments, so the point-to-point RCCL
    #    gather to rank 0 runs exactly as in the product runner.  Rank 0's graph writes its own rows of the gathered
    #    output; every other rank alternates two graphs (one workspace, two send buffers) so a step never overwrites
    #    a buffer whose send may still be in flight (PendingSends(limit=1): the previous step's send is waited on,
    #    stream-ordered, before the next replay).
    graphs, gbufs = [], []
    pending = PendingSends(limit=2)          # eager N > 1: at most two batches in flight per rank
    if not args.eager:
        gws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        if rank == 0:
            gbufs = [out[0:B]]
        else:
            gbufs = [torch.empty((B, len(STEMS), 2, SEG), dtype=torch.float32, device=dev) for _ in range(2)]
            pending = PendingSends(limit=1)
        for buf in gbufs:
            graphs.append(model.capture_prompts(wav, STEMS, out=buf, workspace=gws)[0])
    # further pipelines (N = 1, --pipelines > 1): own model context, batch, output, stream and graph each
    pipes = []
    if world == 1 and graphs and args.pipelines > 1:
        for k in range(1, args.pipelines):
            mk = AudioTextHTDemucs(dtype=args.dtype, text_table=tt, decode_items=dec_items)
            mk.load_state_dict(sd)
            mk = mk.to(dev).eval()
            wk = torch.as_tensor(synthetic_batch(B, SEG, seed0=1000 + B * (world + k))).to(dev)
            gk, _ = mk.capture_prompts(wk, STEMS)
            pipes.append((torch.cuda.Stream(dev), gk, mk, wk))
    nstep = [0]
    ngraph = [0]

    def graph_fwd(w, o):
        k = ngraph[0] % len(graphs)
        ngraph[0] += 1
        graphs[k].replay()
        return gbufs[k]

    def step():
        if pipes:
            k = nstep[0] % (len(pipes) + 1)
            nstep[0] += 1
            if k > 0:
                with torch.cuda.stream(pipes[k - 1][0]):
                    return pipes[k - 1][1].replay()
            return graphs[0].replay()
        if world == 1:
            return graphs[0].replay() if graphs else model.forward_prompts(wav, STEMS, out=out)
        # shard + point-to-point gather of the separated waveforms to rank 0, transfers left in flight
        return separate_segments(model, wav, STEMS, max_batch=B, n_total=N, out=out, pending=pending,
                                 forward_fn=graph_fwd if graphs else None)

    def fwd_only():
        return model.forward_prompts(wav, STEMS)

    # warmup; the last warmup step times every kernel per call site (HIP events) to find the dominant call site
    for i in range(args.warmup):
        if i == args.warmup - 1:
            model.profile_start("@sites")        # (events around eager launches: the graph's launches are baked)
            fwd_only() if graphs else step()
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
    if world > 1:
        t = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    ms = el / args.steps * 1e3
    value = B * world * args.steps / el
    # the timed output, for the parity check below (rank 0's rows of the last step; fwd_only below reuses the
    # model's own workspace and output, not the graph's)
    timed_rows = out[[0, B - 1]].clone() if rank == 0 else None
    peak_mfma = BF16_PEAK_TFLOPS if args.dtype == "bf16" else F32_PEAK_TFLOPS
    flops_step = 2e9 * (ENC_GMAC + 4 * DEC_GMAC) * B
    step_tf = flops_step / (ms * 1e-3) / 1e12
    roofline = roofline_of(model, fwd_only, dominant, peak_mfma, ms, sites, sections=not args.no_extras)
    kernel_sym = roofline["kernel"]
    traffic, traffic_src = pmc_traffic(kernel_sym, B, args.dtype)
    roofline["traffic"] = traffic
    roofline["traffic_note"] = ("PMC bytes per launch of the kernel symbol (all call sites; rocprofv3 cannot split "
                                "them)" if roofline["kernel_all_sites"] and roofline["kernel_all_sites"]["sites"] > 1
                                else "PMC bytes per launch")
    if traffic_src:
        roofline["traffic_source"] = traffic_src
    roofline["step"] = {"achieved_tflops": round(step_tf, 2), "peak": peak_mfma, "frac": round(step_tf / peak_mfma, 4),
                        "basis": "essential FLOPs per step (SURVEY.md §8(d): 256.5 GFLOP per segment x 4 stems) / "
                                 "timed ms per step"}
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
                   "launch": (f"hipGraph replay of one athd_forward_prompts per step ({len(graphs)} graph(s) per rank)"
                              if graphs else "eager"),
                   "pipelines": len(pipes) + 1, "decode_items": dec_items},
        "stems_per_s": round(4 * value, 3),
        "roofline": roofline,
        "step_essential_tflops": round(step_tf, 2),
        "workspace_gb": round(ws_bytes / 1e9, 2),
    }
    if rank == 0 and not args.no_extras:
        full = torch.zeros((B, len(STEMS), 2, SEG), dtype=torch.float32)
        full[[0, B - 1]] = timed_rows.cpu()
        rec["sdr_db_vs_oracle"] = sdr_vs_oracle(full, sd, table, wav.cpu(), rows=(0, B - 1))
        if world == 1 and args.dtype == "bf16":
            m32 = AudioTextHTDemucs(dtype="f32", text_table=tt)
            m32.load_state_dict(sd)
            m32 = m32.to(dev).eval()
            rec["f32"] = f32_line(m32, wav)
            model._ws = None                     # (the bench workspace is not needed for the short split below)
            torch.cuda.empty_cache()
            rec["sdr_delta_benchmark_protocol"] = sdr_delta_split(model, m32)
            del m32
            torch.cuda.empty_cache()
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
