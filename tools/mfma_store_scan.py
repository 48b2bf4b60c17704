"""Static check (tooling): every MFMA result that an LDS / global store reads within 16 wait states of the MFMA.
hipcc (ROCm 7.2) put 10 wait states between v_mfma_f32_16x16x4_f32 and a ds_write of its accumulators in
tdec_tail_kernel, short for the instruction's 40-cycle result latency on gfx950: the store read a stale register
under load (round 5).  Usage: python tools/mfma_store_scan.py [file.s ...] (default: compiles csrc/*.hip to /tmp)."""
import glob
import os
import re
import subprocess
import sys

STORES = ("ds_write", "global_store", "buffer_store", "flat_store", "scratch_store")
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-to-sheet-music_amd", "csrc")


def regs(tok):
    m = re.match(r"([av])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([av])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def scan(fn):
    hits = []
    lines = open(fn).read().splitlines()
    func = "?"
    for k, l in enumerate(lines):
        if re.match(r"^_Z\w+:", l):
            func = l.split(":")[0]
        t = l.strip()
        if not t.startswith("v_mfma"):
            continue
        dst = regs(t.split(None, 1)[1].split(",")[0].strip())
        ws = 0
        for kk in range(k + 1, min(len(lines), k + 60)):
            u = lines[kk].strip()
            if not u or u.startswith(";") or u.startswith("."):
                if u.startswith(".LBB"):
                    break
                continue
            ins = u.split()[0]
            ops = [p.strip() for p in u.split(None, 1)[1].split(",")] if len(u.split(None, 1)) > 1 else []
            srcs = set()
            for o in (ops if ins.startswith(STORES) else ops[1:]):
                srcs |= regs(o)
            if ins.startswith("v_mfma"):
                if dst & regs(ops[0]) and not (dst & srcs):
                    break
                ws += 1
                continue
            if dst & srcs:
                if ins.startswith(STORES) and ws < 16:
                    hits.append((func, t.split()[0], ins, ws))
                break
            ws += (int(ops[0], 0) + 1) if ins == "s_nop" and ops else 1
    return hits


if __name__ == "__main__":
    files = sys.argv[1:]
    if not files:
        for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
            out = "/tmp/mfscan_" + os.path.basename(src)[:-4] + ".s"
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                                   "--cuda-device-only", "-S", src, "-o", out], cwd=CSRC)
            files.append(out)
    n = 0
    for f in files:
        for h in scan(f):
            print(os.path.basename(f), *h)
            n += 1
    print(f"{n} MFMA-result stores within 16 wait states")
    sys.exit(1 if n else 0)
