"""Static check (tooling): inline-asm instructions that read an MFMA or TRANS result too early.

hipcc (ROCm 7.2) pads its own instructions after an MFMA or a transcendental (v_exp / v_rcp / ...) with the wait states
the gfx950 hazard rules ask for.  It inserts nothing before an inline-asm consumer (tools/hazard/README.md).  Examples
from hipcc itself: v_mfma_f32_16x16x4_f32 -> ds_write 9 states, -> VALU / global_store 10; v_exp_f32 -> VALU 1.

The hardware probe tools/hazard/mfma_ds.hip (profiles/r06_hazard.txt) measured 9 states to be enough for the
16x16x4 f32 form, alone and under contention.  So the compiler's own consumers are taken as correct.  This scan
flags every consumer INSIDE an asm block with fewer than NEED wait states after the producer: 10 after an MFMA, 1
after a TRANS instruction.  The consumer may be a VALU read, a store of the register, or an MFMA reading it as
A/B/C.  Round 6 found two such consumers:
  - attn.hip vmax3 on the QK^T accumulators, rounds 2-5;
  - a v_add_f32 row-sum variant reading v_exp results, removed.

Usage: python tools/mfma_store_scan.py [file.s ...]   (default: compiles csrc/*.hip to /tmp)
"""
import glob
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-to-sheet-music_amd", "csrc")
TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")
NEED = {"mfma": 10, "trans": 1}
STORES = ("ds_write", "global_store", "buffer_store", "flat_store", "scratch_store")


def regs(tok):
    m = re.match(r"([av])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"-?\|?([av])(\d+)\|?$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


def operands(u):
    parts = u.split(None, 1)
    return [p.strip() for p in parts[1].split(",")] if len(parts) > 1 else []


def scan(fn):
    hits = []
    lines = open(fn).read().splitlines()
    in_asm = [False] * len(lines)
    a = False
    for k, l in enumerate(lines):
        if ";;#ASMSTART" in l:
            a = True
        elif ";;#ASMEND" in l:
            a = False
        in_asm[k] = a
    labels = {l.split(":")[0]: k for k, l in enumerate(lines) if re.match(r"^\.LBB\w+:", l)}
    func = "?"
    for k, l in enumerate(lines):
        if re.match(r"^_Z\w+:", l):
            func = l.split(":")[0]
        t = l.strip()
        if not t.startswith("v_") or in_asm[k]:
            continue
        op = t.split()[0]
        kind = "mfma" if op.startswith("v_mfma") else "trans" if op.startswith(TRANS) else None
        if kind is None:
            continue
        dst = regs(operands(t)[0]) if operands(t) else set()
        # walk every path (conditional branches: both the fall-through and the target) up to 80 instructions
        stack, seen = [(k + 1, 0, 0)], set()
        while stack:
            kk, ws, steps = stack.pop()
            while kk < len(lines) and steps < 80:
                if (kk, ws) in seen:
                    break
                seen.add((kk, ws))
                u = lines[kk].strip()
                if not u or u.startswith(";") or u.startswith("."):
                    kk += 1
                    continue
                ins = u.split()[0]
                ops = operands(u)
                srcs = set()
                for o in (ops if ins.startswith(STORES) else ops[1:]):
                    srcs |= regs(o)
                if dst & srcs:
                    if in_asm[kk] and ws < NEED[kind]:
                        hits.append((func, op, ins, ws, kk + 1))
                    break
                if ops and dst & regs(ops[0]) and not ins.startswith(STORES):
                    break                                # overwritten before any read
                if ins in ("s_endpgm", "s_setpc_b64"):
                    break
                if ins.startswith("s_cbranch") or ins == "s_branch":
                    tgt = labels.get(ops[0]) if ops else None
                    if tgt is not None:
                        stack.append((tgt, ws + 1, steps + 1))
                    if ins == "s_branch":
                        break
                ws += (int(ops[0], 0) + 1) if ins == "s_nop" and ops else 1
                steps += 1
                kk += 1
    return hits


if __name__ == "__main__":
    files = sys.argv[1:]
    if not files:
        for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
            out = "/tmp/mfscan_" + os.path.basename(src)[:-4] + ".s"
            subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-w",
                                   "--cuda-device-only", "-S", src, "-o", out], cwd=CSRC)
            files.append(out)
    n = 0
    for f in files:
        for h in scan(f):
            print(os.path.basename(f), *h)
            n += 1
    print(f"{n} inline-asm consumers of an MFMA / TRANS result inside the hazard window")
    sys.exit(1 if n else 0)
