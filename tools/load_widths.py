"""Static global-memory load widths per kernel of libathd.so, for the FETCH_SIZE width correction of
tools/pmc_traffic.py (MI355X_MICROARCH.md §HBM: the counter's factor depends on the per-lane access width; the
factors come from tools/pmc_calib.hip).

Compiles every csrc/*.hip to gfx950 device assembly (hipcc --cuda-device-only -S, same flags as the Makefile) and
counts, per kernel symbol, the vector-memory load instructions by bytes per lane:
  2  global/buffer_load_ushort / _short_d16*        4  *_load_dword        8  *_load_dwordx2
  12 *_load_dwordx3                                  16 *_load_dwordx4 and global_load_lds_dwordx4 / buffer ... lds
Static counts in loop bodies stand in for dynamic ones (loop bodies dominate the instruction stream); the result is
each kernel's share of static load BYTES per width.

    python tools/load_widths.py [-o profiles/load_widths.json]
"""
import argparse
import collections
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from knames import short_name  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "audio-to-sheet-music_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-w"]

LOAD = re.compile(r"^\s*(global|buffer)_load_(lds_)?(ubyte|sbyte|ushort|sshort|short_d16\w*|dword|dwordx2|dwordx3|"
                  r"dwordx4)\b(.*)$")
WIDTH = {"ubyte": 1, "sbyte": 1, "ushort": 2, "sshort": 2, "dword": 4, "dwordx2": 8, "dwordx3": 12, "dwordx4": 16}


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True, check=True).stdout.split("\n")
    return dict(zip(names, out))


def widths_of(asm_text):
    per = collections.defaultdict(lambda: collections.Counter())
    cur = None
    for line in asm_text.splitlines():
        m = re.match(r"^(_Z\w+):\s*(;.*)?$", line)
        if m:
            cur = m.group(1)
            continue
        if cur is None:
            continue
        if line.strip().startswith(".Lfunc_end"):
            cur = None
            continue
        m = LOAD.match(line)
        if m:
            kind = m.group(3)
            w = 2 if kind.startswith("short_d16") else WIDTH[kind]
            per[cur][w] += 1
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-o", default=os.path.join(REPO, "profiles", "load_widths.json"))
    a = ap.parse_args()
    allk = {}
    with tempfile.TemporaryDirectory() as td:
        for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
            s = os.path.join(td, os.path.basename(src) + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "--cuda-device-only", "-S", src, "-o", s], check=True,
                           cwd=CSRC)
            for k, c in widths_of(open(s).read()).items():
                allk[k] = c
    dem = demangle(list(allk))
    out = {}
    for k, c in allk.items():
        name = short_name(dem[k])
        tot = sum(w * n for w, n in c.items())
        if tot == 0:
            continue
        agg = out.setdefault(name, collections.Counter())
        agg.update(c)
    res = {}
    for name, c in sorted(out.items()):
        tot = sum(w * n for w, n in c.items())
        res[name] = {"loads": {str(w): n for w, n in sorted(c.items())},
                     "byte_share": {str(w): round(w * n / tot, 4) for w, n in sorted(c.items())}}
    json.dump({"source": "static gfx950 device assembly of audio-to-sheet-music_amd/csrc/*.hip", "kernels": res},
              open(a.o, "w"), indent=1)
    for name, v in res.items():
        print(f"{name:60s} {v['byte_share']}")


if __name__ == "__main__":
    main()
