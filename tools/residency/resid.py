"""Residency microbenchmark driver (tooling): resident workgroups per CU for LDS size x waves per workgroup x VGPRs
on the current GPU.  Prints one line per configuration: spin periods taken by 6 x CUs workgroups -> resident."""
import ctypes
import os
import sys

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libresid.so"))
lib.resid_run.restype = ctypes.c_float
lib.resid_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float]
CUS, K, US = 256, 6, 200.0
for vg in (32, 128):
    for waves in (4, 6, 8):
        row = []
        for kb in (16, 32, 40, 48, 51, 53, 54, 56, 60, 64, 65, 66, 72, 80, 81):
            ms = lib.resid_run(waves, kb * 1024, vg, K * CUS, US)
            periods = round(ms * 1000.0 / US)
            row.append(f"{kb}K:{periods}p")
        print(f"vgpr {vg:3d} waves {waves}: " + " ".join(row), flush=True)
