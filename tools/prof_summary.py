"""Summarise a rocprofv3 --kernel-trace --stats csv directory: top kernels and the per-dispatch sequence of the
last forward (bracketed by stft_kernel launches)."""
import csv
import glob
import os
import sys


def main(d, seq=False, top=25):
    ks = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
    rows = list(csv.DictReader(open(ks)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time {tot / 1e6:.2f} ms")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {float(r['Percentage']):6.2f}% n={r['Calls']:>5} "
              f"avg={float(r['AverageNs']) / 1e3:9.1f}us  {r['Name'][:100]}")
    if seq:
        kt = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
        tr = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
        idx = [i for i, r in enumerate(tr) if "stft_kernel" in r["Kernel_Name"]]
        for r in tr[idx[-1]:]:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"{dur:9.1f}us grid={r['Grid_Size_X']:>8}x{r['Grid_Size_Y']:>4}x{r['Grid_Size_Z']:>3} "
                  f"vgpr={r['VGPR_Count']:>3} lds={r['LDS_Block_Size']:>6} {r['Kernel_Name'].replace('athd::', '')[:70]}")


if __name__ == "__main__":
    main(sys.argv[1], seq="--seq" in sys.argv)
