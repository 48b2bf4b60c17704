"""Kernel sequence (durations) of one decode chunk of the last forward in a rocprofv3 kernel trace."""
import csv
import glob
import os
import sys

d = sys.argv[1]
which = int(sys.argv[2]) if len(sys.argv) > 2 else 1
kt = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
tr = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(tr) if "stft_kernel" in r["Kernel_Name"]]
last = tr[idx[-1]:]
tv = [i for i, r in enumerate(last) if r["Kernel_Name"].startswith("athd::text_vec")] + [len(last)]
tot = 0.0
for r in last[tv[which]:tv[which + 1]]:
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += dur
    print(f"{dur:8.1f} us  {r['Kernel_Name'].replace('athd::', '')[:80]}")
print(f"{tot:8.1f} us  total")
