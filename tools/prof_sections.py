"""Per-section kernel time of the last forward in a rocprofv3 kernel trace: encoder (until pos2d), transformer
(until text_vec), decoder (rest); within each, per kernel name."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
kt = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
tr = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(tr) if "stft_kernel" in r["Kernel_Name"]]
sec = "encoder"
tot = collections.OrderedDict()
for r in tr[idx[-1]:]:
    n = r["Kernel_Name"].replace("athd::", "")
    if n.startswith("pos2d"):
        sec = "transformer"
    if n.startswith("text_vec"):
        sec = "decoder"
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    key = n.split("(")[0][:60]
    tot.setdefault(sec, collections.Counter())[key] += dur
for s, c in tot.items():
    print(f"== {s}: {sum(c.values()) / 1e3:.2f} ms")
    for k, v in c.most_common(8):
        print(f"   {v / 1e3:8.2f} ms  {k}")
