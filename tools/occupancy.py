"""Mean resident waves per CU per kernel from a rocprofv3 PMC pass of SQ_WAVE_CYCLES and GRBM_GUI_ACTIVE (tooling).
The counters' units are calibrated on fenc_row1_kernel, whose one 12-wave workgroup per CU (163 KB of LDS) is
resident for the whole kernel: waves/CU = (SQ_WAVE_CYCLES / GRBM_GUI_ACTIVE) / (that ratio for fenc_row1 / 12).
Usage: python tools/occupancy.py <rocprofv3 output dir> [...]"""
import collections
import csv
import sys


def table(d):
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in rows:
        key = (r["Kernel_Name"][:48], r["Dispatch_Id"])
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[key] = (int(r["LDS_Block_Size"]), int(r["Workgroup_Size"]), int(r["Grid_Size"]))
    last = {}
    for (k, did), v in agg.items():
        last[k] = (v, meta[(k, did)])
    cal = [v for k, (v, m) in last.items() if "fenc_row1_kernel" in k][0]
    unit = cal["SQ_WAVE_CYCLES"] / cal["GRBM_GUI_ACTIVE"] / 12
    out = []
    for k, (v, m) in last.items():
        if v["GRBM_GUI_ACTIVE"] < 2e6:
            continue
        w = v["SQ_WAVE_CYCLES"] / v["GRBM_GUI_ACTIVE"] / unit
        out.append((v["GRBM_GUI_ACTIVE"], k, m, w))
    out.sort(reverse=True)
    return out


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(f"== {d}")
        for g, k, (lds, wg, grid), w in table(d):
            print(f"{k:48s} lds={lds:6d} wg={wg:4d} wgs={grid // wg:6d} waves/CU {w:5.1f}  workgroups/CU {w / (wg / 64):4.2f}")
