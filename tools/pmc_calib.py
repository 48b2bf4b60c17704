"""Counter factors per access width from the rocprofv3 passes over tools/pmc_calib (see tools/pmc_calib.hip).

    python tools/pmc_calib.py <fetch_dir> <write_dir> [-o profiles/pmc_calib.json]

factor = counter bytes (KiB x 1024) / true bytes (1 GiB) per kernel, averaged over its 2 launches; the read kernels
give the FETCH_SIZE factors, the write kernels the WRITE_SIZE factors, keyed by bytes per lane (2, 4, 8, 16)."""
import argparse
import collections
import csv
import glob
import json
import os

TRUE_BYTES = float(1 << 30)
WIDTH = {"read_u16_kernel": 2, "read_kernel<float>": 4, "read_kernel<HIP_vector_type<float, 2u> >": 8,
         "read_kernel<HIP_vector_type<float, 4u> >": 16, "write_u16_kernel": 2, "write_kernel<float>": 4,
         "write_kernel<HIP_vector_type<float, 2u> >": 8, "write_kernel<HIP_vector_type<float, 4u> >": 16}


def collect(d, counter):
    """kernel name -> per-dispatch counter values (rows of one dispatch summed, as tools/pmc_traffic.py does)."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"].replace("void ", "", 1).split("(")[0].strip()
            per[name][(f, r.get("Dispatch_Id", r.get("Correlation_Id")))] += float(r["Counter_Value"])
    return {k: list(v.values()) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("-o", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                               "profiles", "pmc_calib.json"))
    a = ap.parse_args()
    fe, wr = collect(a.fetch_dir, "FETCH_SIZE"), collect(a.write_dir, "WRITE_SIZE")
    out = {"true_bytes_per_kernel": TRUE_BYTES, "fetch": {}, "write": {}, "raw": {}}
    for name, w in WIDTH.items():
        src, key = (fe, "fetch") if name.startswith("read") else (wr, "write")
        vals = src.get(name)
        if not vals:
            continue
        per = sum(vals) / len(vals)
        out["raw"][name] = vals
        out[key][str(w)] = round(per * 1024.0 / TRUE_BYTES, 4)
    json.dump(out, open(a.o, "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("fetch", "write")}))


if __name__ == "__main__":
    main()
