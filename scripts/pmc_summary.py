"""Per-kernel averages of rocprofv3 --pmc passes (run_counter_collection.csv),
with the gfx950 FETCH_SIZE correction (MI355X_MICROARCH.md, HBM section:
FETCH_SIZE reports half the bytes of a coalesced streaming read -> x2).

    python scripts/pmc_summary.py KERNEL dir1 [dir2 ...] > profiles/xxx.json
"""
import collections
import csv
import glob
import json
import os
import sys


def main(kernel, dirs):
    out = {"kernel": kernel, "counters": {}, "launches": {}}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            agg = collections.defaultdict(list)
            for r in csv.DictReader(open(f)):
                if r["Kernel_Name"].split("(")[0] == kernel:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            for k, v in agg.items():
                out["counters"][k] = sum(v) / len(v)
                out["launches"][k] = len(v)
    c = out["counters"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fetch = 2.0 * c["FETCH_SIZE"] * 1024.0      # KiB -> bytes, x2 gfx950 correction
        write = c["WRITE_SIZE"] * 1024.0
        out["hbm_bytes_per_launch"] = {"fetch_corrected": fetch, "write": write, "total": fetch + write}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
