"""Average duration of a kernel over the timed window of a rocprofv3 kernel
trace: its last N launches above 1 % of the longest (phx_iterk's gated
launches dropped) -- the figure to set beside bench.py's roofline.avg_launch_us.
python scripts/trace_window.py <run_kernel_trace.csv> <kernel> <N>"""
import csv
import json
import sys

path, kernel, n = sys.argv[1], sys.argv[2], int(sys.argv[3])


def base(name):
    b = name.split("(")[0].replace("void ", "").split("<")[0].strip()
    return {"k_sp_solve_t": "k_sp_solve"}.get(b, b)


rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path))
              if base(r["Kernel_Name"]) == kernel)
d = [(e - s) / 1e3 for s, e in rows]
top = max(d) if d else 0.0
live = [v for v in d if v > 0.01 * top][-n:]
print(json.dumps({"trace": path, "kernel": kernel, "window": "last %d launches above 1 %% of the longest" % n,
                  "launches": len(live), "avg_us": sum(live) / max(len(live), 1),
                  "min_us": min(live) if live else None, "max_us": max(live) if live else None}))
