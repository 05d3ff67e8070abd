"""Per-kernel averages of rocprofv3 --pmc passes (run_counter_collection.csv),
with the gfx950 FETCH_SIZE correction (MI355X_MICROARCH.md, HBM section:
FETCH_SIZE reports half the bytes of a coalesced streaming read -> x2).

    python scripts/pmc_summary.py KERNEL [--last N] [--skip-idle] dir1 [dir2 ...] > profiles/xxx.json

--last N keeps the last N launches of KERNEL in each pass (by dispatch id): the
timed window of a bench run that ends with its timed iterations (--no-conv).
--skip-idle drops launches below 1 % of the largest (phx_iterk's gated launches).
"""
import collections
import csv
import glob
import json
import os
import sqlite3
import sys


def base_name(name):
    """'void k_wg_warm<false>(phx::Prob, ...)' -> 'k_wg_warm' (template kernels
    count under their template's name)."""
    n = name.split("(")[0].strip()
    if n.startswith("void "):
        n = n[5:]
    n = n.split("<")[0]
    return ALIAS.get(n, n)


# kernels launched under another name than the one bench.py reports
ALIAS = {"k_sp_solve_t": "k_sp_solve"}


def main(kernel, dirs, last=None):
    out = {"kernel": kernel, "counters": {}, "launches": {}, "window": "last %d launches" % last if last else "all"}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            agg = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                if base_name(r["Kernel_Name"]) == kernel:
                    agg[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            add(agg, out, last)
        for f in glob.glob(os.path.join(d, "**", "*results.db"), recursive=True):
            agg = collections.defaultdict(lambda: collections.defaultdict(float))
            con = sqlite3.connect(f)
            for name, disp, ctr, val in con.execute(
                    "select kernel_name, dispatch_id, counter_name, value from counters_collection"):
                if base_name(name) == kernel:
                    agg[ctr][int(disp)] += float(val)
            add(agg, out, last)
    provenance(out, dirs)
    finish(out)


def add(agg, out, last):
    """per-dispatch sums -> mean over the (last) launches"""
    for k, per in agg.items():
        v = [per[i] for i in sorted(per)]
        if SKIP_IDLE and v:
            # gated launches (phx_iterk's pipeline past its stop: the kernel
            # exits at its first load) are not solves
            top = max(v)
            v = [x for x in v if x >= 0.01 * top]
        if last:
            v = v[-last:]
        out["counters"][k] = sum(v) / len(v)
        out["launches"][k] = len(v)


def provenance(out, dirs):
    """The sources the passes measured (src_hash.json written next to each pass
    by scripts/gpu_job.sh on the GPU box) and the git head this summary was
    made at: bench.py uses a summary only while its kernel's sources hash the same."""
    import subprocess
    shas = set()
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "src_hash.json"), recursive=True):
            shas.add(json.load(open(f)).get(out["kernel"]))
    out["source_sha256"] = shas.pop() if len(shas) == 1 else (None if not shas else "mixed")
    try:
        head = subprocess.run(["git", "rev-parse", "HEAD"], capture_output=True, text=True,
                              cwd=os.path.dirname(os.path.abspath(__file__))).stdout.strip()
    except OSError:
        head = None
    out["git_head_at_summary"] = head or None


def finish(out):
    c = out["counters"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fetch = 2.0 * c["FETCH_SIZE"] * 1024.0      # KiB -> bytes, x2 gfx950 correction
        write = c["WRITE_SIZE"] * 1024.0
        out["hbm_bytes_per_launch"] = {"fetch_corrected": fetch, "write": write, "total": fetch + write}
    print(json.dumps(out, indent=1))


SKIP_IDLE = False

if __name__ == "__main__":
    a = sys.argv[1:]
    last = None
    if "--skip-idle" in a:
        a.remove("--skip-idle")
        SKIP_IDLE = True
    if "--last" in a:
        i = a.index("--last")
        last = int(a[i + 1])
        del a[i:i + 2]
    main(a[0], a[1:], last)
