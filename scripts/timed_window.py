"""Kernel timeline of bench.py's TIMED run (Iter0 + K PH iterations) from a
rocprofv3 --kernel-trace [--hip-runtime-trace] database: the run starts at the
2nd seeded first solve (the template interior point: the 2nd phx_lane_cold launch
on one block; the 1st belongs to the warmup object).  Prints every kernel and
copy with its start offset, duration and the gap before it, and a per-phase
summary (Iter0 up to the first k_xbar, then per PH iteration).

    python scripts/timed_window.py gpurun_out/<tag> [occurrence=1] [max_rows=200]
"""
import glob
import sqlite3
import sys


def main():
    d = sys.argv[1]
    occ = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows_max = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    f = glob.glob(d + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(f)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    grid = "grid_x" if "grid_x" in cols else ("grid_size_x" if "grid_size_x" in cols else None)
    q = "select name,start,end%s from kernels order by start" % ("," + grid if grid else "")
    ks = []
    for r in c.execute(q):
        ks.append((r[1], r[2], "K " + r[0].split("(")[0][:44], r[3] if grid else None))
    try:
        ks += [(s, e, "C %d B" % sz, None) for s, e, sz in c.execute("select start,end,size from memory_copies")]
    except sqlite3.Error:
        pass
    ks.sort()
    # template interior points: phx_lane_cold with a grid of one block
    starts = [i for i, k in enumerate(ks) if k[2].startswith("K phx_lane_cold") and not k[2].startswith(
        "K phx_lane_cold_as") and (k[3] is None or k[3] <= 64)]
    if len(starts) <= occ:
        print("only %d seeded solves found" % len(starts))
        return
    i0 = starts[occ]
    i1 = starts[occ + 1] if occ + 1 < len(starts) else len(ks)
    t0 = ks[i0][0]
    prev_end = ks[i0 - 1][1] if i0 > 0 else t0
    phase = "Iter0"
    ph_t = {}
    ph_start = t0
    it = 0
    for n, (s, e, name, g) in enumerate(ks[i0:i1]):
        if name.startswith("K k_xbar") and phase == "Iter0":
            ph_t["Iter0"] = (ph_start, s)
            phase, ph_start, it = "it1", s, 1
        if n < rows_max:
            print("%-50s %9.1f %8.1f  gap %7.1f%s" % (name, (s - t0) / 1e3, (e - s) / 1e3, (s - prev_end) / 1e3,
                                                    "" if g is None else "  grid %d" % g))
        prev_end = max(prev_end, e)
    print("---")
    if "Iter0" in ph_t:
        a, b = ph_t["Iter0"]
        print("Iter0 (first kernel -> first k_xbar start): %.1f us" % ((b - a) / 1e3))
    print("window end (last kernel end - t0): %.1f us" % ((prev_end - t0) / 1e3))
    warm = [(s, e) for s, e, name, g in ks[i0:i1] if name.startswith("K phx_lane_warm")
            and not name.startswith("K phx_lane_warm_list")]
    print("phx_lane_warm launches: %d, us:" % len(warm), " ".join("%.1f" % ((e - s) / 1e3) for s, e in warm))


if __name__ == "__main__":
    main()
