"""C2 (farmer crops_multiplier=10 x 1,000): the device loop (phx_iterk,
workgroup mode) against the Python host loop (native_loop 0), bench timing."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

K = int(os.environ.get("K", "20"))
w = bench.workloads()["C2"]
for so in ({}, {"native_loop": 0}, {"iterk_timing": 0}):
    ph = bench.make_ph(w, w["S"], 1, 1.0, so, K)
    bench.timed_run(ph, K)
    ph = bench.make_ph(w, w["S"], 1, 1.0, so, K)
    T, T0, Tk = bench.timed_run(ph, K)
    st = getattr(ph, "iterk_stats", None)
    print("%-22s T %.2f ms Iter0 %.2f ms iterk %.3f ms/iteration value %.3g steady %.3g %s" % (
        so, T * 1e3, T0 * 1e3, Tk * 1e3 / K, 1000 * (K + 1) / T, 1000 * K / Tk,
        {k: st[k] for k in ("straggler_stops", "stragglers", "wall_s")} if st else "host loop"), flush=True)
