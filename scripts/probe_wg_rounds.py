"""Round budget of the workgroup warm pass (wg_warm) on C2 and C5a: bench timing
(Iter0 + K iterations through phx_iterk)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

K = int(os.environ.get("K", "10"))
W = bench.workloads()
for name in os.environ.get("CONFIGS", "C2,C5a").split(","):
    w = W[name]
    for wg in [int(v) for v in os.environ.get("WG", "16,8,4").split(",")]:
        so = {"wg_warm": wg}
        ph = bench.make_ph(w, w["S"], 1, 1.0, so, K)
        bench.timed_run(ph, K)
        ph = bench.make_ph(w, w["S"], 1, 1.0, so, K)
        T, T0, Tk = bench.timed_run(ph, K)
        st = getattr(ph, "iterk_stats", None) or {}
        print("%-4s wg_warm %2d: T %.2f ms Iter0 %.2f ms iterk %.3f ms/iteration value %.3g steady %.3g stops %s" % (
            name, wg, T * 1e3, T0 * 1e3, Tk * 1e3 / K, w["S"] * (K + 1) / T, w["S"] * K / Tk,
            st.get("straggler_stops")), flush=True)
