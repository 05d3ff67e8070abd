"""The first PH iteration after Iter0 (rescue round budget of its warm pass):
bench timing (Iter0 + K iterations, farmer 100k) for several `rescue_rounds`."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402

S = int(os.environ.get("SCENS", "100000"))
K = int(os.environ.get("K", "20"))
w = {"names": farmer.scenario_names_creator, "creator": farmer.scenario_creator,
     "kw": lambda S, cm: {"num_scens": S, "crops_multiplier": cm}, "nodes": None}
for rr in [int(v) for v in os.environ.get("RR", "0,16,8,4").split(",")]:
    ph = bench.make_ph(w, S, 1, 1.0, {"rescue_rounds": rr}, K)
    bench.timed_run(ph, K)
    ts = [bench.timed_run(ph, K) for _ in range(3)]
    best = min(ts)
    print("rescue_rounds %d: T %.3f ms Iter0 %.3f ms iterk %.3f ms value %.3g stops %d" % (
        rr, best[0] * 1e3, best[1] * 1e3, best[2] * 1e3, S * (K + 1) / best[0],
        ph.iterk_stats["straggler_stops"]), flush=True)
