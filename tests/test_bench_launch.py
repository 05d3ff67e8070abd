"""bench.py's own N-rank launch (the driver's `python bench.py --gpus N` shape): with
no WORLD_SIZE in the environment it starts N ranks itself (torch.distributed.run,
127.0.0.1) before any GPU call.  Run here through the --device cpu test hook (gloo +
the host emulation library): the 2-rank line reports n_gpus = 2 and the same x-bar
and trivial bound as the 1-rank run (scenarios sharded contiguously, one fused
all-reduce per PH iteration)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--device", "cpu", "--scens", "600",
           "--steps", "3", "--warmup", "1", "--no-conv", "--no-cpu-baseline", "--configs", "none", "--ar-probe", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 prints the one JSON line
    return json.loads(lines[0])


def test_bench_launches_ranks_cpu():
    one, two = _bench(1), _bench(2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["scenarios"] == 600 and two["config"]["scenarios_per_gpu"] == 300
    assert two["steps"] == 3 and two["value"] > 0
    a, b = one["final"], two["final"]
    assert np.allclose(a["xbar"]["ROOT"], b["xbar"]["ROOT"], rtol=1e-12, atol=1e-12)
    assert abs(a["trivial_bound"] - b["trivial_bound"]) <= 1e-12 * abs(a["trivial_bound"])
