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


def _bench(n, extra=("--no-conv", "--no-cpu-baseline", "--configs", "none"), tmp=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--device", "cpu", "--scens", "600",
           "--steps", "3", "--warmup", "1", "--ar-probe", "0"] + list(extra)
    if tmp is not None:
        cmd += ["--detail", str(tmp)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 prints the one JSON line
    last = r.stdout.rstrip("\n").splitlines()[-1]
    assert last == lines[0]                            # ... as stdout's LAST line
    assert len(last.encode()) <= 8192, len(last.encode())
    return json.loads(last)


def test_bench_line_compact_cpu(tmp_path):
    """The driver parses stdout's last line (<= 8 KB): the contract keys, the roofline,
    the CPU baseline, conv_time and a per-config summary; the full record goes to
    the --detail file."""
    detail = tmp_path / "detail.json"
    d = _bench(1, extra=("--configs", "C1,C4", "--config-steps", "2", "--cpu-scens", "60", "--cpu-iters", "1",
                         "--cpu-procs", "2", "--conv-max-iters", "50"), tmp=detail)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "roofline",
              "cpu_baseline", "conv_time", "iter0_s", "steady", "configs"):
        assert k in d, k
    assert d["roofline"]["kernel"] and "frac" in d["roofline"] and "traffic_ratio" in d["roofline"]
    assert d["cpu_baseline"]["value"] > 0 and d["cpu_baseline"]["cores"] == 2
    sp = d["cpu_baseline"]["spread"]                 # median of three samples, with their range
    assert sp["samples"] == 3 and sp["min"] <= d["cpu_baseline"]["value"] <= sp["max"]
    for nm in ("C1", "C4"):
        c = d["configs"][nm]
        assert "error" not in c, c
        for k in ("value", "ms_per_step", "frac", "traffic_ratio", "cpu", "avg_launch_us"):
            assert k in c, (nm, k)
    full = json.loads(detail.read_text())
    assert full["configs"]["C4"]["workload"].startswith("aircond")
    assert full["value"] == d["value"] or abs(full["value"] - d["value"]) <= 1e-5 * full["value"]


def test_bench_launches_ranks_cpu():
    one, two = _bench(1), _bench(2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["scenarios"] == 600 and two["config"]["scenarios_per_gpu"] == 300
    assert two["steps"] == 3 and two["value"] > 0
    a, b = one["final"], two["final"]
    assert np.allclose(a["xbar"]["ROOT"], b["xbar"]["ROOT"], rtol=1e-12, atol=1e-12)
    assert abs(a["trivial_bound"] - b["trivial_bound"]) <= 1e-12 * abs(a["trivial_bound"])


def test_compact_line_cap_cpu():
    """whatever the record holds (long error strings, long CPU sample
    text, many configs), the compact line fits LINE_CAP and keeps the contract keys."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bm)
    big = "x" * 20000
    res = {"metric": "m", "value": 1.0, "unit": "u", "n_gpus": 1, "steps": 2, "warmup": 1, "ms_per_step": 1.0,
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64", "data": big,
           "config": {"workload": big}, "roofline": {"kernel": "k", "frac": 0.1, "traffic_ratio": 1.0},
           "cpu_baseline": {"value": 1.0, "unit": "u", "cores": 1, "kind": "port", "sample": big,
                            "whole_host": {"value": 2.0, "how": big, "cap": big},
                            "spread": {"samples": 3, "min": 0.9, "max": 1.1}},
           "configs": {"C%d" % i: {"error": big} for i in range(200)}}
    out = bm.compact_line(res, "detail.json")
    line = json.dumps(out)
    assert len(line.encode()) <= bm.LINE_CAP
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "roofline", "cpu_baseline"):
        assert k in out, k
