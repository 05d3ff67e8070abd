"""Probe: run one BASELINE config through PH on the GPU and print per-solve stats.
    python scripts/probe_config.py <config> <iters> [key=value solver options ...]
config: farmer_cm10 | sslp10k | netdes50_10k | aircond | farmer100k.  Env PHX_SP=0/1 selects
the sparse solver (default: where the dense solvers do not fit)."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
import mpisppy_amd  # noqa: E402,F401
from mpisppy_amd.opt.ph import PH  # noqa: E402
from mpisppy_amd.examples import farmer, sslp, netdes, aircond  # noqa: E402
from mpisppy_amd.utils import sputils  # noqa: E402

CONFIGS = {
    "farmer_cm10": (farmer.scenario_creator, farmer.scenario_names_creator(1000),
                    {"num_scens": 1000, "crops_multiplier": 10}, None),
    "farmer100k": (farmer.scenario_creator, farmer.scenario_names_creator(100000), {"num_scens": 100000}, None),
    "sslp10k": (sslp.scenario_creator, sslp.scenario_names_creator(10000), {"num_scens": 10000}, None),
    "netdes50_10k": (netdes.scenario_creator, netdes.scenario_names_creator(10000),
                     {"instance": "network-50-30-H-01", "num_scens": 10000}, None),
    "aircond": (aircond.scenario_creator, ["scen%d" % i for i in range(1000)], {"branching_factors": [10, 10, 10]},
                sputils.create_nodenames_from_branching_factors([10, 10, 10])),
}


def main():
    cfg, iters = sys.argv[1], int(sys.argv[2])
    so = {}
    for kv in sys.argv[3:]:
        k, v = kv.split("=")
        so[k] = float(v) if "." in v or "e" in v else int(v)
    creator, names, kw, nodes = CONFIGS[cfg]
    opts = {"solver_name": "phx", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": 1e-10, "verbose": False,
            "display_progress": False, "iter0_solver_options": dict(so), "iterk_solver_options": dict(so)}
    t = time.time()
    ph = PH(opts, names, creator, scenario_creator_kwargs=kw, all_nodenames=nodes)
    torch.cuda.synchronize()
    t_setup = time.time() - t
    t = time.time()
    conv, E, tb = ph.ph_main()
    torch.cuda.synchronize()
    print(json.dumps({"config": cfg, "setup_s": t_setup, "ph_main_s": time.time() - t, "tb": tb, "Eobj": E,
                      "conv": conv, "jit": ph._native.jit_info(ph._ctx).decode(),
                      "iterk": getattr(ph, "iterk_stats", None)}))
    keys = ["wall_s", "not_optimal", "pdhg_iters", "lane_certified", "lane_warm_certified", "lane_ms",
            "lane_warm_ms", "wg_certified", "wg_ms", "sp_certified",
            "sp_ms", "sp_ipm_its", "sp_warm_rounds", "sp_cold_rounds", "sp_refine", "pdhg_ms", "ipm_ms", "polish_ms"]
    for i, s in enumerate(ph.solve_stats):
        print(i, json.dumps({k: (round(s[k], 3) if isinstance(s.get(k), float) else s.get(k)) for k in keys}))


if __name__ == "__main__":
    main()
