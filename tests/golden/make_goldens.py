"""Regenerate tests/golden/ref_goldens.json from the reference's own files.

Runs only where /root/reference exists (the build container); the committed
JSON travels instead.  Every value is copied from a reference data file, test
assertion or documentation output — the provenance is recorded per entry.
Loaders execute nothing from the files (csv text, numpy allow_pickle=False).
"""
import csv
import json
import os

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    g = {}
    w_rows = list(csv.reader(open(os.path.join(REF, "mpisppy/tests/examples/w_test_data/w_file.csv"))))[:9]
    x_rows = list(csv.reader(open(os.path.join(REF, "mpisppy/tests/examples/w_test_data/xbar_file.csv"))))[:3]
    g["farmer3_rho1_5iters"] = {
        "source": "mpisppy/tests/examples/w_test_data/{w_file,xbar_file}.csv (first block); "
                  "setup mpisppy/tests/test_w_writer.py:53-76 (farmer 3 scen, rho 1, PHIterLimit 5)",
        "W": [[r[0], r[1], float(r[2])] for r in w_rows],
        "xbar": [[r[0], float(r[1])] for r in x_rows],
        "assert_places": 5,
    }
    g["docs_farmer_rho10_5iters"] = {
        "source": "doc/src/examples.rst:322-338 (gather_var_values_to_rank0 after ph_main, rho 10, 5 iters)",
        "x": {"good": {"X[BEETS]": 280.6489711937925, "X[CORN]": 85.26131687116064, "X[WHEAT]": 134.0897119350402},
              "average": {"X[BEETS]": 283.2796296293019, "X[CORN]": 80.00000000014425,
                          "X[WHEAT]": 136.72037037055298},
              "bad": {"X[BEETS]": 280.64897119379475, "X[CORN]": 85.26131687116226, "X[WHEAT]": 134.08971193504266}},
    }
    g["docs_farmer_ef"] = {"source": "doc/src/examples.rst:225-228, 244-248", "objective": -108390.0,
                           "x": {"X[BEETS]": 250.0, "X[CORN]": 80.0, "X[WHEAT]": 170.0}}
    g["farmer30_trivial_bound"] = {"source": "mpisppy/tests/test_aph.py:246-249 (Scenario1..30, 3 sig)",
                                   "value": -137846, "sig": 3}
    nn = np.load(os.path.join(REF, "mpisppy/tests/examples/rho_test_data/farmer_cyl_nonants.npy"),
                 allow_pickle=False)
    g["farmer3_converged_nonants"] = {"source": "mpisppy/tests/examples/rho_test_data/farmer_cyl_nonants.npy",
                                      "CORN0,SUGAR_BEETS0,WHEAT0": [float(v) for v in nn]}
    g["aircond_ef_bf432"] = {"source": "mpisppy/tests/test_conf_int_aircond.py:199-205 (start_seed 0, 2 sig)",
                             "objective": 970, "sig": 2}
    g["gradient_rho_iter0"] = {"source": "mpisppy/tests/test_gradient_rho.py (w_denom 25 = |x_scen0[CORN0]|)",
                               "scen0_x": {"CORN0": 25.0, "SUGAR_BEETS0": 375.0, "WHEAT0": 100.0}}
    g["farmer_xhat_eval"] = {
        "source": "mpisppy/tests/test_conf_int_farmer.py:63-76, 168-202 (Xhat_Eval over scen0..99 with "
                  "num_scens=10, xhat ROOT=[74,245,181]; 2 sig)",
        "names": 100, "num_scens": 10, "xhat_ROOT": [74.0, 245.0, 181.0],
        "evaluate": -1300000.0, "evaluate_one_scen0": -48000.0, "sig": 2}
    g["aircond_xhat_eval"] = {
        "source": "mpisppy/tests/test_conf_int_aircond.py:38-93, 213-240 (BF [4,3,2], start_seed 0, "
                  "xhat [200,0] at every non-leaf node; 2 sig, 'rebaselined feb 2022')",
        "branching_factors": [4, 3, 2], "xhat_node": [200.0, 0.0],
        "evaluate": 1000.0, "evaluate_one_scen0": 1100.0, "sig": 2}
    g["hydro_ph_bf33"] = {
        "source": "mpisppy/tests/test_ef_ph.py:32-52 (options: rho 1, PHIterLimit 10, convthresh 0.001), "
                  ":545-563 (BF [3,3], Scen1..Scen9, create_nodenames_from_branching_factors), "
                  ":622-640 test_ph_solve (trivial bound 180, Eobjective after disable_W_and_prox 190; 2 sig), "
                  ":581-601 test_ef_solve (EF Scen7.Pgt[2] 60; 1 sig)",
        "branching_factors": [3, 3], "rho": 1.0, "PHIterLimit": 10, "convthresh": 0.001,
        "trivial_bound": 180, "Eobj_W_prox_disabled": 190, "sig": 2,
        "ef_Scen7_Pgt2": 60, "ef_sig": 1}
    with open(os.path.join(HERE, "ref_goldens.json"), "w") as f:
        json.dump(g, f, indent=1)


if __name__ == "__main__":
    main()
