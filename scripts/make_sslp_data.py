"""Extract the sslp_15_45 instance data from the reference's AMPL-style .dat files
(examples/sslp/data/sslp_15_45_{5,10,15}/scenariodata/ScenarioK.dat) into one JSON
data file shipped with the package (mpi-sppy_amd/examples/data/sslp_15_45.json).
Data only: the deterministic parameters (identical in every scenario file — asserted)
and each shipped scenario's ClientPresent vector."""
import glob
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy_amd", "examples",
                   "data", "sslp_15_45.json")


def parse(fname):
    txt = open(fname, "rb").read().decode("latin-1").replace("\r", "")
    out = {}
    for m in re.finditer(r"param\s+(\w+)\s*(:=|:)(.*?);", txt, re.S):
        name, kind, body = m.group(1), m.group(2), m.group(3)
        if kind == ":=" and name in ("NumServers", "NumClients", "Capacity", "Penalty"):
            out[name] = float(body.split()[0])
        elif kind == ":=":                       # 1-D table "i v"
            vals = body.split()
            out[name] = {int(vals[k]): float(vals[k + 1]) for k in range(0, len(vals), 2)}
        else:                                    # 2-D table "cols := rows"
            head, rows = body.split(":=", 1)
            cols = [int(c) for c in head.split()]
            tab = {}
            for line in rows.strip().split("\n"):
                t = line.split()
                if not t:
                    continue
                i = int(t[0])
                for c, v in zip(cols, t[1:]):
                    tab[(i, c)] = float(v)
            out[name] = tab
    return out


def main():
    det = None
    present = {}
    for inst in ("5", "10", "15"):
        d = os.path.join(REF, "examples", "sslp", "data", "sslp_15_45_" + inst, "scenariodata")
        files = sorted(glob.glob(os.path.join(d, "Scenario[0-9]*.dat")), key=lambda f: int(re.findall(r"\d+", os.path.basename(f))[0]))
        present[inst] = []
        for f in files:
            p = parse(f)
            ns, nc = int(p["NumServers"]), int(p["NumClients"])
            cur = {"NumServers": ns, "NumClients": nc, "Capacity": p["Capacity"],
                   "FixedCost": [p["FixedCost"][j] for j in range(1, ns + 1)],
                   "Revenue": [[p["Revenue"].get((i, j), 0.0) for j in range(1, ns + 1)] for i in range(1, nc + 1)],
                   "Demand": [[p["Demand"].get((i, j), 0.0) for j in range(1, ns + 1)] for i in range(1, nc + 1)]}
            if det is None:
                det = cur
            assert cur == det, "deterministic sslp data differ in %s" % f
            present[inst].append([int(p["ClientPresent"].get(i, 1)) for i in range(1, nc + 1)])
    det["Penalty"] = 1000.0          # ReferenceModel.py: Param(default = 1000.0)
    det["ClientPresent"] = present
    det["source"] = ("examples/sslp/data/sslp_15_45_{5,10,15}/scenariodata/ScenarioK.dat; model "
                     "examples/sslp/model/ReferenceModel.py (extracted by scripts/make_sslp_data.py)")
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(det, f)
    print("wrote", OUT, {k: len(v) for k, v in present.items()})


if __name__ == "__main__":
    main()
