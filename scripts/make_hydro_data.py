"""Extract the hydro (elec3) scenario data from the reference's AMPL-style .dat files
(mpisppy/tests/examples/hydro/PySP/scenariodata/Scen{1..9}.dat) into one JSON data file
shipped with the package (mpi-sppy_amd/examples/data/hydro.json).  Data only: every
scalar and 1-D param of each scenario file, keyed by scenario name."""
import glob
import json
import os
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = os.path.join(REF, "mpisppy", "tests", "examples", "hydro", "PySP", "scenariodata")
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy_amd", "examples",
                   "data", "hydro.json")


def parse(fname):
    txt = "\n".join(line.split("#", 1)[0] for line in open(fname).read().splitlines())
    out = {}
    for m in re.finditer(r"param\s+(\w+)\s*:=(.*?);", txt, re.S):
        name, vals = m.group(1), m.group(2).split()
        if len(vals) == 1:
            out[name] = float(vals[0])
        else:
            out[name] = {vals[k]: float(vals[k + 1]) for k in range(0, len(vals), 2)}
    return out


def main():
    data = {}
    for f in sorted(glob.glob(os.path.join(SRC, "Scen[0-9]*.dat"))):
        data[os.path.basename(f)[:-4]] = parse(f)
    assert len(data) == 9, sorted(data)
    with open(OUT, "w") as fo:
        json.dump({"source": "mpisppy/tests/examples/hydro/PySP/scenariodata/Scen{1..9}.dat", "scenarios": data},
                  fo, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
