"""Extract netdes instance data from the reference's text files
(examples/netdes/data/network-NN-KK-DD-ID.dat) into compressed .npz data files shipped
with the package (mpi-sppy_amd/examples/data/netdes_<instance>.npz).  Data only.

File layout, as read by the reference's ``examples/netdes/parse.py:17-74``: header
lines up to one starting with '+'; then N; density; cost ratio; adjacency matrix
(rows separated by ';', entries by ','); first-stage cost matrix c; K; probability
vector p; then per scenario one separator line, the second-stage cost matrix d, the
capacity matrix u and the demand vector b.  Edges are the nonzeros of the adjacency
matrix in row-major order (``np.where(A > 0)``, parse.py:58-59); the .npz stores
every per-edge quantity in that order."""
import os
import sys

import numpy as np

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy_amd", "examples",
                   "data")
INSTANCES = ["network-10-10-H-01", "network-50-30-H-01"]


def _mat(line):
    return np.array([r.split(",") for r in line.strip().split(";")], dtype=np.float64)


def _vec(line):
    return np.array(line.strip().split(","), dtype=np.float64)


def read(fname):
    with open(fname) as f:
        lines = iter(f.read().split("\n"))
    while not next(lines).startswith("+"):
        pass
    N = int(next(lines))
    density = float(next(lines))
    ratio = int(next(lines))
    adj = _mat(next(lines))
    c = _mat(next(lines))
    K = int(next(lines))
    p = _vec(next(lines))
    ix, iy = np.nonzero(adj > 0)
    d, u, b = [], [], []
    for _ in range(K):
        next(lines)
        d.append(_mat(next(lines))[ix, iy])
        u.append(_mat(next(lines))[ix, iy])
        b.append(_vec(next(lines)))
    assert adj.shape == (N, N) and len(p) == K
    return dict(N=np.int64(N), density=np.float64(density), ratio=np.int64(ratio),
                edges=np.stack([ix, iy], 1).astype(np.int32), c=c[ix, iy], p=p,
                d=np.array(d), u=np.array(u), b=np.array(b))


def main():
    os.makedirs(OUT, exist_ok=True)
    for inst in INSTANCES:
        data = read(os.path.join(REF, "examples", "netdes", "data", inst + ".dat"))
        E = len(data["edges"])
        print(inst, "N", int(data["N"]), "E", E, "K", len(data["p"]), "min u", data["u"].min(),
              "d varies", bool(np.any(data["d"] != data["d"][0])), "u varies", bool(np.any(data["u"] != data["u"][0])),
              "sum b", np.abs(data["b"].sum(1)).max())
        np.savez_compressed(os.path.join(OUT, "netdes_%s.npz" % inst), **data)


if __name__ == "__main__":
    main()
