"""Content hashes of the sources each measured kernel is built from, so a
committed PMC summary (profiles/r*_pmc*_<tag>_<kernel>.json) can be matched to
the code it measured (bench.py refuses a summary whose hash differs from the
tree it runs in).  python scripts/src_hash.py  -> JSON {kernel: sha256}"""
import hashlib
import json
import os

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_CSRC = os.path.join(_ROOT, "mpi-sppy_amd", "csrc")
# phx_kernels.hip holds every launch (grids, options, the loop): part of each set
_LANE = ["phx_lane.h", "phx_jit.h", "phx_setup.h", "phx_kernels.hip"]
KERNEL_SOURCES = {
    "phx_lane_warm": _LANE, "phx_lane_warm_fz": _LANE, "phx_lane_warm_fz1": _LANE, "phx_lane_all": _LANE,
    "phx_lane_all_rl": _LANE,
    "phx_lane_all_pk": _LANE,
    "phx_lane_warm_fzr2": _LANE, "phx_lane_warm_fzc": _LANE,
    "k_wg_warm": ["phx_wg.h", "phx_core.h", "phx_setup.h", "phx_kernels.hip"],
    "k_sp_solve": ["phx_sp.h", "phx_core.h", "phx_setup.h", "phx_kernels.hip"],
}


def source_hash(kernel):
    files = KERNEL_SOURCES.get(kernel)
    if not files:
        return None
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(_CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()


def hashes():
    return {k: source_hash(k) for k in KERNEL_SOURCES}


if __name__ == "__main__":
    print(json.dumps(hashes(), indent=1))
