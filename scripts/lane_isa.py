"""Offline look at the JIT lane kernels (no GPU): the farmer (or another model's)
lane source from the host emulation, compiled by hipcc for gfx950 to ISA with
the resource-usage remarks.  python scripts/lane_isa.py [farmer|aircond] [outdir]"""
import ctypes
import os
import subprocess
import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
import mpisppy_amd  # noqa: E402,F401
from mpisppy_amd import _native  # noqa: E402
from mpisppy_amd.examples import farmer, aircond  # noqa: E402
from mpisppy_amd.utils import sputils  # noqa: E402
from helpers import ph_options  # noqa: E402
from mpisppy_amd.opt.ph import PH  # noqa: E402


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "farmer"
    out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/isa"
    os.makedirs(out, exist_ok=True)
    emu = _native.Lib(os.path.join(_ROOT, "tests", "emu", "libphx_emu.so"), prefix="emu_phx_")
    if model == "farmer":
        names, cr, kw, nodes = farmer.scenario_names_creator(12), farmer.scenario_creator, {"num_scens": 12}, None
    else:
        bfs = [3, 3, 3]
        names = ["scen%d" % i for i in range(27)]
        cr, kw, nodes = aircond.scenario_creator, {"branching_factors": bfs}, \
            sputils.create_nodenames_from_branching_factors(bfs)
    ph = PH(ph_options(1), names, cr, scenario_creator_kwargs=kw, all_nodenames=nodes, _native_lib=emu,
            _device="cpu")
    fn = emu.lib.emu_phx_lane_source
    fn.restype = ctypes.c_char_p
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    src = fn(ph._ctx, 2).decode()
    path = os.path.join(out, "lane_%s.hip" % model)
    open(path, "w").write(src)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only", "-S",
           "-I", os.path.join(_ROOT, "mpi-sppy_amd", "csrc"), "-Rpass-analysis=kernel-resource-usage",
           "-o", os.path.join(out, "lane_%s.s" % model), path]
    r = subprocess.run(cmd, capture_output=True, text=True)
    open(os.path.join(out, "lane_%s.remarks" % model), "w").write(r.stderr)
    print(r.returncode, path)


if __name__ == "__main__":
    main()
