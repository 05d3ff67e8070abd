"""The lane solver's JIT source compiles for gfx950 (CPU, no GPU).

The GPU library generates one HIP source per problem STRUCTURE at
phx_set_problem (csrc/phx_jit.h lane_kernel_source) and hands it to hipRTC on
the GPU box, so a compile error there would only surface on the GPU.  The host
emulation builds the same LaneStructure from the same setup code; here its
source goes through hipRTC (libhiprtc, which needs no GPU) with the library's
own options (phx_kernels.hip jit_compile), and every kernel the library loads
must be present in the code object.
"""
import ctypes
import os

import pytest

from helpers import ph_options
from mpisppy_amd.examples import farmer, aircond, hydro
from mpisppy_amd.opt.ph import PH
from mpisppy_amd.utils import sputils

_CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy_amd", "csrc")
_HIPRTC = "/opt/rocm/lib/libhiprtc.so"
KERNELS = ["phx_lane_cold", "phx_lane_cold_as", "phx_lane_warm", "phx_lane_warm_list", "phx_lane_map",
           "phx_fz_tail", "phx_lane_seed", "phx_lane_warm_fz", "phx_lane_warm_fz1", "phx_lane_all",
           "phx_lane_list_all", "phx_lane_all_rl", "phx_lane_all_pk"]


def hiprtc_compile(src):
    rtc = ctypes.CDLL(_HIPRTC)
    prog = ctypes.c_void_p()
    hdr = open(os.path.join(_CSRC, "phx_lane.h"), "rb").read()
    names = (ctypes.c_char_p * 1)(b"phx_lane.h")
    srcs = (ctypes.c_char_p * 1)(hdr)
    assert rtc.hiprtcCreateProgram(ctypes.byref(prog), src.encode(), b"phx_lane_kernel.hip", 1, srcs, names) == 0
    opts = (ctypes.c_char_p * 3)(b"--offload-arch=gfx950", b"-O3", b"-std=c++17")
    rc = rtc.hiprtcCompileProgram(prog, 3, opts)
    size = ctypes.c_size_t()
    rtc.hiprtcGetProgramLogSize(prog, ctypes.byref(size))
    log = ctypes.create_string_buffer(size.value + 1)
    rtc.hiprtcGetProgramLog(prog, log)
    code_size = ctypes.c_size_t()
    code = b""
    if rc == 0:
        rtc.hiprtcGetCodeSize(prog, ctypes.byref(code_size))
        buf = ctypes.create_string_buffer(code_size.value)
        rtc.hiprtcGetCode(prog, buf)
        code = buf.raw
    rtc.hiprtcDestroyProgram(ctypes.byref(prog))
    return rc, log.value.decode(errors="replace"), code


def lane_source(emu, creator, names, kw, nodes=None):
    ph = PH(ph_options(1), names, creator, scenario_creator_kwargs=kw, all_nodenames=nodes,
            _native_lib=emu, _device="cpu")
    fn = emu.lib.emu_phx_lane_source
    fn.restype = ctypes.c_char_p
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    return fn(ph._ctx, 2).decode()


CASES = {
    "farmer": (farmer.scenario_creator, farmer.scenario_names_creator(200), {"num_scens": 200}, None),
    "aircond": (aircond.scenario_creator, ["scen%d" % i for i in range(27)], {"branching_factors": [3, 3, 3]},
                sputils.create_nodenames_from_branching_factors([3, 3, 3])),
    "hydro": (hydro.scenario_creator, hydro.scenario_names_creator(9), {"branching_factors": [3, 3]},
              sputils.create_nodenames_from_branching_factors([3, 3])),
}


@pytest.mark.skipif(not os.path.exists(_HIPRTC), reason="no hipRTC in this image")
@pytest.mark.parametrize("case", sorted(CASES))
def test_lane_source_compiles_gfx950(emu, case):
    creator, names, kw, nodes = CASES[case]
    src = lane_source(emu, creator, names, kw, nodes)
    assert "struct PT" in src, "the lane solver does not serve %s" % case
    rc, log, code = hiprtc_compile(src)
    assert rc == 0, log[-4000:]
    for k in KERNELS:
        assert k.encode() in code, k
