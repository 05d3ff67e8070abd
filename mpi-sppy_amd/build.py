"""Build the native library in-tree (hipcc, gfx950) — no JIT cache, so the
built ``libphx.so`` travels with the repository snapshot to the GPU box."""
import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _newer(target, sources):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(s) <= t for s in sources)


def build_phx(force=False, verbose=True):
    """hipcc --offload-arch=gfx950 -O3 csrc/phx_kernels.hip -> libphx.so"""
    src = os.path.join(_HERE, "csrc", "phx_kernels.hip")
    deps = [src, os.path.join(_HERE, "csrc", "phx_core.h"), os.path.join(_HERE, "csrc", "phx_setup.h"),
            os.path.join(_ROOT, "include", "phx.h")]
    out = os.path.join(_HERE, "libphx.so")
    if not force and _newer(out, deps):
        return out
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-o", out, src]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return out


def build_emu(force=False, verbose=True):
    """Test-only host emulation of the ABI (tests/emu) — g++."""
    src = os.path.join(_ROOT, "tests", "emu", "phx_emu.cpp")
    deps = [src, os.path.join(_HERE, "csrc", "phx_core.h"), os.path.join(_HERE, "csrc", "phx_setup.h"),
            os.path.join(_ROOT, "include", "phx.h")]
    out = os.path.join(_ROOT, "tests", "emu", "libphx_emu.so")
    if not force and _newer(out, deps):
        return out
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", out, src]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    build_phx(force="--force" in sys.argv)
    build_emu(force="--force" in sys.argv)
