"""The workgroup solver's blocked Schur-complement inverse (phx_wg.h
wg_blk_cholesky / wg_blk_trtri / wg_blk_lauum, f64 MFMA tiles on the GPU)
through the phx_debug_spd_inverse hook, against numpy: to rounding on
well-conditioned matrices, and to the Cholesky-based inverse's own accuracy
on the nearly singular complements of degenerate faces (B B^T / reg + reg I
with rank-deficient B, reg = 1e-6: the solver's regularisation)."""
import ctypes

import numpy as np
import pytest

CASES = [(1, 0), (5, 0), (16, 0), (17, 0), (20, 3), (33, 0), (40, 10), (48, 0), (61, 3), (64, 0), (64, 12)]


def spd(ma, deficient, seed):
    rng = np.random.default_rng(seed)
    r = ma - deficient
    B = rng.standard_normal((ma, r))
    if deficient:
        return B @ B.T / 1e-6 + 1e-6 * np.eye(ma)
    return B @ B.T + 0.5 * np.eye(ma)


def run(lib, S):
    ma = S.shape[0]
    S = np.ascontiguousarray(S, dtype=np.float64)
    out = np.zeros_like(S)
    rc = lib.debug_spd_inverse(S.ctypes.data_as(ctypes.c_void_p), ma, out.ctypes.data_as(ctypes.c_void_p))
    return rc, out


def check(lib):
    for k, (ma, deficient) in enumerate(CASES):
        S = spd(ma, deficient, k)
        rc, X = run(lib, S)
        assert rc == 0, (ma, deficient, rc)
        assert np.array_equal(X, X.T), (ma, deficient)          # written as both triangles of one tile
        res = np.max(np.abs(S @ X - np.eye(ma)))
        if deficient:
            # the scalar Cholesky-based inverse's accuracy on these (|S X - I| ~ 1e-3)
            ref = np.linalg.cholesky(S)
            Li = np.linalg.inv(ref)
            res_ref = np.max(np.abs(S @ (Li.T @ Li) - np.eye(ma)))
            assert res < max(20 * res_ref, 1e-2), (ma, deficient, res, res_ref)
        else:
            assert res < 1e-11 * max(1.0, np.linalg.cond(S)), (ma, res)
            assert np.max(np.abs(X - np.linalg.inv(S))) < 1e-10 * np.max(np.abs(np.linalg.inv(S))) * np.linalg.cond(S)
    # not positive definite: refused
    rc, _ = run(lib, -np.eye(7))
    assert rc == 1


def test_blocked_inverse_emu(emu):
    check(emu)


@pytest.mark.gpu
def test_blocked_inverse_gpu(gpu_lib):
    check(gpu_lib)
