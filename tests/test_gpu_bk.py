"""The Bunch-Kaufman variants (bk_wave.hpp: bk_factor_regs_piv in registers, bk_factor_fixed in LDS with unrolled scans
-- k_gkkt_chain's --, bk_factor_regs in natural order with the fixed fallback) against the LDS routine of k_gkkt
(bk_factor_wave), on the device, bit for bit: the lower triangle (L and D), perm, piv and the inertia.

The stage blocks are built like the C2 chain's K = [[Q_uu, h J_n^T], [h J_n, -dc]] (NU = 7 controls, NET = 2 line rows;
a small q-dot diagonal against h J_n is what makes Bunch-Kaufman take 2x2 pivots), plus general symmetric and indefinite
blocks, blocks whose upper triangle differs from the lower in the last bit (K as assembled entry by entry), blocks with
fixed-control identity rows, and singular ones.
"""
import ctypes as C

import numpy as np
import pytest

from mpc_fatigue_amd import _lib

pytestmark = pytest.mark.gpu

M, LD, NU = 9, 10, 7


def _blocks(rng, n):
    out = []
    for t in range(n):
        kind = t % 6
        if kind == 0:  # C2-like: small PSD q-dot block, h J_n rows, dc = 0
            B = rng.normal(size=(NU, NU)) * 10.0 ** rng.uniform(-4, -1)
            Q = B @ B.T + np.diag(10.0 ** rng.uniform(-8, -2, NU))
            h = 0.05
            J = rng.normal(size=(2, NU)) * h
            J[:, 6] = 0.0
            K = np.block([[Q, J.T], [J, -rng.choice([0.0, 1e-8]) * np.eye(2)]])
        elif kind == 1:  # general symmetric
            A = rng.normal(size=(M, M))
            K = A + A.T
        elif kind == 2:  # indefinite Q (a try with the wrong inertia)
            A = rng.normal(size=(NU, NU))
            Q = A + A.T
            J = rng.normal(size=(2, NU)) * 0.05
            K = np.block([[Q, J.T], [J, np.zeros((2, 2))]])
        elif kind == 3:  # stage 0: fixed controls (identity rows and columns)
            A = rng.normal(size=(M, M)) * 1e-3
            K = A @ A.T
            for a in rng.choice(NU, 3, replace=False):
                K[a, :] = 0.0
                K[:, a] = 0.0
                K[a, a] = 1.0
            K[7:, 7:] = 0.0
            K[7:, :7] *= 30.0
            K[:7, 7:] *= 30.0
        elif kind == 4:  # singular: a zero row / column
            A = rng.normal(size=(M, M))
            K = A + A.T
            z = rng.integers(M)
            K[z, :] = 0.0
            K[:, z] = 0.0
        else:  # tiny diagonal everywhere: 2x2 pivots from the first column on
            A = rng.normal(size=(M, M))
            K = A + A.T
            K[np.diag_indices(M)] *= 1e-6
        K = np.array(K, dtype=np.float64)
        if t % 2 == 1:  # upper triangle off by one ulp here and there (entry-by-entry assembly)
            iu = np.triu_indices(M, 1)
            flip = rng.random(len(iu[0])) < 0.5
            up = K[iu]
            K[iu] = np.where(flip, np.nextafter(up, np.inf), up)
        P = np.zeros((M, LD))
        P[:, :M] = K
        out.append(P)
    return np.ascontiguousarray(np.array(out))


@pytest.mark.parametrize("variant", [0, 1, 2, 3], ids=["regs_piv", "lds_fixed", "regs_natural_fixed", "regs_loop"])
def test_bunch_kaufman_variants_match_lds_bit_for_bit(variant):
    rng = np.random.default_rng(7)
    n = 3000
    K = _blocks(rng, n)
    R = np.zeros_like(K)
    W = np.zeros_like(K)
    meta = np.zeros((n, 2 * M + 6), np.int32)
    L = _lib.lib()
    assert _lib.check(L.mf_debug_bk_compare(_lib.dptr(K), n, variant, _lib.dptr(R), _lib.dptr(W), _lib.iptr(meta))) == M
    il = np.tril_indices(M)
    lr = R[:, :, :M][:, il[0], il[1]]
    lw = W[:, :, :M][:, il[0], il[1]]
    same_lower = np.all((lr.view(np.uint64) == lw.view(np.uint64)) | (np.isnan(lr) & np.isnan(lw)), axis=1)
    same_meta = np.all(meta[:, :M] == meta[:, M:2 * M], axis=1) & np.all(meta[:, 2 * M:2 * M + 3] == meta[:, 2 * M + 3:],
                                                                           axis=1)
    piv = meta[:, :M] >> 8
    two = (piv == 2).any(axis=1)
    swapped = np.any((meta[:, :M] & 255) != np.arange(M), axis=1)
    print(f"blocks {n}: 2x2 pivots in {two.sum()}, row swaps in {swapped.sum()}, "
          f"lower triangles equal {same_lower.sum()}, perm/piv/inertia equal {same_meta.sum()}")
    assert two.sum() > n // 4 and swapped.sum() > n // 4
    bad = np.flatnonzero(~(same_lower & same_meta))
    assert bad.size == 0, f"first mismatching blocks {bad[:10]}"
