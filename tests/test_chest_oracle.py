"""CPU checks of the oracle's channel-estimator restatement (oracle/orc_chest.c; chest_dl.c cannot be compiled here,
so these pin the restatement against an independent float64 numpy formulation of the same algorithm):

* INTERPOLATE (SRSLTE_ESTIMATOR_ALG_INTERPOLATE, chest_dl.c:430-567): per-pilot-symbol smoothing with the
  extrapolating same-length convolution (convolution.c:183-220), piecewise-linear frequency interpolation with
  linear extrapolation at both edges (interp.c:259-285, 6 subcarriers per pilot), linear time interpolation
  between the pilot symbols and extrapolation past the last (interp.c:137-188);
* AVERAGE: the same estimate on every OFDM symbol, and both algorithms share the REFS noise estimate.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import ue_dl_chain as uc


def conv_same_ext(x: np.ndarray, f: np.ndarray) -> np.ndarray:
    """convolution.c:183-220 (conv_same_extrapolates_extremes): head outputs read `first`, tail outputs `last`, whose
    extrapolated entries follow the reference's own coefficients."""
    M, N, h = len(f), len(x), len(f) // 2
    first = [(2 + h - i) * x[1] - (1 + h - i) * x[0] if i < h else x[i - h] for i in range(M + h)]
    last = [(2 + i - h) * x[N - 1] - (1 + i - h) * x[N - 2] if i >= M - 1 else x[N - M + i + 1] for i in range(M + h)]
    out = np.zeros(N, complex)
    for i in range(N):
        if i < h:
            seq = first[i: i + M]
        elif i < N - h:
            seq = x[i - h: i - h + M]
        else:
            j = i - (N - h)
            seq = last[j: j + M]
        out[i] = np.dot(np.asarray(seq, complex), f)
    return out


def lin_extrap(xp: np.ndarray, fp: np.ndarray, x: np.ndarray) -> np.ndarray:
    """Piecewise-linear interpolation of (xp, fp) at x with linear extrapolation from the end segments."""
    out = np.interp(x, xp, fp.real) + 1j * np.interp(x, xp, fp.imag)
    lo, hi = x < xp[0], x > xp[-1]
    s0 = (fp[1] - fp[0]) / (xp[1] - xp[0])
    s1 = (fp[-1] - fp[-2]) / (xp[-1] - xp[-2])
    out[lo] = fp[0] + (x[lo] - xp[0]) * s0
    out[hi] = fp[-1] + (x[hi] - xp[-1]) * s1
    return out


def gauss(order: int, sd: float) -> np.ndarray:
    c = order // 2
    f = np.exp(-((np.arange(order + 1) - c) ** 2) / (2 * sd * sd))
    return f / f.sum()


def numpy_interpolate(grid: np.ndarray, nof_prb: int, cell_id: int, sf: int, port: int, filt: np.ndarray | None):
    nre = 12 * nof_prb
    pos = uc.crs_positions(nof_prb, cell_id, port)
    crs = uc.crs_pilots(nof_prb, cell_id, port // 2, sf).astype(np.complex128)
    nsym = 4 if port < 2 else 2
    nref = 2 * nof_prb
    g = grid.astype(np.complex128).reshape(14, nre)
    pe = np.array([g[s, f] for s, f in pos]) * np.conj(crs[: nsym * nref])
    pe = pe.reshape(nsym, nref)
    rows, vals = [], []
    for l in range(nsym):
        s, f0 = pos[l * nref]
        x = pe[l] if filt is None else conv_same_ext(pe[l], filt)
        rows.append(s)
        vals.append(lin_extrap(f0 + 6 * np.arange(nref), x, np.arange(nre, dtype=float)))
    vals = np.array(vals)
    ce = np.zeros((14, nre), complex)
    for k in range(nre):
        ce[:, k] = lin_extrap(np.array(rows, float), vals[:, k], np.arange(14, dtype=float))
    return ce


@pytest.mark.parametrize("nof_prb,cell_id,sf,ft,coef", [(25, 3, 4, 0, (4.0, 1.0)), (50, 7, 0, 1, (0.2, 0.0)),
                                                        (6, 301, 9, 2, (0.0, 0.0)), (100, 1, 5, 0, (6.0, 2.0))])
def test_interpolate_estimator_vs_numpy(nof_prb, cell_id, sf, ft, coef):
    rng = np.random.default_rng(nof_prb + cell_id)
    G = 14 * 12 * nof_prb
    grids = (rng.standard_normal((1, G)) + 1j * rng.standard_normal((1, G))).astype(np.complex64)
    ce, _ = uc.chest_estimate(grids, nof_prb, 2, cell_id, sf, ft, coef, alg=1)
    filt = {0: gauss(int(coef[0]), coef[1]) if ft == 0 else None,
            1: np.array([coef[0], 1 - 2 * coef[0], coef[0]]), 2: None}[ft]
    for p in range(2):
        want = numpy_interpolate(grids[0], nof_prb, cell_id, sf, p, filt)
        got = ce[p, 0].reshape(14, -1)
        rms = np.sqrt(np.mean(np.abs(want) ** 2))
        assert np.abs(got - want).max() <= 2e-5 * rms, (p, np.abs(got - want).max() / rms)


def test_average_and_interpolate_share_noise():
    rng = np.random.default_rng(5)
    G = 14 * 12 * 25
    grids = (rng.standard_normal((2, G)) + 1j * rng.standard_normal((2, G))).astype(np.complex64)
    ce_a, ra = uc.chest_estimate(grids, 25, 2, 3, 4, alg=0)
    ce_i, ri = uc.chest_estimate(grids, 25, 2, 3, 4, alg=1)
    assert ra["noise_estimate"] == ri["noise_estimate"] and ra["rsrp"] == ri["rsrp"]
    rows = ce_a[0, 0].reshape(14, -1)
    assert all(np.array_equal(rows[0], rows[r]) for r in range(14))
    assert not np.array_equal(ce_i[0, 0].reshape(14, -1)[0], ce_i[0, 0].reshape(14, -1)[1])
