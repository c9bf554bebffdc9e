"""Test helper (not product code): a numpy restatement of the 8-bit LLR front end of srslte_pdsch_decode with
llr_is_8bit -- srslte_demod_soft_demodulate_b (demod_soft.c:100-941, SSE/AVX2 build), srslte_scrambling_sb_offset
(scrambling.c:49-53) and the float CSI loop (pdsch.c:661-668) -- pinned to the reference's own outputs by
tests/golden/tdec8.npz (test_oracle_golden.py) and used as the checker of the GPU's int8 LLR kernel."""
from __future__ import annotations

import numpy as np

F = np.float32


def wrap8(v) -> np.ndarray:
    return ((np.asarray(v, np.int64) + 128) % 256) - 128


def sat8(v) -> np.ndarray:
    return np.clip(np.asarray(v, np.int64), -128, 127)


def abs8(v) -> np.ndarray:  # _mm_abs_epi8: |-128| = -128
    v = np.asarray(v, np.int64)
    return np.where(v == -128, -128, np.abs(v))


def trunc(x) -> np.ndarray:
    return np.trunc(x).astype(np.int64)


def demod_b(sym: np.ndarray, qm: int) -> np.ndarray:
    sym = np.asarray(sym, np.complex64)
    n = sym.size
    re, im = sym.real.astype(F), sym.imag.astype(F)
    body = np.arange(n) < n // 8 * 8
    out = np.zeros((n, qm), np.int64)
    if qm == 2:  # srslte_vec_convert_fb: truncation, saturating packs (SIMD body) / wrap (scalar tail)
        s = F(-20 * np.sqrt(2.0))
        for k, x in enumerate((re, im)):
            t = trunc(x * s)
            out[:, k] = np.where(body, sat8(t), wrap8(t))
    elif qm == 4:
        kq = F(60) / np.sqrt(F(10))
        for k, x in enumerate((re, im)):
            sb = sat8(np.rint(x * F(-30.0)))
            y = wrap8(trunc(F(30.0) * x))
            out[:, k] = np.where(body, sb, wrap8(-y))
            out[:, 2 + k] = np.where(body, wrap8(abs8(sb) - 18), wrap8(trunc(np.abs(y).astype(F) - kq)))
    elif qm == 6:
        for k, x in enumerate((re, im)):
            sb = sat8(np.rint(x * F(-40.0)))
            a1 = wrap8(abs8(sb) - 24)
            y = wrap8(trunc(F(40.0) * x))
            t1 = wrap8(wrap8(np.abs(y)) - 24)
            out[:, k] = np.where(body, sb, wrap8(-y))
            out[:, 2 + k] = np.where(body, a1, t1)
            out[:, 4 + k] = np.where(body, wrap8(abs8(a1) - 12), wrap8(wrap8(np.abs(t1)) - 12))
    elif qm == 8:
        ks = [F(c) / np.sqrt(F(170.0)) for c in (8.0, 4.0, 2.0)]
        for k, x in enumerate((re, im)):
            r = -x
            for j in range(4):
                out[:, 2 * j + k] = wrap8(trunc(F(50.0) * r))
                if j < 3:
                    r = (np.abs(r) - ks[j]).astype(F)
    else:
        raise ValueError(qm)
    return out.reshape(-1).astype(np.int8)


def scramble_sb(llr: np.ndarray, c: np.ndarray) -> np.ndarray:
    v = np.asarray(llr, np.int64)
    return np.where(np.asarray(c, bool), wrap8(-v), v).astype(np.int8)


def csi_b(llr: np.ndarray, csi: np.ndarray, qm: int) -> np.ndarray:
    n = csi.size
    cmax = F(np.max(csi[:n]))
    c = (csi.astype(F) / cmax).astype(F)
    v = np.asarray(llr, np.int64).reshape(n, qm).astype(F) * c[:, None]
    return wrap8(trunc(v.astype(F))).reshape(-1).astype(np.int8)
