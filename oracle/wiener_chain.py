"""TEST INFRASTRUCTURE ONLY -- Python handle on oracle/orc_wiener.cpp (the Wiener DL estimator restatement) plus a
synthetic pilot generator for its tests, and a pure-Python restatement of libstdc++'s uniform_int_distribution
(Lemire's nearly divisionless method over a 32-bit generator, bits/uniform_int_dist.h) that the GPU kernel follows."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import lib
from .channel_chain import mt19937


def _declare():
    L = lib()
    if not getattr(L, "_wiener_declared", False):
        L.orc_wiener_new.restype = C.c_void_p
        L.orc_wiener_new.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_wiener_free.argtypes = [C.c_void_p]
        L.orc_wiener_subframe.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_uniform_int_draws.argtypes = [C.c_uint32, C.c_int, C.c_int, C.c_uint32, C.c_void_p]
        L._wiener_declared = True
    return L


class Wiener:
    """One srslte_wiener_dl_t (oracle/orc_wiener.cpp)."""

    def __init__(self, nof_prb: int, nof_ports: int, nof_rx: int):
        self.nof_prb, self.ntx, self.nrx = nof_prb, nof_ports, nof_rx
        self.h = _declare().orc_wiener_new(nof_prb, nof_ports, nof_rx)
        assert self.h

    def subframe(self, pilots: np.ndarray, snr: np.ndarray, shift):
        """pilots [rx][port][4][2 nof_prb] complex64, snr [rx][port] -> (ce [rx][port][14][12 nof_prb], ready, draws)."""
        p = np.ascontiguousarray(pilots, np.complex64)
        s = np.ascontiguousarray(snr, np.float32)
        sh = np.ascontiguousarray(shift, np.uint32)
        ce = np.zeros((self.nrx, self.ntx, 14, 12 * self.nof_prb), np.complex64)
        rd = np.zeros((self.nrx, self.ntx), np.int32)
        draws = _declare().orc_wiener_subframe(self.h, p.ctypes.data, s.ctypes.data, sh.ctypes.data, ce.ctypes.data,
                                               rd.ctypes.data)
        return ce, rd, draws

    def __del__(self):
        if getattr(self, "h", None):
            _declare().orc_wiener_free(self.h)
            self.h = None


def std_uniform_int(seed: int, lo: int, hi: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.int32)
    _declare().orc_uniform_int_draws(seed, lo, hi, n, out.ctypes.data)
    return out


def lemire_uniform_int(seed: int, lo: int, hi: int, n: int) -> list[int]:
    rng = iter(mt19937(seed, 4 * n + 16))
    rngr = (hi - lo + 1) & 0xFFFFFFFF
    out = []
    for _ in range(n):
        prod = next(rng) * rngr
        low = prod & 0xFFFFFFFF
        if low < rngr:
            thr = ((1 << 32) - rngr) % rngr
            while low < thr:
                prod = next(rng) * rngr
                low = prod & 0xFFFFFFFF
        out.append(lo + (prod >> 32))
    return out


def crs_shift(cell_id: int, port: int) -> int:
    """srslte_refsignal_cs_fidx(cell, 0, port, 0) (refsignal_dl.c): (v + cell_id % 6) % 6, v = 0 (port 0) / 3 (port 1)."""
    return ((0 if port == 0 else 3) + cell_id % 6) % 6


def synth_pilots(rng, nof_prb: int, ntx: int, nrx: int, nsf: int, snr_db: float, fd: float = 30.0, taps: int = 6,
                 cell_id: int = 1):
    """LS pilot estimates of nsf subframes of a multipath channel varying over time, at the CRS positions of ports 0/1
    (subcarrier 6 i + (v + cell_id % 6) % 6 of OFDM symbols 0, 4, 7, 11): pilots [sf][rx][port][4][2 nof_prb], snr_lin
    [sf][rx][port] (rsrp / noise / 2) and the true channel H [sf][rx][port][14][12 nof_prb]."""
    nref, nre = 2 * nof_prb, 12 * nof_prb
    delays = np.sort(rng.uniform(0, 1.5e-6, taps))
    pw = np.exp(-np.arange(taps) / 2.0)
    pw /= pw.sum()
    ph = rng.uniform(0, 2 * np.pi, (nrx, ntx, taps, 2))
    fk = (np.arange(nre) - nre // 2) * 15e3
    sigma = np.sqrt(10 ** (-snr_db / 10) / 2)
    sym = [0, 4, 7, 11]
    pil = np.zeros((nsf, nrx, ntx, 4, nref), np.complex64)
    H = np.zeros((nsf, nrx, ntx, 14, nre), np.complex64)
    for s in range(nsf):
        for r in range(nrx):
            for p in range(ntx):
                for l in range(14):
                    t = s * 1e-3 + l * (1e-3 / 14)
                    g = np.sqrt(pw) * np.exp(1j * (2 * np.pi * fd * t * np.cos(ph[r, p, :, 0]) + ph[r, p, :, 1]))
                    H[s, r, p, l] = (g[None, :] * np.exp(-2j * np.pi * fk[:, None] * delays[None, :])).sum(1)
                for li, l in enumerate(sym):
                    v = (0 if (li % 2 == 0) == (p == 0) else 3)
                    k = 6 * np.arange(nref) + (v + cell_id % 6) % 6
                    n = sigma * (rng.standard_normal(nref) + 1j * rng.standard_normal(nref))
                    pil[s, r, p, li] = H[s, r, p, l, k] + n
    snr = np.full((nsf, nrx, ntx), np.float32(1.0 / (2 * sigma ** 2) / 2), np.float32)
    return pil, snr, H
