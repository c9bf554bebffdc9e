"""Python mirror of include/srsran_amd/srslte_tdec.h -- the srslte_tdec_* drop-in.

The class reads like the reference's own test (lib/src/phy/fec/test/turbodecoder_test.c:188-260):
init / init_manual, force_not_sb, new_cb, iteration, run_all, free."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import lib

SRSLTE_TDEC_AUTO = 0
SRSLTE_TDEC_GENERIC = 1


class _Tdec(C.Structure):
    _fields_ = [("max_long_cb", C.c_uint32), ("dec_type", C.c_int), ("force_not_sb", C.c_bool),
                ("current_long_cb", C.c_uint32), ("current_cbidx", C.c_int), ("n_iter", C.c_int),
                ("impl", C.c_void_p)]


def _declare():
    L = lib()
    if getattr(L, "_srslte_declared", False):
        return L
    P = C.POINTER(_Tdec)
    L.mi355_srslte_tdec_init.argtypes = [P, C.c_uint32]
    L.mi355_srslte_tdec_init_manual.argtypes = [P, C.c_uint32, C.c_int]
    L.mi355_srslte_tdec_free.argtypes = [P]
    L.mi355_srslte_tdec_force_not_sb.argtypes = [P]
    L.mi355_srslte_tdec_new_cb.argtypes = [P, C.c_uint32]
    L.mi355_srslte_tdec_get_nof_iterations.argtypes = [P]
    L.mi355_srslte_tdec_autoimp_get_subblocks.restype = C.c_uint32
    L.mi355_srslte_tdec_autoimp_get_subblocks.argtypes = [C.c_uint32]
    L.mi355_srslte_tdec_autoimp_get_subblocks_8bit.restype = C.c_uint32
    L.mi355_srslte_tdec_autoimp_get_subblocks_8bit.argtypes = [C.c_uint32]
    L.mi355_srslte_tdec_iteration.argtypes = [P, C.c_void_p, C.c_void_p]
    L.mi355_srslte_tdec_run_all.argtypes = [P, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]
    L.mi355_srslte_tdec_iteration_8bit.argtypes = [P, C.c_void_p, C.c_void_p]
    L.mi355_srslte_tdec_run_all_8bit.argtypes = [P, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32]
    L._srslte_declared = True
    return L


class SrslteTdec:
    def __init__(self, max_long_cb: int = 6144, dec_type: int | None = None):
        self.L = _declare()
        self.h = _Tdec()
        if dec_type is None:
            rc = self.L.mi355_srslte_tdec_init(C.byref(self.h), max_long_cb)
        else:
            rc = self.L.mi355_srslte_tdec_init_manual(C.byref(self.h), max_long_cb, dec_type)
        if rc != 0:
            raise RuntimeError(f"srslte_tdec_init failed ({rc})")

    def force_not_sb(self):
        self.L.mi355_srslte_tdec_force_not_sb(C.byref(self.h))

    def new_cb(self, K: int) -> int:
        return self.L.mi355_srslte_tdec_new_cb(C.byref(self.h), K)

    def iteration(self, buf: np.ndarray) -> np.ndarray:
        buf = np.ascontiguousarray(buf, np.int16)
        out = np.zeros(self.h.current_long_cb // 8, np.uint8)
        self.L.mi355_srslte_tdec_iteration(C.byref(self.h), buf.ctypes.data, out.ctypes.data)
        return out

    def run_all(self, buf: np.ndarray, nof_iterations: int, K: int) -> np.ndarray:
        buf = np.ascontiguousarray(buf, np.int16)
        out = np.zeros(K // 8, np.uint8)
        rc = self.L.mi355_srslte_tdec_run_all(C.byref(self.h), buf.ctypes.data, out.ctypes.data, nof_iterations, K)
        if rc != 0:
            raise RuntimeError(f"srslte_tdec_run_all failed ({rc})")
        return out

    def iteration_8bit(self, buf: np.ndarray) -> np.ndarray:
        """srslte_tdec_iteration_8bit; buf (int8, the 8-bit decoder layout) receives the tails as in the reference."""
        assert buf.dtype == np.int8 and buf.flags.c_contiguous
        out = np.zeros(self.h.current_long_cb // 8, np.uint8)
        self.L.mi355_srslte_tdec_iteration_8bit(C.byref(self.h), buf.ctypes.data, out.ctypes.data)
        return out

    def run_all_8bit(self, buf: np.ndarray, nof_iterations: int, K: int) -> np.ndarray:
        assert buf.dtype == np.int8 and buf.flags.c_contiguous
        out = np.zeros(K // 8, np.uint8)
        rc = self.L.mi355_srslte_tdec_run_all_8bit(C.byref(self.h), buf.ctypes.data, out.ctypes.data, nof_iterations, K)
        if rc != 0:
            raise RuntimeError(f"srslte_tdec_run_all_8bit failed ({rc})")
        return out

    @property
    def n_iter(self) -> int:
        return self.L.mi355_srslte_tdec_get_nof_iterations(C.byref(self.h))

    def free(self):
        if self.h.impl:
            self.L.mi355_srslte_tdec_free(C.byref(self.h))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
