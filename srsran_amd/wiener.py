"""ctypes mirror of include/srsran_amd/wiener.h -- the Wiener DL estimator (srslte_wiener_dl_t) for many links."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import check, lib
from .tdec import DeviceBuffer


def _declare():
    L = lib()
    if getattr(L, "_wiener_declared", False):
        return L
    vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int
    L.mi355_wiener_dl_create.argtypes = [C.POINTER(vp), i32, u32, u32, u32, u32]
    L.mi355_wiener_dl_free.argtypes = [vp]
    L.mi355_wiener_dl_reset.argtypes = [vp, u32]
    L.mi355_wiener_dl_run_batch.argtypes = [vp, C.POINTER(u32), u32, vp, C.POINTER(C.c_float), C.POINTER(u32), vp,
                                            C.POINTER(C.c_int32), vp]
    L._wiener_declared = True
    return L


class WienerDl:
    def __init__(self, nof_prb: int, nof_ports: int, nof_rx: int, nlinks: int, device: int = 0):
        self.nof_prb, self.ntx, self.nrx, self.nlinks = nof_prb, nof_ports, nof_rx, nlinks
        self.h = C.c_void_p()
        check(_declare().mi355_wiener_dl_create(C.byref(self.h), device, nof_prb, nof_ports, nof_rx, nlinks),
              "mi355_wiener_dl_create")

    def run(self, links, pilots: np.ndarray, snr: np.ndarray, shift):
        """pilots [job][rx][port][4][2 nof_prb] complex64, snr [job][rx][port] -> (ce [job][rx][port][14][12 nof_prb],
        ready [job][rx][port], draws of the first job's link)."""
        n = len(links)
        pil = np.ascontiguousarray(pilots, np.complex64)
        ce = np.zeros((n, self.nrx, self.ntx, 14, 12 * self.nof_prb), np.complex64)
        dp = DeviceBuffer(max(pil.nbytes, 8)).upload(pil)
        dc = DeviceBuffer(max(ce.nbytes, 8))
        ready = np.zeros((n, self.nrx, self.ntx), np.int32)
        s = np.ascontiguousarray(snr, np.float32)
        r = _declare().mi355_wiener_dl_run_batch(
            self.h, (C.c_uint32 * n)(*links), n, dp.ptr, s.ctypes.data_as(C.POINTER(C.c_float)),
            (C.c_uint32 * len(shift))(*shift), dc.ptr, ready.ctypes.data_as(C.POINTER(C.c_int32)), None)
        if r < 0:
            raise RuntimeError(f"mi355_wiener_dl_run_batch failed with {r}")
        dc.download(ce)
        dp.free()
        dc.free()
        return ce, ready, r

    def reset(self, link: int):
        check(_declare().mi355_wiener_dl_reset(self.h, link), "mi355_wiener_dl_reset")

    def close(self):
        if self.h:
            _declare().mi355_wiener_dl_free(self.h)
            self.h = C.c_void_p()
