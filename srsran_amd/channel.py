"""ctypes mirror of include/srsran_amd/channel.h -- the time-domain channel emulators (srslte_channel_fading_t,
srslte_channel_delay_t, srslte_channel_hst_t) batched over links on the GPU.  Buffers are host numpy complex64
arrays here (copied through device buffers); the C ABI itself works on device pointers."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import check, lib
from .tdec import DeviceBuffer


class Timestamp(C.Structure):
    _fields_ = [("full_secs", C.c_int64), ("frac_secs", C.c_double)]


def _declare():
    L = lib()
    if getattr(L, "_channel_declared", False):
        return L
    vp, u32, i32, f32, f64 = C.c_void_p, C.c_uint32, C.c_int, C.c_float, C.c_double
    L.mi355_channel_fading_create.argtypes = [C.POINTER(vp), i32, f64, C.c_char_p, C.POINTER(u32), u32, u32]
    L.mi355_channel_fading_fft_size.argtypes = [vp]
    L.mi355_channel_fading_fft_size.restype = u32
    L.mi355_channel_fading_execute.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), u32, C.POINTER(f64), C.POINTER(f64),
                                               vp]
    L.mi355_channel_fading_free.argtypes = [vp]
    L.mi355_channel_delay_create.argtypes = [C.POINTER(vp), i32, f32, f32, f32, f32, u32, u32, u32]
    L.mi355_channel_delay_update_srate.argtypes = [vp, u32]
    L.mi355_channel_delay_execute.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), u32, C.POINTER(Timestamp),
                                              C.POINTER(u32), vp]
    L.mi355_channel_delay_free.argtypes = [vp]
    L.mi355_channel_hst_execute_batch.argtypes = [i32, f32, f32, f32, u32, C.POINTER(vp), C.POINTER(vp), u32, u32,
                                                  C.POINTER(Timestamp), C.POINTER(f32), vp]
    L._channel_declared = True
    return L


class _Links:
    """Device input / output buffers for nlinks x n complex samples."""

    def __init__(self, nlinks: int, n: int):
        self.nlinks, self.n = nlinks, n
        self.din = [DeviceBuffer(max(8 * n, 8)) for _ in range(nlinks)]
        self.dout = [DeviceBuffer(max(8 * n, 8)) for _ in range(nlinks)]
        self.pin = (C.c_void_p * nlinks)(*[b.ptr for b in self.din])
        self.pout = (C.c_void_p * nlinks)(*[b.ptr for b in self.dout])

    def put(self, x: np.ndarray):
        for b, row in zip(self.din, np.asarray(x, np.complex64).reshape(self.nlinks, -1)):
            b.upload(np.ascontiguousarray(row))

    def get(self, n: int) -> np.ndarray:
        out = np.zeros((self.nlinks, n), np.complex64)
        for b, row in zip(self.dout, out):
            b.download(row)
        return out


class Fading:
    """nlinks srslte_channel_fading_t objects (fading.c): model, srate, seeds[i]; state carried across calls."""

    def __init__(self, srate: float, model: str, seeds, max_nsamples: int, device: int = 0):
        L = _declare()
        self.nlinks = len(seeds)
        self.h = C.c_void_p()
        s = (C.c_uint32 * self.nlinks)(*seeds)
        check(L.mi355_channel_fading_create(C.byref(self.h), device, srate, model.encode(), s, self.nlinks,
                                            max_nsamples), "mi355_channel_fading_create")
        self.N = L.mi355_channel_fading_fft_size(self.h)
        self.io = _Links(self.nlinks, max_nsamples)

    def execute(self, x: np.ndarray, init_time) -> tuple[np.ndarray, np.ndarray]:
        x = np.asarray(x, np.complex64).reshape(self.nlinks, -1)
        n = x.shape[1]
        self.io.put(x)
        t0 = (C.c_double * self.nlinks)(*np.broadcast_to(np.asarray(init_time, np.float64), (self.nlinks,)))
        t1 = (C.c_double * self.nlinks)()
        check(_declare().mi355_channel_fading_execute(self.h, self.io.pin, self.io.pout, n, t0, t1, None),
              "mi355_channel_fading_execute")
        return self.io.get(n), np.array(t1[:])

    def close(self):
        if self.h:
            _declare().mi355_channel_fading_free(self.h)
            self.h = C.c_void_p()


class Delay:
    """nlinks srslte_channel_delay_t objects with one profile (delay.c)."""

    def __init__(self, delay_min_us, delay_max_us, period_s, init_time_s, srate_hz, nlinks, max_len, device=0):
        L = _declare()
        self.nlinks = nlinks
        self.h = C.c_void_p()
        check(L.mi355_channel_delay_create(C.byref(self.h), device, delay_min_us, delay_max_us, period_s, init_time_s,
                                           srate_hz, nlinks, max_len), "mi355_channel_delay_create")
        self.io = _Links(nlinks, max_len)

    def update_srate(self, srate_hz: int):
        check(_declare().mi355_channel_delay_update_srate(self.h, srate_hz), "mi355_channel_delay_update_srate")

    def execute(self, x: np.ndarray, ts) -> tuple[np.ndarray, np.ndarray]:
        x = np.asarray(x, np.complex64).reshape(self.nlinks, -1)
        self.io.put(x)
        tsa = (Timestamp * self.nlinks)(*[Timestamp(int(f), float(r)) for f, r in ts])
        d = (C.c_uint32 * self.nlinks)()
        check(_declare().mi355_channel_delay_execute(self.h, self.io.pin, self.io.pout, x.shape[1], tsa, d, None),
              "mi355_channel_delay_execute")
        return self.io.get(x.shape[1]), np.array(d[:])

    def close(self):
        if self.h:
            _declare().mi355_channel_delay_free(self.h)
            self.h = C.c_void_p()


def hst_execute(x: np.ndarray, fd_hz, period_s, init_time_s, srate_hz, ts, device=0):
    """srslte_channel_hst_execute on every row of x (links) at timestamps ts[i] = (full_secs, frac_secs)."""
    x = np.asarray(x, np.complex64)
    nl, n = x.shape
    io = _Links(nl, n)
    io.put(x)
    tsa = (Timestamp * nl)(*[Timestamp(int(f), float(r)) for f, r in ts])
    fs = (C.c_float * nl)()
    check(_declare().mi355_channel_hst_execute_batch(device, fd_hz, period_s, init_time_s, srate_hz, io.pin, io.pout,
                                                     n, nl, tsa, fs, None), "mi355_channel_hst_execute_batch")
    return io.get(n), np.array(fs[:])
