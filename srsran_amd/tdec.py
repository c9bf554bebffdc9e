"""Python mirror of include/srsran_amd/tdec.h (batched turbo decoder C ABI).

Mirrors the reference's srslte_tdec_run_all semantics (lib/src/phy/fec/turbodecoder.c:537-550):
``nhalf`` is the srslte "iteration" count (one constituent MAP per count), inputs are decoder buffers in
the layout srslte_rm_turbo_rx_lut produces, outputs are K/8 decision bytes.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import check, lib


def tdec_buf_len(K: int) -> int:
    """Decoder input buffer length in int16 (softbuffer.h:50 uses 3*(K+32)+12 for the SB layout)."""
    return 3 * (K + 32) + 12


class DeviceBuffer:
    """A raw hipMalloc'ed buffer owned by the C ABI (no torch needed)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.nbytes = int(nbytes)
        self.ptr = lib().mi355_dev_alloc(self.nbytes, device)
        if not self.ptr:
            raise MemoryError(f"mi355_dev_alloc({nbytes}) failed")

    def upload(self, arr: np.ndarray) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        check(lib().mi355_memcpy_h2d(self.ptr, arr.ctypes.data, arr.nbytes), "mi355_memcpy_h2d")
        return self

    def download(self, arr: np.ndarray) -> np.ndarray:
        assert arr.flags.c_contiguous and arr.nbytes <= self.nbytes
        check(lib().mi355_memcpy_d2h(arr.ctypes.data, self.ptr, arr.nbytes), "mi355_memcpy_d2h")
        return arr

    def free(self) -> None:
        if getattr(self, "ptr", None):
            lib().mi355_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class TdecBatch:
    """Batched GPU turbo decoder bound to one HIP device."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().mi355_tdec_batch_create(C.byref(h), device), "mi355_tdec_batch_create")
        self.h = h
        self.device = device

    @staticmethod
    def subblocks(K: int) -> int:
        return int(lib().mi355_tdec_autoimp_get_subblocks(K))

    def run(self, bufs: np.ndarray, K: int, nhalf: int) -> np.ndarray:
        """Host arrays in/out: bufs is (n, stride) int16, returns (n, K/8) uint8."""
        bufs = np.ascontiguousarray(bufs, np.int16)
        n, stride = bufs.shape
        out = np.zeros((n, K // 8), np.uint8)
        check(lib().mi355_tdec_batch_run(self.h, bufs.ctypes.data, stride, n, K, nhalf,
                                         out.ctypes.data, K // 8), "mi355_tdec_batch_run")
        return out

    def run_dev(self, d_in: int, in_stride: int, n: int, K: int, nhalf: int, d_out: int,
                out_stride: int | None = None, stream: int | None = None) -> None:
        """Device pointers in/out (ints), asynchronous on `stream` (hipStream_t as int, None = own)."""
        check(lib().mi355_tdec_batch_run_dev(self.h, d_in, in_stride, n, K, nhalf, d_out,
                                             out_stride or K // 8, stream), "mi355_tdec_batch_run_dev")

    def set_impl(self, impl: int) -> None:
        """0 = AUTO (by K, as the AVX2 build), 1 = GENERIC on the linear layout for every K."""
        check(lib().mi355_tdec_batch_set_impl(self.h, impl), "mi355_tdec_batch_set_impl")

    def set_generic(self, per_cb: int = -1, warmup: int = 32) -> None:
        """Generic decoder schedule: per_cb 1 = workgroup per code block (chunked, verified), 0 = two blocks per
        lane (serial), -1 = auto; warmup = the chunks' guess warm-up (0: every chunk but the first reruns)."""
        check(lib().mi355_tdec_batch_set_generic(self.h, per_cb, warmup), "mi355_tdec_batch_set_generic")

    def generic_reruns(self) -> int:
        """Chunk reruns of the per-code-block generic decoder since the last call (first call arms, returns 0)."""
        r = C.c_uint32()
        check(lib().mi355_tdec_batch_generic_reruns(self.h, C.byref(r)), "generic_reruns")
        return int(r.value)

    def set_profiling(self, on: bool) -> None:
        lib().mi355_tdec_batch_set_profiling(self.h, 1 if on else 0)

    def kernel_stats(self) -> tuple[float, int]:
        ms, cnt = C.c_double(), C.c_uint32()
        check(lib().mi355_tdec_batch_kernel_stats(self.h, C.byref(ms), C.byref(cnt)), "kernel_stats")
        return ms.value, cnt.value

    def close(self) -> None:
        if getattr(self, "h", None):
            lib().mi355_tdec_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Tdec8Batch:
    """The 8-bit turbo decoder and 8-bit rate dematching on one device (include/srsran_amd/tdec.h mi355_tdec8_*)."""

    def __init__(self, device: int = 0):
        L = lib()
        if not getattr(L, "_tdec8_declared", False):
            vp, u32, sz = C.c_void_p, C.c_uint32, C.c_size_t
            L.mi355_tdec8_create.argtypes = [C.POINTER(vp), C.c_int]
            L.mi355_tdec8_destroy.argtypes = [vp]
            L.mi355_tdec_autoimp_get_subblocks_8bit.restype = u32
            L.mi355_tdec_autoimp_get_subblocks_8bit.argtypes = [u32]
            L.mi355_tdec8_run_dev.argtypes = [vp, vp, sz, u32, u32, u32, vp, sz, vp, vp]
            L.mi355_rm_turbo_rx_8bit_dev.argtypes = [vp, vp, sz, u32, vp, sz, u32, u32, u32, vp]
            L._tdec8_declared = True
        h = C.c_void_p()
        check(L.mi355_tdec8_create(C.byref(h), device), "mi355_tdec8_create")
        self.L, self.h = L, h

    def run_dev(self, d_in: int, in_stride: int, ncb: int, K: int, nhalf: int, d_out: int, out_stride: int,
                d_trace: int | None = None) -> int:
        return self.L.mi355_tdec8_run_dev(self.h, d_in, in_stride, ncb, K, nhalf, d_out, out_stride, d_trace, None)

    def rm_rx_dev(self, d_e: int, e_stride: int, E: int, d_out: int, out_stride: int, ncb: int, K: int, rv: int) -> int:
        return self.L.mi355_rm_turbo_rx_8bit_dev(self.h, d_e, e_stride, E, d_out, out_stride, ncb, K, rv, None)

    def close(self):
        if getattr(self, "h", None):
            self.L.mi355_tdec8_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
