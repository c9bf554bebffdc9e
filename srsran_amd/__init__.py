"""srsran_amd -- MI355X-native (gfx950) srsLTE PDSCH receive hot path.

The product is the C-ABI shared library ``srsran_amd/lib/libsrsran_amd.so`` (HIP kernels + host
runtime, declared in ``include/srsran_amd/*.h``).  This Python package is a thin ctypes mirror of
that ABI used by the tests and bench; it never falls back to a CPU path: if the library is missing
every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# MI355_LIB: an alternative in-tree build of the same library (A/B timing of kernel variants on one box)
LIB_PATH = os.environ.get("MI355_LIB") or os.path.join(HERE, "lib", "libsrsran_amd.so")
_LIB: C.CDLL | None = None


class NativeLibraryMissing(RuntimeError):
    pass


def build(jobs: int = 8) -> str:
    """Compile the HIP library for gfx950 in-tree (cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", "-C", HERE, f"-j{jobs}"], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not built: run `make -C srsran_amd` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        _declare(L)
        _LIB = L
    return _LIB


def _declare(L: C.CDLL) -> None:
    vp, u32, i32, sz = C.c_void_p, C.c_uint32, C.c_int, C.c_size_t
    L.mi355_tdec_batch_create.argtypes = [C.POINTER(vp), i32]
    L.mi355_tdec_batch_destroy.argtypes = [vp]
    L.mi355_tdec_batch_run_dev.argtypes = [vp, vp, sz, u32, u32, u32, vp, sz, vp]
    L.mi355_tdec_batch_run.argtypes = [vp, vp, sz, u32, u32, u32, vp, sz]
    L.mi355_tdec_batch_halfit_dev.argtypes = [vp, vp, sz, u32, u32, u32, vp, sz, vp]
    L.mi355_tdec_batch_set_impl.argtypes = [vp, i32]
    L.mi355_tdec_batch_set_generic.argtypes = [vp, i32, i32]
    L.mi355_dlsch_set_latency_path.argtypes = [i32]
    L.mi355_dlsch_latency_profile.argtypes = [i32, vp]
    L.mi355_tdec_batch_generic_reruns.argtypes = [vp, C.POINTER(u32)]
    L.mi355_tdec_batch_set_profiling.argtypes = [vp, i32]
    L.mi355_tdec_batch_kernel_stats.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(u32)]
    L.mi355_tdec_set_diag.argtypes = [i32]
    L.mi355_tdec_autoimp_get_subblocks.restype = u32
    L.mi355_tdec_autoimp_get_subblocks.argtypes = [u32]
    L.mi355_dev_alloc.restype = vp
    L.mi355_dev_alloc.argtypes = [sz, i32]
    L.mi355_dev_free.argtypes = [vp]
    L.mi355_memcpy_h2d.argtypes = [vp, vp, sz]
    L.mi355_memcpy_d2h.argtypes = [vp, vp, sz]
    L.mi355_memset_dev.argtypes = [vp, i32, sz]
    L.mi355_device_count.restype = i32


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with srslte error code {rc}")


from .tdec import DeviceBuffer, TdecBatch, tdec_buf_len  # noqa: E402,F401
