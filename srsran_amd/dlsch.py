"""Python mirror of include/srsran_amd/dlsch.h -- batched DL-SCH transport-block decode
(srslte_dlsch_decode2, lib/src/phy/phch/sch.c:572-606) with device HARQ softbuffers."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import check, lib
from .tdec import DeviceBuffer


class TbDesc(C.Structure):
    _fields_ = [("tbs", C.c_uint32), ("nof_e_bits", C.c_uint32), ("Qm", C.c_uint32), ("rv", C.c_uint32),
                ("softbuffer", C.c_uint32), ("e_offset", C.c_uint64), ("data_offset", C.c_uint64)]


def _declare():
    L = lib()
    if getattr(L, "_dlsch_declared", False):
        return L
    vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int
    L.mi355_softbuffer_pool_create.argtypes = [C.POINTER(vp), u32, u32, i32]
    L.mi355_softbuffer_pool_destroy.argtypes = [vp]
    L.mi355_softbuffer_reset.argtypes = [vp, u32, vp]
    L.mi355_softbuffer_reset_tbs.argtypes = [vp, u32, u32, vp]
    L.mi355_softbuffer_reset_cb.argtypes = [vp, u32, u32, vp]
    L.mi355_softbuffer_reset_all.argtypes = [vp, vp]
    L.mi355_softbuffer_pool_materialize.argtypes = [vp, u32, u32, vp]
    L.mi355_dlsch_create.argtypes = [C.POINTER(vp), i32]
    L.mi355_dlsch_destroy.argtypes = [vp]
    L.mi355_dlsch_set_max_iterations.argtypes = [vp, u32]
    L.mi355_dlsch_decode_dev.argtypes = [vp, vp, vp, C.POINTER(TbDesc), u32, vp, C.POINTER(C.c_int32),
                                         C.POINTER(C.c_float), vp]
    L.mi355_dlsch_decode8_dev.argtypes = [vp, vp, vp, C.POINTER(TbDesc), u32, vp, C.POINTER(C.c_int32),
                                         C.POINTER(C.c_float), vp]
    L._dlsch_declared = True
    return L


class SoftbufferPool:
    def __init__(self, nof_sb: int, max_cb: int = 32, device: int = 0):
        self.L = _declare()
        h = C.c_void_p()
        check(self.L.mi355_softbuffer_pool_create(C.byref(h), nof_sb, max_cb, device), "softbuffer_pool_create")
        self.h, self.nof_sb, self.max_cb = h, nof_sb, max_cb

    def reset(self, sb: int):
        check(self.L.mi355_softbuffer_reset(self.h, sb, None), "softbuffer_reset")
        lib().mi355_device_sync()

    def reset_all(self):
        check(self.L.mi355_softbuffer_reset_all(self.h, None), "softbuffer_reset_all")
        lib().mi355_device_sync()

    def materialize(self, first: int = 0, n: int | None = None):
        """Zero the unwritten (logically zero) parity rows of softbuffers [first, first + n) so their memory reads as
        the reference's buffers would (mi355_softbuffer_pool_materialize); before raw reads of buffer memory."""
        lib().mi355_device_sync()
        n = self.nof_sb - first if n is None else n
        check(self.L.mi355_softbuffer_pool_materialize(self.h, first, n, None), "softbuffer_pool_materialize")
        lib().mi355_device_sync()

    def close(self):
        if getattr(self, "h", None):
            self.L.mi355_softbuffer_pool_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Dlsch:
    def __init__(self, device: int = 0, max_iterations: int = 10):
        self.L = _declare()
        h = C.c_void_p()
        check(self.L.mi355_dlsch_create(C.byref(h), device), "dlsch_create")
        self.h, self.device = h, device
        check(self.L.mi355_dlsch_set_max_iterations(self.h, max_iterations), "set_max_iterations")

    def set_max_iterations(self, n: int):
        check(self.L.mi355_dlsch_set_max_iterations(self.h, n), "set_max_iterations")

    def decode(self, pool: SoftbufferPool, tbs: list[dict], e_bits: list[np.ndarray], llr8: bool = False):
        """tbs[i] = dict(tbs, Qm, rv, softbuffer); e_bits[i] = int16 LLRs of TB i (int8 with llr8: the
        pdsch_8bit_decoder mode, mi355_dlsch_decode8_dev).  Returns (ret[i], data[i] bytes (tbs/8 + 6),
        avg_iterations[i])."""
        n = len(tbs)
        dt = np.int8 if llr8 else np.int16
        offs = np.cumsum([0] + [e.size for e in e_bits])
        allE = np.concatenate([np.ascontiguousarray(e, dt) for e in e_bits]) if n else np.zeros(1, dt)
        doff = np.cumsum([0] + [t["tbs"] // 8 + 8 for t in tbs])
        d_e = DeviceBuffer(max(allE.nbytes, 2), self.device).upload(allE)
        d_data = DeviceBuffer(max(int(doff[-1]), 1), self.device)
        lib().mi355_memset_dev(d_data.ptr, 0, int(doff[-1]))
        desc = (TbDesc * n)()
        for i, t in enumerate(tbs):
            desc[i] = TbDesc(t["tbs"], int(e_bits[i].size), t["Qm"], t.get("rv", 0), t.get("softbuffer", i),
                             int(offs[i]), int(doff[i]))
        ret = (C.c_int32 * n)()
        its = (C.c_float * n)()
        fn = self.L.mi355_dlsch_decode8_dev if llr8 else self.L.mi355_dlsch_decode_dev
        check(fn(self.h, pool.h, d_e.ptr, desc, n, d_data.ptr, ret, its, None), "dlsch_decode_dev")
        host = np.zeros(int(doff[-1]), np.uint8)
        d_data.download(host)
        datas = [host[doff[i]: doff[i] + tbs[i]["tbs"] // 8 + 6].copy() for i in range(n)]
        return [int(r) for r in ret], datas, [float(v) for v in its]

    def close(self):
        if getattr(self, "h", None):
            self.L.mi355_dlsch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
