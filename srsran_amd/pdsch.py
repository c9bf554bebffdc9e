"""Python mirror of include/srsran_amd/pdsch.h -- batched srslte_pdsch_decode (lib/src/phy/phch/pdsch.c:907-1072).

The ctypes structures carry the reference's field names (srslte_cell_t, srslte_dl_sf_cfg_t, srslte_ra_tb_t,
srslte_pdsch_grant_t, srslte_pdsch_cfg_t, srslte_pdsch_res_t) so test code reads like the reference's
pdsch_test.c.  Sample buffers are device pointers (DeviceBuffer.ptr).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import check, lib
from .dlsch import SoftbufferPool, _declare as _declare_dlsch

MAX_PRB = 110
TXSCHEME_PORT0, TXSCHEME_DIVERSITY, TXSCHEME_SPATIALMUX, TXSCHEME_CDD = range(4)
MOD_BPSK, MOD_QPSK, MOD_16QAM, MOD_64QAM, MOD_256QAM = range(5)
MOD_BITS = {MOD_BPSK: 1, MOD_QPSK: 2, MOD_16QAM: 4, MOD_64QAM: 6, MOD_256QAM: 8}
QM_TO_MOD = {v: k for k, v in MOD_BITS.items()}
MIMO_DECODER_ZF, MIMO_DECODER_MMSE = 0, 1


class Cell(C.Structure):
    _fields_ = [("nof_prb", C.c_uint32), ("nof_ports", C.c_uint32), ("id", C.c_uint32), ("cp", C.c_uint32),
                ("frame_type", C.c_uint32), ("phich_length", C.c_uint32), ("phich_resources", C.c_uint32)]


class DlSfCfg(C.Structure):
    _fields_ = [("tti", C.c_uint32), ("cfi", C.c_uint32)]


class RaTb(C.Structure):
    _fields_ = [("enabled", C.c_uint32), ("mod", C.c_uint32), ("tbs", C.c_int32), ("rv", C.c_uint32),
                ("nof_bits", C.c_uint32), ("cw_idx", C.c_uint32)]


class PdschGrant(C.Structure):
    _fields_ = [("tx_scheme", C.c_uint32), ("pmi", C.c_uint32), ("prb_idx", (C.c_uint8 * MAX_PRB) * 2),
                ("nof_prb", C.c_uint32), ("nof_re", C.c_uint32), ("nof_symb_slot", C.c_uint32 * 2),
                ("tb", RaTb * 2), ("nof_tb", C.c_uint32), ("nof_layers", C.c_uint32)]


class PdschCfg(C.Structure):
    _fields_ = [("grant", PdschGrant), ("rnti", C.c_uint16), ("max_nof_iterations", C.c_uint32),
                ("decoder_type", C.c_uint32), ("p_a", C.c_float), ("p_b", C.c_uint32), ("power_scale", C.c_uint32),
                ("csi_enable", C.c_uint32), ("softbuffer", C.c_uint32 * 2)]


class PdschJob(C.Structure):
    _fields_ = [("sf", DlSfCfg), ("cfg", PdschCfg), ("noise_estimate", C.c_float),
                ("sf_symbols", C.c_void_p * 2), ("ce", (C.c_void_p * 2) * 4), ("payload", C.c_void_p * 2)]


class PdschRes(C.Structure):
    _fields_ = [("crc", C.c_int32), ("avg_iterations_block", C.c_float), ("ret", C.c_int32)]


def _declare():
    L = _declare_dlsch()
    if getattr(L, "_pdsch_declared", False):
        return L
    vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int
    L.mi355_pdsch_create.argtypes = [C.POINTER(vp), C.POINTER(Cell), u32, i32]
    L.mi355_pdsch_destroy.argtypes = [vp]
    L.mi355_pdsch_decode_batch.argtypes = [vp, vp, C.POINTER(PdschJob), u32, C.POINTER(PdschRes), vp]
    L.mi355_pdsch_frontend.argtypes = [vp, C.POINTER(PdschJob), u32, vp]
    L.mi355_pdsch_debug_stage.argtypes = [vp, u32, u32, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)]
    L.mi355_pdsch_set_llr_8bit.argtypes = [vp, C.c_int]
    L.mi355_pdsch_set_ce_invariant.argtypes = [vp, C.c_int]
    L.mi355_pdsch_re_map.restype = u32
    L.mi355_pdsch_re_map.argtypes = [C.POINTER(Cell), C.POINTER(PdschGrant), u32, u32, C.c_void_p]
    L._pdsch_declared = True
    return L


def make_cell(nof_prb: int, nof_ports: int = 1, cell_id: int = 0, cp: int = 0, frame_type: int = 0,
              phich_length: int = 0, phich_resources: int = 0) -> Cell:
    """srslte_cell_t; phich_resources 0 R1/6, 1 R1/2, 2 R1, 3 R2 (only the control-channel REG map reads it)."""
    return Cell(nof_prb, nof_ports, cell_id, cp, frame_type, phich_length, phich_resources)


def re_map(cell: Cell, grant: PdschGrant, cfi: int, sf_idx: int) -> np.ndarray:
    """Host-only: grid indices of the grant's PDSCH REs in srslte_pdsch_get order."""
    L = _declare()
    idx = np.zeros(14 * 12 * cell.nof_prb, np.uint32)
    n = L.mi355_pdsch_re_map(C.byref(cell), C.byref(grant), cfi, sf_idx, idx.ctypes.data)
    return idx[:n].copy()


def make_grant(cell: Cell, prb: np.ndarray, cfi: int, sf_idx: int, tx_scheme: int, nof_layers: int,
               tbs: list[dict], pmi: int = 0) -> PdschGrant:
    """prb: (2, nof_prb) flags.  tbs: per enabled TB dict(mod|qm, tbs, rv, cw_idx).  nof_re / nof_bits filled
    as srslte_ra_dl_grant_to_grant_prb_allocation + ra_dl.c:442 do."""
    g = PdschGrant()
    g.tx_scheme, g.pmi, g.nof_layers = tx_scheme, pmi, nof_layers
    prb = np.asarray(prb, np.uint8).reshape(2, cell.nof_prb)
    for s in range(2):
        for n in range(cell.nof_prb):
            g.prb_idx[s][n] = int(prb[s, n])
    g.nof_prb = int(prb[0].sum())
    nsymb = 6 if cell.cp else 7
    g.nof_symb_slot[0] = g.nof_symb_slot[1] = nsymb
    g.nof_re = int(re_map(cell, g, cfi, sf_idx).size)
    g.nof_tb = 0
    for i, t in enumerate(tbs[:2]):
        if t is None:
            continue
        mod = t["mod"] if "mod" in t else QM_TO_MOD[t["qm"]]
        g.tb[i] = RaTb(1, mod, int(t["tbs"]), int(t.get("rv", 0)), g.nof_re * MOD_BITS[mod], int(t.get("cw_idx", i)))
        g.nof_tb += 1
    return g


class Pdsch:
    """srslte_pdsch_t (UE side) on one MI355X: mi355_pdsch_create / decode_batch."""

    def __init__(self, cell: Cell, nof_rx_antennas: int = 1, device: int = 0):
        self.L = _declare()
        h = C.c_void_p()
        check(self.L.mi355_pdsch_create(C.byref(h), C.byref(cell), nof_rx_antennas, device), "pdsch_create")
        self.h, self.cell, self.nrx, self.device = h, cell, nof_rx_antennas, device

    def decode(self, pool: SoftbufferPool, jobs: list[PdschJob], res: np.ndarray | None = None):
        """Returns a (njobs, 2) array of PdschRes (crc in/out)."""
        n = len(jobs)
        arr = (PdschJob * n)(*jobs)
        out = (PdschRes * (2 * n))()
        if res is not None:
            for i in range(2 * n):
                out[i] = res[i]
        check(self.L.mi355_pdsch_decode_batch(self.h, pool.h, arr, n, out, None), "pdsch_decode_batch")
        return out

    def frontend(self, jobs: list[PdschJob]):
        n = len(jobs)
        arr = (PdschJob * n)(*jobs)
        check(self.L.mi355_pdsch_frontend(self.h, arr, n, None), "pdsch_frontend")

    def set_llr_8bit(self, enable: bool = True):
        """pdsch.llr_is_8bit (srsUE pdsch_8bit_decoder): int8 LLRs and the 8-bit DL-SCH."""
        check(self.L.mi355_pdsch_set_llr_8bit(self.h, int(enable)), "set_llr_8bit")
        self.llr8 = bool(enable)

    def set_ce_invariant(self, enable: bool = True):
        """The estimates of the next decodes are the same in every OFDM symbol (mi355_pdsch_set_ce_invariant)."""
        check(self.L.mi355_pdsch_set_ce_invariant(self.h, int(enable)), "set_ce_invariant")

    def stage(self, job: int, cw: int, nof_re: int, nof_bits: int | None):
        """(d complex64[nof_re], csi float32[nof_re], e int16[nof_bits] (int8 in 8-bit mode) or None) of the last
        call."""
        d, c, e = C.c_void_p(), C.c_void_p(), C.c_void_p()
        check(self.L.mi355_pdsch_debug_stage(self.h, job, cw, C.byref(d), C.byref(c), C.byref(e)), "debug_stage")
        L = lib()
        dd = np.zeros(nof_re, np.complex64)
        cc = np.zeros(nof_re, np.float32)
        check(L.mi355_memcpy_d2h(dd.ctypes.data, d.value, dd.nbytes), "d2h")
        check(L.mi355_memcpy_d2h(cc.ctypes.data, c.value, cc.nbytes), "d2h")
        ee = None
        if nof_bits and e.value:
            ee = np.zeros(nof_bits, np.int8 if getattr(self, "llr8", False) else np.int16)
            check(L.mi355_memcpy_d2h(ee.ctypes.data, e.value, ee.nbytes), "d2h")
        return dd, cc, ee

    def close(self):
        if getattr(self, "h", None):
            self.L.mi355_pdsch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
