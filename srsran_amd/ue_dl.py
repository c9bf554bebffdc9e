"""Python mirror of include/srsran_amd/ue_dl.h -- batched OFDM demodulation, channel estimation and the
srslte_ue_dl-level object (lib/src/phy/ue/ue_dl.c) owning the PDSCH receiver."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import check
from .pdsch import Cell, Pdsch, _declare as _declare_pdsch

MAX_PORTS = 4
CHEST_FILTER_GAUSS, CHEST_FILTER_TRIANGLE, CHEST_FILTER_NONE = range(3)
NOISE_ALG_REFS, NOISE_ALG_PSS, NOISE_ALG_EMPTY = range(3)
MAX_LINKS = 65536


class ChestCfg(C.Structure):
    _fields_ = [("estimator_alg", C.c_uint32), ("noise_alg", C.c_uint32), ("filter_type", C.c_uint32),
                ("filter_coef", C.c_float * 2), ("rsrp_neighbour", C.c_uint32), ("cfo_estimate_enable", C.c_uint32),
                ("sync_error_enable", C.c_uint32), ("cfo_estimate_sf_mask", C.c_uint32)]
CE_ROWS_ALL, CE_ROWS_FIRST = 0, 1


def default_chest_cfg(filter_type: int = CHEST_FILTER_GAUSS, coef=(4.0, 1.0)) -> ChestCfg:
    """phy_dl_test.c:578-586 / srsUE defaults: Gauss order 4 sigma 1, REFS noise, AVERAGE estimator."""
    c = ChestCfg()
    c.filter_type = filter_type
    c.filter_coef[0], c.filter_coef[1] = coef
    return c


F4x4 = (C.c_float * 4) * 4


class ChestRes(C.Structure):
    _fields_ = [("nof_re", C.c_uint32), ("noise_estimate", C.c_float), ("noise_estimate_dbm", C.c_float),
                ("snr_db", C.c_float), ("snr_ant_port_db", F4x4), ("rsrp", C.c_float), ("rsrp_dbm", C.c_float),
                ("rsrp_neigh", C.c_float), ("rsrp_port_dbm", C.c_float * 4), ("rsrp_ant_port_dbm", F4x4),
                ("rsrq", C.c_float), ("rsrq_db", C.c_float), ("rsrq_ant_port_db", F4x4), ("rssi_dbm", C.c_float),
                ("cfo", C.c_float), ("sync_error", C.c_float)]


class DlSfJob(C.Structure):
    _fields_ = [("tti", C.c_uint32), ("in_buffer", C.c_void_p * 2), ("sf_symbols", C.c_void_p * 2),
                ("ce", (C.c_void_p * 2) * 4), ("link", C.c_uint32)]


def _declare():
    L = _declare_pdsch()
    if getattr(L, "_ue_dl_declared", False):
        return L
    vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int
    L.mi355_symbol_sz.restype = u32
    L.mi355_symbol_sz.argtypes = [u32, i32]
    L.mi355_ue_dl_create.argtypes = [C.POINTER(vp), C.POINTER(Cell), u32, i32]
    L.mi355_ue_dl_destroy.argtypes = [vp]
    L.mi355_ue_dl_set_standard_rates.argtypes = [vp, i32]
    L.mi355_ue_dl_reset_link.argtypes = [vp, u32]
    L.mi355_ue_dl_set_chunks.argtypes = [vp, u32]
    L.mi355_ue_dl_set_ce_rows.argtypes = [vp, u32]
    L.mi355_ue_dl_get_stream.restype = vp
    L.mi355_ue_dl_get_stream.argtypes = [vp]
    L.mi355_ofdm_rx_batch.argtypes = [vp, C.POINTER(DlSfJob), u32, vp]
    L.mi355_chest_dl_estimate_batch.argtypes = [vp, C.POINTER(DlSfJob), u32, C.POINTER(ChestCfg),
                                                C.POINTER(ChestRes), vp]
    L.mi355_ue_dl_decode_fft_estimate_batch.argtypes = [vp, C.POINTER(DlSfJob), u32, C.POINTER(ChestCfg),
                                                        C.POINTER(ChestRes), vp]
    L.mi355_ue_dl_pdsch.restype = vp
    L.mi355_ue_dl_pdsch.argtypes = [vp]
    from .pdsch import DlSfCfg, PdschCfg, PdschRes
    L.mi355_ue_dl_decode_pdsch_batch.argtypes = [vp, vp, C.POINTER(DlSfJob), C.POINTER(DlSfCfg), C.POINTER(PdschCfg),
                                                 C.POINTER(ChestRes), C.POINTER(vp), u32, C.POINTER(PdschRes), vp]
    L.mi355_ue_dl_decode_batch.argtypes = [vp, vp, C.POINTER(DlSfJob), C.POINTER(DlSfCfg), C.POINTER(PdschCfg),
                                           C.POINTER(ChestCfg), C.POINTER(ChestRes), C.POINTER(vp), u32,
                                           C.POINTER(PdschRes), vp]
    L._ue_dl_declared = True
    return L


def symbol_sz(nof_prb: int, std: bool = False) -> int:
    return int(_declare().mi355_symbol_sz(nof_prb, int(std)))


class UeDl:
    """srslte_ue_dl_t on one MI355X (FDD, normal subframes)."""

    def __init__(self, cell: Cell, nof_rx_antennas: int = 1, device: int = 0):
        self.L = _declare()
        h = C.c_void_p()
        check(self.L.mi355_ue_dl_create(C.byref(h), C.byref(cell), nof_rx_antennas, device), "ue_dl_create")
        self.h, self.cell, self.nrx, self.device = h, cell, nof_rx_antennas, device
        # the PDSCH receiver owned by the ue_dl object (borrowed handle)
        self.pdsch = Pdsch.__new__(Pdsch)
        self.pdsch.L, self.pdsch.h, self.pdsch.cell, self.pdsch.nrx = self.L, C.c_void_p(
            self.L.mi355_ue_dl_pdsch(self.h)), cell, nof_rx_antennas
        self.pdsch.device = device
        self.pdsch.close = lambda: None

    def stream(self):
        """the object's own stream (its calls given NULL run there): work to order in front of a call goes here"""
        return self.L.mi355_ue_dl_get_stream(self.h)

    def set_chunks(self, n: int):
        """find_and_decode's chunk count (0 = automatic)."""
        check(self.L.mi355_ue_dl_set_chunks(self.h, n), "set_chunks")

    def set_ce_rows(self, n: int):
        """Estimate rows the batched decode calls write (CE_ROWS_ALL / CE_ROWS_FIRST)."""
        check(self.L.mi355_ue_dl_set_ce_rows(self.h, n), "set_ce_rows")

    def reset_link(self, link: int):
        check(self.L.mi355_ue_dl_reset_link(self.h, link), "reset_link")

    def ofdm(self, jobs: list[DlSfJob]):
        arr = (DlSfJob * len(jobs))(*jobs)
        check(self.L.mi355_ofdm_rx_batch(self.h, arr, len(jobs), None), "ofdm_rx_batch")

    def chest(self, jobs: list[DlSfJob], cfg: ChestCfg):
        arr = (DlSfJob * len(jobs))(*jobs)
        res = (ChestRes * len(jobs))()
        check(self.L.mi355_chest_dl_estimate_batch(self.h, arr, len(jobs), C.byref(cfg), res, None), "chest")
        return res

    def fft_estimate(self, jobs: list[DlSfJob], cfg: ChestCfg):
        arr = (DlSfJob * len(jobs))(*jobs)
        res = (ChestRes * len(jobs))()
        check(self.L.mi355_ue_dl_decode_fft_estimate_batch(self.h, arr, len(jobs), C.byref(cfg), res, None),
              "decode_fft_estimate")
        return res

    def decode_pdsch(self, pool, jobs, sfs, cfgs, chest, payloads):
        """mi355_ue_dl_decode_pdsch_batch; payloads: 2 device pointers per job."""
        from .pdsch import DlSfCfg, PdschCfg, PdschRes
        n = len(jobs)
        res = (PdschRes * (2 * n))()
        pays = (C.c_void_p * (2 * n))(*payloads)
        check(self.L.mi355_ue_dl_decode_pdsch_batch(self.h, pool.h, (DlSfJob * n)(*jobs), (DlSfCfg * n)(*sfs),
                                                    (PdschCfg * n)(*cfgs), chest, pays, n, res, None), "decode_pdsch")
        return res

    def decode(self, pool, jobs, sfs, cfgs, cfg: ChestCfg, payloads):
        """mi355_ue_dl_decode_batch (fft + estimate + PDSCH in one call): returns (chest res, PDSCH res)."""
        from .pdsch import DlSfCfg, PdschCfg, PdschRes
        n = len(jobs)
        res = (PdschRes * (2 * n))()
        chest = (ChestRes * n)()
        pays = (C.c_void_p * (2 * n))(*payloads)
        check(self.L.mi355_ue_dl_decode_batch(self.h, pool.h, (DlSfJob * n)(*jobs), (DlSfCfg * n)(*sfs),
                                              (PdschCfg * n)(*cfgs), C.byref(cfg), chest, pays, n, res, None),
              "ue_dl_decode_batch")
        return chest, res

    def close(self):
        if getattr(self, "h", None):
            self.L.mi355_ue_dl_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
