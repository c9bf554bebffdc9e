"""Python mirror of include/srsran_amd/pdcch.h -- the downlink control receiver (PCFICH, PDCCH blind search) and the
host DCI / resource-allocation functions (lib/src/phy/phch/{pcfich,pdcch,dci,ra,ra_dl}.c, ue/ue_dl.c)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import check
from .pdsch import Cell, DlSfCfg, PdschCfg, PdschGrant, PdschRes
from .ue_dl import ChestCfg, ChestRes, DlSfJob, _declare as _declare_ue_dl

DCI_MAX_BITS, MAX_DCI_MSG = 128, 5
FORMAT0, FORMAT1, FORMAT1A, FORMAT1C, FORMAT1B, FORMAT1D, FORMAT2, FORMAT2A, FORMAT2B = range(9)
ALLOC_TYPE0, ALLOC_TYPE1, ALLOC_TYPE2 = range(3)
TM1, TM2, TM3, TM4 = range(4)
SIRNTI, PRNTI, MRNTI = 0xFFFF, 0xFFFE, 0xFFFD


class DciCfg(C.Structure):
    _fields_ = [("multiple_csi_request_enabled", C.c_uint32), ("cif_enabled", C.c_uint32),
                ("cif_present", C.c_uint32), ("srs_request_enabled", C.c_uint32), ("ra_format_enabled", C.c_uint32),
                ("is_not_ue_ss", C.c_uint32)]


class DciLocation(C.Structure):
    _fields_ = [("L", C.c_uint32), ("ncce", C.c_uint32)]


class DciMsg(C.Structure):
    _fields_ = [("payload", C.c_uint8 * DCI_MAX_BITS), ("nof_bits", C.c_uint32), ("location", DciLocation),
                ("format", C.c_uint32), ("rnti", C.c_uint16)]


class DciTb(C.Structure):
    _fields_ = [("mcs_idx", C.c_uint32), ("rv", C.c_int32), ("ndi", C.c_uint32), ("cw_idx", C.c_uint32)]


class _Type0(C.Structure):
    _fields_ = [("rbg_bitmask", C.c_uint32)]


class _Type1(C.Structure):
    _fields_ = [("vrb_bitmask", C.c_uint32), ("rbg_subset", C.c_uint32), ("shift", C.c_uint32)]


class _Type2(C.Structure):
    _fields_ = [("riv", C.c_uint32), ("n_prb1a", C.c_uint32), ("n_gap", C.c_uint32), ("mode", C.c_uint32)]


class _Alloc(C.Union):
    _fields_ = [("type0_alloc", _Type0), ("type1_alloc", _Type1), ("type2_alloc", _Type2)]


class DciDl(C.Structure):
    _anonymous_ = ("alloc",)
    _fields_ = [("rnti", C.c_uint16), ("format", C.c_uint32), ("location", DciLocation), ("ue_cc_idx", C.c_uint32),
                ("alloc_type", C.c_uint32), ("alloc", _Alloc), ("tb", DciTb * 2), ("tb_cw_swap", C.c_uint32),
                ("pinfo", C.c_uint32), ("pconf", C.c_uint32), ("power_offset", C.c_uint32), ("tpc_pucch", C.c_uint8),
                ("is_ra_order", C.c_uint32), ("ra_preamble", C.c_uint32), ("ra_mask_idx", C.c_uint32),
                ("cif", C.c_uint32), ("cif_present", C.c_uint32), ("srs_request", C.c_uint32),
                ("srs_request_present", C.c_uint32), ("pid", C.c_uint32), ("dai", C.c_uint32), ("is_tdd", C.c_uint32),
                ("is_dwpts", C.c_uint32), ("sram_id", C.c_uint32)]


class UeDlCfg(C.Structure):
    _fields_ = [("tm", C.c_uint32), ("dci_common_ss", C.c_uint32), ("dci", DciCfg), ("use_tbs_index_alt", C.c_uint32)]


class CtrlRes(C.Structure):
    _fields_ = [("cfi", C.c_uint32), ("cfi_corr", C.c_float), ("nof_dci", C.c_int32), ("nof_cce", C.c_uint32)]


def _declare():
    L = _declare_ue_dl()
    if getattr(L, "_pdcch_declared", False):
        return L
    vp, u32, i32, u16 = C.c_void_p, C.c_uint32, C.c_int, C.c_uint16
    P = C.POINTER
    L.mi355_dci_format_sizeof.restype = u32
    L.mi355_dci_format_sizeof.argtypes = [P(Cell), P(DciCfg), u32]
    L.mi355_dci_msg_unpack_pdsch.argtypes = [P(Cell), P(DlSfCfg), P(DciCfg), P(DciMsg), P(DciDl)]
    L.mi355_dci_msg_pack_pdsch.argtypes = [P(Cell), P(DlSfCfg), P(DciCfg), P(DciDl), P(DciMsg)]
    L.mi355_ra_dl_dci_to_grant.argtypes = [P(Cell), P(DlSfCfg), u32, u32, P(DciDl), P(PdschGrant)]
    L.mi355_ra_tbs_from_idx.argtypes = [u32, u32]
    L.mi355_ra_type2_to_riv.restype = u32
    L.mi355_ra_type2_to_riv.argtypes = [u32, u32, u32]
    L.mi355_pdcch_ue_locations_ncce.restype = u32
    L.mi355_pdcch_ue_locations_ncce.argtypes = [u32, P(DciLocation), u32, u32, u16]
    L.mi355_pdcch_common_locations_ncce.restype = u32
    L.mi355_pdcch_common_locations_ncce.argtypes = [u32, P(DciLocation), u32]
    L.mi355_regs_pdcch_ncce.argtypes = [P(Cell), u32]
    L.mi355_pcfich_encode_host.argtypes = [P(Cell), P(DlSfCfg), P(vp)]
    L.mi355_pdcch_encode_host.argtypes = [P(Cell), P(DlSfCfg), P(DciMsg), P(vp)]
    L.mi355_ue_dl_find_dl_dci_batch.argtypes = [vp, P(DlSfJob), P(DlSfCfg), P(UeDlCfg), P(u16), P(ChestRes), u32,
                                                P(CtrlRes), P(DciDl), vp]
    L.mi355_ue_dl_find_and_decode_batch.argtypes = [vp, vp, P(DlSfJob), P(DlSfCfg), P(UeDlCfg), P(PdschCfg),
                                                    P(ChestCfg), P(ChestRes), P(vp), u32, P(CtrlRes), P(DciDl),
                                                    P(PdschRes), vp]
    L.mi355_ue_dl_ctrl_llr.argtypes = [vp, u32, vp, u32]
    L.mi355_ue_dl_ctrl_candidates.argtypes = [vp, u32, vp, u32]
    L._pdcch_declared = True
    return L


# ------------------------------------------------------------------ host functions

def dci_sizeof(cell: Cell, fmt: int, cfg: DciCfg | None = None) -> int:
    return int(_declare().mi355_dci_format_sizeof(C.byref(cell), C.byref(cfg) if cfg else None, fmt))


def dci_msg(bits, fmt: int, rnti: int, L: int = 0, ncce: int = 0) -> DciMsg:
    m = DciMsg()
    bits = np.asarray(bits, np.uint8)
    for i, b in enumerate(bits):
        m.payload[i] = int(b)
    m.nof_bits, m.format, m.rnti = bits.size, fmt, rnti
    m.location = DciLocation(L, ncce)
    return m


def msg_bits(m: DciMsg) -> np.ndarray:
    return np.frombuffer(bytes(m.payload), np.uint8)[: m.nof_bits].copy()


def unpack(cell: Cell, msg: DciMsg, tti: int = 0, cfg: DciCfg | None = None) -> DciDl | None:
    d = DciDl()
    sf = DlSfCfg(tti, 1)
    rc = _declare().mi355_dci_msg_unpack_pdsch(C.byref(cell), C.byref(sf), C.byref(cfg) if cfg else None,
                                                C.byref(msg), C.byref(d))
    return d if rc == 0 else None


def pack(cell: Cell, dci: DciDl, tti: int = 0, cfg: DciCfg | None = None) -> DciMsg:
    m = DciMsg()
    sf = DlSfCfg(tti, 1)
    check(_declare().mi355_dci_msg_pack_pdsch(C.byref(cell), C.byref(sf), C.byref(cfg) if cfg else None,
                                              C.byref(dci), C.byref(m)), "dci_msg_pack_pdsch")
    return m


def dci_to_grant(cell: Cell, dci: DciDl, tti: int, cfi: int, tm: int, tbs_alt: bool = False) -> PdschGrant | None:
    g = PdschGrant()
    sf = DlSfCfg(tti, cfi)
    rc = _declare().mi355_ra_dl_dci_to_grant(C.byref(cell), C.byref(sf), tm, int(tbs_alt), C.byref(dci), C.byref(g))
    return g if rc == 0 else None


def ue_locations(nof_cce: int, sf_idx: int, rnti: int) -> list[tuple[int, int]]:
    c = (DciLocation * 16)()
    n = _declare().mi355_pdcch_ue_locations_ncce(nof_cce, c, 16, sf_idx, rnti)
    return [(c[i].L, c[i].ncce) for i in range(n)]


def common_locations(nof_cce: int) -> list[tuple[int, int]]:
    c = (DciLocation * 6)()
    n = _declare().mi355_pdcch_common_locations_ncce(nof_cce, c, 6)
    return [(c[i].L, c[i].ncce) for i in range(n)]


def nof_cce(cell: Cell, cfi: int) -> int:
    return int(_declare().mi355_regs_pdcch_ncce(C.byref(cell), cfi))


def encode_ctrl_host(cell: Cell, tti: int, cfi: int, msgs: list[DciMsg], grids: np.ndarray) -> None:
    """PCFICH + PDCCH messages into host tx grids (ports, 14 * 12 * nof_prb) complex64, in place."""
    assert grids.dtype == np.complex64 and grids.flags["C_CONTIGUOUS"]
    L = _declare()
    ptrs = (C.c_void_p * 4)(*[grids[p].ctypes.data for p in range(grids.shape[0])] + [None] * (4 - grids.shape[0]))
    sf = DlSfCfg(tti, cfi)
    check(L.mi355_pcfich_encode_host(C.byref(cell), C.byref(sf), ptrs), "pcfich_encode")
    for m in msgs:
        check(L.mi355_pdcch_encode_host(C.byref(cell), C.byref(sf), C.byref(m), ptrs), "pdcch_encode")


# ------------------------------------------------------------------ GPU batches

def find_dl_dci(ue, jobs: list[DlSfJob], rntis: list[int], cfgs: list[UeDlCfg], chest):
    """mi355_ue_dl_find_dl_dci_batch: returns (cfis, ctrl results, per-job list of DciDl)."""
    L = _declare()
    n = len(jobs)
    sfs = (DlSfCfg * n)(*[DlSfCfg(j.tti, 0) for j in jobs])
    ctrl = (CtrlRes * n)()
    dci = (DciDl * (n * MAX_DCI_MSG))()
    check(L.mi355_ue_dl_find_dl_dci_batch(ue.h, (DlSfJob * n)(*jobs), sfs, (UeDlCfg * n)(*cfgs),
                                          (C.c_uint16 * n)(*rntis), chest, n, ctrl, dci, None), "find_dl_dci_batch")
    out = [[dci[i * MAX_DCI_MSG + k] for k in range(max(0, ctrl[i].nof_dci))] for i in range(n)]
    return [sfs[i].cfi for i in range(n)], ctrl, out


def find_and_decode(ue, pool, jobs: list[DlSfJob], ue_cfgs: list[UeDlCfg], cfgs: list[PdschCfg], chest_cfg: ChestCfg,
                    payloads: list[int]):
    """mi355_ue_dl_find_and_decode_batch: returns (sfs, chest, ctrl, dci lists, PDSCH res, cfgs with grants)."""
    L = _declare()
    n = len(jobs)
    sfs = (DlSfCfg * n)(*[DlSfCfg(j.tti, 0) for j in jobs])
    carr = (PdschCfg * n)(*cfgs)
    chest = (ChestRes * n)()
    ctrl = (CtrlRes * n)()
    dci = (DciDl * (n * MAX_DCI_MSG))()
    res = (PdschRes * (2 * n))()
    check(L.mi355_ue_dl_find_and_decode_batch(ue.h, pool.h, (DlSfJob * n)(*jobs), sfs, (UeDlCfg * n)(*ue_cfgs), carr,
                                              C.byref(chest_cfg), chest, (C.c_void_p * (2 * n))(*payloads), n, ctrl,
                                              dci, res, None), "find_and_decode_batch")
    out = [[dci[i * MAX_DCI_MSG + k] for k in range(max(0, ctrl[i].nof_dci))] for i in range(n)]
    return sfs, chest, ctrl, out, res, carr


def last_llr(ue, i: int) -> np.ndarray:
    """PDCCH LLRs of subframe i of the previous control-channel call on ue (inspection)."""
    out = np.zeros(8 * 1024, np.float32)
    n = _declare().mi355_ue_dl_ctrl_llr(ue.h, i, out.ctypes.data, out.size)
    if n < 0:
        raise RuntimeError("ctrl_llr failed")
    return out[:n].copy()


CAND_DTYPE = np.dtype([("status", np.uint32), ("crc_rem", np.uint32), ("L", np.uint32), ("ncce", np.uint32),
                       ("bits", np.uint32, 4)])


def last_candidates(ue, i: int) -> np.ndarray:
    """Raw candidate results of subframe i: (22 slots, 2 sizes) records of CAND_DTYPE."""
    out = np.zeros(22 * 2 * 8, np.uint32)
    n = _declare().mi355_ue_dl_ctrl_candidates(ue.h, i, out.ctypes.data, out.size)
    if n < 0:
        raise RuntimeError("ctrl_candidates failed")
    return out.view(CAND_DTYPE).reshape(22, 2)
