"""oracle.pdcch_chain -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the srsLTE downlink control path used as the checker for the GPU control-channel
kernels and the product's DCI host code:
  * REG tables, PCFICH decode, PDCCH LLR extraction, candidate decoding (C, ``orc_pdcch.c``);
  * DCI payload sizes / unpacking / packing (phch/dci.c), the DL grant (phch/ra.c, ra_dl.c) and the UE blind
    search (ue/ue_dl.c:420-730) -- small integer logic, restated here in Python;
  * an eNodeB-side PCFICH + PDCCH synthesiser (pcfich.c:235-272, pdcch.c:548-625) for test subframes.
Wrappers for the reference's own functions (``oracle/_ref``) sit next to the restatement they pin.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass, field

import numpy as np

import oracle

u8p, u16p, u32p, f32p = oracle.u8p, oracle.u16p, oracle.u32p, oracle.f32p
HERE = os.path.dirname(os.path.abspath(__file__))

# srslte_dci_format_t (phy_common.h:288-297)
FORMAT0, FORMAT1, FORMAT1A, FORMAT1C, FORMAT1B, FORMAT1D, FORMAT2, FORMAT2A, FORMAT2B = range(9)
SIRNTI, PRNTI, MRNTI = 0xFFFF, 0xFFFE, 0xFFFD
MAX_NREGS = 1000


def is_user(rnti):  # SRSLTE_RNTI_ISUSER (phy_common.h:92)
    return 0x000B <= rnti <= 0xFFF3


def is_rar(rnti):
    return 0x0001 <= rnti <= 0x000A


_bound = set()


def _bind(L, name, res, args):
    f = getattr(L, name)
    f.restype, f.argtypes = res, args
    return f


def _lib():
    L = oracle.lib()
    if "orc" not in _bound:
        _bind(L, "orc_regs_init", C.c_int, [C.c_uint32] * 7 + [u32p, u32p, C.c_uint32, u32p, C.c_void_p])
        _bind(L, "orc_ctrl_equalize", None, [f32p, f32p, C.c_int, C.c_int, C.c_int, C.c_float, f32p])
        _bind(L, "orc_pcfich_decode", C.c_int, [f32p, f32p, C.c_int, C.c_int, C.c_int, u32p, C.c_uint32, C.c_uint32,
                                                C.c_float, f32p, f32p])
        _bind(L, "orc_pdcch_llr", C.c_int, [f32p, f32p, C.c_int, C.c_int, C.c_int, u32p, C.c_uint32, C.c_uint32,
                                            C.c_uint32, C.c_float, f32p])
        _bind(L, "orc_pdcch_ue_locations", C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, u32p, u32p])
        _bind(L, "orc_pdcch_common_locations", C.c_uint32, [C.c_uint32, u32p, u32p])
        _bind(L, "orc_rm_conv_rx", None, [f32p, C.c_uint32, f32p, C.c_uint32])
        _bind(L, "orc_rm_conv_tx", None, [u8p, C.c_uint32, u8p, C.c_uint32])
        _bind(L, "orc_conv_encode_tb", None, [u8p, C.c_uint32, u8p])
        _bind(L, "orc_viterbi_quant", None, [f32p, C.c_uint32, u16p])
        _bind(L, "orc_viterbi37_tb_decode_us", C.c_int, [u16p, C.c_uint32, u8p])
        _bind(L, "orc_crc16_bits", C.c_uint32, [u8p, C.c_uint32])
        _bind(L, "orc_pdcch_decode_candidate", C.c_int, [f32p, C.c_uint32, C.c_uint32, u8p, C.POINTER(C.c_uint16)])
        _bind(L, "orc_pdcch_encode", None, [u8p, C.c_uint32, C.c_uint32, C.c_uint32, u8p])
        _bound.add("orc")
    return L


def _ref():
    R = oracle.ref()
    if "ref" not in _bound:
        _bind(R, "ref_regs_init", C.c_int, [C.c_uint32] * 6 + [u32p, u32p, C.c_uint32, u32p, C.c_void_p])
        _bind(R, "ref_pcfich_decode", C.c_int, [f32p, f32p, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                                C.c_float, C.POINTER(C.c_float)])
        _bind(R, "ref_pdcch_llr", C.c_int, [f32p, f32p, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                            C.c_uint32, C.c_float, f32p])
        _bind(R, "ref_pdcch_dci_decode", C.c_int, [f32p, C.c_uint32, C.c_uint32, u8p])
        _bind(R, "ref_viterbi_decode_us", C.c_int, [u16p, C.c_uint32, u8p])
        _bind(R, "ref_viterbi_decode_f", C.c_int, [f32p, C.c_uint32, u8p])
        _bind(R, "ref_rm_conv_rx", None, [f32p, C.c_uint32, f32p, C.c_uint32])
        _bind(R, "ref_pdcch_dci_encode", C.c_int, [u8p, C.c_uint32, C.c_uint16, C.c_uint32, u8p])
        _bind(R, "ref_crc16", C.c_uint32, [u8p, C.c_int])
        _bind(R, "ref_ue_locations", C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint16, u32p, u32p])
        _bind(R, "ref_common_locations", C.c_uint32, [C.c_uint32, u32p, u32p])
        _bound.add("ref")
    return R


# ------------------------------------------------------------------ REG tables

@dataclass
class Regs:
    pcfich: np.ndarray          # (16,) grid indices
    pdcch: list                 # per CFI 1..3: (4 * nregs,) grid indices
    nregs: np.ndarray           # (3,) usable REGs per CFI
    phich: np.ndarray           # (ngroups, 12)

    def nof_cce(self, cfi):
        return int(self.nregs[cfi - 1]) // 9


def regs(nof_prb, nof_ports, cell_id, phich_res=2, phich_ext=0, mi=1, use_ref=False) -> Regs:
    """srslte_regs_init_opts tables (CP normal).  phich_res: 0 R1/6, 1 R1/2, 2 R1, 3 R2."""
    pc = np.zeros(16, np.uint32)
    pd = np.zeros(3 * MAX_NREGS * 4, np.uint32)
    nr = np.zeros(3, np.uint32)
    ph = np.zeros(12 * 64, np.uint32)
    if use_ref:
        ng = _ref().ref_regs_init(nof_prb, nof_ports, cell_id, phich_res, phich_ext, mi, pc, pd, MAX_NREGS, nr,
                                  ph.ctypes.data)
    else:
        ng = _lib().orc_regs_init(nof_prb, nof_ports, cell_id, 0, phich_res, phich_ext, mi, pc, pd, MAX_NREGS, nr,
                                  ph.ctypes.data)
    if ng < 0:
        raise ValueError("regs init failed")
    pd = pd.reshape(3, MAX_NREGS * 4)
    return Regs(pc, [pd[c, : 4 * nr[c]].copy() for c in range(3)], nr, ph[: 12 * ng].reshape(ng, 12))


# ------------------------------------------------------------------ receive

def _grid_ce(grids, ce):
    grids = np.ascontiguousarray(grids, np.complex64)
    nof_rx = grids.shape[0]
    ce = np.ascontiguousarray(ce, np.complex64)  # (ports, rx, grid)
    return grids, ce, nof_rx, ce.shape[0], grids.shape[1]


def pcfich_decode(grids, ce, rg: Regs, cell_id, sf_idx, noise):
    grids, ce, nrx, nports, glen = _grid_ce(grids, ce)
    corr = np.zeros(3, np.float32)
    llr = np.zeros(32, np.float32)
    cfi = _lib().orc_pcfich_decode(grids.view(np.float32).ravel(), ce.view(np.float32).ravel(), nrx, nports, glen,
                                   rg.pcfich, cell_id, sf_idx, noise, corr, llr)
    return cfi, corr, llr


def pdcch_llr(grids, ce, rg: Regs, cfi, cell_id, sf_idx, noise):
    grids, ce, nrx, nports, glen = _grid_ce(grids, ce)
    n = int(rg.nregs[cfi - 1])
    llr = np.zeros(8 * n, np.float32)
    _lib().orc_pdcch_llr(grids.view(np.float32).ravel(), ce.view(np.float32).ravel(), nrx, nports, glen,
                         rg.pdcch[cfi - 1], n, cell_id, sf_idx, noise, llr)
    return llr


def ue_locations(nof_cce, sf_idx, rnti, use_ref=False):
    L, n = np.zeros(16, np.uint32), np.zeros(16, np.uint32)
    f = _ref().ref_ue_locations if use_ref else _lib().orc_pdcch_ue_locations
    k = f(nof_cce, sf_idx, rnti, L, n)
    return [(int(L[i]), int(n[i])) for i in range(k)]


def common_locations(nof_cce, use_ref=False):
    L, n = np.zeros(6, np.uint32), np.zeros(6, np.uint32)
    f = _ref().ref_common_locations if use_ref else _lib().orc_pdcch_common_locations
    k = f(nof_cce, L, n)
    return [(int(L[i]), int(n[i])) for i in range(k)]


def decode_candidate(llr, L, ncce, nof_bits):
    """srslte_pdcch_decode_msg for one (location, size): (decoded?, payload bits, crc remainder)."""
    E = 72 << L
    seg = np.ascontiguousarray(llr[72 * ncce: 72 * ncce + E], np.float32)
    pay = np.zeros(nof_bits, np.uint8)
    crc = C.c_uint16(0)
    ok = _lib().orc_pdcch_decode_candidate(seg, E, nof_bits, pay, C.byref(crc))
    return bool(ok), pay, int(crc.value)


# ------------------------------------------------------------------ DCI sizes (dci.c:93-415), FDD

@dataclass
class DciCfg:
    multiple_csi_request_enabled: bool = False
    cif_enabled: bool = False
    srs_request_enabled: bool = False
    is_not_ue_ss: bool = False


def riv_nbits(nof_prb):
    return int(math.ceil(math.log2(nof_prb * (nof_prb + 1) / 2)))


AMBIGUOUS = (12, 14, 16, 20, 24, 26, 32, 40, 44, 56)


def ra_type0_P(nof_prb):
    return 1 if nof_prb <= 10 else 2 if nof_prb <= 26 else 3 if nof_prb <= 63 else 4


def ra_type2_ngap(nof_prb, ngap_is_1):
    if nof_prb <= 10:
        return nof_prb // 2
    if nof_prb == 11:
        return 4
    if nof_prb <= 19:
        return 8
    if nof_prb <= 26:
        return 12
    if nof_prb <= 44:
        return 18
    if nof_prb <= 49:
        return 27
    if nof_prb <= 63:
        return 27 if ngap_is_1 else 9
    if nof_prb <= 79:
        return 32 if ngap_is_1 else 16
    return 48 if ngap_is_1 else 16


def ra_type2_n_rb_step(nof_prb):
    return 2 if nof_prb < 50 else 4


def ra_type2_n_vrb_dl(nof_prb, ngap_is_1):
    ng = ra_type2_ngap(nof_prb, ngap_is_1)
    return 2 * min(ng, nof_prb - ng) if ngap_is_1 else (nof_prb // ng) * 2 * ng


def _f0_raw(nof_prb, cfg):
    n = (3 if cfg.cif_enabled else 0) + 1 + 1 + riv_nbits(nof_prb) + 5 + 1 + 2 + 3
    n += 2 if (cfg.multiple_csi_request_enabled and not cfg.is_not_ue_ss) else 1
    n += 1 if (cfg.srs_request_enabled and not cfg.is_not_ue_ss) else 0
    return n + 1


def _f1a(nof_prb, cfg):
    n = (3 if cfg.cif_enabled else 0) + 1 + 1 + riv_nbits(nof_prb) + 5 + 3 + 1 + 2 + 2
    n += 1 if cfg.srs_request_enabled else 0
    n = max(n, _f0_raw(nof_prb, cfg))
    return n + 1 if n in AMBIGUOUS else n


def dci_sizeof(fmt, nof_prb, nof_ports, cfg=None):
    cfg = cfg or DciCfg()
    cif = 3 if cfg.cif_enabled else 0
    alloc = int(math.ceil(nof_prb / ra_type0_P(nof_prb)))
    big = 1 if nof_prb > 10 else 0
    if fmt == FORMAT0:
        return max(_f0_raw(nof_prb, cfg), _f1a(nof_prb, cfg))
    if fmt == FORMAT1A:
        return _f1a(nof_prb, cfg)
    if fmt == FORMAT1:
        n = alloc + 5 + 3 + 1 + 2 + 2 + cif + big
        while n in (dci_sizeof(FORMAT0, nof_prb, nof_ports, cfg), _f1a(nof_prb, cfg)) or n in AMBIGUOUS:
            n += 1
        return n
    if fmt == FORMAT1C:
        n = riv_nbits(ra_type2_n_vrb_dl(nof_prb, True) // ra_type2_n_rb_step(nof_prb)) + 5
        return n + (1 if nof_prb >= 50 else 0)
    if fmt in (FORMAT1B, FORMAT1D):
        n = cif + 1 + riv_nbits(nof_prb) + 5 + 3 + 1 + 2 + 2 + (2 if nof_ports <= 2 else 4) + 1
        n = max(n, _f0_raw(nof_prb, cfg))
        while n in AMBIGUOUS:
            n += 1
        return n
    if fmt in (FORMAT2, FORMAT2A, FORMAT2B):
        pb = {FORMAT2: 3 if nof_ports <= 2 else 6, FORMAT2A: 0 if nof_ports <= 2 else 2, FORMAT2B: 0}[fmt]
        n = alloc + 2 + 3 + 1 + 2 * (5 + 1 + 2) + pb + cif + big
        while n in AMBIGUOUS:
            n += 1
        return n
    raise ValueError(fmt)


# ------------------------------------------------------------------ DCI unpack / pack (dci.c:582-1335)

def _take(bits, pos, n):
    v = 0
    for i in range(n):
        v = (v << 1) | int(bits[pos + i])
    return v, pos + n


def _put(out, v, n):
    for i in range(n - 1, -1, -1):
        out.append((v >> i) & 1)


def _log2ceil(P):
    return int(math.ceil(math.log2(P)))


def dci_unpack(bits, fmt, rnti, nof_prb, nof_ports, cfg=None) -> dict | None:
    """srslte_dci_msg_unpack_pdsch (dci.c:1283-1335), FDD: returns the srslte_dci_dl_t fields or None on error."""
    cfg = cfg or DciCfg()
    d = dict(rnti=rnti, format=fmt, alloc_type=0, rbg_bitmask=0, vrb_bitmask=0, rbg_subset=0, shift=0, riv=0,
             n_prb1a=0, n_gap=0, mode=0, tb=[dict(mcs_idx=0, rv=0, ndi=0, cw_idx=0), dict(mcs_idx=0, rv=1, ndi=0, cw_idx=0)],
             tb_cw_swap=0, pinfo=0, tpc_pucch=0, is_ra_order=0, ra_preamble=0, ra_mask_idx=0, pid=0, cif=0)
    p = 0
    if cfg.cif_enabled and fmt != FORMAT1C:
        d["cif"], p = _take(bits, p, 3)
    P = ra_type0_P(nof_prb)
    alloc_size = int(math.ceil(nof_prb / P))
    if fmt in (FORMAT1, FORMAT2, FORMAT2A, FORMAT2B):
        if len(bits) != dci_sizeof(fmt, nof_prb, nof_ports, cfg) and fmt == FORMAT1:
            return None
        if nof_prb > 10:
            d["alloc_type"] = int(bits[p]); p += 1
        if d["alloc_type"] == 0:
            d["rbg_bitmask"], p = _take(bits, p, alloc_size)
        elif d["alloc_type"] == 1:
            d["rbg_subset"], p = _take(bits, p, _log2ceil(P))
            d["shift"] = int(bits[p]); p += 1
            d["vrb_bitmask"], p = _take(bits, p, alloc_size - _log2ceil(P) - 1)
        else:
            return None
        if fmt == FORMAT1:
            d["tb"][0]["mcs_idx"], p = _take(bits, p, 5)
            d["pid"], p = _take(bits, p, 3)
            d["tb"][0]["ndi"] = int(bits[p]); p += 1
            d["tb"][0]["rv"], p = _take(bits, p, 2)
            d["tpc_pucch"], p = _take(bits, p, 2)
            return d
        d["tpc_pucch"], p = _take(bits, p, 2)
        d["pid"], p = _take(bits, p, 3)
        d["tb_cw_swap"] = int(bits[p]); p += 1
        nof_tb = 0
        for i in range(2):
            d["tb"][i]["mcs_idx"], p = _take(bits, p, 5)
            d["tb"][i]["ndi"] = int(bits[p]); p += 1
            d["tb"][i]["rv"], p = _take(bits, p, 2)
            nof_tb += tb_enabled(d["tb"][i])
        if fmt == FORMAT2:
            d["pinfo"], p = _take(bits, p, 3 if nof_ports <= 2 else 6)
        elif fmt == FORMAT2A:
            d["pinfo"], p = _take(bits, p, 0 if nof_ports <= 2 else 2)
        for i in range(2):
            d["tb"][i]["cw_idx"] = ((1 if d["tb_cw_swap"] else 0) + i) % nof_tb if nof_tb == 2 else 0
        return d
    if fmt == FORMAT1A:
        if int(bits[p]) != 1:
            return None
        p += 1
        if int(bits[p]) == 0:  # PDCCH order (dci.c:806-830)
            nb = riv_nbits(nof_prb)
            i = 0
            while i < nb and int(bits[p + 1 + i]) == 1:
                i += 1
            if i == nb:
                i = 1 + 10 + nb
                while i < len(bits) - 1 and int(bits[p + i]) == 0:
                    i += 1
                if i == len(bits) - 1:
                    q = p + 1 + nb
                    d["is_ra_order"] = 1
                    d["ra_preamble"], q = _take(bits, q, 6)
                    d["ra_mask_idx"], q = _take(bits, q, 4)
                    return d
        d["alloc_type"] = 2
        d["mode"] = int(bits[p]); p += 1
        nb_gap = 0
        if is_user(rnti) and d["mode"] == 1 and nof_prb >= 50:
            nb_gap = 1
            d["n_gap"] = int(bits[p]); p += 1
        d["riv"], p = _take(bits, p, riv_nbits(nof_prb) - nb_gap)
        d["tb"][0]["mcs_idx"], p = _take(bits, p, 5)
        d["pid"], p = _take(bits, p, 3)
        if not is_user(rnti):
            if nof_prb >= 50 and d["mode"] == 1:
                d["n_gap"] = int(bits[p])
            p += 1
        else:
            d["tb"][0]["ndi"] = int(bits[p]); p += 1
        d["tb"][0]["rv"], p = _take(bits, p, 2)
        if is_user(rnti):
            p += 2
        else:
            p += 1
            d["n_prb1a"] = int(bits[p]); p += 1
        return d
    if fmt == FORMAT1C:
        if len(bits) != dci_sizeof(FORMAT1C, nof_prb, nof_ports, cfg):
            return None
        d["alloc_type"], d["mode"] = 2, 1
        if nof_prb >= 50:
            d["n_gap"] = int(bits[p]); p += 1
        nvrb = ra_type2_n_vrb_dl(nof_prb, d["n_gap"] == 0)
        d["riv"], p = _take(bits, p, riv_nbits(nvrb // ra_type2_n_rb_step(nof_prb)))
        d["tb"][0]["mcs_idx"], p = _take(bits, p, 5)
        d["tb"][0]["rv"] = -1
        return d
    return None


def tb_enabled(tb):  # SRSLTE_DCI_IS_TB_EN
    return not (tb["mcs_idx"] == 0 and tb["rv"] == 1)


def dci_pack(d, nof_prb, nof_ports, cfg=None) -> np.ndarray:
    """srslte_dci_msg_pack_pdsch (dci.c:1238-1282) for formats 1, 1A, 1C, 2, 2A."""
    cfg = cfg or DciCfg()
    fmt, out = d["format"], []
    P = ra_type0_P(nof_prb)
    alloc_size = int(math.ceil(nof_prb / P))
    if fmt in (FORMAT1, FORMAT2, FORMAT2A):
        if nof_prb > 10:
            out.append(d["alloc_type"])
        if d["alloc_type"] == 0:
            _put(out, d["rbg_bitmask"], alloc_size)
        else:
            _put(out, d["rbg_subset"], _log2ceil(P))
            out.append(1 if d["shift"] else 0)
            _put(out, d["vrb_bitmask"], alloc_size - _log2ceil(P) - 1)
        if fmt == FORMAT1:
            _put(out, d["tb"][0]["mcs_idx"], 5)
            _put(out, d["pid"], 3)
            out.append(d["tb"][0]["ndi"])
            _put(out, d["tb"][0]["rv"], 2)
            _put(out, d["tpc_pucch"], 2)
        else:
            _put(out, d["tpc_pucch"], 2)
            _put(out, d["pid"], 3)
            out.append(d["tb_cw_swap"])
            for i in range(2):
                _put(out, d["tb"][i]["mcs_idx"], 5)
                out.append(d["tb"][i]["ndi"])
                _put(out, d["tb"][i]["rv"], 2)
            _put(out, d["pinfo"], (3 if nof_ports <= 2 else 6) if fmt == FORMAT2 else (0 if nof_ports <= 2 else 2))
    elif fmt == FORMAT1A:
        out.append(1)
        out.append(d["mode"])
        nb_gap = 0
        if is_user(d["rnti"]) and d["mode"] == 1 and nof_prb >= 50:
            nb_gap = 1
            out.append(d["n_gap"])
        _put(out, d["riv"], riv_nbits(nof_prb) - nb_gap)
        _put(out, d["tb"][0]["mcs_idx"], 5)
        _put(out, d["pid"], 3)
        if not is_user(d["rnti"]):
            out.append(d["n_gap"] if (nof_prb >= 50 and d["mode"] == 1) else 0)
        else:
            out.append(d["tb"][0]["ndi"])
        _put(out, d["tb"][0]["rv"], 2)
        if is_user(d["rnti"]):
            out += [0, 0]
        else:
            out += [0, d["n_prb1a"]]
    elif fmt == FORMAT1C:
        if nof_prb >= 50:
            out.append(d["n_gap"])
        nvrb = ra_type2_n_vrb_dl(nof_prb, d["n_gap"] == 0)
        _put(out, d["riv"], riv_nbits(nvrb // ra_type2_n_rb_step(nof_prb)))
        _put(out, d["tb"][0]["mcs_idx"], 5)
        return np.array(out, np.uint8)
    else:
        raise ValueError(fmt)
    n = dci_sizeof(fmt, nof_prb, nof_ports, cfg)
    out += [0] * (n - len(out))
    return np.array(out, np.uint8)


# ------------------------------------------------------------------ DL grant (ra.c, ra_dl.c:176-646)

_TBS = None


def tbs_table():
    global _TBS
    if _TBS is None:
        z = np.load(os.path.join(os.path.dirname(HERE), "tests", "golden", "tbs_table.npz"), allow_pickle=False)
        _TBS = (z["tbs"], z["format1c"])
    return _TBS


def tbs_idx_from_mcs(mcs, alt):
    if alt:
        t = [0, 2, 4, 6, 8, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 27, 28, 29, 30, 31, 32, 33]
        return t[mcs] if mcs < 28 else -1
    return (mcs if mcs < 10 else mcs - 1 if mcs < 17 else mcs - 2) if mcs < 29 else -1


def mod_from_mcs(mcs, alt):
    """srslte_ra_dl_mod_from_mcs: bits per symbol"""
    if alt:
        return 2 if (mcs < 5 or mcs == 28) else 4 if (mcs < 11 or mcs == 29) else 6 if (mcs < 20 or mcs == 30) else 8
    return 2 if (mcs < 10 or mcs == 29) else 4 if (mcs < 17 or mcs == 30) else 6


def type2_from_riv(riv, nof_prb, nof_vrb):
    L = riv // nof_prb + 1
    s = riv % nof_prb
    if L > (nof_vrb - s) & 0xFFFFFFFF:  # uint32 arithmetic in ra.c:49-58
        L = nof_prb - riv // nof_prb + 1
        s = nof_prb - riv % nof_prb - 1
    return L, s


def type2_to_riv(L, s, nof_prb):
    return nof_prb * (L - 1) + s if (L - 1) <= nof_prb // 2 else nof_prb * (nof_prb - L + 1) + nof_prb - 1 - s


def prb_allocation(d, nof_prb):
    """srslte_ra_dl_grant_to_grant_prb_allocation (ra_dl.c:176-327): (2, nof_prb) uint8 or None."""
    prb = np.zeros((2, nof_prb), np.uint8)
    P = ra_type0_P(nof_prb)
    at = d["alloc_type"]
    if at == 0:
        nb = int(math.ceil(nof_prb / P))
        for i in range(nb):
            if d["rbg_bitmask"] & (1 << (nb - i - 1)):
                for j in range(P):
                    if i * P + j < nof_prb:
                        prb[0, i * P + j] = 1
        prb[1] = prb[0]
    elif at == 1:
        if d["rbg_subset"] >= P:
            return None
        n1 = int(math.ceil(nof_prb / P)) - _log2ceil(P) - 1
        temp = ((nof_prb - 1) // P) % P
        if d["rbg_subset"] < temp:
            nsub = ((nof_prb - 1) // (P * P)) * P + P
        elif d["rbg_subset"] == temp:
            nsub = ((nof_prb - 1) // (P * P)) * P + ((nof_prb - 1) % P) + 1
        else:
            nsub = ((nof_prb - 1) // (P * P)) * P
        shift = (nsub - n1) if d["shift"] else 0
        for i in range(n1):
            if d["vrb_bitmask"] & (1 << (n1 - i - 1)):
                idx = ((i + shift) // P) * P * P + d["rbg_subset"] * P + (i + shift) % P
                if idx >= nof_prb:
                    return None
                prb[0, idx] = 1
        prb[1] = prb[0]
    else:
        nof_vrb = nof_prb if d["mode"] == 0 else ra_type2_n_vrb_dl(nof_prb, d["n_gap"] == 0)
        if d["format"] == FORMAT1C:
            step = ra_type2_n_rb_step(nof_prb)
            nof_vrb //= step
            L, s = type2_from_riv(d["riv"], nof_vrb, nof_vrb)
            L, s = L * step, s * step
        else:
            L, s = type2_from_riv(d["riv"], nof_prb, nof_vrb)
        if d["mode"] == 0:
            for i in range(L):
                if i + s < nof_prb:
                    prb[0, i + s] = 1
            prb[1] = prb[0]
        else:
            if d["n_gap"] == 0:
                Nt, Ng = ra_type2_n_vrb_dl(nof_prb, True), ra_type2_ngap(nof_prb, True)
            else:
                Nt, Ng = 2 * ra_type2_n_vrb_dl(nof_prb, True), ra_type2_ngap(nof_prb, False)
            Nrow = int(math.ceil(Nt / (4 * P))) * P
            Nnull = 4 * Nrow - Nt
            for i in range(L):
                nv = i + s
                ntv = nv % Nt
                ntp = 2 * Nrow * (ntv % 2) + ntv // 2 + Nt * (nv // Nt)
                nt2 = Nrow * (ntv % 4) + ntv // 4 + Nt * (nv // Nt)
                if Nnull != 0 and ntv >= Nt - Nnull and ntv % 2 == 1:
                    odd = ntp - Nrow
                elif Nnull != 0 and ntv >= Nt - Nnull and ntv % 2 == 0:
                    odd = ntp - Nrow + Nnull // 2
                elif Nnull != 0 and ntv < Nt - Nnull and ntv % 4 >= 2:
                    odd = nt2 - Nnull // 2
                else:
                    odd = nt2
                even = (odd + Nt // 2) % Nt + Nt * (nv // Nt)
                for slot, v in ((0, odd), (1, even)):
                    k = v if v < Nt // 2 else v + Ng - Nt // 2
                    if k >= nof_prb:
                        return None
                    prb[slot, k] = 1
    return prb


def dci_to_grant(d, nof_prb, nof_ports, tm, tbs_alt=False):
    """srslte_ra_dl_dci_to_grant (ra_dl.c:608-645), FDD normal subframes: dict(prb, tbs list, qm list, rv list,
    tx_scheme, nof_layers, pmi) or None.  tm: 0 = TM1 ... 3 = TM4."""
    prb = prb_allocation(d, nof_prb)
    if prb is None:
        return None
    tbs_t, f1c = tbs_table()
    nprb = int(prb[0].sum())
    tbs, qm, rv, en = [0, 0], [2, 2], [d["tb"][0]["rv"], d["tb"][1]["rv"]], [False, False]
    for i in range(2):
        en[i] = (tb_enabled(d["tb"][i]) and d["format"] >= FORMAT2) or (d["format"] < FORMAT2 and i == 0)
    nof_tb = sum(en)
    if not is_user(d["rnti"]) and d["rnti"] != MRNTI:
        if d["format"] == FORMAT1A:
            tbs[0] = int(tbs_t[d["tb"][0]["mcs_idx"], (3 if d["n_prb1a"] else 2) - 1]) if d["tb"][0]["mcs_idx"] < 34 else -1
        elif d["format"] == FORMAT1C:
            tbs[0] = int(f1c[d["tb"][0]["mcs_idx"]])
        else:
            return None
        qm[0] = 2
    else:
        for i in range(2):
            if en[i]:
                qm[i] = mod_from_mcs(d["tb"][i]["mcs_idx"], tbs_alt)
                it = tbs_idx_from_mcs(d["tb"][i]["mcs_idx"], tbs_alt)
                if it < 0:
                    return None  # last_tbs not tracked by the oracle
                tbs[i] = int(tbs_t[it, nprb - 1])
    if d["format"] == FORMAT1C and (is_rar(d["rnti"]) or d["rnti"] == PRNTI):
        rv = [0, 0]
    # config_mimo (ra_dl.c:448-606)
    if tm in (0, 1):
        scheme = 1 if nof_ports > 1 else 0
        if nof_tb != 1:
            return None
    elif tm == 2:
        scheme = 1 if nof_tb == 1 else 3
    elif tm == 3:
        scheme = (1 if d["pinfo"] == 0 else 2) if nof_tb == 1 else 2
    else:
        scheme = 0  # TM5..8: "not implemented" is only logged, the scheme stays port 0 (ra_dl.c:489-499)
    pmi = 0
    if scheme == 2:
        if nof_tb == 1:
            if not 0 < d["pinfo"] < 5:
                return None
            pmi = d["pinfo"] - 1
        else:
            if d["pinfo"] >= 2:
                return None
            pmi = d["pinfo"] % 2
    if (scheme in (0, 1) and nof_tb != 1) or (scheme == 3 and nof_tb != 2):
        return None
    layers = {0: 1, 1: nof_ports, 2: nof_tb, 3: 2}[scheme]
    return dict(prb=prb, nof_prb=nprb, tbs=tbs, qm=qm, rv=rv, enabled=en, nof_tb=nof_tb, tx_scheme=scheme,
                nof_layers=layers, pmi=pmi, cw_idx=[d["tb"][0]["cw_idx"], d["tb"][1]["cw_idx"]])


# ------------------------------------------------------------------ blind search (ue_dl.c:420-730)

UE_FORMATS = {0: (FORMAT1A, FORMAT1), 1: (FORMAT1A, FORMAT1), 2: (FORMAT1A, FORMAT2A), 3: (FORMAT1A, FORMAT2)}
COMMON_FORMATS = (FORMAT1A, FORMAT1C)


def find_dl_dci(llr, nof_cce, sf_idx, rnti, nof_prb, nof_ports, tm=0, cfg=None, dci_common_ss=False):
    """srslte_ue_dl_find_dl_dci: list of (msg dict) in the reference's order; each msg has location, format,
    bits, and the unpacked 'dci'."""
    cfg = cfg or DciCfg()
    allocated, found = [], []

    def overlaps(L, n):
        # dci_location_is_allocated (ue_dl.c:436-448) as written: location.L is the level index (pdcch.c:270) and
        # serves as the width
        for (aL, an) in allocated:
            if (an <= n < an + aL) or (n <= an < n + L):
                return True
        return False

    def search(locs, formats, common):
        c = DciCfg(**vars(cfg))
        if common:
            c.is_not_ue_ss = True  # srslte_dci_cfg_set_common_ss (dci.c:1413-1416)
        out = []
        for (L, n) in locs:
            if overlaps(L, n):
                continue
            for f in formats:
                nb = dci_sizeof(f, nof_prb, nof_ports, c)
                ok, bits, crc = decode_candidate(llr, L, n, nb)
                if not ok or crc != rnti:
                    continue
                fmt = f
                if f in (FORMAT0, FORMAT1A):
                    fmt = FORMAT1A if bits[3 if c.cif_enabled else 0] else FORMAT0
                msg = dict(L=L, ncce=n, format=fmt, bits=bits, nof_bits=nb)
                if fmt == FORMAT0:
                    continue  # kept for the UL search only
                dup = any(m["nof_bits"] == nb and np.array_equal(m["bits"], bits) for m in found + out)
                if not dup:
                    allocated.append((L, n))
                    out.append(msg)
                    break
        return out

    if rnti in (SIRNTI, PRNTI) or is_rar(rnti):
        found += search(common_locations(nof_cce), COMMON_FORMATS, True)
    else:
        found += search(ue_locations(nof_cce, sf_idx, rnti), UE_FORMATS[tm], False)
        if dci_common_ss:
            found += search(common_locations(nof_cce), COMMON_FORMATS[:1], True)
    for m in found:
        m["dci"] = dci_unpack(m["bits"], m["format"], rnti, nof_prb, nof_ports, cfg)
    return found


# ------------------------------------------------------------------ transmitter (test synthesis)

def _qpsk(bits):
    b = np.asarray(bits, np.float32).reshape(-1, 2)
    return ((1 - 2 * b[:, 0]) + 1j * (1 - 2 * b[:, 1])).astype(np.complex64) / np.float32(np.sqrt(2))


def _precode_diversity(d, nof_ports):
    """srslte_layermap_diversity + srslte_precoding_diversity (36.211 6.3.3.3 / 6.3.4.3) -> (ports, n)"""
    n = d.size
    y = np.zeros((nof_ports, n), np.complex64)
    if nof_ports == 1:
        y[0] = d
        return y
    s = np.float32(1 / np.sqrt(2))
    if nof_ports == 2:
        x0, x1 = d[0::2], d[1::2]
        y[0, 0::2], y[1, 0::2] = s * x0, -s * np.conj(x1)
        y[0, 1::2], y[1, 1::2] = s * x1, s * np.conj(x0)
        return y
    x = [d[k::4] for k in range(4)]
    y[0, 0::4], y[2, 0::4] = s * x[0], -s * np.conj(x[1])
    y[0, 1::4], y[2, 1::4] = s * x[1], s * np.conj(x[0])
    y[1, 2::4], y[3, 2::4] = s * x[2], -s * np.conj(x[3])
    y[1, 3::4], y[3, 3::4] = s * x[3], s * np.conj(x[2])
    return y


def ctrl_tx(tx, rg: Regs, cell_id, nof_ports, sf_idx, cfi, msgs):
    """Writes PCFICH (cfi) and each PDCCH message (dict bits, rnti, L, ncce) into tx[port] grids."""
    c = oracle.sequence_lte((sf_idx + 1) * (2 * cell_id + 1) * 512 + cell_id, 32)
    w = [[0, 1, 1], [1, 0, 1], [1, 1, 0]][cfi - 1]
    bits = np.array([w[j % 3] for j in range(32)], np.uint8) ^ c
    y = _precode_diversity(_qpsk(bits), nof_ports)
    for p in range(nof_ports):
        tx[p].ravel()[rg.pcfich] = y[p]
    nregs = int(rg.nregs[cfi - 1])
    seq = oracle.sequence_lte(sf_idx * 512 + cell_id, 8 * nregs)
    for m in msgs:
        E = 72 << m["L"]
        e = np.zeros(E, np.uint8)
        b = np.ascontiguousarray(m["bits"], np.uint8)
        _lib().orc_pdcch_encode(b, b.size, m["rnti"], E, e)
        e ^= seq[72 * m["ncce"]: 72 * m["ncce"] + E]
        y = _precode_diversity(_qpsk(e), nof_ports)
        re = rg.pdcch[cfi - 1][36 * m["ncce"]: 36 * m["ncce"] + E // 2]
        for p in range(nof_ports):
            tx[p].ravel()[re] = y[p]
