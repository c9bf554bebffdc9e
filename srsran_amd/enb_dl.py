"""Python mirror of include/srsran_amd/enb_dl.h -- host PDSCH transmit chain (srslte_pdsch_encode) and CRS
mapping, used to synthesise decodable subframes for the benchmark."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import check
from .pdsch import Cell, DlSfCfg, PdschCfg, _declare as _declare_pdsch


def _declare():
    L = _declare_pdsch()
    if getattr(L, "_enb_declared", False):
        return L
    L.mi355_pdsch_encode_host.argtypes = [C.POINTER(Cell), C.POINTER(DlSfCfg), C.POINTER(PdschCfg),
                                          C.c_void_p * 2, C.c_void_p * 4]
    L.mi355_refsignal_cs_put_sf_host.argtypes = [C.POINTER(Cell), C.c_uint32, C.c_void_p * 4]
    L._enb_declared = True
    return L


def pdsch_encode(cell: Cell, sf: DlSfCfg, cfg: PdschCfg, payloads: list[np.ndarray], grids: np.ndarray) -> None:
    """grids: (nof_ports, nsymb*2*12*nof_prb) complex64, written in place (PDSCH REs)."""
    L = _declare()
    assert grids.dtype == np.complex64 and grids.flags.c_contiguous
    data = (C.c_void_p * 2)()
    keep = []
    for t in range(2):
        if t < len(payloads) and payloads[t] is not None:
            a = np.ascontiguousarray(payloads[t], np.uint8)
            keep.append(a)
            data[t] = a.ctypes.data
    g = (C.c_void_p * 4)()
    for p in range(grids.shape[0]):
        g[p] = grids[p].ctypes.data
    check(L.mi355_pdsch_encode_host(C.byref(cell), C.byref(sf), C.byref(cfg), data, g), "pdsch_encode_host")


def put_refs(cell: Cell, tti: int, grids: np.ndarray) -> None:
    L = _declare()
    g = (C.c_void_p * 4)()
    for p in range(grids.shape[0]):
        g[p] = grids[p].ctypes.data
    check(L.mi355_refsignal_cs_put_sf_host(C.byref(cell), tti, g), "refsignal_cs_put_sf_host")
