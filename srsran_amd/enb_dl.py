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


class EnbPdschJob(C.Structure):
    """mi355_enb_dl_pdsch_job_t: one srslte_enb_dl_put_pdsch call (device payloads and port grids)."""
    _fields_ = [("sf", DlSfCfg), ("cfg", PdschCfg), ("data", C.c_void_p * 2), ("sf_symbols", C.c_void_p * 4)]


def _declare_gpu():
    L = _declare()
    if getattr(L, "_enb_gpu_declared", False):
        return L
    vp, u32, i32 = C.c_void_p, C.c_uint32, C.c_int
    L.mi355_enb_dl_create.argtypes = [C.POINTER(vp), C.POINTER(Cell), i32]
    L.mi355_enb_dl_destroy.argtypes = [vp]
    L.mi355_enb_dl_put_pdsch_batch.argtypes = [vp, C.POINTER(EnbPdschJob), u32, vp]
    L.mi355_enb_dl_put_refs_batch.argtypes = [vp, C.POINTER(u32), C.POINTER(vp), u32, vp]
    L.mi355_enb_dl_gen_signal_batch.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), u32, vp]
    L.mi355_channel_grid_batch.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), u32, u32, C.POINTER(C.c_float),
                                           C.c_float, C.c_uint64, vp]
    L.mi355_channel_grid_batch_at.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), u32, u32, C.POINTER(C.c_float),
                                              C.c_float, C.c_uint64, C.c_uint64, vp]
    L.mi355_enb_synth_payloads.argtypes = [vp, vp, C.c_uint64, u32, u32, u32, C.c_uint64, vp]
    L.mi355_enb_payload_check.argtypes = [vp, vp, C.c_size_t, C.c_uint64, u32, u32, u32, C.c_uint64, vp, vp]
    L.mi355_channel_fading_grid_batch.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), u32, u32, C.c_char_p,
                                                  C.POINTER(C.c_double), C.c_float, u32, vp]
    L._enb_gpu_declared = True
    return L


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = (z + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_payloads_host(first_index: int, n: int, ntb: int, nbytes: int, seed: int) -> np.ndarray:
    """Host restatement of mi355_enb_synth_payloads (checks a sample of a large run): (n, ntb, nbytes) uint8."""
    words = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        it = (np.uint64(first_index) + np.arange(n, dtype=np.uint64))[:, None] << np.uint64(8)
        key = _splitmix64(it | np.arange(ntb, dtype=np.uint64)[None, :])  # (n, ntb)
        z = _splitmix64(np.uint64(seed) ^ (key[:, :, None] + np.arange(words, dtype=np.uint64)[None, None, :]))
    return z.astype("<u8").view(np.uint8).reshape(n, ntb, words * 8)[:, :, :nbytes].copy()


def _arr(t, v):
    return v if isinstance(v, C.Array) else (t * len(v))(*v)


class EnbDl:
    """srslte_enb_dl_t's PDSCH / CRS / IFFT path on one MI355X (mi355_enb_dl_*).  Pointer arguments are device
    addresses (ints, e.g. torch tensor data_ptr()); stream None: synchronous, else asynchronous on that HIP stream."""

    def __init__(self, cell: Cell, device: int = 0):
        self.L = _declare_gpu()
        h = C.c_void_p()
        check(self.L.mi355_enb_dl_create(C.byref(h), C.byref(cell), device), "enb_dl_create")
        self.h, self.cell, self.device = h, cell, device

    # every list argument may also be a prebuilt ctypes array of the same element type (no per-call conversion)
    def put_pdsch(self, jobs, stream=None):
        check(self.L.mi355_enb_dl_put_pdsch_batch(self.h, _arr(EnbPdschJob, jobs), len(jobs), stream),
              "enb_dl_put_pdsch")

    def put_refs(self, ttis, grids, stream=None):
        check(self.L.mi355_enb_dl_put_refs_batch(self.h, _arr(C.c_uint32, ttis), _arr(C.c_void_p, grids), len(ttis),
                                                 stream), "enb_dl_put_refs")

    def gen_signal(self, grids, out, stream=None):
        check(self.L.mi355_enb_dl_gen_signal_batch(self.h, _arr(C.c_void_p, grids), _arr(C.c_void_p, out), len(grids),
                                                   stream), "enb_dl_gen_signal")

    def channel(self, tx, rx, nof_rx: int, H: np.ndarray, sigma: float, seed: int, stream=None, first_index=None):
        """rx grids (nof_rx per job) = H (nof_rx x nof_ports complex) . tx grids (nof_ports per job) + AWGN; with
        first_index the noise of job i is keyed by the global subframe index first_index + i."""
        n = len(rx) // nof_rx
        h = np.ascontiguousarray(np.asarray(H, np.complex64)).view(np.float32).ravel()
        hf = (C.c_float * len(h))(*h.tolist())
        if first_index is None:
            check(self.L.mi355_channel_grid_batch(self.h, _arr(C.c_void_p, tx), _arr(C.c_void_p, rx), n, nof_rx, hf,
                                                  float(sigma), int(seed) & (2**64 - 1), stream), "channel_grid")
        else:
            check(self.L.mi355_channel_grid_batch_at(self.h, _arr(C.c_void_p, tx), _arr(C.c_void_p, rx), n, nof_rx,
                                                     hf, float(sigma), int(seed) & (2**64 - 1), int(first_index),
                                                     stream), "channel_grid_at")

    def synth_payloads(self, out: int, first_index: int, n: int, ntb: int, nbytes: int, seed: int, stream=None):
        """Device payloads of n subframes keyed by their global index (mi355_enb_synth_payloads)."""
        check(self.L.mi355_enb_synth_payloads(self.h, out, int(first_index), n, ntb, nbytes, int(seed) & (2**64 - 1),
                                              stream), "enb_synth_payloads")

    def payload_check(self, rx: int, rx_stride: int, first_index: int, n: int, ntb: int, nbytes: int, seed: int,
                      ok: int, stream=None):
        """ok[i * ntb + t] (device bytes) = 1 iff the decoded bytes at rx + (i * ntb + t) * rx_stride equal the payload
        synth_payloads made for subframe first_index + i, TB t (mi355_enb_payload_check; stream None: synchronous)."""
        check(self.L.mi355_enb_payload_check(self.h, rx, rx_stride, int(first_index), n, ntb, nbytes,
                                             int(seed) & (2**64 - 1), ok, stream), "enb_payload_check")

    def fading(self, tx, rx, nof_rx: int, model: str, t_sf, sigma: float, seed: int, stream=None):
        """Multipath fading (srslte_channel_fading_t: model "epa5", "eva70", "etu300", "none0" ...) + AWGN in the
        grid; job i's subframe starts at t_sf[i] seconds."""
        n = len(rx) // nof_rx
        ts = (C.c_double * max(n, 1))(*[float(t) for t in t_sf][:n])
        check(self.L.mi355_channel_fading_grid_batch(self.h, _arr(C.c_void_p, tx), _arr(C.c_void_p, rx), n, nof_rx,
                                                     model.encode(), ts, float(sigma), int(seed) & 0xFFFFFFFF,
                                                     stream), "channel_fading")

    def close(self):
        if getattr(self, "h", None):
            self.L.mi355_enb_dl_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
