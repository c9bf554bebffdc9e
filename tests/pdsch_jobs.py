"""Test helper: turn an oracle.pdsch_chain.Cfg + synthesized subframe into mi355_pdsch_job_t descriptors with the
grids resident in device memory (through the product's C ABI only)."""
from __future__ import annotations

import numpy as np

from oracle import pdsch_chain as pc
from srsran_amd import pdsch as P
from srsran_amd.tdec import DeviceBuffer


def cell_of(cfg: pc.Cfg) -> P.Cell:
    return P.make_cell(cfg.nof_prb, cfg.nof_ports, cfg.cell_id)


def grant_of(cfg: pc.Cfg) -> P.PdschGrant:
    cell = cell_of(cfg)
    tbs = [dict(qm=cfg.qm[t], tbs=cfg.tbs[t], rv=cfg.rv[t], cw_idx=t) for t in range(cfg.nof_tb)]
    return P.make_grant(cell, cfg.prb_mask(), cfg.cfi, cfg.sf_idx, cfg.scheme, cfg.nof_layers, tbs, pmi=cfg.pmi)


class DevSubframe:
    """Device copies of one subframe's grids + payload buffers (kept alive with the job)."""

    def __init__(self, cfg: pc.Cfg, sf: pc.Subframe, softbuffers=(0, 1), device: int = 0):
        self.cfg, self.sf = cfg, sf
        self.y = [DeviceBuffer(sf.y[r].nbytes, device).upload(sf.y[r]) for r in range(cfg.nof_rx)]
        self.ce = [[DeviceBuffer(sf.ce[p, r].nbytes, device).upload(np.ascontiguousarray(sf.ce[p, r]))
                    for r in range(cfg.nof_rx)] for p in range(cfg.nof_ports)]
        self.payload = [DeviceBuffer(t // 8 + 16, device) for t in cfg.tbs]
        self.job = P.PdschJob()
        j = self.job
        j.sf.tti, j.sf.cfi = cfg.sf_idx, cfg.cfi
        j.cfg.grant = grant_of(cfg)
        j.cfg.rnti = cfg.rnti
        j.cfg.max_nof_iterations = 0
        j.cfg.decoder_type = P.MIMO_DECODER_MMSE if cfg.mmse else P.MIMO_DECODER_ZF
        j.cfg.p_a, j.cfg.p_b, j.cfg.power_scale = cfg.p_a, cfg.p_b, int(cfg.power_scale)
        j.cfg.csi_enable = int(cfg.csi_enable)
        for t in range(2):
            j.cfg.softbuffer[t] = softbuffers[t] if t < len(softbuffers) else 0
        j.noise_estimate = sf.noise
        for r in range(cfg.nof_rx):
            j.sf_symbols[r] = self.y[r].ptr
            for p in range(cfg.nof_ports):
                j.ce[p][r] = self.ce[p][r].ptr
        for t in range(cfg.nof_tb):
            j.payload[t] = self.payload[t].ptr

    def payload_bytes(self, t: int) -> np.ndarray:
        out = np.zeros(self.cfg.tbs[t] // 8 + 16, np.uint8)
        return self.payload[t].download(out)


class DevIqSubframe:
    """Device buffers for one time-domain subframe through the ue_dl front-end: I/Q in, grid + ce out, and a
    PDSCH job over them (noise estimate filled in from the chest result with set_noise)."""

    def __init__(self, cfg: pc.Cfg, iq: np.ndarray, softbuffers=(0, 1), device: int = 0):
        from srsran_amd.ue_dl import DlSfJob
        self.cfg = cfg
        G = 14 * 12 * cfg.nof_prb
        self.iq = [DeviceBuffer(iq[r].nbytes, device).upload(np.ascontiguousarray(iq[r], np.complex64))
                   for r in range(cfg.nof_rx)]
        self.grid = [DeviceBuffer(G * 8, device) for _ in range(cfg.nof_rx)]
        self.ce = [[DeviceBuffer(G * 8, device) for _ in range(cfg.nof_rx)] for _ in range(cfg.nof_ports)]
        self.payload = [DeviceBuffer(t // 8 + 16, device) for t in cfg.tbs]
        self.sfjob = DlSfJob()
        self.sfjob.tti = cfg.sf_idx
        for r in range(cfg.nof_rx):
            self.sfjob.in_buffer[r] = self.iq[r].ptr
            self.sfjob.sf_symbols[r] = self.grid[r].ptr
            for p in range(cfg.nof_ports):
                self.sfjob.ce[p][r] = self.ce[p][r].ptr
        self.job = P.PdschJob()
        j = self.job
        j.sf.tti, j.sf.cfi = cfg.sf_idx, cfg.cfi
        j.cfg.grant = grant_of(cfg)
        j.cfg.rnti = cfg.rnti
        j.cfg.decoder_type = P.MIMO_DECODER_MMSE if cfg.mmse else P.MIMO_DECODER_ZF
        j.cfg.p_a, j.cfg.p_b, j.cfg.power_scale = cfg.p_a, cfg.p_b, int(cfg.power_scale)
        j.cfg.csi_enable = int(cfg.csi_enable)
        for t in range(2):
            j.cfg.softbuffer[t] = softbuffers[t] if t < len(softbuffers) else 0
        for r in range(cfg.nof_rx):
            j.sf_symbols[r] = self.grid[r].ptr
            for p in range(cfg.nof_ports):
                j.ce[p][r] = self.ce[p][r].ptr
        for t in range(cfg.nof_tb):
            j.payload[t] = self.payload[t].ptr

    def set_noise(self, noise: float):
        self.job.noise_estimate = noise

    def grids(self) -> np.ndarray:
        G = 14 * 12 * self.cfg.nof_prb
        return np.stack([b.download(np.zeros(G, np.complex64)) for b in self.grid])

    def ces(self) -> np.ndarray:
        G = 14 * 12 * self.cfg.nof_prb
        return np.stack([np.stack([b.download(np.zeros(G, np.complex64)) for b in row]) for row in self.ce])

    def payload_bytes(self, t: int) -> np.ndarray:
        out = np.zeros(self.cfg.tbs[t] // 8 + 16, np.uint8)
        return self.payload[t].download(out)
