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


def oracle_cfg(cell: P.Cell, nof_rx: int, tti: int, cfi: int, pcfg: P.PdschCfg) -> pc.Cfg:
    """The oracle chain's Cfg for a product PdschCfg (grant from the DCI, the UE's power / CSI / decoder fields)."""
    g = pcfg.grant
    tbs = [t for t in range(2) if g.tb[t].enabled]
    prb = np.array([[g.prb_idx[s][n] for n in range(cell.nof_prb)] for s in range(2)], np.uint8)
    return pc.Cfg(nof_prb=cell.nof_prb, nof_ports=cell.nof_ports, cell_id=cell.id, nof_rx=nof_rx, cfi=cfi,
                  sf_idx=tti % 10, rnti=pcfg.rnti, scheme=g.tx_scheme, nof_layers=g.nof_layers, pmi=g.pmi,
                  qm=[P.MOD_BITS[g.tb[t].mod] for t in tbs], tbs=[g.tb[t].tbs for t in tbs],
                  rv=[g.tb[t].rv for t in tbs] + [0] * (2 - len(tbs)), prb=prb, csi_enable=bool(pcfg.csi_enable),
                  power_scale=bool(pcfg.power_scale), p_a=pcfg.p_a, p_b=pcfg.p_b,
                  mmse=pcfg.decoder_type == P.MIMO_DECODER_MMSE)


def llr_spot_check(rx, k: int, ocfg: pc.Cfg, payload_bytes: list, decoded_job: int | None = None):
    """Subframe k of a DlReceiver's last (single-chunk) call: the GPU's soft bits of every TB equal the oracle
    chain's (oracle/pdsch_chain.rx_front on the GPU's own grid, estimates and noise estimate) bit for bit, and their
    signs equal the codeword the transmitter sent (phy_dl_test.c check_softbits)."""
    import oracle
    from srsran_amd import lib
    G = 14 * 12 * ocfg.nof_prb

    def d2h(ptr):
        out = np.zeros(G, np.complex64)
        lib().mi355_memcpy_d2h(out.ctypes.data, ptr, out.nbytes)
        return out

    grids = np.stack([d2h(rx.grid_ptr(k, r)) for r in range(ocfg.nof_rx)])
    ces = np.stack([np.stack([d2h(rx.ce_ptr(k, p, r)) for r in range(ocfg.nof_rx)]) for p in range(ocfg.nof_ports)])
    if getattr(rx, "ce_rows", 0) == 1:  # row 0 only was written: the AVERAGE estimate of every OFDM symbol
        nre = 12 * ocfg.nof_prb
        ces = np.tile(ces[:, :, :nre], (1, 1, 14))
    noise = rx.chest[k].noise_estimate
    _d, _csi, e_o = pc.rx_front(ocfg, grids, ces, noise)
    j = k if decoded_job is None else decoded_job
    Nl = 2 if ocfg.nof_layers != ocfg.nof_tb else 1
    for t in range(ocfg.nof_tb):
        nbits = e_o[t].size
        nre = nbits // ocfg.qm[t]
        e_g = rx.ue.pdsch.stage(j, t, nre, nbits)[2]
        assert np.array_equal(e_g, e_o[t]), (k, t, int(np.abs(e_g.astype(np.int32) - e_o[t]).max()))
        bits = np.unpackbits(np.asarray(payload_bytes[t], np.uint8))[: ocfg.tbs[t]]
        coded = oracle.dlsch_encode_tb(bits, ocfg.tbs[t], ocfg.qm[t] * Nl, nbits, ocfg.rv[t])
        assert np.array_equal(e_g > 0, coded == 1), (k, t, int(np.sum((e_g > 0) != (coded == 1))))
        if getattr(rx, "last_bound", None) is not None and decoded_job is None:
            softbuffer_check(rx, rx.last_bound[2][k].softbuffer[t], e_o[t], ocfg.tbs[t], ocfg.qm[t] * Nl, ocfg.rv[t],
                             (k, t))


def softbuffer_check(rx, sb: int, e_o: np.ndarray, tbs: int, qm: int, rv: int, what=None):
    """The decoder buffers of softbuffer sb after a fresh-buffer decode (rate dematched by pdsch_eq_rm or
    dlsch_rm_rx) equal the oracle's rate dematching of the oracle's LLRs (orc_dlsch_rm_tb: rm_turbo_rx_lut into
    zeroed buffers), bit for bit over each code block's systematic, parity and tail positions."""
    import ctypes as C
    import oracle
    from srsran_amd import lib
    L = lib()
    buf, stride, mcb = C.POINTER(C.c_int16)(), C.c_uint32(), C.c_uint32()
    L.mi355_softbuffer_pool_buffer.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_int16)), C.POINTER(C.c_uint32),
                                               C.POINTER(C.c_uint32)]
    assert L.mi355_softbuffer_pool_buffer(rx.pool.h, C.byref(buf), C.byref(stride), C.byref(mcb)) == 0
    rx.pool.materialize(sb, 1)  # unwritten empty parity rows of fresh buffers -> the zeros they stand for
    seg = np.zeros(6, np.uint32)
    oracle.lib().orc_cbsegm(tbs, seg)
    Cn = int(seg[0])
    want = np.zeros(Cn * 18600, np.int16)
    e = np.ascontiguousarray(e_o, np.int16)
    assert oracle.lib().orc_dlsch_rm_tb(e, e.size, tbs, qm, rv, want, 18600) == Cn
    got = np.zeros((Cn, stride.value), np.int16)
    base = C.cast(buf, C.c_void_p).value + 2 * sb * mcb.value * stride.value
    L.mi355_memcpy_d2h(got.ctypes.data, base, got.nbytes)
    for c in range(Cn):
        K = int(seg[1]) if c < int(seg[3]) else int(seg[2])
        cols = (np.r_[0:K, K + 32:2 * K + 32, 2 * K + 64:3 * K + 64, 3 * K + 96:3 * K + 108]
                if oracle.lib().orc_tdec_nsb(K) else np.r_[0:3 * K + 12])  # sub-block layout or the natural one
        w = want[c * 18600:(c + 1) * 18600]
        assert np.array_equal(got[c, cols], w[cols]), (what, c, int(np.abs(got[c, cols].astype(np.int32) - w[cols]).max()))
