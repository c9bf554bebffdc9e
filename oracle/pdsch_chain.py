"""oracle.pdsch_chain -- TEST INFRASTRUCTURE ONLY.

* ``synth_subframe``: a transmitted + received PDSCH subframe (eNodeB side of pdsch_test.c,
  lib/src/phy/phch/test/pdsch_test.c): DL-SCH encode (oracle C), bit scrambling, 36.211 7.1 modulation,
  layer mapping (36.211 6.3.3) and precoding (6.3.4) for the schemes srslte_pdsch_decode supports,
  RE mapping in srslte_pdsch_put order, a per-RE channel H and AWGN.  Channel estimates = H (ideal, as
  pdsch_test.c does with its identity ce).
* ``rx_chain``: srslte_pdsch_decode restated over the oracle's C stages (pdsch.c:907-1072 and
  srslte_pdsch_codeword_decode :785-881): RE extraction, rho_b power allocation, equaliser with CSI,
  layer demapping, int16 demapper, descrambling, CSI weighting -> per-TB LLRs, then decode_tb.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import (Softbuffer, cbsegm, csi_correction_s, demod_soft_s, dlsch_decode_tb, dlsch_encode_tb, pdsch_c_init,
               pdsch_re_map, predecode, scramble_s, sequence_lte)

PORT0, DIVERSITY, SPATIALMUX, CDD = range(4)
CELL_SPECIFIC_RATIO = [[1.0, 4 / 5, 3 / 5, 2 / 5], [5 / 4, 1.0, 3 / 4, 1 / 2]]  # pdsch.c:44-46


@dataclass
class Cfg:
    nof_prb: int = 25
    nof_ports: int = 1
    cell_id: int = 1
    nof_rx: int = 1
    cfi: int = 2
    sf_idx: int = 3
    rnti: int = 0x1234
    scheme: int = PORT0
    nof_layers: int = 1
    pmi: int = 0
    qm: list = field(default_factory=lambda: [2])        # per TB
    tbs: list = field(default_factory=lambda: [1000])    # per TB
    rv: list = field(default_factory=lambda: [0, 0])
    prb: np.ndarray | None = None                        # (2, nof_prb)
    csi_enable: bool = False
    power_scale: bool = False
    p_a: float = 0.0
    p_b: int = 0
    mmse: bool = True

    @property
    def nof_tb(self):
        return len(self.tbs)

    @property
    def lstart(self):
        return self.cfi + (1 if self.nof_prb < 10 else 0)

    @property
    def grid_len(self):
        return 14 * 12 * self.nof_prb

    def prb_mask(self):
        return np.ones((2, self.nof_prb), np.uint8) if self.prb is None else np.asarray(self.prb, np.uint8)

    def codebook(self):
        return self.pmi if self.nof_tb == 1 else self.pmi + 1


def valid_tbs(target: int) -> int:
    """Largest TBS <= target (multiple of 8) segmenting like the 36.213 TBS tables do: no filler bits and
    a single code-block size (the reference's transmitter and receiver order mixed sizes differently)."""
    t = max(16, target - target % 8)
    while t > 16:
        s = cbsegm(t)
        if s["F"] == 0 and s["C2"] == 0:
            return t
        t -= 8
    return t


# ------------------------------------------------------------------ 36.211 7.1 modulation
def modulate(bits: np.ndarray, qm: int) -> np.ndarray:
    b = np.asarray(bits, np.int64).reshape(-1, qm)
    s = 1 - 2 * b
    if qm == 1:
        return ((s[:, 0] + 1j * s[:, 0]) / np.sqrt(2)).astype(np.complex64)
    if qm == 2:
        return ((s[:, 0] + 1j * s[:, 1]) / np.sqrt(2)).astype(np.complex64)
    if qm == 4:
        re = s[:, 0] * (2 - s[:, 2])
        im = s[:, 1] * (2 - s[:, 3])
        return ((re + 1j * im) / np.sqrt(10)).astype(np.complex64)
    if qm == 6:
        re = s[:, 0] * (4 - s[:, 2] * (2 - s[:, 4]))
        im = s[:, 1] * (4 - s[:, 3] * (2 - s[:, 5]))
        return ((re + 1j * im) / np.sqrt(42)).astype(np.complex64)
    if qm == 8:
        re = s[:, 0] * (8 - s[:, 2] * (4 - s[:, 4] * (2 - s[:, 6])))
        im = s[:, 1] * (8 - s[:, 3] * (4 - s[:, 5] * (2 - s[:, 7])))
        return ((re + 1j * im) / np.sqrt(170)).astype(np.complex64)
    raise ValueError(qm)


# ------------------------------------------------------------------ 36.211 6.3.3 / 6.3.4
def tx_scales(cfg: Cfg) -> tuple[np.float32, np.float32, np.float32]:
    """srslte_pdsch_encode's rho_a, applied whatever cfg.power_scale says (pdsch.c:1174-1188, :582), and the
    precoders' folded factors rho_a / sqrt(2) (diversity, codebook 0, one layer) and rho_a / 2 (codebooks 1-2,
    CDD) as precoding.c:1945-2200 rounds them (float32)."""
    amp = np.float64(np.float32(10.0) ** np.float32(cfg.p_a / 20.0))
    rho_a = np.float32(amp * (1.0 if cfg.nof_ports == 1 else np.sqrt(2.0)))
    s = rho_a if rho_a != 0 else np.float32(1.0)
    return s, np.float32(np.float64(s) * np.sqrt(0.5)), np.float32(s / np.float32(2.0))


def precode(d: list[np.ndarray], cfg: Cfg, ref_scaling: bool = False) -> np.ndarray:
    """codeword symbols -> per-port transmit symbols (nof_ports, nof_re).  ref_scaling: the reference
    transmitter's amplitudes (rho_a folded in, tx_scales); otherwise unit-power precoders (test channels)."""
    n = d[0].size
    if ref_scaling:
        s0, s1, s2 = tx_scales(cfg)
        m1 = lambda v: (v.real * s1 + 1j * (v.imag * s1)).astype(np.complex64)  # noqa: E731
        m2 = lambda v: (v.real * s2 + 1j * (v.imag * s2)).astype(np.complex64)  # noqa: E731
        if cfg.scheme == PORT0:
            x = d[0]
            return (x if s0 == 1 else (x.real * s0 + 1j * (x.imag * s0)).astype(np.complex64))[None, :].copy()
        if cfg.scheme == DIVERSITY:
            x0, x1 = d[0][0::2], d[0][1::2]
            y = np.zeros((2, n), np.complex64)
            y[0, 0::2], y[1, 0::2] = m1(x0), m1(-np.conj(x1))
            y[0, 1::2], y[1, 1::2] = m1(x1), m1(np.conj(x0))
            return y
        cb = cfg.codebook()
        if cfg.scheme == SPATIALMUX and cfg.nof_layers == 1:
            w1 = {0: 1, 1: -1, 2: 1j, 3: -1j}[cb]
            return np.stack([m1(d[0]), m1(w1 * d[0])]).astype(np.complex64)
        x0, x1 = d[0], d[1]
        if cfg.scheme == SPATIALMUX:
            if cb == 0:
                return np.stack([m1(x0), m1(x1)])
            if cb == 1:
                return np.stack([m2(x0 + x1), m2(x0 - x1)])
            return np.stack([m2(x0 + x1), m2(1j * (x0 - x1))])
        ev = (np.arange(n) % 2) == 0
        return np.stack([m2(x0 + x1), np.where(ev, m2(x0 - x1), m2(x1 - x0))])
    r2 = np.float32(np.sqrt(2.0))
    if cfg.scheme == PORT0:
        return d[0][None, :].copy()
    if cfg.scheme == DIVERSITY:
        assert cfg.nof_ports == 2
        x0, x1 = d[0][0::2], d[0][1::2]
        y = np.zeros((2, n), np.complex64)
        y[0, 0::2], y[1, 0::2] = x0 / r2, -np.conj(x1) / r2
        y[0, 1::2], y[1, 1::2] = x1 / r2, np.conj(x0) / r2
        return y
    cb = cfg.codebook()
    if cfg.scheme == SPATIALMUX and cfg.nof_layers == 1:
        w1 = {0: 1, 1: -1, 2: 1j, 3: -1j}[cb]
        return np.stack([d[0] / r2, w1 * d[0] / r2]).astype(np.complex64)
    x0, x1 = d[0], d[1]
    if cfg.scheme == SPATIALMUX:
        if cb == 0:
            return np.stack([x0 / r2, x1 / r2]).astype(np.complex64)
        if cb == 1:
            return np.stack([(x0 + x1) / 2, (x0 - x1) / 2]).astype(np.complex64)
        return np.stack([(x0 + x1) / 2, (1j * x0 - 1j * x1) / 2]).astype(np.complex64)
    # CDD (large delay, 2 layers): U and D(i) alternate the second port's sign pattern per RE
    ev = (np.arange(n) % 2) == 0
    y0 = (x0 + x1) / 2
    y1 = np.where(ev, (x0 - x1) / 2, (-x0 + x1) / 2)
    return np.stack([y0, y1]).astype(np.complex64)


@dataclass
class Subframe:
    y: np.ndarray         # (nof_rx, grid) complex64
    ce: np.ndarray        # (nof_ports, nof_rx, grid) complex64
    noise: float
    payload: list         # per TB packed bytes
    idx: np.ndarray       # RE map
    nof_re: int


def synth_subframe(cfg: Cfg, rng: np.random.Generator, snr_db: float = 30.0, channel: str = "block",
                   payload_bits: list | None = None) -> Subframe:
    idx = pdsch_re_map(cfg.nof_prb, cfg.nof_ports, cfg.cell_id, cfg.prb_mask(), cfg.lstart, cfg.sf_idx)
    nre = idx.size
    d, payload = [], []
    for t in range(cfg.nof_tb):
        qm, tbs = cfg.qm[t], cfg.tbs[t]
        Nl = 2 if cfg.nof_layers != cfg.nof_tb else 1
        bits = rng.integers(0, 2, tbs, dtype=np.uint8) if payload_bits is None else payload_bits[t]
        G = nre * qm
        coded = dlsch_encode_tb(bits, tbs, qm * Nl, G, cfg.rv[t])
        c = sequence_lte(pdsch_c_init(cfg.rnti, t, cfg.sf_idx, cfg.cell_id), G)
        d.append(modulate(coded ^ c, qm))
        payload.append(np.packbits(bits))
    tx = precode(d, cfg)
    G = cfg.grid_len
    if channel == "rayleigh":  # independent per RE (breaks the SFBC pair assumption)
        h = ((rng.standard_normal((cfg.nof_ports, cfg.nof_rx, G)) + 1j * rng.standard_normal(
            (cfg.nof_ports, cfg.nof_rx, G))) / np.sqrt(2)).astype(np.complex64)
    elif channel == "block":  # Rayleigh, constant over each PRB of each OFDM symbol
        hb = (rng.standard_normal((cfg.nof_ports, cfg.nof_rx, 14 * cfg.nof_prb)) + 1j * rng.standard_normal(
            (cfg.nof_ports, cfg.nof_rx, 14 * cfg.nof_prb))) / np.sqrt(2)
        h = np.repeat(hb, 12, axis=2).astype(np.complex64)
    elif channel == "static":  # Rayleigh, constant over each PRB and the whole subframe (row-invariant estimates)
        hb = (rng.standard_normal((cfg.nof_ports, cfg.nof_rx, cfg.nof_prb)) + 1j * rng.standard_normal(
            (cfg.nof_ports, cfg.nof_rx, cfg.nof_prb))) / np.sqrt(2)
        h = np.tile(np.repeat(hb, 12, axis=2), (1, 1, 14)).astype(np.complex64)
    else:
        h = np.ones((cfg.nof_ports, cfg.nof_rx, G), np.complex64)
    txg = np.zeros((cfg.nof_ports, G), np.complex64)
    txg[:, idx] = tx
    # rho_a / rho_b: transmitted amplitude of the PDSCH REs relative to the CRS (36.213 5.2)
    if cfg.power_scale:
        rho_a = np.float32(10 ** (cfg.p_a / 20) * (1 if cfg.nof_ports == 1 else np.sqrt(2)))
        rho_b = np.float32(np.sqrt(CELL_SPECIFIC_RATIO[0 if cfg.nof_ports == 1 else 1][cfg.p_b]))
        amp = np.full(14, rho_a, np.float32)
        if rho_b != 0 and rho_b != 1:
            for s in range(2):
                for l in (0, 4) + ((1,) if cfg.nof_ports == 4 else ()):
                    amp[s * 7 + l] = rho_a * rho_b
        txg *= np.repeat(amp, 12 * cfg.nof_prb)[None, :]
    sigma2 = 10 ** (-snr_db / 10)
    y = np.einsum("prg,pg->rg", h, txg)
    y += np.sqrt(sigma2 / 2) * (rng.standard_normal(y.shape) + 1j * rng.standard_normal(y.shape))
    return Subframe(y.astype(np.complex64), h, float(sigma2), payload, idx, nre)


def rho_b_mask(cfg: Cfg) -> tuple[np.ndarray, float]:
    """OFDM symbols divided by rho_b (apply_power_allocation, pdsch.c:575-611) and pdsch_scaling (rho_a)."""
    if not cfg.power_scale:
        return np.ones(14, np.float32), 1.0
    rho_a = np.float32(np.float64(np.float32(10.0) ** np.float32(cfg.p_a / 20.0)) *
                       (1.0 if cfg.nof_ports == 1 else np.sqrt(2.0)))
    rho_b = np.sqrt(np.float32(CELL_SPECIFIC_RATIO[0 if cfg.nof_ports == 1 else 1][cfg.p_b]), dtype=np.float32)
    sc = np.ones(14, np.float32)
    if rho_b != 0 and rho_b != 1:
        inv = np.float32(1.0) / rho_b
        for s in range(2):
            for l in (0, 4) + ((1,) if cfg.nof_ports == 4 else ()):
                sc[s * 7 + l] = inv
    scaling = float(rho_a) if (rho_a != 0 and np.isfinite(rho_a)) else 1.0
    return sc, scaling


def rx_front(cfg: Cfg, y: np.ndarray, ce: np.ndarray, noise: float, predecoder=None):
    """Everything of srslte_pdsch_decode up to the DL-SCH: returns (d[cw], csi[cw], e[tb]).  predecoder replaces the
    oracle's equaliser (oracle.ref_predecode_scalar: the compiled reference's scalar path, tests only)."""
    idx = pdsch_re_map(cfg.nof_prb, cfg.nof_ports, cfg.cell_id, cfg.prb_mask(), cfg.lstart, cfg.sf_idx)
    nre = idx.size
    sc, scaling = rho_b_mask(cfg)
    row = 12 * cfg.nof_prb
    ys = (y[:, idx] * sc[idx // row][None, :]).astype(np.complex64)
    hs = ce[:, :, idx]
    nz = noise if cfg.mmse else 0.0
    x, csi = (predecoder or predecode)(ys, hs, cfg.nof_layers, cfg.codebook(), cfg.scheme, scaling, nz)
    d = [np.zeros(nre, np.complex64), np.zeros(nre, np.complex64)]
    if cfg.scheme == DIVERSITY:
        L = cfg.nof_layers
        m = x.shape[1]
        for l in range(L):
            d[0][l:L * m:L] = x[l]
        if cfg.nof_ports == 4:  # quads past m_ap are not equalised (left zero)
            m_ap = ((nre - 2) // 4) if nre % 4 else nre // 4
            d[0][4 * m_ap:] = 0
            csi[0][4 * m_ap:] = 0
    else:
        for l in range(cfg.nof_layers):
            d[l] = x[l]
    e = []
    for t in range(cfg.nof_tb):
        qm = cfg.qm[t]
        cw = t
        llr = demod_soft_s(qm, d[cw])
        llr = scramble_s(pdsch_c_init(cfg.rnti, cw, cfg.sf_idx, cfg.cell_id), llr[:nre * qm])
        if cfg.csi_enable:
            llr = csi_correction_s(qm, llr, csi[cw][:nre])
        e.append(llr)
    return d, csi, e


def rx_decode(cfg: Cfg, e: list[np.ndarray], sbs: list[Softbuffer], max_its: int = 10):
    out = []
    Nl = 2 if cfg.nof_layers != cfg.nof_tb else 1
    for t in range(cfg.nof_tb):
        ret, data, its = dlsch_decode_tb(e[t], cfg.tbs[t], cfg.qm[t] * Nl, cfg.rv[t], max_its, sbs[t])
        out.append((ret, data, its))
    return out
