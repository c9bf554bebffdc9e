"""oracle.ue_dl_chain -- TEST INFRASTRUCTURE ONLY.

The UE downlink front-end restated for parity tests:
  * ``ofdm_rx_sf``: srslte_ofdm_rx_sf (lib/src/phy/dft/ofdm.c:392-471) as a float64 DFT (numpy) of each OFDM
    symbol after its cyclic prefix, FFT-shifted without DC, no normalisation (ue_dl.c:93).  The reference
    uses FFTW (not vendored); the DFT is its mathematical definition, so parity is a float tolerance.
  * ``ofdm_tx_sf``: the inverse (srslte_ofdm_tx_sf semantics) for synthesising time-domain subframes.
  * ``crs_put``: srslte_refsignal_cs_put_sf (refsignal_dl.c:262-283) with the oracle's CRS table.
  * ``chest_estimate``: srslte_chest_dl_estimate_cfg over orc_chest_estimate_port (oracle/orc_chest.c) plus
    fill_res (chest_dl.c:944-972), AVERAGE estimator / REFS noise.
  * ``synth_iq``: a PDSCH subframe (pdsch_chain.synth) with CRS on every port, a time-invariant
    frequency-selective channel and AWGN, returned as time-domain I/Q per rx antenna.
"""
from __future__ import annotations

import math

import numpy as np

from . import f32p, lib, pdsch_re_map  # noqa: F401
from . import pdsch_chain as pc

LIM = (6, 15, 25, 50, 75, 110)


def symbol_sz(nof_prb: int, std: bool = False) -> int:
    """srslte_symbol_sz (phy_common.c:353-380)."""
    ns = (128, 256, 384, 768, 1024, 1536) if not std else (128, 256, 512, 1024, 1536, 2048)
    for lim, n in zip(LIM, ns):
        if nof_prb <= lim:
            return n
    raise ValueError(nof_prb)


def cp_len(N: int, c: int) -> int:
    return int(math.ceil(np.float32(c) * N / np.float32(2048.0)))


def layout(nof_prb: int, cp_ext: bool = False, std: bool = False):
    N = symbol_sz(nof_prb, std)
    nsymb = 6 if cp_ext else 7
    if cp_ext:
        cp0 = cp1 = cp_len(N, 512)
    else:
        cp0, cp1 = cp_len(N, 160), cp_len(N, 144)
    return N, nsymb, cp0, cp1, N * 15 // 2


def ofdm_rx_sf(iq: np.ndarray, nof_prb: int, cp_ext: bool = False, std: bool = False) -> np.ndarray:
    N, nsymb, cp0, cp1, slot = layout(nof_prb, cp_ext, std)
    nre = 12 * nof_prb
    out = np.zeros((2 * nsymb, nre), np.complex64)
    x = np.asarray(iq, np.complex128)
    for s in range(2 * nsymb):
        sl, l = divmod(s, nsymb)
        off = sl * slot + cp0 + l * (N + cp1)
        X = np.fft.fft(x[off:off + N])
        out[s, : nre // 2] = X[N - nre // 2:]
        out[s, nre // 2:] = X[1: nre // 2 + 1]
    return out.reshape(-1)


def ofdm_tx_sf(grid: np.ndarray, nof_prb: int, cp_ext: bool = False, std: bool = False) -> np.ndarray:
    N, nsymb, cp0, cp1, slot = layout(nof_prb, cp_ext, std)
    nre = 12 * nof_prb
    g = np.asarray(grid).reshape(2 * nsymb, nre)
    out = np.zeros(N * 15, np.complex128)
    for s in range(2 * nsymb):
        sl, l = divmod(s, nsymb)
        X = np.zeros(N, np.complex128)
        X[N - nre // 2:] = g[s, : nre // 2]
        X[1: nre // 2 + 1] = g[s, nre // 2:]
        t = np.fft.ifft(X)
        cp = cp0 if l == 0 else cp1
        start = sl * slot + (0 if l == 0 else cp0 + N + (l - 1) * (N + cp1))
        out[start: start + cp] = t[N - cp:]
        out[start + cp: start + cp + N] = t
    return out.astype(np.complex64)


def crs_pilots(nof_prb: int, cell_id: int, pair: int, sf: int, cp_ext: bool = False) -> np.ndarray:
    out = np.zeros(4 * 2 * nof_prb, np.complex64)
    lib().orc_crs_pilots(nof_prb, cell_id, int(cp_ext), pair, sf, out.view(np.float32))
    return out


def _crs_v(port, l):
    return {0: (0, 3), 1: (3, 0)}[port][l % 2] if port < 2 else (0 if (l == 0) == (port == 2) else 3)


def crs_positions(nof_prb: int, cell_id: int, port: int, cp_ext: bool = False):
    """(symbol, subcarrier) of each pilot in srslte_refsignal_cs_get_sf order."""
    nsymb = 6 if cp_ext else 7
    nsym = 4 if port < 2 else 2
    pos = []
    for l in range(nsym):
        s = ((l // 2 + 1) * nsymb - 3 if l % 2 else (l // 2) * nsymb) if port < 2 else 1 + l * nsymb
        f = (_crs_v(port, l) + cell_id % 6) % 6
        for i in range(2 * nof_prb):
            pos.append((s, f + 6 * i))
    return pos


def crs_put(tx: np.ndarray, nof_prb: int, cell_id: int, nof_ports: int, sf: int, cp_ext: bool = False):
    """tx: (nof_ports, grid) -- writes each port's CRS (srslte_refsignal_cs_put_sf)."""
    nre = 12 * nof_prb
    for p in range(nof_ports):
        pil = crs_pilots(nof_prb, cell_id, p // 2, sf, cp_ext)
        for k, (s, f) in enumerate(crs_positions(nof_prb, cell_id, p, cp_ext)):
            tx[p, s * nre + f] = pil[k]


def chest_estimate(grids: np.ndarray, nof_prb: int, nof_ports: int, cell_id: int, sf: int, filter_type: int = 0,
                   coef=(4.0, 1.0), cp_ext: bool = False, rsrp_neighbour: bool = False, alg: int = 0,
                   ce_init: np.ndarray | None = None):
    """grids: (nof_rx, grid).  alg: 0 AVERAGE, 1 INTERPOLATE.  ce_init: (nof_ports, nof_rx, grid) initial content of
    the estimate buffers (INTERPOLATE on ports 2, 3 copies their row 0).  Returns ce (nof_ports, nof_rx, grid) and
    the srslte_chest_dl_res_t scalars."""
    R = grids.shape[0]
    G = grids.shape[1]
    ce = np.zeros((nof_ports, R, G), np.complex64)
    vals = np.zeros((R, nof_ports, 3), np.float32)
    for a in range(R):
        g = np.ascontiguousarray(grids[a], np.complex64)
        for p in range(nof_ports):
            out = np.zeros(G, np.complex64) if ce_init is None else np.array(ce_init[p, a], np.complex64)
            o3 = np.zeros(3, np.float32)
            r = lib().orc_chest_estimate_port(g.view(np.float32), nof_prb, cell_id, int(cp_ext), sf, p, filter_type,
                                              float(coef[0]), float(coef[1]), alg, out.view(np.float32), o3)
            assert r == 0
            ce[p, a] = out
            vals[a, p] = o3
    return ce, fill_res(vals, nof_prb)


class ChestState:
    """The values srslte_chest_dl_t carries from one subframe to the next (chest_dl.c: q->cfo, q->noise_estimate,
    q->sync_err), zero after srslte_chest_dl_init."""

    def __init__(self, nof_rx: int, nof_ports: int):
        self.cfo = np.float32(0)
        self.noise = np.zeros((nof_rx, nof_ports), np.float32)
        self.sync = np.zeros((nof_rx, nof_ports), np.float32)


def chest_estimate_st(grids: np.ndarray, nof_prb: int, nof_ports: int, cell_id: int, tti: int, state: ChestState,
                      filter_type: int = 0, coef=(4.0, 1.0), alg: int = 0, noise_alg: int = 0, cfo_enable=False,
                      cfo_mask: int = 0, sync_enable=False, cp_ext: bool = False, std: bool = False):
    """srslte_chest_dl_estimate_cfg (chest_dl.c:985-1014) with the estimator's state, advanced by one subframe:
    per rx antenna the sync-error correction of the grid (:731-786, when enabled), then per port estimate_port
    (:788-816) -> chest_interpolate_noise_est (:621-728): the CFO (:596-618) where the mask selects the subframe,
    REFS noise before / PSS or EMPTY noise (subframes 0 and 5 only) after the interpolation.
    Returns (corrected grids, ce, res) -- res as chest_estimate's plus "cfo" and "sync_error"."""
    L = lib()
    R = grids.shape[0]
    G = grids.shape[1]
    sf = tti % 10
    N = symbol_sz(nof_prb, std)
    f32 = np.float32
    grids = np.array(grids, np.complex64)
    ce = np.zeros((nof_ports, R, G), np.complex64)
    vals = np.zeros((R, nof_ports, 3), np.float32)
    for a in range(R):
        g = grids[a]
        if sync_enable:
            se = np.zeros(nof_ports, np.float32)
            L.orc_chest_sync_correct(g.view(f32), nof_prb, cell_id, int(cp_ext), sf, nof_ports, N, se)
            state.sync[a, :] = se
        for p in range(nof_ports):
            out = np.zeros(G, np.complex64)
            o3 = np.zeros(3, np.float32)
            r = L.orc_chest_estimate_port_st(g.view(f32), nof_prb, cell_id, int(cp_ext), sf, p, filter_type,
                                             float(coef[0]), float(coef[1]), alg, noise_alg, float(state.noise[a, p]),
                                             out.view(f32), o3)
            assert r == 0
            if cfo_enable and (cfo_mask >> sf) & 1:
                state.cfo = f32(L.orc_chest_cfo(g.view(f32), nof_prb, cell_id, int(cp_ext), sf, p, p if p < 2 else 1,
                                                N))
            if noise_alg == 0:
                state.noise[a, p] = o3[0]
            elif sf in (0, 5):
                state.noise[a, p] = (L.orc_noise_pss(g.view(f32), out.view(f32), nof_prb, int(cp_ext), cell_id,
                                                     nof_ports) if noise_alg == 1
                                     else L.orc_noise_empty(g.view(f32), nof_prb, int(cp_ext)))
            ce[p, a] = out
            vals[a, p] = (state.noise[a, p], o3[1], o3[2])
    res = fill_res(vals, nof_prb)
    res["cfo"] = float(state.cfo)
    res["sync_error"] = float(state.sync[0, 0])
    return grids, ce, res


def fill_res(vals: np.ndarray, nof_prb: int) -> dict:
    """fill_res (chest_dl.c:944-972) incl. get_rsrp's rx-count-indexed port loop (:897-905)."""
    R, P = vals.shape[:2]
    f = np.float32
    noise, rsrp, rssi = vals[..., 0], vals[..., 1], vals[..., 2]
    n = f(0)
    for a in range(R):
        acc = f(0)
        for p in range(P):
            acc = f(acc + noise[a, p])
        n = f(n + f(acc / f(P)))
    n = f(n / f(R))

    def rsrp_port(port):
        if port >= P:
            return f(0)
        s = f(0)
        for j in range(R):
            s = f(s + rsrp[j, port])
        return f(s / f(R))

    rs = max(rsrp_port(i) for i in range(R))
    rq = f(0)
    ri = f(0)
    for a in range(R):
        rq = f(rq + f(f(nof_prb) * rsrp[a, 0] / rssi[a, 0]))
        ri = f(ri + f(f(f(f(4) * rssi[a, 0]) / f(nof_prb)) / f(12)))
    rq, ri = f(rq / f(R)), f(ri / f(R))
    db = lambda v: float(10 * np.log10(v))  # noqa: E731
    # a zero noise estimate (noiseless input) gives +inf dB (nan for 0/0), as the reference's float division does
    with np.errstate(divide="ignore", invalid="ignore"):
        snr = db(rs / n)
    return dict(noise_estimate=float(n), rsrp=float(rs), rsrq=float(rq), rssi_dbm=db(ri) + 30, snr_db=snr,
                noise=noise.copy(), rsrp_ant_port=rsrp.copy(), rssi_ant_port=rssi.copy())


def channel_freq(rng: np.random.Generator, nof_ports: int, nof_rx: int, nof_prb: int, ntaps: int = 3,
                 max_delay: int = 6, common_delays: bool = False) -> np.ndarray:
    """Time-invariant frequency-selective channel: per (port, rx) a few taps within the CP, as per-subcarrier
    gains (nof_ports, nof_rx, 12*nof_prb) in grid order (negative frequencies first).  common_delays: one delay
    profile for every (port, rx) pair (independent gains), as a physical array sees it."""
    nre = 12 * nof_prb
    N = symbol_sz(nof_prb)
    k = np.concatenate([np.arange(-nre // 2, 0), np.arange(1, nre // 2 + 1)])
    h = np.zeros((nof_ports, nof_rx, nre), np.complex128)
    d0 = np.sort(rng.integers(0, max_delay, ntaps)) if common_delays else None
    for p in range(nof_ports):
        for r in range(nof_rx):
            d = d0 if common_delays else np.sort(rng.integers(0, max_delay, ntaps))
            a = (rng.standard_normal(ntaps) + 1j * rng.standard_normal(ntaps)) / np.sqrt(2 * ntaps)
            for t in range(ntaps):
                h[p, r] += a[t] * np.exp(-2j * np.pi * k * d[t] / N)
    return h.astype(np.complex64)


def synth_iq(cfg: pc.Cfg, rng: np.random.Generator, snr_db: float = 30.0, payload_bits=None, max_delay: int = 6,
             channel: str = "taps", ctrl=None, common_delays: bool = False):
    """channel: "taps" (random taps up to max_delay samples) or "cross" (phy_dl_test's flat 2x2 [[1,1],[1,-1]]).
    ctrl: optional callable(tx) writing the control region (PCFICH / PDCCH) into the (ports, grid) tx grids.
    Returns (iq (nof_rx, N*15) complex64, payload bytes per TB, true per-subcarrier channel, noise var)."""
    idx = pdsch_re_map(cfg.nof_prb, cfg.nof_ports, cfg.cell_id, cfg.prb_mask(), cfg.lstart, cfg.sf_idx)
    nre = 12 * cfg.nof_prb
    G = 14 * nre
    # PDSCH part from the same generator as pdsch_chain (flat unit channel -> y == transmitted grid sum)
    d, payload = [], []
    Nl = 2 if cfg.nof_layers != cfg.nof_tb else 1
    for t in range(cfg.nof_tb):
        bits = rng.integers(0, 2, cfg.tbs[t], dtype=np.uint8) if payload_bits is None else payload_bits[t]
        Gb = idx.size * cfg.qm[t]
        coded = pc.dlsch_encode_tb(bits, cfg.tbs[t], cfg.qm[t] * Nl, Gb, cfg.rv[t])
        c = pc.sequence_lte(pc.pdsch_c_init(cfg.rnti, t, cfg.sf_idx, cfg.cell_id), Gb)
        d.append(pc.modulate(coded ^ c, cfg.qm[t]))
        payload.append(np.packbits(bits))
    tx = np.zeros((cfg.nof_ports, G), np.complex64)
    tx[:, idx] = pc.precode(d, cfg)
    crs_put(tx, cfg.nof_prb, cfg.cell_id, cfg.nof_ports, cfg.sf_idx)
    if ctrl is not None:
        ctrl(tx)
    if channel == "cross":
        w = np.array([[1, 1], [1, -1]], np.complex64)[: cfg.nof_ports, : cfg.nof_rx]
        h = np.repeat(w[:, :, None], nre, axis=2).astype(np.complex64)
    else:
        h = channel_freq(rng, cfg.nof_ports, cfg.nof_rx, cfg.nof_prb, max_delay=max_delay, common_delays=common_delays)
    sigma2 = 10 ** (-snr_db / 10)
    iq = []
    for r in range(cfg.nof_rx):
        y = np.zeros((14, nre), np.complex128)
        for p in range(cfg.nof_ports):
            y += tx[p].reshape(14, nre) * h[p, r][None, :]
        y += np.sqrt(sigma2 / 2) * (rng.standard_normal(y.shape) + 1j * rng.standard_normal(y.shape))
        iq.append(ofdm_tx_sf(y.reshape(-1), cfg.nof_prb))
    return np.stack(iq), payload, h, sigma2
