"""Synthetic resource grids for the estimator-state tests (test infrastructure): CRS on every port, the PSS / SSS
region of subframes 0 and 5 (PSS on port 0 of the slot's last symbol, a random SSS stand-in on the symbol before,
the 5 subcarriers either side empty), QPSK data elsewhere, a frequency-selective channel per (port, rx), a timing
offset of `delay` samples (a linear phase over the subcarriers), a carrier offset of `cfo` subcarrier spacings (a
phase advancing with each OFDM symbol's start time) and complex AWGN of power `n0` per RE."""
import numpy as np

import oracle
from oracle import ue_dl_chain as uc


def pss_seq(cell_id: int) -> np.ndarray:
    out = np.zeros(62, np.complex64)
    oracle.lib().orc_pss_generate(cell_id % 3, out.view(np.float32))
    return out


def synth_grids(rng, nof_prb, nof_ports, nof_rx, cell_id, tti, delay=0.0, cfo=0.0, n0=1e-3, std=False, flat=False):
    nre = 12 * nof_prb
    G = 14 * nre
    sf = tti % 10
    tx = np.zeros((nof_ports, G), np.complex64)
    uc.crs_put(tx, nof_prb, cell_id, nof_ports, sf)
    data = ((rng.integers(0, 2, (G,)) * 2 - 1) + 1j * (rng.integers(0, 2, (G,)) * 2 - 1)) / np.sqrt(2)
    occupied = np.zeros(G, bool)
    for p in range(nof_ports):
        occupied |= tx[p] != 0
    # CRS positions of every port are left empty on the other ports (as the reference's RE map does)
    for p in range(4 if nof_ports > 1 else 1):
        for (s, f) in uc.crs_positions(nof_prb, cell_id, p):
            occupied[s * nre + f] = True
    tx[0, ~occupied] = data[~occupied]
    if sf in (0, 5):
        k_sss = 5 * nre + nre // 2 - 31
        k_pss = 6 * nre + nre // 2 - 31
        for k0 in (k_sss, k_pss):
            tx[:, k0 - 5:k0 + 67] = 0
        tx[0, k_pss:k_pss + 62] = pss_seq(cell_id)
        tx[0, k_sss:k_sss + 62] = (rng.integers(0, 2, 62) * 2 - 1).astype(np.complex64)
    h = np.ones((nof_ports, nof_rx, nre), np.complex64) if flat else uc.channel_freq(rng, nof_ports, nof_rx, nof_prb)
    N = uc.symbol_sz(nof_prb, std)
    ng = int(np.ceil(144 * N / 2048))
    kf = np.concatenate([np.arange(-nre // 2, 0), np.arange(1, nre // 2 + 1)])  # subcarrier index around DC
    ramp = np.exp(-2j * np.pi * kf * delay / N)
    tsym = np.arange(14) * (N + ng)
    rot = np.exp(2j * np.pi * cfo * tsym / N)
    grids = np.zeros((nof_rx, G), np.complex64)
    for r in range(nof_rx):
        y = sum(tx[p].reshape(14, nre) * h[p, r][None, :] for p in range(nof_ports))
        y = y * ramp[None, :] * rot[:, None]
        y = y + np.sqrt(n0 / 2) * (rng.standard_normal(y.shape) + 1j * rng.standard_normal(y.shape))
        grids[r] = y.reshape(-1)
    return grids
