"""GPU: the multipath fading test channel of the generator (mi355_channel_fading_grid_batch) --
srslte_channel_fading_t (lib/src/phy/channel/fading.c) evaluated per OFDM symbol in the resource grid.

Pinned pieces:
* the Jakes phases are the reference's own draws: std::mt19937(seed + link) through
  std::uniform_real_distribution<float>(0, 2 pi), tap-major, a before b (fading.c:236-245, random.cpp:32-39).  They
  are restated here with a pure-Python MT19937 (checked against the C++ standard's known answer, [rand.predef]:
  the 10000th output of a default-seeded mt19937 is 4123659995) and libstdc++'s generate_canonical<float, 24>
  (one 32-bit draw converted to float, divided by 2^32, clamped below 1, times (b - a));
* taps, powers (36.104 B.2, fading.c:33-46), alpha = pi (i - 1/2) / (2 ntaps) per tap (fading.c:244) and the gain
  sum of get_doppler_dispersion's generic branch (fading.c:143-152), restated in float64 numpy.  The SSE build of
  the reference reads a 1024-entry sine table instead of cos / sin: its gains differ from these by that
  quantisation, which no test here can pin (fading.c needs FFTW through srslte_dft and is not built here).
Grid-domain semantics (block fading per OFDM symbol, no path delay) are this framework's; the round trip checks that
the product's UE chain decodes through EPA fading.
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import pdsch_chain as pc
from srsran_amd import enb_dl
from srsran_amd import pdsch as P
from srsran_amd.tdec import DeviceBuffer
from tests.pdsch_jobs import cell_of, grant_of
from tests.test_enb_dl_gpu import dev_zeros, enb_job

pytestmark = pytest.mark.gpu

DELAY = {"none": [0], "epa": [0, 30, 70, 90, 110, 190, 410], "eva": [0, 30, 150, 310, 370, 710, 1090, 1730, 2510],
         "etu": [0, 50, 120, 200, 230, 500, 1600, 2300, 5000]}
POWER = {"none": [0.0], "epa": [0.0, -1.0, -2.0, -3.0, -8.0, -17.2, -20.8],
         "eva": [0.0, -1.5, -1.4, -3.6, -0.6, -9.1, -7.0, -12.0, -16.9],
         "etu": [-1.0, -1.0, -1.0, 0.0, 0.0, 0.0, -3.0, -5.0, -7.0]}


def mt19937(seed: int, n: int) -> list[int]:
    mt = [seed & 0xFFFFFFFF]
    for i in range(1, 624):
        mt.append((1812433253 * (mt[-1] ^ (mt[-1] >> 30)) + i) & 0xFFFFFFFF)
    out, idx = [], 624
    for _ in range(n):
        if idx >= 624:
            for i in range(624):
                y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
                mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            idx = 0
        y = mt[idx]
        idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        out.append(y)
    return out


def uniform_2pi(raw: list[int]) -> np.ndarray:
    c = np.asarray(raw, np.float64).astype(np.float32) / np.float32(2.0 ** 32)
    c = np.minimum(c, np.nextafter(np.float32(1), np.float32(0)))
    return (c * (np.float32(2.0) * np.float32(np.pi))).astype(np.float32)


def ref_H(model: str, fd: float, seed: int, link: int, t_sf: float, nre: int) -> np.ndarray:
    """H[l, k] of one link: sum over taps of amp g(t_l) exp(-j 2 pi f_k tau)."""
    ntaps = len(DELAY[model])
    ph = uniform_2pi(mt19937(seed + link, ntaps * 32)).astype(np.float64).reshape(ntaps, 16, 2)
    k = np.arange(nre)
    f = (k - nre // 2 + (k >= nre // 2)) * 15e3
    t = t_sf + (np.arange(14) + 0.5) * (1e-3 / 14)
    H = np.zeros((14, nre), complex)
    for i in range(ntaps):
        amp = 10 ** (POWER[model][i] / 10)
        ca = np.cos(np.pi * (i - 0.5) / (2 * ntaps))
        w = np.pi * fd * ca * t[:, None]
        g = (np.cos(w + ph[i, :, 0]).sum(1) + 1j * np.sin(w + ph[i, :, 1]).sum(1)) * amp / 4
        H += g[:, None] * np.exp(-2j * np.pi * f * DELAY[model][i] * 1e-9)[None, :]
    return H


def test_mt19937_restatement_known_answer():
    assert mt19937(5489, 10000)[-1] == 4123659995


@pytest.mark.parametrize("model,fd,nof_ports,nof_rx,seed", [("epa", 70.0, 1, 1, 17), ("eva", 5.0, 2, 2, 3),
                                                            ("etu", 300.0, 2, 1, 99), ("none", 0.0, 1, 2, 0)])
def test_fading_matches_restatement(model, fd, nof_ports, nof_rx, seed):
    nof_prb = 25
    nre, G = 12 * nof_prb, 14 * 12 * nof_prb
    enb = enb_dl.EnbDl(P.make_cell(nof_prb, nof_ports, 1))
    rng = np.random.default_rng(seed)
    t_sf = [0.0, 0.001, 0.4567]
    n = len(t_sf)
    tx = [(rng.standard_normal(G) + 1j * rng.standard_normal(G)).astype(np.complex64) for _ in range(n * nof_ports)]
    d_tx = [DeviceBuffer(G * 8).upload(t) for t in tx]
    d_rx = [dev_zeros(G * 8) for _ in range(n * nof_rx)]
    mstr = f"{model}{fd:g}"
    enb.fading([t.ptr for t in d_tx], [r.ptr for r in d_rx], nof_rx, mstr, t_sf, 0.0, seed)
    for i in range(n):
        for r in range(nof_rx):
            want = np.zeros((14, nre), complex)
            for p in range(nof_ports):
                H = ref_H(model, fd, seed, r * nof_ports + p, t_sf[i], nre)
                want += H * tx[i * nof_ports + p].reshape(14, nre)
            got = d_rx[i * nof_rx + r].download(np.zeros(G, np.complex64)).reshape(14, nre)
            rms = np.sqrt(np.mean(np.abs(want) ** 2))
            assert np.abs(got - want).max() <= 2e-5 * rms * len(DELAY[model]), (i, r, np.abs(got - want).max() / rms)
    if model == "none":  # one tap: flat in frequency; fd = 0: constant in time
        got = d_rx[0].download(np.zeros(G, np.complex64)).reshape(14, nre) / tx[0].reshape(14, nre)
        assert np.allclose(got, got[0, 0], rtol=1e-4)


def test_fading_rejects_invalid_models():
    enb = enb_dl.EnbDl(P.make_cell(6, 1, 1))
    G = 14 * 72
    d = [dev_zeros(G * 8) for _ in range(2)]
    for bad in ("abc5", "epa", "none", "xyz"):
        with pytest.raises(RuntimeError):
            enb.fading([d[0].ptr], [d[1].ptr], 1, bad, [0.0], 0.0, 1)
    enb.fading([d[0].ptr], [d[1].ptr], 1, "epainf", [0.0], 0.0, 1)  # non-finite Doppler reads as 0 (fading.c:69-71)


def test_generator_round_trip_epa():
    """Device payloads -> GPU generator (2-port transmit diversity + CRS) -> EPA 5 Hz fading, 2 rx, 30 dB AWGN ->
    IFFT -> the product's UE chain: every TB decodes with its payload."""
    from srsran_amd.dlsch import SoftbufferPool
    from srsran_amd.ue_dl import DlSfJob, UeDl, default_chest_cfg, symbol_sz
    cfg0 = pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, cell_id=7, cfi=1, scheme=pc.DIVERSITY, nof_layers=2,
                  qm=[2], tbs=[2984])
    cell = cell_of(cfg0)
    N = symbol_sz(25)
    G = cfg0.grid_len
    enb = enb_dl.EnbDl(cell)
    ue = UeDl(cell, 2)
    rng = np.random.default_rng(5)
    sfs = [1, 2, 3, 4]
    nsf = len(sfs)
    pls, d_pl, tx, rx, iq, jobs = [], [], [], [], [], []
    for i in range(nsf):
        cfg = pc.Cfg(**{**cfg0.__dict__, "sf_idx": sfs[i]})
        pl = [rng.integers(0, 256, t // 8, dtype=np.uint8) for t in cfg.tbs]
        pls.append(pl)
        d_pl.append([DeviceBuffer(p.nbytes).upload(p) for p in pl])
        tx.append([dev_zeros(G * 8) for _ in range(2)])
        rx.append([dev_zeros(G * 8) for _ in range(2)])
        iq.append([dev_zeros(15 * N * 8) for _ in range(2)])
        jobs.append(enb_job(cfg, d_pl[i], tx[i]))
    enb.put_pdsch(jobs)
    enb.put_refs(sfs, [g.ptr for t in tx for g in t])
    sigma = float(np.sqrt(10 ** (-30 / 10) / 2))
    enb.fading([g.ptr for t in tx for g in t], [g.ptr for r in rx for g in r], 2, "epa5", [1e-3 * s for s in sfs],
               sigma, 1234)
    enb.gen_signal([g.ptr for r in rx for g in r], [g.ptr for s in iq for g in s])
    grids = [[dev_zeros(G * 8) for _ in range(2)] for _ in range(nsf)]
    ces = [[[dev_zeros(G * 8) for _ in range(2)] for _ in range(2)] for _ in range(nsf)]
    outs = [DeviceBuffer(cfg0.tbs[0] // 8 + 16) for _ in range(nsf)]
    pool = SoftbufferPool(2 * nsf, max_cb=4)
    sjobs, sfcfgs, pcfgs, pays = [], [], [], []
    for i in range(nsf):
        cfg = pc.Cfg(**{**cfg0.__dict__, "sf_idx": sfs[i]})
        j = DlSfJob()
        j.tti = sfs[i]
        for r in range(2):
            j.in_buffer[r] = iq[i][r].ptr
            j.sf_symbols[r] = grids[i][r].ptr
            for p in range(2):
                j.ce[p][r] = ces[i][p][r].ptr
        sjobs.append(j)
        sfcfgs.append(P.DlSfCfg(sfs[i], 1))
        pc_ = P.PdschCfg()
        pc_.grant = grant_of(cfg)
        pc_.rnti = cfg.rnti
        pc_.decoder_type = P.MIMO_DECODER_MMSE
        pc_.softbuffer[0], pc_.softbuffer[1] = 2 * i, 2 * i + 1
        pcfgs.append(pc_)
        pays += [outs[i].ptr, 0]
    _, res = ue.decode(pool, sjobs, sfcfgs, pcfgs, default_chest_cfg(), pays)
    for i in range(nsf):
        assert res[2 * i].ret == 0 and res[2 * i].crc, i
        got = outs[i].download(np.zeros(cfg0.tbs[0] // 8 + 16, np.uint8))[: cfg0.tbs[0] // 8]
        np.testing.assert_array_equal(got, pls[i][0])
