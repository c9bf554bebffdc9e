"""GPU parity of the estimator's state-carrying stages (include/srsran_amd/ue_dl.h, links) against the stateful
oracle chain (oracle/ue_dl_chain.py chest_estimate_st):
  * sync-error estimation and in-place grid correction (chest_dl.c:731-786): corrected grids within 1e-4 x RMS
    (the reference rotates with a recursive float phasor, the kernel with sincos), sync_error within 1e-3 samples;
  * CFO (chest_estimate_cfo :596-618, 4-port buffer quirk included) in the subframes cfo_estimate_sf_mask selects,
    held in the others: within 1e-5 + 1e-3 relative;
  * PSS / EMPTY noise (:399-430) updated only in subframes 0 and 5, the automatic Gauss sigma reading the previous
    estimate (PSS + automatic sigma takes the segmented launch): noise within 1e-3 relative, ce within 1e-4 x RMS;
  * two links interleaved in one batch, then the sequences continued in a second call (state carried across
    calls) -- each link equals its own sequential oracle run.
"""
import numpy as np
import pytest

from oracle import ue_dl_chain as uc
from srsran_amd import pdsch as P
from srsran_amd.tdec import DeviceBuffer
from srsran_amd.ue_dl import ChestCfg, DlSfJob, UeDl
from tests.chest_synth import synth_grids

pytestmark = pytest.mark.gpu

CASES = [  # nof_prb, ports, nrx, cell, alg, noise_alg, filter (type, coef), sync, cfo mask, delay, cfo
    (100, 2, 2, 1, 0, 0, (0, (4.0, 1.0)), True, 1023, 0.7, 0.004),     # srsUE default + sync correction
    (50, 2, 2, 150, 0, 2, (0, (0.0, 0.0)), False, 0b100001, 0.0, -0.01),  # EMPTY, automatic sigma
    (25, 4, 2, 4, 0, 1, (0, (0.0, 0.0)), True, 1023, -0.9, 0.02),      # PSS + automatic sigma: segmented
    (6, 1, 1, 301, 1, 1, (0, (4.0, 1.0)), True, 0b1010, 1.2, 0.0),     # INTERPOLATE, PSS, 6 PRB
    (15, 2, 1, 2, 1, 2, (1, (0.1, 0.0)), False, 0, 0.0, 0.01),         # triangle filter, EMPTY, CFO masked off
]


def _cfg(alg, noise_alg, filt, sync, mask):
    c = ChestCfg()
    c.estimator_alg, c.noise_alg, c.filter_type = alg, noise_alg, filt[0]
    c.filter_coef[0], c.filter_coef[1] = filt[1]
    c.sync_error_enable = int(sync)
    c.cfo_estimate_enable = int(mask != 0)
    c.cfo_estimate_sf_mask = mask
    return c


def _close(got, want, rel, ab=0.0):
    if np.isnan(want) or np.isnan(got):  # the automatic sigma of a zero state (before the first subframe 0/5) is NaN
        return bool(np.isnan(want) and np.isnan(got))
    return abs(got - want) <= rel * abs(want) + ab


def _max_err(got, want):
    nan_w, nan_g = np.isnan(want), np.isnan(got)
    assert np.array_equal(nan_w, nan_g)
    if nan_w.all():
        return 0.0, 1.0
    ok = ~nan_w
    return np.abs(got[ok] - want[ok]).max(), np.sqrt(np.mean(np.abs(want[ok]) ** 2))


@pytest.mark.parametrize("k", range(len(CASES)))
def test_chest_state_matches_oracle(k):
    nof_prb, ports, nrx, cid, alg, noise_alg, filt, sync, mask, delay, cfo = CASES[k]
    rng = np.random.default_rng(500 + k)
    G = 14 * 12 * nof_prb
    links = 2
    ttis = [list(range(3, 15)), list(range(7, 19))]  # per link: crosses subframes 5 and 0
    seqs = [[synth_grids(rng, nof_prb, ports, nrx, cid, t, delay=delay * (1 + 0.1 * l), cfo=cfo * (1 + 0.2 * l),
                         n0=2e-3 * (1 + (t % 4))) for t in ttis[l]] for l in range(links)]
    # oracle: each link on its own, in order
    want = []
    for l in range(links):
        st = uc.ChestState(nrx, ports)
        want.append([uc.chest_estimate_st(g, nof_prb, ports, cid, t, st, filter_type=filt[0], coef=filt[1], alg=alg,
                                          noise_alg=noise_alg, cfo_enable=mask != 0, cfo_mask=mask,
                                          sync_enable=sync) for g, t in zip(seqs[l], ttis[l])])
    ue = UeDl(P.make_cell(nof_prb, ports, cid), nrx)
    cfg = _cfg(alg, noise_alg, filt, sync, mask)
    n = len(ttis[0])
    order = [(i, l) for i in range(n) for l in range(links)]  # interleaved links
    halves = [order[:n], order[n:]]  # two calls: the state carries over
    for part in halves:
        bufs, jobs = [], []
        for (i, l) in part:
            gb = [DeviceBuffer(G * 8).upload(seqs[l][i][r]) for r in range(nrx)]
            cb = [[DeviceBuffer(G * 8) for _ in range(nrx)] for _ in range(ports)]
            j = DlSfJob()
            j.tti, j.link = ttis[l][i], l
            for r in range(nrx):
                j.sf_symbols[r] = gb[r].ptr
                for p in range(ports):
                    j.ce[p][r] = cb[p][r].ptr
            bufs.append((gb, cb))
            jobs.append(j)
        res = ue.chest(jobs, cfg)
        for q, (i, l) in enumerate(part):
            g_o, ce_o, r_o = want[l][i]
            gb, cb = bufs[q]
            tag = (k, i, l)
            for r in range(nrx):
                got = gb[r].download(np.zeros(G, np.complex64))
                rms = np.sqrt(np.mean(np.abs(g_o[r]) ** 2))
                assert np.abs(got - g_o[r]).max() <= 1e-4 * rms, tag
                for p in range(ports):
                    got = cb[p][r].download(np.zeros(G, np.complex64))
                    err, rms = _max_err(got, ce_o[p, r])
                    assert err <= 1e-4 * rms, (tag, p, r)
            x = res[q]
            assert _close(x.noise_estimate, r_o["noise_estimate"], 1e-3), (tag, x.noise_estimate, r_o["noise_estimate"])
            assert _close(x.cfo, r_o["cfo"], 1e-3, 1e-5), (tag, x.cfo, r_o["cfo"])
            assert _close(x.sync_error, r_o["sync_error"], 1e-3, 1e-3), (tag, x.sync_error, r_o["sync_error"])
            assert _close(x.rsrp, r_o["rsrp"], 1e-4), tag


def test_link_reset_and_bounds():
    ue = UeDl(P.make_cell(6, 1, 1), 1)
    ue.reset_link(0)
    ue.reset_link(65535)
    with pytest.raises(Exception):
        ue.reset_link(65536)
