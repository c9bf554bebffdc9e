"""CPU checks of the estimator-state restatements in oracle/orc_chest.c against independent float64 formulations
and against the physics they estimate (tests/chest_synth.py grids):
  * chest_dl_estimate_correct_sync_error (chest_dl.c:731-786): a timing offset of d samples is estimated as d and
    removed from the grid (a second pass finds < 0.05 samples, below the correction threshold);
  * chest_estimate_cfo (:596-618): a carrier offset of e subcarrier spacings is estimated as e;
  * estimate_noise_empty_sc (:419-430) and estimate_noise_pss (:399-416) equal their float64 formulations;
  * the stateful chain (oracle/ue_dl_chain.py chest_estimate_st): PSS / EMPTY noise and the CFO hold their value
    outside subframes 0 / 5 and outside cfo_estimate_sf_mask, as the reference's srslte_chest_dl_t does.
"""
import numpy as np
import pytest

import oracle
from oracle import ue_dl_chain as uc
from tests.chest_synth import pss_seq, synth_grids

F = np.float32


@pytest.mark.parametrize("nof_prb,ports,delay", [(100, 2, 0.8), (50, 1, -1.3), (25, 4, 0.6), (6, 2, 1.1)])
def test_sync_error_estimate_and_correction(nof_prb, ports, delay):
    rng = np.random.default_rng(1)
    g = synth_grids(rng, nof_prb, ports, 1, 7, 3, delay=delay, n0=1e-6, flat=True)[0]
    N = uc.symbol_sz(nof_prb)
    se = np.zeros(ports, F)
    oracle.lib().orc_chest_sync_correct(g.view(F), nof_prb, 7, 0, 3, ports, N, se)
    assert np.all(np.abs(se - delay) < 0.02), se
    se2 = np.zeros(ports, F)
    g2 = g.copy()
    oracle.lib().orc_chest_sync_correct(g2.view(F), nof_prb, 7, 0, 3, ports, N, se2)
    assert np.all(np.abs(se2) < 0.05), se2
    assert np.array_equal(g2, g)  # below the threshold: no correction


@pytest.mark.parametrize("nof_prb,ports,cfo", [(100, 2, 0.01), (50, 1, -0.03), (15, 2, 0.002)])
def test_cfo_estimate(nof_prb, ports, cfo):
    rng = np.random.default_rng(2)
    g = synth_grids(rng, nof_prb, ports, 1, 11, 1, cfo=cfo, n0=1e-6, flat=True)[0]
    N = uc.symbol_sz(nof_prb)
    est = oracle.lib().orc_chest_cfo(g.view(F), nof_prb, 11, 0, 1, ports - 1, ports - 1, N)
    assert abs(est - cfo) < 1e-3 * max(1.0, abs(cfo) * 100), (est, cfo)


def test_noise_empty_and_pss_formulas():
    rng = np.random.default_rng(3)
    for nof_prb, cid, ports in ((100, 1, 2), (25, 302, 1), (6, 5, 4)):
        nre = 12 * nof_prb
        g = synth_grids(rng, nof_prb, ports, 1, cid, 0, n0=0.01)[0]
        k_sss, k_pss = 5 * nre + nre // 2 - 31, 6 * nre + nre // 2 - 31
        want = sum(np.mean(np.abs(g[k:k + 5].astype(np.complex128)) ** 2)
                   for k in (k_sss - 5, k_sss + 62, k_pss - 5, k_pss + 62))
        got = oracle.lib().orc_noise_empty(g.view(F), nof_prb, 0)
        assert abs(got - want) <= 1e-5 * want
        # PSS: nof_ports * mean |ce * pss - y|^2 / sqrt(2) on the PSS subcarriers
        ce = (rng.standard_normal(g.size) + 1j * rng.standard_normal(g.size)).astype(np.complex64)
        seq = pss_seq(cid).astype(np.complex128)
        want = ports * np.mean(np.abs(ce[k_pss:k_pss + 62] * seq - g[k_pss:k_pss + 62]) ** 2) / np.sqrt(2)
        got = oracle.lib().orc_noise_pss(g.view(F), ce.view(F), nof_prb, 0, cid, ports)
        assert abs(got - want) <= 1e-5 * want


def test_pss_sequence_is_zadoff_chu():
    """36.211 6.11.1.1: d(n) = exp(-j pi u n(n+1)/63), n < 31; exp(-j pi u (n+1)(n+2)/63), n >= 31 -- within the
    reference's float argument rounding (pss.c:363-369 stores the phase, up to ~1000 rad, in a float)."""
    for nid2, u in enumerate((25, 29, 34)):
        n = np.arange(62)
        m = np.where(n < 31, n * (n + 1), (n + 1) * (n + 2))
        want = np.exp(-1j * np.pi * u * m / 63)
        assert np.abs(pss_seq(nid2) - want).max() < 5e-4


def test_state_holds_between_subframes():
    """PSS / EMPTY noise change only in subframes 0 and 5; the CFO only where the mask selects the subframe."""
    rng = np.random.default_rng(4)
    for noise_alg in (1, 2):
        st = uc.ChestState(1, 2)
        prev_noise, prev_cfo = None, None
        for tti in range(3, 14):
            g = synth_grids(rng, 25, 2, 1, 3, tti, cfo=0.01 * (tti % 3), n0=0.01 * (1 + tti))
            _g, _ce, res = uc.chest_estimate_st(g, 25, 2, 3, tti, st, noise_alg=noise_alg, cfo_enable=True,
                                                cfo_mask=0b100001)
            sf = tti % 10
            if prev_noise is not None and sf not in (0, 5):
                assert res["noise_estimate"] == prev_noise
            if prev_cfo is not None and sf not in (0, 5):
                assert res["cfo"] == prev_cfo
            if sf in (0, 5):
                assert res["noise_estimate"] > 0
            prev_noise, prev_cfo = res["noise_estimate"], res["cfo"]
