"""GPU: the Wiener DL estimator (mi355_wiener_dl_*, srsran_amd/csrc/wiener_kernels.hip) against its CPU restatement
oracle/orc_wiener.cpp on identical inputs: three links interleaved in a batch (each its own srslte_wiener_dl_t),
several subframes of a link in one call and across calls, 1/2 ports x 1/2 rx, 6..100 PRB.  Both sides evaluate the
same float operations in the same order (-ffp-contract=off), so the Wiener rows agree to float rounding of the
transcendental-free path (checked at 1e-5 relative RMS, bit-exact in practice) and the ready flags and sub-band draw
counts are equal."""
import numpy as np
import pytest

from oracle import wiener_chain as wc
from srsran_amd.wiener import WienerDl

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nof_prb,ntx,nrx", [(25, 2, 2), (6, 1, 1), (100, 2, 2), (15, 1, 2)])
def test_wiener_matches_oracle(nof_prb, ntx, nrx):
    rng = np.random.default_rng(100 + nof_prb)
    nl, nsf = 3, 8
    data = [wc.synth_pilots(rng, nof_prb, ntx, nrx, nsf, snr_db=snr) for snr in (12.0, 20.0, 30.0)]
    shift = [wc.crs_shift(7, p) for p in range(ntx)]
    gpu = WienerDl(nof_prb, ntx, nrx, nl)
    refs = [wc.Wiener(nof_prb, ntx, nrx) for _ in range(nl)]
    # calls of 2 subframes per link, links interleaved inside each call
    worst, nready = 0.0, 0
    for s0 in range(0, nsf, 2):
        links = [l for s in (s0, s0 + 1) for l in range(nl)]
        pil = np.stack([data[l][0][s] for s in (s0, s0 + 1) for l in range(nl)])
        snr = np.stack([data[l][1][s] for s in (s0, s0 + 1) for l in range(nl)])
        ce, ready, _ = gpu.run(links, pil, snr, shift)
        for j, (l, s) in enumerate([(l, s) for s in (s0, s0 + 1) for l in range(nl)]):
            ce_o, rd_o, _ = refs[l].subframe(data[l][0][s], data[l][1][s], shift)
            assert np.array_equal(ready[j], rd_o), (s, l)
            nready += int(rd_o.sum())
            err = np.sqrt(np.mean(np.abs(ce[j] - ce_o) ** 2) / max(np.mean(np.abs(ce_o) ** 2), 1e-30))
            worst = max(worst, err)
    assert worst < 1e-5, worst
    assert nready > 0
    gpu.close()


def test_wiener_reset_restarts_link():
    rng = np.random.default_rng(9)
    pil, snr, _ = wc.synth_pilots(rng, 25, 1, 1, 3, snr_db=20.0)
    gpu = WienerDl(25, 1, 1, 1)
    a = [gpu.run([0], pil[s][None], snr[s][None], [1]) for s in range(3)]
    gpu.reset(0)
    b = [gpu.run([0], pil[s][None], snr[s][None], [1]) for s in range(3)]
    for x, y in zip(a, b):
        assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) and x[2] == y[2]
    gpu.close()
