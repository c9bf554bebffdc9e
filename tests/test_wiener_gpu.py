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


@pytest.mark.parametrize("nof_ports,scheme,check_decode", [(2, "SPATIALMUX", False), (1, "PORT0", True)])
def test_ue_chain_wiener_estimator(nof_ports, scheme, check_decode):
    """The UE chain with estimator_alg = WIENER (chest_dl.c:648-676) over 6 subframes of one link (25 PRB, 2 rx, a
    static multipath channel with one delay profile for every antenna pair, 25 dB): until the link is ready the
    estimates are the AVERAGE estimator's (equal to a second receiver configured with AVERAGE), afterwards they are
    the Wiener rows -- equal (1e-4 relative RMS) to oracle/orc_wiener.cpp fed with the LS pilots of the GPU's own
    OFDM grids and the chain's per-port SNR.  With one port the TBs decode once the matrices have averaged a few
    training rounds.  (With two ports the reference trains its shared matrices with the last port's CRS shift,
    wiener_dl.c:506-521 called as chest_dl.c:651 does, and applies them to port 0 as well, whose estimates are then
    biased by the three-subcarrier offset; the restatement keeps that, so no decode is required there.)"""
    from oracle import pdsch_chain as pc
    from oracle import ue_dl_chain as uc
    from srsran_amd.dlsch import SoftbufferPool
    from srsran_amd.ue_dl import UeDl, default_chest_cfg
    from tests.pdsch_jobs import DevIqSubframe, cell_of

    nsf, prb = 6, 25
    if nof_ports == 2:
        cfg0 = pc.Cfg(nof_prb=prb, nof_ports=2, nof_rx=2, cell_id=5, cfi=1, scheme=pc.SPATIALMUX, nof_layers=2,
                      qm=[4, 4], tbs=[pc.valid_tbs(5000)] * 2, csi_enable=True)
    else:
        cfg0 = pc.Cfg(nof_prb=prb, nof_ports=1, nof_rx=2, cell_id=5, cfi=1, scheme=pc.PORT0, nof_layers=1,
                      qm=[4], tbs=[pc.valid_tbs(5000)], csi_enable=True)
    cell = cell_of(cfg0)
    subs = []
    for s in range(nsf):
        cfg = pc.Cfg(**{**cfg0.__dict__, "sf_idx": 1 + s})
        iq, payload, _h, _s2 = uc.synth_iq(cfg, np.random.default_rng(77), snr_db=25, max_delay=8, common_delays=True)
        subs.append((cfg, iq, payload))
    ue_w, ue_a = UeDl(cell, 2), UeDl(cell, 2)
    cw, ca = default_chest_cfg(), default_chest_cfg()
    cw.estimator_alg = 2
    pool = SoftbufferPool(4 * nsf, max_cb=8)  # fresh softbuffers for every subframe (no HARQ combining)
    P = nof_ports
    oracle_w = wc.Wiener(prb, P, 2)
    shift = [wc.crs_shift(cfg0.cell_id, p) for p in range(P)]
    nref = 2 * prb
    wiener_seen = 0
    for s, (cfg, iq, payload) in enumerate(subs):
        dw, da = DevIqSubframe(cfg, iq, softbuffers=(4 * s, 4 * s + 1)), DevIqSubframe(cfg, iq, softbuffers=(4 * s + 2, 4 * s + 3))
        pays = [dw.job.payload[0], dw.job.payload[1] if cfg.nof_tb > 1 else 0]
        chest, res = ue_w.decode(pool, [dw.sfjob], [dw.job.sf], [dw.job.cfg], cw, pays)
        ue_a.fft_estimate([da.sfjob], ca)
        grids, ce_w, ce_a = dw.grids(), dw.ces(), da.ces()
        # the oracle's inputs: LS pilots of the GPU grid, snr_lin = rsrp / noise / 2 from the chain's result
        pil = np.zeros((2, P, 4, nref), np.complex64)
        snr = np.zeros((2, P), np.float32)
        for r in range(2):
            for p in range(P):
                ref = uc.crs_pilots(prb, cfg.cell_id, 0, cfg.sf_idx)
                pos = uc.crs_positions(prb, cfg.cell_id, p)
                x = np.array([grids[r][sy * 12 * prb + f] for sy, f in pos], np.complex64)
                pil[r, p] = (x * np.conj(ref)).reshape(4, nref)
                snr[r, p] = np.float32(10 ** (chest[0].snr_ant_port_db[r][p] / 10) / 2)
        ce_o, rd_o, _ = oracle_w.subframe(pil, snr, shift)
        for r in range(2):
            for p in range(P):
                got = ce_w[p][r].reshape(14, -1)
                if rd_o[r, p]:
                    wiener_seen += 1
                    err = np.sqrt(np.mean(np.abs(got - ce_o[r, p]) ** 2) / np.mean(np.abs(ce_o[r, p]) ** 2))
                    assert err < 1e-4, (s, r, p, err)
                else:
                    assert np.array_equal(ce_w[p][r], ce_a[p][r]), (s, r, p)
        if check_decode and (s == 0 or s >= 3):
            for t in range(cfg.nof_tb):
                assert res[t].ret == 0 and res[t].crc, (s, t)
                assert np.array_equal(dw.payload_bytes(t)[: cfg.tbs[t] // 8], payload[t])
    assert wiener_seen >= 4 * P
