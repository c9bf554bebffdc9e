"""GPU parity of the UE downlink front-end (include/srsran_amd/ue_dl.h) against the oracle
(oracle/ue_dl_chain.py):
  * OFDM demodulation vs a float64 DFT of the same samples: max |error| <= 1e-5 x RMS of the grid (the
    reference's FFTW float transform is pinned only by tolerance);
  * channel estimation vs orc_chest.c on the SAME grid: max |error| <= 2e-5 x RMS(ce) (float summation order),
    noise / RSRP / RSRQ within 1e-3 relative;
  * end to end from time-domain I/Q through OFDM, estimation, MMSE equalisation and the DL-SCH: every TB
    decodes with the transmitted payload; soft bits against the oracle chain within +-2 (fraction < 1e-3).
"""
import numpy as np
import pytest

import oracle
from oracle import pdsch_chain as pc
from oracle import ue_dl_chain as uc
from srsran_amd import pdsch as P
from srsran_amd.dlsch import SoftbufferPool
from srsran_amd.tdec import DeviceBuffer
from srsran_amd.ue_dl import DlSfJob, UeDl, default_chest_cfg
from tests.pdsch_jobs import DevIqSubframe, cell_of

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nof_prb,std", [(6, False), (15, False), (25, False), (50, False), (75, False),
                                         (100, False), (100, True), (25, True)])
def test_ofdm_matches_dft(nof_prb, std):
    rng = np.random.default_rng(nof_prb)
    N = uc.symbol_sz(nof_prb, std)
    nrx = 2
    iq = ((rng.standard_normal((nrx, 15 * N)) + 1j * rng.standard_normal((nrx, 15 * N))) / np.sqrt(2)).astype(
        np.complex64)
    cell = P.make_cell(nof_prb, 1, 3)
    ue = UeDl(cell, nrx)
    if std:
        assert ue.L.mi355_ue_dl_set_standard_rates(ue.h, 1) == 0
    G = 14 * 12 * nof_prb
    bin_ = [DeviceBuffer(iq[r].nbytes).upload(iq[r]) for r in range(nrx)]
    bout = [DeviceBuffer(G * 8) for _ in range(nrx)]
    j = DlSfJob()
    for r in range(nrx):
        j.in_buffer[r], j.sf_symbols[r] = bin_[r].ptr, bout[r].ptr
    ue.ofdm([j])
    for r in range(nrx):
        got = bout[r].download(np.zeros(G, np.complex64))
        want = uc.ofdm_rx_sf(iq[r], nof_prb, std=std)
        rms = np.sqrt(np.mean(np.abs(want) ** 2))
        err = np.abs(got - want).max() / rms
        assert err < 1e-5, (nof_prb, std, r, err)


CHEST = [  # (nof_prb, ports, cell_id, nrx, sf, filter, coef)
    (100, 2, 1, 2, 4, 0, (4.0, 1.0)), (100, 1, 0, 1, 0, 0, (4.0, 1.0)), (50, 1, 5, 2, 3, 1, (0.1, 0.0)),
    (25, 4, 4, 2, 7, 0, (4.0, 1.0)), (15, 2, 2, 1, 9, 2, (0.0, 0.0)), (6, 1, 301, 1, 5, 0, (0.0, 0.0)),
    (75, 2, 8, 2, 1, 0, (6.0, 2.0)),
]


@pytest.mark.parametrize("k", range(len(CHEST)))
def test_chest_matches_oracle(k):
    nof_prb, ports, cid, nrx, sf, ft, coef = CHEST[k]
    rng = np.random.default_rng(200 + k)
    cfg = pc.Cfg(nof_prb=nof_prb, nof_ports=ports, cell_id=cid, nof_rx=nrx, sf_idx=sf, cfi=2,
                 scheme=0 if ports == 1 else 1, nof_layers=ports, qm=[2], tbs=[pc.valid_tbs(500)])
    G = 14 * 12 * nof_prb
    nre = 12 * nof_prb
    tx = np.zeros((ports, G), np.complex64)
    uc.crs_put(tx, nof_prb, cid, ports, sf)
    h = uc.channel_freq(rng, ports, nrx, nof_prb)
    grids = np.zeros((nrx, G), np.complex64)
    for r in range(nrx):
        y = sum(tx[p].reshape(14, nre) * h[p, r][None, :] for p in range(ports))
        y = y + 0.02 * (rng.standard_normal(y.shape) + 1j * rng.standard_normal(y.shape))
        grids[r] = y.reshape(-1)
    ce_o, res_o = uc.chest_estimate(grids, nof_prb, ports, cid, sf, ft, coef)
    ue = UeDl(P.make_cell(nof_prb, ports, cid), nrx)
    gb = [DeviceBuffer(G * 8).upload(grids[r]) for r in range(nrx)]
    cb = [[DeviceBuffer(G * 8) for _ in range(nrx)] for _ in range(ports)]
    j = DlSfJob()
    j.tti = sf
    for r in range(nrx):
        j.sf_symbols[r] = gb[r].ptr
        for p in range(ports):
            j.ce[p][r] = cb[p][r].ptr
    res = ue.chest([j], default_chest_cfg(ft, coef))[0]
    for p in range(ports):
        for r in range(nrx):
            got = cb[p][r].download(np.zeros(G, np.complex64))
            rms = np.sqrt(np.mean(np.abs(ce_o[p, r]) ** 2))
            err = np.abs(got - ce_o[p, r]).max() / rms
            assert err < 2e-5, (k, p, r, err)
    assert abs(res.noise_estimate - res_o["noise_estimate"]) <= 1e-3 * res_o["noise_estimate"]
    assert abs(res.rsrp - res_o["rsrp"]) <= 1e-4 * res_o["rsrp"]
    assert abs(res.rsrq - res_o["rsrq"]) <= 1e-4 * res_o["rsrq"]
    assert abs(res.snr_db - res_o["snr_db"]) < 0.01


E2E = [
    pc.Cfg(nof_prb=100, nof_ports=1, nof_rx=1, cell_id=1, cfi=1, sf_idx=3, scheme=0, nof_layers=1, qm=[2],
           tbs=[15840]),
    pc.Cfg(nof_prb=100, nof_ports=2, nof_rx=2, cell_id=1, cfi=1, sf_idx=4, scheme=2, nof_layers=2, qm=[8, 8],
           tbs=[97896, 97896], csi_enable=True),
    pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, cell_id=7, cfi=2, sf_idx=0, scheme=1, nof_layers=2, qm=[4],
           tbs=[4968]),
    pc.Cfg(nof_prb=50, nof_ports=2, nof_rx=2, cell_id=5, cfi=3, sf_idx=5, scheme=3, nof_layers=2, qm=[6, 6],
           tbs=[20616, 20616]),
]


def test_ue_dl_end_to_end():
    rng = np.random.default_rng(77)
    for k, cfg in enumerate(E2E):
        for t in cfg.tbs:
            assert pc.valid_tbs(t) == t, t
        iq, payload, _h, _s2 = uc.synth_iq(cfg, rng, snr_db=32, max_delay=3)
        ue = UeDl(cell_of(cfg), cfg.nof_rx)
        ds = DevIqSubframe(cfg, iq)
        res = ue.fft_estimate([ds.sfjob], default_chest_cfg())[0]
        ds.set_noise(res.noise_estimate)
        pool = SoftbufferPool(2, max_cb=32)
        out = ue.pdsch.decode(pool, [ds.job])
        # oracle chain from the same I/Q
        grids = np.stack([uc.ofdm_rx_sf(iq[r], cfg.nof_prb) for r in range(cfg.nof_rx)])
        ce_o, res_o = uc.chest_estimate(grids, cfg.nof_prb, cfg.nof_ports, cfg.cell_id, cfg.sf_idx)
        _, _, e_o = pc.rx_front(cfg, grids, ce_o, res_o["noise_estimate"])
        nre = ds.job.cfg.grant.nof_re
        for t in range(cfg.nof_tb):
            assert out[t].ret == 0 and out[t].crc, (k, t)
            np.testing.assert_array_equal(ds.payload_bytes(t)[: cfg.tbs[t] // 8], payload[t])
            e_g = ue.pdsch.stage(0, t, nre, nre * cfg.qm[t])[2]
            diff = np.abs(e_g.astype(np.int32) - e_o[t].astype(np.int32))
            assert diff.max() <= 2 and (diff > 0).mean() < 1e-3, (k, t, diff.max(), (diff > 0).mean())


FUSED = [  # (cfg, sf indices): the fused call's equaliser+LLR path (port 0, SM) and its two-kernel path (SFBC, CDD)
    (E2E[1], (1, 4, 0)),
    (pc.Cfg(nof_prb=50, nof_ports=1, nof_rx=2, cell_id=3, cfi=2, sf_idx=0, scheme=0, nof_layers=1, qm=[6],
            tbs=[pc.valid_tbs(18000)], csi_enable=True), (2, 5, 7)),
    (pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, cell_id=9, cfi=1, sf_idx=0, scheme=2, nof_layers=1, qm=[4],
            tbs=[pc.valid_tbs(5000)], pmi=2, csi_enable=True), (3, 6, 9)),
    (pc.Cfg(nof_prb=50, nof_ports=2, nof_rx=2, cell_id=5, cfi=3, sf_idx=0, scheme=3, nof_layers=2, qm=[6, 6],
            tbs=[20616, 20616], csi_enable=True), (1, 2, 8)),
    (pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, cell_id=7, cfi=2, sf_idx=0, scheme=1, nof_layers=2, qm=[4],
            tbs=[4968], csi_enable=True), (0, 4, 5)),
]


@pytest.mark.parametrize("k", range(len(FUSED)))
def test_fused_decode_matches_two_step(k):
    """mi355_ue_dl_decode_batch (noise kept on the device, channel estimates read from their first row, the
    equaliser and LLR fused for port 0 / spatial multiplexing) == decode_fft_estimate followed by decode_pdsch:
    same chest results, CRCs, payloads and LLRs, over a batch mixing subframes."""
    rng = np.random.default_rng(5 + k)
    cfg0, sfl = FUSED[k]
    subs = []
    for sf in sfl:
        cfg = pc.Cfg(**{**cfg0.__dict__, "sf_idx": sf})
        iq, payload, _h, _s2 = uc.synth_iq(cfg, rng, snr_db=34, channel="cross")
        subs.append((cfg, iq, payload))
    ntb = cfg0.nof_tb
    outs = []
    for fused in (False, True):
        ue = UeDl(cell_of(cfg0), cfg0.nof_rx)
        ds = [DevIqSubframe(c, iq, softbuffers=(2 * j, 2 * j + 1)) for j, (c, iq, _) in enumerate(subs)]
        pool = SoftbufferPool(6, max_cb=16)
        jobs = [d.sfjob for d in ds]
        sfs = [d.job.sf for d in ds]
        cfgs = [d.job.cfg for d in ds]
        pays = [p for d in ds for p in (d.job.payload[0], d.job.payload[1])]
        if fused:
            chest, res = ue.decode(pool, jobs, sfs, cfgs, default_chest_cfg(), pays)
        else:
            chest = ue.fft_estimate(jobs, default_chest_cfg())
            res = ue.decode_pdsch(pool, jobs, sfs, cfgs, chest, pays)
        e = [ue.pdsch.stage(j, t, ds[j].job.cfg.grant.nof_re, ds[j].job.cfg.grant.nof_re * cfg0.qm[t])[2]
             for j in range(3) for t in range(ntb)]
        outs.append(([chest[j].noise_estimate for j in range(3)], [(r.crc, r.avg_iterations_block) for r in res],
                     e))
        for j, (c, _, payload) in enumerate(subs):
            for t in range(ntb):
                assert res[2 * j + t].crc, (k, fused, j, t)
                np.testing.assert_array_equal(ds[j].payload_bytes(t)[: c.tbs[t] // 8], payload[t])
    assert outs[0][0] == outs[1][0]
    assert outs[0][1] == outs[1][1]
    for a, b in zip(outs[0][2], outs[1][2]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("k", range(len(CHEST)))
def test_chest_interpolate_matches_oracle(k):
    """srslte_chest_dl_estimate with SRSLTE_ESTIMATOR_ALG_INTERPOLATE (chest_dl.c:430-531): per-symbol smoothing,
    frequency interpolation of each pilot symbol, linear time interpolation (ports 0/1); ports 2/3 reproduce the
    reference copying the never-written row 0 of the estimate buffer over the others (random initial content)."""
    nof_prb, ports, cid, nrx, sf, ft, coef = CHEST[k]
    rng = np.random.default_rng(400 + k)
    G = 14 * 12 * nof_prb
    nre = 12 * nof_prb
    tx = np.zeros((ports, G), np.complex64)
    uc.crs_put(tx, nof_prb, cid, ports, sf)
    h = uc.channel_freq(rng, ports, nrx, nof_prb)
    grids = np.zeros((nrx, G), np.complex64)
    for r in range(nrx):
        # a time-varying channel: the estimate rows differ
        tv = (1 + 0.05 * np.arange(14))[:, None]
        y = sum(tx[p].reshape(14, nre) * h[p, r][None, :] * tv for p in range(ports))
        y = y + 0.02 * (rng.standard_normal(y.shape) + 1j * rng.standard_normal(y.shape))
        grids[r] = y.reshape(-1)
    init = (rng.standard_normal((ports, nrx, G)) + 1j * rng.standard_normal((ports, nrx, G))).astype(np.complex64)
    ce_o, res_o = uc.chest_estimate(grids, nof_prb, ports, cid, sf, ft, coef, alg=1, ce_init=init)
    ue = UeDl(P.make_cell(nof_prb, ports, cid), nrx)
    gb = [DeviceBuffer(G * 8).upload(grids[r]) for r in range(nrx)]
    cb = [[DeviceBuffer(G * 8).upload(init[p, r]) for r in range(nrx)] for p in range(ports)]
    j = DlSfJob()
    j.tti = sf
    for r in range(nrx):
        j.sf_symbols[r] = gb[r].ptr
        for p in range(ports):
            j.ce[p][r] = cb[p][r].ptr
    cfg = default_chest_cfg(ft, coef)
    cfg.estimator_alg = 1
    res = ue.chest([j], cfg)[0]
    for p in range(ports):
        for r in range(nrx):
            got = cb[p][r].download(np.zeros(G, np.complex64))
            rms = np.sqrt(np.mean(np.abs(ce_o[p, r]) ** 2))
            err = np.abs(got - ce_o[p, r]).max() / rms
            assert err < 2e-5, (k, p, r, err)
            if ports == 4 and p >= 2:
                assert np.array_equal(got.reshape(14, nre)[5], init[p, r][:nre])
    assert abs(res.noise_estimate - res_o["noise_estimate"]) <= 1e-3 * res_o["noise_estimate"]
    assert abs(res.rsrp - res_o["rsrp"]) <= 1e-4 * res_o["rsrp"]


def test_ue_dl_decode_interpolate():
    """mi355_ue_dl_decode_batch with the INTERPOLATE estimator on a time-varying channel (no fused equaliser: the
    estimate rows differ): every TB decodes with its payload."""
    from srsran_amd.dlsch import SoftbufferPool
    rng = np.random.default_rng(91)
    for k, cfg in enumerate([E2E[0], E2E[1], E2E[3]]):
        # 40 dB: per-symbol estimates are not averaged over the 4 pilot symbols, and QAM256 at 32 dB on this
        # channel fails the CRC in the oracle chain with either estimator
        iq, payload, _h, _s2 = uc.synth_iq(cfg, rng, snr_db=40, max_delay=3)
        ue = UeDl(cell_of(cfg), cfg.nof_rx)
        ds = DevIqSubframe(cfg, iq)
        ccfg = default_chest_cfg()
        ccfg.estimator_alg = 1
        pool = SoftbufferPool(2, max_cb=32)
        _, res = ue.decode(pool, [ds.sfjob], [ds.job.sf], [ds.job.cfg], ccfg, [ds.job.payload[0], ds.job.payload[1]])
        for t in range(cfg.nof_tb):
            assert res[t].ret == 0 and res[t].crc, (k, t)
            np.testing.assert_array_equal(ds.payload_bytes(t)[: cfg.tbs[t] // 8], payload[t])


@pytest.mark.parametrize("ctrl", [False, True], ids=["decode_batch", "find_and_decode"])
def test_ce_rows_first_only(ctrl):
    """mi355_ue_dl_set_ce_rows(1) (AVERAGE): the batched calls write row 0 of every estimate only -- the other
    13 rows keep whatever the buffer held -- and every result is the one of the all-rows run: estimator outputs,
    CFI / DCIs, CRCs, iteration counts, payloads and the soft bits of a sample."""
    import bench
    from srsran_amd import lib
    cell = bench.tm4_setup()
    B = 24
    src = bench.Tm4Source(cell, B, 0, ctrl=ctrl)
    src.generate(3000, B, 30.0, 5)
    outs = []
    for rows in (0, 1):
        from srsran_amd.synth import DlReceiver
        rx = DlReceiver(cell, 2, B, bench.NB, 0, ctrl=ctrl, ce_rows=rows)
        rx.ue.set_chunks(1)
        lib().mi355_memset_dev(rx.d_ce.ptr, 0xFF, rx.d_ce.nbytes)  # NaN sentinel
        bound = rx.bind(src, 0, B)
        rx.step(bound)
        ce = rx.d_ce.download(np.zeros(rx.d_ce.nbytes // 8, np.complex64)).reshape(B, 4, 14, 1200)
        chest = np.ctypeslib.as_array(rx.chest)[:B].copy()
        res = np.ctypeslib.as_array(rx.res)[: 2 * B].copy()
        e = [rx.ue.pdsch.stage(k, t, 14400, 14400 * 8)[2] for k in (0, 7, 23) for t in range(2)]
        ctl = np.ctypeslib.as_array(rx.ctrl_res)[:B].copy() if ctrl else None
        outs.append((ce, chest, res, rx.received(B), e, ctl))
        rx.close()
    (ce0, ch0, r0, p0, e0, c0), (ce1, ch1, r1, p1, e1, c1) = outs
    assert np.array_equal(ce1[:, :, 0], ce0[:, :, 0])
    assert np.isnan(ce1[:, :, 1:].view(np.float32)).all()  # untouched
    assert np.array_equal(ce0[:, :, 1:], np.repeat(ce0[:, :, :1], 13, axis=2))
    assert ch0.tobytes() == ch1.tobytes()
    assert r0.tobytes() == r1.tobytes() and r0["crc"].all()
    assert np.array_equal(p0, p1)
    for a, b in zip(e0, e1):
        assert np.array_equal(a, b)
    if ctrl:
        assert c0.tobytes() == c1.tobytes() and (c0["nof_dci"] == 1).all()
    src.close()
