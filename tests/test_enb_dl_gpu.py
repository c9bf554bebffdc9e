"""GPU parity of the eNodeB-side generator (mi355_enb_dl_*) against its host chain, which
tests/test_enb_dl_host.py pins to the oracle transmitter and the reference's turbo-encoder known answer:

* put_pdsch grids equal to mi355_pdsch_encode_host's bit for bit (coded bits, scrambling, modulation,
  precoding and RE mapping are integer / exact-float work) over every supported scheme, multi-job batches;
* put_refs equal to the host CRS;
* gen_signal against a float64 numpy IDFT with srslte_ofdm_tx_sf's bin mapping and CP, x 0.05/sqrt(nof_prb);
* the test channel: exact mixing at sigma 0, noise statistics and determinism at sigma > 0;
* round trip: GPU generator -> channel -> IFFT -> the product's UE chain decodes every TB with the payload.
"""
from __future__ import annotations

import zlib

import numpy as np
import pytest

from oracle import pdsch_chain as pc
from srsran_amd import enb_dl
from srsran_amd import pdsch as P
from srsran_amd.tdec import DeviceBuffer
from tests.pdsch_jobs import cell_of, grant_of
from tests.test_enb_dl_host import host_tx_grid, tx_configs

pytestmark = pytest.mark.gpu


def dev_zeros(nbytes: int) -> DeviceBuffer:
    return DeviceBuffer(nbytes).upload(np.zeros(nbytes, np.uint8))


def enb_job(cfg: pc.Cfg, payloads: list[DeviceBuffer], grids: list[DeviceBuffer], sf_idx=None) -> enb_dl.EnbPdschJob:
    j = enb_dl.EnbPdschJob()
    j.sf.tti = cfg.sf_idx if sf_idx is None else sf_idx
    j.sf.cfi = cfg.cfi
    j.cfg.grant = grant_of(cfg)
    j.cfg.rnti = cfg.rnti
    j.cfg.p_a = cfg.p_a  # the transmitter scales by rho_a whatever power_scale says (pdsch.c:1174-1188)
    for t, b in enumerate(payloads):
        j.data[t] = b.ptr
    for p, g in enumerate(grids):
        j.sf_symbols[p] = g.ptr
    return j


@pytest.mark.parametrize("name,cfg", tx_configs(), ids=[n for n, _ in tx_configs()])
def test_put_pdsch_matches_host(name, cfg):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    pl = [rng.integers(0, 256, t // 8, dtype=np.uint8) for t in cfg.tbs]
    ref = host_tx_grid(cfg, pl)
    enb = enb_dl.EnbDl(cell_of(cfg))
    d_pl = [DeviceBuffer(p.nbytes).upload(p) for p in pl]
    d_g = [dev_zeros(cfg.grid_len * 8) for _ in range(cfg.nof_ports)]
    enb.put_pdsch([enb_job(cfg, d_pl, d_g)])
    got = np.stack([g.download(np.zeros(cfg.grid_len, np.complex64)) for g in d_g])
    bad = np.nonzero(got.view(np.uint64) != ref.view(np.uint64))
    assert bad[0].size == 0, (bad[0].size, bad[1][:8], got[bad][:4], ref[bad][:4])


def test_put_pdsch_batch_tm4():
    """One call, 12 TM4 QAM256 jobs of a 100-PRB cell over every subframe index and rv (32 code blocks of K=6144
    each): every grid equals the host encoder's."""
    base = pc.Cfg(nof_prb=100, nof_ports=2, nof_rx=2, cell_id=1, cfi=1, scheme=pc.SPATIALMUX, nof_layers=2,
                  qm=[8, 8], tbs=[97896, 97896])
    enb = enb_dl.EnbDl(cell_of(base))
    rng = np.random.default_rng(5)
    jobs, keep, refs = [], [], []
    for i in range(12):
        cfg = pc.Cfg(**{**base.__dict__, "sf_idx": i % 10, "rv": [i % 4, (i + 1) % 4], "rnti": 0x1234 + i})
        pl = [rng.integers(0, 256, t // 8, dtype=np.uint8) for t in cfg.tbs]
        refs.append(host_tx_grid(cfg, pl))
        d_pl = [DeviceBuffer(p.nbytes).upload(p) for p in pl]
        d_g = [dev_zeros(cfg.grid_len * 8) for _ in range(2)]
        keep.append((d_pl, d_g))
        jobs.append(enb_job(cfg, d_pl, d_g))
    enb.put_pdsch(jobs)
    for i, (_, d_g) in enumerate(keep):
        got = np.stack([g.download(np.zeros(base.grid_len, np.complex64)) for g in d_g])
        assert np.array_equal(got.view(np.uint32), refs[i].view(np.uint32)), i


def test_put_pdsch_rejects_invalid():
    cfg = pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, scheme=pc.SPATIALMUX, nof_layers=2, qm=[4, 4],
                 tbs=[pc.valid_tbs(5000)] * 2)
    enb = enb_dl.EnbDl(cell_of(cfg))
    d_pl = [DeviceBuffer(t // 8) for t in cfg.tbs]
    d_g = [dev_zeros(cfg.grid_len * 8) for _ in range(2)]
    j = enb_job(cfg, d_pl, d_g)
    j.cfg.grant.nof_re += 1  # inconsistent with the allocation
    with pytest.raises(RuntimeError):
        enb.put_pdsch([j])
    j = enb_job(cfg, d_pl, d_g)
    j.data[1] = None  # missing payload of an enabled TB
    with pytest.raises(RuntimeError):
        enb.put_pdsch([j])


@pytest.mark.parametrize("nof_prb,nof_ports,cell_id", [(6, 1, 1), (25, 2, 7), (100, 2, 1), (50, 4, 301)])
def test_put_refs_matches_host(nof_prb, nof_ports, cell_id):
    cell = P.make_cell(nof_prb, nof_ports, cell_id)
    G = 14 * 12 * nof_prb
    enb = enb_dl.EnbDl(cell)
    ttis = list(range(10))
    grids = [dev_zeros(G * 8) for _ in range(10 * nof_ports)]
    enb.put_refs(ttis, [g.ptr for g in grids])
    for sf in ttis:
        ref = np.zeros((nof_ports, G), np.complex64)
        enb_dl.put_refs(cell, sf, ref)
        got = np.stack([grids[sf * nof_ports + p].download(np.zeros(G, np.complex64)) for p in range(nof_ports)])
        assert np.array_equal(got, ref), sf


def ofdm_tx_ref(grid: np.ndarray, nof_prb: int) -> np.ndarray:
    from srsran_amd.ue_dl import symbol_sz
    N = symbol_sz(nof_prb)
    nre = 12 * nof_prb
    cp0, cp1 = int(np.ceil(160 * N / 2048)), int(np.ceil(144 * N / 2048))
    out = np.zeros(15 * N, np.complex128)
    g = grid.reshape(14, nre).astype(np.complex128)
    for s in range(14):
        sl, l = divmod(s, 7)
        X = np.zeros(N, np.complex128)
        X[N - nre // 2:] = g[s, : nre // 2]
        X[1: nre // 2 + 1] = g[s, nre // 2:]
        x = N * np.fft.ifft(X) * (0.05 / np.sqrt(nof_prb))
        cp = cp0 if l == 0 else cp1
        start = sl * (15 * N // 2) + (0 if l == 0 else cp0 + N + (l - 1) * (N + cp1))
        out[start: start + cp] = x[N - cp:]
        out[start + cp: start + cp + N] = x
    return out


@pytest.mark.parametrize("nof_prb", [6, 15, 25, 50, 75, 100])
def test_gen_signal_matches_idft(nof_prb):
    from srsran_amd.ue_dl import symbol_sz
    cell = P.make_cell(nof_prb, 1, 3)
    N = symbol_sz(nof_prb)
    G = 14 * 12 * nof_prb
    rng = np.random.default_rng(nof_prb)
    enb = enb_dl.EnbDl(cell)
    grids = [(rng.standard_normal(G) + 1j * rng.standard_normal(G)).astype(np.complex64) for _ in range(3)]
    d_g = [DeviceBuffer(G * 8).upload(g) for g in grids]
    d_o = [dev_zeros(15 * N * 8) for _ in grids]
    enb.gen_signal([g.ptr for g in d_g], [o.ptr for o in d_o])
    for g, o in zip(grids, d_o):
        ref = ofdm_tx_ref(g, nof_prb)
        got = o.download(np.zeros(15 * N, np.complex64))
        rms = np.sqrt(np.mean(np.abs(ref) ** 2))
        assert np.abs(got - ref).max() <= 1e-5 * rms, (np.abs(got - ref).max(), rms)


def test_channel_grid():
    cell = P.make_cell(25, 2, 1)
    G = 14 * 12 * 25
    enb = enb_dl.EnbDl(cell)
    rng = np.random.default_rng(3)
    n = 3
    tx = [(rng.standard_normal(G) + 1j * rng.standard_normal(G)).astype(np.complex64) for _ in range(2 * n)]
    d_tx = [DeviceBuffer(G * 8).upload(t) for t in tx]
    d_rx = [dev_zeros(G * 8) for _ in range(2 * n)]
    H = np.array([[1, 1], [1, -1]], np.complex64) * np.complex64(0.5 + 0.25j)
    enb.channel([t.ptr for t in d_tx], [r.ptr for r in d_rx], 2, H, 0.0, 1)
    for i in range(n):
        for r in range(2):
            got = d_rx[2 * i + r].download(np.zeros(G, np.complex64))
            ref = H[r, 0] * tx[2 * i] + H[r, 1] * tx[2 * i + 1]
            np.testing.assert_allclose(got, ref, rtol=0, atol=1e-5)
    # AWGN: zero-mean, per-dimension variance sigma^2, reproducible for a seed, different across seeds / jobs
    zero = [dev_zeros(G * 8) for _ in range(2 * n)]
    sigma = 0.3
    enb.channel([t.ptr for t in zero], [r.ptr for r in d_rx], 2, H, sigma, 7)
    a = np.stack([r.download(np.zeros(G, np.complex64)) for r in d_rx])
    enb.channel([t.ptr for t in zero], [r.ptr for r in d_rx], 2, H, sigma, 7)
    b = np.stack([r.download(np.zeros(G, np.complex64)) for r in d_rx])
    enb.channel([t.ptr for t in zero], [r.ptr for r in d_rx], 2, H, sigma, 8)
    c = np.stack([r.download(np.zeros(G, np.complex64)) for r in d_rx])
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert not np.array_equal(a[0], a[2]) and not np.array_equal(a[0], a[1])
    v = np.concatenate([a.real.ravel(), a.imag.ravel()])
    assert abs(v.mean()) < 0.01 and abs(v.std() - sigma) < 0.01 * sigma * 3


def test_generator_round_trip_tm4():
    """Device payloads -> GPU generator (PDSCH + CRS) -> crossed 2x2 channel + 30 dB AWGN -> IFFT -> the
    product's UE chain (mi355_ue_dl_decode_batch): every TB decodes with its payload."""
    from srsran_amd.dlsch import SoftbufferPool
    from srsran_amd.ue_dl import DlSfJob, UeDl, default_chest_cfg, symbol_sz
    cfg0 = pc.Cfg(nof_prb=100, nof_ports=2, nof_rx=2, cell_id=1, cfi=1, scheme=pc.SPATIALMUX, nof_layers=2,
                  qm=[8, 8], tbs=[97896, 97896], csi_enable=True)
    cell = cell_of(cfg0)
    N = symbol_sz(100)
    G = cfg0.grid_len
    enb = enb_dl.EnbDl(cell)
    ue = UeDl(cell, 2)
    rng = np.random.default_rng(11)
    nsf = 6
    sfs = [1, 2, 3, 4, 6, 7]
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
    H = np.array([[1, 1], [1, -1]], np.complex64)
    sigma = float(np.sqrt(10 ** (-30 / 10) / 2))
    enb.channel([g.ptr for t in tx for g in t], [g.ptr for r in rx for g in r], 2, H, sigma, 1234)
    enb.gen_signal([g.ptr for r in rx for g in r], [g.ptr for s in iq for g in s])
    # UE side
    grids = [[dev_zeros(G * 8) for _ in range(2)] for _ in range(nsf)]
    ces = [[[dev_zeros(G * 8) for _ in range(2)] for _ in range(2)] for _ in range(nsf)]
    outs = [[DeviceBuffer(t // 8 + 16) for t in cfg0.tbs] for _ in range(nsf)]
    pool = SoftbufferPool(2 * nsf, max_cb=16)
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
        pc_.csi_enable = 1
        pc_.power_scale, pc_.p_a, pc_.p_b = 1, 0.0, 1  # undo the transmitter's rho_a, rho_b = 1 (as phy_dl_test)
        pc_.softbuffer[0], pc_.softbuffer[1] = 2 * i, 2 * i + 1
        pcfgs.append(pc_)
        pays += [outs[i][0].ptr, outs[i][1].ptr]
    _, res = ue.decode(pool, sjobs, sfcfgs, pcfgs, default_chest_cfg(), pays)
    for i in range(nsf):
        for t in range(2):
            assert res[2 * i + t].ret == 0 and res[2 * i + t].crc, (i, t)
            got = outs[i][t].download(np.zeros(cfg0.tbs[t] // 8 + 16, np.uint8))[: cfg0.tbs[t] // 8]
            np.testing.assert_array_equal(got, pls[i][t])


def test_indexed_synthesis_is_shard_invariant():
    """bench.py --total-subframes: payloads (mi355_enb_synth_payloads) equal their host restatement, and the AWGN of
    mi355_channel_grid_batch_at depends on the global subframe index only -- one call over [10, 14) equals two calls
    over [10, 12) and [12, 14); first_index 0 equals the plain call."""
    cell = P.make_cell(6, 2, 1)
    G = 14 * 12 * 6
    enb = enb_dl.EnbDl(cell)
    d = dev_zeros(5 * 2 * 1001)
    enb.synth_payloads(d.ptr, (1 << 40) + 3, 5, 2, 1001, 99)
    got = d.download(np.zeros(5 * 2 * 1001, np.uint8)).reshape(5, 2, 1001)
    assert np.array_equal(got, enb_dl.synth_payloads_host((1 << 40) + 3, 5, 2, 1001, 99))
    assert not np.array_equal(got[0, 0], got[0, 1]) and not np.array_equal(got[0, 0], got[1, 0])
    H = np.array([[1, 1], [1, -1]], np.complex64)
    zero = [dev_zeros(G * 8) for _ in range(2 * 4)]
    one = [dev_zeros(G * 8) for _ in range(2 * 4)]
    two = [dev_zeros(G * 8) for _ in range(2 * 4)]
    enb.channel([t.ptr for t in zero], [r.ptr for r in one], 2, H, 0.5, 77, first_index=10)
    enb.channel([t.ptr for t in zero[:4]], [r.ptr for r in two[:4]], 2, H, 0.5, 77, first_index=10)
    enb.channel([t.ptr for t in zero[4:]], [r.ptr for r in two[4:]], 2, H, 0.5, 77, first_index=12)
    a = np.stack([r.download(np.zeros(G, np.complex64)) for r in one])
    b = np.stack([r.download(np.zeros(G, np.complex64)) for r in two])
    assert np.array_equal(a, b) and np.abs(a).max() > 0
    enb.channel([t.ptr for t in zero], [r.ptr for r in one], 2, H, 0.5, 77, first_index=0)
    enb.channel([t.ptr for t in zero], [r.ptr for r in two], 2, H, 0.5, 77)
    a = np.stack([r.download(np.zeros(G, np.complex64)) for r in one])
    b = np.stack([r.download(np.zeros(G, np.complex64)) for r in two])
    assert np.array_equal(a, b)
