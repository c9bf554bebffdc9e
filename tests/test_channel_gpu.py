"""GPU: the time-domain channel emulators (mi355_channel_{fading,delay,hst}_*, srsran_amd/csrc/channel_*) against
the CPU restatement oracle/channel_chain.py on the same inputs:
* fading (fading.c): several links with their own seeds, EPA / EVA / ETU at 1.92 / 23.04 / 30.72 Msps, two
  consecutive calls (overlap-add state and time carried), a ragged last segment.  Tap gains are the same float32
  sine-table arithmetic on both sides; the FFTs are float32 (GPU) vs float64 (oracle): relative RMS <= 2e-6.
* delay (delay.c): pure sample moves, so bit-exact, across calls whose delay grows and shrinks.
* hst (hst.c): frequency shift, within 1e-5 of the float64 phasor (the reference's recursive float phasor itself
  drifts by ~1e-7 per 8 samples).
"""
import numpy as np
import pytest

from oracle import channel_chain as cc
from srsran_amd import channel as ch

pytestmark = pytest.mark.gpu


def rel_rms(a, b):
    return float(np.sqrt(np.mean(np.abs(a - b) ** 2) / np.mean(np.abs(b) ** 2)))


@pytest.mark.parametrize("model,srate,n1,n2", [("epa5", 23.04e6, 23040, 11520 + 100), ("eva70", 30.72e6, 7000, 30720),
                                              ("etu300", 1.92e6, 1920, 1000), ("epa300", 1.92e6, 333, 1587)])
def test_fading_matches_oracle(model, srate, n1, n2):
    rng = np.random.default_rng(5)
    seeds = [0x1234 * i + 7 for i in range(3)]
    q = ch.Fading(srate, model, seeds, max(n1, n2))
    refs = [cc.Fading(srate, model, s) for s in seeds]
    assert q.N == refs[0].N
    t0 = np.array([0.0, 0.0123, 1.5])
    for n in (n1, n2):
        x = ((rng.standard_normal((3, n)) + 1j * rng.standard_normal((3, n))) / np.sqrt(2)).astype(np.complex64)
        y, t1 = q.execute(x, t0)
        for i, r in enumerate(refs):
            yo, to = r.execute(x[i].astype(complex), t0[i])
            assert t1[i] == to
            assert rel_rms(y[i], yo) < 2e-6, (model, n, i, rel_rms(y[i], yo))
        t0 = t1
    q.close()


def test_fading_rejects_bad_inputs():
    with pytest.raises(RuntimeError):
        ch.Fading(23.04e6, "none0", [1], 100)
    with pytest.raises(RuntimeError):
        ch.Fading(23.04e6, "xyz5", [1], 100)


def test_delay_bit_exact():
    rng = np.random.default_rng(6)
    q = ch.Delay(1.0, 8.0, 0.01, 0.0, 1_920_000, nlinks=2, max_len=2000)
    refs = [cc.Delay(1.0, 8.0, 0.01, 0.0, 1_920_000) for _ in range(2)]
    for call, (n, frac) in enumerate([(1920, 0.0), (1920, 0.0025), (700, 0.004), (1920, 0.0061), (1920, 0.0081)]):
        x = (rng.standard_normal((2, n)) + 1j * rng.standard_normal((2, n))).astype(np.complex64)
        ts = [(0, frac), (1, frac + 0.001)]
        y, d = q.execute(x, ts)
        for i in range(2):
            yo = refs[i].execute(x[i].astype(complex), *ts[i])
            assert d[i] == refs[i].delay_samples(*ts[i])
            assert np.array_equal(y[i], yo.astype(np.complex64)), (call, i)
    q.close()


def test_hst_matches_oracle():
    rng = np.random.default_rng(7)
    n = 23040
    x = (rng.standard_normal((3, n)) + 1j * rng.standard_normal((3, n))).astype(np.complex64)
    ts = [(0, 0.0), (0, 0.3), (2, 0.7)]
    y, fs = ch.hst_execute(x, 750.0, 0.5, 0.0, 23_040_000, ts)
    for i in range(3):
        r = cc.Hst(750.0, 0.5, 0.0, 23_040_000)
        assert fs[i] == pytest.approx(r.shift_hz(*ts[i]), rel=1e-6, abs=1e-6)
        yo = r.execute(x[i].astype(complex), *ts[i])
        assert np.max(np.abs(y[i] - yo)) < 1e-5 * np.max(np.abs(yo))


def test_generator_round_trip_time_domain_epa():
    """Device payloads -> GPU generator (1 port, 25 PRB, 16QAM) -> IFFT -> time-domain EPA 5 Hz fading on the
    continuous sample stream (5.76 Msps, N = 96, path delay 24 + 2.4 samples, inside the 27-sample CP) -> a receiver
    synchronised to the path delay -> the product's UE chain: every TB decodes with its payload."""
    from oracle import pdsch_chain as pc
    from srsran_amd import enb_dl
    from srsran_amd import pdsch as P
    from srsran_amd.dlsch import SoftbufferPool
    from srsran_amd.tdec import DeviceBuffer
    from srsran_amd.ue_dl import DlSfJob, UeDl, default_chest_cfg, symbol_sz
    from tests.pdsch_jobs import cell_of, grant_of
    from tests.test_enb_dl_gpu import dev_zeros, enb_job

    cfg0 = pc.Cfg(nof_prb=25, nof_ports=1, nof_rx=1, cell_id=11, cfi=2, scheme=pc.PORT0, nof_layers=1, qm=[4],
                  tbs=[pc.valid_tbs(5000)])
    cell = cell_of(cfg0)
    Nfft = symbol_sz(25)
    SF = 15 * Nfft
    G = cfg0.grid_len
    enb = enb_dl.EnbDl(cell)
    ue = UeDl(cell, 1)
    rng = np.random.default_rng(9)
    sfs = [0, 1, 2, 3, 4]
    pls, d_pl, tx, iq, jobs = [], [], [], [], []
    for i, sf in enumerate(sfs):
        cfg = pc.Cfg(**{**cfg0.__dict__, "sf_idx": sf})
        pl = [rng.integers(0, 256, t // 8, dtype=np.uint8) for t in cfg.tbs]
        pls.append(pl)
        d_pl.append([DeviceBuffer(p.nbytes).upload(p) for p in pl])
        tx.append([dev_zeros(G * 8)])
        iq.append([dev_zeros(SF * 8)])
        jobs.append(enb_job(cfg, d_pl[i], tx[i]))
    enb.put_pdsch(jobs)
    enb.put_refs(sfs, [t[0].ptr for t in tx])
    enb.gen_signal([t[0].ptr for t in tx], [s[0].ptr for s in iq])
    stream = np.concatenate([s[0].download(np.zeros(SF, np.complex64)) for s in iq] + [np.zeros(SF, np.complex64)])
    srate = 1.92e6 * Nfft / 128
    fad = ch.Fading(srate, "epa5", [77], len(stream))
    y, _ = fad.execute(stream[None, :], 0.0)
    fad.close()
    pd = fad.N // 4
    nsf = len(sfs)
    rx = [DeviceBuffer(SF * 8).upload(np.ascontiguousarray(y[0, i * SF + pd: (i + 1) * SF + pd])) for i in range(nsf)]
    grids = [dev_zeros(G * 8) for _ in range(nsf)]
    ces = [dev_zeros(G * 8) for _ in range(nsf)]
    outs = [DeviceBuffer(cfg0.tbs[0] // 8 + 16) for _ in range(nsf)]
    pool = SoftbufferPool(nsf, max_cb=4)
    sjobs, sfcfgs, pcfgs, pays = [], [], [], []
    for i, sf in enumerate(sfs):
        cfg = pc.Cfg(**{**cfg0.__dict__, "sf_idx": sf})
        j = DlSfJob()
        j.tti = sf
        j.in_buffer[0] = rx[i].ptr
        j.sf_symbols[0] = grids[i].ptr
        j.ce[0][0] = ces[i].ptr
        sjobs.append(j)
        sfcfgs.append(P.DlSfCfg(sf, cfg.cfi))
        pc_ = P.PdschCfg()
        pc_.grant = grant_of(cfg)
        pc_.rnti = cfg.rnti
        pc_.softbuffer[0] = i
        pcfgs.append(pc_)
        pays += [outs[i].ptr, 0]
    _, res = ue.decode(pool, sjobs, sfcfgs, pcfgs, default_chest_cfg(), pays)
    for i in range(nsf):
        assert res[2 * i].ret == 0 and res[2 * i].crc, i
        got = outs[i].download(np.zeros(cfg0.tbs[0] // 8 + 16, np.uint8))[: cfg0.tbs[0] // 8]
        np.testing.assert_array_equal(got, pls[i][0])
