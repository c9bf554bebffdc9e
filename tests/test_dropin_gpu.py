"""The srslte_* drop-in on the GPU, exercised from a caller compiled against the REFERENCE headers
(tests/dropin/caller.c -> libdropin_caller.so -> libsrslte_mi355.so -> libsrsran_amd.so).

* srslte_tdec_init_manual / run_all / get_nof_iterations / free (turbodecoder_test.c's calls) on the reference's
  golden code blocks: decisions bit-exact with the reference decoder's, AUTO and GENERIC.
* phy_dl_test's work_ue (srslte_ue_dl_decode_fft_estimate -> find_dl_dci -> dci_to_pdsch_grant -> decode_pdsch)
  on subframes carrying a PCFICH, a DCI on the PDCCH and the PDSCH: the CFI, the DCI, the grant and every
  transport block (CRC ok, payload equal to the transmitted one); the same PDSCH through srslte_pdsch_decode on
  the ue_dl's host copies of the grid and estimates, and srslte_ue_dl_find_and_decode, give the same bytes.
* srslte_pdsch_decode on a stand-alone srslte_pdsch_t with host buffers, with the softbuffer carried across calls
  (the second call finds every code block already decoded; as in the reference, their bytes were not saved because
  the TB passed, so the TB CRC fails).
"""
import ctypes as C
import os

import numpy as np
import pytest

from golden_io import tdec_auto_cases, tdec_generic_cases
from oracle import pdcch_chain as P
from oracle import pdsch_chain as pc
from oracle import ue_dl_chain as uc

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CALLER = os.path.join(ROOT, "tests", "dropin", "libdropin_caller.so")


class CallerCfg(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("nof_prb", "nof_ports", "nof_rx", "cell_id", "rnti", "tm",
                                          "use_tbs_index_alt", "decoder_type", "csi_enable", "max_nof_iterations",
                                          "cfo_estimate_enable", "estimator_alg", "noise_alg",
                                          "sync_error_enable", "power_scale")]


class SfRes(C.Structure):
    _fields_ = [("ret_fft", C.c_int32), ("cfi", C.c_int32), ("nof_dci", C.c_int32), ("ret_grant", C.c_int32),
                ("ret_pdsch", C.c_int32), ("crc", C.c_int32 * 2), ("avg_its", C.c_float * 2), ("ret_host", C.c_int32),
                ("crc_host", C.c_int32 * 2)] + \
               [(n, C.c_int32) for n in ("nof_re", "nof_tb")] + [("tbs", C.c_int32 * 2)] + \
               [(n, C.c_int32) for n in ("tx_scheme", "nof_layers", "dci_format", "dci_ncce", "dci_L", "ret_fad")] + \
               [("ack_fad", C.c_int32 * 2)] + [(n, C.c_float) for n in ("noise_estimate", "snr_db", "rsrp", "cfo")]


class RaTb(C.Structure):  # srslte_ra_tb_t
    _fields_ = [("mod", C.c_int), ("tbs", C.c_int), ("rv", C.c_int), ("nof_bits", C.c_uint32), ("cw_idx", C.c_uint32),
                ("enabled", C.c_bool), ("mcs_idx", C.c_uint32)]


class Grant(C.Structure):  # srslte_pdsch_grant_t
    _fields_ = [("tx_scheme", C.c_int), ("pmi", C.c_uint32), ("prb_idx", (C.c_bool * 110) * 2), ("nof_prb", C.c_uint32),
                ("nof_re", C.c_uint32), ("nof_symb_slot", C.c_uint32 * 2), ("tb", RaTb * 2), ("last_tbs", C.c_int * 2),
                ("nof_tb", C.c_uint32), ("nof_layers", C.c_uint32)]


def _caller():
    if not os.path.exists(CALLER):
        pytest.fail(f"{CALLER} missing: build it where the reference headers exist (make -C tests/dropin)")
    L = C.CDLL(CALLER)
    L.caller_install_crash_handler()
    L.caller_tdec_run_all.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.POINTER(C.c_int)]
    L.caller_ue_dl.argtypes = [C.POINTER(CallerCfg), C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                               C.POINTER(SfRes)]
    # (c, tti, cfi, grant, grid, ce, noise, ncalls, rvs, payload, crc_out, its_out): every pointer declared -- an
    # undeclared trailing argument is passed as a 32-bit C int and truncates the address
    L.caller_tti_latency.argtypes = [C.POINTER(CallerCfg), C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p,
                                     C.c_void_p]
    L.caller_pdsch_decode.argtypes = [C.POINTER(CallerCfg), C.c_uint32, C.c_uint32, C.POINTER(Grant), C.c_void_p,
                                      C.c_void_p, C.c_float, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p]
    return L


def test_grant_mirror_size():
    assert C.sizeof(Grant) == 316 and C.sizeof(RaTb) == 28


def test_tdec_drop_in_matches_reference_goldens():
    L = _caller()
    for c in tdec_auto_cases():
        K, trace = c["K"], c["trace"]
        buf = np.ascontiguousarray(c["buf"].astype(np.int16))
        for nit in (1, 4, len(trace)):
            out = np.zeros(K // 8, np.uint8)
            n = C.c_int(0)
            r = L.caller_tdec_run_all(buf.ctypes.data, out.ctypes.data, K, nit, 0, C.byref(n))
            assert r == 0 and n.value == nit
            assert np.array_equal(out, trace[nit - 1]), (K, nit)
    for c in tdec_generic_cases():
        K, want = c["K"], c["trace"]
        buf = np.ascontiguousarray(c["lin"].astype(np.int16))
        out = np.zeros(K // 8, np.uint8)
        n = C.c_int(0)
        assert L.caller_tdec_run_all(buf.ctypes.data, out.ctypes.data, K, len(want), 1, C.byref(n)) == 0
        assert np.array_equal(out, want[-1]), K
    # the reference rejects K outside the 36.212 table and unsupported implementations with -1
    out = np.zeros(800, np.uint8)
    n = C.c_int(0)
    assert L.caller_tdec_run_all(np.zeros(20000, np.int16).ctypes.data, out.ctypes.data, 6145, 2, 0, C.byref(n)) == -1
    assert L.caller_tdec_run_all(np.zeros(20000, np.int16).ctypes.data, out.ctypes.data, 6144, 2, 7, C.byref(n)) == -100


# (name, nof_prb, ports, rx, tm, DCI format, mcs, tbs_alt, cell id)
CASES = [("tm4_sm_256qam_100prb", 100, 2, 2, 3, P.FORMAT2, 27, True, 1),
         ("tm1_siso_qpsk", 25, 1, 1, 0, P.FORMAT1, 9, False, 3),
         ("tm2_sfbc_16qam", 50, 2, 2, 1, P.FORMAT1, 14, False, 11)]


def _synth(case, ttis, rnti):
    from srsran_amd import pdcch as D
    from srsran_amd import pdsch as S
    from test_pdcch_gpu import _make_dci, _with_rnti
    name, nprb, ports, nrx, tm, fmt, mcs, alt, cid = case
    rng = np.random.default_rng(nprb * 3 + tm)
    cell = S.make_cell(nprb, ports, cid, phich_resources=2)  # SRSLTE_PHICH_R_1, as phy_dl_test's cell
    iqs, expect = [], []
    for tti in ttis:
        sf_idx = tti % 10
        cfi = 1 if mcs == 27 else 1 + sf_idx % 3
        d = _make_dci(D, cell, fmt, mcs, rnti)
        m = D.pack(cell, d, sf_idx)
        g = D.dci_to_grant(cell, D.unpack(cell, _with_rnti(m, rnti), sf_idx), sf_idx, cfi, tm, alt)
        locs = D.ue_locations(D.nof_cce(cell, cfi), sf_idx, rnti)
        L_, n_ = next((lv for lv in locs if lv[0] == 2), locs[-1])
        m.location = D.DciLocation(L_, n_)
        m.rnti = rnti
        prb = np.array([[g.prb_idx[s][k] for k in range(nprb)] for s in range(2)], np.uint8)
        cfg = pc.Cfg(nof_prb=nprb, nof_ports=ports, cell_id=cid, nof_rx=nrx, cfi=cfi, sf_idx=sf_idx, rnti=rnti,
                     scheme=g.tx_scheme, nof_layers=g.nof_layers, pmi=g.pmi,
                     qm=[[1, 2, 4, 6, 8][g.tb[t].mod] for t in range(g.nof_tb)],
                     tbs=[g.tb[t].tbs for t in range(g.nof_tb)], rv=[0, 0], prb=prb, csi_enable=True)

        def ctrl(tx, m=m, sf_idx=sf_idx, cfi=cfi):
            D.encode_ctrl_host(cell, sf_idx, cfi, [m], tx)

        chan, snr = ("cross", 40) if mcs == 27 else ("taps", 32)
        iq, payload, _h, _s2 = uc.synth_iq(cfg, rng, snr_db=snr, ctrl=ctrl, channel=chan)
        iqs.append(iq.astype(np.complex64))
        expect.append((cfg, payload, g, m))
    return np.ascontiguousarray(np.stack(iqs)), expect


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_ue_dl_drop_in_phy_dl_test_flow(case):
    L = _caller()
    name, nprb, ports, nrx, tm, fmt, mcs, alt, cid = case
    rnti = 0x46
    ttis = [10 * 7 + 0, 10 * 7 + 3, 10 * 8 + 6, 10 * 9 + 9]
    iq, expect = _synth(case, ttis, rnti)
    # srsUE's set_ue_dl_cfg defaults (phy_common.cc:78-108, main.cc:317-318): CFO estimation on in every subframe
    # (cfo_ref_mask 1023), REFS noise, AVERAGE; sync-error correction (an option, off by default) on every other case
    sync = CASES.index(case) % 2
    c = CallerCfg(nof_prb=nprb, nof_ports=ports, nof_rx=nrx, cell_id=cid, rnti=rnti, tm=tm, use_tbs_index_alt=int(alt),
                  decoder_type=1, csi_enable=1, max_nof_iterations=10, cfo_estimate_enable=1, estimator_alg=0,
                  noise_alg=0, sync_error_enable=sync)
    nsf = len(ttis)
    maxb = max(t for e in expect for t in e[0].tbs) // 8 + 16
    pay = np.zeros((nsf, 3, 2, maxb), np.uint8)
    res = (SfRes * nsf)()
    tt = np.array(ttis, np.uint32)
    assert L.caller_ue_dl(C.byref(c), iq.ctypes.data, tt.ctypes.data, nsf, pay.ctypes.data, maxb, res) == 0
    for i, (cfg, payload, g, m) in enumerate(expect):
        o = res[i]
        assert o.ret_fft == 0 and o.cfi == cfg.cfi, (name, i, o.ret_fft, o.cfi)
        assert o.nof_dci == 1 and o.dci_format == m.format and o.dci_ncce == m.location.ncce, (name, i, o.nof_dci)
        assert o.ret_grant == 0
        assert (o.nof_re, o.nof_tb, o.tx_scheme, o.nof_layers) == (g.nof_re, g.nof_tb, g.tx_scheme, g.nof_layers)
        assert o.ret_pdsch == 0 and o.ret_host == 0 and o.ret_fad == 1, (o.ret_pdsch, o.ret_host, o.ret_fad)
        # the chest result scalars are filled (noise tracks the 32 / 40 dB AWGN)
        assert o.noise_estimate > 0 and np.isfinite(o.snr_db) and o.rsrp > 0
        assert np.isfinite(o.cfo) and abs(o.cfo) < 0.05  # no carrier offset in the synthetic channel
        for t in range(cfg.nof_tb):
            nb = cfg.tbs[t] // 8
            assert o.crc[t] and o.crc_host[t] and o.ack_fad[t], (name, i, t)
            assert 0 < o.avg_its[t] <= 10
            for k in range(3):
                assert np.array_equal(pay[i, k, t, :nb], payload[t][:nb]), (name, i, k, t)


def test_ctrl_stage_failure_does_not_rerun_estimation():
    """srslte_ue_dl_decode_fft_estimate runs estimation + the control stage in one library call; when only the
    control stage fails (MI355_ERROR_SECOND_STAGE, injected here on the first TTI), the drop-in re-runs the control
    stage alone.  Re-running the estimation would advance the per-link estimator state (CFO average, noise
    history) twice for one TTI, so every later TTI's estimates and decodes must equal a run without the fault."""
    from srsran_amd import lib
    L = _caller()
    case = CASES[0]
    name, nprb, ports, nrx, tm, fmt, mcs, alt, cid = case
    rnti = 0x46
    ttis = [10 * 7 + 0, 10 * 7 + 3, 10 * 8 + 6, 10 * 9 + 9]
    iq, expect = _synth(case, ttis, rnti)
    c = CallerCfg(nof_prb=nprb, nof_ports=ports, nof_rx=nrx, cell_id=cid, rnti=rnti, tm=tm, use_tbs_index_alt=int(alt),
                  decoder_type=1, csi_enable=1, max_nof_iterations=10, cfo_estimate_enable=1, estimator_alg=0,
                  noise_alg=0, sync_error_enable=0)
    nsf, maxb = len(ttis), max(t for e in expect for t in e[0].tbs) // 8 + 16
    tt = np.array(ttis, np.uint32)
    fail = lib().mi355_debug_fail_ctrl_stages
    lib().mi355_debug_fail_ctrl_stages.argtypes = [C.c_int]
    lib().mi355_debug_fail_ctrl_stages.restype = C.c_int
    runs = []
    for nfail in (0, 1):
        pay = np.zeros((nsf, 3, 2, maxb), np.uint8)
        res = (SfRes * nsf)()
        fail(nfail)
        assert L.caller_ue_dl(C.byref(c), iq.ctypes.data, tt.ctypes.data, nsf, pay.ctypes.data, maxb, res) == 0
        assert fail(0) == 0, "the injected control-stage failure was not consumed"
        runs.append((bytes(res), pay))
    assert runs[0][0] == runs[1][0], "a control-stage failure changed the estimates or decodes of later TTIs"
    assert np.array_equal(runs[0][1], runs[1][1])
    r = (SfRes * nsf).from_buffer_copy(runs[1][0])
    assert all(r[i].ret_fft == 0 and r[i].nof_dci == 1 and r[i].crc[0] and r[i].crc[1] for i in range(nsf))


def test_pdsch_drop_in_host_buffers_and_softbuffer_reuse():
    """srslte_pdsch_decode with a stand-alone object and host grids (pdsch_test.c:498); the second call on the same
    softbuffers skips every code block (cb_crc, sch.c:385) and restores bytes that were never saved (sch.c:462-484)."""
    L = _caller()
    cfg = pc.Cfg(nof_prb=50, nof_ports=2, nof_rx=2, cell_id=21, cfi=2, sf_idx=4, scheme=2, nof_layers=2,
                 qm=[6, 6], tbs=[pc.valid_tbs(30000)] * 2, csi_enable=True)
    rng = np.random.default_rng(5)
    iq, payload, _h, _s2 = uc.synth_iq(cfg, rng, snr_db=36, channel="cross")
    grids = np.stack([uc.ofdm_rx_sf(iq[r], cfg.nof_prb) for r in range(2)]).astype(np.complex64)
    ce, res = uc.chest_estimate(grids, cfg.nof_prb, 2, cfg.cell_id, cfg.sf_idx)
    ce = np.ascontiguousarray(ce.astype(np.complex64))
    grids = np.ascontiguousarray(grids)
    from pdsch_jobs import grant_of
    mg = grant_of(cfg)
    g = Grant()
    g.tx_scheme, g.pmi, g.nof_prb, g.nof_re = mg.tx_scheme, mg.pmi, mg.nof_prb, mg.nof_re
    for s in range(2):
        g.nof_symb_slot[s] = mg.nof_symb_slot[s]
        for k in range(110):
            g.prb_idx[s][k] = bool(mg.prb_idx[s][k])
    for t in range(2):
        g.tb[t].mod, g.tb[t].tbs, g.tb[t].nof_bits = mg.tb[t].mod, mg.tb[t].tbs, mg.tb[t].nof_bits
        g.tb[t].cw_idx, g.tb[t].enabled = mg.tb[t].cw_idx, bool(mg.tb[t].enabled)
    g.nof_tb, g.nof_layers = mg.nof_tb, mg.nof_layers
    c = CallerCfg(nof_prb=50, nof_ports=2, nof_rx=2, cell_id=21, rnti=cfg.rnti, tm=3, decoder_type=1, csi_enable=1,
                  max_nof_iterations=10)
    ncall = 2
    pay = np.zeros((ncall * 2, cfg.tbs[0] // 8 + 8), np.uint8)
    crc = np.zeros(2 * ncall, np.int32)
    its = np.zeros(2 * ncall, np.float32)
    rvs = np.zeros(ncall, np.int32)
    r = L.caller_pdsch_decode(C.byref(c), cfg.sf_idx, cfg.cfi, C.byref(g), grids.ctypes.data, ce.ctypes.data,
                              float(res["noise_estimate"]), ncall, rvs.ctypes.data, pay.ctypes.data, crc.ctypes.data,
                              its.ctypes.data)
    assert r == 0
    for t in range(2):
        nb = cfg.tbs[t] // 8
        assert crc[t] == 1, t
        assert np.array_equal(pay[t, :nb], payload[t][:nb]), t
    assert its[0] > 0
    # second call on the same softbuffers: every code block is skipped (cb_crc) and its bytes "restored" from the
    # softbuffer, but sch.c:476-483 saves them only when the TB failed, so the reference's TB CRC fails here
    assert crc[2] == 0 and crc[3] == 0 and its[2] == 0 and its[3] == 0


def test_tti_latency_flow_decodes_every_tti():
    """caller_tti_latency (srsUE's per-TTI worker flow, bench.py's dropin_tti_latency field): 10 distinct TM4
    subframes cycled over 30 TTIs, every TB decodes, every stage timed."""
    L = _caller()
    case = CASES[0]
    name, nprb, ports, nrx, tm, fmt, mcs, alt, cid = case
    rnti = 0x46
    iq, _expect = _synth(case, list(range(10)), rnti)
    c = CallerCfg(nof_prb=nprb, nof_ports=ports, nof_rx=nrx, cell_id=cid, rnti=rnti, tm=tm, use_tbs_index_alt=int(alt),
                  decoder_type=1, csi_enable=1, max_nof_iterations=10, cfo_estimate_enable=1, estimator_alg=0,
                  noise_alg=0, sync_error_enable=0)
    n = 30
    us = np.zeros((n, 3), np.float32)
    ok = np.zeros(n, np.int32)
    assert L.caller_tti_latency(C.byref(c), iq.ctypes.data, 10, 2, n, us.ctypes.data, ok.ctypes.data) == 0
    assert np.all(ok == 2), ok
    assert np.all(us > 0) and np.all(np.isfinite(us))


def test_concurrent_workers_match_single_thread():
    """srsUE runs up to 3 sf_worker threads, each calling the ue_dl / pdsch API on its own srslte_ue_dl_t at the same
    time (srsue/src/phy/phy.cc:135-189, sf_worker.cc:182, thread_pool.cc:215-230).  Three host threads, each with its
    own objects and softbuffers (caller_ue_dl: decode_pdsch, pdsch_decode on host copies, find_and_decode), decode
    distinct TM4 subframes concurrently while a fourth runs srslte_tdec_run_all on the reference goldens: every
    outcome and payload equals the single-thread run's.  ctypes releases the GIL around each foreign call, so the
    drop-in really is entered from several threads at once."""
    import threading
    L = _caller()
    case = CASES[0]
    name, nprb, ports, nrx, tm, fmt, mcs, alt, cid = case
    rnti = 0x46
    groups = [[10 * 3 + 1, 10 * 3 + 4, 10 * 4 + 8], [10 * 5 + 2, 10 * 5 + 5, 10 * 6 + 7], [10 * 6 + 0, 10 * 7 + 6, 10 * 8 + 9]]
    synth = [_synth(case, g, rnti) for g in groups]
    c = CallerCfg(nof_prb=nprb, nof_ports=ports, nof_rx=nrx, cell_id=cid, rnti=rnti, tm=tm, use_tbs_index_alt=int(alt),
                  decoder_type=1, csi_enable=1, max_nof_iterations=10, cfo_estimate_enable=1, estimator_alg=0,
                  noise_alg=0, sync_error_enable=0)
    maxb = max(t for _iq, ex in synth for e in ex for t in e[0].tbs) // 8 + 16

    def run(k, out):
        iq, _ex = synth[k]
        nsf = iq.shape[0]
        pay = np.zeros((nsf, 3, 2, maxb), np.uint8)
        res = (SfRes * nsf)()
        tt = np.array(groups[k], np.uint32)
        rc = L.caller_ue_dl(C.byref(c), iq.ctypes.data, tt.ctypes.data, nsf, pay.ctypes.data, maxb, res)
        out[k] = (rc, pay, [(r.ret_pdsch, r.ret_host, r.ret_fad, tuple(r.crc), tuple(r.crc_host), tuple(r.ack_fad))
                            for r in res])

    single = {}
    for k in range(3):
        run(k, single)
    auto = tdec_auto_cases()
    tdec_bad = []

    def tdec_loop():
        for _ in range(3):
            for cs in auto:
                K, trace = cs["K"], cs["trace"]
                buf = np.ascontiguousarray(cs["buf"].astype(np.int16))
                out = np.zeros(K // 8, np.uint8)
                n = C.c_int(0)
                if L.caller_tdec_run_all(buf.ctypes.data, out.ctypes.data, K, len(trace), 0, C.byref(n)) != 0 or \
                        not np.array_equal(out, trace[-1]):
                    tdec_bad.append(K)

    for rep in range(2):
        conc = {}
        th = [threading.Thread(target=run, args=(k, conc)) for k in range(3)] + [threading.Thread(target=tdec_loop)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in th), "a worker thread hung"
        assert not tdec_bad, tdec_bad
        for k in range(3):
            rc, pay, outc = conc[k]
            assert rc == 0 and outc == single[k][2], (rep, k, outc, single[k][2])
            assert np.array_equal(pay, single[k][1]), (rep, k)
            _iq, ex = synth[k]
            for i, (cfg, payload, g, m) in enumerate(ex):
                for t in range(cfg.nof_tb):
                    nb = cfg.tbs[t] // 8
                    assert outc[i][3][t] and outc[i][5][t], (rep, k, i, t)
                    for j in range(3):
                        assert np.array_equal(pay[i, j, t, :nb], payload[t][:nb]), (rep, k, i, j, t)
