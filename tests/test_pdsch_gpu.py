"""GPU parity of the batched PDSCH receiver (mi355_pdsch_decode_batch / mi355_pdsch_frontend) against the
oracle's restatement of srslte_pdsch_decode (oracle/pdsch_chain.py over the oracle C stages, themselves
pinned to the compiled reference by tests/golden/pdsch_stages.npz).

Parity (north star: bit-exact decoded bits / CRCs, soft values within 1e-4):
  * equalised symbols, CSI and LLRs: BIT-EXACT against the oracle.  Both evaluate the reference's exact
    (non-SIMD) fp32 formulas operation by operation in the same order, with correctly rounded division and
    no FMA contraction (-ffp-contract=off on both sides), so there is nothing left to differ.  (Against the
    reference's own AVX2 build the equaliser differs by its rcp approximation, <= 1e-3 relative: pinned in
    tests/test_pdsch_oracle.py.)
  * decoded payloads, CRC flags, iteration counts: identical to the oracle chain.
"""
import numpy as np
import pytest

import oracle
from oracle import pdsch_chain as pc
from srsran_amd import pdsch as P
from srsran_amd.dlsch import SoftbufferPool
from tests.pdsch_jobs import DevSubframe, cell_of

pytestmark = pytest.mark.gpu

CFGS = [
    pc.Cfg(nof_prb=25, nof_ports=1, nof_rx=1, scheme=0, nof_layers=1, qm=[2], tbs=[1480]),
    pc.Cfg(nof_prb=25, nof_ports=1, nof_rx=2, scheme=0, nof_layers=1, qm=[6], tbs=[8888], csi_enable=True),
    pc.Cfg(nof_prb=6, nof_ports=1, nof_rx=1, scheme=0, nof_layers=1, qm=[4], tbs=[776], sf_idx=0, cfi=3),
    pc.Cfg(nof_prb=100, nof_ports=1, nof_rx=2, scheme=0, nof_layers=1, qm=[8], tbs=[75376], csi_enable=True),
    pc.Cfg(nof_prb=50, nof_ports=2, nof_rx=2, scheme=1, nof_layers=2, qm=[4], tbs=[7992], sf_idx=0),
    pc.Cfg(nof_prb=15, nof_ports=2, nof_rx=1, scheme=1, nof_layers=2, qm=[2], tbs=[1480], sf_idx=5, csi_enable=True),
    pc.Cfg(nof_prb=50, nof_ports=2, nof_rx=2, scheme=2, nof_layers=2, qm=[8, 8], tbs=[19848, 19848],
           csi_enable=True),
    pc.Cfg(nof_prb=50, nof_ports=2, nof_rx=2, scheme=2, nof_layers=2, qm=[6, 4], tbs=[11960, 7992], pmi=1),
    pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, scheme=2, nof_layers=2, qm=[2, 6], tbs=[1480, 5992], pmi=0,
           csi_enable=True),
    pc.Cfg(nof_prb=15, nof_ports=2, nof_rx=2, scheme=2, nof_layers=1, qm=[4], tbs=[2984], pmi=3, csi_enable=True),
    pc.Cfg(nof_prb=15, nof_ports=2, nof_rx=2, scheme=2, nof_layers=1, qm=[2], tbs=[1480], pmi=0),
    pc.Cfg(nof_prb=15, nof_ports=2, nof_rx=2, scheme=3, nof_layers=2, qm=[2, 2], tbs=[1480, 1480], sf_idx=5),
    pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, scheme=1, nof_layers=2, qm=[6], tbs=[6968], power_scale=True,
           p_a=-3.0, p_b=1),
    pc.Cfg(nof_prb=25, nof_ports=1, nof_rx=1, scheme=0, nof_layers=1, qm=[4], tbs=[4008], power_scale=True,
           p_a=-6.0, p_b=2, csi_enable=True),
    pc.Cfg(nof_prb=27, nof_ports=2, nof_rx=2, scheme=2, nof_layers=2, qm=[4, 4], tbs=[5992, 5992], pmi=1,
           sf_idx=0, csi_enable=True, mmse=False),
]


def _stage_check(pd, k, cfg, sf, job=0, predecoder=None):
    d_o, csi_o, e_o = pc.rx_front(cfg, sf.y, sf.ce, sf.noise, predecoder=predecoder)
    nre = sf.nof_re
    ncw = cfg.nof_layers if cfg.scheme in (2, 3) else 1
    for cw in range(ncw):
        qm = cfg.qm[cw] if cw < cfg.nof_tb else 2
        d, csi, e = pd.stage(job, cw, nre, nre * qm if cw < cfg.nof_tb else None)
        bad = d.view(np.uint64) != d_o[cw].view(np.uint64)
        assert not bad.any(), (k, cw, int(bad.sum()), (d - d_o[cw])[bad][:4], d_o[cw][bad][:4])
        np.testing.assert_array_equal(csi.view(np.uint32), csi_o[cw][:nre].view(np.uint32), err_msg=f"csi {k} {cw}")
        if cw < cfg.nof_tb:
            np.testing.assert_array_equal(e, e_o[cw], err_msg=f"cfg {k} cw {cw}")


@pytest.mark.parametrize("k", range(len(CFGS)))
def test_frontend_matches_oracle(k):
    cfg = CFGS[k]
    sf = pc.synth_subframe(cfg, np.random.default_rng(700 + k), snr_db=25)
    ds = DevSubframe(cfg, sf)
    pd = P.Pdsch(cell_of(cfg), cfg.nof_rx)
    assert ds.job.cfg.grant.nof_re == sf.nof_re
    pd.frontend([ds.job])
    _stage_check(pd, k, cfg, sf)


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("k", range(len(CFGS)))
def test_frontend_matches_reference_scalar_equaliser(k):
    """The GPU's equalised symbols, CSI and LLRs against the same chain with the equaliser taken from the COMPILED
    reference (oracle/_ref: srslte_predecoding_type in chunks below one AVX2 vector, i.e. its exact-division scalar
    path, precoding.c / mat.c) instead of the oracle restatement: bit-exact, every scheme of CFGS."""
    cfg = CFGS[k]
    sf = pc.synth_subframe(cfg, np.random.default_rng(700 + k), snr_db=25)
    ds = DevSubframe(cfg, sf)
    pd = P.Pdsch(cell_of(cfg), cfg.nof_rx)
    pd.frontend([ds.job])
    _stage_check(pd, k, cfg, sf, predecoder=oracle.ref_predecode_scalar)


def test_decode_batch_matches_oracle():
    """One batch with every configuration of CFGS (one cell per Pdsch object: group by cell)."""
    rng = np.random.default_rng(42)
    groups = {}
    for k, cfg in enumerate(CFGS):
        groups.setdefault((cfg.nof_prb, cfg.nof_ports, cfg.cell_id, cfg.nof_rx), []).append(k)
    for key, ks in groups.items():
        pool = SoftbufferPool(2 * len(ks), max_cb=16)
        subs = []
        for j, k in enumerate(ks):
            cfg = CFGS[k]
            sf = pc.synth_subframe(cfg, rng, snr_db=28)
            subs.append(DevSubframe(cfg, sf, softbuffers=(2 * j, 2 * j + 1)))
        pd = P.Pdsch(cell_of(CFGS[ks[0]]), CFGS[ks[0]].nof_rx)
        res = pd.decode(pool, [s.job for s in subs])
        for j, (k, s) in enumerate(zip(ks, subs)):
            cfg = s.cfg
            # the DL-SCH part is bit-exact: decode the GPU's own LLRs with the oracle (the front-end parity is
            # test_frontend_matches_oracle's business)
            e_g = [pd.stage(j, t, s.sf.nof_re, s.sf.nof_re * cfg.qm[t])[2] for t in range(cfg.nof_tb)]
            want = pc.rx_decode(cfg, e_g, [oracle.Softbuffer() for _ in cfg.tbs])
            for t in range(cfg.nof_tb):
                r = res[2 * j + t]
                ret, data, its = want[t]
                assert r.ret == 0
                assert bool(r.crc) == (ret == 0), (k, t)
                assert r.crc, (k, t)  # 28 dB: every configuration decodes
                n = cfg.tbs[t] // 8
                np.testing.assert_array_equal(s.payload_bytes(t)[:n], s.sf.payload[t], err_msg=f"cfg {k} tb {t}")
                np.testing.assert_array_equal(s.payload_bytes(t)[:n], data[:n])
                assert abs(r.avg_iterations_block - its) < 1e-5


def test_harq_retransmissions_match_oracle():
    """Low SNR: rv 0, 2, 3, 1 accumulate in the device softbuffer exactly like the oracle's."""
    base = pc.Cfg(nof_prb=50, nof_ports=2, nof_rx=2, scheme=2, nof_layers=2, qm=[6, 6], tbs=[25456, 25456],
                  csi_enable=True)
    pool = SoftbufferPool(2, max_cb=16)
    pd = P.Pdsch(cell_of(base), 2)
    sbs = [oracle.Softbuffer(), oracle.Softbuffer()]
    rng = np.random.default_rng(9)
    bits = [rng.integers(0, 2, t, dtype=np.uint8) for t in base.tbs]
    res_in = None
    for step, rv in enumerate((0, 2, 3, 1)):
        cfg = pc.Cfg(**{**base.__dict__, "rv": [rv, rv]})
        sf = pc.synth_subframe(cfg, rng, snr_db=9.0, payload_bits=bits)
        ds = DevSubframe(cfg, sf, softbuffers=(0, 1))
        res = pd.decode(pool, [ds.job], res_in)
        for t in range(2):
            if res_in is not None and res_in[t].crc:
                continue
            e_g = pd.stage(0, t, sf.nof_re, sf.nof_re * cfg.qm[t])[2]
            ret, data, its = oracle.dlsch_decode_tb(e_g, cfg.tbs[t], cfg.qm[t], rv, 10, sbs[t])
            assert bool(res[t].crc) == (ret == 0), (step, t)
            assert abs(res[t].avg_iterations_block - its) < 1e-5
            if ret == 0:
                np.testing.assert_array_equal(ds.payload_bytes(t)[: cfg.tbs[t] // 8], data[: cfg.tbs[t] // 8])
        res_in = res


def test_invalid_configs_rejected():
    cfg = pc.Cfg(nof_prb=25, nof_ports=1, nof_rx=1, scheme=0, nof_layers=1, qm=[2], tbs=[1480])
    sf = pc.synth_subframe(cfg, np.random.default_rng(1), snr_db=20)
    ds = DevSubframe(cfg, sf)
    pd = P.Pdsch(cell_of(cfg), 1)
    pool = SoftbufferPool(2, max_cb=4)
    bad = P.PdschJob.from_buffer_copy(ds.job)
    bad.cfg.grant.nof_re += 1  # "Error expecting %d symbols but got %d"
    with pytest.raises(RuntimeError):
        pd.decode(pool, [bad])
    bad = P.PdschJob.from_buffer_copy(ds.job)
    bad.cfg.grant.tx_scheme = P.TXSCHEME_SPATIALMUX  # 1 port: predecoding error
    with pytest.raises(RuntimeError):
        pd.decode(pool, [bad])


@pytest.mark.parametrize("k", [k for k, c in enumerate(CFGS) if c.scheme in (0, 2)])
def test_ce_invariant_matches_per_symbol_path(k):
    """mi355_pdsch_set_ce_invariant (the drop-in sets it on its own AVERAGE estimates): estimates equal in every OFDM
    symbol decoded through the fused equaliser (row 0 read) and through the per-symbol two-kernel path -- the same
    CRCs, iteration counts, payloads and decoder buffers."""
    from srsran_amd import lib
    import ctypes as C
    cfg = CFGS[k]
    sf = pc.synth_subframe(cfg, np.random.default_rng(900 + k), snr_db=26, channel="static")
    out = []
    for inv in (False, True):
        ds = DevSubframe(cfg, sf)
        pool = SoftbufferPool(2, max_cb=16)
        pd = P.Pdsch(cell_of(cfg), cfg.nof_rx)
        pd.set_ce_invariant(inv)
        res = pd.decode(pool, [ds.job])
        pool.materialize()
        buf, stride, mcb = C.POINTER(C.c_int16)(), C.c_uint32(), C.c_uint32()
        L = lib()
        L.mi355_softbuffer_pool_buffer.argtypes = [C.c_void_p, C.POINTER(C.POINTER(C.c_int16)),
                                                   C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.mi355_softbuffer_pool_buffer(pool.h, C.byref(buf), C.byref(stride), C.byref(mcb))
        sb = np.zeros((2 * mcb.value, stride.value), np.int16)
        L.mi355_memcpy_d2h(sb.ctypes.data, C.cast(buf, C.c_void_p).value, sb.nbytes)
        out.append(([(int(res[t].crc), res[t].avg_iterations_block) for t in range(cfg.nof_tb)],
                    [ds.payload_bytes(t)[:cfg.tbs[t] // 8] for t in range(cfg.nof_tb)], sb))
        pool.close()
    assert out[0][0] == out[1][0], (k, out[0][0], out[1][0])
    assert all(c for c, _ in out[0][0]), k  # 26 dB, static channel: every TB decodes
    for t in range(cfg.nof_tb):
        np.testing.assert_array_equal(out[0][1][t], out[1][1][t], err_msg=f"cfg {k} tb {t}")
        np.testing.assert_array_equal(out[1][1][t], sf.payload[t][:cfg.tbs[t] // 8], err_msg=f"cfg {k} tb {t}")
    for t in range(cfg.nof_tb):  # the TB's code blocks (slots t * max_cb + c), decoder buffer 3 (K + 32) + 12
        sg = oracle.cbsegm(cfg.tbs[t])
        for c in range(sg["C"]):
            n = 3 * ((sg["K1"] if c < sg["C1"] else sg["K2"]) + 32) + 12
            np.testing.assert_array_equal(out[0][2][16 * t + c, :n], out[1][2][16 * t + c, :n],
                                          err_msg=f"cfg {k} tb {t} cb {c} decoder buffer")
