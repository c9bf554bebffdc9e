"""CPU: the oracle's PDSCH stage restatements against the compiled reference's golden vectors
(tests/golden/pdsch_stages.npz, made by tests/golden/make_golden.py from oracle/_ref), the product's host-side
RE extraction map against the oracle's, and the oracle TX/RX chain round trip.

  * demapper (demod_soft.c, AVX2 build) and descrambler: bit-exact;
  * equaliser (precoding.c/mat.c): the oracle states the exact formulas; the reference's SIMD bodies use
    an approximate reciprocal, so x and CSI agree within 1e-3 relative (the tolerance of the north star's
    soft-value parity is on LLRs: see test_pdsch_gpu.py), and BIT-EXACTLY where the reference takes its
    scalar path (n smaller than one AVX2 vector of 8 complex values; full 100-PRB vectors through that path in
    tests/test_ref_pins.py);
  * RE map (pdsch.c:83-228, not compilable here: it includes the generated srslte/version.h): product
    (C++) == oracle (C), two restatements, plus RE counts against an independent per-PRB formula.
"""
import os

import numpy as np
import pytest

import oracle
from oracle import pdsch_chain as pc

GOLD = os.path.join(os.path.dirname(__file__), "golden", "pdsch_stages.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD)


def test_demod_golden(g):
    for k in range(int(g["demod_n"])):
        qm = int(g[f"demod{k}_qm"])
        got = oracle.demod_soft_s(qm, g[f"demod{k}_sym"])
        np.testing.assert_array_equal(got, g[f"demod{k}_llr"], err_msg=f"case {k} qm={qm}")


def test_scrambling_golden(g):
    for k in range(int(g["scr_n"])):
        got = oracle.scramble_s(int(g[f"scr{k}_cinit"]), g[f"scr{k}_in"])
        np.testing.assert_array_equal(got, g[f"scr{k}_out"])


def test_predecoding_golden(g):
    for k in range(int(g["pre_n"])):
        scheme, ports, rx, layers, cb, n = [int(v) for v in g[f"pre{k}_cfg"]]
        scaling, noise = [float(v) for v in g[f"pre{k}_sc"]]
        x, csi = oracle.predecode(g[f"pre{k}_y"], g[f"pre{k}_h"], layers, cb, scheme, scaling, noise)
        xr, cr = g[f"pre{k}_x"], g[f"pre{k}_csi"]
        used = 2 if (layers == 2 and scheme >= 2) else 1
        if n < 8:  # the reference's scalar path: bit-exact
            np.testing.assert_array_equal(x.view(np.uint32), xr.view(np.uint32), err_msg=f"case {k}")
            np.testing.assert_array_equal(csi[:used].view(np.uint32), cr[:used].view(np.uint32), err_msg=f"case {k}")
            continue
        ex = np.abs(x - xr) / (np.abs(xr) + 1e-3)
        assert ex.max() < 1e-3, (k, scheme, layers, cb, n, ex.max())
        ec = np.abs(csi[:used] - cr[:used]) / (np.abs(cr[:used]) + 1e-3)
        assert ec.max() < 1e-3, (k, ec.max())


def test_gold_sequence_linear_form():
    """The product's Gold table factorises c(n) = x1(n+Nc) ^ <mask(n+Nc), c_init>: check the oracle's
    sequence is linear in c_init over GF(2) on top of the fixed x1 part (what the table relies on)."""
    n = 3000
    z = oracle.sequence_lte(0, n)
    a, b = 0x12345, 0x0abcdef
    ca, cb_, cab = oracle.sequence_lte(a, n), oracle.sequence_lte(b, n), oracle.sequence_lte(a ^ b, n)
    np.testing.assert_array_equal(ca ^ cb_ ^ z, cab)


def test_re_map_product_vs_oracle():
    from srsran_amd import pdsch as P
    rng = np.random.default_rng(0)
    for nof_prb in (6, 7, 15, 25, 27, 50, 75, 100):
        for ports in (1, 2, 4):
            for cid in (0, 1, 2, 5, 301):
                for cfi in (1, 2, 3):
                    for sf in (0, 1, 5, 6, 3):
                        for ft in (0, 1):
                            cell = P.make_cell(nof_prb, ports, cid, 0, ft)
                            prb = (rng.random((2, nof_prb)) < 0.6).astype(np.uint8)
                            prb[1] = prb[0]
                            gr = P.make_grant(cell, prb, cfi, sf, 0, 1, [dict(qm=2, tbs=100)])
                            a = P.re_map(cell, gr, cfi, sf)
                            b = oracle.pdsch_re_map(nof_prb, ports, cid, prb, cfi + (nof_prb < 10), sf, tdd=bool(ft))
                            np.testing.assert_array_equal(a, b)
                            assert np.unique(a).size == a.size


@pytest.mark.parametrize("ports,refs", [(1, 2), (2, 4), (4, 4)])
def test_re_count_formula(ports, refs):
    """Full allocation, FDD, a subframe without PSS/SSS/PBCH: per PRB, slot 0 has (7 - cfi) symbols minus the
    CRS of l=4 (and l=1 for 4 ports when not in the control region), slot 1 has 7 symbols minus CRS on
    l=0, l=4 (and l=1)."""
    from srsran_amd import pdsch as P
    cell = P.make_cell(50, ports, 3)
    prb = np.ones((2, 50), np.uint8)
    for cfi in (1, 2, 3):
        gr = P.make_grant(cell, prb, cfi, 3, 0, 1, [dict(qm=2, tbs=100)])
        s0 = (7 - cfi) * 12 - refs - (refs if (ports == 4 and cfi <= 1) else 0)
        s1 = 84 - 2 * refs - (refs if ports == 4 else 0)
        assert gr.nof_re == 50 * (s0 + s1)


CHAIN = [
    pc.Cfg(nof_prb=25, nof_ports=1, nof_rx=1, scheme=0, nof_layers=1, qm=[2], tbs=[1480]),
    pc.Cfg(nof_prb=25, nof_ports=1, nof_rx=2, scheme=0, nof_layers=1, qm=[6], tbs=[8888], csi_enable=True),
    pc.Cfg(nof_prb=50, nof_ports=2, nof_rx=2, scheme=1, nof_layers=2, qm=[4], tbs=[7992], sf_idx=0),
    pc.Cfg(nof_prb=50, nof_ports=2, nof_rx=2, scheme=2, nof_layers=2, qm=[8, 8], tbs=[19848, 19848],
           csi_enable=True),
    pc.Cfg(nof_prb=15, nof_ports=2, nof_rx=2, scheme=2, nof_layers=1, qm=[4], tbs=[2984], pmi=3),
    pc.Cfg(nof_prb=15, nof_ports=2, nof_rx=2, scheme=3, nof_layers=2, qm=[2, 2], tbs=[1480, 1480], sf_idx=5),
    pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, scheme=1, nof_layers=2, qm=[6], tbs=[6968], power_scale=True,
           p_a=-3.0, p_b=1),
]


@pytest.mark.parametrize("k", range(len(CHAIN)))
def test_oracle_chain_roundtrip(k):
    cfg = CHAIN[k]
    for t in cfg.tbs:
        assert pc.valid_tbs(t) == t
    sf = pc.synth_subframe(cfg, np.random.default_rng(50 + k), snr_db=30)
    _, _, e = pc.rx_front(cfg, sf.y, sf.ce, sf.noise)
    res = pc.rx_decode(cfg, e, [oracle.Softbuffer() for _ in cfg.tbs])
    for t, (ret, data, _its) in enumerate(res):
        assert ret == 0
        np.testing.assert_array_equal(data[: cfg.tbs[t] // 8], sf.payload[t])
