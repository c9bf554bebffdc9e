"""CPU: the oracle (and the product's host-side RE map) pinned to the compiled reference where the reference's own
code for a stage compiles here (tests/golden/ref_pins.npz, made by ``tests/golden/make_golden.py pins`` from
oracle/_ref):

  * equaliser (a5): oracle.predecode == the reference's scalar path of srslte_predecoding_type, BIT-EXACT, over full
    100-PRB vectors (14,400 REs) for every branch srslte_pdsch_decode takes -- SISO (precoding.c:309-357 tail),
    SFBC, TM4 2x2 MMSE codebooks 0-2 (:1519-1548 -> mat.c:63-109), 2x1 MRC codebooks 0-3 (:1802-1820), CDD, MMSE
    and ZF.  The reference's SIMD bodies use rcp_ps (host-CPU dependent, <= 1e-3: tests/test_pdsch_oracle.py);
    the scalar path is the exact-division arithmetic the product and the oracle evaluate;
  * RE extraction (a3): oracle.pdsch_re_map == product mi355_pdsch_re_map == the map through the reference's
    compiled prb_dl.c primitives (prb_cp_ref / prb_cp / prb_cp_half, oracle/ref/ref_prb.c) for 6-110 PRB x 1/2/4
    ports x 5 cell ids x CFI 1-3 x subframes 0/1/5/6 x FDD/TDD, full and partial allocations;
  * estimator smoothing filters (a2): oracle.chest_filter == chest_common.c's Gauss and 3-tap filters, bit-exact.

The fixtures hold SHA-256 digests of the reference outputs plus the equaliser's first 64 values; inputs are
regenerated from their seeds and their digests checked first, so a numpy RNG change is told apart from a numeric
mismatch.  Where oracle/_ref is built (this container), the same comparisons also run live against it.
"""
import hashlib
import os
import sys

import numpy as np
import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden as mg  # noqa: E402

GOLD = os.path.join(HERE, "golden", "ref_pins.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD)


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("k", range(len(mg.PIN_CASES)))
def test_equaliser_full_size_bit_exact_vs_reference_scalar(g, k):
    scheme, ports, rx, layers, cb, scaling, noise = mg.PIN_CASES[k]
    y, h = mg.pin_inputs(9000 + k, scheme, ports, rx, mg.PIN_N)
    assert _sha(y) + _sha(h) == str(g[f"eq{k}_in_sha"]), "input regeneration changed (numpy RNG), not a numeric diff"
    x, csi = oracle.predecode(y, h, layers, cb, scheme, scaling, noise)
    used = 2 if (layers == 2 and scheme >= 2) else 1
    np.testing.assert_array_equal(x[:, :64].view(np.uint32), g[f"eq{k}_x_head"].view(np.uint32))
    np.testing.assert_array_equal(csi[:used, :64].view(np.uint32), g[f"eq{k}_csi_head"].view(np.uint32))
    assert _sha(x) == str(g[f"eq{k}_x_sha"]), k
    assert _sha(csi[:used]) == str(g[f"eq{k}_csi_sha"]), k


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built")
def test_equaliser_live_vs_reference_scalar():
    """Fresh random inputs (other amplitudes, odd lengths) against the live reference scalar path."""
    rng = np.random.default_rng(77)
    for (scheme, ports, rx, layers, cb, scaling, noise) in mg.PIN_CASES:
        for n, amp in ((1206, 1.0), (614, 40.0), (300, 1e-3)):
            n -= n % 2 if scheme == 1 else 0
            y = (amp * (rng.standard_normal((rx, n)) + 1j * rng.standard_normal((rx, n)))).astype(np.complex64)
            h = (rng.standard_normal((ports, rx, n)) + 1j * rng.standard_normal((ports, rx, n))).astype(np.complex64)
            x, csi = oracle.predecode(y, h, layers, cb, scheme, scaling, noise)
            xr, cr = oracle.ref_predecode_scalar(y, h, layers, cb, scheme, scaling, noise)
            used = 2 if (layers == 2 and scheme >= 2) else 1
            np.testing.assert_array_equal(x.view(np.uint32), xr.view(np.uint32), err_msg=str((scheme, cb, n)))
            np.testing.assert_array_equal(csi[:used].view(np.uint32), cr[:used].view(np.uint32))


def test_re_map_oracle_and_product_vs_reference_prb_primitives(g):
    from srsran_amd import pdsch as P
    digests = g["map_sha"]
    assert digests.shape[0] == len(mg.PIN_MAPS)
    for k, (nof_prb, ports, cid, cfi, sf, tdd, seed) in enumerate(mg.PIN_MAPS):
        prb = mg.pin_alloc(nof_prb, seed)
        a = oracle.pdsch_re_map(nof_prb, ports, cid, prb, cfi + (nof_prb < 10), sf, tdd=bool(tdd))
        want = digests[k].tobytes().hex()
        assert _sha(a.astype(np.uint32)) == want, (nof_prb, ports, cid, cfi, sf, tdd, seed)
        if k % 7 == 0:  # the product's host map (C++), a sample of the cases
            cell = P.make_cell(nof_prb, ports, cid, 0, tdd)
            gr = P.make_grant(cell, prb, cfi, sf, 0, 1, [dict(qm=2, tbs=100)])
            b = P.re_map(cell, gr, cfi, sf)
            assert _sha(np.asarray(b, np.uint32)) == want, ("product", nof_prb, ports, cid, cfi, sf, tdd, seed)


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built")
def test_re_map_live_vs_reference_prb_primitives():
    rng = np.random.default_rng(5)
    for nof_prb in (6, 9, 13, 51, 99, 100):
        for ports in (1, 2, 4):
            for cfi in (1, 2, 3):
                for sf in range(10):
                    prb = (rng.random((2, nof_prb)) < 0.5).astype(np.uint8)
                    prb[1] = prb[0] if sf % 2 else prb[1]  # distributed-style per-slot allocations too
                    cid = int(rng.integers(0, 504))
                    a = oracle.pdsch_re_map(nof_prb, ports, cid, prb, cfi + (nof_prb < 10), sf)
                    b = oracle.ref_pdsch_re_map(nof_prb, ports, cid, prb, cfi + (nof_prb < 10), sf)
                    np.testing.assert_array_equal(a, b, err_msg=str((nof_prb, ports, cid, cfi, sf)))


def test_smoothing_filters_vs_reference_chest_common(g):
    for order in range(1, 15):
        for j, sd in enumerate((0.1, 0.5, 1.0, 2.0, 3.7, 10.0)):
            got = oracle.chest_filter(0, float(order), sd)
            np.testing.assert_array_equal(got.view(np.uint32), g[f"gauss{order}_{j}"].view(np.uint32),
                                          err_msg=f"gauss order {order} sigma {sd}")
    for j, w in enumerate((0.0, 0.1, 0.25, 0.3333)):
        np.testing.assert_array_equal(oracle.chest_filter(1, w, 0.0), g[f"tri3_{j}"])


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built")
def test_smoothing_filter_auto_sigma_live():
    """filter_coef[0] <= 0: order 4, sigma = 200 x noise (chest_dl.c:641-645 -> chest_common.c:70-88)."""
    for noise in (1e-4, 3e-3, 0.01, 0.2):
        got = oracle.chest_filter(0, 0.0, 0.0, noise)
        want = oracle.ref_chest_filter(0, 4, noise * 200.0)
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg=str(noise))


@pytest.mark.skipif(not oracle.ref_available(), reason="oracle/_ref not built")
@pytest.mark.parametrize("snr_db", [5.5, 5.7, 5.9, 6.0, 7.0, 9.0])
def test_reference_early_stop_matches_oracle_decode_tb(snr_db):
    """oracle.ref_dlsch_decode_cbs (bench's crc_parity_vs_avx2 checker: the reference's AVX2 decoder under sch.c's
    per-CB early stop) == the oracle's decode_tb restatement, on a TM4 QAM256 TB (C = 16, K = 6144) from the waterfall
    (some blocks fail) to the clean regime: TB CRC, payload, average half-iterations."""
    rng = np.random.default_rng(int(snr_db * 10))
    tbs, Qm, G = 97896, 8, 115200
    payload, llr = oracle.make_tb(rng, tbs, Qm, G, 0, snr_db)
    ret, data, its = oracle.dlsch_decode_tb(llr, tbs, Qm, 0, 10, oracle.Softbuffer())
    bufs = np.stack([oracle.rm_turbo_rx(llr[c * 7200:(c + 1) * 7200], 6144, 0) for c in range(16)])
    tb_ok, rdata, cb_ok, cb_its = oracle.ref_dlsch_decode_cbs(bufs, 6144, tbs, 10)
    assert tb_ok == (ret == 0)
    assert abs(cb_its.sum() / 16 - its) < 1e-5
    if tb_ok:
        assert np.array_equal(rdata[: tbs // 8], data[: tbs // 8]) and np.array_equal(rdata[: tbs // 8], payload)
