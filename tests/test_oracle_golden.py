"""CPU: the oracle (our scalar C restatement) against the reference's golden vectors.

This pins the checker itself before any GPU result is compared with it."""
import numpy as np
import pytest

import oracle
from golden_io import load, tdec_auto_cases, tdec_generic_cases


@pytest.mark.parametrize("case", tdec_auto_cases(), ids=lambda c: f"K{c['K']}-{c['kind']}-{c['ebno']}")
def test_oracle_tdec_auto_matches_reference_every_half_iteration(case):
    K = case["K"]
    out, tr = oracle.tdec_run(case["buf"], K, case["trace"].shape[0], trace=True)
    np.testing.assert_array_equal(tr, case["trace"])
    np.testing.assert_array_equal(out, case["trace"][-1])


@pytest.mark.parametrize("case", tdec_generic_cases(), ids=lambda c: f"K{c['K']}")
def test_oracle_tdec_generic_matches_reference(case):
    out = oracle.tdec_run_generic(case["lin"], case["K"], case["trace"].shape[0])
    np.testing.assert_array_equal(out, case["trace"][-1])


def test_golden_decodes_at_high_snr():
    # sanity of the fixtures themselves: the 4 dB (test units) AWGN cases are (nearly) error-free
    for c in tdec_auto_cases():
        if c["kind"] == "awgn" and c["ebno"] >= 4.0:
            assert np.mean(np.unpackbits(c["trace"][-1]) != c["bits"]) < 0.05, c["K"]


def test_tcod_known_answer():
    z = load("tcod_known.npz")
    enc = oracle.tcod_encode(z["known_data"], 504)
    np.testing.assert_array_equal(enc, z["ref_encoder_out"])
    # the reference's fixture differs from the reference encoder only in the first tail bit
    diff = np.nonzero(enc != z["known_data_encoded"])[0]
    assert list(diff) == list(z["fixture_vs_encoder_diff"]) == [1512]


def test_crc_and_cbsegm():
    z = load("crc_cbsegm.npz")
    polys = {"crc24a": oracle.CRC24A, "crc24b": oracle.CRC24B, "crc16": oracle.CRC16, "crc8": oracle.CRC8}
    for i in range(int(z["nmsg"])):
        m = z[f"msg{i}"]
        for name, po in polys.items():
            assert oracle.crc(m, 8 * m.size, po) == int(z[f"msg{i}_{name}"]), (i, name)
    for t, row in zip(z["tbs"], z["cbsegm"]):
        s = oracle.cbsegm(int(t))
        assert [s[k] for k in ("C", "K1", "K2", "C1", "C2", "F")] == [int(v) for v in row], t


def test_qpp_is_permutation_and_contention_free():
    for K in oracle.cb_sizes():
        pi = oracle.qpp(K).astype(np.int64)
        assert np.array_equal(np.sort(pi), np.arange(K))
        nsb = oracle.tdec_nsb(K)
        if nsb:
            L = K // nsb
            w = np.arange(nsb)
            for j in range(0, L, max(1, L // 7)):
                assert len(set(pi[w * L + j] // L)) == nsb  # windows read distinct windows


from golden_io import rm_cases, rm_harq, rm_init_softbuffer  # noqa: E402


@pytest.mark.parametrize("case", rm_cases(), ids=lambda c: f"K{c['K']}-rv{c['rv']}-E{c['e'].size}")
def test_oracle_rate_dematch_matches_reference(case):
    out = oracle.rm_turbo_rx(case["e"], case["K"], case["rv"], rm_init_softbuffer())
    np.testing.assert_array_equal(out[: case["out"].size], case["out"])


def test_oracle_rate_dematch_harq_accumulation():
    h = rm_harq()
    acc = oracle.rm_turbo_rx(h["e0"], h["K"], 0)
    oracle.rm_turbo_rx(h["e2"], h["K"], 2, acc)
    np.testing.assert_array_equal(acc[: h["out"].size], h["out"])


def test_tdec8_goldens_sane():
    """The 8-bit reference goldens: every high-SNR case decodes its transmitted bits after 2 half-iterations (the
    reference's 8-bit decoder is weaker than the 16-bit one and oscillates later), inputs are in the 8-bit layout."""
    z = load("tdec8.npz")
    hi = 0
    for i in range(int(z["ncases"])):
        K = int(z[f"c{i}_K"])
        assert z[f"c{i}_buf"].dtype == np.int8 and z[f"c{i}_buf"].size == 3 * (K + 32) + 12
        assert z[f"c{i}_trace"].shape == (int(z["nhalf"]), K // 8)
        if float(z[f"c{i}_ebno"]) >= 10.0:
            hi += 1
            assert (np.unpackbits(z[f"c{i}_trace"][1]) != z[f"c{i}_bits"]).mean() < 2e-3
    assert hi == 3


def test_llr8_restatement_matches_reference_goldens():
    """tests/llr8_ref.py (the checker of the GPU int8 LLR kernel) against srslte_demod_soft_demodulate_b and
    srslte_scrambling_sb_offset as the reference computes them (SIMD bodies, scalar tails, saturation, wrap)."""
    import oracle
    from tests import llr8_ref
    z = load("tdec8.npz")
    for k in range(int(z["dm_n"])):
        got = llr8_ref.demod_b(z[f"dm{k}_sym"], int(z[f"dm{k}_qm"]))
        np.testing.assert_array_equal(got, z[f"dm{k}_llr"], err_msg=f"demod case {k} qm={int(z[f'dm{k}_qm'])}")
    for k in range(int(z["sb_n"])):
        n = z[f"sb{k}_in"].size
        c = oracle.sequence_lte(int(z[f"sb{k}_cinit"]), n)
        np.testing.assert_array_equal(llr8_ref.scramble_sb(z[f"sb{k}_in"], c), z[f"sb{k}_out"])
