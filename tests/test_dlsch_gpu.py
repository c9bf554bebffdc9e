"""GPU parity of the batched DL-SCH decoder (rate dematching + turbo with CRC early stop + TB CRC)
against the oracle's restatement of decode_tb (sch.c:363-570), whose rate matcher, decoder and CRC are
pinned to the compiled reference by tests/golden/.  Bit-exact: return codes, payload bytes (including the
trailing CB-CRC bytes), average iteration counts, HARQ softbuffer evolution."""
import numpy as np
import pytest

import oracle
from srsran_amd import check, lib
from srsran_amd.dlsch import Dlsch, SoftbufferPool

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[512, 0], ids=["latency", "throughput"], autouse=True)
def dlsch_path(request):
    """Every test on both turbo paths: the latency path (tdec_win_lat: a wave per code block, all half-iterations in
    one launch, for calls of at most 512 code blocks) and the half-iteration-per-launch throughput path."""
    from srsran_amd import lib
    old = lib().mi355_dlsch_set_latency_path(request.param)
    yield
    lib().mi355_dlsch_set_latency_path(old)

# (tbs, Qm, G, snr_db): SISO QPSK MCS9 (C=3, K=5312), TM4 QAM256 MCS27 codeword (C=16, K=6144),
# gamma != 0 cases, 16-window and 8-window and generic single-CB sizes
CASES = [(15840, 2, 30000, 3.0), (97896, 8, 115200, 9.0), (97896, 8, 115200, 5.5), (30576, 6, 36300, 4.5),
         (1000, 2, 3010, 1.0), (456, 2, 1500, 0.5), (40, 2, 200, -1.0), (6120, 4, 14402, 2.0),
         (75376, 6, 86400, 5.0), (2600, 2, 7800, 0.0),
         # E several times the circular buffer (rate-dematching wrap-around sums): the SIB sizes of the real signal
         (144, 2, 1080, 0.0), (256, 2, 1080, -2.0), (40, 2, 600, -3.0)]


def _oracle(llrs, cases, rvs, max_its, sbs):
    out = []
    for i, (tbs, Qm, G, _) in enumerate(cases):
        out.append(oracle.dlsch_decode_tb(llrs[i], tbs, Qm, rvs[i], max_its, sbs[i]))
    return out


def _check(got, want, cases):
    rets, datas, its = got
    for i, (tbs, *_r) in enumerate(cases):
        r, d, a = want[i]
        C = oracle.cbsegm(tbs)["C"]
        n = tbs // 8 + (6 if C > 1 else 3)
        assert rets[i] == r, (i, tbs)
        np.testing.assert_array_equal(datas[i][:n], d[:n], err_msg=f"tb {i} tbs={tbs}")
        assert abs(its[i] - a) < 1e-5, (i, its[i], a)


@pytest.mark.parametrize("max_its", [1, 4, 10])
def test_dlsch_batch_matches_oracle(max_its):
    rng = np.random.default_rng(100 + max_its)
    llrs = [oracle.make_tb(rng, t, q, g, 0, snr)[1] for (t, q, g, snr) in CASES]
    dl = Dlsch(0, max_its)
    pool = SoftbufferPool(len(CASES), 32)
    got = dl.decode(pool, [dict(tbs=t, Qm=q, rv=0, softbuffer=i) for i, (t, q, g, s) in enumerate(CASES)], llrs)
    want = _oracle(llrs, CASES, [0] * len(CASES), max_its, [oracle.Softbuffer() for _ in CASES])
    _check(got, want, CASES)
    assert any(r == 0 for r in got[0]) and any(r == -1 for r in got[0])


def test_dlsch_harq_retransmission_matches_oracle():
    rng = np.random.default_rng(7)
    cases = [(97896, 8, 115200, 4.0), (15840, 2, 30000, 0.0), (30576, 6, 36300, 2.5)]
    dl = Dlsch(0, 8)
    pool = SoftbufferPool(len(cases), 32)
    sbs = [oracle.Softbuffer() for _ in cases]
    payload_llr = []
    for t, q, g, snr in cases:
        bits = rng.integers(0, 2, t, dtype=np.uint8)
        payload_llr.append(bits)
    for rv in (0, 2, 3, 1):
        llrs = []
        for (t, q, g, snr), bits in zip(cases, payload_llr):
            coded = oracle.dlsch_encode_tb(bits, t, q, g, rv)
            y = np.where(coded.astype(bool), 1.0, -1.0) + 10 ** (-snr / 20) * rng.standard_normal(g)
            llrs.append(np.trunc(100 * y).clip(-32768, 32767).astype(np.int16))
        got = dl.decode(pool, [dict(tbs=t, Qm=q, rv=rv, softbuffer=i) for i, (t, q, g, s) in enumerate(cases)],
                        llrs)
        want = _oracle(llrs, cases, [rv] * len(cases), 8, sbs)
        _check(got, want, cases)


def test_dlsch_invalid_and_empty():
    dl = Dlsch(0, 4)
    pool = SoftbufferPool(2, 4)
    e = np.zeros(1000, np.int16)
    # tbs 97896 needs 16 CBs > max_cb 4 -> invalid; tbs 0 -> success with nothing decoded
    rets, _, _ = dl.decode(pool, [dict(tbs=97896, Qm=8, rv=0, softbuffer=0), dict(tbs=0, Qm=2, rv=0, softbuffer=1)],
                           [e, e])
    assert rets == [-2, 0]


@pytest.mark.parametrize("max_its", [2, 3, 6])
def test_dlsch_speculative_dec2_matches_oracle(max_its):
    """Speculative DEC2 half-iterations (dlsch_runtime.cpp spec_policy): the a-priori of the next DEC1 is written only
    by a rerun for the code blocks the check leaves unfinished, and the policy follows the previous batch.  Batches of
    the mixed cases alternate with all-high-SNR ones on one decoder, so the rerun runs with many, few and no blocks
    and the policy changes between calls; every batch must still be the oracle's."""
    dl = Dlsch(0, max_its)
    pool = SoftbufferPool(len(CASES), 32)
    hi = [(t, q, g, 30.0) for (t, q, g, _s) in CASES]
    for k, cases in enumerate((CASES, hi, hi, CASES, hi)):
        rng = np.random.default_rng(1000 * max_its + k)
        llrs = [oracle.make_tb(rng, t, q, g, 0, snr)[1] for (t, q, g, snr) in cases]
        pool.reset_all()
        got = dl.decode(pool, [dict(tbs=t, Qm=q, rv=0, softbuffer=i) for i, (t, q, g, s) in enumerate(cases)], llrs)
        want = _oracle(llrs, cases, [0] * len(cases), max_its, [oracle.Softbuffer() for _ in cases])
        _check(got, want, cases)


def test_dlsch_many_distinct_tb_sizes_one_call():
    """the TB epilogue's per-size CRC factor tables (dlsch_runtime.cpp tb_crc_scales) must stay valid for
    every TB planned in a call.  530 distinct TB sizes (more than the old 512-entry cap) in one batch, then the first
    100 again in a second call; every TB passes its CRC with the transmitted payload.  Sizes: no filler bits and one
    code-block size per TB (the reference's TX orders mixed K+/K- blocks K- first and its RX K+ first, sch.c:255-265 vs
    :387, so mixed-size TBs do not decode in the reference either), 40 .. 275,608 bits, 1 to 46 code blocks."""
    sizes = []
    t = 40
    while len(sizes) < 530:
        sg = oracle.cbsegm(t)
        if sg["F"] == 0 and sg["C2"] == 0:
            sizes.append(t)
        t += 8
    rng = np.random.default_rng(512)
    dl = Dlsch(0, 6)
    pool = SoftbufferPool(len(sizes), 46)
    for call, sz in enumerate((sizes, sizes[:100])):
        pays, llrs = [], []
        for t in sz:
            p, e = oracle.make_tb(rng, t, 2, 3 * t + 120, 0, 20.0)
            pays.append(p)
            llrs.append(e)
        pool.reset_all()
        rets, datas, _its = dl.decode(pool, [dict(tbs=t, Qm=2, rv=0, softbuffer=i) for i, t in enumerate(sz)], llrs)
        assert rets == [0] * len(sz), (call, [i for i, r in enumerate(rets) if r != 0][:8])
        for i, t in enumerate(sz):
            np.testing.assert_array_equal(datas[i][: t // 8], pays[i][: t // 8], err_msg=f"call {call} tbs {t}")


@pytest.mark.parametrize("kind", ["reset", "reset_range", "reset_tbs_batch"])
def test_null_stream_reset_done_before_decode(kind):
    """dlsch.h: a softbuffer reset given stream NULL has completed when the call returns.  The null stream does not
    order against the decoder's own (non-blocking) stream, so a reset left pending there could land after the next
    decode's rate dematcher read the CB CRC flags: that decode would skip every code block as already passed and
    return the previous TB (profiles/r05/reset_race).  Each round: a clean TB decodes into softbuffer 0 (its flags
    set), the raw C reset with NULL (no device sync around it), then pure-noise LLRs decode into the same softbuffer
    at once; the result must be the oracle's decode of the noise from a fresh softbuffer (CRC failure)."""
    import ctypes as C
    L = lib()
    L.mi355_softbuffer_reset_range.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.mi355_softbuffer_reset_tbs_batch.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                                   C.c_uint32, C.c_void_p]
    tbs, Qm, G = 15840, 2, 30000
    rng = np.random.default_rng(77)
    dl = Dlsch(0, 4)
    pool = SoftbufferPool(2, 32)
    desc = [dict(tbs=tbs, Qm=Qm, rv=0, softbuffer=0)]
    for rnd in range(6):
        pay, good = oracle.make_tb(rng, tbs, Qm, G, 0, 20.0)
        pool.reset(0)
        r, d, _ = dl.decode(pool, desc, [good])
        assert r == [0] and np.array_equal(d[0][: tbs // 8], pay[: tbs // 8]), rnd
        if kind == "reset":
            check(L.mi355_softbuffer_reset(pool.h, 0, None), "softbuffer_reset")
        elif kind == "reset_range":
            check(L.mi355_softbuffer_reset_range(pool.h, 0, 2, None), "softbuffer_reset_range")
        else:
            sbs, tb = (C.c_uint32 * 1)(0), (C.c_uint32 * 1)(tbs)
            check(L.mi355_softbuffer_reset_tbs_batch(pool.h, sbs, tb, 1, None), "softbuffer_reset_tbs_batch")
        noise = rng.integers(-300, 301, G).astype(np.int16)
        got = dl.decode(pool, desc, [noise])
        want = _oracle([noise], [(tbs, Qm, G, 0.0)], [0], 4, [oracle.Softbuffer()])
        _check(got, want, [(tbs, Qm, G, 0.0)])
        assert got[0] == [-1], (rnd, got[0])
