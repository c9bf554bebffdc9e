"""GPU: the DL-SCH decode in srsUE's pdsch_8bit_decoder mode (mi355_dlsch_decode8_dev: sch.c:403-423 with
llr_is_8bit) -- int8 LLRs, srslte_rm_turbo_rx_lut_8bit into the softbuffers, srslte_tdec_iteration_8bit with the
CB / TB CRC logic the 16-bit decode shares.  Its two stages are pinned to the reference's own 8-bit code by
tests/test_tdec8_gpu.py; here the orchestration is checked by composition (the decoded payload of a single-code-block
TB equals what the golden-pinned rate dematcher + 8-bit decoder give for its LLRs, iteration count included),
end to end (multi-CB TBs of both 8-bit window decoders and the K <= 400 fallback decode their payloads, HARQ
combining over rv 0, 2 rescues a failing first transmission), and on the rejected K range."""
import numpy as np
import pytest

import oracle
from srsran_amd.dlsch import Dlsch, SoftbufferPool
from srsran_amd.tdec import DeviceBuffer, Tdec8Batch

pytestmark = pytest.mark.gpu


def llr8(coded: np.ndarray, snr_db: float, rng, amp: float = 20.0) -> np.ndarray:
    y = np.where(coded.astype(bool), 1.0, -1.0) + 10 ** (-snr_db / 20) * rng.standard_normal(coded.size)
    return np.clip(np.round(amp * y), -127, 127).astype(np.int8)


# (tbs, Qm, G): TM4 QAM256 codeword (C=16, K=6144) and C=3 K=5312 (32 windows), single-CB K=3008 (32 windows),
# K=6144, K=1024 (16 windows), K=280 (the 16-bit fallback)
CASES8 = [(97896, 8, 115200), (15840, 2, 30000), (2984, 2, 9000), (6120, 4, 14400), (1000, 2, 3010), (256, 2, 1080)]


def test_dlsch8_decodes_payloads():
    rng = np.random.default_rng(8)
    bits = [rng.integers(0, 2, t, dtype=np.uint8) for t, _, _ in CASES8]
    llrs = [llr8(oracle.dlsch_encode_tb(b, t, q, g, 0), 12.0, rng) for b, (t, q, g) in zip(bits, CASES8)]
    dl = Dlsch(0, 10)
    pool = SoftbufferPool(len(CASES8), 32)
    rets, datas, its = dl.decode(pool, [dict(tbs=t, Qm=q, rv=0, softbuffer=i) for i, (t, q, g) in enumerate(CASES8)],
                                 llrs, llr8=True)
    for i, (t, q, g) in enumerate(CASES8):
        assert rets[i] == 0, (i, t, rets[i])
        np.testing.assert_array_equal(datas[i][: t // 8], np.packbits(bits[i]), err_msg=f"tbs={t}")
        assert 1 <= its[i] <= 10


def test_dlsch8_single_cb_composition():
    """C = 1 (tbs 6120 -> K = 6144): the decode equals rm_turbo_rx_lut_8bit + the 8-bit decoder run for the
    reported number of half-iterations, decision bytes identical."""
    rng = np.random.default_rng(81)
    t, q, g = 6120, 4, 14400
    K = 6144
    bits = rng.integers(0, 2, t, dtype=np.uint8)
    e = llr8(oracle.dlsch_encode_tb(bits, t, q, g, 1), 3.5, rng, amp=12.0)
    dl = Dlsch(0, 10)
    pool = SoftbufferPool(1, 4)
    rets, datas, its = dl.decode(pool, [dict(tbs=t, Qm=q, rv=1, softbuffer=0)], [e], llr8=True)
    nh = int(round(its[0]))
    t8 = Tdec8Batch()
    blen = 3 * (K + 32) + 12
    d_buf = DeviceBuffer(blen + 256).upload(np.zeros(blen + 256, np.int8))
    d_e = DeviceBuffer(e.size).upload(e)
    assert t8.rm_rx_dev(d_e.ptr, e.size, e.size, d_buf.ptr, blen, 1, K, 1) == 0
    d_out = DeviceBuffer(K // 8)
    assert t8.run_dev(d_buf.ptr, blen, 1, K, nh, d_out.ptr, K // 8) == 0
    dec = d_out.download(np.zeros(K // 8, np.uint8))
    np.testing.assert_array_equal(datas[0][: K // 8], dec)  # C = 1: the K bits (TB + CRC) at data[0]
    assert rets[0] == (0 if np.array_equal(np.unpackbits(dec)[:t], bits) else -1)


def test_dlsch8_harq_rescues_first_transmission():
    """rv 0 alone at code rate 1.3 cannot decode; rv 0 + rv 2 combined in the int8 softbuffer (rate 0.66) does."""
    rng = np.random.default_rng(82)
    t, q, g = 15840, 2, 12000
    bits = rng.integers(0, 2, t, dtype=np.uint8)
    dl = Dlsch(0, 8)
    pool = SoftbufferPool(1, 32)
    results = []
    for rv in (0, 2):
        e = llr8(oracle.dlsch_encode_tb(bits, t, q, g, rv), 10.0, rng, amp=20.0)
        rets, datas, _ = dl.decode(pool, [dict(tbs=t, Qm=q, rv=rv, softbuffer=0)], [e], llr8=True)
        results.append(rets[0])
    assert results[0] == -1 and results[1] == 0, results
    np.testing.assert_array_equal(datas[0][: t // 8], np.packbits(bits))


def test_dlsch8_rejects_unconverted_range():
    rng = np.random.default_rng(83)
    t, q, g = 456, 2, 1500  # K = 480: 400 < K <= 800
    e = llr8(oracle.dlsch_encode_tb(rng.integers(0, 2, t, dtype=np.uint8), t, q, g, 0), 10.0, rng)
    dl = Dlsch(0, 4)
    pool = SoftbufferPool(1, 4)
    rets, _, _ = dl.decode(pool, [dict(tbs=t, Qm=q, rv=0, softbuffer=0)], [e], llr8=True)
    assert rets[0] == -2
