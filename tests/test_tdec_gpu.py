"""GPU parity: the HIP turbo decoder (through the C ABI) against the reference golden vectors and the
oracle.  Bit-exact: decision bytes must be identical after every half-iteration count, for passing and
failing code blocks, saturating and full-range inputs, every decoder regime (generic / 8 / 16 windows)."""
import numpy as np
import pytest

import oracle
import srsran_amd
from golden_io import tdec_auto_cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dec():
    d = srsran_amd.TdecBatch(0)
    yield d
    d.close()


def _stack(bufs, K):
    stride = srsran_amd.tdec_buf_len(K)
    a = np.zeros((len(bufs), stride), np.int16)
    for i, b in enumerate(bufs):
        a[i, : b.size] = b
    return a


def test_golden_every_half_iteration(dec):
    cases = tdec_auto_cases()
    byK = {}
    for c in cases:
        byK.setdefault(c["K"], []).append(c)
    for K, cs in byK.items():
        bufs = _stack([c["buf"] for c in cs], K)
        for nh in range(1, cs[0]["trace"].shape[0] + 1):
            out = dec.run(bufs, K, nh)
            for i, c in enumerate(cs):
                np.testing.assert_array_equal(out[i], c["trace"][nh - 1],
                                              err_msg=f"K={K} {c['kind']} {c['ebno']} nhalf={nh}")


KS = [40, 48, 104, 200, 256, 400, 408, 480, 512, 528, 800, 816, 1024, 1056, 2048, 3072, 4096, 5312, 6144]


@pytest.mark.parametrize("K", KS)
def test_random_vs_oracle(dec, K):
    rng = np.random.default_rng(K)
    bufs = []
    for i in range(13):  # odd count: exercises the unpaired generic lane
        eb = [0.0, 0.5, 1.0, 2.0, 6.0][i % 5]
        if i == 12:
            lin = rng.integers(-32768, 32768, 3 * K + 12, dtype=np.int16)
            bufs.append(oracle.tdec_pack_input(lin, K))
        else:
            bufs.append(oracle.make_cb(rng, K, eb, scale=100.0 if i % 3 else 900.0)[2])
    arr = _stack(bufs, K)
    for nh in (1, 2, 3, 8):
        out = dec.run(arr, K, nh)
        for i, b in enumerate(bufs):
            np.testing.assert_array_equal(out[i], oracle.tdec_run(b, K, nh), err_msg=f"K={K} cb={i} nhalf={nh}")


def test_large_batch_is_batch_size_independent(dec):
    """16384 x K=6144: tiled copies of 32 distinct code blocks must decode exactly like the pool."""
    K, nh = 6144, 8
    rng = np.random.default_rng(7)
    pool = _stack([oracle.make_cb(rng, K, eb)[2] for eb in np.linspace(0.0, 3.0, 32)], K)
    want = np.stack([oracle.tdec_run(b, K, nh) for b in pool])
    n = 16384
    big = np.ascontiguousarray(np.tile(pool, (n // pool.shape[0], 1)))
    out = dec.run(big, K, nh)
    np.testing.assert_array_equal(out, np.tile(want, (n // pool.shape[0], 1)))


def test_single_and_tiny_batches(dec):
    rng = np.random.default_rng(3)
    for K in (40, 512, 6144):
        for n in (1, 2, 3):
            bufs = [oracle.make_cb(rng, K, 1.0)[2] for _ in range(n)]
            out = dec.run(_stack(bufs, K), K, 5)
            for i, b in enumerate(bufs):
                np.testing.assert_array_equal(out[i], oracle.tdec_run(b, K, 5))


def test_invalid_inputs_are_rejected(dec):
    L = srsran_amd.lib()
    buf = np.zeros((1, srsran_amd.tdec_buf_len(6144)), np.int16)
    out = np.zeros((1, 768), np.uint8)
    # K not in the 36.212 table, nhalf == 0, odd stride, short stride
    assert L.mi355_tdec_batch_run(dec.h, buf.ctypes.data, buf.shape[1], 1, 6000, 8, out.ctypes.data, 768) == -2
    assert L.mi355_tdec_batch_run(dec.h, buf.ctypes.data, buf.shape[1], 1, 6144, 0, out.ctypes.data, 768) == -2
    assert L.mi355_tdec_batch_run_dev(dec.h, 1, 18541, 1, 6144, 8, 1, 768, None) == -2
    assert L.mi355_tdec_batch_run_dev(dec.h, 1, 100, 1, 6144, 8, 1, 768, None) == -2
    # n == 0 is a successful no-op
    assert L.mi355_tdec_batch_run(dec.h, buf.ctypes.data, buf.shape[1], 0, 6144, 8, out.ctypes.data, 768) == 0


def test_kernel_profiling_counts_launches(dec):
    rng = np.random.default_rng(11)
    arr = _stack([oracle.make_cb(rng, 6144, 2.0)[2] for _ in range(4)], 6144)
    dec.set_profiling(True)
    dec.run(arr, 6144, 6)
    ms, n = dec.kernel_stats()
    dec.set_profiling(False)
    assert n == 6 and ms > 0
