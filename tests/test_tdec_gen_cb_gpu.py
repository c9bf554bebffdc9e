"""GPU: the generic decoder with one workgroup per code block (tdec_gen_cb.hip) -- chunked recursions started from
guessed states and rerun until every chunk boundary agrees -- against the reference's generic decoder
(turbodecoder_gen.c:58-198 via tests/golden/tdec_generic.npz) and the oracle's restatement of it, after every
half-iteration, for every schedule knob: the default warm-up, a short one and none at all (every chunk but the
first then starts from a wrong guess, so the rerun path carries the whole decode)."""
import numpy as np
import pytest

import oracle
from golden_io import tdec_generic_cases
from srsran_amd.srslte import SRSLTE_TDEC_GENERIC, SrslteTdec
from srsran_amd.tdec import TdecBatch

pytestmark = pytest.mark.gpu


def _lin_batch(lins, K):
    stride = (3 * K + 12 + 7) // 8 * 8
    host = np.zeros((len(lins), stride), np.int16)
    for i, l in enumerate(lins):
        host[i, : l.size] = l
    return host


def _decoder(per_cb, warm):
    dec = TdecBatch(0)
    dec.set_impl(1)  # GENERIC on the linear layout (turbodecoder_test -d 1)
    dec.set_generic(per_cb, warm)
    dec.generic_reruns()
    return dec


@pytest.mark.parametrize("warm", [32, 8, 0])
def test_golden_blocks_every_warmup(warm):
    dec = _decoder(1, warm)
    for c in tdec_generic_cases():
        K, tr = c["K"], c["trace"]
        host = _lin_batch([c["lin"]], K)
        for n in range(1, tr.shape[0] + 1):
            out = dec.run(host, K, n)
            np.testing.assert_array_equal(out[0], tr[n - 1], err_msg=f"K={K} warm={warm} half-iteration {n}")
    reruns = dec.generic_reruns()
    if warm == 0:
        assert reruns > 0  # the rerun path was taken (and the decode stayed exact)
    dec.close()


def _random_lins(rng, K, n):
    """Encoded blocks over a range of Eb/N0 (waterfall and below), plus adversarial inputs: all-zero, constant,
    random full-range int16 (wrapping sums), and LLRs scaled to saturate the recursion."""
    lins = []
    for i in range(n):
        kind = i % 6
        if kind < 3:
            lins.append(oracle.make_cb(rng, K, (-1.0, 0.8, 3.0)[kind])[1])
        elif kind == 3:
            lins.append(rng.integers(-32768, 32768, 3 * K + 12).astype(np.int16))
        elif kind == 4:
            lins.append(np.full(3 * K + 12, 0 if i % 12 == 4 else 7, np.int16))
        else:
            lins.append(oracle.make_cb(rng, K, 6.0, scale=3000.0)[1])
    return lins


@pytest.mark.parametrize("K", [40, 104, 400, 1024, 3264, 6144])
def test_random_batch_matches_oracle_each_half_iteration(K):
    rng = np.random.default_rng(K)
    lins = _random_lins(rng, K, 12)
    host = _lin_batch(lins, K)
    for per_cb, warm in ((1, 32), (1, 4), (0, 32)):
        dec = _decoder(per_cb, warm)
        for nhalf in (1, 2, 3, 6):
            out = dec.run(host, K, nhalf)
            for i, l in enumerate(lins):
                want = oracle.tdec_run_generic(l, K, nhalf)
                np.testing.assert_array_equal(out[i], want, err_msg=f"K={K} cb={i} per_cb={per_cb} warm={warm} "
                                                                    f"nhalf={nhalf}")
        dec.close()


def test_iteration_api_continues_across_calls():
    """srslte_tdec_iteration one half-iteration per call (the workspace carries E and A1 between launches), the
    decision after each equal to the reference trace."""
    dec = SrslteTdec(6144, SRSLTE_TDEC_GENERIC)
    dec.force_not_sb()
    for c in tdec_generic_cases():
        K = c["K"]
        buf = np.zeros(3 * (K + 32) + 12, np.int16)
        buf[: c["lin"].size] = c["lin"]
        assert dec.new_cb(K) == 0
        for n in range(c["trace"].shape[0]):
            np.testing.assert_array_equal(dec.iteration(buf), c["trace"][n], err_msg=f"K={K} half-iteration {n + 1}")
    dec.free()


def test_large_batch_sampled():
    """Thousands of code blocks in one launch (one workgroup each), sampled against the oracle."""
    K, n = 6144, 2048
    rng = np.random.default_rng(5)
    base = [oracle.make_cb(rng, K, e)[1] for e in (0.6, 1.0, 2.0, 4.0)]
    lins = [base[i % 4] for i in range(n)]
    host = _lin_batch(lins, K)
    dec = _decoder(-1, 32)
    out = dec.run(host, K, 8)
    want = [oracle.tdec_run_generic(b, K, 8) for b in base]
    for i in range(n):
        np.testing.assert_array_equal(out[i], want[i % 4], err_msg=f"cb {i}")
    dec.close()
