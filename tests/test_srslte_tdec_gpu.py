"""GPU: the srslte_tdec_* drop-in API, exercised the way the reference's own callers use it:
turbodecoder_test.c (GENERIC + force_not_sb + run_all on linear input, config 1) and sch.c:415-450
(new_cb + iteration, decision after every half-iteration)."""
import numpy as np
import pytest

from golden_io import tdec_auto_cases, tdec_generic_cases
from srsran_amd.srslte import SRSLTE_TDEC_GENERIC, SrslteTdec

pytestmark = pytest.mark.gpu


def test_run_all_generic_force_not_sb_matches_reference():
    dec = SrslteTdec(6144, SRSLTE_TDEC_GENERIC)
    dec.force_not_sb()
    for c in tdec_generic_cases():
        buf = np.zeros(3 * (c["K"] + 32) + 12, np.int16)
        buf[: c["lin"].size] = c["lin"]
        out = dec.run_all(buf, c["trace"].shape[0], c["K"])
        np.testing.assert_array_equal(out, c["trace"][-1])
    dec.free()


def test_iteration_api_matches_reference_trace():
    dec = SrslteTdec(6144)
    for c in tdec_auto_cases()[::3]:
        assert dec.new_cb(c["K"]) == 0
        for n in range(c["trace"].shape[0]):
            out = dec.iteration(c["buf"])
            np.testing.assert_array_equal(out, c["trace"][n], err_msg=f"K={c['K']} half-iteration {n + 1}")
        assert dec.n_iter == c["trace"].shape[0]
    dec.free()


def test_new_cb_errors_like_reference():
    dec = SrslteTdec(1024)
    assert dec.new_cb(2048) == -1   # > max_long_cb
    assert dec.new_cb(1000) == -1   # not a 36.212 size
    assert dec.new_cb(1024) == 0
    dec.free()


def test_iteration_8bit_api_matches_reference_trace():
    """srslte_tdec_iteration_8bit as sch.c:421-423 calls it with llr_is_8bit, against the reference's own 8-bit
    decoder (tests/golden/tdec8.npz), and run_all_8bit's final decision."""
    from golden_io import load
    z = load("tdec8.npz")
    dec = SrslteTdec(6144)
    for i in range(0, int(z["ncases"]), 2):
        K, tr = int(z[f"c{i}_K"]), z[f"c{i}_trace"]
        buf = z[f"c{i}_buf"].copy()
        assert dec.new_cb(K) == 0
        for n in range(tr.shape[0]):
            np.testing.assert_array_equal(dec.iteration_8bit(buf), tr[n], err_msg=f"K={K} half-iteration {n + 1}")
        assert dec.n_iter == tr.shape[0]
        np.testing.assert_array_equal(dec.run_all_8bit(z[f"c{i}_buf"].copy(), tr.shape[0], K), tr[-1])
    with pytest.raises(RuntimeError):  # 400 < K <= 800: the reference decodes a partly unconverted buffer
        dec.run_all_8bit(np.zeros(3 * (512 + 32) + 12, np.int8), 2, 512)
    dec.free()
