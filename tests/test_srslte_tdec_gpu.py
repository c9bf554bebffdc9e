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
