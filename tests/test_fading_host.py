"""CPU checks of the fading-channel test restatement (tests/test_enb_fading_gpu.py): the Python MT19937 against the
C++ standard's known answer, and the phase draws' range and libstdc++ float conversion."""
import numpy as np

from tests.test_enb_fading_gpu import mt19937, uniform_2pi


def test_mt19937_known_answer():
    assert mt19937(5489, 10000)[-1] == 4123659995  # [rand.predef]


def test_uniform_2pi_draws():
    x = uniform_2pi(mt19937(17, 4096))
    assert x.dtype == np.float32 and x.min() >= 0 and x.max() < np.float32(2 * np.pi)
    assert abs(float(x.mean()) - np.pi) < 0.1
    top = uniform_2pi([0xFFFFFFFF])[0]  # rounds to 2^32 in float: clamped below 1 before scaling
    assert top == np.nextafter(np.float32(1), np.float32(0)) * (np.float32(2.0) * np.float32(np.pi))
