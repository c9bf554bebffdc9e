"""CPU: the time-domain channel emulator restatement (oracle/channel_chain.py) -- fading FFT sizes and segment
timing (fading.c:227-232, 334-367), the FIFO semantics of the delay emulator (delay.c:95-133) against a direct
sample-delay model, and the high-speed-train Doppler profile (hst.c:47-80).  The reference's fading.c needs FFTW
(not vendored, not installed), so it cannot be built here: the fading restatement is pinned by these structural
properties and, on the GPU, by agreement of two independent implementations (tests/test_channel_gpu.py)."""
import numpy as np
import pytest

from oracle import channel_chain as cc


@pytest.mark.parametrize("model,srate,N", [("epa5", 1.92e6, 32), ("epa5", 23.04e6, 384), ("epa5", 30.72e6, 512),
                                           ("eva70", 23.04e6, 512), ("etu300", 23.04e6, 1024),
                                           ("etu300", 1.92e6, 64)])
def test_fft_size(model, srate, N):
    assert cc.fft_size(model, srate) == N


def test_model_parsing():
    assert cc.parse_model("epa5") == ("epa", 5.0)
    assert cc.parse_model("etu300") == ("etu", 300.0)
    assert cc.parse_model("evaX") == ("eva", 0.0)
    for bad in ("foo5", "epa"):
        with pytest.raises(ValueError):
            cc.parse_model(bad)
    with pytest.raises(ValueError):
        cc.fft_size("none0", 23.04e6)


def test_mt19937_known_answer():
    assert cc.mt19937(5489, 10000)[-1] == 4123659995


def test_fading_time_advance_and_state():
    """execute returns init_time + sum of float(n) / srate over its segments; two calls over halves of a stream
    equal one call over the whole stream (the overlap-add state carries the tail)."""
    rng = np.random.default_rng(1)
    x = (rng.standard_normal(5000) + 1j * rng.standard_normal(5000)) / np.sqrt(2)
    f1 = cc.Fading(23.04e6, "epa5", 3)
    y_all, t_all = f1.execute(x, 0.25)
    n = f1.N // 2
    segs = [n] * (5000 // n) + ([5000 % n] if 5000 % n else [])
    t = 0.25
    for s in segs:
        t += float(np.float32(s) / np.float32(23.04e6))
    assert t_all == pytest.approx(t, abs=0)
    f2 = cc.Fading(23.04e6, "epa5", 3)
    cut = 6 * n  # segment boundary: the same segments, so the same tap times
    ya, ta = f2.execute(x[:cut], 0.25)
    yb, _ = f2.execute(x[cut:], ta)
    assert np.allclose(np.concatenate([ya, yb]), y_all, rtol=0, atol=1e-12)


def test_fading_static_channel_is_lti():
    """With zero Doppler the taps are constant: the emulator is then linear and time-invariant up to its
    block structure -- delaying the input by one segment delays the output by one segment."""
    rng = np.random.default_rng(2)
    f = cc.Fading(1.92e6, "eva0", 9)
    n = f.N // 2
    x = rng.standard_normal(8 * n) + 1j * rng.standard_normal(8 * n)
    y, _ = cc.Fading(1.92e6, "eva0", 9).execute(x, 0.0)
    y2, _ = cc.Fading(1.92e6, "eva0", 9).execute(np.concatenate([np.zeros(n), x]), 0.0)
    assert np.allclose(y2[n:], y[: len(y2) - n], atol=1e-12)
    y3, _ = cc.Fading(1.92e6, "eva0", 9).execute(2 * x, 0.0)
    assert np.allclose(y3, 2 * y, atol=1e-12)


def test_delay_fifo_matches_sample_delay():
    """A constant delay d: the output stream is the input stream delayed by d samples (zeros first), whatever
    the call lengths."""
    rng = np.random.default_rng(3)
    q = cc.Delay(10.0, 10.0, 0.0, 0.0, 1_920_000)
    d = q.delay_samples(0, 0.0)
    assert d == round(10.0 * 1.92)
    xs = [rng.standard_normal(k) + 0j for k in (7, 40, 3, 25, 19)]
    out = np.concatenate([q.execute(x, 0, 0.0) for x in xs])
    full = np.concatenate(xs)
    assert np.array_equal(out, np.concatenate([np.zeros(d), full])[: len(full)])


def test_delay_profile_and_resize():
    q = cc.Delay(1.0, 5.0, 1.0, 0.0, 1_920_000)
    ds = [q.delay_samples(0, f) for f in (0.0, 0.25, 0.5, 0.75)]
    assert ds == [round(3.0 * 1.92), round(5.0 * 1.92), round(3.0 * 1.92), round(1.0 * 1.92)]
    x = np.arange(1, 11) + 0j
    y1 = q.execute(x, 0, 0.25)  # d = 10: all zeros out, FIFO = x
    assert np.array_equal(y1, np.zeros(10))
    y2 = q.execute(x + 10, 0, 0.75)  # d = 2: the two newest samples of the FIFO come out first
    assert np.array_equal(y2, np.r_[9, 10, np.arange(11, 19)] + 0j)


def test_hst_profile():
    q = cc.Hst(750.0, 1.0, 0.0, 1_920_000)
    assert q.shift_hz(0, 0.0) == pytest.approx(750.0, rel=1e-4)     # approaching: +fd
    assert abs(q.shift_hz(0, 0.25)) < 1e-3                           # passing the eNodeB
    assert q.shift_hz(0, 0.5 - 1e-6) == pytest.approx(-750.0, rel=1e-3)
    x = np.ones(64, complex)
    y = q.execute(x, 0, 0.0)
    fs = q.shift_hz(0, 0.0)
    assert np.allclose(y, np.exp(-2j * np.pi * fs / 1.92e6 * np.arange(64)), atol=1e-6)
