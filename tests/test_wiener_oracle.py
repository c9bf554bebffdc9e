"""CPU: the Wiener DL estimator restatement (oracle/orc_wiener.cpp, wiener_dl.c) -- the sub-band draws equal the
standard library's (and the Lemire restatement the GPU kernel follows), the estimator trains and then switches to its
Wiener output as chest_dl.c:648-676 does, and the trained estimate tracks the channel better than the raw pilots.
wiener_dl.c cannot be built here (srslte.h -> CMake-generated version.h; FFTW absent), so the restatement itself is
pinned by these properties, not by reference outputs ("parity unpinned" against the reference)."""
import numpy as np
import pytest

from oracle import wiener_chain as wc


def test_stdlib_draws_are_libstdcxx_lemire():
    """The restatement's sub-band draws come from the host's standard library: libstdc++ with Lemire's
    uniform_int_distribution (GCC 11 and later, __GLIBCXX__ >= 20210427), which the GPU kernel restates.  The
    reference's srslte_random_uniform_int_dist draws the same only when built against such a library."""
    import ctypes
    import oracle
    f = oracle.lib().orc_stdlib_glibcxx
    f.restype, f.argtypes = ctypes.c_long, []
    v = f()
    if v < 20210427:
        pytest.skip(f"oracle built against {'libstdc++ ' + str(v) if v else 'a non-libstdc++ library'}: its "
                    "uniform_int_distribution is not Lemire's, so the Wiener sub-band draws are not the GPU's")
    assert v >= 20210427


@pytest.mark.parametrize("hi", [3, 12, 50, 1, 0])
def test_uniform_int_is_lemire(hi):
    std = wc.std_uniform_int(0xDEAD, 0, hi, 300)
    assert list(std) == wc.lemire_uniform_int(0xDEAD, 0, hi, 300)


def test_rejects_unsupported():
    with pytest.raises(AssertionError):
        wc.Wiener(6, 4, 1)


@pytest.mark.parametrize("nof_prb,ntx,nrx", [(25, 2, 2), (6, 1, 1), (50, 1, 2)])
def test_trains_then_tracks(nof_prb, ntx, nrx):
    """A time-varying multipath channel at 15 dB: the estimator is not ready in its first subframe (chest_dl.c then
    outputs the AVERAGE estimate), ready from the third on, and its Wiener rows then track the true channel with a
    relative MSE well below the LS pilots' noise (2 sigma^2 = 0.032)."""
    rng = np.random.default_rng(nof_prb)
    pil, snr, H = wc.synth_pilots(rng, nof_prb, ntx, nrx, 12, snr_db=15.0)
    w = wc.Wiener(nof_prb, ntx, nrx)
    shift = [wc.crs_shift(1, p) for p in range(ntx)]
    mse = []
    for s in range(12):
        ce, rd, draws = w.subframe(pil[s], snr[s], shift)
        assert np.all(np.isfinite(ce))
        if s == 0:
            assert not rd.any()
        if s >= 2:
            assert rd.all()
        mse.append(float(np.mean(np.abs(ce - H[s]) ** 2) / np.mean(np.abs(H[s]) ** 2)))
    assert draws > 0
    ls_noise = 10 ** (-15 / 10)  # relative variance of an LS pilot estimate
    assert max(mse[5:]) < 0.5 * ls_noise, mse


def test_state_carries_between_calls():
    """Feeding subframes one by one equals feeding the same subframes to a second object (determinism)."""
    rng = np.random.default_rng(3)
    pil, snr, _ = wc.synth_pilots(rng, 15, 2, 1, 6, snr_db=20.0)
    a, b = wc.Wiener(15, 2, 1), wc.Wiener(15, 2, 1)
    for s in range(6):
        ca, ra, da = a.subframe(pil[s], snr[s], [1, 4])
        cb, rb, db = b.subframe(pil[s], snr[s], [1, 4])
        assert np.array_equal(ca, cb) and np.array_equal(ra, rb) and da == db
