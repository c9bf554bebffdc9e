"""The latency kernel's distributed trellis (srsran_amd/csrc/tdec_win_lat.hip: Lane8, partner<D>, dstep, dnorm) against
the register form of the window decoder's recursions (turbodecoder_win.h:640-676 beta, :771-800 alpha; the kernel's
bstep / acands): the 8 states of a window pair over 8 lanes, lane q holding state rotl3(q, K) (beta) or rotr3(q, K)
(alpha) at phase K, each lane combining its own and its partner lane's (q ^ D) metric with the branch metric its held
state selects.  Saturating int16 arithmetic throughout; CPU only (the GPU suites check the kernel itself)."""
import numpy as np
import pytest

INF = 10000


def sat(v):
    return max(-32768, min(32767, int(v)))


def sadd(a, b):
    return sat(a + b)


def bstep(s, x, y):  # turbodecoder_win.h:640-676 (tdec_win_lat.hip bstep<true>)
    xy = sadd(x, y)
    return [max(sadd(s[4], xy), s[0]), max(s[4], sadd(s[0], xy)), max(sadd(s[5], y), sadd(s[1], x)),
            max(sadd(s[5], x), sadd(s[1], y)), max(sadd(s[6], x), sadd(s[2], y)), max(sadd(s[6], y), sadd(s[2], x)),
            max(s[7], sadd(s[3], xy)), max(sadd(s[7], xy), s[3])]


def astep(o, x, y):  # turbodecoder_win.h:771-800 (tdec_win_lat.hip acands + max)
    xy = sadd(x, y)
    c0 = [o[0], sadd(o[3], y), sadd(o[4], y), o[7], o[1], sadd(o[2], y), sadd(o[5], y), o[6]]
    c1 = [sadd(o[1], xy), sadd(o[2], x), sadd(o[5], x), sadd(o[6], xy), sadd(o[0], xy), sadd(o[3], x), sadd(o[4], x),
          sadd(o[7], xy)]
    return [max(a, b) for a, b in zip(c0, c1)]


def snorm(s):  # turbodecoder_win.h:480-498, 16-bit: subtract state 0
    return [0] + [sat(v - s[0]) for v in s[1:]]


def rotl3(q, k):
    return ((q << k) | (q >> ((3 - k) % 3))) & 7


def rotr3(q, k):
    return ((q >> k) | (q << ((3 - k) % 3))) & 7


def held(q, k, beta):  # Lane8::held
    return rotl3(q, k) if beta else rotr3(q, k)


def g(code, x, y):  # sat((x & mx) + (y & my))
    return sadd(x if code & 1 else 0, y if code & 2 else 0)


def dstep(lanes, k, beta, x, y):  # tdec_win_lat.hip dstep<BETA, PH>
    d = (4 >> k) if beta else (1 << k)
    out = []
    for q in range(8):
        s = held(q, k, beta)
        go = (s & 3) if beta else (s >> 1)
        out.append(max(sadd(lanes[q], g(go, x, y)), sadd(lanes[q ^ d], g(3 - go, x, y))))
    return out


def dnorm(lanes):  # state 0 always in lane 0 of the group
    return [sat(v - lanes[0]) for v in lanes]


@pytest.mark.parametrize("beta", [False, True], ids=["alpha", "beta"])
def test_distributed_step_equals_register_step(beta):
    rng = np.random.default_rng(7 + beta)
    for trial in range(300):
        s = [int(v) for v in rng.integers(-4000, 4000, 8)]
        if trial % 3 == 0:
            s = [0] + [-INF] * 7  # the window boundaries' initial states
        k0 = int(rng.integers(0, 3))
        lanes = [s[held(q, k0, beta)] for q in range(8)]
        for step in range(12):
            k = (k0 + step) % 3
            lim = 32767 if trial % 2 else 300  # saturating and small inputs
            x, y = (int(v) for v in rng.integers(-lim, lim + 1, 2))
            s = (bstep if beta else astep)(s, x, y)
            lanes = dstep(lanes, k, beta, x, y)
            if step % 2:
                s, lanes = snorm(s), dnorm(lanes)
            k1 = (k + 1) % 3
            assert held(0, k1, beta) == 0
            assert lanes == [s[held(q, k1, beta)] for q in range(8)], (trial, step)


def test_partner_exchanges_are_involutions_within_groups():
    # the DPP patterns of partner<D>: quad_perm [1,0,3,2] (D = 1), [2,3,0,1] (D = 2), row_shr:4 into lanes 4-7 and
    # row_shl:4 into lanes 0-3 of every 8 (D = 4) -- lane q of a group of 8 reads lane q ^ D of the same group
    def perm(d, lane):
        q, base = lane & 7, lane & ~7
        if d == 1:
            return (lane & ~3) | [1, 0, 3, 2][lane & 3]
        if d == 2:
            return (lane & ~3) | [2, 3, 0, 1][lane & 3]
        return lane - 4 if q >= 4 else lane + 4

    for d in (1, 2, 4):
        for lane in range(64):
            assert perm(d, lane) == (lane ^ d)
            assert perm(d, lane) >> 3 == lane >> 3
