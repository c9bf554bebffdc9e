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


def lane_logical(gl):  # tdec_win_lat.hip lane_logical: group lane -> logical lane
    return gl ^ (3 if gl & 4 else 0)


def dstep_n_phys(phys, k, beta, x, y):
    """The kernel's dstep_n on group lanes: partner by group-lane xor (1, 2, 7), the new state 0 from the old states
    of logical lanes 0 and D (group lanes 0 and 1 / 2 / 7), subtracted."""
    d = (4 >> k) if beta else (1 << k)
    gd = 7 if d == 4 else d
    s0 = max(phys[0], sadd(phys[gd], sadd(x, y)))
    out = []
    for gl in range(8):
        s = held(lane_logical(gl), k, beta)
        go = (s & 3) if beta else (s >> 1)
        new = max(sadd(phys[gl], g(go, x, y)), sadd(phys[gl ^ gd], g(3 - go, x, y)))
        out.append(sat(new - s0))
    return out


@pytest.mark.parametrize("beta", [False, True], ids=["alpha", "beta"])
def test_group_lane_relabelling_and_early_normalisation(beta):
    # M is a linear involution with M(0) = 0 mapping the logical partner distances 1, 2, 4 to group-lane xors 1, 2, 7
    for a in range(8):
        assert lane_logical(lane_logical(a)) == a
        for b in range(8):
            assert lane_logical(a ^ b) == lane_logical(a) ^ lane_logical(b)
    assert lane_logical(0) == 0 and [lane_logical(d) for d in (1, 2, 4)] == [1, 2, 7]
    rng = np.random.default_rng(11 + beta)
    for trial in range(300):
        s = [int(v) for v in rng.integers(-4000, 4000, 8)]
        k0 = int(rng.integers(0, 3))
        phys = [s[held(lane_logical(gl), k0, beta)] for gl in range(8)]
        for step in range(9):
            k = (k0 + step) % 3
            lim = 32767 if trial % 2 else 300
            x, y = (int(v) for v in rng.integers(-lim, lim + 1, 2))
            s = snorm((bstep if beta else astep)(s, x, y))
            phys = dstep_n_phys(phys, k, beta, x, y)
            k1 = (k + 1) % 3
            assert phys == [s[held(lane_logical(gl), k1, beta)] for gl in range(8)], (trial, step)


def test_partner_exchanges_are_involutions_within_groups():
    # the DPP patterns of partner<D>: quad_perm [1,0,3,2] (D = 1), [2,3,0,1] (D = 2), row_half_mirror (D = 4: group
    # lane g reads 7 - g) -- a lane reads group lane g ^ (1, 2, 7) of its own group of 8
    def perm(d, lane):
        g = lane & 7
        if d == 1:
            return (lane & ~3) | [1, 0, 3, 2][lane & 3]
        if d == 2:
            return (lane & ~3) | [2, 3, 0, 1][lane & 3]
        return (lane & ~7) | (7 - g)

    for d, x in ((1, 1), (2, 2), (4, 7)):
        for lane in range(64):
            assert perm(d, lane) == (lane ^ x)
            assert perm(d, lane) >> 3 == lane >> 3
