#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the srsLTE reference compiled from its own
sources (``make -C oracle ref`` -> oracle/_ref/libsrslte_ref.so).  Run in the survey container only
(needs /root/reference); the resulting .npz files are committed and are the parity anchor on the GPU box.

    python tests/golden/make_golden.py

Contents
  tdec_auto.npz      AUTO-mode decoder (generic / 8-window / 16-window by K): inputs in the softbuffer
                     layout, decision bytes after every half-iteration 1..8 (srslte_tdec_iteration),
                     including failing code blocks, saturating and full-range int16 inputs.
  tdec8.npz          the 8-bit AUTO decoder (srslte_tdec_iteration_8bit: 32-window AVX8 for K % 32 == 0 && K > 2048,
                     16-window SSE8 for K % 16 == 0 && K > 800) on int8 inputs in the 8-bit sub-block layout,
                     decision bytes after every half-iteration 1..8, incl. saturating and full-range int8 inputs;
                     plus srslte_rm_turbo_rx_lut_8bit (E below / at / above the circular buffer, every rv, HARQ).
  tdec_generic.npz   GENERIC manual decoder + force_not_sb on linear input (turbodecoder_test -d 1).
  tcod_known.npz     the reference test's own known-answer vector (turbodecoder_test.h:69-125).
  crc_cbsegm.npz     CRC24A/24B/16/8 checksums and CB segmentation for a TBS sweep.
  rm_turbo.npz       srslte_rm_turbo_rx_lut (AVX build): E LLRs -> decoder buffer, every rv, E below /
                     at / above the circular buffer (wrap-around), plus HARQ accumulation rv0 + rv2.
  pdcch.npz          downlink control channels: REG maps (srslte_regs_init_opts: PCFICH / PHICH / per-CFI PDCCH),
                     UE / common search spaces, CRC16, the tail-biting Viterbi decoder on u16 symbols
                     (srslte_viterbi_decode_us, AVX2 16-bit build), srslte_pdcch_dci_decode on noisy LLRs,
                     srslte_pdcch_dci_encode, and srslte_pcfich_decode / srslte_pdcch_extract_llr on synthetic
                     control regions (1 / 2 / 4 ports, 1 / 2 rx).  ``make_golden.py pdcch`` regenerates only this.
  pdsch_stages.npz   srslte_demod_soft_demodulate_s for every modulation (SIMD bodies and scalar tails,
                     saturating amplitudes), srslte_scrambling_s_offset (PDSCH c_init), and
                     srslte_predecoding_type with CSI (AVX2 build, MMSE) for every scheme srslte_pdsch_decode
                     uses -- the equaliser output is pinned within the reference's rcp tolerance.
  ref_pins.npz       (``make_golden.py pins``) the reference's scalar equaliser path over full 100-PRB vectors
                     (srslte_predecoding_type on chunks shorter than one AVX2 vector: precoding.c scalar tails,
                     mat.c:63-109) for SISO 1/2 rx, SFBC 2 ports 1/2 rx, TM4 2x2 codebooks 0-2, 2x1 MRC codebooks
                     0-3 and CDD, MMSE and ZF, inputs regenerated from their seeds (input SHA-256 recorded), outputs
                     as SHA-256 plus their first 64 values; the PDSCH RE -> grid map through the compiled prb_dl.c
                     primitives (oracle/ref/ref_prb.c) for 6-110 PRB x 1/2/4 ports x CFI 1-3 x subframes x FDD/TDD
                     (SHA-256 per case); and the estimator's smoothing filters from the compiled chest_common.c.
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF_TEST_H = "/root/reference/lib/src/phy/fec/test/turbodecoder_test.h"
NHALF = 8


def gen_tdec_auto(rng):
    ref = oracle.RefTdec()
    cases = []
    # (K, kind, ebno)  kind: awgn (scale 100 as turbodecoder_test), big (scale 4000 -> saturation),
    #                        rand (uniform full-range int16 -> saturation + wrap everywhere)
    Ks = [40, 104, 400, 408, 512, 800, 816, 1024, 1056, 2048, 5312, 6144]
    for K in Ks:
        cases += [(K, "awgn", 0.5), (K, "awgn", 4.0)]
    cases += [(6144, "big", 2.0), (512, "big", 2.0), (200, "big", 2.0),
              (6144, "rand", 0.0), (512, "rand", 0.0), (104, "rand", 0.0)]
    data = {}
    for ci, (K, kind, eb) in enumerate(cases):
        if kind == "rand":
            bits = np.zeros(K, np.uint8)
            lin = rng.integers(-32768, 32768, 3 * K + 12, dtype=np.int16)
            buf = oracle.tdec_pack_input(lin, K)
        else:
            bits, lin, buf = oracle.make_cb(rng, K, eb, scale=100.0 if kind == "awgn" else 4000.0)
        out, tr = ref.run(buf, K, NHALF, trace=True)
        data[f"c{ci}_K"] = np.int32(K)
        data[f"c{ci}_kind"] = np.array(kind)
        data[f"c{ci}_ebno"] = np.float32(eb)
        data[f"c{ci}_bits"] = bits
        data[f"c{ci}_buf"] = buf
        data[f"c{ci}_trace"] = tr
    data["ncases"] = np.int32(len(cases))
    data["nhalf"] = np.int32(NHALF)
    np.savez_compressed(os.path.join(OUT, "tdec_auto.npz"), **data)
    print("tdec_auto.npz:", len(cases), "cases")


def pack8(lin: np.ndarray, K: int, nsb: int) -> np.ndarray:
    """Encoder-order LLRs (x z z' per step, 12 tails) -> the 8-bit decoder buffer: stream s at s*(K+32), step
    w*L + j of window w at j*nsb + w, tails at 3*(K+32) in encoder order (rm_turbo_rx_lut_8bit's layout)."""
    L = K // nsb
    buf = np.zeros(3 * (K + 32) + 12, np.int8)
    m = np.arange(K)
    pos = (m % L) * nsb + m // L
    for s in range(3):
        buf[s * (K + 32) + pos] = lin[s: 3 * K: 3]
    buf[3 * (K + 32):] = lin[3 * K:]
    return buf


def gen_tdec8(rng):
    R = oracle.ref()
    h = R.ref_tdec8_new(6144)
    cases = []
    # (K, kind, ebno, scale): awgn int8 LLRs round(scale * y) clipped to +-127; rand: uniform full-range int8
    for K in (6144, 3072, 2112, 2048, 1024, 848):
        cases += [(K, "awgn", 0.5, 16.0), (K, "awgn", 2.0, 16.0)]
    cases += [(6144, "awgn", 6.0, 60.0), (1024, "awgn", 2.0, 90.0), (6144, "awgn", 10.0, 30.0), (1024, "awgn", 10.0, 30.0),
              (2112, "awgn", 10.0, 30.0), (6144, "rand", 0.0, 0.0), (848, "rand", 0.0, 0.0)]
    data = {}
    for ci, (K, kind, eb, sc) in enumerate(cases):
        nsb = 32 if (K % 32 == 0 and K > 2048) else 16
        if kind == "rand":
            bits = np.zeros(K, np.uint8)
            lin = rng.integers(-128, 128, 3 * K + 12, dtype=np.int8)
        else:
            bits = rng.integers(0, 2, K, dtype=np.uint8)
            enc = oracle.tcod_encode(bits, K)
            sigma = 10 ** (-(eb + 10 * np.log10(1 / 3)) / 20)
            y = np.where(enc.astype(bool), 1.0, -1.0) + sigma * rng.standard_normal(enc.size)
            lin = np.clip(np.round(sc * y), -127, 127).astype(np.int8)
        buf = pack8(lin, K, nsb)
        out = np.zeros(K // 8, np.uint8)
        tr = np.zeros((NHALF, K // 8), np.uint8)
        work = buf.copy()
        assert R.ref_tdec8_run(h, work, K, NHALF, out, tr.ctypes.data) == 0
        data[f"c{ci}_K"] = np.int32(K)
        data[f"c{ci}_kind"] = np.array(kind)
        data[f"c{ci}_ebno"] = np.float32(eb)
        data[f"c{ci}_bits"] = bits
        data[f"c{ci}_buf"] = buf
        data[f"c{ci}_trace"] = tr
    R.ref_tdec8_free(h)
    data["ncases"] = np.int32(len(cases))
    data["nhalf"] = np.int32(NHALF)
    # srslte_rm_turbo_rx_lut_8bit: (K, rv, E, amplitude) into a zero buffer, then a second (HARQ) accumulation
    rm = []
    for K in (6144, 2112, 1024, 848):
        N = 3 * K + 12
        for rv in range(4):
            for E in (N // 3, N, N + N // 2 + 7):
                rm.append((K, rv, E))
    for ri, (K, rv, E) in enumerate(rm):
        e1 = rng.integers(-40, 41, E, dtype=np.int8)
        e2 = rng.integers(-128, 128, E, dtype=np.int8)
        out = np.zeros(3 * (K + 32) + 12 + 64, np.int8)
        assert R.ref_rm_turbo_rx_8bit(e1, E, out, K, rv) == 0
        first = out.copy()
        assert R.ref_rm_turbo_rx_8bit(e2, E, out, K, (rv + 2) % 4) == 0
        data[f"rm{ri}_K"], data[f"rm{ri}_rv"], data[f"rm{ri}_E"] = np.int32(K), np.int32(rv), np.int32(E)
        data[f"rm{ri}_e1"], data[f"rm{ri}_e2"] = e1, e2
        data[f"rm{ri}_out1"], data[f"rm{ri}_out2"] = first[: 3 * (K + 32) + 12], out[: 3 * (K + 32) + 12]
    data["rm_n"] = np.int32(len(rm))
    # srslte_demod_soft_demodulate_b (SSE bodies / scalar tails, saturation and int8 wrap) and srslte_scrambling_sb_offset
    k = 0
    for qm in (2, 4, 6, 8):
        for n in (1, 3, 7, 8, 9, 16, 17, 100, 301):
            for amp in (1.0, 3.0, 9.0):
                sym = (amp * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)).astype(np.complex64)
                iq = np.ascontiguousarray(sym.view(np.float32))
                out = np.zeros(qm * n + 64, np.int8)
                assert R.ref_demod_soft_b(qm, iq, out, n) == 0
                data[f"dm{k}_qm"], data[f"dm{k}_sym"], data[f"dm{k}_llr"] = np.int32(qm), sym, out[: qm * n].copy()
                k += 1
    data["dm_n"] = np.int32(k)
    k = 0
    for (rnti, cw, sf, cid, n) in [(0x1234, 0, 3, 1, 1000), (0xffff, 1, 9, 503, 4097), (61, 0, 0, 0, 33)]:
        c_init = oracle.pdsch_c_init(rnti, cw, sf, cid)
        llr = rng.integers(-128, 128, n, dtype=np.int8)
        llr[:4] = [-128, 127, 0, -1]
        out = llr.copy()
        assert R.ref_scramble_sb(c_init, out, 0, n) == 0
        data[f"sb{k}_cinit"], data[f"sb{k}_in"], data[f"sb{k}_out"] = np.uint32(c_init), llr, out
        k += 1
    data["sb_n"] = np.int32(k)
    np.savez_compressed(os.path.join(OUT, "tdec8.npz"), **data)
    print("tdec8.npz:", len(cases), "decoder cases,", len(rm), "rate-dematching cases")


def gen_tdec_generic(rng):
    ref = oracle.RefTdec(generic=True)
    data = {}
    cases = [(6144, 6.0), (6144, 1.0), (1024, 1.0)]
    for ci, (K, eb) in enumerate(cases):
        bits, lin, _ = oracle.make_cb(rng, K, eb)
        buf = np.zeros(oracle.tdec_buf_len(K), np.int16)
        buf[: 3 * K + 12] = lin
        out, tr = ref.run(buf, K, NHALF, trace=True)
        data[f"c{ci}_K"] = np.int32(K)
        data[f"c{ci}_lin"] = lin
        data[f"c{ci}_bits"] = bits
        data[f"c{ci}_trace"] = tr
    data["ncases"] = np.int32(len(cases))
    np.savez_compressed(os.path.join(OUT, "tdec_generic.npz"), **data)
    print("tdec_generic.npz:", len(cases), "cases")


def gen_tcod_known():
    """The reference's own fixture: 504 info bits and their 1524 coded bits."""
    txt = open(REF_TEST_H).read()

    def arr(name):
        m = re.search(name + r"\[[A-Z_0-9 *+]*\]\s*=\s*\{([^}]*)\}", txt)
        return np.array([int(v) for v in m.group(1).replace("\n", " ").split(",") if v.strip()], np.uint8)

    kd, kde = arr("known_data"), arr("known_data_encoded")
    assert kd.size == 504 and kde.size == 3 * 504 + 12, (kd.size, kde.size)
    # cross-check with the compiled reference encoder
    out = np.zeros(kde.size, np.uint8)
    oracle.ref().ref_tcod_encode(kd.copy(), out, 504)
    # Finding: the fixture differs from the reference encoder (srslte_tcod_encode) in exactly one bit,
    # index 1512 = the first tail bit x_K.  turbodecoder_test -k only feeds the fixture to the decoder
    # and never compares it with the encoder, so the discrepancy is latent in the reference.
    diff = np.nonzero(out != kde)[0]
    assert list(diff) == [1512], diff
    np.savez_compressed(os.path.join(OUT, "tcod_known.npz"), known_data=kd, known_data_encoded=kde,
                        ref_encoder_out=out, fixture_vs_encoder_diff=diff.astype(np.int32))
    print("tcod_known.npz")


def gen_crc_cbsegm(rng):
    L = oracle.ref()
    polys = {"crc24a": (0x1864CFB, 24), "crc24b": (0x1800063, 24), "crc16": (0x11021, 16), "crc8": (0x19B, 8)}
    data = {}
    msgs = [rng.integers(0, 256, n, dtype=np.uint8) for n in (1, 3, 5, 64, 768, 12243)]
    for i, m in enumerate(msgs):
        data[f"msg{i}"] = m
        for name, (p, o) in polys.items():
            data[f"msg{i}_{name}"] = np.uint32(L.ref_crc_byte(p, o, m.copy(), 8 * m.size))
    data["nmsg"] = np.int32(len(msgs))
    tbs = np.array([0, 16, 40, 104, 1000, 6120, 6144, 6168, 15840, 30576, 75376, 97896, 149776, 391656], np.uint32)
    seg = np.zeros((tbs.size, 6), np.uint32)
    for i, t in enumerate(tbs):
        r = np.zeros(6, np.uint32)
        assert L.ref_cbsegm(int(t), r) == 0
        seg[i] = r
    data["tbs"] = tbs
    data["cbsegm"] = seg
    np.savez_compressed(os.path.join(OUT, "crc_cbsegm.npz"), **data)
    print("crc_cbsegm.npz")


def rm_init_softbuffer():
    """Deterministic non-zero softbuffer content (same formula in tests/golden_io.py)."""
    i = np.arange(oracle.SOFTBUFFER_SIZE, dtype=np.int64)
    return ((i * 7919) % 60001 - 30000).astype(np.int16)


def gen_rm(rng):
    L = oracle.ref()
    data = {}
    cases = []
    for K in (40, 104, 512, 816, 2048, 6144):
        N = 3 * K + 12
        for rv in range(4):
            for E in ((N // 3, 2 * N + 17) if K < 2048 else (7200,) if rv else (7200, N + 501)):
                cases.append((K, rv, E))
    for ci, (K, rv, E) in enumerate(cases):
        e = rng.integers(-20000, 20000, E).astype(np.int16)
        out = rm_init_softbuffer()  # non-zero softbuffer: exercises the wrapping +=
        assert L.ref_rm_turbo_rx(e.copy(), E, out, K, rv) == 0
        blen = 3 * (K + 32) + 12
        assert (out[blen:] == rm_init_softbuffer()[blen:]).all()
        data[f"c{ci}_K"], data[f"c{ci}_rv"] = np.int32(K), np.int32(rv)
        data[f"c{ci}_e"], data[f"c{ci}_out"] = e, out[:blen]
    data["ncases"] = np.int32(len(cases))
    # HARQ: rv 0 then rv 2 into a zeroed buffer, K = 5312 (SISO QPSK config: E = 10000)
    K = 5312
    e0 = rng.integers(-300, 300, 10000).astype(np.int16)
    e2 = rng.integers(-300, 300, 10000).astype(np.int16)
    acc = np.zeros(oracle.SOFTBUFFER_SIZE, np.int16)  # after srslte_softbuffer_rx_reset
    L.ref_rm_turbo_rx(e0.copy(), e0.size, acc, K, 0)
    L.ref_rm_turbo_rx(e2.copy(), e2.size, acc, K, 2)
    data.update(harq_K=np.int32(K), harq_e0=e0, harq_e2=e2, harq_out=acc[: 3 * (K + 32) + 12])
    np.savez_compressed(os.path.join(OUT, "rm_turbo.npz"), **data)
    print("rm_turbo.npz:", len(cases), "cases")


def gen_pdsch_stages(rng):
    R = oracle.ref()
    data = {}
    k = 0
    for qm in (1, 2, 4, 6, 8):
        for n in (1, 3, 4, 7, 16, 17, 100, 301):
            for amp in (1.0, 60.0, 3e5):
                sym = (amp * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)).astype(np.complex64)
                iq = np.ascontiguousarray(sym.view(np.float32))
                out = np.zeros(qm * n, np.int16)
                R.ref_demod_soft_s(qm, iq, out, n)
                data[f"demod{k}_qm"] = np.int32(qm)
                data[f"demod{k}_sym"] = sym
                data[f"demod{k}_llr"] = out
                k += 1
    data["demod_n"] = np.int32(k)
    k = 0
    for (rnti, cw, sf, cid, n) in [(0x1234, 0, 3, 1, 1000), (0xffff, 1, 9, 503, 4097), (61, 0, 0, 0, 33),
                                   (0x4601, 1, 5, 77, 20000)]:
        c_init = oracle.pdsch_c_init(rnti, cw, sf, cid)
        llr = rng.integers(-32768, 32768, n, dtype=np.int16)
        llr[:4] = [-32768, 32767, 0, -1]
        out = llr.copy()
        R.ref_scramble_s(c_init, out, 0, n)
        data[f"scr{k}_cinit"] = np.uint32(c_init)
        data[f"scr{k}_in"] = llr
        data[f"scr{k}_out"] = out
        k += 1
    data["scr_n"] = np.int32(k)
    k = 0
    # (scheme, ports, rx, layers, codebooks)
    cfgs = [(0, 1, 1, 1, [0]), (0, 1, 2, 1, [0]), (1, 2, 1, 2, [0]), (1, 2, 2, 2, [0]), (2, 2, 2, 2, [0, 1, 2]),
            (2, 2, 2, 1, [0, 1, 2, 3]), (3, 2, 2, 2, [0])]
    for (scheme, ports, rx, layers, cbs) in cfgs:
        for cb in cbs:
            for n in (6, 258):
                y = ((rng.standard_normal((rx, n)) + 1j * rng.standard_normal((rx, n))) / np.sqrt(2)).astype(
                    np.complex64)
                h = ((rng.standard_normal((ports, rx, n)) + 1j * rng.standard_normal((ports, rx, n))) /
                     np.sqrt(2)).astype(np.complex64)
                scaling, noise = 0.8, 0.03
                x, csi = oracle.ref_predecode(y, h, layers, cb, scheme, scaling, noise)
                data[f"pre{k}_cfg"] = np.array([scheme, ports, rx, layers, cb, n], np.int32)
                data[f"pre{k}_sc"] = np.array([scaling, noise], np.float32)
                data[f"pre{k}_y"] = y
                data[f"pre{k}_h"] = h
                data[f"pre{k}_x"] = x
                data[f"pre{k}_csi"] = csi
                k += 1
    data["pre_n"] = np.int32(k)
    np.savez_compressed(os.path.join(OUT, "pdsch_stages.npz"), **data)
    print("pdsch_stages.npz:", data["demod_n"], "demod,", data["scr_n"], "scrambling,", k, "predecoding cases")


PIN_N = 14400  # PDSCH REs of a full-allocation 100-PRB 2-port subframe, CFI 1, no PBCH / sync (sf 1)


def pin_inputs(seed: int, scheme: int, ports: int, rx: int, n: int):
    """Inputs of one equaliser pin case (regenerated by tests/test_ref_pins.py from the same seed)."""
    rng = np.random.default_rng(seed)
    y = ((rng.standard_normal((rx, n)) + 1j * rng.standard_normal((rx, n))) / np.sqrt(2)).astype(np.complex64)
    h = ((rng.standard_normal((ports, rx, n)) + 1j * rng.standard_normal((ports, rx, n))) / np.sqrt(2)).astype(
        np.complex64)
    return y, h


# (scheme, ports, rx, layers, codebook, scaling, noise): every srslte_predecoding_type branch srslte_pdsch_decode takes
PIN_CASES = [(0, 1, 1, 1, 0, 1.0, 0.01), (0, 1, 2, 1, 0, 0.8, 0.03), (0, 1, 2, 1, 0, 1.0, 0.0),
             (1, 2, 1, 2, 0, 1.0, 0.0), (1, 2, 2, 2, 0, 0.7079, 0.0),
             (2, 2, 2, 2, 0, 1.0, 0.02), (2, 2, 2, 2, 1, 1.0, 0.02), (2, 2, 2, 2, 2, 0.8, 0.05),
             (2, 2, 2, 2, 1, 1.0, 0.0),
             (2, 2, 2, 1, 0, 1.0, 0.02), (2, 2, 2, 1, 1, 1.0, 0.02), (2, 2, 2, 1, 2, 1.0, 0.02),
             (2, 2, 2, 1, 3, 0.8, 0.02), (3, 2, 2, 2, 0, 1.0, 0.02)]

# RE map pins: (nof_prb, ports, cell_id, cfi, sf, tdd, allocation seed or -1 for full)
PIN_MAPS = [(p, a, c, f, s, t, -1 if k % 2 == 0 else k)
            for k, (p, a, c, f, s, t) in enumerate(
                (p, a, c, f, s, t) for p in (6, 7, 15, 25, 27, 50, 75, 100, 110) for a in (1, 2, 4)
                for c in (0, 1, 2, 5, 301) for f in (1, 2, 3) for s in (0, 1, 5, 6) for t in (0, 1))]


def pin_alloc(nof_prb: int, seed: int) -> np.ndarray:
    if seed < 0:
        return np.ones((2, nof_prb), np.uint8)
    prb = (np.random.default_rng(seed).random(nof_prb) < 0.6).astype(np.uint8)
    return np.stack([prb, prb])


def sha(a: np.ndarray) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def gen_ref_pins():
    data = {}
    for k, (scheme, ports, rx, layers, cb, scaling, noise) in enumerate(PIN_CASES):
        y, h = pin_inputs(9000 + k, scheme, ports, rx, PIN_N)
        x, csi = oracle.ref_predecode_scalar(y, h, layers, cb, scheme, scaling, noise)
        used = 2 if (layers == 2 and scheme >= 2) else 1
        data[f"eq{k}_in_sha"] = np.array(sha(y) + sha(h))
        data[f"eq{k}_x_sha"] = np.array(sha(x))
        data[f"eq{k}_csi_sha"] = np.array(sha(csi[:used]))
        data[f"eq{k}_x_head"] = x[:, :64].copy()
        data[f"eq{k}_csi_head"] = csi[:used, :64].copy()
    data["eq_n"] = np.int32(len(PIN_CASES))
    shas = []
    for (nof_prb, ports, cid, cfi, sf, tdd, seed) in PIN_MAPS:
        m = oracle.ref_pdsch_re_map(nof_prb, ports, cid, pin_alloc(nof_prb, seed), cfi + (nof_prb < 10), sf,
                                    tdd=bool(tdd))
        shas.append(np.frombuffer(bytes.fromhex(sha(m.astype(np.uint32))), np.uint8))
    data["map_sha"] = np.stack(shas)  # (cases, 32) SHA-256 digests
    # smoothing filters: Gauss order 1..14 x sigma, 3-tap w, triangle lengths
    for order in range(1, 15):
        for j, sd in enumerate((0.1, 0.5, 1.0, 2.0, 3.7, 10.0)):
            data[f"gauss{order}_{j}"] = oracle.ref_chest_filter(0, order, sd)
    for j, w in enumerate((0.0, 0.1, 0.25, 0.3333)):
        data[f"tri3_{j}"] = oracle.ref_chest_filter(1, 3, 0.0, w)
    np.savez_compressed(os.path.join(OUT, "ref_pins.npz"), **data)
    print("ref_pins.npz:", len(PIN_CASES), "equaliser cases,", len(PIN_MAPS), "RE maps")


def gen_pdcch(rng):
    import ctypes as C

    from oracle import pdcch_chain as P
    R = P._ref()
    data = {}
    cells = [(6, 1, 1, 2), (15, 2, 0, 0), (25, 2, 3, 1), (50, 4, 7, 3), (75, 1, 301, 2), (100, 2, 1, 0),
             (100, 4, 503, 1), (100, 1, 77, 2)]
    for k, (nprb, ports, cid, res) in enumerate(cells):
        rg = P.regs(nprb, ports, cid, res, use_ref=True)
        data[f"regs{k}_cell"] = np.array([nprb, ports, cid, res], np.int32)
        data[f"regs{k}_pcfich"] = rg.pcfich
        data[f"regs{k}_nregs"] = rg.nregs
        for c in range(3):
            data[f"regs{k}_pdcch{c}"] = rg.pdcch[c]
        data[f"regs{k}_phich"] = rg.phich
    data["regs_n"] = np.int32(len(cells))
    locs = []
    for ncce in (1, 2, 5, 8, 17, 21, 43, 86, 88):
        for sf in range(10):
            for rnti in (0x1234, 0x000B, 0xFFF3, 0x4601):
                u = P.ue_locations(ncce, sf, rnti, use_ref=True)
                locs.append([ncce, sf, rnti, len(u)] + [v for lv in u for v in lv] + [0] * (32 - 2 * len(u)))
        c = P.common_locations(ncce, use_ref=True)
        locs.append([ncce, 0, 0xFFFF, len(c)] + [v for lv in c for v in lv] + [0] * (32 - 2 * len(c)))
    data["locations"] = np.array(locs, np.int32)
    k = 0
    for n in (1, 7, 8, 15, 16, 27, 43, 57, 61, 128):
        for _ in range(2):
            b = rng.integers(0, 2, n, dtype=np.uint8)
            data[f"crc{k}_bits"] = b
            data[f"crc{k}_crc"] = np.uint32(R.ref_crc16(b, n))
            k += 1
    data["crc_n"] = np.int32(k)
    k = 0
    for F in (28, 37, 43, 57, 60, 72, 144):
        for kind in ("noisy", "rand", "edge"):
            if kind == "rand":
                sym = rng.integers(0, 65536, 3 * F, dtype=np.uint16)
            elif kind == "edge":
                sym = rng.choice(np.array([0, 1, 32767, 32768, 65534, 65535], np.uint16), 3 * F)
            else:
                bits = rng.integers(0, 2, F, dtype=np.uint8)
                coded = np.zeros(3 * F, np.uint8)
                P._lib().orc_conv_encode_tb(bits, F, coded)
                sym = np.clip(32767.5 + (1 - 2 * coded.astype(np.float64)) * 700 + rng.normal(0, 600, 3 * F), 0,
                              65535).astype(np.uint16)
            out = np.zeros(F, np.uint8)
            R.ref_viterbi_decode_us(sym, F, out)
            data[f"vit{k}_sym"] = sym
            data[f"vit{k}_bits"] = out
            k += 1
    data["vit_n"] = np.int32(k)
    k = 0
    for nb in (8, 21, 27, 31, 43, 57, 61):
        for L in range(4):
            E = 72 << L
            bits = rng.integers(0, 2, nb, dtype=np.uint8)
            e = np.zeros(E, np.uint8)
            R.ref_pdcch_dci_encode(bits.copy(), nb, 0x1234, E, e)
            data[f"enc{k}_bits"] = bits
            data[f"enc{k}_e"] = e
            for snr in (0.4, 1.0, 2.5):
                llr = ((1 - 2 * e.astype(np.float32)) * snr + rng.normal(0, 1, E)).astype(np.float32)
                pay = np.zeros(nb + 16, np.uint8)
                crc = R.ref_pdcch_dci_decode(llr, E, nb, pay)
                data[f"dec{k}_{snr}_llr"] = llr
                data[f"dec{k}_{snr}_out"] = pay
                data[f"dec{k}_{snr}_crc"] = np.int32(crc)
            k += 1
    data["enc_n"] = np.int32(k)
    k = 0
    for (nprb, ports, nrx, cid, sf, cfi, snr) in [(6, 1, 1, 1, 0, 1, 30), (6, 2, 2, 4, 5, 3, 10),
                                                  (25, 2, 2, 3, 3, 2, 20), (50, 1, 2, 7, 9, 3, 15),
                                                  (100, 2, 2, 1, 1, 1, 25), (100, 4, 2, 5, 7, 3, 18),
                                                  (15, 4, 1, 0, 2, 2, 12), (100, 1, 1, 77, 4, 2, 3)]:
        rg = P.regs(nprb, ports, cid, 0)
        glen = 14 * 12 * nprb
        tx = np.zeros((ports, glen), np.complex64)
        msgs = []
        nb = P.dci_sizeof(P.FORMAT1A, nprb, ports)
        if rg.nof_cce(cfi) >= 4:
            b = rng.integers(0, 2, nb, dtype=np.uint8)
            b[0] = 1
            msgs.append(dict(bits=b, rnti=0xFFFF, L=2, ncce=0))
        P.ctrl_tx(tx, rg, cid, ports, sf, cfi, msgs)
        h = ((rng.normal(size=(ports, nrx, glen)) + 1j * rng.normal(size=(ports, nrx, glen))) / np.sqrt(2)).astype(
            np.complex64)
        y = np.einsum("prg,pg->rg", h, tx).astype(np.complex64)
        sd = 10 ** (-snr / 20) / np.sqrt(2)
        y += (sd * (rng.normal(size=y.shape) + 1j * rng.normal(size=y.shape))).astype(np.complex64)
        noise = np.float32(2 * sd * sd)
        corr = C.c_float()
        cf = R.ref_pcfich_decode(y.view(np.float32).ravel(), h.view(np.float32).ravel(), nrx, nprb, ports, cid, sf,
                                 noise, C.byref(corr))
        llr = np.zeros(8 * int(rg.nregs[cf - 1]), np.float32)
        R.ref_pdcch_llr(y.view(np.float32).ravel(), h.view(np.float32).ravel(), nrx, nprb, ports, cid, cf, sf, noise,
                        llr)
        ctrl = 4 * 12 * nprb  # only the first 4 OFDM symbols are stored (the control region)
        data[f"sf{k}_cfg"] = np.array([nprb, ports, nrx, cid, sf, cfi], np.int32)
        data[f"sf{k}_y"] = y[:, :ctrl].copy()
        data[f"sf{k}_h"] = h[:, :, :ctrl].copy()
        data[f"sf{k}_noise"] = noise
        data[f"sf{k}_cfi"] = np.int32(cf)
        data[f"sf{k}_corr"] = np.float32(corr.value)
        data[f"sf{k}_llr"] = llr
        data[f"sf{k}_msg"] = msgs[0]["bits"] if msgs else np.zeros(0, np.uint8)
        k += 1
    data["sf_n"] = np.int32(k)
    np.savez_compressed(os.path.join(OUT, "pdcch.npz"), **data)
    print("pdcch.npz:", len(cells), "REG maps,", len(locs), "search spaces,", data["vit_n"], "Viterbi,",
          data["enc_n"], "DCI encode/decode,", k, "control regions")


def main():
    oracle.build(ref=True)
    if not oracle.ref_available():
        sys.exit("oracle/_ref/libsrslte_ref.so is not available (needs /root/reference)")
    if sys.argv[1:] == ["pdcch"]:
        gen_pdcch(np.random.default_rng(4004))
        return
    if sys.argv[1:] == ["pins"]:
        gen_ref_pins()
        return
    if sys.argv[1:] == ["tdec8"]:
        gen_tdec8(np.random.default_rng(8008))
        return
    rng = np.random.default_rng(20201010)
    gen_tdec_auto(rng)
    gen_tdec_generic(rng)
    gen_tcod_known()
    gen_crc_cbsegm(rng)
    gen_rm(np.random.default_rng(1212))
    gen_pdsch_stages(np.random.default_rng(3003))
    gen_pdcch(np.random.default_rng(4004))
    gen_tdec8(np.random.default_rng(8008))
    gen_ref_pins()


if __name__ == "__main__":
    main()
