"""oracle -- TEST INFRASTRUCTURE ONLY.

ctypes access to
  * ``liboracle.so``            -- our scalar C restatement of the srsLTE receive path (the checker,
                                   and bench.py's ``cpu_baseline`` "port");
  * ``_ref/libsrslte_ref.so``   -- the srsLTE 20.10.1 reference compiled from its own sources
                                   (``make -C oracle ref``), used to generate/validate golden vectors and
                                   as the "reference" CPU baseline where the .so is present.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import this
package, and only as the checker -- the product path (``srsran_amd``) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

i16p = np.ctypeslib.ndpointer(np.int16, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")


def build(ref: bool = False) -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref and os.path.isdir("/root/reference/lib"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def lib() -> C.CDLL:
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_cb_index.argtypes = [C.c_uint32]
        L.orc_cb_size.restype = C.c_uint32
        L.orc_cb_size.argtypes = [C.c_int]
        L.orc_qpp.argtypes = [C.c_uint32, u16p]
        L.orc_tdec_nsb.restype = C.c_uint32
        L.orc_tdec_nsb.argtypes = [C.c_uint32]
        L.orc_tdec_buf_len.restype = C.c_uint32
        L.orc_tdec_buf_len.argtypes = [C.c_uint32]
        L.orc_tdec_pack_input.argtypes = [i16p, C.c_uint32, i16p]
        L.orc_tdec_run.argtypes = [i16p, C.c_uint32, C.c_uint32, u8p, C.c_void_p, C.c_void_p]
        L.orc_tdec_run_generic.argtypes = [i16p, C.c_uint32, C.c_uint32, u8p]
        L.orc_tcod_encode.argtypes = [u8p, C.c_uint32, u8p]
        L.orc_crc.restype = C.c_uint32
        L.orc_crc.argtypes = [u8p, C.c_uint32, C.c_uint32, C.c_uint32]
        L.orc_cbsegm.argtypes = [C.c_uint32, u32p]
        L.orc_tdec_run_batch.argtypes = [i16p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u8p, C.c_int]
        L.orc_rm_turbo_table.argtypes = [C.c_uint32, C.c_uint32, u16p]
        L.orc_rm_turbo_rx.argtypes = [i16p, C.c_uint32, i16p, C.c_uint32, C.c_uint32]
        L.orc_dlsch_decode_tb.argtypes = [i16p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                          i16p, u8p, u8p, u8p, C.POINTER(C.c_float)]
        L.orc_rm_turbo_tx.argtypes = [u8p, C.c_uint32, C.c_uint32, C.c_uint32, u8p]
        L.orc_dlsch_encode_tb.argtypes = [u8p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u8p]
        L.orc_sequence_lte.argtypes = [C.c_uint32, C.c_uint32, u8p]
        L.orc_demod_soft_s.argtypes = [C.c_int, f32p, i16p, C.c_int]
        L.orc_scramble_s.argtypes = [C.c_uint32, i16p, C.c_uint32]
        L.orc_csi_correction_s.argtypes = [C.c_int, i16p, f32p, C.c_uint32]
        L.orc_pdsch_re_map.restype = C.c_uint32
        L.orc_pdsch_re_map.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_uint32,
                                       C.c_uint32, u8p, C.c_uint32, C.c_uint32, u32p]
        L.orc_chest_filter.restype = C.c_uint32
        L.orc_chest_filter.argtypes = [C.c_int, C.c_float, C.c_float, C.c_float, f32p]
        L.orc_crs_pilots.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, f32p]
        L.orc_chest_estimate_port.argtypes = [f32p, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, C.c_int,
                                              C.c_float, C.c_float, C.c_int, f32p, f32p]
        L.orc_chest_estimate_port_st.argtypes = [f32p, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32,
                                                 C.c_int, C.c_float, C.c_float, C.c_int, C.c_int, C.c_float, f32p,
                                                 f32p]
        L.orc_chest_sync_correct.argtypes = [f32p, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32,
                                             C.c_uint32, f32p]
        L.orc_chest_cfo.restype = C.c_float
        L.orc_chest_cfo.argtypes = [f32p, C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.c_uint32]
        L.orc_noise_empty.restype = C.c_float
        L.orc_noise_empty.argtypes = [f32p, C.c_uint32, C.c_int]
        L.orc_pss_generate.argtypes = [C.c_uint32, f32p]
        L.orc_noise_pss.restype = C.c_float
        L.orc_noise_pss.argtypes = [f32p, f32p, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32]
        L.orc_predecode.argtypes = [f32p, f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float,
                                    C.c_float, f32p, f32p, f32p]
        L.orc_ofdm_rx_sf.argtypes = [f32p, C.c_uint32, f32p]
        L.orc_ue_dl_front.argtypes = [C.POINTER(FrontCfg), C.c_void_p * 2, C.c_void_p * 2, C.POINTER(C.c_float)]
        L.orc_dlsch_rm_tb.argtypes = [i16p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, i16p, C.c_uint32]
        L.orc_ue_dl_rx_batch.argtypes = [C.POINTER(FrontCfg), C.c_uint32, f32p, C.c_size_t, i16p, C.c_uint32,
                                         C.c_uint32, C.c_int]
        L.orc_front_set_stages.argtypes = [C.c_void_p]
        _LIB = L
    return _LIB


class FrontCfg(C.Structure):
    """orc_front_cfg_t (oracle.h)."""
    _fields_ = [(n, C.c_uint32) for n in ("nof_prb", "nof_ports", "nof_rx", "cell_id", "cfi", "sf_idx", "rnti",
                                          "scheme", "nof_layers", "cb", "nof_tb")] + \
               [("qm", C.c_uint32 * 2), ("tbs", C.c_uint32 * 2), ("rv", C.c_uint32 * 2), ("csi_enable", C.c_int32),
                ("power_scale", C.c_int32), ("mmse", C.c_int32), ("p_a", C.c_float), ("p_b", C.c_uint32)]


def front_cfg(cfg) -> FrontCfg:
    """pdsch_chain.Cfg -> orc_front_cfg_t."""
    f = FrontCfg()
    for n in ("nof_prb", "nof_ports", "nof_rx", "cell_id", "cfi", "sf_idx", "rnti", "scheme", "nof_layers"):
        setattr(f, n, int(getattr(cfg, n)))
    f.cb, f.nof_tb = cfg.codebook(), cfg.nof_tb
    for t in range(cfg.nof_tb):
        f.qm[t], f.tbs[t], f.rv[t] = cfg.qm[t], cfg.tbs[t], cfg.rv[t]
    f.csi_enable, f.power_scale, f.mmse = int(cfg.csi_enable), int(cfg.power_scale), int(cfg.mmse)
    f.p_a, f.p_b = float(cfg.p_a), int(cfg.p_b)
    return f


class FrontStages(C.Structure):
    """orc_front_stages_t (oracle.h): the front end's replaceable stage functions, as raw addresses."""
    _fields_ = [(n, C.c_void_p) for n in ("predecode", "demod_soft_s", "scramble_s", "rm_turbo_rx")]


def front_use_reference(on: bool = True) -> bool:
    """Run orc_ue_dl_front's equaliser, demapper, descrambler and rate dematcher through the reference's own AVX2
    code (oracle/ref/ref_front.c, ref_pdsch.c, ref_harness.c in oracle/_ref) instead of the restatement's (on=False:
    back to the restatement).  Returns whether the reference stages are installed."""
    L = lib()
    if not on or not ref_available():
        L.orc_front_set_stages(None)
        return False
    R = ref()
    addr = lambda f: C.cast(f, C.c_void_p).value  # noqa: E731
    st = FrontStages(addr(R.ref_front_predecode), addr(R.ref_demod_soft_s), addr(R.ref_front_scramble_s),
                     addr(R.ref_rm_turbo_rx))
    L.orc_front_set_stages(C.byref(st))
    return True


def _aligned_i16(n: int, align: int = 64) -> np.ndarray:
    buf = np.zeros(n + align, np.int16)
    off = (-buf.ctypes.data % align) // 2
    return buf[off: off + n]


def ue_dl_front(cfg, iq: np.ndarray):
    """orc_ue_dl_front: iq (nof_rx, 15 N) complex64 -> (e per TB int16, noise)."""
    iq = np.ascontiguousarray(iq, np.complex64)
    e = [_aligned_i16(8 * 14 * 1200) for _ in range(2)]  # 64-byte aligned: the reference stages' SIMD stores
    ip = (C.c_void_p * 2)(iq[0].ctypes.data, iq[min(1, iq.shape[0] - 1)].ctypes.data)
    ep = (C.c_void_p * 2)(e[0].ctypes.data, e[1].ctypes.data)
    noise = C.c_float()
    f = front_cfg(cfg)
    nre = lib().orc_ue_dl_front(C.byref(f), ip, ep, C.byref(noise))
    if nre < 0:
        raise ValueError("orc_ue_dl_front: invalid configuration")
    return [e[t][: nre * cfg.qm[t]].copy() for t in range(cfg.nof_tb)], float(noise.value)


def ref_available() -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", "libsrslte_ref.so"))


def ref() -> C.CDLL:
    global _REF
    if _REF is None:
        L = C.CDLL(os.path.join(HERE, "_ref", "libsrslte_ref.so"))
        i8p = np.ctypeslib.ndpointer(np.int8, flags="C_CONTIGUOUS")
        L.ref_tdec_new.restype = C.c_void_p
        L.ref_tdec_new.argtypes = [C.c_uint32, C.c_int]
        L.ref_tdec_free.argtypes = [C.c_void_p]
        L.ref_tdec_run.argtypes = [C.c_void_p, i16p, C.c_uint32, C.c_uint32, u8p, C.c_void_p]
        L.ref_tcod_encode.argtypes = [u8p, u8p, C.c_uint32]
        L.ref_crc_byte.restype = C.c_uint32
        L.ref_crc_byte.argtypes = [C.c_uint32, C.c_int, u8p, C.c_int]
        L.ref_cbsegm.argtypes = [C.c_uint32, u32p]
        L.ref_rm_turbo_rx.argtypes = [i16p, C.c_uint32, i16p, C.c_uint32, C.c_uint32]
        L.ref_tdec8_new.restype = C.c_void_p
        L.ref_tdec8_new.argtypes = [C.c_uint32]
        L.ref_tdec8_free.argtypes = [C.c_void_p]
        L.ref_tdec8_run.argtypes = [C.c_void_p, i8p, C.c_uint32, C.c_uint32, u8p, C.c_void_p]
        L.ref_rm_turbo_rx_8bit.argtypes = [i8p, C.c_uint32, i8p, C.c_uint32, C.c_uint32]
        L.ref_tdec_run_batch.argtypes = [i16p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u8p, C.c_int]
        L.ref_demod_soft_s.argtypes = [C.c_int, f32p, i16p, C.c_int]
        L.ref_scramble_s.argtypes = [C.c_uint32, i16p, C.c_int, C.c_int]
        L.ref_demod_soft_b.argtypes = [C.c_int, f32p, i8p, C.c_int]
        L.ref_scramble_sb.argtypes = [C.c_uint32, i8p, C.c_int, C.c_int]
        L.ref_predecoding.argtypes = [C.c_void_p] * 10 + [C.c_int] * 6 + [C.c_float, C.c_float, C.c_int]
        L.ref_front_predecode.argtypes = [f32p, f32p] + [C.c_int] * 6 + [C.c_float, C.c_float, f32p, f32p, f32p]
        L.ref_front_scramble_s.argtypes = [C.c_uint32, i16p, C.c_int]
        L.ref_pdsch_get_map.restype = C.c_int
        L.ref_pdsch_get_map.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int, C.c_uint32, C.c_uint32,
                                        u8p, C.c_uint32, C.c_uint32, u32p]
        L.ref_chest_filter.restype = C.c_uint32
        L.ref_chest_filter.argtypes = [C.c_int, C.c_uint32, C.c_float, C.c_float, f32p]
        L.ref_chest_noise_pilots.restype = C.c_float
        L.ref_chest_noise_pilots.argtypes = [f32p, f32p, f32p, C.c_uint32]
        _REF = L
    return _REF


# ------------------------------------------------------------------ thin helpers

def cb_sizes() -> list[int]:
    L = lib()
    return [int(L.orc_cb_size(i)) for i in range(188)]


def qpp(K: int) -> np.ndarray:
    out = np.zeros(K, np.uint16)
    assert lib().orc_qpp(K, out) == 0
    return out


def tdec_nsb(K: int) -> int:
    return int(lib().orc_tdec_nsb(K))


def tdec_buf_len(K: int) -> int:
    return int(lib().orc_tdec_buf_len(K))


def tdec_pack_input(lin: np.ndarray, K: int) -> np.ndarray:
    buf = np.zeros(tdec_buf_len(K), np.int16)
    lib().orc_tdec_pack_input(np.ascontiguousarray(lin, np.int16), K, buf)
    return buf


def tdec_run(buf: np.ndarray, K: int, nhalf: int, trace: bool = False, llr: bool = False):
    out = np.zeros(K // 8, np.uint8)
    tr = np.zeros((nhalf, K // 8), np.uint8) if trace else None
    lo = np.zeros(K, np.int16) if llr else None
    rc = lib().orc_tdec_run(np.ascontiguousarray(buf, np.int16), K, nhalf, out,
                            tr.ctypes.data if tr is not None else None,
                            lo.ctypes.data if lo is not None else None)
    assert rc == 0
    res = [out]
    if trace:
        res.append(tr)
    if llr:
        res.append(lo)
    return res[0] if len(res) == 1 else tuple(res)


def tdec_run_generic(lin: np.ndarray, K: int, nhalf: int) -> np.ndarray:
    out = np.zeros(K // 8, np.uint8)
    assert lib().orc_tdec_run_generic(np.ascontiguousarray(lin, np.int16), K, nhalf, out) == 0
    return out


def tdec_run_batch(bufs: np.ndarray, K: int, nhalf: int, nthreads: int) -> np.ndarray:
    bufs = np.ascontiguousarray(bufs, np.int16)
    out = np.zeros((bufs.shape[0], K // 8), np.uint8)
    lib().orc_tdec_run_batch(bufs, bufs.shape[1], bufs.shape[0], K, nhalf, out, nthreads)
    return out


def tcod_encode(bits: np.ndarray, K: int) -> np.ndarray:
    out = np.zeros(3 * K + 12, np.uint8)
    assert lib().orc_tcod_encode(np.ascontiguousarray(bits, np.uint8), K, out) == 0
    return out


CRC24A = (0x1864CFB, 24)
CRC24B = (0x1800063, 24)
CRC16 = (0x11021, 16)
CRC8 = (0x19B, 8)


def crc(data_bytes: np.ndarray, nbits: int, poly_order=CRC24A) -> int:
    return int(lib().orc_crc(np.ascontiguousarray(data_bytes, np.uint8), nbits, poly_order[0], poly_order[1]))


def cbsegm(tbs: int) -> dict:
    r = np.zeros(6, np.uint32)
    assert lib().orc_cbsegm(tbs, r) == 0
    return dict(zip(["C", "K1", "K2", "C1", "C2", "F"], [int(v) for v in r]))


SOFTBUFFER_SIZE = 18600


def rm_turbo_table(K: int, rv: int) -> np.ndarray:
    t = np.zeros(3 * K + 12, np.uint16)
    lib().orc_rm_turbo_table(K, rv, t)
    return t


def rm_turbo_rx(e: np.ndarray, K: int, rv: int, out: np.ndarray | None = None) -> np.ndarray:
    """srslte_rm_turbo_rx_lut: accumulate (wrapping) into out (a SOFTBUFFER_SIZE int16 buffer)."""
    if out is None:
        out = np.zeros(SOFTBUFFER_SIZE, np.int16)
    e = np.ascontiguousarray(e, np.int16)
    assert lib().orc_rm_turbo_rx(e, e.size, out, K, rv) == 0
    return out


class Softbuffer:
    """srslte_softbuffer_rx_t equivalent (softbuffer.h:37-43) for the oracle TB decoder."""

    def __init__(self, max_cb: int = 32):
        self.buf = np.zeros((max_cb, SOFTBUFFER_SIZE), np.int16)
        self.cb_crc = np.zeros(max_cb, np.uint8)
        self.data = np.zeros((max_cb, 768), np.uint8)

    def reset(self):
        self.buf[:] = 0
        self.cb_crc[:] = 0
        self.data[:] = 0


def dlsch_decode_tb(e_bits: np.ndarray, tbs: int, Qm: int, rv: int, max_its: int, sb: Softbuffer):
    """decode_tb (sch.c:503-570): returns (ret, data bytes, avg half-iterations)."""
    e = np.ascontiguousarray(e_bits, np.int16)
    data = np.zeros(tbs // 8 + 8, np.uint8)
    its = C.c_float()
    ret = lib().orc_dlsch_decode_tb(e, e.size, tbs, Qm, rv, max_its, sb.buf, sb.cb_crc, sb.data, data,
                                    C.byref(its))
    return ret, data, its.value


def dlsch_encode_tb(payload_bits: np.ndarray, tbs: int, Qm: int, G: int, rv: int) -> np.ndarray:
    """TB -> G coded bits (CRC24A, segmentation + CRC24B, turbo coding, rate matching)."""
    e = np.zeros(G, np.uint8)
    assert lib().orc_dlsch_encode_tb(np.ascontiguousarray(payload_bits, np.uint8), tbs, Qm, G, rv, e) == 0
    return e


def make_tb(rng: np.random.Generator, tbs: int, Qm: int, G: int, rv: int, snr_db: float, scale: float = 100.0):
    """Random TB -> int16 LLRs of its G coded bits over BPSK/AWGN (positive = bit 1), plus payload bytes."""
    bits = rng.integers(0, 2, tbs, dtype=np.uint8)
    coded = dlsch_encode_tb(bits, tbs, Qm, G, rv)
    sigma = 10 ** (-snr_db / 20)
    y = np.where(coded.astype(bool), 1.0, -1.0) + sigma * rng.standard_normal(G)
    llr = np.trunc(scale * y).clip(-32768, 32767).astype(np.int16)
    return np.packbits(bits), llr


def sequence_lte(c_init: int, n: int) -> np.ndarray:
    c = np.zeros(n, np.uint8)
    lib().orc_sequence_lte(c_init, n, c)
    return c


def demod_soft_s(qm: int, symbols: np.ndarray) -> np.ndarray:
    iq = np.ascontiguousarray(np.asarray(symbols, np.complex64).view(np.float32))
    out = np.zeros(qm * (iq.size // 2), np.int16)
    assert lib().orc_demod_soft_s(qm, iq, out, iq.size // 2) == 0
    return out


def scramble_s(c_init: int, llr: np.ndarray) -> np.ndarray:
    out = np.array(llr, np.int16, copy=True)
    lib().orc_scramble_s(c_init, out, out.size)
    return out


def csi_correction_s(qm: int, e: np.ndarray, csi: np.ndarray) -> np.ndarray:
    out = np.array(e, np.int16, copy=True)
    lib().orc_csi_correction_s(qm, out, np.ascontiguousarray(csi, np.float32), out.size)
    return out


def pdsch_re_map(nof_prb: int, nof_ports: int, cell_id: int, prb: np.ndarray, lstart: int, sf_idx: int,
                 tdd: bool = False, cp_ext: bool = False, nof_symb_slot=(0, 0)) -> np.ndarray:
    """Grid indices of the PDSCH REs in srslte_pdsch_get order (pdsch.c:136-228); prb: (2, nof_prb) bool."""
    prb = np.ascontiguousarray(np.asarray(prb, np.uint8).reshape(2, nof_prb))
    idx = np.zeros(14 * 12 * nof_prb, np.uint32)
    n = lib().orc_pdsch_re_map(nof_prb, nof_ports, cell_id, int(tdd), int(cp_ext), nof_symb_slot[0],
                               nof_symb_slot[1], prb, lstart, sf_idx, idx)
    return idx[:n].copy()


def predecode(y: np.ndarray, h: np.ndarray, nof_layers: int, cb: int, tx_scheme: int, scaling: float,
              noise: float):
    """orc_predecode: y (nof_rx, n) complex64, h (nof_ports, nof_rx, n) complex64 ->
    (x (nof_layers, n_layer) complex64, csi (2, n) float32)."""
    y = np.ascontiguousarray(y, np.complex64)
    nof_rx, n = y.shape
    nof_ports = h.shape[0]
    hh = np.zeros((nof_ports, 2, n), np.complex64)
    hh[:, :nof_rx] = h
    x = np.zeros((max(nof_layers, 1), n), np.complex64)
    csi = np.zeros((2, n), np.float32)
    r = lib().orc_predecode(y.view(np.float32), hh.view(np.float32).reshape(-1), nof_rx, nof_ports, nof_layers,
                            cb, n, tx_scheme, scaling, noise, x.view(np.float32).reshape(-1), csi[0], csi[1])
    if r < 0:
        raise ValueError("orc_predecode: invalid configuration")
    nl = n // nof_ports if tx_scheme == 1 else n
    return x[:, :nl].copy(), csi


def _aligned(a: np.ndarray, align: int = 64) -> np.ndarray:
    """Copy into an `align`-byte aligned buffer (the reference's SIMD kernels use aligned loads)."""
    a = np.asarray(a)
    raw = np.zeros(a.nbytes + align, np.uint8)
    off = (-raw.ctypes.data) % align
    out = raw[off:off + a.nbytes].view(a.dtype).reshape(a.shape)
    out[...] = a
    return out


def ref_predecode(y: np.ndarray, h: np.ndarray, nof_layers: int, cb: int, tx_scheme: int, scaling: float,
                  noise: float):
    """The reference's srslte_predecoding_type (AVX2 build) through oracle/_ref, same layout as predecode()."""
    y = np.ascontiguousarray(y, np.complex64)
    nof_rx, n = y.shape
    nof_ports = h.shape[0]
    H = [[_aligned(h[p, r].astype(np.complex64)) if p < nof_ports and r < nof_rx else None
          for r in range(2)] for p in range(2)]
    x = [_aligned(np.zeros(n, np.complex64)) for _ in range(2)]
    csi = [_aligned(np.zeros(n, np.float32)) for _ in range(2)]
    ptr = lambda a: None if a is None else a.ctypes.data
    ys = [_aligned(y[0]), _aligned(y[1]) if nof_rx > 1 else None]
    r = ref().ref_predecoding(ptr(ys[0]), ptr(ys[1]), ptr(H[0][0]), ptr(H[0][1]), ptr(H[1][0]), ptr(H[1][1]),
                              ptr(x[0]), ptr(x[1]), ptr(csi[0]), ptr(csi[1]), nof_rx, nof_ports, nof_layers, cb, n,
                              tx_scheme, scaling, noise, 1)
    if r < 0:
        raise ValueError("ref_predecoding failed")
    nl = n // nof_ports if tx_scheme == 1 else n
    return np.stack(x)[:nof_layers, :nl].copy(), np.stack(csi)


def chest_filter(filter_type: int, coef0: float, coef1: float, noise: float = 0.0) -> np.ndarray:
    """orc_chest_filter: the estimator's smoothing taps (Gauss / 3-tap / none) as chest_dl.c sets them up."""
    f = np.zeros(32, np.float32)
    n = lib().orc_chest_filter(filter_type, coef0, coef1, noise, f)
    return f[:n].copy()


def ref_chest_filter(kind: int, order: int, sigma: float = 0.0, w: float = 0.0) -> np.ndarray:
    """chest_common.c compiled from the reference (oracle/_ref): 0 Gauss(order, sigma), 1 3-tap(w), 2 triangle."""
    f = np.zeros(64, np.float32)
    n = ref().ref_chest_filter(kind, order, sigma, w, f)
    return f[:n].copy()


def ref_pdsch_re_map(nof_prb: int, nof_ports: int, cell_id: int, prb: np.ndarray, lstart: int, sf_idx: int,
                     tdd: bool = False, cp_ext: bool = False, nof_symb_slot=(0, 0)) -> np.ndarray:
    """The RE -> grid map in extraction order through the reference's compiled prb_dl.c primitives
    (oracle/ref/ref_prb.c); same arguments as pdsch_re_map()."""
    prb = np.ascontiguousarray(np.asarray(prb, np.uint8).reshape(2, nof_prb))
    idx = np.zeros(14 * 12 * nof_prb, np.uint32)
    n = ref().ref_pdsch_get_map(nof_prb, nof_ports, cell_id, int(tdd), int(cp_ext), nof_symb_slot[0],
                                nof_symb_slot[1], prb, lstart, sf_idx, idx)
    if n < 0:
        raise ValueError("ref_pdsch_get_map: invalid configuration")
    return idx[:n].copy()


def ref_predecode_scalar(y: np.ndarray, h: np.ndarray, nof_layers: int, cb: int, tx_scheme: int, scaling: float,
                         noise: float):
    """The reference's srslte_predecoding_type on chunks shorter than one AVX2 vector (8 complex values), so every RE
    takes the scalar bodies (precoding.c:309-357 single_csi tail, :1519-1548 2x2 MMSE tail -> mat.c:63-109,
    :1802-1820 2x1 MRC tail, the diversity / CDD tails): the exact-division path, independent of the host CPU's
    rcp_ps.  Same layout as predecode(); chunks are whole SFBC groups (4 REs for 4 ports, else 6)."""
    y = np.ascontiguousarray(y, np.complex64)
    n = y.shape[1]
    nof_ports = h.shape[0]
    ch = 4 if (tx_scheme == 1 and nof_ports == 4) else 6
    xs, cs = [], []
    for a in range(0, n, ch):
        b = min(n, a + ch)
        x, c = ref_predecode(y[:, a:b], h[:, :, a:b], nof_layers, cb, tx_scheme, scaling, noise)
        xs.append(x)
        cs.append(c[:, : b - a])
    return np.concatenate(xs, 1), np.concatenate(cs, 1)


def pdsch_c_init(rnti: int, cw: int, sf: int, cell_id: int) -> int:
    """srslte_sequence_pdsch (phch/sequences.c:61-64) with nslot = 2*sf."""
    return (rnti << 14) + (cw << 13) + (sf << 9) + cell_id


# ------------------------------------------------------------------ test-vector synthesis

def awgn_llrs(rng: np.random.Generator, coded_bits: np.ndarray, ebno_db: float, scale: float = 100.0) -> np.ndarray:
    """BPSK + AWGN at Eb/N0 for a rate-1/3 code, LLR = int16(scale * (+-1 + sigma*n)) as
    turbodecoder_test.c:236-247 does (positive = bit 1).  numpy RNG replaces glibc rand()."""
    esno_db = ebno_db + 10 * np.log10(1.0 / 3.0)
    sigma = 10 ** (-esno_db / 20)
    sym = np.where(coded_bits.astype(bool), 1.0, -1.0).astype(np.float32)
    y = sym + np.float32(sigma) * rng.standard_normal(sym.shape).astype(np.float32)
    return np.trunc(scale * y).clip(-32768, 32767).astype(np.int16)


def make_cb(rng: np.random.Generator, K: int, ebno_db: float, scale: float = 100.0):
    """Random info bits -> encoder-ordered int16 LLRs (3K+12) -> AUTO-layout decoder buffer."""
    bits = rng.integers(0, 2, K, dtype=np.uint8)
    coded = tcod_encode(bits, K)
    lin = awgn_llrs(rng, coded, ebno_db, scale)
    return bits, lin, tdec_pack_input(lin, K)


# ------------------------------------------------------------------ reference wrappers

class RefTdec:
    """The reference decoder (AUTO, or GENERIC manual + force_not_sb)."""

    def __init__(self, generic: bool = False, max_K: int = 6144):
        self.L = ref()
        self.h = self.L.ref_tdec_new(max_K, 1 if generic else 0)

    def run(self, buf: np.ndarray, K: int, nhalf: int, trace: bool = False):
        b = np.array(buf, np.int16, copy=True)
        out = np.zeros(K // 8, np.uint8)
        tr = np.zeros((nhalf, K // 8), np.uint8) if trace else None
        assert self.L.ref_tdec_run(self.h, b, K, nhalf, out, tr.ctypes.data if tr is not None else None) == 0
        return (out, tr) if trace else out

    def __del__(self):
        try:
            self.L.ref_tdec_free(self.h)
        except Exception:
            pass


def ref_dlsch_decode_cbs(bufs: np.ndarray, K: int, tbs: int, max_half: int = 10, dec: "RefTdec | None" = None):
    """decode_tb_cb + decode_tb of the reference (sch.c:382-486, :531-556) on fresh softbuffers, through the
    REFERENCE's own AVX2 turbo decoder (oracle/_ref) and its CRC: every code block is decoded half-iteration by
    half-iteration (srslte_tdec_iteration) until the CRC24B of its K decision bits (the TB CRC24A when C == 1) is zero
    or max_half half-iterations ran; the TB passes when every block passed and the TB CRC over tbs bits equals the
    transmitted parity and is non-zero (sch.c:543-549).  bufs: (C, stride) int16 decoder buffers of one TB (the
    16-window layout).  Returns (tb_ok, data bytes (tbs/8 + 3), per-CB passed (C,), per-CB half-iterations (C,))."""
    L = ref()
    dec = dec or RefTdec()
    C = bufs.shape[0]
    rlen = K - 24 if C > 1 else K
    data = np.zeros(C * rlen // 8 + K // 8, np.uint8)
    ok = np.zeros(C, bool)
    its = np.zeros(C, np.int32)
    for c in range(C):
        _, tr = dec.run(bufs[c], K, max_half, trace=True)
        for h in range(max_half):
            nb, poly = (K, CRC24B) if C > 1 else (tbs + 24, CRC24A)
            if L.ref_crc_byte(poly[0], poly[1], np.ascontiguousarray(tr[h]), nb) == 0:
                ok[c], its[c] = True, h + 1
                break
        else:
            its[c] = max_half
        data[c * rlen // 8: c * rlen // 8 + K // 8] = tr[its[c] - 1]
    out = data[: tbs // 8 + 3].copy()
    tb_ok = bool(ok.all())
    if tb_ok:
        par_rx = int(L.ref_crc_byte(CRC24A[0], CRC24A[1], np.ascontiguousarray(out), tbs))
        par_tx = (int(out[tbs // 8]) << 16) | (int(out[tbs // 8 + 1]) << 8) | int(out[tbs // 8 + 2])
        tb_ok = par_rx == par_tx and par_rx != 0
    return tb_ok, out, ok, its
