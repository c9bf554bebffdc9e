"""GPU: srslte_pdsch_decode with llr_is_8bit (srsUE pdsch_8bit_decoder) -- mi355_pdsch_set_llr_8bit.  The int8 LLRs
of every codeword are bit-exact with tests/llr8_ref.py (a restatement pinned to the reference's own
srslte_demod_soft_demodulate_b / srslte_scrambling_sb_offset by tests/golden/tdec8.npz) applied to the GPU's own
equalised symbols and CSI (whose parity with the oracle is test_pdsch_gpu.py's business), and every transport block
without CSI weighting decodes through the 8-bit DL-SCH with its payload.  With CSI weighting the reference's int8
path often crushes the LLRs (e * csi / max(csi), truncated: mean |e| ~ 1 on faded 16QAM) and fails the CRC; there the
CRC result of a single-code-block TB must equal what the reference's own srslte_rm_turbo_rx_lut_8bit +
srslte_tdec_iteration_8bit (oracle/_ref) make of the same int8 LLRs within 10 half-iterations."""
import numpy as np
import pytest

import oracle
from oracle import pdsch_chain as pc
from srsran_amd import pdsch as P
from srsran_amd.dlsch import SoftbufferPool
from tests import llr8_ref
from tests.pdsch_jobs import DevSubframe, cell_of
from tests.test_pdsch_gpu import CFGS

pytestmark = pytest.mark.gpu


def ok8(tbs: int) -> bool:
    s = oracle.cbsegm(tbs)
    return all(K <= 400 or (K % 16 == 0 and K > 800) for K in (s["K1"], s["K2"]) if K)


CFGS8 = [c for c in CFGS if all(ok8(t) for t in c.tbs)]


def test_cfgs8_cover_the_schemes():
    assert len(CFGS8) >= 8 and {c.scheme for c in CFGS8} == {0, 1, 2, 3}
    assert {q for c in CFGS8 for q in c.qm} == {2, 4, 6, 8}


@pytest.mark.parametrize("k", range(len(CFGS8)))
def test_pdsch_8bit_llrs_and_decode(k):
    cfg = CFGS8[k]
    rng = np.random.default_rng(800 + k)
    sf = pc.synth_subframe(cfg, rng, snr_db=35)
    ds = DevSubframe(cfg, sf)
    pd = P.Pdsch(cell_of(cfg), cfg.nof_rx)
    pd.set_llr_8bit(True)
    pool = SoftbufferPool(2, max_cb=16)
    res = pd.decode(pool, [ds.job])
    for t in range(cfg.nof_tb):
        qm = cfg.qm[t]
        d, csi, e8 = pd.stage(0, t, sf.nof_re, sf.nof_re * qm)
        want = llr8_ref.demod_b(d, qm)
        c = oracle.sequence_lte(oracle.pdsch_c_init(cfg.rnti, t, cfg.sf_idx, cfg.cell_id), sf.nof_re * qm)
        want = llr8_ref.scramble_sb(want, c)
        if cfg.csi_enable:
            want = llr8_ref.csi_b(want, csi, qm)
        np.testing.assert_array_equal(e8, want, err_msg=f"cfg {k} tb {t}")
        assert res[t].ret == 0, (k, t)
        n = cfg.tbs[t] // 8
        if not cfg.csi_enable:
            assert res[t].crc, (k, t)
        elif oracle.cbsegm(cfg.tbs[t])["C"] == 1 and oracle.ref_available():
            assert bool(res[t].crc) == ref_decodes(e8, cfg.tbs[t], sf.payload[t]), (k, t)
        if res[t].crc:
            np.testing.assert_array_equal(ds.payload_bytes(t)[:n], sf.payload[t], err_msg=f"cfg {k} tb {t}")


def ref_decodes(e8: np.ndarray, tbs: int, payload: np.ndarray) -> bool:
    """The reference's 8-bit rate dematching + decoder on these LLRs (rv 0, C = 1): payload within 10 half-its."""
    R = oracle.ref()
    K = oracle.cbsegm(tbs)["K1"]
    buf = np.zeros(3 * (K + 32) + 12 + 64, np.int8)
    assert R.ref_rm_turbo_rx_8bit(np.ascontiguousarray(e8), e8.size, buf, K, 0) == 0
    h = R.ref_tdec8_new(6144)
    tr = np.zeros((10, K // 8), np.uint8)
    out = np.zeros(K // 8, np.uint8)
    assert R.ref_tdec8_run(h, buf[: 3 * (K + 32) + 12].copy(), K, 10, out, tr.ctypes.data) == 0
    R.ref_tdec8_free(h)
    want = np.unpackbits(np.asarray(payload, np.uint8))[:tbs]
    return any(np.array_equal(np.unpackbits(tr[i])[:tbs], want) for i in range(10))
