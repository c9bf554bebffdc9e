"""CPU tests of the eNodeB-side generator's host chain (include/srsran_amd/enb_dl.h, mi355_*_host), which the GPU
generator (mi355_enb_dl_*) must reproduce bit for bit:

* mi355_tcod_encode_host against the reference's own turbo encoder output (tests/golden/tcod_known.npz, recorded
  from srslte_tcod_encode, turbocoder.c:76-186) and against the oracle encoder for every 40 <= K <= 6144 class;
* mi355_pdsch_encode_host grids against the oracle transmitter (oracle/pdsch_chain.py: dlsch_encode_tb =
  encode_tb_off sch.c:250-355 + rm_turbo_tx, scrambling, 36.211 modulation, layermap/precoding, RE map) --
  with the reference transmitter's amplitudes (rho_a folded into the precoders whatever power_scale says,
  pdsch.c:1174-1188): equal within float rounding;
* mi355_refsignal_cs_put_sf_host against the oracle-side CRS values the estimator tests use.
"""
from __future__ import annotations

import ctypes as C
import zlib

import numpy as np
import pytest

import oracle
from oracle import pdsch_chain as pc
from srsran_amd import enb_dl
from srsran_amd import pdsch as P
from tests.golden_io import load
from tests.pdsch_jobs import cell_of, grant_of


def _tcod_host(bits: np.ndarray, K: int) -> np.ndarray:
    L = enb_dl._declare()
    L.mi355_tcod_encode_host.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    out = np.zeros(3 * K + 12, np.uint8)
    b = np.ascontiguousarray(bits, np.uint8)
    assert L.mi355_tcod_encode_host(b.ctypes.data, K, out.ctypes.data) == 0
    return out


def test_tcod_host_matches_reference_encoder():
    z = load("tcod_known.npz")
    assert np.array_equal(_tcod_host(z["known_data"], 504), z["ref_encoder_out"])


@pytest.mark.parametrize("K", [40, 48, 512, 1024, 2048, 5312, 6144])
def test_tcod_host_matches_oracle(K):
    rng = np.random.default_rng(K)
    bits = rng.integers(0, 2, K, dtype=np.uint8)
    assert np.array_equal(_tcod_host(bits, K), oracle.tcod_encode(bits, K))


def tx_configs():
    """(name, Cfg): every transmit scheme / modulation the generator supports, single and multi code-block TBs,
    every rv, partial allocations, subframes with PBCH / synchronisation signals (0, 5)."""
    out = []
    for qm in (2, 4, 6, 8):
        out.append((f"port0_q{qm}", pc.Cfg(nof_prb=25, cfi=2, sf_idx=3, qm=[qm], tbs=[pc.valid_tbs(700 * qm)],
                                            rv=[qm // 2 - 1, 0])))
    out.append(("port0_sf0_c3", pc.Cfg(nof_prb=25, cfi=1, sf_idx=0, qm=[6], tbs=[pc.valid_tbs(14000)], rv=[2, 0])))
    out.append(("sfbc_sf5", pc.Cfg(nof_prb=15, nof_ports=2, cfi=3, sf_idx=5, scheme=pc.DIVERSITY, nof_layers=2,
                                   qm=[4], tbs=[pc.valid_tbs(4000)], rv=[1, 0])))
    for pmi in (0, 1):  # two codewords: codebook pmi + 1 (pdsch.c / precoding.c:1945-2270)
        out.append((f"sm2_pmi{pmi}", pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, cfi=1, sf_idx=7, scheme=pc.SPATIALMUX,
                                            nof_layers=2, pmi=pmi, qm=[8, 6],
                                            tbs=[pc.valid_tbs(20000), pc.valid_tbs(15000)], rv=[0, 3])))
    for cb in range(4):
        out.append((f"sm1_cb{cb}", pc.Cfg(nof_prb=6, nof_ports=2, nof_rx=2, cfi=2, sf_idx=9, scheme=pc.SPATIALMUX,
                                          nof_layers=1, pmi=cb, qm=[2], tbs=[pc.valid_tbs(600)], rv=[3, 0])))
    out.append(("cdd", pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, cfi=2, sf_idx=1, scheme=pc.CDD, nof_layers=2,
                              qm=[4, 4], tbs=[pc.valid_tbs(8000), pc.valid_tbs(8000)], rv=[0, 1])))
    prb = np.zeros((2, 50), np.uint8)
    prb[:, 3:40:3] = 1
    out.append(("sm2_pa_m3", pc.Cfg(nof_prb=25, nof_ports=2, nof_rx=2, cfi=1, sf_idx=2, scheme=pc.SPATIALMUX,
                                    nof_layers=2, pmi=1, qm=[6, 6], tbs=[pc.valid_tbs(9000)] * 2, p_a=-3.0)))
    out.append(("port0_pa_m6", pc.Cfg(nof_prb=15, cfi=2, sf_idx=6, qm=[4], tbs=[pc.valid_tbs(3000)], p_a=-6.0)))
    out.append(("partial_alloc", pc.Cfg(nof_prb=50, cfi=2, sf_idx=4, qm=[6], tbs=[pc.valid_tbs(5000)], rv=[0, 0],
                                        prb=prb)))
    return out


def oracle_tx_grid(cfg: pc.Cfg, bits: list[np.ndarray]) -> np.ndarray:
    """Per-port grids of the oracle transmitter (the TX half of pc.synth_subframe)."""
    idx = oracle.pdsch_re_map(cfg.nof_prb, cfg.nof_ports, cfg.cell_id, cfg.prb_mask(), cfg.lstart, cfg.sf_idx)
    nre = idx.size
    d = []
    for t in range(cfg.nof_tb):
        qm, tbs = cfg.qm[t], cfg.tbs[t]
        Nl = 2 if cfg.nof_layers != cfg.nof_tb else 1
        G = nre * qm
        coded = oracle.dlsch_encode_tb(bits[t], tbs, qm * Nl, G, cfg.rv[t])
        c = oracle.sequence_lte(oracle.pdsch_c_init(cfg.rnti, t, cfg.sf_idx, cfg.cell_id), G)
        d.append(pc.modulate(coded ^ c, qm))
    tx = pc.precode(d, cfg, ref_scaling=True)
    g = np.zeros((cfg.nof_ports, cfg.grid_len), np.complex64)
    g[:, idx] = tx
    return g


def host_tx_grid(cfg: pc.Cfg, payloads: list[np.ndarray]) -> np.ndarray:
    cell = cell_of(cfg)
    pcfg = P.PdschCfg()
    pcfg.grant = grant_of(cfg)
    pcfg.rnti = cfg.rnti
    pcfg.p_a = cfg.p_a
    g = np.zeros((cfg.nof_ports, cfg.grid_len), np.complex64)
    enb_dl.pdsch_encode(cell, P.DlSfCfg(cfg.sf_idx, cfg.cfi), pcfg, payloads, g)
    return g


@pytest.mark.parametrize("name,cfg", tx_configs(), ids=[n for n, _ in tx_configs()])
def test_pdsch_encode_host_matches_oracle(name, cfg):
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    bits = [rng.integers(0, 2, t, dtype=np.uint8) for t in cfg.tbs]
    ref = oracle_tx_grid(cfg, bits)
    got = host_tx_grid(cfg, [np.packbits(b) for b in bits])
    assert np.array_equal(ref != 0, got != 0)
    np.testing.assert_allclose(got, ref, rtol=0, atol=5e-7)  # 1-2 float32 ulps of |x| <= 1.5


@pytest.mark.parametrize("nof_prb,nof_ports,cell_id,sf", [(6, 1, 1, 0), (25, 2, 7, 5), (100, 2, 1, 3),
                                                          (50, 4, 301, 9)])
def test_crs_host_matches_oracle(nof_prb, nof_ports, cell_id, sf):
    from oracle import ue_dl_chain as uc
    cell = P.make_cell(nof_prb, nof_ports, cell_id)
    G = 14 * 12 * nof_prb
    got = np.zeros((nof_ports, G), np.complex64)
    enb_dl.put_refs(cell, sf, got)
    ref = np.zeros((nof_ports, G), np.complex64)
    uc.crs_put(ref, nof_prb, cell_id, nof_ports, sf)
    assert np.array_equal(got, ref)
