"""Second reference-held known answer: lib/src/phy/phch/test/signal.10M.dat (copied verbatim as
tests/golden/signal_10M.c64), the recording pcfich_file_test decodes (phch/test/CMakeLists.txt:437:
-c 150 -n 50 -p 2, i.e. cell 150, 50 PRB, 2 ports, PHICH normal / R1 as pcfich_file_test.c:33-38 sets them).
Its pass criterion (pcfich_file_test.c:247-256): CFI 2 with a correlation above 2.8, after srslte_ofdm_rx_sf and
srslte_chest_dl_estimate with a zeroed srslte_chest_dl_cfg_t (Gauss filter with the automatic sigma, AVERAGE,
REFS noise) on subframe 0.  This pins the OFDM demodulator, the 2-port CRS estimator at 50 PRB and the PCFICH --
on the CPU oracle chain and on the GPU product.

The file holds 7,681 samples, fewer than the 11,520 of a 50-PRB subframe (symbol size 768): the test reads
them into a malloc'd buffer whose tail it never writes; the tail is taken as zeros here (a fresh heap block)."""
import os

import numpy as np
import pytest

from oracle import pdcch_chain as pd
from oracle import ue_dl_chain as uc

HERE = os.path.dirname(os.path.abspath(__file__))
NPRB, CELL, PORTS = 50, 150, 2
SF_LEN = 15 * uc.symbol_sz(NPRB)


def _iq():
    raw = np.fromfile(os.path.join(HERE, "golden", "signal_10M.c64"), np.complex64)
    iq = np.zeros(SF_LEN, np.complex64)
    iq[:raw.size] = raw
    return raw.size, iq


def test_fixture_shape():
    n, _ = _iq()
    assert n == 7681 and SF_LEN == 11520


def test_oracle_pcfich_known_answer():
    _, iq = _iq()
    grid = uc.ofdm_rx_sf(iq, NPRB)[None, :]
    ce, res = uc.chest_estimate(grid, NPRB, PORTS, CELL, 0, filter_type=0, coef=(0.0, 0.0))
    rg = pd.regs(NPRB, PORTS, CELL, 2)
    cfi, corr, _ = pd.pcfich_decode(grid, ce, rg, CELL, 0, res["noise_estimate"])
    assert cfi == 2 and corr.max() > 2.8, (cfi, corr)


@pytest.mark.gpu
def test_product_pcfich_known_answer():
    from srsran_amd import lib
    from srsran_amd import pdcch as D
    from srsran_amd import pdsch as P
    from srsran_amd.tdec import DeviceBuffer
    from srsran_amd.ue_dl import ChestCfg, DlSfJob, UeDl

    _, iq = _iq()
    ue = UeDl(P.make_cell(NPRB, PORTS, CELL, phich_resources=2), 1)
    G = 14 * 12 * NPRB
    d_iq, d_grid = DeviceBuffer(iq.nbytes), DeviceBuffer(G * 8)
    d_ce = [DeviceBuffer(G * 8) for _ in range(PORTS)]
    lib().mi355_memcpy_h2d(d_iq.ptr, iq.ctypes.data, iq.nbytes)
    j = DlSfJob()
    j.tti = 0
    j.in_buffer[0], j.sf_symbols[0] = d_iq.ptr, d_grid.ptr
    for p in range(PORTS):
        j.ce[p][0] = d_ce[p].ptr
    chest = ue.fft_estimate([j], ChestCfg())  # srslte_chest_dl_estimate: zeroed configuration
    cfis, ctrl, _dci = D.find_dl_dci(ue, [j], [0xFFFF], [D.UeDlCfg()], chest)
    assert cfis[0] == 2 and ctrl[0].cfi == 2 and ctrl[0].cfi_corr > 2.8, (cfis[0], ctrl[0].cfi_corr)
    # the same correlation as the oracle chain on the same samples
    grid = uc.ofdm_rx_sf(iq, NPRB)[None, :]
    ce, res = uc.chest_estimate(grid, NPRB, PORTS, CELL, 0, filter_type=0, coef=(0.0, 0.0))
    _cfi, corr, _ = pd.pcfich_decode(grid, ce, pd.regs(NPRB, PORTS, CELL, 2), CELL, 0, res["noise_estimate"])
    assert abs(ctrl[0].cfi_corr - corr.max()) <= 1e-3 * corr.max()
    assert abs(chest[0].noise_estimate - res["noise_estimate"]) <= 1e-3 * res["noise_estimate"]
    ue.close()
