"""The reference's own end-to-end test matrix on the GPU: lib/test/phy/CMakeLists.txt:33-58 runs phy_dl_test over
6/15/25/50/75/100 PRB x 64QAM/256QAM tables x TM1-4 x MCS 0/7/14/21/28 (27, or 26 at 15 PRB, with 256QAM):
240 cases, each over one frame's worth of UE-specific PDCCH locations (phy_dl_test.c:412-429), every TB required to
decode with its payload (BLER 0, :600-633).

Here every case's subframes come from the product's GPU eNodeB generator (srsran_amd.synth.phy_dl_test_plans:
the test's DCI formats, type-0 allocation of every RBG, the DCI at location (sf / 10) % nof_locations, its MCS
rules for 6 / 15 PRB, p_a 0 dB / p_b 1 and no noise, the crossed 2x2 channel for TM2-4), and the UE side is ONE
mi355_ue_dl_find_and_decode_batch per (PRB, port count) over all of its cases' subframes (up to 4,800): OFDM,
estimation, PCFICH / PDCCH blind search, DCI -> grant (tm, 256QAM table per subframe), PDSCH, DL-SCH.

Pass criterion, per TB, as phy_dl_test: exactly one DCI found, CRC ok, payload equal.  Soft bits: on two subframes
of every case, the GPU's LLRs equal the oracle chain's (rx_front on the GPU's own grid / estimates / noise) bit for
bit and their signs equal the transmitted codeword (check_softbits, phy_dl_test.c:257-292)."""
import numpy as np
import pytest

from srsran_amd import synth
from tests.pdsch_jobs import llr_spot_check, oracle_cfg

pytestmark = pytest.mark.gpu

CROSSED = [[1, 1], [1, -1]]  # phy_dl_test.c:549-563


def _group(nof_prb: int, tms: tuple):
    cases = [c for c in synth.phy_dl_test_matrix() if c[0] == nof_prb and c[2] in tms]
    cell, nrx = synth.phy_dl_test_cell(nof_prb, tms[0] - 1)
    plans, case_of, first_of = [], [], []
    for prb, a256, tm, mcs in cases:
        p = synth.phy_dl_test_plans(cell, tm - 1, mcs, a256)
        first_of.append(len(plans))
        plans += p
        case_of += [(prb, a256, tm, mcs)] * len(p)
    return cell, nrx, cases, plans, case_of, first_of


@pytest.mark.parametrize("nof_prb", [6, 15, 25, 50, 75, 100])
@pytest.mark.parametrize("tms", [(1,), (2, 3, 4)], ids=["tm1", "tm2-4"])
def test_phy_dl_test_matrix(nof_prb, tms):
    cell, nrx, cases, plans, case_of, first_of = _group(nof_prb, tms)
    n = len(plans)
    nbytes = max(max(synth.tb_bytes(p.cfg)) for p in plans)
    src = synth.DlSource(cell, nrx, n, nbytes, H=[[1]] if nrx == 1 else CROSSED)
    src.generate(0, plans, None, seed=1000 + nof_prb, ctrl=True)
    rx = synth.DlReceiver(cell, nrx, n, nbytes, ctrl=True, max_cb=16)
    rx.ue.set_chunks(1)  # the LLR spot checks read the single chunk's soft bits
    bound = rx.bind(src, 0, n)
    rx.step(bound)
    ctrl = np.ctypeslib.as_array(rx.ctrl_res)[:n]
    res = np.ctypeslib.as_array(rx.res)[: 2 * n].reshape(n, 2)
    got, want = rx.received(n), src.payloads(0, n)
    failures, count_tbs = [], 0
    for k, pl in enumerate(plans):
        nb = synth.tb_bytes(pl.cfg)
        for t in range(2):
            if not nb[t]:
                continue
            count_tbs += 1
            if ctrl[k]["nof_dci"] != 1 or not res[k, t]["crc"] or res[k, t]["ret"] != 0 or \
                    not np.array_equal(got[k, t, : nb[t]], want[k, t, : nb[t]]):
                failures.append((case_of[k], k, t, int(ctrl[k]["nof_dci"]), int(res[k, t]["crc"])))
    assert not failures, (len(failures), count_tbs, failures[:8])
    assert count_tbs == sum(2 if p.tm >= 2 else 1 for p in plans)
    # soft bits of two subframes per case (the first of the case and one in subframe 5 or after)
    for ci, case in enumerate(cases):
        k0 = first_of[ci]
        for k in (k0, k0 + 5):
            pl = plans[k]
            ocfg = oracle_cfg(cell, nrx, pl.tti, pl.cfi, pl.cfg)
            llr_spot_check(rx, k, ocfg, [want[k, t, : ocfg.tbs[t] // 8] for t in range(ocfg.nof_tb)])
    rx.close()
    src.close()
