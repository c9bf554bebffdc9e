"""find_and_decode's pipelined chunks (mi355_ue_dl_find_and_decode_batch, ue_dl_runtime.cpp): a batch split into 1,
2 or 3 chunks -- chunk c's PDSCH/DL-SCH left in flight while the host replays chunk c+1's blind search -- must give
exactly the results of one chunk: every TB's CRC flag, return code, average iteration count and payload bytes.

The batch mixes max_nof_iterations per subframe (srslte_sch_set_max_noi persists, pdsch.c:930-932), so a chunk's
DL-SCH decode runs as several iteration-count groups sharing the descriptor scratch while earlier groups are still
queued; and in the multi-chunk runs subframe k and k + B/2 share their softbuffers (every TB is reset before its
decode, ue_dl.c:1522-1529), so chunk c+1's softbuffer resets must land after chunk c's decodes."""
import numpy as np
import pytest

import bench
from srsran_amd import lib

pytestmark = pytest.mark.gpu

B = 40
ITS = [10, 1, 3, 0, 2, 10, 4, 0, 1]  # per subframe, cyclic; 0 keeps the previous setting


def _run(src, rx, chunks: int, shared: bool):
    bound = rx.bind(src, 0, B)
    _jobs, _sfs, cfgs, n, _ = bound
    for k in range(B):
        sb = k % (B // 2) if shared else k
        cfgs[k].softbuffer[0], cfgs[k].softbuffer[1] = 2 * sb, 2 * sb + 1
        cfgs[k].max_nof_iterations = ITS[k % len(ITS)]
    rx.ue.set_chunks(chunks)
    lib().mi355_memset_dev(rx.d_pay.ptr, 0, B * 2 * rx.plen)
    rx.step(bound)
    res = np.ctypeslib.as_array(rx.res)[: 2 * B].copy()
    ctrl = np.ctypeslib.as_array(rx.ctrl_res)[:B].copy()
    return res, ctrl, rx.received(B)


def test_chunking_does_not_change_results():
    cell = bench.tm4_setup()
    src = bench.Tm4Source(cell, B, 0, ctrl=True)
    # 26 dB on the crossed channel: the decoder needs a varying number of half-iterations, so the per-subframe
    # iteration caps change outcomes
    src.generate(500, B, 26.0, 77)
    rx = bench.Tm4Rx(cell, B, 0, ctrl=True)
    base = _run(src, rx, 1, shared=False)
    r0, c0, p0 = base
    assert (c0["nof_dci"] == 1).all()
    assert r0["crc"].sum() >= B // 2, r0["crc"].sum()  # many TBs decode ...
    assert r0["crc"].sum() < 2 * B  # ... and the 1-iteration caps make some fail
    assert len(set(np.round(r0["avg_iterations_block"], 3))) > 2
    for chunks, shared in ((2, False), (2, True), (3, True), (1, False)):
        r, c, p = _run(src, rx, chunks, shared)
        assert np.array_equal(c["nof_dci"], c0["nof_dci"]) and np.array_equal(c["cfi"], c0["cfi"]), chunks
        for f in ("crc", "ret", "avg_iterations_block"):
            assert np.array_equal(r[f], r0[f]), (chunks, shared, f)
        ok = r0["crc"].reshape(B, 2) != 0
        assert np.array_equal(p[ok], p0[ok]), (chunks, shared)
    want = src.payloads(0, B)
    got = p0[:, :, : bench.NB]
    assert all(np.array_equal(got[k, t], want[k, t]) for k in range(B) for t in range(2) if ok[k, t])
    rx.close()
    src.close()
