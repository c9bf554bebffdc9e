"""GPU tests of pdsch_eq_rm (pdsch_kernels.hip: equaliser, LLRs and rate dematching in one kernel, used when every job
of a batch qualifies) against the two-kernel path (pdsch_eq_llr + dlsch_rm_rx, forced by MI355_NO_EQRM), whose
parity with the oracle test_pdsch_gpu / test_dlsch_gpu / the LLR spot checks hold: a HARQ retransmission combined
into old (not fresh) softbuffers, where pdsch_eq_rm takes its read-modify-write path, must leave the same decoder
buffers and give the same CRC results."""
import ctypes as C

import numpy as np
import pytest

import bench

pytestmark = pytest.mark.gpu


def _two_transmissions(monkeypatch, eqrm: bool, B=6, snr=8.0):
    from srsran_amd import check, lib
    if eqrm:
        monkeypatch.delenv("MI355_NO_EQRM", raising=False)
    else:
        monkeypatch.setenv("MI355_NO_EQRM", "1")
    cell = bench.tm4_setup()
    src = bench.Tm4Source(cell, B, 0)
    src.generate(0, B, snr, 77)  # low SNR: most 256QAM code blocks fail the first time
    rx = bench.Tm4Rx(cell, B, 0)
    bound = rx.bind(src, 0, B)
    rx.step(bound)  # rv 0 into fresh softbuffers (reset first)
    crc1 = rx.crc_bits(B).copy()
    # the retransmission as rv 2 (the same I/Q: the combining arithmetic is what is under test), no reset: the TBs
    # that passed are skipped (res), the others' code blocks not decoded yet are read-modified
    jobs, sfs, cfgs, n, _ = bound
    for k in range(n):
        for t in range(2):
            cfgs[k].grant.tb[t].rv = 2
    check(rx.L.mi355_ue_dl_decode_batch(rx.ue.h, rx.pool.h, jobs, sfs, cfgs, C.byref(rx.chest_cfg), rx.chest,
                                        rx.pays, n, rx.res, None), "ue_dl_decode_batch")
    crc2 = rx.crc_bits(B).copy()
    ptr, stride = bench.softbuffer_contents(rx, 0)
    buflen = 3 * (6144 + 32) + 12
    sb = np.zeros((2 * B * 16, stride), np.int16)  # Tm4Rx: max_cb 16, softbuffers 2k, 2k + 1
    lib().mi355_memcpy_d2h(sb.ctypes.data, ptr, sb.nbytes)
    rx.close()
    src.close()
    return crc1, crc2, sb[:, :buflen]


def test_harq_combining_matches_two_kernel_path(monkeypatch):
    on = _two_transmissions(monkeypatch, True)
    off = _two_transmissions(monkeypatch, False)
    assert np.array_equal(on[0], off[0]) and np.array_equal(on[1], off[1])
    assert on[0].sum() < on[0].size  # some TBs failed the first transmission: the second combined into old buffers
    assert np.array_equal(on[2], off[2])
