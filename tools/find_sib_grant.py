#!/usr/bin/env python3
"""Search the reference's real-signal test vector for the PDSCH grants it carries (GPU).

lib/src/phy/phch/test/pdsch_pdcch_file_test.c decodes SI-RNTI transmissions from signal.1.92M.amar.dat
(CMakeLists.txt:440: cell id 1, 6 PRB, 1 port, CFI 3) after blind PDCCH decoding, which is out of this
framework's scope.  Instead every plausible DCI-1A grant is tried directly on the product path: each subframe
is demodulated and estimated once (mi355_ue_dl_decode_fft_estimate_batch), then one PDSCH job per (localized
allocation, redundancy version, TBS) is decoded in a batch and the transport-block CRC24A picks the right one
(a false pass has probability 2^-24 per try).  Hits are written to gpurun_out/sib_grants.json; the fixture
tests/golden/real_signal_sib.json (with the signal bytes of the hit subframes) is made from it by
tests/golden/make_golden.py (gen_real_signal).

Run: python tools/find_sib_grant.py tests/golden/signal_1.92M_amar.c64  (the reference test's data file, copied
verbatim: /root/reference does not exist on the GPU box).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from srsran_amd import pdsch as P  # noqa: E402
from srsran_amd.dlsch import SoftbufferPool  # noqa: E402
from srsran_amd.tdec import DeviceBuffer  # noqa: E402
from srsran_amd.ue_dl import DlSfJob, UeDl, default_chest_cfg, symbol_sz  # noqa: E402

NPRB, CELL_ID, CFI = 6, 1, 3
SI_RNTI = 0xFFFF


def main():
    path = sys.argv[1]
    iq = np.fromfile(path, np.complex64)
    N = symbol_sz(NPRB)
    sf_len = 15 * N
    nsf = iq.size // sf_len
    cell = P.make_cell(NPRB, 1, CELL_ID)
    ue = UeDl(cell, 1)
    G = 14 * 12 * NPRB
    d_iq = DeviceBuffer(iq.nbytes).upload(iq)
    d_grid = DeviceBuffer(nsf * G * 8)
    d_ce = DeviceBuffer(nsf * G * 8)
    sfjobs = []
    for s in range(nsf):
        j = DlSfJob()
        j.tti = s
        j.in_buffer[0] = d_iq.ptr + s * sf_len * 8
        j.sf_symbols[0] = d_grid.ptr + s * G * 8
        j.ce[0][0] = d_ce.ptr + s * G * 8
        sfjobs.append(j)
    chest = ue.fft_estimate(sfjobs, default_chest_cfg())
    allocs = [(s, L) for L in range(1, NPRB + 1) for s in range(NPRB - L + 1)]
    tbs_list = list(range(16, 2217, 8))
    hits = []
    for s in range(nsf):
        cands = [(a, rv, t) for a in allocs for rv in range(4) for t in tbs_list]
        pool = SoftbufferPool(len(cands), max_cb=1)
        pay = DeviceBuffer(len(cands) * 300)
        jobs = []
        for k, ((st, L), rv, t) in enumerate(cands):
            prb = np.zeros((2, NPRB), np.uint8)
            prb[:, st:st + L] = 1
            job = P.PdschJob()
            job.sf.tti, job.sf.cfi = s, CFI
            job.cfg.grant = P.make_grant(cell, prb, CFI, s, P.TXSCHEME_PORT0, 1,
                                         [dict(qm=2, tbs=t, rv=rv, cw_idx=0)])
            job.cfg.rnti = SI_RNTI
            job.cfg.decoder_type = P.MIMO_DECODER_MMSE
            job.cfg.softbuffer[0] = k
            job.noise_estimate = chest[s].noise_estimate
            job.sf_symbols[0] = d_grid.ptr + s * G * 8
            job.ce[0][0] = d_ce.ptr + s * G * 8
            job.payload[0] = pay.ptr + k * 300
            jobs.append(job)
        res = ue.pdsch.decode(pool, jobs)
        host = np.zeros(len(cands) * 300, np.uint8)
        pay.download(host)
        for k, c in enumerate(cands):
            if res[2 * k].crc:
                (st, L), rv, t = c
                hits.append({"sf": s, "prb_start": st, "nof_prb": L, "rv": rv, "tbs": t,
                             "payload_hex": host[k * 300: k * 300 + t // 8].tobytes().hex(),
                             "noise_estimate": float(chest[s].noise_estimate)})
                print("hit", hits[-1], flush=True)
        pool.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "sib_grants.json"), "w") as f:
        json.dump({"cell": {"nof_prb": NPRB, "id": CELL_ID, "ports": 1}, "cfi": CFI, "rnti": SI_RNTI,
                   "hits": hits}, f, indent=1)
    print(len(hits), "hits")


if __name__ == "__main__":
    main()
