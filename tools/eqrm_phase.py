"""pdsch_eq_rm phase profile (run on the GPU box): per-workgroup shader cycles of the prologue (descriptors, flags,
parity-row bitmaps), the equaliser (RE pairs -> LLR images in LDS) and the rate dematching (table walk -> softbuffers),
averaged over the bench's default batch (2,048 TM4 subframes, 3 decodes):  python3 tools/eqrm_phase.py [subframes]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from srsran_amd import lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
cell = bench.tm4_setup()
src = bench.Tm4Source(cell, B, 0, False)
src.generate(0, B, 40.0, 4242)
rx = bench.Tm4Rx(cell, B, 0, False)
b = rx.bind(src, 0, B)
for _ in range(2):
    rx.step(b)
L = lib()
L.mi355_pdsch_eqrm_profile.argtypes = [C.c_int, C.c_void_p]
assert L.mi355_pdsch_eqrm_profile(1, None) == 0
for _ in range(3):
    rx.step(b)
out = (C.c_uint64 * 4)()
assert L.mi355_pdsch_eqrm_profile(0, out) == 0
wg = max(1, out[0])
res = {"subframes": B, "workgroups": int(out[0]), "avg_cycles": {"prologue": out[1] / wg, "equaliser": out[2] / wg,
                                                               "rate_dematching": out[3] / wg}}
print(json.dumps(res))
