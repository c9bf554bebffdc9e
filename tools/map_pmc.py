#!/usr/bin/env python3
"""The MAP kernel's launches of one bench roofline probe, alone, for rocprofv3 --pmc passes (tools/gpu/map_pmc.sh):
    python3 tools/map_pmc.py e2e | siso | tdec
e2e: the default workload's probe (bench.map_probe): the rate-dematched TM4 softbuffers of one 2,048-subframe step
(65,536 CBs of K = 6144, parity-row bitmaps), 8 half-iterations without early stop; siso: the same for configs[2]
(8,192 subframes x 3 CBs of K = 5312); tdec: configs[1]'s synthetic 65,536-CB batch (full parity), 8 half-iterations.
One warm run, then three measured runs (24 launches) -- tools/map_pmc_summary.py averages the last 16."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from srsran_amd import lib  # noqa: E402
from srsran_amd.tdec import DeviceBuffer, TdecBatch  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "e2e"
if mode == "e2e":
    cell = bench.tm4_setup()
    B, K = 2048, 6144
    src = bench.Tm4Source(cell, B, 0)
    src.generate(0, B, 40.0, 4242)
    rx = bench.Tm4Rx(cell, B, 0)
    rx.step(rx.bind(src, 0, B))
    ncb = 32 * B
    ptr, stride = bench.softbuffer_contents(rx, ncb)
elif mode == "siso":
    from srsran_amd import synth
    cell, nrx = synth.phy_dl_test_cell(100, 0)
    B, K = 8192, bench.SISO_K
    plans = synth.phy_dl_test_plans(cell, 0, 9, False, nof_subframes=B, first=0)
    src = synth.DlSource(cell, nrx, B, bench.SISO_TBS // 8, 0)
    src.generate(0, plans, None, 4242, ctrl=True)
    rx = synth.DlReceiver(cell, nrx, B, bench.SISO_TBS // 8, 0, ctrl=True, max_cb=bench.SISO_C, ce_rows=1)
    rx.step(rx.bind(src, 0, B, tb_major=True))
    ncb = bench.SISO_C * B
    ptr, stride = bench.softbuffer_contents(rx, ncb)
else:
    K, ncb = 6144, 65536
    stride = bench.tdec_stride(K)
    pool = bench.make_cb_pool(K, 256, 6.0, seed=bench.shard_seed(0))
    host = np.ascontiguousarray(np.tile(pool, (ncb // 256 + 1, 1))[:ncb])
    d_in = DeviceBuffer(host.nbytes, 0).upload(host)
    del host
    ptr = d_in.ptr
lib().mi355_device_sync()
d_out = DeviceBuffer(ncb * (K // 8), 0)
dec = TdecBatch(0)
for _ in range(4):
    dec.run_dev(ptr, stride, ncb, K, 8, d_out.ptr)
    lib().mi355_device_sync()
print(f"map_pmc {mode}: {ncb} CBs of K={K}, 4 x 8 half-iterations", flush=True)
