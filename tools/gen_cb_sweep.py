#!/usr/bin/env python3
"""Per-code-block generic decoder (tdec_gen_cb.hip): time and chunk reruns vs the guess warm-up, for one K = 6144 block
(latency, device buffers) and 16,384 blocks (throughput), at several Eb/N0; every output checked against the oracle.
    python3 tools/gen_cb_sweep.py > gpurun_out/.../gen_cb_sweep.json"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from srsran_amd import lib  # noqa: E402
from srsran_amd.tdec import DeviceBuffer, TdecBatch  # noqa: E402

K, NH = 6144, 8
stride = (3 * K + 12 + 7) // 8 * 8
rng = np.random.default_rng(3)
res = []
for eb in (0.5, 1.0, 2.0, 4.0):
    lin = oracle.make_cb(rng, K, eb)[1]
    want = oracle.tdec_run_generic(lin, K, NH)
    for n in (1, 16384):
        host = np.zeros((n, stride), np.int16)
        host[:, : lin.size] = lin
        d_in = DeviceBuffer(host.nbytes, 0).upload(host)
        d_out = DeviceBuffer(n * (K // 8), 0)
        for W in (16, 32, 48, 64):
            tb = TdecBatch(0)
            tb.set_impl(1)
            tb.set_generic(1, W)
            tb.run_dev(d_in.ptr, stride, n, K, NH, d_out.ptr)
            lib().mi355_device_sync()
            tb.generic_reruns()
            reps = 20 if n == 1 else 3
            t0 = time.perf_counter()
            for _ in range(reps):
                tb.run_dev(d_in.ptr, stride, n, K, NH, d_out.ptr)
            lib().mi355_device_sync()
            dt = (time.perf_counter() - t0) / reps
            rr = tb.generic_reruns() / reps / n
            out = d_out.download(np.zeros((n, K // 8), np.uint8))
            ok = bool((out == want[None, :]).all())
            res.append({"ebno": eb, "n": n, "warm": W, "us_per_call": round(dt * 1e6, 1),
                        "cb_per_s": round(n / dt, 1), "reruns_per_cb": round(rr, 1), "exact": ok})
            print(json.dumps(res[-1]), flush=True)
            tb.close()
        d_in.free()
        d_out.free()
