#!/usr/bin/env python3
"""DL-SCH latency path (tdec_win_lat) vs the throughput path on one TM4 subframe's transport blocks (2 x TBS 97,896,
16 code blocks each): host time per call, and the latency kernel's phase counters (shader cycles per code block and
half-iteration, rerun rounds).  python3 tools/lat_probe.py"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from srsran_amd import lib  # noqa: E402
from srsran_amd.dlsch import Dlsch, SoftbufferPool  # noqa: E402

NAMES = ["load", "first_halves", "second_halves", "decisions", "check", "simd_alpha", "simd_beta", "same_simd", "owave_shares_simd", "half_its", "cbs"]
rng = np.random.default_rng(1)
QUICK = os.environ.get("LAT_PROBE_QUICK") == "1"  # the 30 dB latency case only
if os.environ.get("LAT_PROBE_SWEEP") == "1":  # crossover: host time per call of both paths vs transport blocks per call
    for snr in (30.0, 9.0):
        base = [oracle.make_tb(rng, 97896, 8, 115200, 0, snr)[1] for _ in range(2)]
        for ntb in (1, 2, 4, 8, 12, 16, 24):
            llrs = [base[i % 2] for i in range(ntb)]
            tbs = [dict(tbs=97896, Qm=8, rv=0, softbuffer=i) for i in range(ntb)]
            res = {"snr": snr, "tbs": ntb, "cbs": 16 * ntb}
            for path in ("throughput", "latency"):
                lib().mi355_dlsch_set_latency_path(100000 if path == "latency" else 0)
                dl = Dlsch(0, 10)
                pool = SoftbufferPool(ntb, 32)
                pool.reset_all()
                dl.decode(pool, tbs, llrs)
                n = 10
                t0 = time.perf_counter()
                for _ in range(n):
                    pool.reset_all()  # (a decoded softbuffer is skipped by the next call)
                    got = dl.decode(pool, tbs, llrs)
                res[path + "_us"] = round((time.perf_counter() - t0) / n * 1e6, 1)
                res[path + "_ok"] = sum(1 for r in got[0] if r == 0)
            print(json.dumps(res), flush=True)
    sys.exit(0)
for snr in ((30.0,) if QUICK else (9.0, 5.5, 30.0)):
    cases = [(97896, 8, 115200, snr)] * 2
    llrs = [oracle.make_tb(rng, t, q, g, 0, s)[1] for (t, q, g, s) in cases]
    for path in (("latency",) if QUICK else ("throughput", "latency")):
        lib().mi355_dlsch_set_latency_path(512 if path == "latency" else 0)
        dl = Dlsch(0, 10)
        pool = SoftbufferPool(2, 32)
        tbs = [dict(tbs=t, Qm=q, rv=0, softbuffer=i) for i, (t, q, g, s) in enumerate(cases)]
        got = dl.decode(pool, tbs, llrs)
        lib().mi355_dlsch_latency_profile(1, None)
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            pool.reset_all() if hasattr(pool, "reset_all") else None
            got = dl.decode(pool, tbs, llrs)
        dt = (time.perf_counter() - t0) / n
        out = (C.c_uint64 * 11)()
        lib().mi355_dlsch_latency_profile(0, C.addressof(out))
        v = list(out)
        res = {"snr": snr, "path": path, "us_per_call": round(dt * 1e6, 1), "rets": list(got[0]),
               "its": [round(float(x), 2) for x in got[2]]}
        if path == "latency" and v[10]:
            cb, hi = v[10], max(v[9], 1)
            res["per_cb_half_it_kcycles"] = {NAMES[k]: round(v[k] / hi / 1e3, 2) for k in (1, 2, 3, 4)}
            res["load_kcycles_per_cb"] = round(v[0] / cb / 1e3, 2)
            res["half_its_per_cb"] = round(hi / cb, 2)
            res["simd"] = {NAMES[k]: round(v[k] / cb - (k < 7), 2) for k in (5, 6, 7, 8)}
        print(json.dumps(res), flush=True)
        dl.close() if hasattr(dl, "close") else None
