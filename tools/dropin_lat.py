#!/usr/bin/env python3
"""The drop-in's per-TTI latency loop alone (bench.dropin_tti_latency), for kernel / copy traces:
    python3 tools/dropin_lat.py [ntti]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

args = bench.parse(["--snr", "40"])
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
print(json.dumps(bench.dropin_tti_latency(args, bench.tm4_setup(), 0, ntti=n, nwarm=20)))
