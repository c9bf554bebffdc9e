#!/usr/bin/env python3
"""SNR sweep of the bench's decoder-bound e2e field (EPA 5 Hz fading, TM4 QAM256): mean half-iterations and CRC-ok
TBs per SNR on 512 subframes, to choose bench.py --waterfall-snr.  GPU box: python3 tools/waterfall_sweep.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    from srsran_amd import lib
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    snrs = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [22, 24, 26, 28, 30, 32, 35]
    cell = bench.tm4_setup()
    src = bench.Tm4Source(cell, B, 0)
    rx = bench.Tm4Rx(cell, B, 0)
    for snr in snrs:
        src.generate(10_000_000, B, snr, 4243, fading="epa5")
        b = rx.bind(src, 0, B)
        rx.step(b)
        lib().mi355_device_sync()
        t0 = time.perf_counter()
        rx.step(b)
        lib().mi355_device_sync()
        dt = time.perf_counter() - t0
        print(json.dumps({"snr": snr, "avg_half_its": round(rx.avg_its(B), 3), "crc_ok": int(rx.crc_bits(B).sum()),
                          "tbs": 2 * B, "ms": round(dt * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
