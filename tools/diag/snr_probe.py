"""TM4 find_and_decode / decode_batch CRC counts vs SNR (diagnostic)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import bench
cell = bench.tm4_setup()
B = 40
for ctrl in (False, True):
    src = bench.Tm4Source(cell, B, 0, ctrl=ctrl)
    rx = bench.Tm4Rx(cell, B, 0, ctrl=ctrl)
    for snr in (40, 32, 28, 26, 24):
        src.generate(500, B, snr, 77)
        b = rx.bind(src, 0, B)
        rx.step(b)
        r = np.ctypeslib.as_array(rx.res)[: 2 * B]
        print("ctrl", ctrl, "snr", snr, "crc", int(r["crc"].sum()), "its", float(r["avg_iterations_block"].mean()),
              "noise", rx.chest[0].noise_estimate, flush=True)
