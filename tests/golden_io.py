"""Readers for the committed golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py
from the srsLTE reference compiled from its own sources)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def tdec_auto_cases():
    z = load("tdec_auto.npz")
    out = []
    for i in range(int(z["ncases"])):
        out.append(dict(K=int(z[f"c{i}_K"]), kind=str(z[f"c{i}_kind"]), ebno=float(z[f"c{i}_ebno"]),
                        bits=z[f"c{i}_bits"], buf=z[f"c{i}_buf"], trace=z[f"c{i}_trace"]))
    return out


def tdec_generic_cases():
    z = load("tdec_generic.npz")
    return [dict(K=int(z[f"c{i}_K"]), lin=z[f"c{i}_lin"], bits=z[f"c{i}_bits"], trace=z[f"c{i}_trace"])
            for i in range(int(z["ncases"]))]


def rm_init_softbuffer():
    """Deterministic non-zero softbuffer content used when the rm_turbo goldens were made."""
    i = np.arange(18600, dtype=np.int64)
    return ((i * 7919) % 60001 - 30000).astype(np.int16)


def rm_cases():
    z = load("rm_turbo.npz")
    return [dict(K=int(z[f"c{i}_K"]), rv=int(z[f"c{i}_rv"]), e=z[f"c{i}_e"], out=z[f"c{i}_out"])
            for i in range(int(z["ncases"]))]


def rm_harq():
    z = load("rm_turbo.npz")
    return dict(K=int(z["harq_K"]), e0=z["harq_e0"], e2=z["harq_e2"], out=z["harq_out"])
