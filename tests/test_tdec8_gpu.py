"""GPU parity of the 8-bit turbo decoder and 8-bit rate dematching against the reference's own
8-bit path (tests/golden/tdec8.npz, recorded from srslte_tdec_iteration_8bit -- AVX8 32-window and SSE8 16-window
decoders -- and srslte_rm_turbo_rx_lut_8bit of the srsLTE sources compiled here): decision bytes after every
half-iteration 1..8 bit-exact, including failing blocks and full-range int8 inputs; rate-dematched buffers
bit-exact incl. wrap-around (E > N) and HARQ accumulation."""
from __future__ import annotations

import numpy as np
import pytest

from srsran_amd.tdec import DeviceBuffer, Tdec8Batch
from tests.golden_io import load

pytestmark = pytest.mark.gpu


def cases():
    z = load("tdec8.npz")
    return z, int(z["ncases"])


def test_tdec8_matches_reference_goldens():
    z, n = cases()
    nh = int(z["nhalf"])
    dec = Tdec8Batch()
    byK: dict[int, list[int]] = {}
    for i in range(n):
        byK.setdefault(int(z[f"c{i}_K"]), []).append(i)
    for K, idx in byK.items():  # every K as one batch of its cases
        blen = 3 * (K + 32) + 12
        stride = (blen + 255) // 256 * 256
        host = np.zeros((len(idx), stride), np.int8)
        for r, i in enumerate(idx):
            host[r, :blen] = z[f"c{i}_buf"]
        d_in = DeviceBuffer(host.nbytes).upload(host)
        d_out = DeviceBuffer(len(idx) * (K // 8))
        d_tr = DeviceBuffer(len(idx) * nh * (K // 8))
        assert dec.run_dev(d_in.ptr, stride, len(idx), K, nh, d_out.ptr, K // 8, d_tr.ptr) == 0
        tr = d_tr.download(np.zeros((len(idx), nh, K // 8), np.uint8))
        out = d_out.download(np.zeros((len(idx), K // 8), np.uint8))
        for r, i in enumerate(idx):
            want = z[f"c{i}_trace"]
            for h in range(nh):
                assert np.array_equal(tr[r, h], want[h]), (K, str(z[f"c{i}_kind"]), float(z[f"c{i}_ebno"]), h)
            assert np.array_equal(out[r], want[nh - 1])


def test_tdec8_rejects_other_K():
    dec = Tdec8Batch()
    d = DeviceBuffer(3 * (512 + 32) + 12 + 256)
    o = DeviceBuffer(64)
    assert dec.run_dev(d.ptr, 3 * (512 + 32) + 12, 1, 512, 2, o.ptr, 64) != 0   # 16-bit fallback K
    assert dec.run_dev(d.ptr, 3 * (512 + 32) + 12, 1, 513, 2, o.ptr, 64) != 0   # not a code-block size


def test_rm_turbo_rx_8bit_matches_reference_goldens():
    z = load("tdec8.npz")
    dec = Tdec8Batch()
    for i in range(int(z["rm_n"])):
        K, rv, E = int(z[f"rm{i}_K"]), int(z[f"rm{i}_rv"]), int(z[f"rm{i}_E"])
        blen = 3 * (K + 32) + 12
        d_out = DeviceBuffer(blen).upload(np.zeros(blen, np.int8))
        d_e1 = DeviceBuffer(E).upload(z[f"rm{i}_e1"])
        d_e2 = DeviceBuffer(E).upload(z[f"rm{i}_e2"])
        assert dec.rm_rx_dev(d_e1.ptr, E, E, d_out.ptr, blen, 1, K, rv) == 0
        got1 = d_out.download(np.zeros(blen, np.int8))
        assert np.array_equal(got1, z[f"rm{i}_out1"]), (K, rv, E)
        assert dec.rm_rx_dev(d_e2.ptr, E, E, d_out.ptr, blen, 1, K, (rv + 2) % 4) == 0
        got2 = d_out.download(np.zeros(blen, np.int8))
        assert np.array_equal(got2, z[f"rm{i}_out2"]), (K, rv, E, "harq")
