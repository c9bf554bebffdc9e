import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import bench, oracle
from srsran_amd.tdec import DeviceBuffer, TdecBatch
from tests.golden_io import tdec_auto_cases
K = 6144
stride = bench.tdec_stride(K)
pool = [bench.make_cb_pool(K, 8, 6.0, 11), bench.make_cb_pool(K, 8, 4.0, 12)]
for c in [c for c in tdec_auto_cases() if c["K"] == K]:
    row = np.zeros((1, stride), np.int16); row[0, : c["buf"].size] = c["buf"]; pool.append(row)
pool = np.ascontiguousarray(np.concatenate(pool)); n = pool.shape[0]
dec = TdecBatch(0)
d_in = DeviceBuffer(pool.nbytes).upload(pool); d_out = DeviceBuffer(n * 768)
dec.run_dev(d_in.ptr, stride, n, K, 8, d_out.ptr)
got = d_out.download(np.zeros((n, 768), np.uint8))
print("ref available", oracle.ref_available())
w1 = np.zeros((n, 768), np.uint8); oracle.lib().orc_tdec_run_batch(pool, stride, n, K, 8, w1, 1)
print("oracle rows equal", [bool(np.array_equal(got[i], w1[i])) for i in range(n)])
if oracle.ref_available():
    for nt in (1, 8):
        w2 = np.zeros((n, 768), np.uint8); oracle.ref().ref_tdec_run_batch(pool, stride, n, K, 8, w2, nt)
        print("ref", nt, [bool(np.array_equal(got[i], w2[i])) for i in range(n)])
h = dec.run(pool, K, 8)
print("host-run rows equal", [bool(np.array_equal(got[i], h[i])) for i in range(n)])
