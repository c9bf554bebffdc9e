"""BASELINE.json's configurations at their stated sizes, through the product's C ABI:

* configs[1] -- 65,536 x K=6144 code blocks, 8 half-iterations, one mi355_tdec_batch_run_dev launch set: the batch
  tiles a pool of distinct code blocks (Eb/N0 6.0 and 4.0, plus the reference's K=6144 golden inputs); every copy
  of a pool block must decode to the same bits (no cross-block interference at full occupancy), the pool's
  decisions equal the oracle / reference decoder and the golden traces bit for bit;
* configs[2] -- phy_dl_test -p 100 -t 1 -m 9 (20 MHz SISO QPSK, TBS 15,840): 1,000 subframes through
  mi355_ue_dl_find_and_decode_batch, every TB decoded with its payload, LLRs of a sample equal to the oracle chain;
* configs[3] -- one 2,048-subframe TM4 2x2 QAM256 batch through mi355_ue_dl_decode_batch (the bench step): every
  TB decoded with its payload, LLRs of a sample equal to the oracle chain;
* configs[4]'s code path -- bench.run_pdsch with --total-subframes at N = 1 over two resident sets (shard
  regeneration by global index, batch loop, CRC-bitmap bookkeeping)."""
import numpy as np
import pytest

import bench
import oracle
from srsran_amd import lib, synth
from tests.golden_io import tdec_auto_cases
from tests.pdsch_jobs import llr_spot_check, oracle_cfg

pytestmark = pytest.mark.gpu


def test_config1_batched_turbo_65536():
    from srsran_amd.tdec import DeviceBuffer, TdecBatch
    K, ncb, nh = 6144, 65536, 8
    stride = bench.tdec_stride(K)
    pool = [bench.make_cb_pool(K, 40, 6.0, 11), bench.make_cb_pool(K, 40, 4.0, 12)]
    gold = [c for c in tdec_auto_cases() if c["K"] == K]
    assert gold
    for c in gold:
        row = np.zeros((1, stride), np.int16)
        row[0, : c["buf"].size] = c["buf"]
        pool.append(row)
    pool = np.ascontiguousarray(np.concatenate(pool))
    npool = pool.shape[0]
    tile_rows = npool * (4096 // npool)
    tile = np.ascontiguousarray(np.tile(pool, (tile_rows // npool, 1)))
    d_in = DeviceBuffer(ncb * stride * 2)
    for r0 in range(0, ncb, tile_rows):
        m = min(tile_rows, ncb - r0)
        lib().mi355_memcpy_h2d(d_in.ptr + r0 * stride * 2, tile.ctypes.data, m * stride * 2)
    d_out = DeviceBuffer(ncb * (K // 8))
    dec = TdecBatch(0)
    dec.run_dev(d_in.ptr, stride, ncb, K, nh, d_out.ptr)  # asynchronous on the decoder's stream
    lib().mi355_device_sync()
    got = d_out.download(np.zeros((ncb, K // 8), np.uint8))
    dec.close()
    # every copy of a pool block decodes identically
    first = got[:npool]
    for r0 in range(0, ncb, npool):
        m = min(npool, ncb - r0)
        assert np.array_equal(got[r0:r0 + m], first[:m]), r0
    # the pool's decisions: oracle (or the reference decoder where oracle/_ref is built) and the golden traces
    want = np.zeros((npool, K // 8), np.uint8)
    if oracle.ref_available():
        oracle.ref().ref_tdec_run_batch(pool, stride, npool, K, nh, want, 8)
    else:
        oracle.lib().orc_tdec_run_batch(pool, stride, npool, K, nh, want, 8)
    assert np.array_equal(first, want)
    for i, c in enumerate(gold):
        assert np.array_equal(first[80 + i], c["trace"][-1]), i
    # Eb/N0 4.0 leaves some blocks undecoded after 8 half-iterations (configs[1] "13 % fail") -- the bits checked
    # are then the decoder's, not the payload's; Eb/N0 6.0 decodes: nothing more to assert here


def test_config2_siso_qpsk_1000_subframes():
    cell, nrx = synth.phy_dl_test_cell(100, 0)
    plans = synth.phy_dl_test_plans(cell, 0, 9, False, nof_subframes=1000)
    assert {p.cfg.grant.tb[0].tbs for p in plans} == {15840}
    n, nb = len(plans), 15840 // 8
    src = synth.DlSource(cell, nrx, n, nb)
    src.generate(0, plans, None, seed=9, ctrl=True)
    rx = synth.DlReceiver(cell, nrx, n, nb, ctrl=True, max_cb=4)
    rx.ue.set_chunks(1)
    bound = rx.bind(src, 0, n)
    rx.step(bound)
    assert rx.payload_ok(src, bound) == n
    want = src.payloads(0, n)
    for k in (0, 1, 5, 499, 999):
        pl = plans[k]
        llr_spot_check(rx, k, oracle_cfg(cell, nrx, pl.tti, pl.cfi, pl.cfg), [want[k, 0, :nb]])
    rx.close()
    src.close()


def test_config3_tm4_2048_subframe_batch():
    cell = bench.tm4_setup()
    B = 2048
    src = bench.Tm4Source(cell, B, 0)
    src.generate(0, B, 40.0, 4242)
    rx = bench.Tm4Rx(cell, B, 0)
    bound = rx.bind(src, 0, B)
    rx.step(bound)
    assert rx.payload_ok(src, bound) == 2 * B
    want = src.payloads(0, B)
    for k in (0, 3, 1024, 2047):
        pl = src.plans[k]
        cfg = bound[2][k]
        llr_spot_check(rx, k, oracle_cfg(cell, 2, pl.tti, pl.cfi, cfg), [want[k, t] for t in range(2)])
    rx.close()
    src.close()


def test_config4_total_subframes_two_resident_sets():
    args = bench.parse(["--total-subframes", "600", "--subframes", "256", "--resident-gb", "0.1", "--no-cpu",
                        "--snr", "40"])
    res = bench.run_pdsch(args, 1, 0, 0, None)
    assert res["resident_sets"] == 3
    assert res["crc_ok_tbs"] == "1200/1200"
    assert res["crc_bitmap"]["length_bits"] == 1200 and res["crc_bitmap"]["ok_tbs"] == 1200
    assert res["payload_checked_tbs"] == "1200/1200"  # every TB's bytes, checked on the GPU after its call
    assert res["config"]["workers_per_gpu"] == 3  # the PHY worker pool takes the resident sets' batches in turn
