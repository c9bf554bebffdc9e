#!/bin/bash
# r04b: new per-CB generic decoder tests first; then as r04a (GPU suite, bench, row-mask A/B, fan-out, SISO trace, eq_rm SQ counters)
# skip (MI355_NO_ROWMASK); fan-out at world 1; configs[2] SISO QPSK trace + host phases; pdsch_eq_rm SQ counters
set -e
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tdec_gen_cb_gpu.py tests/test_srslte_tdec_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gen_cb.log 2>&1 || { rc=$?; echo gen_cb rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 200 python3 -u tools/gen_cb_sweep.py > $OUT/gen_cb_sweep.jsonl 2> $OUT/gen_cb_sweep.err || { rc=$?; echo sweep rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --deselect tests/test_tdec_gen_cb_gpu.py --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_suite.log 2>&1 || { rc=$?; echo suite rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 400 python3 -u bench.py --no-waterfall > $OUT/bench.json 2> $OUT/bench.err
for i in 1 2; do
  MI355_NO_ROWMASK=1 timeout -k 10 200 python3 -u bench.py --no-cpu --no-waterfall --no-roofline > $OUT/ab_off_$i.json 2>> $OUT/ab.err
  timeout -k 10 200 python3 -u bench.py --no-cpu --no-waterfall --no-roofline > $OUT/ab_on_$i.json 2>> $OUT/ab.err
done
timeout -k 10 300 python3 -u bench.py --fanout --steps 3 --warmup 1 --subframes 1024 > $OUT/fanout.json 2> $OUT/fanout.err
MI355_HOST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/siso -o tr -- python3 bench.py --workload siso_qpsk --steps 3 --warmup 1 --no-cpu --no-roofline > $OUT/siso.json 2> $OUT/siso.err
timeout -k 10 300 python3 -u bench.py --workload siso_qpsk --steps 5 --warmup 2 --no-cpu --no-roofline > $OUT/siso_plain.json 2> $OUT/siso_plain.err
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d $OUT/sq1 -o sq -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/sq1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq2 -o sq -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/sq2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/lat -o lat -- python3 tools/dropin_lat.py 200 > $OUT/lat.log 2>&1
echo rc=0
