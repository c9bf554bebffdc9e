# round 6 h: instruction mix of pdsch_eq_rm (compact image) and the MAP launches of the default step (SQ counters)
set -o pipefail
OUT=gpurun_out/r06h
mkdir -p $OUT
export TMPDIR=/tmp
PA="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
PB="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
i=0
for P in "$PA" "$PB"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "pdsch_eq_rm|tdec_win_halfit" --output-format csv \
    -d $OUT/p$i -o c -- python3 bench.py --workers 1 --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline \
    > $OUT/p$i.log 2>&1 || exit 1
done
echo rc=0
