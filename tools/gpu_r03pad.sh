#!/bin/bash
# padded LDS image in the rate dematchers + pdsch_eq_rm: parity suites, kernel times (fused on / off), A/B vs cpb1
set -e
OUT=gpurun_out/r03pad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dlsch_gpu.py tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_pdsch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
MI355_NO_EQRM=1 timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_noeqrm.log 2>&1
bash tools/gpu_eqtrace.sh srsran_amd/lib_var/pad.so srsran_amd/lib_var/cpb1.so > $OUT/et.txt 2>&1
MI355_NO_EQRM=1 bash tools/gpu_eqtrace.sh srsran_amd/lib_var/pad.so > $OUT/et_off.txt 2>&1
for f in gpurun_out/rt/0 gpurun_out/rt/1; do python3 - $f <<'PY' >> $OUT/k.txt
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("pdsch_eq_rm", "dlsch_rm_rx", "pdsch_eq_llr")):
        print(sys.argv[1], r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
echo rc=0
