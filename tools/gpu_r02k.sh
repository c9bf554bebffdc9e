#!/bin/bash
# r02k: smoke, GPU suite, MAP PMC for the current sources, default bench, e2e kernel stats
mkdir -p gpurun_out/r02k
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r02k/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02k/gputest.log 2>&1 || { echo suite failed; exit 1; }
bash tools/profile_tdec.sh r02k > gpurun_out/r02k/prof.log 2>&1 || { echo profile failed; exit 1; }
cp profiles/r02_tdec_pmc.json profiles/r02k_pmc_summary.json gpurun_out/r02k/ 2>/dev/null
timeout -k 10 300 python -u bench.py > gpurun_out/r02k/bench.json 2> gpurun_out/r02k/bench.err && bash tools/e2e_stats.sh r02k
echo rc=$?
