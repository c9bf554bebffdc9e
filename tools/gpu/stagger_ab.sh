mkdir -p gpurun_out/stg2
for st in 0 1 0 1 0 1 0 1; do
  BENCH_STAGGER_MS=$st BENCH_CALL_TRACE=gpurun_out/stg2/calls_$st.json timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --workers 3 --no-cpu --no-roofline --no-waterfall > gpurun_out/stg2/b.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/stg2/b.json').read().strip().splitlines()[-1]); t=json.load(open('gpurun_out/stg2/calls_$st.json')); t.sort(key=lambda r:r[1]); print('stagger $st', d['ms_per_step'], d['worker_calls'], ['%.1f'%(b-a) for w,a,b in t[:4]])"
done
