#!/bin/bash
# Round measurement: the four bench workloads (default = the headline OD pipeline) + rocprof kernel
# stats of the OD pipeline.  Outputs under gpurun_out/ (copied into profiles/ by hand).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u bench.py > gpurun_out/bench_od.json.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_od.json.log > gpurun_out/bench_od.json
timeout -k 10 600 python3 -u bench.py --workload si_pipeline > gpurun_out/bench_si.json.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_si.json.log > gpurun_out/bench_si.json
timeout -k 10 600 python3 -u bench.py --workload si_pipeline --classes 8 > gpurun_out/bench_si8.json.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_si8.json.log > gpurun_out/bench_si8.json
timeout -k 10 600 python3 -u bench.py --workload od_features > gpurun_out/bench_fe.json.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_fe.json.log > gpurun_out/bench_fe.json
timeout -k 10 600 python3 -u bench.py --workload noise_gate > gpurun_out/bench_nr.json.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_nr.json.log > gpurun_out/bench_nr.json
rm -rf gpurun_out/prof_bench
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o od -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/prof_bench.log 2>&1 || exit $?
python3 - <<'PY'
import json
for f in ('od', 'si', 'si8', 'fe', 'nr'):
    d = json.load(open(f'gpurun_out/bench_{f}.json'))
    print(f, d['value'], d['unit'], 'ms/step', round(d['ms_per_step'], 2), 'roof', {k: d['roofline'][k] for k in ('kernel', 'achieved', 'peak', 'frac') if k in d['roofline']}, 'cpu', (d.get('cpu_baseline') or {}).get('value'))
PY
# keep only the stats summaries (traces exceed gpurun's copy-back limit)
find gpurun_out/prof_bench -type f ! -name '*_stats.csv' -delete
