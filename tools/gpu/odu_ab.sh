#!/bin/bash
# dev (round 5): odu tests, then the OD bench line with the fused blocks 4-9 and with the conv_h3 pairs
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" > gpurun_out/quick.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/quick.log; exit 1; }
tail -3 gpurun_out/quick.log
for r in 1 2; do
for v in 0 1; do
  MMLA_NO_ODU=$v timeout -k 10 600 python bench.py --no-cpu-baseline --no-latency --no-f32 --no-parity > gpurun_out/bench_odu$v.json 2> gpurun_out/bench_odu$v.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_odu$v.err; exit 1; }
  python - $v <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/bench_odu{sys.argv[1]}.json').read())
print('NO_ODU', sys.argv[1], 'value', round(d['value']), 'roof', round(d['roofline']['frac'], 4), 'conv ms', d['stages']['conv']['ms'])
PY
done
done
