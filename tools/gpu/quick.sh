#!/bin/bash
# dev: a few GPU test files (args) then the default bench line without the CPU baseline
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" > gpurun_out/quick.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/quick.log; exit 1; }
tail -3 gpurun_out/quick.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-latency > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_q.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/bench_q.json').read())
print('value', d['value'], 'roof', d['roofline']['frac'], 'stages', d['stages'])
print('parity', {k: d['parity'][k] for k in ('logp_err_net', 'logp_max_abs_err', 'img_lsb_pixels', 'argmax_agree')})
print('f32', d['precision_f32']['value'], d['precision_f32']['argmax_differs_from_f16x3'])
PY
