#!/bin/bash
# round 6: the new tests first, then the GPU suite, then the default bench line (no CPU leg)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_tf_compat.py tests/test_gpu_range_guard.py tests/test_gpu_batching.py > gpurun_out/new.log 2>&1 || { echo "new tests rc=$?"; tail -40 gpurun_out/new.log; exit 1; }
tail -3 gpurun_out/new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1 || { echo "suite rc=$?"; tail -30 gpurun_out/suite.log; exit 1; }
tail -3 gpurun_out/suite.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_od.json 2> gpurun_out/bench_od.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_od.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/bench_od.json').read())
print('value', d['value'], 'roof', d['roofline']['frac'], 'fe', d['fe']['roofline']['frac'])
print('stages', d['stages'])
print('parity', {k: d['parity'][k] for k in ('logp_err_net', 'logp_max_abs_err', 'img_lsb_pixels', 'argmax_agree')})
PY
