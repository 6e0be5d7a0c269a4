#!/bin/bash
# rbs (rolling strips) vs resblk tiles: tests, then the bench line with each (MMLA_RB_TILE), twice
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_rbs.py tests/test_gpu_parity.py -k "rbs or layerwise or precision_modes" > gpurun_out/rbs_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/rbs_tests.log; exit 1; }
tail -3 gpurun_out/rbs_tests.log
for r in 1 2; do
  for t in 1 0; do
    MMLA_RB_TILE=$t timeout -k 10 300 python bench.py --no-cpu-baseline --no-f32 --no-latency > gpurun_out/ab_${t}_${r}.json 2> gpurun_out/ab_err.log || { echo "bench rc=$?"; tail -20 gpurun_out/ab_err.log; exit 1; }
    python -c "
import json,sys
d=json.loads(open('gpurun_out/ab_${t}_${r}.json').read())
p=d['parity']
print('tile=$t', round(d['value']), 'conv_ms', d['stages']['conv']['ms'], 'frac', round(d['roofline']['frac'],4), 'logp_net', p['logp_err_net'], 'agree', p['argmax_agree'])
"
  done
done
