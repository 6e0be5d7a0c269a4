#!/bin/bash
# dev (round 5): the OD parity-drift bisect (tools/parity_drift.py) + the split-BiLSTM timeout tests
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python tools/parity_drift.py head .
for s in ed28c4c 908a92d 85696f2; do
  timeout -k 10 200 python tools/parity_drift.py $s bisect/$s --pcm gpurun_out/drift_pcm.npy
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_batching.py -k "split or timeout" 
