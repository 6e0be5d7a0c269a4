#!/bin/bash
# round 4: host-mapped outputs / range flag for small host-pointer calls (MMLA_NO_PIN_OUT): the whole
# GPU suite, then batch-1 latency with and without
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pin_pytest.log 2>&1 || { tail -30 gpurun_out/pin_pytest.log; exit 1; }
tail -1 gpurun_out/pin_pytest.log
for i in 1 2; do
  echo "pin on"; timeout -k 10 120 python3 tools/latency_probe.py || exit 1
  echo "pin off"; MMLA_NO_PIN_OUT=1 timeout -k 10 120 python3 tools/latency_probe.py || exit 1
done
