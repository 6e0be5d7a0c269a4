#!/bin/bash
# SI change check: the SI GPU tests, then A/B of the SI line against a reference build ($1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sc_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/sc_pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/sc_pytest.log | head -20; exit 1; }
timeout -k 10 300 python3 bench.py --workload si_pipeline --no-cpu-baseline --no-f32 --no-latency > gpurun_out/sc_bench.log 2>&1 || { tail -20 gpurun_out/sc_bench.log; exit 1; }
grep '^{' gpurun_out/sc_bench.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('parity', d['parity'])"
bash tools/gpu/ab.sh si_pipeline $1 mmla_audio_amd/libmmla.so 3 || exit 1
