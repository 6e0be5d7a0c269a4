#!/bin/bash
# HEAD check: GPU suite, the config-2 front-end line, the v3 front-end phase timeline (libmmla_exp.so)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/hc_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/hc_pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/hc_pytest.log | head -30; exit 1; }
bash tools/gpu/fe_quick.sh || exit 1
timeout -k 10 200 python3 -u tools/fe3_timeline.py 16 > gpurun_out/hc_tl.log 2>&1 || { tail -20 gpurun_out/hc_tl.log; exit 1; }
cat gpurun_out/hc_tl.log
bash tools/gpu/pmc_kernels.sh od_features 4096 r3fe > gpurun_out/hc_pmc.log 2>&1 || { tail -20 gpurun_out/hc_pmc.log; exit 1; }
grep -A30 "fe3" gpurun_out/pmc_r3fe_summary.txt | head -40
