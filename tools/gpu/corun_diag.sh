#!/bin/bash
# dev: co-run matrix after the front-end store-wait fix, then the full GPU suite
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/corun_diag4.py > gpurun_out/corun4.log 2>&1 || { tail -20 gpurun_out/corun4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/corun4.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1
rc=$?; tail -3 gpurun_out/suite.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/suite.log | head; exit $rc; }
