#!/bin/bash
# Round-end measurement, part 1: GPU suite, the four bench lines + OD rocprof stats (bench_all.sh),
# rocprof stats of the SI and front-end lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1 || { tail -30 gpurun_out/fin_pytest.log; exit 1; }
tail -1 gpurun_out/fin_pytest.log
bash tools/gpu/bench_all.sh || exit $?
WL=si_pipeline TAG=si BENCH_ARGS="--no-latency" bash tools/gpu/prof_line.sh || exit $?
WL=od_features TAG=fe BENCH_ARGS="--no-latency" bash tools/gpu/prof_line.sh || exit $?
find gpurun_out -type f -size +8M -print -delete; du -sh gpurun_out
