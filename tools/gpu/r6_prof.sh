#!/bin/bash
# Round-6 checkpoint, part 3: rocprof kernel stats of the SI and front-end bench lines, SQ counters of
# the SI pipeline (part 4, r6_pmc_od.sh: the OD pipeline's)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
WL=si_pipeline TAG=si_pipeline BENCH_ARGS="--no-latency" bash tools/gpu/prof_line.sh || exit $?
WL=od_features TAG=od_features BENCH_ARGS="--no-latency" bash tools/gpu/prof_line.sh || exit $?
bash tools/gpu/pmc_kernels.sh si_pipeline 65536 r6si > gpurun_out/pmc_r6si.log 2>&1 || { tail -20 gpurun_out/pmc_r6si.log; exit 1; }
