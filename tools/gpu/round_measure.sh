#!/bin/bash
# Round measurement: bench suite (4 workloads) + rocprof kernel stats (OD, SI) + PMC traffic
cd $GRAFT_REPO_ROOT
bash tools/gpu/bench_all.sh || exit $?
bash tools/gpu/prof_si.sh || exit $?
bash tools/gpu/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || exit $?
echo measured
