#!/bin/bash
# rocprof kernel stats of the OD and SI bench lines (3xFP16 path only: --no-f32 --no-parity, so the
# conv-stage average is comparable with the bench line's roofline.avg_launch_ms)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_bench
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o od -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/prof_bench.log 2>&1 || exit $?
find gpurun_out/prof_bench -type f ! -name '*_stats.csv' -delete
bash tools/gpu/prof_si.sh > gpurun_out/prof_si_summary.txt 2>&1 || exit $?
echo profiled
