#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu3.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python bench.py > gpurun_out/bench_od.log 2>&1 || exit $?
echo "bench od done"; tail -1 gpurun_out/bench_od.log
timeout -k 10 900 python bench.py --workload si_pipeline > gpurun_out/bench_si.log 2>&1 || exit $?
echo "bench si done"; tail -1 gpurun_out/bench_si.log
timeout -k 10 600 python bench.py --workload od_features --steps 5 > gpurun_out/bench_fe.log 2>&1 || exit $?
echo "bench fe done"; tail -1 gpurun_out/bench_fe.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r1 -o od -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_od.log 2>&1 || exit $?
echo "rocprof done"; ls -R gpurun_out/prof_r1 | head -20
