cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "od_" > gpurun_out/tq.log 2>&1; rc=$?; tail -3 gpurun_out/tq.log; [ $rc = 0 ] || { grep -E "Error|assert|err" gpurun_out/tq.log | head -20; exit 1; }
timeout -k 10 200 python bench.py --workload od_features --no-cpu-baseline --no-parity --no-latency --steps 50 > gpurun_out/fq.log 2>&1 || exit 1
python3 -c "
import json
l=[x for x in open('gpurun_out/fq.log') if x.startswith('{')][-1]; d=json.loads(l); print('fe', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
