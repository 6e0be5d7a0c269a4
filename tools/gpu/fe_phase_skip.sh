cd $GRAFT_REPO_ROOT
for v in ${SKIPS:-0 1 2 4 8 16}; do
  if [ $v = 0 ]; then lib=mmla_audio_amd/libmmla.so; else lib=mmla_audio_amd/ab/libmmla_skip$v.so; fi
  timeout -k 10 200 python tools/bench_with_lib.py $lib --workload od_features --no-cpu-baseline --no-parity --no-latency --steps 50 > gpurun_out/skip$v.log 2>&1 || exit 1
  python3 -c "
import json
l=[x for x in open('gpurun_out/skip$v.log') if x.startswith('{')][-1]; d=json.loads(l); print('skip $v', d['roofline']['avg_launch_ms'])"
done
