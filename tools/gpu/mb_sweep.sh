cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for mb in 16384 32768 65536 16384 65536; do
  timeout -k 10 300 python3 bench.py --workload si_pipeline --no-cpu-baseline --microbatch $mb > gpurun_out/mb_si_$mb.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/mb_si_$mb.log') if l.startswith('{')][-1]); print('si mb $mb', round(d['value']), round(d['ms_per_step'],2))"
done
