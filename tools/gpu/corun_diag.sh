#!/bin/bash
# dev: FE corruption next to resblk: register-capped FE with packed FP32 (minb3); FE throughput of
# the product build, the no-packed-FP32 build and the capped build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MMLA_LIB=mmla_audio_amd/ab/libmmla_minb3.so timeout -k 10 300 python3 -u tools/corun_diag7.py > gpurun_out/corun7d.log 2>&1 || { tail -20 gpurun_out/corun7d.log; exit 1; }
grep -v amdgpu.ids gpurun_out/corun7d.log
for lib in mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_nopk.so mmla_audio_amd/ab/libmmla_minb3.so; do
  for n in 4096 65536; do
    timeout -k 10 300 python3 tools/bench_with_lib.py $lib --workload od_features --clips $n --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fe_ab.log 2>&1 || exit $?
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/fe_ab.log') if l.startswith('{')][0]);r=d['roofline'];print('$lib',$n,'clips/s',round(d['value']),'frac',round(r['frac'],4))"
  done
done
