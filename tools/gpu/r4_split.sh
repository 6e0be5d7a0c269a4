#!/bin/bash
# round 4: the small-batch BiLSTM split (bilstm_h3_split_kernel): bit-identity + parity tests, then
# batch-1 latency with and without it (MMLA_NO_LSTM_SPLIT), and a kernel trace of each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batching.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r4_split.log 2>&1
rc=$?; tail -5 gpurun_out/r4_split.log; [ $rc = 0 ] || exit 1
for i in 1 2; do
  echo "split on"; timeout -k 10 120 python3 tools/latency_probe.py || exit 1
  echo "split off"; MMLA_NO_LSTM_SPLIT=1 timeout -k 10 120 python3 tools/latency_probe.py || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/lat_split -o lat -- python3 tools/lat_od1.py > gpurun_out/lat_split.log 2>&1 || exit 1
MMLA_NO_LSTM_SPLIT=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/lat_nosplit -o lat -- python3 tools/lat_od1.py > gpurun_out/lat_nosplit.log 2>&1 || exit 1
for d in lat_split lat_nosplit; do
  echo "== $d"; python3 tools/kstats_db.py $(find gpurun_out/$d -name '*.db' | head -1) 6 || exit 1
done
