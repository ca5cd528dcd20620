#!/bin/bash
# Single-evaluation latency vs the 128-tile thresholds of the update / panel solve launches
set -u
for spec in "512 256" "128 256" "2048 256" "512 64" "512 1024"; do
  set -- $spec
  for a in "value 8192 1" "value 4096 1"; do
    GPK_UPD_T128_MIN=$1 GPK_TRSM_T128_MIN=$2 timeout -k 10 100 python tools/exp_grad.py $a > gpurun_out/tt.log 2>&1 || exit 1
    echo "upd_t128_min=$1 trsm_t128_min=$2 $a: $(grep 'per call' gpurun_out/tt.log | sed 's/ (.*//')"
  done
done
