#!/bin/bash
# split_rl on/off: bitwise fingerprint, then single-evaluation latency
set -u
for v in 0 1; do
  GPK_SPLIT_RL=$v timeout -k 10 120 python tools/variant_fingerprint.py > gpurun_out/fp_split$v.log 2>&1 || { tail -3 gpurun_out/fp_split$v.log; exit 1; }
done
if diff <(grep '^n=' gpurun_out/fp_split0.log) <(grep '^n=' gpurun_out/fp_split1.log) > /dev/null; then echo "split_rl: bitwise identical"; else echo "split_rl: DIFFERS"; diff <(grep '^n=' gpurun_out/fp_split0.log) <(grep '^n=' gpurun_out/fp_split1.log) | head; fi
for v in 0 1 0 1; do
  for a in "value 8192 1 4" "value 4096 1" "8192 1" "4096 1"; do
    GPK_SPLIT_RL=$v timeout -k 10 100 python tools/exp_grad.py $a > gpurun_out/sp.log 2>&1 || exit 1
    echo "split_rl=$v $a: $(grep 'per call' gpurun_out/sp.log | sed 's/ (.*//' | tr '\n' ';')"
  done
done
