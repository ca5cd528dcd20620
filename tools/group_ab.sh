#!/bin/bash
# Single-evaluation latency vs panel group size: bash tools/group_ab.sh "8 4 2" ["value 8192 1"]
set -u
for g in $1; do
  GPK_GROUP=$g GPK_GROUP_FIRST=$g timeout -k 10 100 python tools/exp_grad.py ${2:-value 8192 1} > gpurun_out/grp.log 2>&1 || exit 1
  echo "group=$g ${2:-value 8192 1}: $(grep 'per call' gpurun_out/grp.log | sed 's/ (.*//' | tr '\n' ';')"
done
