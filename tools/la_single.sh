#!/bin/bash
# Single-evaluation latency (batch 1, no pipelining) under look-ahead / panel-stream variants.
# NS: problem sizes; VARIANTS: env assignments per run (LA=0|1 picks bench --lookahead).
set -e
mkdir -p gpurun_out
for n in ${NS:-4096 8192}; do
 for v in ${VARIANTS:-"LA=0" "LA=1 GPK_PANEL_STREAM=0" "LA=1 GPK_PANEL_STREAM=1" "LA=1 GPK_PANEL_STREAM=2" "LA=1 GPK_PANEL_STREAM=1 GPK_RESERVE_CUS=0"}; do
  tag=$(echo "$n $v" | tr ' =' '__')
  env $v timeout -k 10 120 python bench.py --config C2 --n $n --batch ${BATCH:-1} --pipeline 1 --lookahead $(echo "$v" | sed 's/.*LA=\([012]\).*/\1/') \
      --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline --roofline-steps 1 > gpurun_out/la_$tag.log 2>&1
  echo "n=$n batch=${BATCH:-1} $v: $(grep '^{' gpurun_out/la_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
 done
done
