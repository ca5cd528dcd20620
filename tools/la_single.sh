#!/bin/bash
# Single-evaluation latency (batch BATCH, no pipelining) under schedule variants.
# NS: problem sizes; VARIANTS: space-separated variants, each a comma-separated list of env
# assignments (LA=0|1|2 picks bench --lookahead, default 2 = auto).
set -e
mkdir -p gpurun_out
for n in ${NS:-4096 8192}; do
 for v in ${VARIANTS:-LA=0 LA=1 LA=2}; do
  tag=$(echo "$n $v" | tr ' =,' '___')
  la=$(echo ",$v," | sed -n 's/.*,LA=\([012]\),.*/\1/p'); la=${la:-2}
  env $(echo "$v" | tr ',' ' ') timeout -k 10 120 python bench.py --config C2 --n $n --batch ${BATCH:-1} --pipeline 1 --lookahead $la \
      --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline --roofline-steps 1 > gpurun_out/la_$tag.log 2>&1
  echo "n=$n batch=${BATCH:-1} $v: $(grep '^{' gpurun_out/la_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
 done
done
