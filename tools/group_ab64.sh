#!/bin/bash
# Panel-group size at the default metric bench (64 x 2): two alternating passes.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
for g in ${GS:-8 12 16}; do
  GPK_GROUP=$g timeout -k 10 300 python bench.py --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/g64.log 2>&1 || exit 1
  echo "group $g: $(grep '^{' gpurun_out/g64.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"])')"
done
done
