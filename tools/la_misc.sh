#!/bin/bash
# Look-ahead on / off for the C4 sweep and the gradient path (ms per step).
set -e
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 120 python bench.py "$@" --no-cpu-baseline --roofline-steps 1 > gpurun_out/lam_$tag.log 2>&1
  echo "$tag: $(grep '^{' gpurun_out/lam_$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; }
for la in 0 1; do
  run c4_la$la --config C4 --pipeline 1 --lookahead $la --steps 10 --warmup 2
  run c4b16_la$la --config C4 --batch 16 --pipeline 1 --lookahead $la --steps 20 --warmup 2
  run grad4096_la$la --config C2 --mode grad --n 4096 --batch 1 --pipeline 1 --lookahead $la --steps 30 --warmup 3
  run grad2048b4_la$la --config C2 --mode grad --n 2048 --batch 4 --pipeline 1 --lookahead $la --steps 30 --warmup 3
done
