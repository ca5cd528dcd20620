#!/bin/bash
# C4 strong-scaling projection on one GPU: rank 0's slice of the 128-candidate N = 4096 sweep at
# W = 1 / 2 / 4 / 8 ranks (bench.py --config C4 --slice-of W), one JSON line per W.
set -u
OUT=${1:-gpurun_out/c4_slices.jsonl}
: > "$OUT"
for W in 1 2 4 8; do
  timeout -k 10 240 python bench.py --config C4 --slice-of $W --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline \
      --roofline-steps 1 ${BENCH_ARGS:-} > gpurun_out/c4_slice_$W.log 2>&1
  rc=$?
  echo "W=$W rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  grep '^{' gpurun_out/c4_slice_$W.log >> "$OUT"
done
