#!/bin/bash
# A/B of prebuilt libgpk variants on single-evaluation latency (batch 1, no pipelining, look-ahead auto).
# usage: NAMES="base x" [NS="1024 4096"] [CHECK="x"] bash tools/ab_single.sh
set -u
mkdir -p gpurun_out
for v in ${CHECK:-}; do
  GPK_LIB=variants/libgpk_$v.so timeout -k 10 300 python -m pytest tests -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "${CHECK_K:-schedule or golden or diag_versions or fused_panel}" > gpurun_out/abs_chk_$v.log 2>&1
  rc=$?; echo "check $v rc=$rc $(tail -1 gpurun_out/abs_chk_$v.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
for rep in 1 2; do
 for n in ${NS:-1024 4096}; do
  for v in ${NAMES}; do
   GPK_LIB=variants/libgpk_$v.so timeout -k 10 120 python bench.py --config C2 --n $n --batch 1 --pipeline 1 --steps ${STEPS:-50} \
      --warmup 5 --no-cpu-baseline --roofline-steps 1 > gpurun_out/abs_${v}_$n.log 2>&1
   rc=$?
   echo "rep $rep n=$n $v: $(grep '^{' gpurun_out/abs_${v}_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["check"])')"
   case $rc in 124|134|137|139) exit $rc;; esac
  done
 done
done
