#!/bin/bash
# Ragged-batch timing per prebuilt variant: NAMES="base x" bash tools/ab_ragged.sh [n] [members]
set -u
mkdir -p gpurun_out
for v in ${NAMES}; do
  GPK_LIB=variants/libgpk_$v.so timeout -k 10 200 python tools/bench_ragged.py "$@" > gpurun_out/rg_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/rg_$v.log; exit $rc; }
  grep '^{' gpurun_out/rg_$v.log | sed "s/^/$v /"
done
