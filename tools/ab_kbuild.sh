#!/bin/bash
# K-build timing per prebuilt variant: NAMES="base x" bash tools/ab_kbuild.sh [cases]
set -u
for v in ${NAMES}; do
  GPK_LIB=variants/libgpk_$v.so timeout -k 10 200 python tools/bench_kbuild.py "$@" > gpurun_out/kb_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/kb_$v.log; exit $rc; }
  grep '^{' gpurun_out/kb_$v.log | sed "s/^/$v /"
done
