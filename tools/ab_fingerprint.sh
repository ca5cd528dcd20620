#!/bin/bash
# Bitwise A/B of prebuilt libgpk variants: NAMES="base x" bash tools/ab_fingerprint.sh
set -u
mkdir -p gpurun_out
for n in ${NAMES}; do
  GPK_LIB=variants/libgpk_$n.so timeout -k 10 120 python tools/variant_fingerprint.py > gpurun_out/fp_$n.log 2>&1
  rc=$?; echo "fingerprint $n rc=$rc"
  case $rc in 0) ;; *) tail -5 gpurun_out/fp_$n.log; exit $rc;; esac
done
set -- ${NAMES}
ref=$1; shift
for n in "$@"; do
  if diff <(grep '^n=' gpurun_out/fp_$ref.log) <(grep '^n=' gpurun_out/fp_$n.log) > /dev/null; then
    echo "$n: bitwise identical to $ref"
  else
    echo "$n: DIFFERS from $ref"; diff <(grep '^n=' gpurun_out/fp_$ref.log) <(grep '^n=' gpurun_out/fp_$n.log) | head -8
  fi
done
