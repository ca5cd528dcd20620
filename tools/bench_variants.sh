#!/bin/bash
# Run bench.py under several environment variants (timing only, no CPU baseline).
# usage: VARIANTS="NAME=ENV[@ARGS] ..." bash tools/bench_variants.sh
#        ENV like GPK_X=1,GPK_Y=2 (or -), ARGS like --batch,4 (commas become spaces)
set -u
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  name=${v%%=*}; envs=${v#*=}
  vargs=""
  case "$envs" in *@*) vargs=$(echo "${envs#*@}" | tr ',' ' '); envs=${envs%%@*};; esac
  envline=$(echo "$envs" | tr ',' ' ')
  [ "$envs" = "-" ] && envline=""
  env $envline timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} $vargs > gpurun_out/var_$name.log 2>&1
  rc=$?
  echo "== $name ($envline) rc=$rc"
  python -c "
import json,sys
l=[x for x in open('gpurun_out/var_$name.log') if x.startswith('{')]
if l:
  d=json.loads(l[-1]); print('  value', d['value'], 'ms', d['ms_per_step'], 'upd TF', d['roofline']['achieved'] if d['roofline'] else None, d['kernel_ms_per_step'])
"
  case $rc in 124|134|137|139) exit $rc;; esac
done
