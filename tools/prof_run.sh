#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run into gpurun_out/$1 (extra bench args after it).
set -u
ROOT=$(pwd); export TMPDIR=/tmp
name=$1; shift
mkdir -p gpurun_out
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$ROOT/gpurun_out/$name" -o run -- python "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline "$@" \
    > gpurun_out/$name.log 2>&1
rc=$?; echo "prof $name rc=$rc"; grep '^{' gpurun_out/$name.log | cut -c1-300
exit $rc
