#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one counter group per pass, kernel trace only).
set -u
ROOT=$(pwd); export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
i=0
for grp in "${PMC_GROUPS[@]:-}"; do :; done
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pmc/p$i" -o run \
     -- python "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-events ${BENCH_ARGS:-} > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done < "${PMC_FILE:-tools/pmc_groups.txt}"
