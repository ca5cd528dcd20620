#!/bin/bash
# Final tree check on one GPU box: GPU tests, smoke(), default bench (with CPU baseline), rocprofv3 stats.
# usage: bash tools/final_check.sh TAG
set -u
tag=${1:-fin}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1 || { tail -5 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -5 gpurun_out/${tag}_smoke.log; exit 1; }
grep smoke: gpurun_out/${tag}_smoke.log
timeout -k 10 900 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -5 gpurun_out/${tag}_bench.log; exit 1; }
grep '^{' gpurun_out/${tag}_bench.log | cut -c1-200
bash tools/prof_run.sh ${tag}_prof || exit 1
