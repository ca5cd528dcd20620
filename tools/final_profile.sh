#!/bin/bash
# End-of-round measurement set on one GPU box (everything under gpurun_out/):
#   GPU tests -> PMC passes (traffic counters, then the SQ / TCC groups) -> pmc_traffic.json ->
#   default bench.py (with the CPU baseline) -> rocprofv3 kernel-trace --stats of a short bench.
# usage: bash tools/final_profile.sh [tag]
set -u
tag=${1:-fin}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${tag}_tests.log 2>&1 || { tail -5 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
rm -rf gpurun_out/pmc
GPK_LOOKAHEAD=0 PMC_FILE=tools/pmc_traffic.txt bash tools/pmc_pass.sh || exit 1
python tools/pmc_traffic.py metric_b${BATCH:-64} gpurun_out/pmc profiles/pmc_traffic.json || exit 1
cp profiles/pmc_traffic.json gpurun_out/${tag}_pmc_traffic.json
mv gpurun_out/pmc gpurun_out/pmc_traffic_passes
GPK_LOOKAHEAD=0 PMC_FILE=tools/pmc_groups.txt bash tools/pmc_pass.sh || exit 1
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/${tag}_pmc_summary.txt || exit 1
timeout -k 10 900 python bench.py > gpurun_out/${tag}_bench.log 2>&1 || { tail -5 gpurun_out/${tag}_bench.log; exit 1; }
grep '^{' gpurun_out/${tag}_bench.log | cut -c1-300
bash tools/prof_run.sh ${tag}_prof || exit 1
