#!/bin/bash
# LDS counters of the single-evaluation chain (get_metric at N, look-ahead off: diag2 fused panel solve,
# thin updates): one rocprofv3 --pmc pass, CSV under gpurun_out/$1.
set -u
OUT=${1:-diag_pmc}; N=${2:-4096}
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d "gpurun_out/$OUT" -o run -- python tools/bench_api_latency.py --no-grad $N \
  > "gpurun_out/$OUT.log" 2>&1
