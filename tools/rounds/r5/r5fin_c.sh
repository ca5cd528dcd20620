# round 5 final tree (3/3): PMC passes of the metric config (look-ahead off: the roofline post-pass's update
# launches) -> HBM bytes per update launch (profiles/pmc_traffic.json key metric_b64) + MFMA / LDS summary
set -o pipefail
GPK_LOOKAHEAD=0 BENCH_ARGS="--pipeline 1 --lookahead 0" bash tools/pmc_pass.sh || exit 1
mkdir -p gpurun_out/r05fin && python tools/pmc_traffic.py metric_b64 gpurun_out/pmc gpurun_out/r05fin/pmc_traffic.json || exit 1
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/r05fin/pmc_summary.txt 2>&1; cat gpurun_out/r05fin/pmc_summary.txt | head -30
