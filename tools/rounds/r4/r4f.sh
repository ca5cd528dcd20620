set -o pipefail
export TMPDIR=/tmp
KB=gpurun_out/kb2 bash tools/r4d_kbuild_pmc.sh || exit 1
GPK_LOOKAHEAD=0 PMC_FILE=tools/pmc_traffic.txt BENCH_ARGS="" bash tools/pmc_pass.sh > gpurun_out/pmc_pass.log 2>&1 || exit 1
