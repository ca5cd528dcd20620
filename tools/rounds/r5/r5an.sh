# round 5: the committed library vs the refactored fast kernel (grid launch) and one-column-block passes at 4 / 5
# workgroups per CU (tools/build_variant.sh -DGPK_FAST_H=1 -DGPK_FAST_MINB=4|5), C5 K build, alternating
set -o pipefail
mkdir -p gpurun_out
NAMES="base new h1m4 h1m5 base new h1m4 h1m5 base new h1m4 h1m5" bash tools/ab_kbuild.sh C5
