# round 5: timing-only ablations of the C5 fast read-out (variants built with -DGPK_FAST_ABLATE=1|2|3: no table
# read in the exp / no stores / no exps), against the committed build; C5 K build, alternating
set -o pipefail
mkdir -p gpurun_out
NAMES="base abl1 abl2 abl3 base abl1 abl2 abl3" bash tools/ab_kbuild.sh C5
