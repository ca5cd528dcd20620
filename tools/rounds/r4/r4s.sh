# rocprofv3 kernel stats of 33 single N = 4096 evaluations (persistent factorisation) + their HIP-event spans
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd); O=gpurun_out/r4s; mkdir -p $O
SETS='{"chain":1}' timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- python tools/single_sched.py 4096 > $O/sched.log 2>&1 || exit 1
