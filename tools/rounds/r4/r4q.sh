# round-4 measurement set on the current tree: full GPU tests + smoke + default bench + rocprof stats,
# API latency (persistent and launch path), C2 by batch / launches in flight
set -o pipefail
bash tools/gpu_final.sh r04q || exit 1
bash tools/r4o.sh || exit 1
