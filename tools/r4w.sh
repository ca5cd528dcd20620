# round-4 final measurement set on the current tree (tests + smoke + bench + rocprof + API latency + C2)
set -o pipefail
bash tools/gpu_final.sh r04w || exit 1
R4O_OUT=gpurun_out/r4w_c2 bash tools/r4o.sh || exit 1
