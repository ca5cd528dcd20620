# round-4 final measurement set on the current tree (tests + smoke + bench + rocprof + API latency + C2)
set -o pipefail
bash tools/gpu_final.sh ${TAG:-r04w} || exit 1
R4O_OUT=gpurun_out/${TAG:-r04w}_c2x bash tools/r4o.sh || exit 1
