# final tree: full check (tests, smoke, bench, rocprof), API latency, C2 with and without pipelining
set -o pipefail
T=${1:-r03p}
bash tools/final_check.sh $T || exit 1
timeout -k 10 300 python tools/bench_api_latency.py 256 1024 2048 4096 6144 8192 > gpurun_out/${T}_api.log 2>&1 || { tail -5 gpurun_out/${T}_api.log; exit 1; }
grep "^{" gpurun_out/${T}_api.log
GPK_CHAIN=0 timeout -k 10 300 python tools/bench_api_latency.py --no-grad 256 1024 2048 4096 6144 > gpurun_out/${T}_api_launch.log 2>&1 || { tail -5 gpurun_out/${T}_api_launch.log; exit 1; }
grep "^{" gpurun_out/${T}_api_launch.log
timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_c2.log 2>&1 || { tail -5 gpurun_out/${T}_c2.log; exit 1; }
grep "^{" gpurun_out/${T}_c2.log | cut -c1-200
timeout -k 10 300 python bench.py --config C2 --pipeline 1 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${T}_c2_p1.log 2>&1 || { tail -5 gpurun_out/${T}_c2_p1.log; exit 1; }
grep "^{" gpurun_out/${T}_c2_p1.log | cut -c1-200
