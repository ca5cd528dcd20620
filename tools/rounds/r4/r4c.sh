set -o pipefail
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_kbuild.py tests/test_gpu_parity.py tests/test_gpu_approx_grad.py tests/test_gpu_syevd.py tests/test_gpu_strategies.py -m gpu > gpurun_out/r4c_tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r4c_tests.log
timeout -k 10 300 python tools/chain_batch_ab.py 1024 2048 4096 > gpurun_out/r4c_chain_batch.jsonl 2>&1
timeout -k 10 200 python bench.py --config C5 --steps 30 --warmup 3 --no-cpu-baseline --no-check > gpurun_out/r4c_c5.json 2>gpurun_out/r4c_c5.err
timeout -k 10 200 python tools/bench_api_latency.py --no-grad 1024 4096 6144 8192 12288 > gpurun_out/r4c_api.jsonl 2>&1
bash tools/r4d_kbuild_pmc.sh
