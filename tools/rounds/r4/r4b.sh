set -o pipefail
timeout -k 10 800 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_grad_handlings.py tests/test_gpu_approx_grad.py tests/test_gpu_syevd.py tests/test_gpu_strategies.py -m gpu > gpurun_out/r4b_tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r4b_tests.log
SETS='{"chain":0};{"chain":2,"chain_max_p":100000,"chain_group":1};{"chain":2,"chain_max_p":100000,"chain_group":4};{"chain":2,"chain_max_p":100000,"chain_group":8}' timeout -k 10 300 python tools/single_sched.py 4096 6144 8192 12288 > gpurun_out/r4b_sched.jsonl 2>&1 || exit 1
for g in 0 64; do
  GPK_CHAIN_GRID=$g timeout -k 10 120 python bench.py --config C2 --steps 400 --warmup 20 --chain 2 --pipeline 4 --no-cpu-baseline --no-check > gpurun_out/r4b_c2_g$g.json 2>gpurun_out/r4b_c2_g$g.err || exit 1
done
timeout -k 10 120 python bench.py --config C2 --steps 400 --warmup 20 --pipeline 4 --no-cpu-baseline --no-check > gpurun_out/r4b_c2_launch.json 2>gpurun_out/r4b_c2_launch.err
