set -o pipefail
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_grad_handlings.py -m gpu > gpurun_out/r4a_tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r4a_tests.log
for g in 0 64 128; do
  GPK_CHAIN_GRID=$g timeout -k 10 120 python bench.py --config C2 --steps 400 --warmup 20 --chain 2 --pipeline 4 --no-cpu-baseline --no-check > gpurun_out/r4a_c2_g$g.json 2>gpurun_out/r4a_c2_g$g.err || exit 1
done
timeout -k 10 120 python bench.py --config C2 --steps 400 --warmup 20 --pipeline 4 --no-cpu-baseline --no-check > gpurun_out/r4a_c2_launch.json 2>gpurun_out/r4a_c2_launch.err
