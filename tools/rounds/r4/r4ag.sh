# auto chain_group: tests and spans
set -o pipefail
O=gpurun_out/r4ag; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed" >> $O/tests.log; exit 1; }
SETS='{"chain":1}' timeout -k 10 400 python tools/single_sched.py 4096 8192 10240 12288 > $O/ab.jsonl 2>&1 || exit 1
