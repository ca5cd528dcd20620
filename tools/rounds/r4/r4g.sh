# UQ (quarter updates of the next diagonal block) in the persistent factorisation: correctness, then A/B
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed" >> $O/tests.log; exit 1; }
SETS='{"chain_uq":1};{"chain_uq":0};{"chain_uq":1};{"chain_uq":0}' timeout -k 10 300 python tools/single_sched.py 2048 4096 6144 8192 12288 > $O/ab.jsonl 2>&1 || exit 1
GPK_CHAIN_UQ=1 timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof_uq1.txt 2>&1 || exit 1
GPK_CHAIN_UQ=0 timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof_uq0.txt 2>&1 || exit 1
