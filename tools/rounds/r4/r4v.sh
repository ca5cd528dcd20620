# one Newton step (per-pivot bad bookkeeping kept): probe, tests, spans
set -o pipefail
O=gpurun_out/r4v; mkdir -p $O
timeout -k 5 30 ./tools/probe/potf2_n1 > $O/probe.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_diag_versions.py tests/test_gpu_strategies.py tests/test_gpu_grad_handlings.py tests/test_gpu_dropin.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed" >> $O/tests.log; exit 1; }
SETS='{"chain":1};{"chain":0,"lookahead":2}' timeout -k 10 300 python tools/single_sched.py 1024 2048 4096 6144 8192 > $O/ab.jsonl 2>&1 || exit 1
timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof.txt 2>&1 || exit 1
