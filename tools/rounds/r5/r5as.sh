# round 5: one host-to-device copy for hyperparameters + noise, a fresh read-out buffer per evaluation (no clone):
# full GPU suite, drop-in API latency, and the N = 256 device trace again
set -o pipefail
O=gpurun_out/r5as; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/bench_api_latency.py 128 256 512 1024 2048 4096 8192 > $O/api.log 2>&1 || { tail -3 $O/api.log; exit 1; }
grep '^{' $O/api.log
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$(pwd)/$O/n256" -o run -- python tools/api_profile.py 256 200 > $O/n256.log 2>&1 || { tail -3 $O/n256.log; exit 1; }
grep "us per call" $O/n256.log
