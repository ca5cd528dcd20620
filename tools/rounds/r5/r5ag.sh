# round 5: pair-path tests (ragged, gradient) on the final tree
set -o pipefail
O=gpurun_out/r5ag; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_kbuild_pair.py -m gpu -s > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error|pair MFMA" $O/tests.log | tail -20; exit $rc
