# round 5: the held-result independence test of the clone-free read-out, and the drop-in tests around it
set -o pipefail
O=gpurun_out/r5aw; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dropin.py tests/test_gpu_grad.py > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
