# round 6: the whole GPU suite on the f32-chain tree (+ smoke)
set -o pipefail
O=${O:-gpurun_out/r6l}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
exit 0
