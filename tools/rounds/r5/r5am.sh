# round 5: the persistent fast-tile kernel (asm_fast_persist): bitwise vs the grid kernel, then C5 K build A/B
set -o pipefail
O=gpurun_out/r5am; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kbuild_pair.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for g in 0 512 768 1024 1536 2048 0; do
  GPK_FAST_PERSIST=$g timeout -k 10 120 python tools/bench_kbuild.py C5 > $O/kb_$g.log 2>&1 || { tail -3 $O/kb_$g.log; exit 1; }
  grep '^{' $O/kb_$g.log | sed "s/^{/{\"persist\": $g, /"
done
