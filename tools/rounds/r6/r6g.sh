# round 6: C5 K build with the column features double-buffered by LDS-DMA (GPK_FAST_DMA, default) against the round-5
# form (variants/libgpk_fastdma0.so, -DGPK_FAST_DMA=0), alternating; the pair-path tests on the default build
set -o pipefail
O=${O:-gpurun_out/r6g}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kbuild_pair.py tests/test_gpu_kbuild.py -m gpu -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 120 python tools/bench_kbuild.py C5 > $O/dma1_$rep.json 2> $O/e.err || { tail -3 $O/e.err; exit 1; }
  GPK_LIB=variants/libgpk_fastdma0.so timeout -k 10 120 python tools/bench_kbuild.py C5 > $O/dma0_$rep.json 2> $O/e.err || { tail -3 $O/e.err; exit 1; }
  echo "rep $rep dma1 $(tail -1 $O/dma1_$rep.json | cut -c1-120) | dma0 $(tail -1 $O/dma0_$rep.json | cut -c1-120)"
done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/stats" -o run -- python tools/bench_kbuild.py C5 > $O/stats.log 2>&1 || exit 1
f=$(find $O/stats -name "*kernel_stats.csv" | head -1); grep -h "pair_\|assemble" "$f" | cut -c1-160
exit 0
