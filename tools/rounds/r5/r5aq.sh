# round 5: the fast-tile kernel over chunks of consecutive lower tiles (row features loaded once per tile row):
# pair tests on the in-tree build (chunk 1) and on the chunk-4 variant, then C5 K build A/B of chunk 1 (base =
# the previous build, new = in-tree) / 2 / 4 / 8 (variants -DGPK_FAST_CHUNK=2|4|8)
set -o pipefail
O=gpurun_out/r5aq; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kbuild_pair.py tests/test_gpu_kbuild.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GPK_LIB=variants/libgpk_ch4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kbuild_pair.py > $O/pytest_ch4.log 2>&1 || { tail -20 $O/pytest_ch4.log; exit 1; }
tail -1 $O/pytest_ch4.log
cp gaussianprocessfundamentals_amd/libgpk.so variants/libgpk_new.so
NAMES="base new ch2 ch4 ch8 base new ch2 ch4 ch8" bash tools/ab_kbuild.sh C5
