set -o pipefail
mkdir -p gpurun_out/r4e
timeout -k 10 200 python tools/bench_kbuild.py C5 C3 SE8192 > gpurun_out/r4e/kbuild_pair.jsonl 2>&1 || exit 1
GPK_ASM_PAIR=0 timeout -k 10 200 python tools/bench_kbuild.py C5 > gpurun_out/r4e/kbuild_nopair.jsonl 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > gpurun_out/r4e/tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r4e/tests.log
