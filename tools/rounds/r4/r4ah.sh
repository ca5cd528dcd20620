# exactly symmetric periodic entries (separately rounded products): K-build timing, then the full GPU suite + smoke
set -o pipefail
O=gpurun_out/r4ah; mkdir -p $O
timeout -k 10 200 python tools/bench_kbuild.py C5 C3 SE8192 > $O/kbuild.jsonl 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed" >> $O/tests.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
