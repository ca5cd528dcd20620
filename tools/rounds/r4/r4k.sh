# potf2 pivot column by DPP row_newbcast: correctness, spans vs the LDS form, D phase timeline
# (historical A/B script of round 4: the variant libraries it names were built with tools/build_variant.sh and removed after the measurement -- see DESIGN §4 for the outcome)
set -o pipefail
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_diag_versions.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed" >> $O/tests.log; exit 1; }
SETS='{"chain":1};{"chain":0,"lookahead":2}' timeout -k 10 300 python tools/single_sched.py 1024 2048 4096 8192 > $O/ab_dpp.jsonl 2>&1 || exit 1
GPK_LIB=variants/libgpk_potf0.so SETS='{"chain":1};{"chain":0,"lookahead":2}' timeout -k 10 300 python tools/single_sched.py 1024 2048 4096 8192 > $O/ab_lds.jsonl 2>&1 || exit 1
GPK_LIB=variants/libgpk_dprof.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/dphase.txt 2>&1 || exit 1
timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof.txt 2>&1 || exit 1
