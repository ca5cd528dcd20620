# persistent factorisation: GPU tests, per-task profile at N = 4096, single-evaluation span vs the launch path
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c2_tests.log 2>&1 || { tail -20 gpurun_out/c2_tests.log; exit 1; }
tail -1 gpurun_out/c2_tests.log
timeout -k 10 120 python tools/chain_prof.py 4096 > gpurun_out/c2_prof.log 2>&1 || { tail -5 gpurun_out/c2_prof.log; exit 1; }
grep -v "^INFO\|amdgpu.ids" gpurun_out/c2_prof.log
SETS='{"chain":0,"lookahead":0};{"chain":1}' timeout -k 10 200 python tools/single_sched.py ${SIZES:-1024 2048 4096} > gpurun_out/c2_sched.log 2>&1 || { tail -5 gpurun_out/c2_sched.log; exit 1; }
grep '^{' gpurun_out/c2_sched.log
