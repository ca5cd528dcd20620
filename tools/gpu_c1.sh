set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c1_tests.log 2>&1 || { tail -20 gpurun_out/c1_tests.log; exit 1; }
tail -1 gpurun_out/c1_tests.log
timeout -k 10 120 python tools/chain_prof.py 4096 > gpurun_out/c1_prof_inl.log 2>&1 || { tail -5 gpurun_out/c1_prof_inl.log; exit 1; }
grep -v "^INFO\|amdgpu.ids" gpurun_out/c1_prof_inl.log | head -8
GPK_LIB=$PWD/gaussianprocessfundamentals_amd/libgpk_noinl.so timeout -k 10 120 python tools/chain_prof.py 4096 > gpurun_out/c1_prof_noinl.log 2>&1 || { tail -5 gpurun_out/c1_prof_noinl.log; exit 1; }
grep -v "^INFO\|amdgpu.ids" gpurun_out/c1_prof_noinl.log | head -8
SETS='{"chain":0,"lookahead":0};{"chain":1}' timeout -k 10 200 python tools/single_sched.py 1024 4096 8192 > gpurun_out/c1_sched.log 2>&1 || { tail -5 gpurun_out/c1_sched.log; exit 1; }
grep '^{' gpurun_out/c1_sched.log
