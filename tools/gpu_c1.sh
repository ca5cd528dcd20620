# A/B of the persistent factorisation: default build vs $VARLIB (tests, per-task profile, single-evaluation span)
set -o pipefail
VARLIB=${VARLIB:-$PWD/gaussianprocessfundamentals_amd/libgpk_sc1ld.so}
for v in base var; do
  if [ $v = var ]; then export GPK_LIB=$VARLIB; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c_${v}_tests.log 2>&1 || { tail -20 gpurun_out/c_${v}_tests.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/c_${v}_tests.log)"
  timeout -k 10 120 python tools/chain_prof.py 4096 > gpurun_out/c_${v}_prof.log 2>&1 || { tail -5 gpurun_out/c_${v}_prof.log; exit 1; }
  grep -v "^INFO\|amdgpu.ids" gpurun_out/c_${v}_prof.log | head -7
  SETS='{"chain":0,"lookahead":0};{"chain":1}' timeout -k 10 200 python tools/single_sched.py 1024 2048 4096 > gpurun_out/c_${v}_sched.log 2>&1 || { tail -5 gpurun_out/c_${v}_sched.log; exit 1; }
  grep '^{' gpurun_out/c_${v}_sched.log
done
