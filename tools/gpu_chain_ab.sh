# A/B of the persistent factorisation: default build vs $VARLIB (GPU tests, per-task profile, span)
set -o pipefail
: "${VARLIB:?}"
for v in base var; do
  if [ $v = var ]; then export GPK_LIB=$VARLIB; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cab_${v}_tests.log 2>&1 || { tail -20 gpurun_out/cab_${v}_tests.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/cab_${v}_tests.log)"
  timeout -k 10 120 python tools/chain_prof.py 4096 > gpurun_out/cab_${v}_prof.log 2>&1 || { tail -5 gpurun_out/cab_${v}_prof.log; exit 1; }
  grep -v "^INFO\|amdgpu.ids\|ready / done\|k=5" gpurun_out/cab_${v}_prof.log
done
