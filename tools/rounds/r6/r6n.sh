# round 6: the diagonal body's QR phase ended by an LDS counter among waves 1..7 (GPK_DIAG_QR_LDSBAR) -- tests, then
# chain_prof / get_metric against the barrier form (variants/libgpk_qrbar0.so), alternating, and the phase timeline
set -o pipefail
O=${O:-gpurun_out/r6n}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_chain_f32.py tests/test_gpu_diag_versions.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export GPK_LIB=variants/libgpk_qrbar0.so; else unset GPK_LIB; fi
    timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof_${v}_$rep.log 2>&1 || { tail -5 $O/prof_${v}_$rep.log; exit 1; }
    timeout -k 10 200 python tools/bench_api_latency.py 2048 4096 8192 > $O/api_${v}_$rep.jsonl 2>&1 || { tail -5 $O/api_${v}_$rep.jsonl; exit 1; }
    echo "$v rep $rep: $(grep 'mean over' $O/prof_${v}_$rep.log)"
    grep '^{' $O/api_${v}_$rep.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('   ', {k: d[k] for k in d if k in ('n','get_metric_ms','get_metric_and_gradient_ms','value_ms','grad_ms')} or d)"
  done
done
unset GPK_LIB
GPK_LIB=variants/libgpk_dprof.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/phase.log 2>&1 || { tail -5 $O/phase.log; exit 1; }
grep -v "INFO\|amdgpu.ids" $O/phase.log | head -12
exit 0
