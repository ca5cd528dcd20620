# round 6: fresh per-step breakdown of the single-evaluation chain (N = 4096, 8192) and the D task's phase timeline
set -o pipefail
O=${O:-gpurun_out/r6m}; mkdir -p $O
for n in 4096 8192; do
  timeout -k 10 120 python tools/chain_prof.py $n > $O/prof_$n.log 2>&1 || { tail -5 $O/prof_$n.log; exit 1; }
  echo "== chain_prof $n"; grep -v "INFO\|amdgpu.ids" $O/prof_$n.log
done
GPK_LIB=variants/libgpk_dprof.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/phase.log 2>&1 || { tail -5 $O/phase.log; exit 1; }
echo "== diag_phase_prof 4096"; grep -v "INFO\|amdgpu.ids" $O/phase.log
exit 0
