# round 6 final tree, set C: PMC traffic of the trailing update (roofline.traffic), PMC of the C3 f32 K build, the
# value + gradient kernel stats, rocprofv3 stats of C2 / C3 / C5
set -o pipefail
T=${T:-r06fin}; O=gpurun_out/$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -m gpu -q --timeout 240 --timeout-method thread > $O/tests_chain.log 2>&1 || { tail -5 $O/tests_chain.log; exit 1; }
tail -1 $O/tests_chain.log
rm -rf gpurun_out/pmc
GPK_LOOKAHEAD=0 PMC_FILE=tools/pmc_traffic.txt bash tools/pmc_pass.sh || exit 1
python tools/pmc_traffic.py metric_b64 gpurun_out/pmc profiles/pmc_traffic.json || exit 1
cp profiles/pmc_traffic.json $O/pmc_traffic.json
KB=$O/pmc_kb_c3; mkdir -p $KB; i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  [ $i -eq 3 ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$(pwd)/$KB/p$i" -o run -- python tools/bench_kbuild.py C3 > $KB/p$i.log 2>&1 || exit 1
done < tools/pmc_kbuild.txt
python tools/pmc_kbuild_summary.py $KB 8192 4 4 > $O/kbuild_c3_pmc.txt 2>&1; cat $O/kbuild_c3_pmc.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/prof_grad" -o g -- python3 tools/grad_profile.py 8192 20 > $O/prof_grad.log 2>&1 || { tail -5 $O/prof_grad.log; exit 1; }
grep median $O/prof_grad.log
for c in C2 C3 C5; do
  st=$([ $c = C5 ] && echo 8 || echo 40)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/prof_$c" -o run -- python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline --no-check > $O/prof_$c.log 2>&1 || { tail -3 $O/prof_$c.log; exit 1; }
  grep '^{' $O/prof_$c.log | cut -c1-120
done
echo done
