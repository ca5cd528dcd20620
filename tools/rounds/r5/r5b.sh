# round 5: full GPU suite + smoke + short bench (r5a), then A/B of the chain's hand-off loads:
# plain loads behind one agent acquire per task (default) vs sc1 loads without the acquire (GPK_CHAIN_SC1LD)
set -o pipefail
O=gpurun_out/r5b; mkdir -p $O
O=$O RUN_BENCH=1 bash tools/rounds/r5/r5a.sh || exit 1
GPK_LIB=variants/libgpk_sc1ld.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_chain.py -m gpu -k "bitwise or matches" > $O/tests_sc1ld.log 2>&1 || { tail -5 $O/tests_sc1ld.log; exit 1; }
tail -1 $O/tests_sc1ld.log
for v in "" sc1ld "" sc1ld; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  GPK_LIB=$L SETS='{"chain":1}' timeout -k 10 300 python tools/single_sched.py 1024 2048 4096 8192 >> $O/ab_${v:-base}.jsonl 2>&1 || exit 1
done
grep -h "^{" $O/ab_base.jsonl $O/ab_sc1ld.jsonl | cut -c1-160
timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof_base.txt 2>&1 || exit 1
GPK_LIB=variants/libgpk_sc1ld.so timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof_sc1ld.txt 2>&1 || exit 1
tail -1 $O/prof_base.txt; tail -1 $O/prof_sc1ld.txt
