# S prefetch on by default (tests), then the diagonal body's split accumulators / paired trailing tiles
# (historical A/B script of round 4: the variant libraries it names were built with tools/build_variant.sh and removed after the measurement -- see DESIGN §4 for the outcome)
set -o pipefail
O=gpurun_out/r4p; mkdir -p $O
true
true
for v in "" qrsplit trail2 qrsplit_t2 ""; do
  L=gaussianprocessfundamentals_amd/libgpk.so; [ -n "$v" ] && L=variants/libgpk_$v.so
  GPK_LIB=$L SETS='{"chain":1};{"chain":0,"lookahead":2}' timeout -k 10 300 python tools/single_sched.py 1024 4096 8192 >> $O/ab_${v:-base}.jsonl 2>&1 || exit 1
done
GPK_LIB=variants/libgpk_dprofqt.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/dphase_qt.txt 2>&1 || exit 1
GPK_LIB=variants/libgpk_dprof.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/dphase_base.txt 2>&1 || exit 1
timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof.txt 2>&1 || exit 1
