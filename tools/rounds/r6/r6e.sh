# round 6: schedules with 16 hardware queues -- C2 persistent launches in flight x CU share, C3 / C5 pipelines;
# C3 K build kernel stats; API latency with the eye plans' 8-panel groups
set -o pipefail
O=${O:-gpurun_out/r6e}; mkdir -p $O
v() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(d['value'])" $1; }
for ps in "8 4" "12 4" "12 6" "16 4" "16 8"; do set -- $ps
  GPK_BENCH_PERSIST_P=$1 GPK_BENCH_PERSIST_SHARE=$2 timeout -k 10 200 python bench.py --config C2 --steps 300 --warmup 20 --no-cpu-baseline --no-check > $O/c2_p$1_s$2.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "C2 P$1 share1/$2 $(v $O/c2_p$1_s$2.json)"
done
for P in 4 6 8; do
  timeout -k 10 200 python bench.py --config C3 --steps 100 --warmup 10 --pipeline $P --no-cpu-baseline --no-check > $O/c3_p$P.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "C3 P$P $(v $O/c3_p$P.json)"
done
for P in 3 4 6; do
  timeout -k 10 200 python bench.py --config C5 --steps 12 --warmup 3 --pipeline $P --no-cpu-baseline --no-check > $O/c5_p$P.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "C5 P$P $(v $O/c5_p$P.json)"
done
timeout -k 10 200 python tools/bench_api_latency.py 2048 4096 8192 > $O/api.jsonl 2> $O/api.err || { tail -3 $O/api.err; exit 1; }
cat $O/api.jsonl
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kb -o kb -- python3 tools/bench_kbuild.py C3 > $O/prof_kb.log 2>&1 || { tail -5 $O/prof_kb.log; exit 1; }
f=$(find $O/prof_kb -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -5 $f | cut -c1-180
exit 0
