# round 6: persistent schedules (launches in flight x CU share) for C2 / C3 under the new planner
set -o pipefail
O=${O:-gpurun_out/r6y}; mkdir -p $O
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'])"; }
for rep in 1 2; do
  for ps in "8 4" "6 3" "10 5" "8 5" "12 6" "6 4"; do
    set -- $ps
    GPK_BENCH_PERSIST_P=$1 GPK_BENCH_PERSIST_SHARE=$2 timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline > $O/c2.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    GPK_BENCH_PERSIST_P=$1 GPK_BENCH_PERSIST_SHARE=$2 timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/c3.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    echo "rep $rep P=$1 share=1/$2: C2 $(val $O/c2.json) C3 $(val $O/c3.json)"
  done
done
exit 0
