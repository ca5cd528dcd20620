# round 6: C3 (8 f32 persistent launches) depth / near / look-ahead sweep under the full new planner
set -o pipefail
O=${O:-gpurun_out/r6ac}; mkdir -p $O
val() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['value'])"; }
for rep in 1 2; do
  for v in "0 2 2" "0 2 1" "12 4 2" "16 4 2" "0 4 2" "16 4 1"; do
    set -- $v
    GPK_CHAIN_GROUP=$1 GPK_CHAIN_GROUP_NEAR=$2 GPK_CHAIN_GROUP_LA=$3 timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 --no-cpu-baseline > $O/c3.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
    echo "rep $rep group=$1 near=$2 la=$3: C3 $(val $O/c3.json)"
  done
done
exit 0
