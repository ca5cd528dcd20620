# round 6: single-evaluation knobs at N = 4096 / 8192 under the new planner: chain_uq 0 / 1 / 2, near sub-groups off
set -o pipefail
O=${O:-gpurun_out/r6ab}; mkdir -p $O
for rep in 1 2; do
  for v in "1 2" "2 2" "0 2" "1 1"; do
    set -- $v
    GPK_CHAIN_UQ=$1 GPK_CHAIN_GROUP_NEAR=$2 timeout -k 10 300 python tools/bench_api_latency.py --no-grad 2048 4096 8192 > $O/api.log 2>&1 || exit 1
    echo "rep $rep uq=$1 near=$2: $(grep '^{' $O/api.log | python -c "
import json,sys
print(' '.join('%d: %.3f' % (d['n'], d['get_metric_ms']) for d in map(json.loads, sys.stdin)))")"
  done
done
exit 0
