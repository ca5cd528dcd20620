# round 6: value + gradient at N = 4096 / 8192 under forced block-row updates / solves (the auto rule keeps slices at 4096)
set -o pipefail
O=${O:-gpurun_out/r6aa}; mkdir -p $O
for rep in 1 2; do
  for v in "2 2" "1 0" "1 1" "0 0"; do
    set -- $v
    GPK_CHAIN_U128=$1 GPK_CHAIN_S128=$2 timeout -k 10 300 python tools/bench_api_latency.py 4096 8192 > $O/api.log 2>&1 || exit 1
    echo "rep $rep u128=$1 s128=$2: $(grep '^{' $O/api.log | python -c "
import json,sys
print(' '.join('%d: %.3f / %.3f' % (d['n'], d['get_metric_ms'], d['get_metric_and_gradient_ms']) for d in map(json.loads, sys.stdin)))")"
  done
done
exit 0
