# round 6: API latency after the identity-augmented block-row-solve threshold 64 (alternating box noise: two passes)
set -o pipefail
O=${O:-gpurun_out/r6z2}; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python tools/bench_api_latency.py 4096 6144 8192 > $O/api.log 2>&1 || exit 1
  grep '^{' $O/api.log
done
exit 0
