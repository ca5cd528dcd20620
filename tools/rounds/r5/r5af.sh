# round 5: C5 (N = 16384) as persistent launches side by side (chain_max_p raised for the experiment)
set -o pipefail
O=gpurun_out/r5af; mkdir -p $O; : > $O/c5.txt
for pg in "4 64" "8 32" "6 64" "4 128"; do
  set -- $pg
  GPK_CHAIN_MAX_P=16640 GPK_CHAIN_GRID=$2 timeout -k 10 300 python bench.py --config C5 --pipeline $1 --chain 2 --steps 24 --warmup 8 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -3 $O/c5.log; exit 1; }
  echo "P=$1 grid=$2 $(grep '^{' $O/c5.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["check"]["rel_vs_oracle"])')" | tee -a $O/c5.txt
done
