# round 5: C2 with concurrent persistent launches on CU fractions, now that run() no longer synchronises per launch
set -o pipefail
O=gpurun_out/r5u; mkdir -p $O; : > $O/c2.txt
for pg in "4 0 0" "4 64 2" "2 128 2" "3 85 2" "4 0 2" "8 32 2"; do
  set -- $pg
  GPK_CHAIN_GRID=$2 timeout -k 10 200 python bench.py --config C2 --pipeline $1 --chain $3 --steps 200 --warmup 20 --no-cpu-baseline --no-check > $O/c2_p$1_g$2_c$3.log 2>&1 || { tail -3 $O/c2_p$1_g$2_c$3.log; exit 1; }
  echo "P=$1 grid=$2 chain=$3 $(grep '^{' $O/c2_p$1_g$2_c$3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/c2.txt
done
