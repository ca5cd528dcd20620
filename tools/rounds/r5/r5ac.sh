# round 5: C2 persistent side by side -- larger CU shares at 8 in flight, 7 in flight
set -o pipefail
O=gpurun_out/${OUTD:-r5ac}; mkdir -p $O; : > $O/c2.txt
for pg in ${PGS:-"8 64" "8 48" "8 64" "8 96" "8 128" "6 64" "8 64"}; do
  set -- $pg
  GPK_CHAIN_GRID=$2 timeout -k 10 200 python bench.py --config C2 --pipeline $1 --chain 2 --steps 300 --warmup 30 --no-cpu-baseline --no-check > $O/c2.log 2>&1 || { tail -3 $O/c2.log; exit 1; }
  echo "P=$1 grid=$2 $(grep '^{' $O/c2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/c2.txt
done
