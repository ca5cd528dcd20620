# round 5: metric config -- candidates per step x batches in flight (memory: 64 x 2 = 71 GB of the 288 GB)
set -o pipefail
O=gpurun_out/r5aj; mkdir -p $O; : > $O/metric.txt
for bp in "64 2" "96 2" "128 2" "64 3" "80 2" "64 2"; do
  set -- $bp
  timeout -k 10 400 python bench.py --batch $1 --pipeline $2 --steps 12 --warmup 3 --no-cpu-baseline --no-check --no-events > $O/m.log 2>&1 || { tail -3 $O/m.log; exit 1; }
  echo "B=$1 P=$2 $(grep '^{' $O/m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/metric.txt
done
