set -u
for rep in 1 2; do
for b in 32 48 64; do
  timeout -k 10 300 python bench.py --batch $b --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/bs.log 2>&1 || exit 1
  echo "batch $b: $(grep '^{' gpurun_out/bs.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["achieved"])')"
done
done
