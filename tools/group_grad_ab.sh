set -u
for g in 8 4 8 4; do
  GPK_GROUP=$g GPK_GROUP_FIRST=$g timeout -k 10 200 python bench.py --mode grad --batch 8 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/gb.log 2>&1 || exit 1
  echo "group=$g grad b8: $(grep '^{' gpurun_out/gb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["achieved"])')"
done
bash tools/group_ab.sh "8 4" "4096 1 4"
