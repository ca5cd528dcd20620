# round 5: every BASELINE config on the final tree, each with roofline + cpu_baseline, the C4
# per-rank slices, rocprofv3 --stats of each config, the drop-in API latency.  -> gpurun_out/r5cfg/
set -o pipefail
O=gpurun_out/r5cfg; mkdir -p $O; : > $O/configs.jsonl
export TMPDIR=/tmp
for spec in "metric 10" "C2 100" "C3 60" "C4 20" "C5 20"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --steps $2 --warmup 3 --cpu-seconds 10 > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  grep '^{' $O/$1.log >> $O/configs.jsonl
  python - $1 <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/r5cfg/configs.jsonl")][-1])
r, c = d.get("roofline", {}), d.get("cpu_baseline", {})
print(sys.argv[1], d["value"], d["unit"], "roofline frac", r.get("frac"), "cpu", c.get("value"), "kbuild", d.get("kbuild_roofline"))
PY
done
timeout -k 10 300 python bench.py --config C2 --batch 1 --pipeline 1 --steps 100 --warmup 5 --no-cpu-baseline > $O/C2_single.log 2>&1 || exit 1
grep '^{' $O/C2_single.log >> $O/configs.jsonl
timeout -k 10 300 python bench.py --mode grad --steps 6 --warmup 2 --no-cpu-baseline > $O/grad.log 2>&1 || exit 1
grep '^{' $O/grad.log >> $O/configs.jsonl
OUT=$O/c4_slices.jsonl bash -c 'for W in 1 2 4 8; do timeout -k 10 240 python bench.py --config C4 --slice-of $W --steps 20 --warmup 3 --no-cpu-baseline --roofline-steps 1 > gpurun_out/r5cfg/c4_slice_$W.log 2>&1 || exit 1; grep "^{" gpurun_out/r5cfg/c4_slice_$W.log >> $OUT; done' || exit 1
timeout -k 10 300 python tools/bench_api_latency.py > $O/api.log 2>&1 || exit 1
for c in metric C2 C3 C4 C5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/prof_$c" -o run -- python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-check > $O/prof_$c.log 2>&1 || exit 1
done
echo done
