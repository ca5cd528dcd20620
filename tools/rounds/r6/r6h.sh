# round 6: the f32 persistent factorisation (chain_kernel<float>) -- its GPU tests, then C3 on it against the launch path
set -o pipefail
O=${O:-gpurun_out/r6h}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain_f32.py -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -c PASSED $O/tests.log; tail -2 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config C3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3_chain_$rep.json 2> $O/c3_chain_$rep.err || { tail -5 $O/c3_chain_$rep.err; exit 1; }
  timeout -k 10 300 python bench.py --config C3 --steps 40 --warmup 5 --no-cpu-baseline --chain 0 > $O/c3_launch_$rep.json 2> $O/c3_launch_$rep.err || { tail -5 $O/c3_launch_$rep.err; exit 1; }
  python - $O/c3_chain_$rep.json $O/c3_launch_$rep.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d.get("roofline", {}).get("frac"))
PY
done
for pp in "4 4" "6 4" "8 3" "6 3" "4 2"; do
  set -- $pp
  GPK_BENCH_PERSIST_P=$1 GPK_BENCH_PERSIST_SHARE=$2 timeout -k 10 300 python bench.py --config C3 --steps 40 --warmup 5 --no-cpu-baseline > $O/c3_p$1_s$2.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  echo "P=$1 share=1/$2 $(python -c "import json;d=json.loads(open('$O/c3_p$1_s$2.json').read().strip().splitlines()[-1]);print(d['value'])")"
done
exit 0
