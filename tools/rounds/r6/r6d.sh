# round 6: f32 K build without the edge list (C3 shape), its kernel stats; bench hardware queues 8 vs 16 on the
# metric, C2 and C2 --dist
set -o pipefail
O=${O:-gpurun_out/r6d}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kbuild.py tests/test_gpu_parity.py -m gpu -q \
  --timeout 240 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_kbuild.py C3 > $O/kb_c3.json 2> $O/kb.err || { tail -3 $O/kb.err; exit 1; }
tail -1 $O/kb_c3.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_kb -o kb -- python3 tools/bench_kbuild.py C3 > $O/prof_kb.log 2>&1 || { tail -5 $O/prof_kb.log; exit 1; }
find $O/prof_kb -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -6 {} | cut -c1-200'
for q in 8 16; do
  GPK_BENCH_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check > $O/metric_q$q.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  GPK_BENCH_HW_QUEUES=$q timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 --no-cpu-baseline --no-check > $O/c2_q$q.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  GPK_BENCH_HW_QUEUES=$q timeout -k 10 300 python bench.py --config C2 --dist --steps 200 --warmup 20 --no-cpu-baseline --no-check > $O/c2d_q$q.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
  echo "q$q metric $(python -c "import json;print(json.loads(open('$O/metric_q$q.json').read().splitlines()[-1])['value'])") C2 $(python -c "import json;print(json.loads(open('$O/c2_q$q.json').read().splitlines()[-1])['value'])") C2dist $(python -c "import json;print(json.loads(open('$O/c2d_q$q.json').read().splitlines()[-1])['value'])")"
done
exit 0
