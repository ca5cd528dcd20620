# round 6: r6a (the touched GPU tests + C2 bench) plus the XCD hand-off probe, the identity-augmented planner
# knob sweep (value + gradient, N = 8192) and the C2 --dist rehearsal with 16 hardware queues
set -o pipefail
O=${O:-gpurun_out/r6b}; mkdir -p $O
timeout -k 10 60 tools/probe/xcd_handoff_probe > $O/xcd_probe.txt 2>&1 || { tail -5 $O/xcd_probe.txt; exit 1; }
cat $O/xcd_probe.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_syevd.py tests/test_gpu_nystroem_indefinite.py \
  tests/test_gpu_approx_metrics.py tests/test_gpu_strategies.py tests/test_gpu_kbuild.py tests/test_gpu_parity.py -m gpu -v --timeout 240 --timeout-method thread -rf -s \
  > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error|m = 16400|n = 16400|duplicate" $O/tests.log | tail -30
[ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] && exit $rc
timeout -k 10 300 python bench.py --config C3 --steps 100 --warmup 10 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c3.json').read().strip().splitlines()[-1]); print('C3', d['value'], d['kbuild_roofline'], d['check']['rel_vs_oracle'])"
GPK_BENCH_HW_QUEUES=16 timeout -k 10 300 python bench.py --config C3 --steps 100 --warmup 10 --pipeline 2 --lookahead 1 --la-per-stream --no-cpu-baseline > $O/bench_c3_la2.json 2> $O/bench_c3_la2.err || { tail -5 $O/bench_c3_la2.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c3_la2.json').read().strip().splitlines()[-1]); print('C3 P2 la per-stream', d['value'], d['check']['rel_vs_oracle'])"
GPK_BENCH_HW_QUEUES=16 timeout -k 10 300 python bench.py --config C3 --steps 100 --warmup 10 --pipeline 3 --lookahead 1 --la-per-stream --no-cpu-baseline > $O/bench_c3_la3.json 2> $O/bench_c3_la3.err || { tail -5 $O/bench_c3_la3.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c3_la3.json').read().strip().splitlines()[-1]); print('C3 P3 la per-stream', d['value'], d['check']['rel_vs_oracle'])"
timeout -k 10 300 python bench.py --config C2 --steps 200 --warmup 20 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print('C2', d['value'], d['check'])"
GPK_BENCH_HW_QUEUES=16 timeout -k 10 300 python bench.py --config C2 --dist --steps 200 --warmup 20 > $O/bench_c2_dist16.json 2> $O/bench_c2_dist16.err || { tail -5 $O/bench_c2_dist16.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c2_dist16.json').read().strip().splitlines()[-1]); print('C2 dist hwq16', d['value'], d['check'])"
timeout -k 10 400 python tools/grad_knob_sweep.py 8192 > $O/grad_sweep_8192.jsonl 2> $O/grad_sweep.err || { tail -5 $O/grad_sweep.err; exit 1; }
python -c "
import json
rows=[json.loads(l) for l in open('$O/grad_sweep_8192.jsonl')]
rows.sort(key=lambda r: r['ms_median'])
for r in rows[:6]+[x for x in rows if x['chain_group']==0 and x['chain_group_corner']==16 and x['chain_corner_tail']==8 and x['chain_group_la']==2]: print(r)
print('max dev', max(r['max_rel_vs_first'] for r in rows))"
exit $rc
