# round 6: two-list chain (chain_xcd) bitwise + A/B, f32 K build chunk sweep, C2 --dist at 8 queues, C4 W = 8 slice
# schedule sweep, value-path chain_group_la A/B
set -o pipefail
O=${O:-gpurun_out/r6c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_kbuild.py tests/test_gpu_grad.py -m gpu -q \
  --timeout 240 --timeout-method thread -rf > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/chain_xcd_ab.py 2048 4096 8192 > $O/chain_xcd_ab.jsonl 2> $O/chain_xcd_ab.err || { tail -3 $O/chain_xcd_ab.err; exit 1; }
cat $O/chain_xcd_ab.jsonl
for c in 1 2 4 8 16; do
  GPK_ASM_F32_CHUNK=$c timeout -k 10 120 python tools/bench_kbuild.py C3 > $O/kb_c3_chunk$c.json 2> $O/kb.err || { tail -3 $O/kb.err; exit 1; }
  echo "chunk $c $(tail -1 $O/kb_c3_chunk$c.json | cut -c1-200)"
done
for la in 2 1; do
  GPK_CHAIN_GROUP_LA=$la timeout -k 10 200 python tools/bench_api_latency.py --no-grad 4096 8192 > $O/api_la$la.jsonl 2> $O/api.err || { tail -3 $O/api.err; exit 1; }
  echo "la $la $(cat $O/api_la$la.jsonl | tr '\n' ' ')"
done
timeout -k 10 300 python bench.py --config C2 --dist --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_c2_dist8.json 2> $O/bench_c2_dist8.err || { tail -5 $O/bench_c2_dist8.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c2_dist8.json').read().strip().splitlines()[-1]); print('C2 dist hwq8', d['value'], d['check']['allgather_ok'])"
for P in 4 6 8; do
  GPK_BENCH_HW_QUEUES=16 timeout -k 10 200 python bench.py --config C4 --slice-of 8 --steps 60 --warmup 10 --pipeline $P --no-cpu-baseline --no-check > $O/c4_s8_p$P.json 2> $O/c4.err || { tail -3 $O/c4.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c4_s8_p$P.json').read().strip().splitlines()[-1]); print('C4 slice8 P$P', d['ms_per_step'], d['slice'])"
done
for ig in 1 2; do
  GPK_INGROUP=$ig timeout -k 10 200 python bench.py --config C4 --slice-of 8 --steps 60 --warmup 10 --no-cpu-baseline --no-check > $O/c4_s8_ig$ig.json 2> $O/c4.err || { tail -3 $O/c4.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/c4_s8_ig$ig.json').read().strip().splitlines()[-1]); print('C4 slice8 ingroup$ig', d['ms_per_step'])"
done
timeout -k 10 200 python bench.py --config C4 --steps 20 --warmup 3 --no-cpu-baseline --no-check > $O/c4_full.json 2> $O/c4.err || { tail -3 $O/c4.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c4_full.json').read().strip().splitlines()[-1]); print('C4 full', d['ms_per_step'])"
exit 0
