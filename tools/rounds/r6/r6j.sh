# round 6: C3 on the f32 persistent launch -- deferred-update depth and schedule sweep (bench.py, one candidate per step)
set -o pipefail
O=${O:-gpurun_out/r6j}; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config C3 --steps 40 --warmup 5 --no-cpu-baseline > $O/$tag.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  echo "$tag $(python -c "import json;d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['frac'])")"
}
run g8_p8s4 GPK_CHAIN_GROUP=8
run g16_p8s4 GPK_CHAIN_GROUP=16
run g12_p8s4 GPK_CHAIN_GROUP=12
run g16_p6s3 GPK_CHAIN_GROUP=16 GPK_BENCH_PERSIST_P=6 GPK_BENCH_PERSIST_SHARE=3
run g16_p4s2 GPK_CHAIN_GROUP=16 GPK_BENCH_PERSIST_P=4 GPK_BENCH_PERSIST_SHARE=2
run g16_p12s6 GPK_CHAIN_GROUP=16 GPK_BENCH_PERSIST_P=12 GPK_BENCH_PERSIST_SHARE=6
run g16_la1 GPK_CHAIN_GROUP=16 GPK_CHAIN_GROUP_LA=1
run launch GPK_CHAIN_F32=0
exit 0
