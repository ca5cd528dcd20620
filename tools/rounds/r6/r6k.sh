# round 6: f32 persistent launch with the f32 BLK DMA at the top of the chunk and 8-panel deferred updates
set -o pipefail
O=${O:-gpurun_out/r6k}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain_f32.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --config C3 --warmup 5 --no-cpu-baseline "$@" > $O/$tag.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
  echo "$tag $(python -c "import json;d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'])")"
}
run chain_p8_1 --steps 40
run launch_p4_1 --steps 40 --chain 0
run chain_p8_2 --steps 40
run launch_p4_2 --steps 40 --chain 0
run chain_p1 --steps 20 --pipeline 1
run launch_p1 --steps 20 --pipeline 1 --chain 0
timeout -k 10 120 python tools/chain_util.py 8192 f32 grid=64 > $O/u.log 2>&1 && grep -v "INFO\|amdgpu.ids" $O/u.log
timeout -k 10 120 python tools/chain_util.py 8192 f32 > $O/u2.log 2>&1 && grep -v "INFO\|amdgpu.ids" $O/u2.log
exit 0
