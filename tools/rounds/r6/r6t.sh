# round 6: where the 64-workgroup launches spend their time now (C2 f64 N = 4096, C3 f32 N = 8192), and the bench's C3 line
set -o pipefail
O=${O:-gpurun_out/r6t}; mkdir -p $O
for a in "4096 grid=64" "8192 f32 grid=64" "8192 grid=64" "8192"; do
  echo "== chain_util $a"
  timeout -k 10 120 python tools/chain_util.py $a > $O/u.log 2>&1 || { tail -5 $O/u.log; exit 1; }
  grep -v "INFO\|amdgpu.ids" $O/u.log
done
timeout -k 10 300 python bench.py --config C3 --steps 60 --warmup 10 > $O/c3.json 2> $O/e.err || { tail -5 $O/e.err; exit 1; }
tail -1 $O/c3.json | cut -c1-400
exit 0
