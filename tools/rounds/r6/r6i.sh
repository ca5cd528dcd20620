# round 6: where the f32 persistent launch spends its time (tools/chain_util.py) against the f64 one, full grid and 64
set -o pipefail
O=${O:-gpurun_out/r6i}; mkdir -p $O
for a in "8192" "8192 f32" "8192 grid=64" "8192 f32 grid=64" "4096 f32"; do
  echo "== $a"
  timeout -k 10 120 python tools/chain_util.py $a > $O/u.log 2>&1 || { tail -5 $O/u.log; exit 1; }
  grep -v "INFO\|amdgpu.ids" $O/u.log
done
exit 0
