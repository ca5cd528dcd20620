# round 6: chain_util of the value + gradient launch (N = 8192, identity rows) and of the single evaluation (4096, 8192)
set -o pipefail
O=${O:-gpurun_out/r6w}; mkdir -p $O
for a in "8192 eye" "4096 eye" "4096"; do
  echo "== chain_util $a"
  timeout -k 10 120 python tools/chain_util.py $a > $O/u.log 2>&1 || { tail -5 $O/u.log; exit 1; }
  grep -v "INFO\|amdgpu.ids" $O/u.log
done
exit 0
