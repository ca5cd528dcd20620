# C2 one candidate per step: persistent launches on a fraction of the CUs, several in flight
set -o pipefail
O=gpurun_out/r4ae; mkdir -p $O
for pg in "2 128" "3 85" "4 64" "2 0"; do
  set -- $pg
  GPK_CHAIN_GRID=$2 timeout -k 10 200 python bench.py --config C2 --pipeline $1 --chain 2 --steps 200 --warmup 20 --no-cpu-baseline --no-check > $O/c2_p$1_g$2.log 2>&1 || exit 1
  echo "P=$1 grid=$2 $(grep '^{' $O/c2_p$1_g$2.log | cut -c1-140)"
done
