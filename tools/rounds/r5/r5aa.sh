# round 5: C4 (128-candidate sweep, N = 4096) -- sweeps in flight and group knobs
set -o pipefail
O=gpurun_out/r5aa; mkdir -p $O; : > $O/c4.txt
run() {
  env $2 timeout -k 10 200 python bench.py --config C4 --steps 20 --warmup 4 --no-cpu-baseline --no-check $3 > $O/c4.log 2>&1 || { tail -3 $O/c4.log; exit 1; }
  echo "$1 $(grep '^{' $O/c4.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')" | tee -a $O/c4.txt
}
run base "X=1" ""
run p2 "X=1" "--pipeline 2"
run p3 "X=1" "--pipeline 3"
run p6 "X=1" "--pipeline 6"
run g4 "GPK_GROUP=4" ""
run g16 "GPK_GROUP=16" ""
run ing3 "GPK_INGROUP=3" ""
run base2 "X=1" ""
