# round 5: C5 (SE-ARD+PER D=8, N=16384 fp64, one candidate per step) schedule knobs
set -o pipefail
O=gpurun_out/r5x; mkdir -p $O; : > $O/c5.txt
run() {  # label, env, args
  env $2 timeout -k 10 200 python bench.py --config C5 --steps 24 --warmup 6 --no-cpu-baseline --no-check $3 > $O/c5.log 2>&1 || { tail -3 $O/c5.log; exit 1; }
  echo "$1 $(grep '^{' $O/c5.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')" | tee -a $O/c5.txt
}
run base "X=1" ""
run p3 "X=1" "--pipeline 3"
run p2 "X=1" "--pipeline 2"
run p6 "X=1" "--pipeline 6"
run g16 "GPK_GROUP=16" ""
run g4 "GPK_GROUP=4" ""
run gf4 "GPK_GROUP_FIRST=4" ""
run p1la2 "X=1" "--pipeline 1 --lookahead 2"
run base2 "X=1" ""
