# round 5: C3 (f32, one candidate per step) -- factorisations in flight and group knobs
set -o pipefail
O=gpurun_out/r5y; mkdir -p $O; : > $O/c3.txt
run() {
  env $2 timeout -k 10 200 python bench.py --config C3 --steps 80 --warmup 10 --no-cpu-baseline --no-check $3 > $O/c3.log 2>&1 || { tail -3 $O/c3.log; exit 1; }
  echo "$1 $(grep '^{' $O/c3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"])')" | tee -a $O/c3.txt
}
run base "X=1" ""
run p3 "X=1" "--pipeline 3"
run p5 "X=1" "--pipeline 5"
run p6 "X=1" "--pipeline 6"
run p8 "X=1" "--pipeline 8"
run g16 "GPK_GROUP=16" ""
run g4 "GPK_GROUP=4" ""
run t128_256 "GPK_UPD_T128_MIN=256" ""
run t128_1024 "GPK_UPD_T128_MIN=1024" ""
run base2 "X=1" ""
