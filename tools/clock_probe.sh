#!/bin/bash
# Effective shader clock under the bench load: rocm-smi's current clocks sampled while a long
# bench.py run is in its timed region, plus a GRBM_GUI_ACTIVE PMC pass (busy cycles per update
# dispatch / its duration).  Read-only: nothing here changes a clock or power setting.
set -u
mkdir -p gpurun_out/clk
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 300 --warmup 3 --no-cpu-baseline --no-events > gpurun_out/clk/bench.log 2>&1 &
pid=$!
sleep 12
for i in 1 2 3 4 5; do rocm-smi -c > gpurun_out/clk/smi_$i.txt 2>&1; sleep 1; done
wait $pid
rc=$?
echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d "$(pwd)/gpurun_out/clk/pmc" -o run \
  -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-events --pipeline 1 --lookahead 0 > gpurun_out/clk/pmc.log 2>&1
echo "pmc rc=$?"
