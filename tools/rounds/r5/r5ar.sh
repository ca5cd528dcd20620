# round 5: what one small-N get_metric costs on the device (kernel count, kernel time, span, gaps), N = 256 / 1024
set -o pipefail
O=gpurun_out/r5ar; mkdir -p $O
export TMPDIR=/tmp
for n in 256 1024; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$(pwd)/$O/n$n" -o run -- python tools/api_profile.py $n 200 > $O/n$n.log 2>&1 || { tail -3 $O/n$n.log; exit 1; }
  grep "us per call" $O/n$n.log
  f=$(ls $O/n$n/*kernel_trace.csv $O/n$n/*/*kernel_trace.csv 2>/dev/null | head -1)
  python tools/api_trace_summary.py "$f" 200 | tee $O/summary_n$n.txt
done
