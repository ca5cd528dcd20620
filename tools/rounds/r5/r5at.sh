# round 5: host-side HIP API time of one small-N get_metric (rocprofv3 --hip-trace), N = 256
set -o pipefail
O=gpurun_out/r5at; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --hip-trace --output-format csv -d "$(pwd)/$O/n256" -o run -- python tools/api_profile.py 256 200 > $O/n256.log 2>&1 || { tail -3 $O/n256.log; exit 1; }
grep "us per call" $O/n256.log
f=$(ls $O/n256/*hip_api_trace.csv $O/n256/*/*hip_api_trace.csv 2>/dev/null | head -1)
python tools/hip_api_summary.py "$f" 200 | tee $O/summary.txt
