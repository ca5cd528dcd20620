# round 6: where the value + gradient call's time goes at N = 8192 (rocprofv3 kernel stats + trace)
set -o pipefail
O=${O:-gpurun_out/r6f}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o g -- python3 tools/grad_profile.py 8192 20 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep median $O/prof.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 $f | cut -c1-160
exit 0
