# round 5 last tree: C5 K build PMC passes (tools/pmc_kbuild.txt, as r5q.sh) and rocprofv3 stats, chunked fast kernel
set -o pipefail
O=gpurun_out/r5ax; mkdir -p $O
export TMPDIR=/tmp
KB=$O/pmc; mkdir -p $KB; i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  [ $i -eq 3 ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$(pwd)/$KB/p$i" -o run -- python tools/bench_kbuild.py C5 > $KB/p$i.log 2>&1 || exit 1
done < tools/pmc_kbuild.txt
python tools/pmc_kbuild_summary.py $KB 16384 8 > $KB/summary.txt 2>&1; cat $KB/summary.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$(pwd)/$O/stats" -o run -- python tools/bench_kbuild.py C5 > $O/stats.log 2>&1 || exit 1
f=$(ls $O/stats/*kernel_stats.csv $O/stats/*/*kernel_stats.csv 2>/dev/null | head -1); grep -h "pair_\|assemble" "$f" | cut -c1-200
