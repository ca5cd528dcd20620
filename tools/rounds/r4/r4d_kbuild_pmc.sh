# K build of C5 (tools/bench_kbuild.py C5) under rocprofv3: kernel stats, then one PMC pass per counter group
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
KB=${KB:-gpurun_out/kb}; mkdir -p $KB
timeout -k 10 120 python tools/bench_kbuild.py C5 C3 SE8192 > $KB/kbuild.jsonl 2>&1 || exit 1
timeout -k 10 60 rocprofv3 -L > $KB/counters.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$KB/stats" -o run -- python tools/bench_kbuild.py C5 > $KB/stats.log 2>&1 || exit 1
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$ROOT/$KB/p$i" -o run -- python tools/bench_kbuild.py C5 > $KB/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc" >> $KB/passes.txt
  case $rc in 0) ;; *) exit $rc;; esac
done < tools/pmc_kbuild.txt
