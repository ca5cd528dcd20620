# K build of C5 (tools/bench_kbuild.py C5) under rocprofv3: kernel stats, then one PMC pass per counter group
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
mkdir -p gpurun_out/kb
timeout -k 10 120 python tools/bench_kbuild.py C5 C3 SE8192 > gpurun_out/kb/kbuild.jsonl 2>&1 || exit 1
timeout -k 10 60 rocprofv3 -L > gpurun_out/kb/counters.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/kb/stats" -o run -- python tools/bench_kbuild.py C5 > gpurun_out/kb/stats.log 2>&1 || exit 1
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$ROOT/gpurun_out/kb/p$i" -o run -- python tools/bench_kbuild.py C5 > gpurun_out/kb/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc" >> gpurun_out/kb/passes.txt
  case $rc in 0) ;; *) exit $rc;; esac
done < tools/pmc_kbuild.txt
