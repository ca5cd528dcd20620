# round 5: PMC of the C5 K build, MFMA pair path (GPK_ASM3_MINB=3) vs the VALU form
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
for v in asm3minb3 nopairmfma; do
  KB=gpurun_out/r5k_$v; mkdir -p $KB
  export GPK_LIB=variants/libgpk_$v.so
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    [ $i -gt 2 ] && [ $i -lt 4 ] && continue
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$ROOT/$KB/p$i" -o run -- python tools/bench_kbuild.py C5 > $KB/p$i.log 2>&1
    rc=$?; echo "$v pass $i rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done < tools/pmc_kbuild.txt
  python tools/pmc_kbuild_summary.py $KB 16384 8 > $KB/summary.txt 2>&1; cat $KB/summary.txt
done
