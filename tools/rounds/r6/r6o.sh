# round 6: PMC of the single-evaluation persistent launch (get_metric N = 4096): LDS bank conflicts per LDS instruction
# and MFMA busy of chain_kernel, one counter group per pass; plus chain_util at N = 4096 / 8192 (f64, f32)
set -o pipefail
O=${O:-gpurun_out/r6o}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d "$(pwd)/$O/p1" -o run -- python tools/bench_api_latency.py --no-grad 4096 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d "$(pwd)/$O/p2" -o run -- python tools/bench_api_latency.py --no-grad 4096 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python tools/pmc_kernel_ratio.py $(find $O/p1 -name "*counter_collection.csv" | head -1)
python - $(find $O/p2 -name "*counter_collection.csv" | head -1) <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(int)
for r in csv.DictReader(open(sys.argv[1])):
    fam = r["Kernel_Name"].split("(")[0].split("::")[-1][:28]
    acc[fam][r["Counter_Name"]] += float(r["Counter_Value"])
for fam, c in acc.items():
    g = c.get("GRBM_GUI_ACTIVE", 0)
    if g <= 0: continue
    busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    print("%-28s MFMA busy %.1f %% of (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); F64 MFMA MOPs %.3e" % (fam, 100 * busy / (1024 * g / 8), c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0)))
PY
for a in "4096" "4096 f32" "8192" "8192 f32"; do
  echo "== chain_util $a"
  timeout -k 10 120 python tools/chain_util.py $a > $O/u.log 2>&1 || { tail -5 $O/u.log; exit 1; }
  grep -v "INFO\|amdgpu.ids" $O/u.log
done
exit 0
