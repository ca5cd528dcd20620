"""Per-kernel-family sums of rocprofv3 --pmc counters from a counter_collection.csv:
python tools/pmc_kernel_ratio.py <csv>  -> SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS per family."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    fam = ("diag2" if "diag2" in name else "trsm" if "gemm_kernel<double, 1" in name else
           "update" if "gemm_kernel" in name else name.split("(")[0].split("::")[-1][:28])
    acc[fam][r["Counter_Name"]] += float(r["Counter_Value"])
for fam, c in sorted(acc.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
    lds = c.get("SQ_INSTS_LDS", 0)
    conf = c.get("SQ_LDS_BANK_CONFLICT", 0)
    print("%-30s LDS insts %12.0f  bank-conflict cycles %12.0f  per LDS inst %.3f" % (fam, lds, conf, conf / lds if lds else 0))
