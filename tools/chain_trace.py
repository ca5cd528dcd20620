"""Per-kernel sequence of the last single evaluation in a rocprofv3 kernel trace (one stream, no overlap):
name class, duration and the gap before each dispatch, plus per-class sums.
usage: python tools/chain_trace.py gpurun_out/x/run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "assemble_kernel" in r["Kernel_Name"]]
seq = rows[starts[-1]:]
t0 = int(seq[0]["Start_Timestamp"])
prev_end = t0
sums, gaps = defaultdict(float), 0.0
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"]
    k = ("diag2" if "diag2" in name else "trsm" if "gemm_kernel<double, 1" in name else
         "update" if "gemm_kernel" in name else name.split("(")[0].split("::")[-1][:30])
    g = max(0, s - prev_end) / 1e3
    gaps += g
    sums[k] += (e - s) / 1e3
    print("%-32s %8.1f us  gap %6.1f  grid %s" % (k, (e - s) / 1e3, g, r.get("Grid_Size", r.get("Grid_Size_X", ""))))
    prev_end = max(prev_end, e)
print("span %.1f us, gaps %.1f us" % ((prev_end - t0) / 1e3, gaps))
for k, v in sorted(sums.items(), key=lambda kv: -kv[1]):
    print("  %-30s %8.1f us" % (k, v))
