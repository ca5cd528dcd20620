"""Timeline of the last single evaluation in a rocprofv3 kernel trace, all queues: start / end offsets
(us from the evaluation's first dispatch), duration, queue, class, grid; then, per class, the busy sum and
the time during which only the panel chain runs (no update on the bulk queue).
usage: python tools/la_trace.py gpurun_out/x/run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "assemble_kernel" in r["Kernel_Name"]]
seq = rows[starts[-1]:]
t0 = int(seq[0]["Start_Timestamp"])


def klass(n):
    return ("diag2" if "diag2" in n else "trsm" if "gemm_kernel<double, 1" in n else
            "update" if "gemm_kernel" in n else n.split("(")[0].split("::")[-1][:24])


sums = defaultdict(float)
end = t0
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    end = max(end, e)
    k = klass(r["Kernel_Name"])
    sums[k] += (e - s) / 1e3
    print("%9.1f %9.1f %7.1f  q%-3s %-10s grid %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3,
                                                   r.get("Queue_Id", "?"), k, r.get("Grid_Size_X", r.get("Grid_Size", ""))))
print("span %.1f us" % ((end - t0) / 1e3))
for k, v in sorted(sums.items(), key=lambda kv: -kv[1]):
    print("  %-24s %9.1f us" % (k, v))
