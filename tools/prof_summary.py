"""Group a rocprofv3 --kernel-trace --stats run into libgpk's timing classes.

usage: python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv [steps]

Prints per class (assemble / diag / trsm / update / finalize / trsv) the launch count, total and
average duration, so the class averages can be checked against the HIP-event figures that
bench.py reports (roofline.avg_launch_us is the 'update' class average).
"""
import collections
import csv
import re
import sys


def klass(name):
    if "assemble_kernel" in name:
        return "assemble"
    if "diag_kernel" in name or "diag2_kernel" in name:
        return "diag"
    m = re.search(r"gemm_kernel<\w+, (\d)", name)
    if m:
        return "update" if m.group(1) == "0" else "trsm"
    if "finalize_kernel" in name:
        return "finalize"
    if "trsv" in name:
        return "trsv"
    return None


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
    calls = collections.Counter()
    total = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = klass(r["Name"])
        if k is None:
            continue
        calls[k] += int(r["Calls"])
        total[k] += float(r["TotalDurationNs"])
    print("%-9s %8s %14s %12s %s" % ("class", "calls", "total_ms", "avg_us", "ms/step" if steps else ""))
    for k in ("assemble", "diag", "trsm", "update", "finalize", "trsv"):
        if calls[k]:
            line = "%-9s %8d %14.3f %12.2f" % (k, calls[k], total[k] * 1e-6, total[k] * 1e-3 / calls[k])
            if steps:
                line += " %10.3f" % (total[k] * 1e-6 / steps)
            print(line)


if __name__ == "__main__":
    main()
