"""Per-call GPU picture of the drop-in API at small N from a rocprofv3 kernel trace of tools/api_profile.py (its
timed loop of `calls` get_metric calls): kernels per call, summed kernel time, device span and the gaps between
dependent kernels.  usage: python tools/api_trace_summary.py TRACE.csv CALLS"""
import csv
import re
import statistics
import sys
from collections import Counter


def main(path, calls):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    # the last 2 * calls calls' worth of kernels: the script's timed loop and its profiled loop
    ks = [(s, e, re.sub(r"\(anonymous namespace\)::", "", n).split("(")[0][:70]) for s, e, n in ks]
    per_call = len(ks) / (2 * calls + 20)
    tail = ks[-int(per_call * calls):]
    busy = sum(e - s for s, e, _ in tail) / calls / 1e3
    gaps = [tail[i + 1][0] - tail[i][1] for i in range(len(tail) - 1)]
    print("kernels %d, ~%.1f per call; per call: kernel time %.1f us, span %.1f us; median gap %.2f us" %
          (len(ks), per_call, busy, (tail[-1][1] - tail[0][0]) / calls / 1e3, statistics.median(gaps) / 1e3))
    durs = Counter()
    cnt = Counter()
    for s, e, n in tail:
        durs[n] += (e - s) / 1e3
        cnt[n] += 1
    for n, d in durs.most_common(12):
        print("  %-70s %6d  %8.2f us per call  %6.2f us avg" % (n, cnt[n], d / calls, d / cnt[n]))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
