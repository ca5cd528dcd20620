"""Host-side HIP API time per call of the drop-in API from a rocprofv3 --hip-trace CSV of tools/api_profile.py:
API name, calls per get_metric, summed microseconds per get_metric (the last `calls` get_metric's worth).
usage: python tools/hip_api_summary.py HIP_API_TRACE.csv CALLS"""
import csv
import sys
from collections import Counter


def main(path, calls):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the script's last two loops of `calls` get_metric each: from the (2 calls)-th last memset of info (one per
    # get_metric, gpk_nlml's first call) to the end
    ms = [i for i, r in enumerate(rows) if r["Function"] == "hipMemsetAsync"]
    tail = rows[ms[-2 * calls]:]
    calls *= 2
    t = Counter()
    c = Counter()
    for r in tail:
        t[r["Function"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c[r["Function"]] += 1
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
    print("span per get_metric %.1f us; HIP API time per get_metric %.1f us" % (span / calls, sum(t.values()) / calls))
    for f, v in t.most_common(20):
        print("  %-40s %6.2f calls  %8.2f us" % (f, c[f] / calls, v / calls))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
