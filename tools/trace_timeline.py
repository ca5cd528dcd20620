"""Timeline of one factorisation step from a rocprofv3 kernel trace.

usage: python tools/trace_timeline.py gpurun_out/prof/run_kernel_trace.csv [step_index_from_end]

Steps are delimited by assemble_kernel dispatches.  Prints, for the chosen step, its wall span,
the busy time of the bulk-update kernels, the time during which no update kernel runs (the
critical-path exposure of the panel chain) and the per-class sums, to show where the step time goes
beyond the trailing update.
"""
import csv
import sys


def klass(name):
    if "assemble_kernel" in name:
        return "assemble"
    if "diag_kernel" in name or "diag2_kernel" in name:
        return "diag"
    if "gemm_kernel<double, 1" in name or "gemm_kernel<float, 1" in name:
        return "trsm"
    if "gemm_kernel" in name:
        return "update"
    if "finalize" in name:
        return "finalize"
    return "other"


def union(intervals):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(intervals):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    path = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows = []
    meta = {}
    for r in csv.DictReader(open(path)):
        key = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), klass(r["Kernel_Name"]))
        rows.append(key)
        meta[key] = (r["Queue_Id"], r["Grid_Size_X"], r["Grid_Size_Y"])
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2] == "assemble"]
    i0 = starts[-back]
    i1 = starts[-back + 1] if back > 1 else len(rows)
    step = rows[i0:i1]
    t0 = step[0][0]
    t1 = max(r[1] for r in step)
    span = t1 - t0
    print("step span %.3f ms, %d kernels" % (span / 1e6, len(step)))
    for c in ("assemble", "diag", "trsm", "update", "finalize"):
        iv = [(s, e) for s, e, k in step if k == c]
        print("  %-9s n=%4d  sum %.3f ms  union %.3f ms" % (c, len(iv), sum(e - s for s, e in iv) / 1e6,
                                                           union(iv) / 1e6))
    upd = union([(s, e) for s, e, k in step if k == "update"])
    anyk = union([(s, e) for s, e, k in step])
    print("  no update running: %.3f ms; no kernel at all: %.3f ms" % ((span - upd) / 1e6, (span - anyk) / 1e6))
    # exposure in windows of the step (where the chain is critical)
    nwin = 8
    for w in range(nwin):
        a, b = t0 + span * w // nwin, t0 + span * (w + 1) // nwin
        clip = [(max(s, a), min(e, b)) for s, e, k in step if k == "update" and e > a and s < b]
        print("  window %d: update busy %.0f%%" % (w, 100.0 * union(clip) / (b - a)))
    if len(sys.argv) > 3:
        # kernel sequence of the last N kernels of the step: queue, class, start offset, duration, grid
        nlast = int(sys.argv[3])
        for s_, e_, k_ in sorted(step)[-nlast:]:
            q, gx, gy = meta[(s_, e_, k_)]
            print("    q%-3s %-9s +%9.1f us  %7.1f us  grid %s x %s" % (q, k_, (s_ - t0) / 1e3, (e_ - s_) / 1e3, gx, gy))


if __name__ == "__main__":
    main()
