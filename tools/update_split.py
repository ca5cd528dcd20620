"""Split the update launches of the last look-ahead-off step of a rocprofv3 trace into the group
(bulk, K = 128 G) launches and the thin (K = 128) in-group launches, with their achieved TF/s.

usage: python tools/update_split.py gpurun_out/prof/run_kernel_trace.csv N BATCH [G]
Flops per launch: 2 K x (lower-triangle elements of the updated 128-tiles) x batch, from the
launch order of gpk_potrf_aug (per group: G-1 left-looking thin updates between the G diag / trsm pairs, then the group update).
"""
import csv
import sys


def main():
    path, n, batch = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    G = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    starts = [i for i, r in enumerate(rows) if "assemble_kernel" in r[2]]
    step = rows[starts[-1]:]
    nb = n // 128
    upd = [(s, e) for s, e, k in step if "gemm_kernel<double, 0" in k or "gemm_kernel<float, 0" in k]
    seq = []
    for g0 in range(0, nb, G):
        gend = min(g0 + G, nb)
        for k in range(g0 + 1, gend):
            # left-looking: block column k with the group's panels g0 .. k-1 (depth 128 (k - g0))
            rows_ = (nb - k) * 128
            elems = sum(rows_ - r for r in range(128))
            seq.append(("thin", 2.0 * 128 * (k - g0) * elems * batch))
        rK = (nb - gend) * 128
        seq.append(("group", 2.0 * 128 * (gend - g0) * rK * (rK + 1) / 2 * batch))
    if len(seq) != len(upd):
        print("launch count mismatch: trace %d, model %d" % (len(upd), len(seq)))
    tot = {"thin": [0.0, 0.0, 0], "group": [0.0, 0.0, 0]}
    for (s, e), (kind, fl) in zip(upd, seq):
        t = tot[kind]
        t[0] += (e - s) * 1e-9
        t[1] += fl
        t[2] += 1
    for kind, (sec, fl, cnt) in tot.items():
        print("%-5s %3d launches  %.3f ms  %.1f TF/s" % (kind, cnt, sec * 1e3, fl / max(sec, 1e-12) / 1e12))
    big = [(e - s, fl) for (s, e), (kind, fl) in zip(upd, seq) if kind == "group"]
    for dt, fl in big[:6]:
        print("   group launch %.1f us  %.1f TF/s" % (dt / 1e3, fl / (dt * 1e-9) / 1e12))
    for dt, fl in big[-6:]:
        print("   group launch %.1f us  %.1f TF/s" % (dt / 1e3, fl / max(dt * 1e-9, 1e-12) / 1e12))


if __name__ == "__main__":
    main()


def thin_by_depth(path, n, batch, G):
    """Per-depth average rate of the thin (left-looking in-group) launches of the last step."""
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    starts = [i for i, r in enumerate(rows) if "assemble_kernel" in r[2]]
    step = rows[starts[-1]:]
    nb = n // 128
    upd = [(s, e) for s, e, k in step if "gemm_kernel<double, 0" in k or "gemm_kernel<float, 0" in k]
    i = 0
    acc = {}
    for g0 in range(0, nb, G):
        gend = min(g0 + G, nb)
        for k in range(g0 + 1, gend):
            rows_ = (nb - k) * 128
            elems = sum(rows_ - r for r in range(128))
            s, e = upd[i]
            d = k - g0
            a = acc.setdefault(d, [0.0, 0.0, 0])
            a[0] += (e - s) * 1e-9
            a[1] += 2.0 * 128 * d * elems * batch
            a[2] += 1
            i += 1
        i += 1
    for d in sorted(acc):
        sec, fl, cnt = acc[d]
        print("   thin depth %4d: %2d launches, avg %.1f us, %.1f TF/s" % (128 * d, cnt, sec / cnt * 1e6, fl / sec / 1e12))


if __name__ == "__main__" and len(sys.argv) > 5 and sys.argv[5] == "depth":
    thin_by_depth(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))
