"""Split the update launches of the last look-ahead-off step of a rocprofv3 trace into the group
(bulk, K = 128 G) launches and the in-group launches, with their achieved TF/s.

usage: python tools/update_split.py gpurun_out/prof/run_kernel_trace.csv N BATCH [G] [INGROUP] [depth]
INGROUP: 3 two-level left-looking (the default schedule for batches that fill the chip), 1 left-looking.
Flops per launch: 2 K x (lower-triangle elements of the updated columns over the K rows), from the launch
order of gpk_potrf_aug (gpk_abi.hip potrf_impl):
  left-looking (1): per group, before panel k > g0 one update of block column k with panels g0 .. k-1;
  two-level (3):    the group split at gmid = g0 + ceil(G / 2); each half left-looking within itself, and
                    before panel gmid ONE update of columns gmid .. gend-1 with panels g0 .. gmid-1 ("half");
then the group update of the trailing matrix with all G panels.  "depth" adds a per-depth table.
"""
import csv
import sys


def elems(n, row0, w):
    """lower-triangle elements of block columns [row0, row0 + 128 w) over rows [row0, n)"""
    ra, cb = n - row0, min(128 * w, n - row0)
    return cb * ra - (cb - 1.0) * cb / 2.0


def model(n, G, ingroup):
    nb = n // 128
    seq = []
    for g0 in range(0, nb, G):
        gend = min(g0 + G, nb)
        gmid = min(g0 + (gend - g0 + 1) // 2, gend) if ingroup == 3 else gend
        for k in range(g0, gend):
            h0 = g0 if k < gmid else gmid
            if ingroup == 3 and k == gmid and gmid > g0:
                d = gmid - g0
                seq.append(("half", 128 * d, 2.0 * 128 * d * elems(n, 128 * gmid, gend - gmid)))
            if k > h0:
                d = k - h0
                seq.append(("thin", 128 * d, 2.0 * 128 * d * elems(n, 128 * k, 1)))
        rows = n - 128 * gend
        seq.append(("group", 128 * (gend - g0), 2.0 * 128 * (gend - g0) * rows * (rows + 1) / 2))
    return seq


def main():
    path, n, batch = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    G = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    ingroup = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    starts = [i for i, r in enumerate(rows) if "assemble_kernel" in r[2]]
    step = rows[starts[-1]:]
    upd = [(s, e) for s, e, k in step if "gemm_kernel<double, 0" in k or "gemm_kernel<float, 0" in k]
    seq = model(n, G, ingroup)
    if len(seq) != len(upd):
        print("launch count mismatch: trace %d, model %d" % (len(upd), len(seq)))
    tot = {}
    bydepth = {}
    for (s, e), (kind, depth, fl) in zip(upd, seq):
        fl *= batch
        t = tot.setdefault(kind, [0.0, 0.0, 0])
        t[0] += (e - s) * 1e-9
        t[1] += fl
        t[2] += 1
        if kind != "group":
            b = bydepth.setdefault((kind, depth), [0.0, 0.0, 0])
            b[0] += (e - s) * 1e-9
            b[1] += fl
            b[2] += 1
    for kind, (sec, fl, cnt) in tot.items():
        print("%-5s %3d launches  %.3f ms  %.1f TF/s" % (kind, cnt, sec * 1e3, fl / max(sec, 1e-12) / 1e12))
    big = [(e - s, fl * batch) for (s, e), (kind, _, fl) in zip(upd, seq) if kind == "group"]
    for dt, fl in big[:4] + big[-3:]:
        print("   group launch %.1f us  %.1f TF/s" % (dt / 1e3, fl / max(dt * 1e-9, 1e-12) / 1e12))
    if "depth" in sys.argv[6:]:
        for (kind, depth), (sec, fl, cnt) in sorted(bydepth.items()):
            print("   %-4s depth %4d: %2d launches, avg %6.1f us, %.1f TF/s"
                  % (kind, depth, cnt, sec / cnt * 1e6, fl / sec / 1e12))


if __name__ == "__main__":
    main()
