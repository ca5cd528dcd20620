"""Summary of tools/rounds/r4/r4d_kbuild_pmc.sh (rocprofv3 PMC passes over tools/bench_kbuild.py C5): per assemble_kernel
dispatch, the VALU / SALU / LDS instruction counts per matrix element, the VALU issue utilisation, and HBM bytes
(2 x FETCH_SIZE + WRITE_SIZE, gfx950 FETCH correction) against the algorithmic bytes and 8 TB/s.

The K build of the C5 tree is three launches since round 5 (pair_feat_kernel, pair_fast_kernel, the leftover
assemble_kernel): the counters are summed over every K-build kernel of one build (dispatches grouped per launch of
the build), and the duration is the sum of their median durations.

usage: python tools/pmc_kbuild_summary.py [dir] [n] [d] [element bytes: 8, or 4 for C3's f32 build]"""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kb"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
d = int(sys.argv[3]) if len(sys.argv) > 3 else 8
es = int(sys.argv[4]) if len(sys.argv) > 4 else 8
p = -(-(n + 1) // 128) * 128          # augmented rows (m = 0)
ntile = p // 64
elements = ntile * (ntile + 1) // 2 * 64 * 64
alg_bytes = es * p * (p + 64) / 2 + 8 * n * d
tot = collections.defaultdict(float)
cnt = collections.Counter()
dur = []
KB = ("assemble_kernel", "pair_fast_kernel", "pair_feat_kernel", "f32_fast_kernel")


def fam(name):
    return next((k for k in KB if k in name), None)


for f in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        k = fam(r["Kernel_Name"])
        if k:
            key = (k, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for (k, _), dd in per.items():
        for c, v in dd.items():
            tot[(k, c)] += v
            cnt[(k, c)] += 1
durs = collections.defaultdict(list)
for f in sorted(glob.glob(root + "/p*/run_kernel_trace.csv"))[:1]:
    for r in csv.DictReader(open(f)):
        k = fam(r["Kernel_Name"])
        if k:
            durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
med = {k: sorted(v)[len(v) // 2] for k, v in durs.items()}
for k in KB:
    if k in med:
        print("  %-17s median %.1f us over %d dispatches" % (k, med[k], len(durs[k])))
avg = collections.defaultdict(float)
for (k, c), v in tot.items():
    avg[c] += v / cnt[(k, c)]        # per build: the sum over its kernels of each one's per-dispatch mean
dur = [d for v in durs.values() for d in v]
us = sum(med.values()) if med else float("nan")
we = elements / 64.0   # wave-elements (one element per lane)
print("K build (all its kernels), N = %d, D = %d: %.1f us (sum of medians), %.3g elements" % (n, d, us, elements))
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
    if k in avg:
        print("  %-14s %.4g per dispatch = %.1f per element (per lane)" % (k, avg[k], avg[k] / we))
if "GRBM_GUI_ACTIVE" in avg:
    clk = avg["GRBM_GUI_ACTIVE"] / 8 / (us * 1e-6) / 1e9
    print("  effective clock %.2f GHz (GRBM_GUI_ACTIVE / 8 XCDs / duration)" % clk)
    if "SQ_INSTS_VALU" in avg:
        per_simd = avg["SQ_INSTS_VALU"] / 1024
        cyc = avg["GRBM_GUI_ACTIVE"] / 8
        print("  VALU wave-instructions per SIMD per cycle %.3f (f64 VALU: 4 cycles each -> at most 0.25)" % (per_simd / cyc))
    if "SQ_ACTIVE_INST_VALU" in avg:
        # SQ_ACTIVE_INST_VALU counts quad-cycles (one per wave64 VALU instruction issued: 3.26e8 against
        # SQ_INSTS_VALU 3.22e8 on C5); VALU busy = its cycles over the SIMD-cycles of the dispatch (256 CUs x 4 SIMDs)
        busy = avg["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * avg["GRBM_GUI_ACTIVE"] / 8)
        print("  VALU busy %.1f %% of the SIMD cycles (SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x cycles)): the kernel's "
              "roofline is the VALU issue rate" % (100 * busy))
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    hbm = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
    print("  HBM bytes (2 FETCH + WRITE) %.4g vs algorithmic %.4g (%.2fx); %.0f GB/s = %.1f %% of 8 TB/s" % (
        hbm, alg_bytes, hbm / alg_bytes, hbm / (us * 1e-6) / 1e9, 100 * hbm / (us * 1e-6) / 8e12))
