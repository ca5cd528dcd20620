"""Summarise rocprofv3 PMC passes (gpurun_out/pmc/p*/run_counter_collection.csv) per kernel.

Prints, per kernel family, the mean over dispatches of each counter, plus derived figures:
MFMA busy fraction, HBM bytes (FETCH_SIZE doubled per the gfx950 guide + WRITE_SIZE, in KiB
units x 1024) and bytes per dispatch.
"""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"


def family(name):
    name = name.replace("void gpk::(anonymous namespace)::", "")
    return re.sub(r"\([^()]*\)$", "", name)


data = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(root + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        fam = family(r["Kernel_Name"])
        data[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] in ("GRBM_GUI_ACTIVE", "FETCH_SIZE"):
            dur[fam].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)

for fam, ctrs in sorted(data.items()):
    if "gpk" not in fam and "kernel" not in fam:
        continue
    print("== %s  (dispatches %d)" % (fam, max(len(v) for v in ctrs.values())))
    mean = {k: sum(v) / len(v) for k, v in ctrs.items()}
    for k in sorted(mean):
        print("   %-30s %.4g" % (k, mean[k]))
    if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "GRBM_GUI_ACTIVE" in mean:
        # MFMA busy is summed over SIMDs (1024); GRBM_GUI_ACTIVE over XCDs (8)
        gui = mean["GRBM_GUI_ACTIVE"] / 8.0
        print("   -> MFMA busy fraction      %.3f" % (mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * 1024.0)))
    if "FETCH_SIZE" in mean:
        print("   -> HBM read  (2 x FETCH)   %.1f MB/dispatch" % (2 * mean["FETCH_SIZE"] * 1024 / 1e6))
    if "WRITE_SIZE" in mean:
        print("   -> HBM write               %.1f MB/dispatch" % (mean["WRITE_SIZE"] * 1024 / 1e6))
    if "TCC_HIT_sum" in mean:
        h, m = mean["TCC_HIT_sum"], mean.get("TCC_MISS_sum", 0.0)
        print("   -> L2 hit rate             %.3f" % (h / max(1.0, h + m)))
    if "SQ_WAVE_CYCLES" in mean:
        w = mean["SQ_WAVE_CYCLES"]
        print("   -> wait_any %.2f  wait_inst %.2f  active %.2f (fractions of wave cycles)" % (
            mean.get("SQ_WAIT_ANY", 0) / w, mean.get("SQ_WAIT_INST_ANY", 0) / w, mean.get("SQ_ACTIVE_INST_ANY", 0) / w))
