# D phase timeline: potf2 modes 0 / 1 / 2, with the other waves' P work on (dbg 0) and off (dbg 13)
# (historical A/B script of round 4: the variant libraries it names were built with tools/build_variant.sh and removed after the measurement -- see DESIGN §4 for the outcome)
set -o pipefail
O=gpurun_out/r4l; mkdir -p $O
for m in 0 1 ""; do for d in 0 13; do
  GPK_CHAIN_DBG=$d GPK_LIB=variants/libgpk_dprof$m.so timeout -k 10 120 python tools/diag_phase_prof.py 4096 > $O/dphase_m${m}_d$d.txt 2>&1 || exit 1
done; done
