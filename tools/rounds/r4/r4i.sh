# D-task ablation inside the persistent factorisation (GPK_CHAIN_DBG bits of diag2_body; timing only)
set -o pipefail
O=gpurun_out/r4i; mkdir -p $O
for d in 0 2 1 4 8 32 16 34 6; do
  GPK_CHAIN_DBG=$d timeout -k 10 120 python tools/chain_prof.py 4096 > $O/prof_$d.txt 2>&1 || exit 1
done
timeout -k 10 120 python tools/exp_diag.py 1 4096 > $O/exp_diag.txt 2>&1 || exit 1
