# deferred-update depth (chain_group) at the larger single-evaluation sizes on the round-4 tree
set -o pipefail
O=gpurun_out/r4af; mkdir -p $O
SETS='{"chain_group":4};{"chain_group":8};{"chain_group":6};{"chain_group":4};{"chain_group":8}' timeout -k 10 400 python tools/single_sched.py 8192 10240 12288 > $O/ab.jsonl 2>&1 || exit 1
