# round 5: C2's persistent schedule through the N > 1 code path (RCCL group, per-step all-gather) on one GPU
set -o pipefail
O=gpurun_out/r5z; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_chain.py -k "unsettled or side_by_side" -m gpu > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29557 bench.py --gpus 1 --config C2 --steps 200 --warmup 20 --dist --no-cpu-baseline > $O/c2_dist.log 2>&1 || { tail -5 $O/c2_dist.log; exit 1; }
grep '^{' $O/c2_dist.log > $O/c2_dist.json; python -c "import json; d=json.load(open('$O/c2_dist.json')); print(d['value'], d['check'])"
