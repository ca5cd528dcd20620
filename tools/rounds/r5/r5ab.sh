# round 5 final tree: posterior (mu + full Sigma) latency, single-evaluation device spans chain vs launch path
set -o pipefail
O=gpurun_out/r05fin; mkdir -p $O
timeout -k 10 300 python tools/bench_posterior.py 4096 1024 10 > $O/posterior_4096.log 2>&1 || { tail -3 $O/posterior_4096.log; exit 1; }
timeout -k 10 300 python tools/bench_posterior.py 8192 2048 5 > $O/posterior_8192.log 2>&1 || { tail -3 $O/posterior_8192.log; exit 1; }
grep -v INFO $O/posterior_4096.log $O/posterior_8192.log | grep -v amdgpu.ids | tail -6
SETS='{"chain":1};{"chain":0,"lookahead":2}' timeout -k 10 300 python tools/single_sched.py 1024 2048 4096 6144 8192 12288 > $O/spans.jsonl 2>&1 || { tail -3 $O/spans.jsonl; exit 1; }
grep '^{' $O/spans.jsonl
