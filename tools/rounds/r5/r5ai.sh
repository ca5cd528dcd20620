# round 5: host-side profile of get_metric at small N
set -o pipefail
O=gpurun_out/r5ai; mkdir -p $O
timeout -k 10 300 python tools/api_profile.py 256 400 > $O/prof256.txt 2>&1 || { tail -5 $O/prof256.txt; exit 1; }
grep -v INFO $O/prof256.txt | head -60
