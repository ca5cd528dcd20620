# round 5: device write / copy ceilings (the K build's roofline)
set -o pipefail
mkdir -p gpurun_out/r5ao
timeout -k 10 120 python tools/probe/write_ceiling.py > gpurun_out/r5ao/write_ceiling.jsonl 2>&1 || { tail -5 gpurun_out/r5ao/write_ceiling.jsonl; exit 1; }
cat gpurun_out/r5ao/write_ceiling.jsonl
