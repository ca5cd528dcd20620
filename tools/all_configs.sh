#!/bin/bash
# Every bench config once (no CPU baseline): one JSON line each into gpurun_out/$1.jsonl
set -u
out=gpurun_out/${1:-cfgs}.jsonl; : > $out
for spec in "C2 200" "C3 100" "C4 20" "C5 20" "C3 40 --batch 16"; do
  set -- $spec
  c=$1; st=$2; shift 2
  timeout -k 10 300 python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline "$@" > gpurun_out/cfg.log 2>&1 || { tail -3 gpurun_out/cfg.log; exit 1; }
  grep '^{' gpurun_out/cfg.log >> $out
  python - "$c" "$*" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/cfg.log") if l.startswith("{")][-1])
k = d.get("kernel_ms_per_step", {})
print(sys.argv[1], sys.argv[2], d["value"], d["unit"], "assemble ms/step", k.get("assemble"), "kbuild GB/s", k.get("kbuild_GBps"))
PY
done
