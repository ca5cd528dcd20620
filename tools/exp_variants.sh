#!/bin/bash
# A/B of prebuilt libgpk variants (variants/libgpk_<name>.so): quick parity, then bench lines.
# usage: NAMES="old base cfirst" [CHECK="base cfirst"] [BENCH_ARGS=...] bash tools/exp_variants.sh
set -u
mkdir -p gpurun_out
for n in ${CHECK:-}; do
  GPK_LIB=variants/libgpk_$n.so timeout -k 10 300 python -m pytest tests -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "schedule or golden_c2 or golden_c3 or grad_matches" > gpurun_out/chk_$n.log 2>&1
  rc=$?; echo "check $n rc=$rc $(tail -1 gpurun_out/chk_$n.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
for n in ${NAMES}; do
  for cfg in ${CFGS:-metric}; do
    GPK_LIB=variants/libgpk_$n.so timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 \
        --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/v_${n}_$cfg.log 2>&1
    rc=$?
    python - "$n" "$cfg" <<'PY'
import json, sys
n, cfg = sys.argv[1], sys.argv[2]
l = [x for x in open("gpurun_out/v_%s_%s.log" % (n, cfg)) if x.startswith("{")]
if l:
    d = json.loads(l[-1]); r = d["roofline"] or {}
    print("%-8s %-7s value %9.3f ms %8.3f upd %.2f TF (%.1f us) ovl %s" % (n, cfg, d["value"], d["ms_per_step"],
          r.get("achieved", 0), r.get("avg_launch_us", 0), r.get("overlapped_achieved")))
else:
    print(n, cfg, "no line")
PY
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
