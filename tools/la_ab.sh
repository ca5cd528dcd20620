set -u
for la in 0 1 0 1; do
  for a in "value 8192 1 4" "value 4096 1" "8192 1"; do
    GPK_LA_FIRST=$la timeout -k 10 100 python tools/exp_grad.py $a > gpurun_out/la.log 2>&1 || exit 1
    echo "la_first=$la $a: $(grep 'per call' gpurun_out/la.log | sed 's/ (.*//' | tr '\n' ';')"
  done
done
