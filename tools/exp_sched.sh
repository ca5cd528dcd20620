set -u
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
VARIANTS="noev=-@--no-events G2=GPK_GROUP=2@--no-events G8=GPK_GROUP=8@--no-events R0=GPK_RESERVE_CUS=0@--no-events R16=GPK_RESERVE_CUS=16@--no-events LA0=GPK_LOOKAHEAD=0@--no-events b16=-@--batch,16,--no-events b1=-@--batch,1,--no-events C2b8=-@--config,C2,--batch,8 C3=-@--config,C3 C4=-@--config,C4 C5=-@--config,C5" bash tools/bench_variants.sh || exit $?
GPK_LOOKAHEAD=0 PMC_FILE=tools/pmc_traffic.txt bash tools/pmc_pass.sh || exit $?
python tools/pmc_traffic.py metric_b8 gpurun_out/pmc gpurun_out/pmc_traffic.json
