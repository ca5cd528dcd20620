#!/bin/bash
# One GPU-box session: build check, GPU parity tests, short bench, optional rocprofv3 trace.
# Stops at the first step that faults / aborts / times out (exit 124, 134, 137, 139);
# ordinary test failures continue.
set -u
ROOT=$(pwd)
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1
rc=$?; echo "build rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/build.log; exit $rc; }
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -8 gpurun_out/gpu_tests.log
  fatal $rc && exit $rc
fi
if [ "${RUN_BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
  fatal $rc && exit $rc
fi
if [ "${RUN_PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$ROOT/gpurun_out/prof" -o run -- python "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline ${PROF_ARGS:-} \
      > gpurun_out/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/prof.log
  fatal $rc && exit $rc
fi
exit 0
