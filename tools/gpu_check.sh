#!/bin/bash
# One GPU-box session: build check, GPU parity tests, short bench.  Stops at the first step
# that faults / aborts / times out (exit 124, 134, 137, 139); ordinary test failures continue.
set -u
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1
rc=$?; echo "build rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
fatal $rc && exit $rc
if [ "${RUN_BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
  fatal $rc && exit $rc
fi
exit 0
