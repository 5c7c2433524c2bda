#!/bin/bash
# SERIAL (render()'s reference-identical mode) on one GPU: the SERIAL parity
# tests, then the coalescing block search against the count pass on the
# 960x540x16 frames (tools/serial_probe.py).  Every GPU step has its own time
# limit; a failure ends the session.  EXTRA: more env for the coalescing run.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
CASES_AB="${CASES_AB:-c_raytracer:960x540x16/8,rtow:960x540x16/8,world:960x540x16/8}"
if [ -z "$NO_TESTS" ]; then
    timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_serial.py \
        > gpurun_out/serial_tests.log 2>&1 || { tail -30 gpurun_out/serial_tests.log; exit 1; }
    tail -3 gpurun_out/serial_tests.log
fi
env $EXTRA RT_AMD_SERIAL_DEBUG=1 CASES="$CASES_AB" timeout -k 10 300 python -u tools/serial_probe.py \
    > gpurun_out/probe_coalesce.log 2>&1 || { tail -30 gpurun_out/probe_coalesce.log; exit 1; }
grep -v amdgpu.ids gpurun_out/probe_coalesce.log
if [ -z "$NO_COUNT" ]; then
    RT_AMD_SERIAL_COALESCE=0 CASES="$CASES_AB" timeout -k 10 300 python -u tools/serial_probe.py \
        > gpurun_out/probe_count.log 2>&1 || { tail -30 gpurun_out/probe_count.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/probe_count.log
fi
