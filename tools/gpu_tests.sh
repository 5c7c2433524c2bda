#!/bin/bash
# GPU test session: smoke, the -m gpu suite (one process, per-test time
# limit), then a short bench unless NO_BENCH=1.  Every GPU step has its own
# time limit; a crash/timeout ends the session (no retries).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>: rc 0/1 continue, anything else stops
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.txt" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -5 "gpurun_out/$name.txt"
    if [ $rc -gt 1 ]; then exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS}
[ -n "$NO_BENCH" ] || step bench 600 python bench.py --steps 5 --warmup 2
