#!/bin/bash
# One GPU session: VALU issue-rate microbench, smoke, GPU parity tests, bench.
# Every GPU step has its own time limit; a crash/timeout ends the session.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>: rc 0/1 continue, anything else stops
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.txt" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -3 "gpurun_out/$name.txt"
    if [ $rc -gt 1 ]; then exit $rc; fi
}
[ -x tools/ubench_valu ] && step ubench 120 ./tools/ubench_valu
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1200 python -m pytest tests -q -m gpu -x
step bench 600 python bench.py --steps 3 --warmup 1
