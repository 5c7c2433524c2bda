#!/bin/bash
# RT_RNG_SERIAL tuning sweep (iteration length L x window half-width z sigma)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for L in ${LS:-4096 8192 16384}; do
  for Z in ${ZS:-10 15 20}; do
    echo "== L=$L z=$Z"
    RT_AMD_SERIAL_DEBUG=1 RT_AMD_SERIAL_CHUNK=$L RT_AMD_SERIAL_Z10=$Z REPS=1 timeout -k 10 120 python3 tools/serial_probe.py 2>&1 | grep -E "call|debug" || exit 1
  done
done
