#!/bin/bash
# one WRITE_SIZE/TCC_REQ pass per variant (env settings), C2 bench, 2 steps
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/pmc_ab"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in "fused:RT_AMD_FUSED=1" "p4:RT_AMD_RESOLVE_PIX=4" "slab:RT_AMD_FUSED=0"; do
  name=${v%%:*}; kv=${v#*:}
  env "$kv" timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_REQ_sum -d "$OUT/$name" -o "$name" --output-format csv -- python3 "$REPO/bench.py" --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/$name.log" 2>&1 || exit 1
  python3 - "$OUT/$name" "$name" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/*counter_collection.csv")[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "trace_kernel" in r["Kernel_Name"]:
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: sum(v) / len(v) for k, v in agg.items()})
PY
done
