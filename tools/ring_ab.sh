#!/bin/bash
# C2 ring traffic against pixels per chunk (RT_AMD_RESOLVE_PIX): FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes of the timed (lean) trace kernel, then an
# interleaved A/B of the frame times in one process (tools/ab.py).
# usage: tools/ring_ab.sh <outdir> [config]
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/${1:-gpurun_out/ring_ab}"
CFG=${2:-c2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for px in 8 4 2; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    name=px${px}_$ctr
    env RT_AMD_RESOLVE_PIX=$px timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d "$OUT/$name" -o "$name" \
        --output-format csv -- python3 "$REPO/bench.py" --config $CFG --no-cpu-baseline --no-serial --steps 3 --warmup 1 \
        > "$OUT/$name.log" 2>&1 || exit 1
    python3 - "$OUT/$name" "$name" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/*counter_collection.csv")[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].replace(" ", "")
    if "trace_kernel<" in n and n.split("trace_kernel<", 1)[1].split(">", 1)[0].split(",")[4] == "false":
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: sum(v) / len(v) for k, v in agg.items()}, flush=True)
PY
  done
done
cd "$REPO"
timeout -k 10 300 python3 tools/ab.py --config $CFG --rounds 7 --variant px8=rust-swift-raytracer_amd/lib/libraytracer.so:RT_AMD_RESOLVE_PIX=8 \
    --variant px4=rust-swift-raytracer_amd/lib/libraytracer.so:RT_AMD_RESOLVE_PIX=4 \
    --variant px2=rust-swift-raytracer_amd/lib/libraytracer.so:RT_AMD_RESOLVE_PIX=2 > "$OUT/ab.log" 2>&1 || exit 1
grep -v amdgpu "$OUT/ab.log" | cut -c1-220
