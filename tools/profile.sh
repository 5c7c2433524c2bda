#!/bin/bash
# rocprofv3 evidence for bench.py: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md, rocprofv3 PMC slots).
# usage: tools/profile.sh <tag> [bench args...]
TAG=${1:-r01}; shift
REPO="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$REPO/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
# the binary these counters describe (bench.py compares it with the one it loads)
sha256sum "$REPO/rust-swift-raytracer_amd/lib/libraytracer.so" | cut -d' ' -f1 > "$OUT/lib_sha256.txt"
# ... and the hash of the frame trace kernels' machine code (tools/kernel_hash.py),
# which unrelated edits to the library do not change
python3 "$REPO/tools/kernel_hash.py" | head -1 > "$OUT/kernel_sha256.txt"
cd /tmp && export TMPDIR=/tmp
run() {  # run <name> <secs> <rocprof args...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv \
        -- python3 "$REPO/bench.py" --no-cpu-baseline --no-serial "${BENCH_ARGS[@]}" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -2 "$OUT/$name.log"
    [ $rc -eq 0 ] || exit $rc
}
BENCH_ARGS=("$@")
run trace 600 --kernel-trace --stats
run pmc_fetch 600 --kernel-trace --pmc FETCH_SIZE
run pmc_write 600 --kernel-trace --pmc WRITE_SIZE
run pmc_valu 600 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU
run pmc_wait 600 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
run pmc_l2 600 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum
run pmc_tcp 600 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD TCP_PENDING_STALL_CYCLES_sum
find "$OUT" -name "*.csv" | head -20
