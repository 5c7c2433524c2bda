"""Summarise a tools/profile.sh output directory (rocprofv3 CSVs) into JSON.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KB
from separate --pmc passes; on gfx950 FETCH_SIZE reads 1/2 of the bytes of
wide coalesced streaming reads, so fetched bytes are reported both raw and
x2-corrected; WRITE_SIZE is exact for 16-B-per-lane stores.

usage: python tools/pmc_summary.py gpurun_out/prof_r01 profiles/r01 [config]
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def short(name):
    # trace_kernel<kBvh, kLds, kStep, kMesh, kCount, kSerial>: the timed frames
    # run the kCount=false variant ("trace_kernel"); frames with stats run
    # "trace_kernel[count]", SERIAL passes "trace_kernel[serial]"
    if "trace_kernel" in name:
        args = name.split("trace_kernel<", 1)[-1].split(">", 1)[0].replace(" ", "").split(",")
        if len(args) >= 6 and args[5] == "true":
            return "trace_kernel[serial]"
        return "trace_kernel[count]" if len(args) >= 5 and args[4] == "true" else "trace_kernel"
    if "resolve_kernel" in name:
        return "resolve_kernel"
    return name[:60]


def main(src, dst, config="c2"):
    os.makedirs(dst, exist_ok=True)
    out = {"source": os.path.basename(src.rstrip("/")), "kernels": {}}
    for key in ("lib_sha256", "kernel_sha256"):
        sha = os.path.join(src, key + ".txt")
        if os.path.exists(sha):
            out[key] = open(sha).read().strip()
            shutil.copy(sha, os.path.join(dst, key + ".txt"))
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            k = out["kernels"].setdefault(short(r["Name"]), {})
            k["calls"] = int(r["Calls"])
            k["avg_ns"] = float(r["AverageNs"])
            k["pct_time"] = float(r["Percentage"])
    for f in glob.glob(os.path.join(src, "pmc_*", "*counter_collection.csv")):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (kern, ctr), v in agg.items():
            if kern in ("trace_kernel", "trace_kernel[count]", "resolve_kernel"):
                out["kernels"].setdefault(kern, {})[ctr] = sum(v) / len(v)
    for k in out["kernels"].values():
        if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
            k["hbm_fetch_bytes_raw"] = k["FETCH_SIZE"] * 1024
            k["hbm_fetch_bytes_x2"] = 2 * k["FETCH_SIZE"] * 1024
            k["hbm_write_bytes"] = k["WRITE_SIZE"] * 1024
            k["hbm_bytes_per_launch"] = k["hbm_fetch_bytes_x2"] + k["hbm_write_bytes"]
    # the bench line of the kernel-trace pass: the profiled run's schedule
    # (launch settings) and its timing, kept with the counters
    logf = os.path.join(src, "trace.log")
    bline = None
    if os.path.exists(logf):
        for line in open(logf):
            if line.startswith("{") and '"metric"' in line:
                bline = json.loads(line)
    if bline:
        out["launch"] = bline.get("launch_settings")
        out["bench_ms_per_step"] = bline.get("ms_per_step")
        out["bench_avg_launch_ms"] = (bline.get("roofline") or {}).get("avg_launch_ms")
        out["rays_per_frame"] = bline.get("rays_per_frame")
    # the timed region's launches: bench.py's last `steps` lean trace_kernel
    # dispatches of the frame's grid (before them: warm-up frames, after them
    # only counting-variant frames), their mean beside the all-dispatch average
    # rocprof's stats give.  Only valid when the bench skipped its SERIAL legs
    # (--no-serial, as tools/profile.sh runs it): their REPLAY frames are lean
    # trace_kernel dispatches too, after the timed region.
    traces = glob.glob(os.path.join(src, "trace", "*kernel_trace.csv"))
    steps = bline.get("steps") if bline else None
    if bline and "serial" in bline:
        print("pmc_summary: the profiled bench ran its SERIAL legs; timed_avg_ns not computed "
              "(run bench.py with --no-serial)", file=sys.stderr)
        steps = None
    if traces and steps:
        ls = (bline or {}).get("launch_settings") or {}
        grid = ls.get("blocks", 0) * ls.get("block_threads", 0)

        def frame_grid(r):
            g = r.get("Grid_Size_X") or r.get("Grid_Size")
            return not grid or g is None or int(g) == grid

        lean = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                      for r in csv.DictReader(open(traces[0]))
                      if short(r["Kernel_Name"]) == "trace_kernel" and frame_grid(r))
        timed = [d for _, d in lean[-steps:]]
        if timed and "trace_kernel" in out["kernels"]:
            out["kernels"]["trace_kernel"]["timed_launches"] = len(timed)
            out["kernels"]["trace_kernel"]["timed_avg_ns"] = sum(timed) / len(timed)
    # VALU evidence of the timed (lean) kernel: lanes active per VALU
    # instruction, VALU lane-slots per ray, and the issue rate against the
    # v_add_f32 microbenchmark (profiles/valu_ceiling.json, tools/ubench_valu)
    tk = out["kernels"].get("trace_kernel", {})
    if "SQ_INSTS_VALU" in tk and "SQ_THREAD_CYCLES_VALU" in tk:
        v = {"insts_valu": tk["SQ_INSTS_VALU"],
             "lanes_active": tk["SQ_THREAD_CYCLES_VALU"] / (64.0 * tk["SQ_INSTS_VALU"])}
        rays = out.get("rays_per_frame")
        if rays:
            v["lane_slots_per_ray"] = tk["SQ_INSTS_VALU"] * 64.0 / rays
        t_ns = tk.get("timed_avg_ns") or tk.get("avg_ns")
        if t_ns:
            v["issue_wave_insts_per_s"] = tk["SQ_INSTS_VALU"] / (t_ns * 1e-9)
            cf = os.path.join(os.path.dirname(dst.rstrip("/")), "valu_ceiling.json")
            if os.path.exists(cf):
                ceil = json.load(open(cf))["v_add_f32_wave_insts_per_s"]
                v["issue_frac_of_v_add_rate"] = v["issue_wave_insts_per_s"] / ceil
        if "SQ_WAIT_ANY" in tk and "SQ_WAVE_CYCLES" in tk:
            v["wait_frac"] = tk["SQ_WAIT_ANY"] / tk["SQ_WAVE_CYCLES"]
        out["valu"] = v
    with open(os.path.join(dst, "summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    tr = out["kernels"].get("trace_kernel", {})
    if "hbm_bytes_per_launch" in tr:
        path = os.path.join(os.path.dirname(dst.rstrip("/")), "hbm_traffic.json")
        allc = json.load(open(path)) if os.path.exists(path) else {}
        allc[config] = {"trace_bytes_per_launch": tr["hbm_bytes_per_launch"],
                        "from": os.path.relpath(dst, os.path.dirname(path)),
                        "lib_sha256": out.get("lib_sha256"),
                        "trace_kernel_sha256": out.get("kernel_sha256"),
                        "launch": out.get("launch"),
                        "profile_ms_per_step": out.get("bench_ms_per_step"),
                        "timed_avg_launch_ms": (tr.get("timed_avg_ns") or 0) * 1e-6 or None,
                        "valu": out.get("valu")}
        with open(path, "w") as fh:
            json.dump(allc, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
