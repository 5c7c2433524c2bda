"""Static ISA breakdown of one trace_kernel instance (tuning tool, not product).

Compiles render.hip for gfx950 to assembly with line tables (-g changes no
code: the instruction count is checked against the plain build), then counts
the instructions of one kernel by class (VALU, SALU, vector memory, LDS,
scalar memory, branches, waits) and by the source region of their innermost
location: the helper functions of render.hip and the sections of the
trace_kernel loop (ray setup, sphere walk, triangle walk, shading, sample
store, fused resolve, refill, direction normalisation).  Static counts weigh
every instruction once; tools/stamps.py gives the dynamic (cycle) shares.

  python tools/isa_breakdown.py [--kernel 1,1,0,0,0,0] [--defs "-DX"] [--asm file.s]
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rust-swift-raytracer_amd", "csrc", "render.hip")
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "--offload-arch=gfx950",
         "--cuda-device-only", "-S"]


def compile_asm(defs, debug):
    out = tempfile.NamedTemporaryFile(suffix=".s", delete=False).name
    cmd = ["/opt/rocm/bin/hipcc"] + FLAGS + (["-g"] if debug else []) + defs + [SRC, "-o", out]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return out


def kernel_body(lines, flags):
    """Instruction lines (with their .loc) of trace_kernel<flags>."""
    tag = "trace_kernelI" + "".join(("Li%sE" if k == 3 else "Lb%sE") % f for k, f in enumerate(flags)) + "EEvNS_11TraceParamsE:"
    start = next(i for i, l in enumerate(lines) if l.startswith("_ZN") and tag in l)
    body = []
    loc = None
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith(".Lfunc_end"):
            break
        if s.startswith(".loc"):
            parts = s.split()
            loc = (int(parts[1]), int(parts[2]))
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        body.append((s.split()[0], loc))
    return body


def klass(op):
    if op.startswith("v_"):
        return "VALU"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "VMEM"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "SMEM"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
        return "branch"
    if op.startswith("s_waitcnt") or op in ("s_nop", "s_barrier", "s_sleep"):
        return "wait/sync"
    if op.startswith("s_"):
        return "SALU"
    return "other"


def regions():
    """(first line, last line, name) of render.hip's functions and loop sections."""
    src = open(SRC).read().split("\n")
    out = []
    head = re.compile(r"^(?:__device__|__global__|static|RT_HOST_DEVICE|void|hipError_t|uint32_t|size_t)\b")
    skip = {"__launch_bounds__", "amdgpu_waves_per_eu", "__attribute__", "if", "for"}
    starts = []
    for i, l in enumerate(src, 1):
        if not head.match(l) or l.rstrip().endswith(";"):
            continue
        names = [n for n in re.findall(r"(\w+)\s*\(", l) if n not in skip]
        if names:
            starts.append((i, names[0]))
    for k, (i, name) in enumerate(starts):
        end = starts[k + 1][0] - 1 if k + 1 < len(starts) else len(src)
        out.append((i, end, name))
    # sections of trace_kernel's loop, by the comments that open them
    marks = [("---- ray_color's bounce loop", "loop: ray setup"),
             ("kStep: at most p.steps node visits", "loop: sphere walk"),
             ("if (phase == kTriInit)", "loop: triangle walk"),
             ("if (phase == kShade)", "loop: shading"),
             ("if (done) {", "loop: sample store (+ SERIAL counts)"),
             ("---- fused resolve, at refill points", "loop: fused resolve"),
             ("---- refill lanes whose path ended", "loop: refill"),
             ("if (renorm) dir = unit(vdir);", "loop: direction normalisation"),
             ("---- per-wave statistics", "after the loop")]
    tk = next((a, b) for a, b, n in out if n == "trace_kernel")
    pos = []
    for text, name in marks:
        for i in range(tk[0], tk[1] + 1):
            if text in src[i - 1]:
                pos.append((i, name))
                break
    pos.sort()
    sec = []
    for k, (i, name) in enumerate(pos):
        end = pos[k + 1][0] - 1 if k + 1 < len(pos) else tk[1]
        sec.append((i, end, name))
    pre = (tk[0], pos[0][0] - 1, "kernel entry (LDS staging)") if pos else None
    return out, ([pre] if pre else []) + sec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="1,1,0,0,0,0",
                    help="trace_kernel<kBvh,kLds,kStep,kMesh,kCount,kSerial> flags (default: C2's lean kernel)")
    ap.add_argument("--defs", default="")
    ap.add_argument("--asm", default=None)
    args = ap.parse_args()
    flags = args.kernel.split(",")
    defs = args.defs.split() if args.defs else []
    asm = args.asm or compile_asm(defs, True)
    plain = compile_asm(defs, False)
    body = kernel_body(open(asm).read().split("\n"), flags)
    nplain = len(kernel_body(open(plain).read().split("\n"), flags))
    files = {}
    for l in open(asm):
        if l.lstrip().startswith(".file"):
            p = l.split()
            files[int(p[1])] = p[-3].strip('"') if p[-2] == "md5" else p[-1].strip('"')
    funcs, secs = regions()
    by_class = collections.Counter(klass(op) for op, _ in body)
    by_region = collections.defaultdict(collections.Counter)
    for op, loc in body:
        name = "?"
        if loc is not None:
            f = files.get(loc[0], "?")
            if f.endswith("render.hip"):
                line = loc[1]
                name = next((n for a, b, n in secs if a <= line <= b), None) or \
                    next((n for a, b, n in funcs if a <= line <= b), "render.hip")
            else:
                name = os.path.basename(f)
            if loc[1] == 0:
                name = "(no line)"
        by_region[name][klass(op)] += 1
    print(f"trace_kernel<{args.kernel}>: {len(body)} instructions with -g, {nplain} without "
          f"({'same code' if len(body) == nplain else 'DIFFERENT code: counts approximate'})")
    print("by class: " + ", ".join(f"{k} {v}" for k, v in by_class.most_common()))
    print(f"{'region (innermost source location)':44s} {'total':>6s} {'VALU':>6s} {'SALU':>6s} "
          f"{'VMEM':>5s} {'LDS':>5s} {'SMEM':>5s} {'br':>5s}")
    for name, c in sorted(by_region.items(), key=lambda kv: -sum(kv[1].values())):
        print(f"{name[:44]:44s} {sum(c.values()):6d} {c['VALU']:6d} {c['SALU']:6d} {c['VMEM']:5d} "
              f"{c['LDS']:5d} {c['SMEM']:5d} {c['branch']:5d}")
    if args.asm is None:
        os.unlink(asm)
    os.unlink(plain)


if __name__ == "__main__":
    sys.exit(main())
