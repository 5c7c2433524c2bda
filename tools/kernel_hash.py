"""sha256 of the frame trace kernels' machine code inside libraytracer.so
(measurement bookkeeping, not product code).

bench.py quotes roofline.traffic from a separate rocprofv3 PMC run
(profiles/hbm_traffic.json).  Keying that figure on the whole .so made any
unrelated edit (a SERIAL kernel, host code) flip `same_binary`; this hashes
only what the counters describe: the gfx950 code of the lean frame variants
of trace_kernel (render.hip trace_kernel<..., kCount = false, kSerial =
false>), i.e. the bytes of each such function symbol plus its kernel
descriptor (less its position-dependent code-entry offset), taken from the
clang offload bundle in the .hip_fatbin section.

  python tools/kernel_hash.py [lib.so]      -> prints the hash and the symbols
"""
import hashlib
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "rust-swift-raytracer_amd", "lib", "libraytracer.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# trace_kernel<kBvh, kLds, kStep, kMesh, kCount=false, kSerial=false>: the
# mangled template argument list ends in Lb0ELb0E (the last two bools)
FRAME_SUFFIX = "ELb0ELb0EEEvNS_11TraceParamsE"


def _bundles(blob):
    """(triple, bytes) of every entry of every offload bundle in blob."""
    pos = blob.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", blob, pos + 24)
        off = pos + 32
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", blob, off)
            triple = blob[off + 24:off + 24 + tlen].decode()
            off += 24 + tlen
            yield triple, blob[pos + eoff:pos + eoff + esize]
        pos = blob.find(MAGIC, pos + 24)


def _elf_symbols(elf):
    """{name: bytes} of the FUNC and OBJECT symbols of a 64-bit ELF."""
    if elf[:4] != b"\x7fELF":
        return {}
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    out = {}
    for sec in secs:
        if sec[1] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[sec[6]]
        for k in range(sec[5] // sec[9]):
            name_off, info, _other, shndx, value, size = struct.unpack_from("<IBBHQQ", elf, sec[4] + k * sec[9])
            if size == 0 or shndx == 0 or shndx >= len(secs) or (info & 0xF) not in (1, 2):
                continue
            s0 = strtab[4] + name_off
            name = elf[s0:elf.index(b"\0", s0)].decode()
            host = secs[shndx]
            start = host[4] + (value - host[3])
            out[name] = elf[start:start + size]
    return out


def frame_kernel_hash(lib=LIB):
    """(sha256 hex, [symbol names]) of the lean frame trace kernels, or (None, [])."""
    with open(lib, "rb") as fh:
        blob = fh.read()
    syms = {}
    for triple, code in _bundles(blob):
        if "gfx950" in triple:
            syms.update(_elf_symbols(code))
    names = sorted(n for n in syms if "trace_kernel" in n and n.endswith(FRAME_SUFFIX))
    if not names:
        return None, []
    h = hashlib.sha256()
    for n in names:
        h.update(n.encode())
        h.update(syms[n])
        # the kernel descriptor (register counts, LDS / scratch / kernarg sizes)
        # without kernel_code_entry_byte_offset (bytes 16-23): that field is the
        # distance from the descriptor to the code, which moves whenever any
        # other kernel of the library changes size
        kd = bytearray(syms.get(n + ".kd", b""))
        if len(kd) >= 24:
            kd[16:24] = bytes(8)
        h.update(bytes(kd))
    return h.hexdigest(), names


if __name__ == "__main__":
    digest, names = frame_kernel_hash(sys.argv[1] if len(sys.argv) > 1 else LIB)
    print(digest)
    for n in names:
        print("  ", n)
