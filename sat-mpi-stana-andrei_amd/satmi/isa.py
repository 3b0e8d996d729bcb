"""Machine-code identity of a kernel in libsatmi.so (no GPU, no HIP calls).

The bench's issue rooflines come from SQ counter passes taken on one build of
a kernel (profiles/sq_issue.json).  Whether an entry still describes the
kernel that runs is a question about the code object, not the source text: a
comment edit must not mark it stale, a changed instruction must.  So the key
is a hash of the kernel's gfx950 machine code, read from the library itself:

    libsatmi.so  .hip_fatbin: one clang offload bundle per translation unit
      bundle entry "hipv4-amdgcn-amd-amdhsa--gfx950": an AMDGPU ELF code object
        .symtab: the kernel functions (STT_FUNC) and their descriptors (*.kd)

`kernel_code_sha(base)` hashes, in symbol-name order, the bytes of every
function symbol and kernel descriptor whose name contains `base` (every
template instance of that kernel).  A descriptor's kernel_code_entry_byte_offset
(bytes 16-23: the distance from the descriptor to the code) is zeroed first:
it moves whenever another kernel of the same code object changes size, while
the instructions themselves (branches are PC-relative) do not.
"""
import hashlib
import os
import struct

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_ARCH = b"hipv4-amdgcn-amd-amdhsa--gfx950"


def code_objects(data):
    """The gfx950 code objects (bytes) of every offload bundle in `data`."""
    out = []
    i = data.find(_BUNDLE_MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl]
            p += tl
            if triple == _ARCH and size:
                out.append(data[i + off:i + off + size])
        i = data.find(_BUNDLE_MAGIC, i + 1)
    return out


def elf_symbols(co):
    """[(name, bytes)] of the sized function / object symbols of an ELF64 code object."""
    shoff, = struct.unpack_from("<Q", co, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", co, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", co, shoff + k * shentsize) for k in range(shnum)]
    out = []
    for (_, stype, _, _, off, size, link, _, _, entsize) in secs:
        if stype != 2:   # SHT_SYMTAB
            continue
        stroff = secs[link][4]
        for j in range(size // entsize):
            name_off, info, _, shndx, value, ssize = struct.unpack_from("<IBBHQQ", co, off + j * entsize)
            if ssize == 0 or (info & 0xF) not in (1, 2) or shndx == 0 or shndx >= shnum:   # OBJECT, FUNC
                continue
            end = co.index(b"\0", stroff + name_off)
            name = co[stroff + name_off:end].decode("ascii", "replace")
            sec = secs[shndx]   # value is a virtual address: its offset in the file via the section
            foff = sec[4] + (value - sec[3])
            out.append((name, co[foff:foff + ssize]))
    return out


def kernel_code_sha(base, lib_path=None):
    """16 hex digits of sha256 over the machine code of the kernels named
    `base` (e.g. "dpll_fixed_kernel", "dpll_scan_kernel", "cdcl_kernel",
    "res_pass"); None if the library or the kernel is absent."""
    if lib_path is None:
        from . import _capi
        lib_path = _capi.LIB_PATH
    if not os.path.exists(lib_path):
        return None
    with open(lib_path, "rb") as fh:
        data = fh.read()
    h = hashlib.sha256()
    found = False
    for co in code_objects(data):
        for name, code in sorted(elf_symbols(co)):
            if base in name:
                if name.endswith(".kd") and len(code) == 64:
                    code = code[:16] + bytes(8) + code[24:]
                h.update(name.encode() + b"\0" + code)
                found = True
    return h.hexdigest()[:16] if found else None
