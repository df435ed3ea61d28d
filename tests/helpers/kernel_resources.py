"""Per-kernel resources of the built library, read from its gfx950 code objects: for every kernel, the scratch
bytes per lane (`.private_segment_fixed_size`) and the VGPR count (`.vgpr_count`) from the AMDGPU metadata note.
The library's `.hip_fatbin` section holds one clang offload bundle per source file; each gfx950 entry is an ELF
code object whose notes `llvm-readelf --notes` prints. Host-only: nothing here touches a GPU."""
import os
import re
import struct
import subprocess
import tempfile

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _section(path, name):
    b = open(path, "rb").read()
    shoff = struct.unpack_from("<Q", b, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    stro = secs[shstrndx][4]
    for s in secs:
        if b[stro + s[0]: b.index(b"\0", stro + s[0])].decode() == name:
            return b[s[4]: s[4] + s[5]]
    return None


def kernel_resources(lib, arch="gfx950"):
    """{mangled kernel name: (scratch bytes per lane, VGPRs)} over every code object for `arch` in `lib`."""
    fat = _section(lib, ".hip_fatbin")
    if fat is None:
        raise RuntimeError(f"{lib}: no .hip_fatbin section")
    res, pos = {}, 0
    while True:
        i = fat.find(_MAGIC, pos)
        if i < 0:
            break
        n = struct.unpack_from("<Q", fat, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24: p + 24 + tl].decode()
            p += 24 + tl
            if arch not in triple:
                continue
            with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
                f.write(fat[i + off: i + off + size])
            try:
                out = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True, check=True).stdout
            finally:
                os.unlink(f.name)
            for blk in out.split("  - .")[1:]:
                m = re.search(r"\.name:\s+(\S+)", blk)
                s = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
                v = re.search(r"\.vgpr_count:\s+(\d+)", blk)
                if m and s and v:
                    res[m.group(1)] = (int(s.group(1)), int(v.group(1)))
        pos = i + 32
    return res
