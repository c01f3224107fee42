"""Per-kernel resources of the shipped gfx950 code objects, read from libchiara.so itself.

The library's `.hip_fatbin` section holds one clang offload bundle per HIP translation unit; each bundle's gfx950
entry is an ELF code object whose NT_AMDGPU_METADATA note lists every kernel's `.vgpr_count`, `.agpr_count`,
`.private_segment_fixed_size` (scratch) and `.group_segment_fixed_size` (static LDS).  No GPU is needed.

Why it matters: beside RCCL a tree grid runs three one-wave workgroups per SIMD (12 per CU), and
rcclGenericKernel's wave needs ~288 of the SIMD's 512 VGPRs: a tree kernel above 72 VGPRs (8-register granules)
starves it.  A change of operand order once moved the bf16 trees from 66 to 80 without any test noticing
(DESIGN §4.2); tests/test_kernel_resources.py now checks the budget on every build.

    python3 tools/kernel_resources.py [libchiara.so]      -> one JSON object {kernel: {vgpr, agpr, scratch, lds}}
"""
import json
import os
import struct
import subprocess
import sys
import tempfile

import yaml

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
OBJCOPY = "/opt/rocm/lib/llvm/bin/llvm-objcopy"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
DEFAULT_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                           "configurable-hierarchical-allreduce-algorithms_amd", "chiara_amd", "libchiara.so")


def _bundles(fat):
    """(offset, size) of every gfx950 code object in an (uncompressed) offload-bundle stream."""
    out, pos = [], 0
    while True:
        i = fat.find(MAGIC, pos)
        if i < 0:
            return out
        off = i + len(MAGIC)
        (n,) = struct.unpack_from("<Q", fat, off)
        off += 8
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", fat, off)
            off += 24
            triple = fat[off:off + tl].decode()
            off += tl
            if triple.endswith("gfx950") and sz:
                out.append((i + o, sz))
        pos = i + 1


def kernel_resources(lib=DEFAULT_LIB):
    with tempfile.TemporaryDirectory() as tmp:
        fat_path = os.path.join(tmp, "fat.bin")
        subprocess.run([OBJCOPY, "--dump-section", f".hip_fatbin={fat_path}", lib, os.path.join(tmp, "stripped")],
                       check=True, capture_output=True)
        fat = open(fat_path, "rb").read()
        if fat.startswith(b"CCOB"):
            raise RuntimeError("compressed offload bundle: build without --offload-compress")
        res = {}
        for k, (o, sz) in enumerate(_bundles(fat)):
            co = os.path.join(tmp, f"co{k}.o")
            with open(co, "wb") as f:
                f.write(fat[o:o + sz])
            notes = subprocess.run([READELF, "--notes", co], check=True, capture_output=True, text=True).stdout
            text = notes[notes.index("---"):]
            text = text[:text.index("\n...") + 4] if "\n..." in text else text
            meta = yaml.safe_load(text)
            for kern in meta["amdhsa.kernels"]:
                res[kern[".name"]] = {"vgpr": kern[".vgpr_count"], "agpr": kern.get(".agpr_count", 0),
                                      "scratch": kern[".private_segment_fixed_size"],
                                      "lds": kern[".group_segment_fixed_size"]}
        return res


def alloc_vgprs(r):
    """Registers a wave of this kernel takes from the SIMD's 512: VGPRs and AGPRs share the file (AGPRs start at a
    4-aligned offset), allocated in granules of 8."""
    v = r["vgpr"]
    if r["agpr"]:
        v = (v + 3) // 4 * 4 + r["agpr"]
    return (v + 7) // 8 * 8


if __name__ == "__main__":
    print(json.dumps(kernel_resources(sys.argv[1] if len(sys.argv) > 1 else DEFAULT_LIB), sort_keys=True))
