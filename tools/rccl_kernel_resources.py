#!/usr/bin/env python3
"""Workgroup size, LDS, VGPRs and scratch of the gfx950 kernels in an RCCL library, read from the
AMDGPU metadata of its embedded code objects (no GPU needed).  The two RCCLs a process here can
load: torch's bundled one (Python processes import torch first) and ROCm 7.2's (the C++ harnesses).

    python tools/rccl_kernel_resources.py [librccl.so ...]   (default: both)
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
DEFAULT = ["/usr/local/lib/python3.10/dist-packages/torch/lib/librccl.so", "/opt/rocm/lib/librccl.so.1"]


def kernels(lib, tmp):
    fb = os.path.join(tmp, "fatbin.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", lib], check=True)
    d = open(fb, "rb").read()
    offs = sorted(m.start() for pat in (b"__CLANG_OFFLOAD_BUNDLE__", b"CCOB")
                  for m in re.finditer(re.escape(pat), d) if m.start() % 4096 == 0)
    rows = []
    for i, o in enumerate(offs):
        part, co = os.path.join(tmp, "p.bin"), os.path.join(tmp, "p.co")
        open(part, "wb").write(d[o:offs[i + 1] if i + 1 < len(offs) else len(d)])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode:
            continue
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
        for b in re.split(r"\n  - \.agpr_count", notes)[1:]:
            def f(k):
                m = re.search(r"\." + k + r":\s+(\S+)", b)
                return m.group(1) if m else None
            rows.append((f("name"), int(f("group_segment_fixed_size")), int(f("max_flat_workgroup_size")),
                         int(f("vgpr_count")), int(f("private_segment_fixed_size"))))
    return rows


def main():
    libs = sys.argv[1:] or DEFAULT
    with tempfile.TemporaryDirectory() as tmp:
        for lib in libs:
            if not os.path.exists(lib):
                print(f"{lib}: absent")
                continue
            rows = kernels(lib, tmp)
            print(f"{lib}: {len(rows)} gfx950 kernels")
            print("  the collective / send-recv kernels (every ncclSend/ncclRecv group launches one):")
            for name, lds, wg, vgpr, scratch in rows:
                if "Generic" in name:
                    print(f"    {name[:60]:60s} LDS {lds:6d} B  max WG {wg:4d}  VGPR+AGPR {vgpr:4d}  scratch {scratch} B")
            fam = collections.Counter((re.sub(r"_(Sum|Prod|MinMax|PreMulSum|SumPostDiv)_.*", "_*", n)[:40], lds, wg)
                                      for n, lds, wg, _, _ in rows if "Generic" not in n)
            print("  other kernel families (name prefix, LDS, max WG): count")
            for k, v in sorted(fam.items()):
                print(f"    {k}: {v}")


if __name__ == "__main__":
    main()
