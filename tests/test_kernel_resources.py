"""Register and scratch budget of the shipped gfx950 kernels, read from libchiara.so's code objects (no GPU).

Beside RCCL every streaming reduction runs one-wave workgroups at 12 per CU (CoresidentScope):
three waves per SIMD, and rcclGenericKernel's wave needs ~288 of the SIMD's 512 VGPRs, so a streaming kernel
may take at most 72 (granules of 8).  Above that the RCCL-sized kernel waits for the reduction launch to drain
(U = 2 trees at 82-90: admission 4 -> 170 us, profiles/r05/cores_u/; bf16 trees at 80 after the NaN-payload fix:
median admission 29-48 -> 5.5-14 us once back at 61, profiles/r05/cores_ab_bf16/)."""
import os
import re
import shutil
import sys

import pytest

from chiara_amd import _lib

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import kernel_resources as kr  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists(kr.READELF), reason="llvm-readelf not in this image")

DT = ["f32", "f64", "i32", "bf16", "i8", "u8", "i16", "u16", "u32", "i64", "u64", "fi", "di", "li", "2i", "si",
      "cf", "cd"]
OP = ["sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor", "maxloc", "minloc"]
RCCL_ROOM_VGPRS = 72
# Until round 5's SWAR 8-bit code (reduce_common.hpp apply_vec) the int8 / uint8 MAX / MIN kernels held 88-152
# and the u8 two-leaf trees 96: no exception is left.


@pytest.fixture(scope="module")
def res():
    return kr.kernel_resources(_lib.LIB_PATH)


def _streaming(res):
    """(kind, dtype, op, shape) -> allocated VGPRs for the one-wave streaming kernels (the shapes CoresidentScope
    launches beside RCCL): k_reduce_tree<DT, OP, NL, U, true, 64> and k_reduce_vec<DT, OP, M, U, true, true, 64>."""
    out = {}
    for name, r in res.items():
        m = re.search(r"k_reduce_treeILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb1ELi64E", name)
        if m:
            dt, op, nl, u = map(int, m.groups())
            out[("tree", DT[dt], OP[op] if op < len(OP) else op, (nl, u))] = kr.alloc_vgprs(r)
        m = re.search(r"k_reduce_vecILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb1ELb1ELi64E", name)
        if m:
            dt, op, mm, u = map(int, m.groups())
            out[("vec", DT[dt], OP[op] if op < len(OP) else op, (mm, u))] = kr.alloc_vgprs(r)
    return out


def test_every_kernel_found_and_none_uses_scratch(res):
    assert len(res) > 2000
    scratch = {n: r["scratch"] for n, r in res.items() if r["scratch"]}
    assert not scratch, f"kernels with a private segment: {sorted(scratch)[:5]}"


def test_streaming_kernels_leave_rccl_its_registers(res):
    s = _streaming(res)
    assert len(s) > 500
    over = sorted((k, v) for k, v in s.items() if v > RCCL_ROOM_VGPRS)
    assert not over, f"streaming kernels above {RCCL_ROOM_VGPRS} VGPRs: {over[:8]}"


@pytest.mark.parametrize("dt", ["f32", "bf16", "f64", "i32", "i8", "u8"])
def test_the_configs_kernels_in_budget(res, dt):
    """C4 / C5's 8-leaf trees, the N = 4 / N = 2 lines' 4- and 2-leaf trees and every fold width, per dtype the
    reference's harnesses use (and bf16), and the 8-bit types whose per-lane code used to be the outliers."""
    s = _streaming(res)
    mine = {k: v for k, v in s.items() if k[1] == dt}
    assert {k[0] for k in mine} == {"tree", "vec"}
    if dt in ("f32", "bf16", "f64", "i32"):
        for nl, u in ((8, 1), (4, 2), (2, 4)):
            for op in ("sum", "prod", "max", "min"):
                assert ("tree", dt, op, (nl, u)) in mine
    for key, v in mine.items():
        assert v <= RCCL_ROOM_VGPRS, (key, v)
    if dt in ("f32", "bf16"):  # C4 / C5 themselves: 58 / 61 in round 5
        assert s[("tree", dt, "sum", (8, 1))] <= 64


def test_alloc_granule():
    assert kr.alloc_vgprs({"vgpr": 58, "agpr": 0}) == 64
    assert kr.alloc_vgprs({"vgpr": 61, "agpr": 0}) == 64
    assert kr.alloc_vgprs({"vgpr": 80, "agpr": 0}) == 80
    assert kr.alloc_vgprs({"vgpr": 10, "agpr": 4}) == 16
    assert shutil.which("nm")
