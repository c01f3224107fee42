"""Host-side checks of the fused expression-tree path (no GPU): the flat plan compiler
emits one tree op per chunk where the kernel's limits allow, CHR_TREE=0 falls back to one
fold per launch with identical results, and chr_reduce_tree validates programs."""
import ctypes
import os

import numpy as np
import pytest

import chiara_amd as ca
import plan_sim
import pyoracle as po
from tree_util import random_program


def _trees(mode, n, k, b, count, rank=0):
    p = ca.parse_plan(ca.describe_plan(mode, n, rank, k, b, count))
    return [op for st in p["steps"] for op in st["post"] if op[0] == "tree"], p


def test_c4_plan_is_one_tree_per_chunk():
    trees, p = _trees(ca.MODE_ALLREDUCE, 8, 4, 4, 8 * 4096)
    # 2 chunks (nnodes = 2) per slice: recexch fold of 4 + fold of 4, then the lane fold
    assert len(trees) == 2 * p["header"]["slices"]
    for op in trees:
        assert op[5] == ([0, 1, 1, 1, 0, 1, 1, 2], [0] * 7)
        assert op[1][0] == "RECV"  # the root lands straight in recvbuf
    reds = [op for st in p["steps"] for op in st["post"] if op[0].startswith("reduce")]
    assert not reds


@pytest.mark.parametrize("n,k,b", [(8, 2, 8), (8, 4, 8), (8, 2, 2), (6, 2, 3), (4, 2, 4)])
def test_tree_within_limits(n, k, b):
    trees, _ = _trees(ca.MODE_ALLREDUCE, n, k, b, n * 2048)
    assert trees
    for op in trees:
        comb, swaps = op[5]
        assert len(comb) == n and sum(comb) == n - 1 and len(swaps) == n - 1


def test_wide_trees_fall_back_to_folds():
    """16 leaves exceed the kernel's 8: one k_reduce_vec launch per reference fold."""
    trees, p = _trees(ca.MODE_ALLREDUCE, 16, 2, 16, 16 * 1024)
    assert not trees
    assert any(op[0] == "reduce" for st in p["steps"] for op in st["post"])


@pytest.mark.parametrize("mode,n,k,b,dt", [(ca.MODE_ALLREDUCE, 8, 4, 4, "f32"), (ca.MODE_ALLREDUCE, 8, 2, 8, "bf16"),
                                          (ca.MODE_REDUCE_SCATTER, 8, 4, 8, "f32"),
                                          (ca.MODE_ALLREDUCE, 6, 2, 3, "f64")])
def test_tree_and_fold_plans_bit_identical(monkeypatch, mode, n, k, b, dt):
    rc = 96
    count = rc * n
    sends = [po.fill(count if mode == ca.MODE_ALLREDUCE else rc * n, dt, 0, 21, r) for r in range(n)]
    f = po.allreduce_radix_batch if mode == ca.MODE_ALLREDUCE else po.reduce_scatter_radix_batch
    ref = f(sends, k, b, dt, "sum")
    got_tree = plan_sim.simulate(mode, sends, k, b, dt, "sum")
    monkeypatch.setenv("CHR_TREE", "0")
    assert not _trees(mode, n, k, b, count if mode == ca.MODE_ALLREDUCE else rc)[0]
    got_fold = plan_sim.simulate(mode, sends, k, b, dt, "sum")
    for r in range(n):
        assert np.array_equal(got_tree[r].view(np.uint8), ref[r].view(np.uint8))
        assert np.array_equal(got_fold[r].view(np.uint8), ref[r].view(np.uint8))


def _call(comb, swaps, nl=None):
    nl = len(comb) if nl is None else nl
    leaves = (ctypes.c_void_p * max(1, nl))(*([0x1000] * nl))
    cb = bytes(bytearray(comb))
    sb = bytes(bytearray(swaps)) if swaps is not None else None
    return ca.lib().chr_reduce_tree(0x2000, leaves, nl, cb, sb, 0, ca.FLOAT32, ca.SUM, None)


def test_reduce_tree_program_validation():
    assert _call([0, 1, 1, 1, 0, 1, 1, 2], [0] * 7) == 0      # valid, n = 0: nothing to do
    assert _call([0, 1, 0, 2, 0, 1, 0, 3], None) == 0
    assert _call([1, 0], [0]) == 8                             # combine with one value on the stack
    assert _call([0, 0, 1], [0]) == 8                          # two values left
    assert _call([0, 0, 0, 0, 0, 3, 1], [0] * 4) == 8          # depth 5 > 4
    assert _call([0] + [1] * 8, [0] * 8) == 8                  # 9 leaves > 8
    assert _call([0, 1], [0], nl=0) == 1                       # no leaves


@pytest.mark.parametrize("seed", range(20))
def test_random_programs_are_valid(seed):
    rng = np.random.default_rng(seed)
    comb, swaps = random_program(rng, int(rng.integers(1, 9)))
    assert _call(comb, swaps) == 0
