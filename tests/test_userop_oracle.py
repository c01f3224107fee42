"""The user-op path's oracle against the reference itself: a user-defined, non-commutative MPI_Op
(MPI_Op_create(halfadd, commute = 0): inout = in * 0.5f + inout on MPI_FLOAT, in * 0.5 + inout on MPI_DOUBLE,
3 * in + inout on MPI_INT) through the reference's radix/batch
allreduce and reduce-scatter and CHiArA's phases, compiled unchanged against MPICH 3.3.2
(tests/golden/userop_outputs.npz, tests/golden/gen_golden.py userop).  Every operand order the reference takes shows
in the bits of a non-commutative op; the oracle restates the op once (chiara_oracle.c ORC_USER_HALFADD) and must
reproduce every case bit for bit.  The device path (chr_op_create, tests/userop/halfadd_op.hip) is checked against
the same goldens in tests/test_gpu_user_op.py."""
import json
import os

import numpy as np
import pytest

import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
MAN = json.load(open(os.path.join(HERE, "golden", "userop_manifest.json")))
FIX = np.load(os.path.join(HERE, "golden", "userop_outputs.npz"), allow_pickle=False)


def oracle_outputs(c):
    """All ranks' outputs of golden case c by the oracle (rank-major, as the fixture stores them)."""
    n, k, b, count, mode = c["n"], c["k"], c["b"], c["count"], c["mode"]
    ip = bool(c["inplace"])
    if mode in ("irs", "ilr"):
        in_n, _ = po.phase_sizes(mode, n, b, count)
        xs = [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r, in_n) for r in range(n)]
        return po.phase_collective(mode, xs, c["dtype"], c["op"], k, b, count, inplace=ip)
    in_n = count * n if mode == "rs" else count
    xs = [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r, in_n) for r in range(n)]
    if mode == "ar":
        return po.allreduce_radix_batch(xs, k, b, c["dtype"], c["op"], inplace=ip)
    assert mode == "rs", mode
    return po.reduce_scatter_radix_batch(xs, k, b, c["dtype"], c["op"], inplace=ip)


def test_fixture_is_non_commutative_in_the_bits():
    """The op is non-commutative, so the fixture pins operand order: swapping in / inout changes results."""
    x = po.fill(4096, "f32", po.PAT_UNIFORM, 5, 0)
    y = po.fill(4096, "f32", po.PAT_UNIFORM, 5, 1)
    a, b2 = y.copy(), x.copy()
    po.reduce_local(x, a, "f32", "user_halfadd")
    po.reduce_local(y, b2, "f32", "user_halfadd")
    assert not np.array_equal(a.view(np.uint32), b2.view(np.uint32))
    assert len(MAN["cases"]) >= 200 and {c["mode"] for c in MAN["cases"]} == {"ar", "rs", "irs", "ilr"}
    assert {c["dtype"] for c in MAN["cases"]} == {"f32", "f64", "i32"}


@pytest.mark.parametrize("case", MAN["cases"], ids=lambda c: c["id"])
def test_oracle_matches_reference_with_user_op(case):
    got = np.concatenate([np.asarray(o).ravel() for o in oracle_outputs(case)])
    want = FIX[case["id"]]
    assert got.dtype == want.dtype and np.array_equal(got.view(np.uint8), want.view(np.uint8))
