"""The oracle's restatement of MPICH's pair (MAXLOC / MINLOC) and complex (SUM / PROD) element
semantics against MPICH's own MPI_Reduce_local outputs (tests/golden/pairs_reduce_local.npz, made by
tests/golden/gen_pairs.py from oracle/ref_pairs_probe) -- inputs with ties, -0 / +0, NaN payloads,
infinities and integer extremes.  Bit-exact, except that for complex results that are NaN only the
NaN-ness is compared: an x86 invalid operation (inf - inf, 0 * inf) yields the negative default
NaN, and which operand's NaN payload survives an SSE add is instruction-order dependent, neither of
which C (or the device) pins down."""
import json
import os

import numpy as np
import pytest

import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
MAN = json.load(open(os.path.join(HERE, "golden", "pairs_manifest.json")))
FIX = np.load(os.path.join(HERE, "golden", "pairs_reduce_local.npz"), allow_pickle=False)


def complex_equal(a, b):
    """Bitwise, except NaN parts compare by NaN-ness."""
    ok = True
    for part in ("real", "imag"):
        x, y = getattr(a, part), getattr(b, part)
        nan = np.isnan(x) & np.isnan(y)
        ok &= bool(np.all(nan | (x.view(f"u{x.itemsize}") == y.view(f"u{y.itemsize}"))))
    return ok


def test_manifest_is_mpichs_table():
    t = MAN["table"]
    for d in po.PAIR_DTYPES:
        assert t[d]["ops"] == ["maxloc", "minloc"] and t[d]["extent"] == po.NP_DTYPES[d].itemsize
    for d in po.COMPLEX_DTYPES:
        assert t[d]["ops"] == ["sum", "prod"] and t[d]["extent"] == np.dtype(po.NP_DTYPES[d]).itemsize
    # the three types whose MPI_Type_size differs from their extent (the reference addresses its
    # buffers with MPI_Type_size, all_reduce_radix_batch.cpp:238-256)
    assert {d for d in t if t[d]["size"] != t[d]["extent"]} >= {"di", "li", "si"}
    for d in po.PAIR_DTYPES + po.COMPLEX_DTYPES:
        for op in po.OPS:
            assert po.valid(d, op) == (op in t[d]["ops"]), (d, op)


@pytest.mark.parametrize("case", MAN["cases"], ids=lambda c: f"{c['type']}_{c['op']}")
def test_oracle_matches_mpich_reduce_local(case):
    key = f"{case['type']}_{case['op']}"
    npdt = po.NP_DTYPES[case["type"]]
    # copy as bytes: a copy of a structured array does not keep its padding bytes
    x = FIX[key + "_in"].copy().view(npdt)
    y = FIX[key + "_inout"].copy().view(npdt)
    want = FIX[key + "_out"].view(npdt)
    po.reduce_local(x, y, case["type"], case["op"])
    if case["type"] in po.COMPLEX_DTYPES:
        assert complex_equal(y, want)
    else:
        assert np.array_equal(y.view(np.uint8), want.view(np.uint8))
