"""The oracle's restatement of MPICH's pair (MAXLOC / MINLOC) and complex (SUM / PROD) element
semantics against MPICH's own MPI_Reduce_local outputs (tests/golden/pairs_reduce_local.npz, made by
tests/golden/gen_pairs.py from oracle/ref_pairs_probe) -- inputs with ties, -0 / +0, NaN payloads,
infinities and integer extremes -- and against the NaN fixture (tests/golden/nan_reduce_local.npz, made by
tests/golden/gen_nan_payloads.py): two-NaN, one-NaN and invalid operations on every floating type x op.  Bit-exact
everywhere, complex NaN parts included: the oracle writes x86's NaN rules out (orc_x86f / orc_x86d: the first
operand's NaN survives, an invalid operation gives the default NaN with its sign set) with the operand order of
MPICH's compiled loops and of libgcc's __mulsc3, as the fixture pins them."""
import json
import os

import numpy as np
import pytest

import pyoracle as po

HERE = os.path.dirname(os.path.abspath(__file__))
MAN = json.load(open(os.path.join(HERE, "golden", "pairs_manifest.json")))
FIX = np.load(os.path.join(HERE, "golden", "pairs_reduce_local.npz"), allow_pickle=False)


NAN_MAN = json.load(open(os.path.join(HERE, "golden", "nan_manifest.json")))
NAN_FIX = np.load(os.path.join(HERE, "golden", "nan_reduce_local.npz"), allow_pickle=False)


def complex_equal(a, b):
    """Bitwise, except NaN parts compare by NaN-ness (kept for callers that want the weaker check)."""
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
    assert np.array_equal(y.view(np.uint8), want.view(np.uint8))


@pytest.mark.parametrize("case", NAN_MAN["cases"], ids=lambda c: f"{c['type']}_{c['op']}")
def test_oracle_matches_mpich_nan_payloads(case):
    """Every NaN payload, NaN sign and default NaN MPICH's MPI_Reduce_local produces, byte for byte."""
    key = f"{case['type']}_{case['op']}"
    npdt = po.NP_DTYPES[case["type"]]
    x = NAN_FIX[key + "_in"].copy().view(npdt)
    y = NAN_FIX[key + "_inout"].copy().view(npdt)
    po.reduce_local(x, y, case["type"], case["op"])
    assert np.array_equal(y.view(np.uint8), NAN_FIX[key + "_out"])


def test_nan_fixture_covers_the_rules():
    """The fixture holds what it is for: two-NaN operations with distinct payloads, one-NaN operations and invalid
    operations (default NaN), in both complex parts, and the complex SUM keeps in's NaN where MPI_FLOAT's SUM keeps
    inout's."""
    def parts(key, fl):
        ut = np.uint32 if fl == np.float32 else np.uint64
        return (NAN_FIX[key + "_in"].view(ut), NAN_FIX[key + "_inout"].view(ut), NAN_FIX[key + "_out"].view(ut))
    for t, fl, dn in (("f32", np.float32, 0xFFC00000), ("cf", np.float32, 0xFFC00000),
                      ("f64", np.float64, 0xFFF8000000000000), ("cd", np.float64, 0xFFF8000000000000)):
        mb = 23 if fl == np.float32 else 52
        q = 1 << (mb - 1)
        x, y, w = parts(f"{t}_sum", fl)
        xn, yn = np.isnan(x.view(fl)), np.isnan(y.view(fl))
        both = xn & yn
        assert both.sum() > 500
        survivor = x if t in ("cf", "cd") else y
        assert np.array_equal(w[both], survivor[both] | np.array(q, dtype=x.dtype))
        assert (~xn & ~yn & np.isnan(w.view(fl))).sum() > 0 and set(w[~xn & ~yn & np.isnan(w.view(fl))]) == {dn}
        if t in ("cf", "cd"):
            for part in (0, 1):
                assert both.reshape(-1, 2)[:, part].sum() > 200
