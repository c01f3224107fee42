"""Pin the oracle (CPU restatement) against the real reference's golden vectors.

tests/golden/ was produced by tests/golden/gen_golden.py, which runs the reference's
all_reduce_radix_batch.cpp / reduce_scatter_radix_batch.cpp unchanged under MPICH.
Every case must match bit-for-bit (sha256 of all ranks' outputs).
"""
import hashlib

import numpy as np
import pytest

import pyoracle as po


def _run_oracle(c):
    n = c["n"]
    in_n = c["count"] * n if c["mode"] == "rs" else c["count"]
    sends = [po.fill(in_n, c["dtype"], c["pattern"], c["seed"], r) for r in range(n)]
    if c["mode"] == "ag":
        return po.allgather_radix_batch(sends, c["k"], c["b"], c["dtype"], inplace=bool(c["inplace"]))
    f = po.allreduce_radix_batch if c["mode"] == "ar" else po.reduce_scatter_radix_batch
    return f(sends, c["k"], c["b"], c["dtype"], c["op"], inplace=bool(c["inplace"]))


def test_golden_manifest_is_complete(golden):
    cases, arrays = golden
    assert len(cases) > 1000
    assert len({c["id"] for c in cases}) == len(cases)
    modes = {(c["mode"], c["dtype"], c["op"]) for c in cases}
    for need in [("ar", "i32", "sum"), ("ar", "f32", "sum"), ("ar", "bf16", "sum"), ("rs", "f32", "sum"),
                 ("ag", "i32", "sum"), ("ag", "f64", "sum"),
                 ("ar", "f32", "max"), ("ar", "f64", "sum"), ("rs", "bf16", "sum")]:
        assert need in modes


def test_oracle_matches_reference_bit_exact(golden):
    cases, arrays = golden
    bad = []
    for c in cases:
        outs = _run_oracle(c)
        h = hashlib.sha256(b"".join(o.tobytes() for o in outs)).hexdigest()
        if h != c["sha256"]:
            bad.append(c["id"])
        elif c["stored"]:
            np.testing.assert_array_equal(np.concatenate(outs), arrays[c["id"]])
    assert not bad, f"{len(bad)} oracle/reference mismatches, e.g. {bad[:5]}"


def test_reference_exact_on_integers(golden):
    """The reference harness's own is_correct: int32 results equal MPI's collective."""
    cases, _ = golden
    ints = [c for c in cases if c["dtype"] == "i32"]
    assert ints and all(c["n_diff_vs_lib"] == 0 for c in ints)


def test_reference_allgather_equals_mpi_allgather(golden):
    """allgather_radix_batch is pure data movement: on every golden geometry its bytes equal
    MPI_Allgather's (which is why the product may route blocks differently)."""
    cases, _ = golden
    ag = [c for c in cases if c["mode"] == "ag"]
    assert len(ag) > 150 and all(c["sha256"] == c["sha256_lib"] for c in ag)


def test_float_tolerance_vs_library(golden):
    """fp32 SUM vs MPI_Allreduce is not bit-exact for n>2 (different association);
    bound: |x - lib| <= (n-1) * 2^-23 * sum|x_i|, with |x_i| < 1 here."""
    cases, _ = golden
    for c in cases:
        if c["dtype"] == "f32" and c["op"] == "sum":
            assert c["max_abs_diff_vs_lib"] <= (c["n"] - 1) * 2.0 ** -23 * c["n"] * 2
            if c["n"] <= 2:
                assert c["n_diff_vs_lib"] == 0


def test_reduce_local_semantics():
    # MPICH 3.3.2 loop (MPIR_OP_TYPE_REDUCE_CASE, a = inoutvec, b = invec):
    # inout = inout > in ? inout : in -- `in` wins on ties and whenever a NaN is compared.
    # Pinned by the PAT_TIES golden cases (gen_golden.py), which the reference produced.
    a = np.array([1.0, -0.0, np.nan, 3.0], dtype=np.float32)
    b = np.array([2.0, 0.0, 1.0, np.nan], dtype=np.float32)
    out = po.reduce_local(a, b.copy(), "f32", "max")
    assert out[0] == 2.0 and np.signbit(out[1])
    assert np.isnan(out[2]) and out[3] == 3.0
    out = po.reduce_local(a, b.copy(), "f32", "min")
    assert out[0] == 1.0 and np.signbit(out[1])
    assert np.isnan(out[2]) and out[3] == 3.0


def test_golden_has_tie_cases(golden):
    cases, _ = golden
    ties = [c for c in cases if c["pattern"] == po.PAT_TIES]
    assert {(c["mode"], c["dtype"], c["op"]) for c in ties} >= {("ar", "f32", "max"), ("ar", "bf16", "min"),
                                                               ("rs", "f64", "max")}


@pytest.mark.parametrize("mode,n,k,b,dtype", [
    ("ar", 8, 4, 4, "f32"), ("ar", 8, 4, 4, "bf16"), ("ar", 8, 2, 2, "f32"), ("ar", 8, 4, 8, "f32"),
    ("ar", 6, 2, 3, "bf16"), ("ar", 12, 3, 4, "f32"), ("ar", 16, 4, 4, "i32"), ("rs", 8, 4, 4, "f32"),
    ("rs", 2, 2, 1, "f32"), ("rs", 6, 3, 6, "bf16"),
])
def test_block_window_property(mode, n, k, b, dtype):
    """The full-size parity tests check BASELINE-size outputs window by window: every rank's
    output restricted to the window [off, off+w) of each recvcount block equals the collective
    run on the inputs restricted to the same windows (pyoracle.window_inputs).  Pinned here on
    the oracle itself, windows at the start, middle and end of the blocks, fold geometries
    (b not a power of k) included."""
    per = 96  # recvcount of the full call
    count = per * n
    full_in = [po.fill(count, dtype, po.PAT_UNIFORM, 11, r) for r in range(n)]
    f = po.allreduce_radix_batch if mode == "ar" else po.reduce_scatter_radix_batch
    full = f(full_in, k, b, dtype, "sum")
    for off, w in ((0, 8), (40, 16), (per - 5, 5)):
        win_in = po.window_inputs(n, count, off, w, dtype, po.PAT_UNIFORM, 11)
        for r in range(n):
            np.testing.assert_array_equal(win_in[r], full_in[r][po.block_window(n, per, off, w)])
        got = f(win_in, k, b, dtype, "sum")
        for r in range(n):
            want = full[r][po.block_window(n, per, off, w)] if mode == "ar" else full[r][off:off + w]
            np.testing.assert_array_equal(got[r].view(np.uint8), want.view(np.uint8))


def _oracle_outputs(c):
    n, dt = c["n"], c["dtype"]
    mode = {"ar_lib": "ar", "rs_lib": "rs"}.get(c["mode"], c["mode"])  # MPI's collective: same result
    in_n = c["count"] * n if mode == "rs" else c["count"]
    sends = [po.fill(in_n, dt, c["pattern"], c["seed"], r) for r in range(n)]
    ip = bool(c["inplace"])
    c = dict(c, mode=mode)
    if c["mode"] == "ar":
        return po.allreduce_radix_batch(sends, c["k"], c["b"], dt, c["op"], ip)
    if c["mode"] == "rs":
        return po.reduce_scatter_radix_batch(sends, c["k"], c["b"], dt, c["op"], ip)
    if c["mode"] == "ag":
        return po.allgather_radix_batch(sends, c["k"], c["b"], dt, ip)
    return po.mpich_allreduce(c["mode"], sends, dt, c["op"], k=c["k"], inplace=ip)


def test_oracle_matches_reference_on_integer_types_and_logical_bitwise_ops(golden_types):
    """MPI_Datatype x MPI_Op beyond int32 SUM (all_reduce_radix_batch.cpp:202-204, :234-277):
    (u)int8/16/64, uint32 and LAND/LOR/LXOR/BAND/BOR/BXOR through the radix/batch collectives and
    three MPICH baselines, every case bit-exact vs the reference run here under MPICH 3.3.2, and
    the reference equal to MPI's own collective (integer ops are associative)."""
    cases, arrays = golden_types
    assert len(cases) > 1500
    assert {c["dtype"] for c in cases} == {"i8", "u8", "i16", "u16", "i32", "u32", "i64", "u64", "f32", "f64"}
    assert {c["op"] for c in cases} >= {"sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor"}
    bad = [c["id"] for c in cases
           if hashlib.sha256(b"".join(o.tobytes() for o in _oracle_outputs(c))).hexdigest() != c["sha256"]]
    assert not bad, bad[:5]
    assert all(c["n_diff_vs_lib"] == 0 for c in cases)
    # the logical ops produce both values somewhere (the SPARSE / TIES patterns make them non-trivial)
    for op in ("land", "lor", "lxor"):
        vals = set()
        for c in cases:
            if c["op"] == op:
                vals |= set(np.unique(arrays[c["id"]]).tolist())
        assert vals == {0, 1}, (op, vals)


def test_oracle_matches_reference_on_pair_and_complex_types(golden_pairtypes):
    """MPI_MAXLOC / MPI_MINLOC on the five pair types and SUM / PROD on the C complex types through the
    radix/batch collectives, allgather and three MPICH baselines: bit-exact vs the reference run here
    under MPICH 3.3.2 (MPI_FLOAT_INT, MPI_2INT, complex; the TIES pattern's -0 / +0 and NaN make the
    operand order visible) and vs MPI's own collective for MPI_DOUBLE_INT / MPI_LONG_INT /
    MPI_SHORT_INT, whose MPI_Type_size (12 / 12 / 6) the reference would take for their stride
    (all_reduce_radix_batch.cpp:238-256, gen_golden.py pairs_cases_for)."""
    cases, arrays = golden_pairtypes
    assert len(cases) > 700
    assert {c["dtype"] for c in cases} == set(po.PAIR_DTYPES + po.COMPLEX_DTYPES)
    bad = [c["id"] for c in cases
           if hashlib.sha256(b"".join(o.tobytes() for o in _oracle_outputs(c))).hexdigest() != c["sha256"]]
    assert not bad, bad[:5]
    # without NaN / signed zeros the reference's MAXLOC / MINLOC equal MPI's collective (order-free)
    assert all(c["n_diff_vs_lib"] == 0 for c in cases if c["dtype"] in ("fi", "2i") and c["pattern"] == 0)
