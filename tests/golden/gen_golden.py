#!/usr/bin/env python3
"""Generate golden vectors from the REAL reference (container-only).

Builds oracle/_ref/ref_driver (the reference's algorithm files, compiled unchanged
from /root/reference against the container's MPICH 3.3.2) and runs it under
`mpiexec -n N` for a grid of (mode, n, k, b, count, dtype, op, pattern, inplace) cases.
Writes:
  tests/golden/manifest.json  one record per case: parameters, sha256 of all ranks'
                              outputs (rank-major), sha256 of the MPI library collective,
                              and the library-vs-reference difference statistics
  tests/golden/outputs.npz    full outputs (rank-major) for the small cases
Inputs are not stored: they are regenerated from (dtype, pattern, seed, rank) with the
shared generator (oracle/chiara_oracle.h).  Rerun: python tests/golden/gen_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ORACLE = os.path.join(REPO, "oracle")
sys.path.insert(0, ORACLE)
import pyoracle  # noqa: E402

MPIEXEC = "/opt/conda/bin/mpiexec"
SEED = 0xC41A5EED
STORE_LIMIT = 64 * 1024  # bytes of rank-major output stored in full


def divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


def cases_for(n):
    """Case grid for communicator size n (ids are unique across the whole grid)."""
    out = []
    ks = [2, 3, 4, 5, 8]

    def add(mode, k, b, count, dt, op, pat, inplace):
        cid = f"{mode}_n{n}_k{k}_b{b}_c{count}_{dt}_{op}_p{pat}_ip{inplace}"
        out.append(dict(id=cid, mode=mode, n=n, k=k, b=b, count=count, dtype=dt, op=op,
                        pattern=pat, seed=SEED, inplace=inplace))

    for b in divisors(n):
        for k in ks:
            if k > max(b, 2) + 1 and k != 2:
                continue  # k is clamped to b (all_reduce_radix_batch.cpp:19-21); keep one clamp probe
            # allreduce: the reference harness's own int32 pattern, plus fp32/bf16/f64 uniform
            add("ar", k, b, n * 3, "i32", "sum", pyoracle.PAT_SEQ, 0)
            add("ar", k, b, n * 64, "f32", "sum", pyoracle.PAT_UNIFORM, 0)
            add("ar", k, b, n * 5, "bf16", "sum", pyoracle.PAT_UNIFORM, 0)
            # reduce-scatter (block): recvcount odd and even
            add("rs", k, b, 7, "i32", "sum", pyoracle.PAT_SEQ, 0)
            add("rs", k, b, 33, "f32", "sum", pyoracle.PAT_UNIFORM, 0)
            # allgather_radix_batch (Allgather/main.cpp's int32 pattern; op unused)
            add("ag", k, b, 6, "i32", "sum", pyoracle.PAT_SEQ, 0)
        # a few extra dtypes / ops / in-place per geometry at k = 2 and 3
        for k in (2, 3):
            add("ar", k, b, n * 16, "f64", "sum", pyoracle.PAT_UNIFORM, 0)
            add("ar", k, b, n * 16, "i32", "sum", pyoracle.PAT_UNIFORM, 0)
            add("ar", k, b, n * 16, "f32", "max", pyoracle.PAT_UNIFORM, 0)
            add("ar", k, b, n * 16, "f32", "min", pyoracle.PAT_UNIFORM, 1)
            add("ar", k, b, n * 16, "f32", "prod", pyoracle.PAT_UNIFORM, 0)
            add("ar", k, b, n * 16, "f32", "sum", pyoracle.PAT_UNIFORM, 1)
            add("rs", k, b, 16, "bf16", "sum", pyoracle.PAT_UNIFORM, 0)
            add("rs", k, b, 16, "f32", "sum", pyoracle.PAT_UNIFORM, 1)
            add("rs", k, b, 16, "i32", "max", pyoracle.PAT_UNIFORM, 0)
            # MAX/MIN operand order: ties, signed zeros, NaN payloads (PAT_TIES)
            add("ar", k, b, n * 16, "f32", "max", pyoracle.PAT_TIES, 0)
            add("ar", k, b, n * 16, "bf16", "min", pyoracle.PAT_TIES, 0)
            add("rs", k, b, 16, "f64", "max", pyoracle.PAT_TIES, 1)
            add("ag", k, b, 33, "f32", "sum", pyoracle.PAT_UNIFORM, 0)
            add("ag", k, b, 7, "bf16", "sum", pyoracle.PAT_UNIFORM, 0)
            add("ag", k, b, 5, "f64", "sum", pyoracle.PAT_TIES, 0)
    return out


LARGE = [
    # BASELINE geometries at sizes the reference finishes in seconds (hash-only)
    dict(mode="ar", n=8, k=4, b=4, count=1 << 20, dtype="f32", op="sum"),
    dict(mode="ar", n=8, k=4, b=4, count=1 << 20, dtype="bf16", op="sum"),
    dict(mode="ar", n=8, k=2, b=2, count=1 << 20, dtype="f32", op="sum"),
    dict(mode="ar", n=8, k=4, b=8, count=1 << 20, dtype="f32", op="sum"),
    dict(mode="ar", n=8, k=3, b=4, count=1 << 20, dtype="bf16", op="sum"),
    dict(mode="ar", n=8, k=2, b=4, count=1 << 20, dtype="bf16", op="sum"),
    dict(mode="ar", n=2, k=2, b=1, count=1024, dtype="f32", op="sum"),
    dict(mode="ar", n=2, k=2, b=2, count=1024, dtype="f32", op="sum"),
    dict(mode="rs", n=2, k=2, b=1, count=1 << 18, dtype="f32", op="sum"),
    dict(mode="rs", n=2, k=2, b=2, count=1 << 18, dtype="f32", op="sum"),
    dict(mode="ar", n=4, k=2, b=2, count=1 << 18, dtype="f32", op="sum"),
    dict(mode="ar", n=4, k=4, b=4, count=1 << 18, dtype="f32", op="sum"),
    dict(mode="ag", n=8, k=4, b=4, count=1 << 16, dtype="f32", op="sum"),
    dict(mode="ag", n=16, k=3, b=4, count=1 << 14, dtype="bf16", op="sum"),
]


def mpich_cases_for(n):
    """testing/main.cpp baselines: ring, recursive doubling,
    reduce-scatter+allgather (Rabenseifner), recursive exchange and k-reduce-scatter-allgather
    (k, single_phase_recv), recursive multiplying (k)."""
    out = []

    def add(mode, k, b, count, dt, op, pat, inplace):
        cid = f"{mode}_n{n}_k{k}_b{b}_c{count}_{dt}_{op}_p{pat}_ip{inplace}"
        out.append(dict(id=cid, mode=mode, n=n, k=k, b=b, count=count, dtype=dt, op=op,
                        pattern=pat, seed=SEED, inplace=inplace))

    for mode in ("ring", "rd", "rsag"):
        for count in (1, 7, 3 * n + 1, 256, 1000):
            add(mode, 0, 0, count, "f32", "sum", pyoracle.PAT_UNIFORM, 0)
        add(mode, 0, 0, 96, "f64", "sum", pyoracle.PAT_UNIFORM, 0)   # testing/main.cpp uses double
        add(mode, 0, 0, 64, "i32", "sum", pyoracle.PAT_SEQ, 0)
        add(mode, 0, 0, 64, "bf16", "sum", pyoracle.PAT_UNIFORM, 0)
        add(mode, 0, 0, 64, "f32", "max", pyoracle.PAT_UNIFORM, 0)
        add(mode, 0, 0, 64, "f32", "sum", pyoracle.PAT_UNIFORM, 1)
        add(mode, 0, 0, 64, "f32", "max", pyoracle.PAT_TIES, 0)
        add(mode, 0, 0, 64, "f64", "min", pyoracle.PAT_TIES, 1)
        add(mode, 0, 0, 64, "bf16", "max", pyoracle.PAT_TIES, 0)
    for k in (2, 3, 4, 5):
        for spr in (0, 1):
            for count in (1, 33, 500):
                add("rx", k, spr, count, "f32", "sum", pyoracle.PAT_UNIFORM, 0)
            add("rx", k, spr, 64, "f64", "sum", pyoracle.PAT_UNIFORM, 0)
            add("rx", k, spr, 64, "i32", "sum", pyoracle.PAT_SEQ, 0)
            add("rx", k, spr, 64, "f32", "prod", pyoracle.PAT_UNIFORM, 1)
            # MPICH_do_reduce runs the running value as the FIRST operand: order-sensitive
            add("rx", k, spr, 64, "f32", "max", pyoracle.PAT_TIES, 0)
            add("rx", k, spr, 64, "f32", "min", pyoracle.PAT_TIES, 1)
            add("rx", k, spr, 64, "bf16", "max", pyoracle.PAT_TIES, 0)
            # k-reduce-scatter-allgather (k, single_phase_recv)
            for count in (1, 33, 500):
                add("krsag", k, spr, count, "f32", "sum", pyoracle.PAT_UNIFORM, 0)
            add("krsag", k, spr, 64, "f64", "sum", pyoracle.PAT_UNIFORM, 1)
            add("krsag", k, spr, 64, "i32", "sum", pyoracle.PAT_SEQ, 0)
            add("krsag", k, spr, 64, "f32", "max", pyoracle.PAT_TIES, 0)
            add("krsag", k, spr, 64, "bf16", "sum", pyoracle.PAT_UNIFORM, 0)
        # recursive multiplying (k)
        for count in (1, 33, 500):
            add("rm", k, 0, count, "f32", "sum", pyoracle.PAT_UNIFORM, 0)
        add("rm", k, 0, 64, "f64", "sum", pyoracle.PAT_UNIFORM, 1)
        add("rm", k, 0, 64, "i32", "sum", pyoracle.PAT_SEQ, 0)
        add("rm", k, 0, 64, "f32", "max", pyoracle.PAT_TIES, 0)
        add("rm", k, 0, 64, "f32", "min", pyoracle.PAT_TIES, 1)
        add("rm", k, 0, 64, "bf16", "max", pyoracle.PAT_TIES, 0)
        add("rm", k, 0, 64, "bf16", "sum", pyoracle.PAT_UNIFORM, 0)
    return out


TYPE_OPS = {  # MPI's predefined op/type table: arithmetic on every integer type, logical/bitwise too
    "i8": ("sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor"),
    "u8": ("sum", "max", "min", "land", "bxor"),
    "i16": ("sum", "prod", "max", "min", "lor", "band"),
    "u16": ("sum", "max", "min", "lxor", "bor"),
    "i32": ("land", "lor", "lxor", "band", "bor", "bxor"),
    "u32": ("sum", "prod", "max", "min", "land", "bxor"),
    "i64": ("sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor"),
    "u64": ("sum", "max", "min", "lor", "band"),
    # MPICH 3.3.2 accepts the logical ops on float and double too (C truth values; TIES data:
    # +-0, +-1, 0.5, NaN)
    "f32": ("land", "lor", "lxor"),
    "f64": ("land", "lxor"),
}


def types_cases_for(n):
    """The reference is generic over MPI_Datatype x MPI_Op (all_reduce_radix_batch.cpp:202-204,
    :234-277): the integer types beyond int32 and the logical / bitwise ops, through the radix/batch
    collectives and a few MPICH baselines.  LOR/LXOR run on the TIES pattern ({0, 1, -1, 2, 7}: zeros
    are frequent), LAND on SPARSE (1/8 zeros, so its results mix 0 and 1), arithmetic and bitwise
    ops on full-width random bits (SUM/PROD wrap)."""
    out = []

    def add(mode, k, b, count, dt, op, pat, inplace):
        cid = f"{mode}_n{n}_k{k}_b{b}_c{count}_{dt}_{op}_p{pat}_ip{inplace}"
        out.append(dict(id=cid, mode=mode, n=n, k=k, b=b, count=count, dtype=dt, op=op,
                        pattern=pat, seed=SEED, inplace=inplace))

    for dt, ops in TYPE_OPS.items():
        for op in ops:
            pat = {"land": pyoracle.PAT_SPARSE, "lor": pyoracle.PAT_TIES, "lxor": pyoracle.PAT_TIES}.get(
                op, pyoracle.PAT_UNIFORM)
            if dt in ("f32", "f64"):
                pat = pyoracle.PAT_TIES
            for i, b in enumerate(divisors(n)):
                k = (2, 3, 4)[i % 3]
                add("ar", k, b, n * 24 + (n if i % 2 else 0), dt, op, pat, i % 2)
                add("rs", k, b, 13 + i, dt, op, pat, 0)
            if op in ("sum", "max", "band", "land"):
                add("rx", 3, 0, 40, dt, op, pat, 0)
                add("ring", 0, 0, 3 * n + 5, dt, op, pat, 0)
                add("rm", 2, 0, 33, dt, op, pat, 1)
        add("ag", 2, n if n < 4 else 2, 9, dt, "sum", pyoracle.PAT_UNIFORM, 0)
    return out


def pairs_cases_for(n):
    """MPI's pair types under MAXLOC / MINLOC and the C complex types under SUM / PROD through the
    radix/batch collectives and three MPICH baselines (the reference is generic over MPI_Datatype x
    MPI_Op, all_reduce_radix_batch.cpp:202-204; its arithmetic is MPICH's MPI_Reduce_local).  The
    reference addresses its buffers with MPI_Type_size as the element stride (:238-256), which is the
    C struct's size only for MPI_FLOAT_INT, MPI_2INT and the complex types; for MPI_DOUBLE_INT,
    MPI_LONG_INT and MPI_SHORT_INT (size 12 / 12 / 6, extent 16 / 16 / 8) the expected output is MPI's
    own collective instead (modes ar_lib / rs_lib; MAXLOC / MINLOC on these values are associative
    and commutative, so every correct schedule gives those bits).  fi also runs the TIES pattern
    (-0 / +0, NaN): MPICH keeps inout on ties and NaN compares, so the operand order shows."""
    out = []

    def add(mode, k, b, count, dt, op, pat, inplace):
        cid = f"{mode}_n{n}_k{k}_b{b}_c{count}_{dt}_{op}_p{pat}_ip{inplace}"
        out.append(dict(id=cid, mode=mode, n=n, k=k, b=b, count=count, dtype=dt, op=op,
                        pattern=pat, seed=SEED, inplace=inplace))

    ref_ok = {"fi": ("maxloc", "minloc"), "2i": ("maxloc", "minloc"), "cf": ("sum", "prod"), "cd": ("sum", "prod")}
    for dt, ops in ref_ok.items():
        for op in ops:
            pats = [pyoracle.PAT_UNIFORM] + ([pyoracle.PAT_TIES] if dt == "fi" else [])
            for pat in pats:
                for i, b in enumerate(divisors(n)):
                    k = (2, 3, 4)[i % 3]
                    add("ar", k, b, n * 12 + (n if i % 2 else 0), dt, op, pat, i % 2)
                    add("rs", k, b, 7 + i, dt, op, pat, 0)
                add("rx", 3, 0, 40, dt, op, pat, 0)
                add("ring", 0, 0, 3 * n + 5, dt, op, pat, 0)
                add("rm", 2, 0, 33, dt, op, pat, 1)
        add("ag", 2, 2 if n >= 4 and n % 2 == 0 else n, 9, dt, ops[0], pyoracle.PAT_UNIFORM, 0)
    for dt in ("di", "li", "si"):
        for op in ("maxloc", "minloc"):
            for i, b in enumerate(divisors(n)):
                k = (2, 3, 4)[i % 3]
                add("ar_lib", k, b, n * 12 + (n if i % 2 else 0), dt, op, pyoracle.PAT_UNIFORM, 0)
                add("rs_lib", k, b, 7 + i, dt, op, pyoracle.PAT_UNIFORM, 0)
    return out


def rsmpich_cases_for(n):
    """testing/mpich_implementations/reduce_scatter/: radix (k), recursive halving, recursive
    doubling (relays for non-powers of two) and pairwise, driven by that directory's main.cpp
    (MPI_DOUBLE, MPI_SUM, MPI_Reduce_scatter_block semantics; count = recvcount)."""
    out = []

    def add(mode, k, count, dt, op, pat, inplace):
        cid = f"{mode}_n{n}_k{k}_c{count}_{dt}_{op}_p{pat}_ip{inplace}"
        out.append(dict(id=cid, mode=mode, n=n, k=k, b=0, count=count, dtype=dt, op=op,
                        pattern=pat, seed=SEED, inplace=inplace))

    for mode in ("rs_halving", "rs_doubling", "rs_pairwise"):
        for count in (1, 7, 33):
            add(mode, 0, count, "f64", "sum", pyoracle.PAT_UNIFORM, 0)  # the harness's datatype
            add(mode, 0, count, "f32", "sum", pyoracle.PAT_UNIFORM, count % 2)
        add(mode, 0, 16, "i32", "sum", pyoracle.PAT_SEQ, 0)
        add(mode, 0, 16, "bf16", "sum", pyoracle.PAT_UNIFORM, 0)
        add(mode, 0, 16, "f32", "max", pyoracle.PAT_TIES, 0)
        add(mode, 0, 16, "f64", "min", pyoracle.PAT_TIES, 1)
        add(mode, 0, 16, "bf16", "max", pyoracle.PAT_TIES, 1)
        add(mode, 0, 16, "i64", "bxor", pyoracle.PAT_UNIFORM, 0)
    for k in (2, 3, 4, 5, 8):
        for count in (1, 13):
            add("rs_radix", k, count, "f64", "sum", pyoracle.PAT_UNIFORM, 0)
            add("rs_radix", k, count, "f32", "sum", pyoracle.PAT_UNIFORM, 1)
        add("rs_radix", k, 16, "i32", "sum", pyoracle.PAT_SEQ, 0)
        add("rs_radix", k, 16, "bf16", "sum", pyoracle.PAT_UNIFORM, 0)
        add("rs_radix", k, 16, "f32", "max", pyoracle.PAT_TIES, 0)
        add("rs_radix", k, 16, "f64", "min", pyoracle.PAT_TIES, 1)
        add("rs_radix", k, 16, "u16", "land", pyoracle.PAT_SPARSE, 0)
    return out


def phases_cases_for(n):
    """CHiArA's phases as stand-alone functions (testing/custom_implementations/work_dir/reduce_scatter/):
    irs = intra_reduce_scatter_radix_batch (k, b), ilr = inter_reduce_linear (b), isc =
    intra_scatter_radix_batch (k, b); count = recvcount.  Every divisor b of n (stages, leftover
    stages, step-1 folds of b not a power of k), the self-tests' own parameters (irs: recvcount 1, k 2,
    b 4; ilr: b 2; isc: k 7, b 9, recvcount 7)."""
    out = []

    def add(mode, k, b, count, dt, op, pat, inplace):
        cid = f"{mode}_n{n}_k{k}_b{b}_c{count}_{dt}_{op}_p{pat}_ip{inplace}"
        out.append(dict(id=cid, mode=mode, n=n, k=k, b=b, count=count, dtype=dt, op=op,
                        pattern=pat, seed=SEED, inplace=inplace))

    for b in divisors(n):
        for k in (2, 3, 4):
            add("irs", k, b, 3, "f32", "sum", pyoracle.PAT_UNIFORM, 0)
            add("irs", k, b, 5, "i32", "sum", pyoracle.PAT_SEQ, k % 2)
            add("isc", k, b, 5, "i32", "sum", pyoracle.PAT_SEQ, 0)
        add("irs", 2, b, 16, "f64", "max", pyoracle.PAT_TIES, 0)
        add("irs", 3, b, 16, "bf16", "sum", pyoracle.PAT_UNIFORM, 1)
        add("irs", 4, b, 16, "f32", "min", pyoracle.PAT_TIES, 0)
        add("irs", 2, b, 33, "u8", "bxor", pyoracle.PAT_UNIFORM, 0)
        add("ilr", 0, b, 3, "f32", "sum", pyoracle.PAT_UNIFORM, 0)
        add("ilr", 0, b, 7, "i32", "sum", pyoracle.PAT_SEQ, 0)
        add("ilr", 0, b, 16, "f64", "max", pyoracle.PAT_TIES, 0)
        add("ilr", 0, b, 16, "bf16", "sum", pyoracle.PAT_UNIFORM, 0)
        add("isc", 2, b, 16, "f64", "sum", pyoracle.PAT_UNIFORM, 0)
        add("isc", 5, b, 33, "u8", "sum", pyoracle.PAT_UNIFORM, 0)
        # MPI's pair types (MAXLOC / MINLOC, ties) and C complex types whose MPI_Type_size is their extent
        # (the reference strides its buffers by MPI_Type_size, intra_reduce_scatter_radix.cpp:238)
        add("irs", 2, b, 5, "fi", "maxloc", pyoracle.PAT_TIES, 0)
        add("irs", 3, b, 5, "cf", "sum", pyoracle.PAT_UNIFORM, 0)
        add("ilr", 0, b, 5, "2i", "minloc", pyoracle.PAT_TIES, 0)
        add("ilr", 0, b, 4, "cd", "prod", pyoracle.PAT_UNIFORM, 0)
        add("isc", 2, b, 3, "cd", "sum", pyoracle.PAT_UNIFORM, 0)
    if n % 4 == 0:
        add("irs", 2, 4, 1, "i32", "sum", pyoracle.PAT_SEQ, 0)  # intra_reduce_scatter_radix.cpp:564-566
    if n % 2 == 0:
        add("ilr", 0, 2, 1, "i32", "sum", pyoracle.PAT_SEQ, 0)  # inter_linear_reduce.cpp:102-103
    if n % 9 == 0:
        add("isc", 7, 9, 7, "i32", "sum", pyoracle.PAT_SEQ, 0)  # intra_scatter_radix_batch.cpp:155-157
    return out


def userop_cases_for(n):
    """A user-defined, non-commutative MPI op (MPI_Op_create(halfadd, commute = 0): inout = in * 0.5f + inout on
    MPI_FLOAT, oracle/ref_driver.cpp) through CHiArA's own collectives: the radix/batch allreduce and
    reduce-scatter at every divisor b (in place too) and the stand-alone phases.  The reference is generic over
    MPI_Op (all_reduce_radix_batch.cpp:202-204) and reduces with MPI_Reduce_local, which calls the user function; a
    non-commutative op makes every operand order visible in the bits.  (The MPICH baselines, which branch on
    MPI_Op_commutative, have their own suite: usermpich_cases_for.)"""
    out = []

    def add(mode, k, b, count, inplace, dt="f32"):
        cid = f"{mode}_n{n}_k{k}_b{b}_c{count}_{dt}_user_halfadd_p0_ip{inplace}"
        out.append(dict(id=cid, mode=mode, n=n, k=k, b=b, count=count, dtype=dt, op="user_halfadd",
                        pattern=pyoracle.PAT_UNIFORM, seed=SEED, inplace=inplace))

    for i, b in enumerate(divisors(n)):
        for k in (2, 3, 4):
            add("ar", k, b, n * 16 + (n if k == 3 else 0), (i + k) % 2)
            add("rs", k, b, 9 + k, 0)
        # the same function on MPI_DOUBLE (in * 0.5 + inout) and MPI_INT (3 * in + inout, wrapping): the user-op
        # path at 8- and 4-byte integer elements
        for j, dt in enumerate(("f64", "i32")):
            k = (2, 3, 4)[(i + j) % 3]
            add("ar", k, b, n * 8 + (n if j else 0), (i + j) % 2, dt)
            add("rs", k, b, 7 + j, 0, dt)
    for b in divisors(n):
        add("irs", 2, b, 5, 0)
        add("ilr", 0, b, 4, 0)
        add("irs", 3, b, 6, 0, "f64")
        add("ilr", 0, b, 3, 0, "i32")
    return out


def usermpich_cases_for(n):
    """The MPICH baselines (testing/mpich_implementations/{all_reduce,reduce_scatter}/) with a user-defined op: the
    halfadd function created non-commutative (user_halfadd) and commutative (user_halfadd_c).  The baselines branch
    on MPI_Op_commutative (allreduce_recursive_doubling.cpp:69, reduce_scatter_recursive_doubling.cpp:134,
    allreduce_recexch.cpp:343, :378) or refuse a non-commutative op with MPI_ERR_OP
    (allreduce_k_reduce_scatter_allgather.cpp:279-283; allreduce_recursive_multiplying.cpp:46-49 at a size that is
    not a power of k); the arithmetic is non-commutative either way, so both paths show in the bits.  The reference's
    return codes are recorded (ref_rc)."""
    out = []

    def add(mode, k, b, count, op, inplace):
        cid = f"{mode}_n{n}_k{k}_b{b}_c{count}_f32_{op}_p0_ip{inplace}"
        out.append(dict(id=cid, mode=mode, n=n, k=k, b=b, count=count, dtype="f32", op=op,
                        pattern=pyoracle.PAT_UNIFORM, seed=SEED, inplace=inplace))

    for j, op in enumerate(("user_halfadd", "user_halfadd_c")):
        for mode in ("ring", "rd", "rsag"):
            for i, count in enumerate((7, 3 * n + 1, 64)):
                add(mode, 0, 0, count, op, (i + j) % 2)
        for k in (2, 3, 4, 5):
            for spr in (0, 1):
                add("rx", k, spr, 33, op, (k + spr) % 2)
        for k in (2, 3, 4):
            add("krsag", k, 0, 33, op, 0)
            add("rm", k, 0, 33, op, k % 2)
        for mode in ("rs_halving", "rs_doubling", "rs_pairwise"):
            for i, count in enumerate((1, 7, 16)):
                add(mode, 0, 0, count, op, (i + j) % 2)
        for k in (2, 3, 4, 5):
            add("rs_radix", k, 0, 13, op, k % 2)
    return out


def run_n(n, cases, tmp):
    cf = os.path.join(tmp, f"cases_{n}.txt")
    with open(cf, "w") as f:
        for c in cases:
            f.write(f"{c['id']} {c['mode']} {c['k']} {c['b']} {c['count']} {c['dtype']} {c['op']} "
                    f"{c['pattern']} {c['seed']} {c['inplace']}\n")
    cmd = [MPIEXEC, "-n", str(n)]
    if n <= os.cpu_count():
        cmd[1:1] = ["-bind-to", "core"]
    cmd += [os.path.join(ORACLE, "_ref", "ref_driver"), cf, tmp]
    subprocess.check_call(cmd, timeout=600)


def main():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "ref", "liboracle.so"])
    which = sys.argv[1] if len(sys.argv) > 1 else "radix_batch"
    all_cases = []
    if which == "mpich":
        for n in (1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 16):
            all_cases += mpich_cases_for(n)
        prefix = "mpich_"
    elif which == "rsmpich":
        for n in (1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 16):
            all_cases += rsmpich_cases_for(n)
        prefix = "rsmpich_"
    elif which == "phases":
        for n in (1, 2, 3, 4, 5, 6, 8, 9, 12, 16, 18):
            all_cases += phases_cases_for(n)
        prefix = "phases_"
    elif which == "types":
        for n in (2, 3, 4, 6, 8):
            all_cases += types_cases_for(n)
        prefix = "types_"
    elif which == "userop":
        for n in (2, 3, 4, 6, 8):
            all_cases += userop_cases_for(n)
        prefix = "userop_"
    elif which == "usermpich":
        for n in (1, 2, 3, 4, 5, 6, 7, 8, 9):
            all_cases += usermpich_cases_for(n)
        prefix = "usermpich_"
    elif which == "pairs":
        for n in (2, 3, 4, 5, 6, 8):
            all_cases += pairs_cases_for(n)
        prefix = "pairtypes_"
    else:
        prefix = ""
        for n in (1, 2, 3, 4, 5, 6, 8, 9, 12, 16):
            all_cases += cases_for(n)
        for c in LARGE:
            c = dict(c, pattern=pyoracle.PAT_UNIFORM, seed=SEED, inplace=0)
            c["id"] = (f"{c['mode']}_n{c['n']}_k{c['k']}_b{c['b']}_c{c['count']}_{c['dtype']}_{c['op']}"
                       f"_p{c['pattern']}_ip0_large")
            all_cases.append(c)
    manifest, arrays = [], {}
    with tempfile.TemporaryDirectory() as tmp:
        by_n = {}
        for c in all_cases:
            by_n.setdefault(c["n"], []).append(c)
        for n, cs in sorted(by_n.items()):
            print(f"n={n}: {len(cs)} cases", flush=True)
            run_n(n, cs, tmp)
        for c in all_cases:
            out = open(os.path.join(tmp, c["id"] + ".out"), "rb").read()
            libb = open(os.path.join(tmp, c["id"] + ".lib"), "rb").read()
            rec = dict(c)
            if which == "usermpich":  # every rank's return code (MPI_ERR_OP where the baseline refuses the op)
                rec["ref_rc"] = [int(x) for x in open(os.path.join(tmp, c["id"] + ".rc")).read().split()]
            rec["sha256"] = hashlib.sha256(out).hexdigest()
            rec["sha256_lib"] = hashlib.sha256(libb).hexdigest()
            npdt = pyoracle.NP_DTYPES[c["dtype"]]
            a = np.frombuffer(out, dtype=npdt)
            lb = np.frombuffer(libb, dtype=npdt)
            if c["dtype"] in pyoracle.PAIR_DTYPES + pyoracle.COMPLEX_DTYPES:
                # element-wise byte comparison (structured / complex elements)
                isz = np.dtype(npdt).itemsize
                ab = np.frombuffer(out, dtype=np.uint8).reshape(-1, isz)
                lbb = np.frombuffer(libb, dtype=np.uint8).reshape(-1, isz)
                rec["n_diff_vs_lib"] = int(np.count_nonzero((ab != lbb).any(axis=1)))
                if c["dtype"] in pyoracle.COMPLEX_DTYPES:
                    d = np.abs(a.astype(np.complex128) - lb.astype(np.complex128))
                    rec["max_abs_diff_vs_lib"] = float(np.max(d[np.isfinite(d)])) if np.isfinite(d).any() else 0.0
                else:
                    rec["max_abs_diff_vs_lib"] = 0.0 if rec["n_diff_vs_lib"] == 0 else float("nan")
                rec["stored"] = len(out) <= STORE_LIMIT
                if rec["stored"]:
                    arrays[c["id"]] = np.frombuffer(out, dtype=np.uint8).copy()
                    arrays[c["id"] + "__lib"] = np.frombuffer(libb, dtype=np.uint8).copy()
                manifest.append(rec)
                continue
            if c["dtype"] == "bf16":
                af = (a.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
                lf = (lb.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
            elif c["dtype"] in ("i64", "u64"):  # exact integer difference (doubles lose bits)
                af, lf = a.view(np.int64).astype(object), lb.view(np.int64).astype(object)
            else:
                af, lf = a.astype(np.float64), lb.astype(np.float64)
            rec["n_diff_vs_lib"] = int(np.count_nonzero(a != lb))
            if af.dtype == object:
                rec["max_abs_diff_vs_lib"] = float(max((abs(int(x) - int(y)) for x, y in zip(af, lf)), default=0))
            else:
                ok = np.isfinite(af) & np.isfinite(lf)
                rec["max_abs_diff_vs_lib"] = float(np.max(np.abs(af[ok] - lf[ok]))) if ok.any() else 0.0
            rec["stored"] = len(out) <= STORE_LIMIT
            if rec["stored"]:
                arrays[c["id"]] = a.copy()
                arrays[c["id"] + "__lib"] = lb.copy()
            manifest.append(rec)
    ref_desc = ("testing/custom_implementations/work_dir/reduce_scatter/{intra_reduce_scatter_radix,"
                "inter_linear_reduce,intra_scatter_radix_batch}.cpp" if which == "phases" else
                "testing/mpich_implementations/reduce_scatter/{reduce_scatter_radix,"
                "reduce_scatter_recursive_halving,reduce_scatter_recursive_doubling,reduce_scatter_pairwise}.cpp"
                if which == "rsmpich" else
                "Fugaku_experiments/{Allreduce,Reduce-scatter,Allgather} + testing/mpich_implementations/"
                "all_reduce/{allreduce_ring,allreduce_recexch,allreduce_recursive_multiplying}.cpp, integer types "
                "beyond int32 and the logical/bitwise ops" if which == "types" else
                "Fugaku_experiments/{Allreduce,Reduce-scatter,Allgather} + testing/mpich_implementations/"
                "all_reduce/{allreduce_ring,allreduce_recexch,allreduce_recursive_multiplying}.cpp, MPI pair types "
                "(MAXLOC/MINLOC) and C complex types (SUM/PROD); ar_lib/rs_lib: MPI_Allreduce / "
                "MPI_Reduce_scatter_block (see pairs_cases_for)" if which == "pairs" else
                "Fugaku_experiments/{Allreduce,Reduce-scatter} + testing/custom_implementations/work_dir/"
                "reduce_scatter/{intra_reduce_scatter_radix,inter_linear_reduce}.cpp, with a user-defined "
                "non-commutative MPI_Op (see userop_cases_for)" if which == "userop" else
                "testing/mpich_implementations/{all_reduce,reduce_scatter}/*.cpp with a user-defined MPI_Op, created "
                "non-commutative and commutative (see usermpich_cases_for)" if which == "usermpich" else
                "testing/mpich_implementations/all_reduce/{allreduce_ring,allreduce_recursive_doubling,"
                "allreduce_reduce_scatter_allgather,allreduce_recexch,allreduce_k_reduce_scatter_allgather,"
                "allreduce_recursive_multiplying}.cpp" if which == "mpich" else
                "Fugaku_experiments/{Allreduce/all_reduce_radix_batch.cpp,Reduce-scatter/reduce_scatter_radix_batch.cpp,"
                "Allgather/all_gather_radix_batch_1_0.cpp}")
    with open(os.path.join(HERE, prefix + "manifest.json"), "w") as f:
        json.dump({"generator": f"tests/golden/gen_golden.py {which}",
                   "reference": ref_desc + " @ 2025-11-21, MPICH 3.3.2", "seed": SEED, "cases": manifest},
                  f, indent=0)
    np.savez_compressed(os.path.join(HERE, prefix + "outputs.npz"), **arrays)
    print(f"{len(manifest)} cases, {len(arrays) // 2} stored in full")


if __name__ == "__main__":
    main()
