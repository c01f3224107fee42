#!/usr/bin/env python3
"""Fixture of MPICH's NaN and invalid-operation results, container-only: MPI_Reduce_local(in, inout) computed by
MPICH 3.3.2 itself (oracle/_ref/ref_pairs_probe, `make -C oracle ref_pairs`) on inputs made here, for every floating
type x op where the result can carry a NaN:

* f32 / f64 SUM and PROD (MPI_FLOAT / MPI_DOUBLE);
* cf / cd SUM and PROD (MPI_C_FLOAT_COMPLEX / MPI_C_DOUBLE_COMPLEX), the real and the imaginary part drawn
  independently;
* fi / di MAXLOC and MINLOC (MPI_FLOAT_INT / MPI_DOUBLE_INT).

Every NaN carries a payload that names its side (in = 1, inout = 2), its part (re = 1, im = 2) and its element, and
comes quiet or signalling with either sign; the other values are +-0, +-inf, +-1, 2.5, values whose products
overflow, and normal random numbers, so the fixture holds two-NaN operations (whose survivor IEEE 754 leaves open),
one-NaN operations, and invalid operations (inf - inf, 0 * inf: x86's default NaN) on both sides of every add,
subtract and multiply of MPICH's loops, libgcc's complex multiply included.  The first 512 elements are NaN in every
part on both sides.  Writes tests/golden/nan_reduce_local.npz (inputs and MPICH's outputs, raw bytes) and
tests/golden/nan_manifest.json.  Rerun: python tests/golden/gen_nan_payloads.py
"""
import json
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PROBE = os.path.join(REPO, "oracle", "_ref", "ref_pairs_probe")
N = 4096
ALL_NAN = 512
SEED = 20261018

FLOAT = {"f32": (np.float32, np.uint32, 23, 0x7F800000), "f64": (np.float64, np.uint64, 52, 0x7FF0000000000000)}
CASES = [("f32", "sum"), ("f32", "prod"), ("f64", "sum"), ("f64", "prod"),
         ("cf", "sum"), ("cf", "prod"), ("cd", "sum"), ("cd", "prod"),
         ("fi", "maxloc"), ("fi", "minloc"), ("di", "maxloc"), ("di", "minloc")]
PART_FLOAT = {"f32": "f32", "f64": "f64", "cf": "f32", "cd": "f64", "fi": "f32", "di": "f64"}
PAIR_LAYOUT = {"fi": (4, 8), "di": (8, 16)}  # index offset, extent


def nan_bits(fl, side, part, idx, rng):
    """NaN whose payload is (side, part, element): quiet or signalling (then the payload is non-zero anyway), either
    sign."""
    ft, ut, mb, exp = FLOAT[fl]
    quiet = rng.random(idx.size) < 0.5
    pay = (np.uint64(side) << np.uint64(mb - 4)) | (np.uint64(part) << np.uint64(mb - 7)) | (idx.astype(np.uint64) & np.uint64(0x3FF))
    pay |= np.uint64(1)
    qbit = np.uint64(1) << np.uint64(mb - 1)
    pay = np.where(quiet, pay | qbit, pay & ~qbit)
    sign = (rng.random(idx.size) < 0.3).astype(np.uint64) << np.uint64(np.dtype(ut).itemsize * 8 - 1)
    return (np.uint64(exp) | pay | sign).astype(ut)


def values(fl, side, part, rng, n=N):
    ft, ut, mb, exp = FLOAT[fl]
    big = 1e30 if ft == np.float32 else 1e300
    pool = np.array([0.0, -0.0, np.inf, -np.inf, 1.0, -1.0, 2.5, big, -big, 1e-30 if ft == np.float32 else 1e-300],
                    dtype=ft)
    v = rng.standard_normal(n).astype(ft)
    r = rng.random(n)
    pick = r < 0.4
    v[pick] = pool[rng.integers(0, len(pool), pick.sum())]
    bits = v.view(ut).copy()
    nan = (r >= 0.4) & (r < 0.75)
    nan[:ALL_NAN] = True
    idx = np.arange(n)
    bits[nan] = nan_bits(fl, side, part, idx[nan], rng)
    return bits.view(ft)


def inputs(t, side, rng):
    fl = PART_FLOAT[t]
    if t in ("f32", "f64"):
        return values(fl, side, 1, rng).view(np.uint8)
    if t in ("cf", "cd"):
        re, im = values(fl, side, 1, rng), values(fl, side, 2, rng)
        z = np.empty(2 * N, dtype=re.dtype)
        z[0::2], z[1::2] = re, im
        return z.view(np.uint8)
    ioff, ext = PAIR_LAYOUT[t]
    raw = np.full((N, ext), 0xAB, dtype=np.uint8)  # padding marker
    v = values(fl, side, 1, rng)
    # ties of equal non-NaN values (+-0 included) on some elements, so MAXLOC / MINLOC's equal branch runs too
    raw[:, :v.itemsize] = v.view(np.uint8).reshape(N, -1)
    idx = rng.integers(-3, 12, N).astype("<i4")
    raw[:, ioff:ioff + 4] = idx.view(np.uint8).reshape(N, 4)
    return raw.reshape(-1)


def main():
    rng = np.random.default_rng(SEED)
    arrays, cases = {}, []
    with tempfile.TemporaryDirectory() as tmp:
        for t, op in CASES:
            a, b = inputs(t, 1, rng), inputs(t, 2, rng)
            if t in PAIR_LAYOUT:  # copy a fifth of inout's values into in: ties
                ext = PAIR_LAYOUT[t][1]
                vs = 4 if t == "fi" else 8
                tie = np.flatnonzero(rng.random(N) < 0.2)
                a2, b2 = a.reshape(N, ext), b.reshape(N, ext)
                a2[tie, :vs] = b2[tie, :vs]
            fin, fio, fout = (os.path.join(tmp, x) for x in ("in", "io", "out"))
            a.tofile(fin)
            b.tofile(fio)
            subprocess.check_call([PROBE, "reduce", t, op, str(N), fin, fio, fout])
            key = f"{t}_{op}"
            arrays[key + "_in"], arrays[key + "_inout"] = a, b
            arrays[key + "_out"] = np.fromfile(fout, dtype=np.uint8)
            cases.append({"type": t, "op": op, "n": N})
    np.savez_compressed(os.path.join(HERE, "nan_reduce_local.npz"), **arrays)
    with open(os.path.join(HERE, "nan_manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_nan_payloads.py (MPICH 3.3.2 MPI_Reduce_local via "
                                "oracle/ref_pairs_probe)", "seed": SEED, "all_nan_prefix": ALL_NAN, "cases": cases}, f,
                  indent=1)
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
