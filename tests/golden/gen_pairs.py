#!/usr/bin/env python3
"""Fixtures of MPICH's own element semantics for the pair types (MAXLOC / MINLOC) and the C complex
types (SUM / PROD), container-only: MPI_Reduce_local(in, inout) computed by MPICH 3.3.2 itself
(oracle/_ref/ref_pairs_probe, built by `make -C oracle ref_pairs`) on inputs made here, with ties,
signed zeros, NaN / infinity and integer extremes, and padding bytes set to a marker so the fixture
also shows what MPICH does with them.  Writes tests/golden/pairs_reduce_local.npz (inputs and
MPICH's outputs, raw bytes) and tests/golden/pairs_manifest.json (MPICH's size / extent / valid-op
table for these types).  Rerun: python tests/golden/gen_pairs.py
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

# C layouts (x86-64 and gfx950 agree): value, then the int index at the value's alignment
LAYOUT = {
    "fi": ("<f4", 0, 4, 8), "di": ("<f8", 0, 8, 16), "li": ("<i8", 0, 8, 16),
    "2i": ("<i4", 0, 4, 8), "si": ("<i2", 0, 4, 8),
}
COMPLEX = {"cf": np.complex64, "cd": np.complex128}


def pair_inputs(t, rng):
    vfmt, voff, ioff, size = LAYOUT[t]
    raw = np.full((2, N, size), 0xAB, dtype=np.uint8)  # padding marker
    for s in range(2):
        if vfmt[1] == "f":
            pool = np.array([-1.0, 0.0, -0.0, 1.0, 2.5, np.inf, -np.inf, np.nan], dtype=vfmt)
            v = np.where(rng.random(N) < 0.75, pool[rng.integers(0, len(pool), N)],
                         rng.standard_normal(N).astype(vfmt)).astype(vfmt)
            if vfmt == "<f4":  # a NaN with a per-side payload
                vb = v.view(np.uint32)
                vb[np.isnan(v)] = 0x7FC00000 | (0x11 + s)
        else:
            info = np.iinfo(np.dtype(vfmt))
            pool = np.array([info.min, info.max, -1, 0, 1, 2], dtype=vfmt)
            v = np.where(rng.random(N) < 0.3, pool[rng.integers(0, len(pool), N)],
                         rng.integers(-3, 4, N)).astype(vfmt)
        idx = np.where(rng.random(N) < 0.2, rng.integers(-5, 0, N), rng.integers(0, 12, N)).astype("<i4")
        raw[s, :, voff:voff + np.dtype(vfmt).itemsize] = v.view(np.uint8).reshape(N, -1)
        raw[s, :, ioff:ioff + 4] = idx.view(np.uint8).reshape(N, 4)
    return raw[0].reshape(-1), raw[1].reshape(-1)


def complex_inputs(t, rng):
    ct = COMPLEX[t]
    ft = np.float32 if ct == np.complex64 else np.float64
    out = []
    for s in range(2):
        re = rng.standard_normal(N).astype(ft)
        im = rng.standard_normal(N).astype(ft)
        sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e30 if ft == np.float32 else 1e300,
                       1e-30 if ft == np.float32 else 1e-300], dtype=ft)
        m = rng.random(N) < 0.15
        re[m] = sp[rng.integers(0, len(sp), m.sum())]
        m = rng.random(N) < 0.15
        im[m] = sp[rng.integers(0, len(sp), m.sum())]
        z = np.empty(N, dtype=ct)
        z.real, z.imag = re, im
        out.append(z.view(np.uint8))
    return out


def main():
    table = json.loads(subprocess.check_output([PROBE, "table"]).decode())
    rng = np.random.default_rng(20261017)
    arrays, cases = {}, []
    with tempfile.TemporaryDirectory() as tmp:
        for t in list(LAYOUT) + list(COMPLEX):
            for op in table[t]["ops"]:
                a, b = (pair_inputs(t, rng) if t in LAYOUT else complex_inputs(t, rng))
                fin, fio, fout = (os.path.join(tmp, x) for x in ("in", "io", "out"))
                a.tofile(fin)
                b.tofile(fio)
                subprocess.check_call([PROBE, "reduce", t, op, str(N), fin, fio, fout])
                out = np.fromfile(fout, dtype=np.uint8)
                key = f"{t}_{op}"
                arrays[key + "_in"], arrays[key + "_inout"], arrays[key + "_out"] = a, b, out
                cases.append({"type": t, "op": op, "n": N, "extent": table[t]["extent"]})
    np.savez_compressed(os.path.join(HERE, "pairs_reduce_local.npz"), **arrays)
    with open(os.path.join(HERE, "pairs_manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_pairs.py (MPICH 3.3.2 MPI_Reduce_local via oracle/ref_pairs_probe)",
                   "table": table, "cases": cases}, f, indent=1)
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
