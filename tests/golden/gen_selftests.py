"""Expected outputs of the reference's DEBUG_MODE self-test mains for CHiArA's stand-alone phases
(testing/custom_implementations/work_dir/reduce_scatter/{intra_reduce_scatter_radix, inter_linear_reduce,
intra_scatter_radix_batch}.cpp): each file compiled unchanged with -DDEBUG_MODE against MPICH 3.3.2
(`make -C oracle selftests`, oracle/_ref/selftest_<name>_mpi) and run here under mpiexec with one
stdout file per rank (`-outfile-pattern`; `-l` labels would split the mains' piecewise printf lines
at arbitrary points).  The printed lines of every rank (BEFORE and AFTER buffers; the scatter's RESULT line) go to
selftest_outputs.json; tests/test_gpu_ref_harness.py runs the same mains linked against libchiara
through the shim on MI355X and compares line for line.  Geometries whose output the reference leaves
uninitialised (intra_reduce_scatter's leftover-stage chunk on lanes >= nu is malloc'd and printed
unwritten) are avoided: every printed value is defined."""
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle")
MPIEXEC = "/opt/conda/bin/mpiexec"

# (binary, nranks, argv): the mains' own argument order
#   intra_reduce_scatter_radix: recvcount k b (:562-566, defaults 1 2 4)
#   inter_linear_reduce:        b recvcount   (:102-103, defaults 2 1)
#   intra_scatter_radix_batch:  k b recvcount (:155-160, defaults 7 9 7)
CONFIGS = [
    ("intra_reduce_scatter_radix", 4, ["1", "2", "2"]),
    ("intra_reduce_scatter_radix", 8, ["3", "2", "2"]),
    ("intra_reduce_scatter_radix", 9, ["2", "2", "3"]),
    ("inter_linear_reduce", 8, ["2", "2"]),
    ("inter_linear_reduce", 6, ["2", "3"]),
    ("inter_linear_reduce", 9, ["3", "1"]),
    ("intra_scatter_radix_batch", 9, ["7", "9", "7"]),
    ("intra_scatter_radix_batch", 8, ["2", "4", "3"]),
    ("intra_scatter_radix_batch", 6, ["3", "3", "2"]),
]


def key(name, n, args):
    return f"{name}_n{n}_" + "_".join(args)


def per_rank(outdir, n):
    """The per-rank stdout files of `-outfile-pattern out.%r` -> each rank's lines in order."""
    lines = {}
    for r in range(n):
        with open(os.path.join(outdir, f"out.{r}"), encoding="utf-8") as f:
            lines[str(r)] = [ln.rstrip() for ln in f.read().splitlines()]
    return lines


def main():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "selftests"])
    out = {}
    for name, n, args in CONFIGS:
        exe = os.path.join(ORACLE, "_ref", f"selftest_{name}_mpi")
        with tempfile.TemporaryDirectory() as tmp:
            subprocess.run([MPIEXEC, "-outfile-pattern", "out.%r", "-n", str(n), exe] + args, cwd=tmp, timeout=300,
                           check=True)
            out[key(name, n, args)] = {"binary": name, "nranks": n, "args": args, "lines": per_rank(tmp, n)}
        print(key(name, n, args), sum(len(v) for v in out[key(name, n, args)]["lines"].values()), "lines")
    with open(os.path.join(HERE, "selftest_outputs.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_selftests.py",
                   "reference": "testing/custom_implementations/work_dir/reduce_scatter/{intra_reduce_scatter_radix,"
                                "inter_linear_reduce,intra_scatter_radix_batch}.cpp -DDEBUG_MODE @ 2025-11-21, "
                                "MPICH 3.3.2", "runs": out}, f, indent=0)


if __name__ == "__main__":
    main()
