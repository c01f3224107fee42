"""Expected outputs of the reference's DEBUG_MODE self-test mains: CHiArA's stand-alone phases
(testing/custom_implementations/work_dir/reduce_scatter/), all_reduce_radix_batch.cpp and the MPICH baselines
(testing/mpich_implementations/): each file compiled unchanged with -DDEBUG_MODE against MPICH 3.3.2
(`make -C oracle selftests`, oracle/selftests.sh, oracle/_ref/selftest_<name>_mpi) and run here under mpiexec with one
stdout file per rank (`-outfile-pattern`; `-l` labels would split the mains' piecewise printf lines
at arbitrary points).  The printed lines of every rank (buffers, PASS / FAIL lines; normalised by tests/selftest_util.py) and the files
a main writes go to selftest_outputs.json; tests/test_gpu_ref_harness.py runs the same mains linked against libchiara
through the shim on MI355X and compares line for line.  Geometries whose output the reference leaves
uninitialised (intra_reduce_scatter's leftover-stage chunk on lanes >= nu is malloc'd and printed
unwritten) are avoided: every printed value is defined."""
import json
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import selftest_util  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle")
MPIEXEC = "/opt/conda/bin/mpiexec"

# (binary, nranks, argv, files the main writes): the mains' own argument order
#   intra_reduce_scatter_radix: recvcount k b (:562-566, defaults 1 2 4)
#   inter_linear_reduce:        b recvcount   (:102-103, defaults 2 1)
#   intra_scatter_radix_batch:  k b recvcount (:155-160, defaults 7 9 7)
#   all_reduce_radix_batch:     n_iter [b=..] (Fugaku_experiments/Allreduce, :844-876): results0.csv
#   reduce_scatter_radix:       k             (testing/mpich_implementations/reduce_scatter, default 3)
#   reduce_scatter_recursive_halving: r b     (writes all_buffers.txt)
#   the allreduce baselines:    their defaults (count 10 / 100, k 3)
CONFIGS = [
    ("intra_reduce_scatter_radix", 4, ["1", "2", "2"], []),
    ("intra_reduce_scatter_radix", 8, ["3", "2", "2"], []),
    ("intra_reduce_scatter_radix", 9, ["2", "2", "3"], []),
    ("inter_linear_reduce", 8, ["2", "2"], []),
    ("inter_linear_reduce", 6, ["2", "3"], []),
    ("inter_linear_reduce", 9, ["3", "1"], []),
    ("intra_scatter_radix_batch", 9, ["7", "9", "7"], []),
    ("intra_scatter_radix_batch", 8, ["2", "4", "3"], []),
    ("intra_scatter_radix_batch", 6, ["3", "3", "2"], []),
    ("all_reduce_radix_batch", 6, ["3", "b=2"], ["results0.csv"]),
    ("reduce_scatter_radix", 6, ["3"], []),
    ("reduce_scatter_recursive_halving", 6, ["2", "2"], ["all_buffers.txt"]),
    ("reduce_scatter_pairwise", 6, [], []),
    ("allreduce_ring", 6, [], []),
    ("allreduce_recursive_doubling", 6, [], []),
    ("allreduce_reduce_scatter_allgather", 6, [], []),
    ("allreduce_recexch", 6, [], []),
    ("allreduce_k_reduce_scatter_allgather", 6, [], []),
    ("allreduce_recursive_multiplying", 6, [], []),
]


def key(name, n, args):
    return f"{name}_n{n}_" + "_".join(a.replace("=", "") for a in args)


def per_rank(outdir, n):
    """The per-rank stdout files of `-outfile-pattern out.%r` -> each rank's normalised lines."""
    lines = {}
    for r in range(n):
        path = os.path.join(outdir, f"out.{r}")  # a rank that prints nothing leaves no file
        text = open(path, encoding="utf-8").read() if os.path.exists(path) else ""
        lines[str(r)] = selftest_util.normalize(text)
    return lines


def written(outdir, files):
    out = {}
    for name in files:
        with open(os.path.join(outdir, name), encoding="utf-8") as f:
            text = f.read()
        out[name] = selftest_util.normalize_csv(text) if name.endswith(".csv") else text.splitlines()
    return out


def main():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "selftests"])
    out = {}
    for name, n, args, files in CONFIGS:
        exe = os.path.join(ORACLE, "_ref", f"selftest_{name}_mpi")
        with tempfile.TemporaryDirectory() as tmp:
            subprocess.run([MPIEXEC, "-outfile-pattern", "out.%r", "-n", str(n), exe] + args, cwd=tmp, timeout=300,
                           check=True)
            out[key(name, n, args)] = {"binary": name, "nranks": n, "args": args, "lines": per_rank(tmp, n),
                                       "files": written(tmp, files)}
        print(key(name, n, args), sum(len(v) for v in out[key(name, n, args)]["lines"].values()), "lines")
    with open(os.path.join(HERE, "selftest_outputs.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_selftests.py",
                   "reference": "the DEBUG_MODE mains of testing/custom_implementations/work_dir/reduce_scatter/"
                                "{intra_reduce_scatter_radix,inter_linear_reduce,intra_scatter_radix_batch}.cpp, "
                                "Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp, testing/mpich_implementations/"
                                "{reduce_scatter/reduce_scatter_{radix,recursive_halving,pairwise},all_reduce/allreduce_"
                                "{ring,recursive_doubling,reduce_scatter_allgather,recexch,k_reduce_scatter_allgather,"
                                "recursive_multiplying}}.cpp @ 2025-11-21, MPICH 3.3.2 (oracle/selftests.sh)",
                   "runs": out}, f, indent=0)


if __name__ == "__main__":
    main()
