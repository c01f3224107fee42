// ref_reduce_local.cpp -- TEST INFRASTRUCTURE ONLY (bench.py cpu_baseline, kind=reference).
//
// Times the reference's actual hot-path call, MPICH 3.3.2's MPI_Reduce_local(in, inout,
// n, MPI_FLOAT, MPI_SUM) (all_reduce_radix_batch.cpp:364 etc.), single rank, single
// thread, on an n-element fp32 bucket for about `seconds` seconds.
// Usage: mpiexec -n 1 ref_reduce_local <n_elems> <seconds>
// Prints one JSON object: {"gbps": ..., "calls": ..., "seconds": ..., "bytes_per_call": ...}
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    const long n = argc > 1 ? std::atol(argv[1]) : (16L << 20);
    const double seconds = argc > 2 ? std::atof(argv[2]) : 10.0;
    std::vector<float> in(n), inout(n);
    for (long i = 0; i < n; ++i) {
        in[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
        inout[i] = (float)((i * 40503u) % 1000) * 1e-3f - 0.5f;
    }
    MPI_Reduce_local(in.data(), inout.data(), (int)n, MPI_FLOAT, MPI_SUM);  // warm-up / first touch
    long calls = 0;
    const double t0 = MPI_Wtime();
    double t1 = t0;
    while (t1 - t0 < seconds) {
        MPI_Reduce_local(in.data(), inout.data(), (int)n, MPI_FLOAT, MPI_SUM);
        ++calls;
        t1 = MPI_Wtime();
    }
    const double bytes = 3.0 * (double)n * sizeof(float);
    std::printf("{\"gbps\": %.4f, \"calls\": %ld, \"seconds\": %.4f, \"bytes_per_call\": %.0f, \"checksum\": %.6g}\n",
                bytes * calls / (t1 - t0) / 1e9, calls, t1 - t0, bytes, (double)inout[n / 2]);
    MPI_Finalize();
    return 0;
}
