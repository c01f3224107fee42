// ref_reduce_local.cpp -- TEST INFRASTRUCTURE ONLY (bench.py cpu_baseline, kind=reference).
//
// Times the reference's actual hot-path call, MPICH 3.3.2's MPI_Reduce_local(in, inout,
// n, MPI_FLOAT, MPI_SUM) (all_reduce_radix_batch.cpp:364 etc.), single rank, on an n-element
// fp32 bucket for about `seconds` seconds.  threads = 1: one thread over the whole bucket
// (the reference's own call).  threads = T > 1: the bucket is cut into T contiguous slices,
// each thread first-touches and reduces its own slice with MPI_Reduce_local
// (MPI_THREAD_MULTIPLE) -- the all-cores variant SURVEY §8(d) asks for, labelled as such.
// Usage: ref_reduce_local <n_elems> <seconds> [threads]
// Prints one JSON object: {"gbps": ..., "calls": ..., "seconds": ..., "bytes_per_call": ..., "threads": T}
#include <mpi.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

static void init_slice(float* in, float* inout, long lo, long hi) {
    for (long i = lo; i < hi; ++i) {
        in[i] = (float)((i * 2654435761u) % 1000) * 1e-3f - 0.5f;
        inout[i] = (float)((i * 40503u) % 1000) * 1e-3f - 0.5f;
    }
}

int main(int argc, char** argv) {
    int provided = 0;
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &provided);
    const long n = argc > 1 ? std::atol(argv[1]) : (16L << 20);
    const double seconds = argc > 2 ? std::atof(argv[2]) : 10.0;
    int T = argc > 3 ? std::atoi(argv[3]) : 1;
    if (T < 1 || provided < MPI_THREAD_MULTIPLE) T = 1;
    float* in = static_cast<float*>(std::malloc(n * sizeof(float)));
    float* inout = static_cast<float*>(std::malloc(n * sizeof(float)));
    std::vector<long> calls(T, 0);
    std::atomic<int> ready{0};
    double t0 = 0, t1 = 0;
    auto worker = [&](int t) {
        const long lo = n * t / T, hi = n * (t + 1) / T;
        init_slice(in, inout, lo, hi);  // first touch by the thread that streams the slice
        MPI_Reduce_local(in + lo, inout + lo, (int)(hi - lo), MPI_FLOAT, MPI_SUM);  // warm-up
        ready.fetch_add(1);
        while (ready.load() < T + 1) {}
        const double s0 = MPI_Wtime();
        while (MPI_Wtime() - s0 < seconds) {
            MPI_Reduce_local(in + lo, inout + lo, (int)(hi - lo), MPI_FLOAT, MPI_SUM);
            ++calls[t];
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) pool.emplace_back(worker, t);
    while (ready.load() < T) {}
    t0 = MPI_Wtime();
    ready.fetch_add(1);
    for (auto& th : pool) th.join();
    t1 = MPI_Wtime();
    // every thread ran `seconds`; total bytes = sum over threads of calls x slice bytes
    double bytes = 0;
    long total_calls = 0;
    for (int t = 0; t < T; ++t) {
        bytes += 3.0 * (double)(n * (t + 1) / T - n * t / T) * sizeof(float) * (double)calls[t];
        total_calls += calls[t];
    }
    std::printf("{\"gbps\": %.4f, \"calls\": %ld, \"seconds\": %.4f, \"bytes_per_call\": %.0f, \"threads\": %d, "
                "\"checksum\": %.6g}\n",
                bytes / (t1 - t0) / 1e9, total_calls / T, t1 - t0, 3.0 * (double)n * sizeof(float), T,
                (double)inout[n / 2]);
    std::free(in);
    std::free(inout);
    MPI_Finalize();
    return 0;
}
