// ref_timer.cpp -- TEST INFRASTRUCTURE ONLY (bench.py's N>1 cpu_baseline, kind=reference).
//
// Times the REAL reference collective on the host's cores: all_reduce_radix_batch /
// reduce_scatter_radix_batch compiled unchanged from
//   /root/reference/Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp
//   /root/reference/Fugaku_experiments/Reduce-scatter/reduce_scatter_radix_batch.cpp
// against MPICH 3.3.2, one MPI rank per core (`mpiexec -bind-to core`), fp32 SUM, the same
// (n, k, b) geometry as the GPU line.  One warm-up call, then `reps` calls bracketed by
// MPI_Barrier, max over ranks (as bench.py takes the max over GPU ranks).
// Usage: mpiexec -n N ref_timer <ar|rs> <k> <b> <count> <reps>   (count: allreduce elements per
// rank, or reduce-scatter recvcount).  Rank 0 prints one JSON object.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

int all_reduce_radix_batch(char* sendbuf, char* recvbuf, int aCount, MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                           int k, int b);
int reduce_scatter_radix_batch(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                               MPI_Op op, MPI_Comm comm, int k, int b);

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int rank, n;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &n);
    if (argc != 6) {
        if (rank == 0) std::fprintf(stderr, "usage: ref_timer ar|rs k b count reps\n");
        MPI_Finalize();
        return 1;
    }
    const std::string mode = argv[1];
    const int k = std::atoi(argv[2]), b = std::atoi(argv[3]), reps = std::atoi(argv[5]);
    const long long count = std::atoll(argv[4]);
    const bool ar = mode == "ar";
    const long long sendn = ar ? count : count * n, recvn = count;
    std::vector<float> send((size_t)sendn), recv((size_t)recvn);
    for (long long i = 0; i < sendn; ++i) send[(size_t)i] = (float)((rank * 131 + i) % 1021) * 1e-3f;
    auto call = [&]() {
        if (ar)
            all_reduce_radix_batch((char*)send.data(), (char*)recv.data(), (int)count, MPI_FLOAT, MPI_SUM,
                                   MPI_COMM_WORLD, k, b);
        else
            reduce_scatter_radix_batch(send.data(), recv.data(), (MPI_Aint)count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD,
                                       k, b);
    };
    call();  // warm-up (first touch of the reference's per-call scratch happens on every call anyway)
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    for (int r = 0; r < reps; ++r) call();
    MPI_Barrier(MPI_COMM_WORLD);
    double el = MPI_Wtime() - t0, mx = 0;
    MPI_Reduce(&el, &mx, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    if (rank == 0)
        std::printf("{\"mode\": \"%s\", \"nranks\": %d, \"k\": %d, \"b\": %d, \"count\": %lld, \"reps\": %d, "
                    "\"seconds_per_call\": %.9f, \"bytes_per_rank\": %lld}\n",
                    mode.c_str(), n, k, b, count, reps, mx / reps, sendn * 4);
    MPI_Finalize();
    return 0;
}
