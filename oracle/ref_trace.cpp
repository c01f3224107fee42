// ref_trace.cpp -- TEST INFRASTRUCTURE ONLY, container-only.
//
// Message trace of the REAL reference collectives, compiled unchanged from
//   /root/reference/Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp
//   /root/reference/Fugaku_experiments/Reduce-scatter/reduce_scatter_radix_batch.cpp
// against the container's MPICH 3.3.2.  MPI_Isend / MPI_Irecv / MPI_Send / MPI_Recv are
// intercepted through the standard PMPI profiling interface: every point-to-point call the
// algorithm makes is logged as (rank, direction, peer, bytes) in call order, then forwarded
// to PMPI_*.  The trace pins the communication pattern of libchiara's `exact` schedule
// (tests/test_exact_schedule.py, fixture tests/golden/msg_trace.json, made by
// tests/golden/gen_trace.py).
//
// Usage: mpiexec -n N ref_trace <ar|rs> <k> <b> <count>    (fp32 SUM; count = allreduce
// count or reduce-scatter recvcount).  Rank 0 prints one JSON object per rank, one per line.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

int all_reduce_radix_batch(char* sendbuf, char* recvbuf, int aCount, MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                           int k, int b);
int reduce_scatter_radix_batch(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                               MPI_Op op, MPI_Comm comm, int k, int b);

namespace {
bool g_on = false;
std::vector<long long> g_log;  // triples: dir (0 send, 1 recv), peer, bytes

void note(int dir, int peer, int count, MPI_Datatype dt) {
    if (!g_on) return;
    int sz = 0;
    PMPI_Type_size(dt, &sz);
    g_log.push_back(dir);
    g_log.push_back(peer);
    g_log.push_back((long long)count * sz);
}
}  // namespace

extern "C" {
int MPI_Isend(const void* buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request* req) {
    note(0, dest, count, dt);
    return PMPI_Isend(buf, count, dt, dest, tag, comm, req);
}
int MPI_Irecv(void* buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Request* req) {
    note(1, source, count, dt);
    return PMPI_Irecv(buf, count, dt, source, tag, comm, req);
}
int MPI_Send(const void* buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm) {
    note(0, dest, count, dt);
    return PMPI_Send(buf, count, dt, dest, tag, comm);
}
int MPI_Recv(void* buf, int count, MPI_Datatype dt, int source, int tag, MPI_Comm comm, MPI_Status* st) {
    note(1, source, count, dt);
    return PMPI_Recv(buf, count, dt, source, tag, comm, st);
}
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int rank, n;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &n);
    if (argc != 5) {
        if (rank == 0) std::fprintf(stderr, "usage: ref_trace ar|rs k b count\n");
        MPI_Finalize();
        return 1;
    }
    const std::string mode = argv[1];
    const int k = std::atoi(argv[2]), b = std::atoi(argv[3]);
    const long long count = std::atoll(argv[4]);
    const long long sendn = mode == "ar" ? count : count * n;
    const long long recvn = mode == "ar" ? count : count;
    std::vector<float> send((size_t)sendn), recv((size_t)recvn);
    for (long long i = 0; i < sendn; ++i) send[(size_t)i] = (float)((rank * 7 + i) % 13);
    MPI_Barrier(MPI_COMM_WORLD);
    g_on = true;
    if (mode == "ar")
        all_reduce_radix_batch((char*)send.data(), (char*)recv.data(), (int)count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD,
                               k, b);
    else
        reduce_scatter_radix_batch(send.data(), recv.data(), (MPI_Aint)count, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD, k, b);
    g_on = false;
    // gather the logs at rank 0 (these calls are not logged)
    int len = (int)g_log.size();
    std::vector<int> lens(n);
    PMPI_Gather(&len, 1, MPI_INT, lens.data(), 1, MPI_INT, 0, MPI_COMM_WORLD);
    std::vector<int> displs(n, 0);
    int tot = 0;
    for (int r = 0; r < n; ++r) {
        displs[r] = tot;
        tot += lens[r];
    }
    std::vector<long long> all((size_t)(rank == 0 ? tot : 0) + 1);
    PMPI_Gatherv(g_log.data(), len, MPI_LONG_LONG, all.data(), lens.data(), displs.data(), MPI_LONG_LONG, 0,
                 MPI_COMM_WORLD);
    if (rank == 0) {
        for (int r = 0; r < n; ++r) {
            std::printf("{\"rank\": %d, \"msgs\": [", r);
            for (int i = 0; i < lens[r]; i += 3) {
                const long long* t = &all[(size_t)(displs[r] + i)];
                std::printf("%s[%lld, %lld, %lld]", i ? ", " : "", t[0], t[1], t[2]);
            }
            std::printf("]}\n");
        }
    }
    MPI_Finalize();
    return 0;
}
