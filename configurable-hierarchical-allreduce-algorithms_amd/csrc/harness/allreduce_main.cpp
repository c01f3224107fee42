// allreduce_main.cpp -- drop-in for Fugaku_experiments/Allreduce/main.cpp on MI355X.
//
//   mpiexec -n 8 bin/chiara_allreduce <n_iter> [--overwrite] [b=4] [base=..] [num_nodes=..]
//                                     [radix_increment=..] [dtype=..] [mem=host|device] [k=..]
// Same CLI keys, same CSV file name and schema (algorithm_name,k,b,nprocs,send_count,time,
// is_correct), same per-rep protocol: fill recv 0 -> MPI_Barrier -> MPI_Wtime -> collective
// -> MPI_Barrier -> MPI_Wtime; is_correct against the MPI library's MPI_Allreduce on the
// same inputs (Allreduce/main.cpp:43-76).  The collective is chr_allreduce_radix_batch.
#include "harness_common.hpp"

using namespace harness;

static void run_k2(const Options& o, Ctx& c, std::ofstream& csv, const char* name, int k, int count) {
    const chr_dtype dt = to_chr(o.dtype);
    const size_t es = esize(dt);
    std::vector<char> send, ref(count * es), recv(count * es);
    fill_input(send, count, dt, c.rank, count, o.pattern);
    MPI_Allreduce(send.data(), ref.data(), count, dt == CHR_BFLOAT16 ? c.bf16 : mpi_type(dt),
                  dt == CHR_BFLOAT16 ? c.bf16_sum : MPI_SUM, MPI_COMM_WORLD);
    std::vector<double> sumabs(count);
    MPI_Allreduce(abs_values(send, count, dt).data(), sumabs.data(), count, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
    const bool dev = o.mem == "device";
    DevBuf dsend(dev ? count * es : 0), drecv(dev ? count * es : 0);
    if (dev) {
        (void)hipMemcpy(dsend.p, send.data(), count * es, hipMemcpyHostToDevice);
        (void)hipDeviceSynchronize();
    }
    const int reps = o.reps > 0 ? o.reps : 50;
    for (int rep = 0; rep < reps; ++rep) {
        std::fill(recv.begin(), recv.end(), 0);
        if (dev) {
            (void)hipMemset(drecv.p, 0, count * es);
            (void)hipDeviceSynchronize();  // NULL-stream memset vs the comm's non-blocking stream
        }
        MPI_Barrier(MPI_COMM_WORLD);
        const double t0 = MPI_Wtime();
        const int err = chr_allreduce_radix_batch(dev ? dsend.p : send.data(), dev ? drecv.p : recv.data(),
                                                  (size_t)count, dt, CHR_SUM, c.comm, k, o.b);
        MPI_Barrier(MPI_COMM_WORLD);
        const double t1 = MPI_Wtime();
        if (dev) (void)hipMemcpy(recv.data(), drecv.p, count * es, hipMemcpyDeviceToHost);
        const bool correct = err == CHR_SUCCESS && check_correctness(recv, ref, sumabs, count, dt, c.nprocs);
        if (err != CHR_SUCCESS && c.rank == 0 && rep == 0)
            std::fprintf(stderr, "%s k=%d b=%d count=%d: %s\n", name, k, o.b, count, chr_error_string(err));
        if (c.rank == 0)
            csv << name << "," << k << "," << o.b << "," << c.nprocs << "," << count / c.nprocs << "," << (t1 - t0)
                << "," << (correct ? 1 : 0) << "\n" << std::flush;
    }
}

static void run_no_k(const Options& o, Ctx& c, std::ofstream& csv, int count) {
    const chr_dtype dt = to_chr(o.dtype);
    if (dt == CHR_BFLOAT16) return;
    const size_t es = esize(dt);
    std::vector<char> send, recv(count * es), ref(count * es);
    fill_input(send, count, dt, c.rank, count, o.pattern);
    MPI_Allreduce(send.data(), ref.data(), count, mpi_type(dt), MPI_SUM, MPI_COMM_WORLD);
    std::vector<double> sumabs(count);
    MPI_Allreduce(abs_values(send, count, dt).data(), sumabs.data(), count, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
    const int reps = o.reps > 0 ? o.reps : 50;
    for (int rep = 0; rep < reps; ++rep) {
        std::fill(recv.begin(), recv.end(), 0);
        MPI_Barrier(MPI_COMM_WORLD);
        const double t0 = MPI_Wtime();
        const int err = MPI_Allreduce(send.data(), recv.data(), count, mpi_type(dt), MPI_SUM, MPI_COMM_WORLD);
        MPI_Barrier(MPI_COMM_WORLD);
        const double t1 = MPI_Wtime();
        const bool correct = err == MPI_SUCCESS && check_correctness(recv, ref, sumabs, count, dt, c.nprocs);
        if (c.rank == 0)
            csv << "MPICH_allreduce,0,0," << c.nprocs << "," << count / c.nprocs << "," << (t1 - t0) << ","
                << (correct ? 1 : 0) << "\n" << std::flush;
    }
}

int main(int argc, char** argv) {
    setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 0);  // dmabuf IPC for RCCL, before any HIP call (api.cpp)
    MPI_Init(&argc, &argv);
    Options o;
    Ctx c;
    MPI_Comm_rank(MPI_COMM_WORLD, &c.rank);
    if (!parse(argc, argv, &o, c.rank)) {
        MPI_Finalize();
        return EXIT_FAILURE;
    }
    if (init(&c, o) != CHR_SUCCESS) {
        std::fprintf(stderr, "rank %d: communicator init failed\n", c.rank);
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    std::ofstream csv = open_csv(o, c.rank, c.nprocs);
    const int base = o.base * c.nprocs;  // Allreduce/main.cpp:185
    for (int i = 0; i < o.n_iter; ++i) {
        const int count = base << i;
        if (o.k_only) {
            run_k2(o, c, csv, "all_reduce_radix_batch", o.k_only, count);
        } else {
            for (int k = 2; k < o.b; k += o.radix_increment)  // Allreduce/main.cpp:190
                run_k2(o, c, csv, "all_reduce_radix_batch", k, count);
        }
        run_no_k(o, c, csv, count);
    }
    if (c.rank == 0) csv.close();
    chr_comm_destroy(c.comm);
    MPI_Finalize();
    return EXIT_SUCCESS;
}
