// reduce_scatter_main.cpp -- drop-in for Fugaku_experiments/Reduce-scatter/main.cpp on MI355X.
//
//   mpiexec -n 2 bin/chiara_reduce_scatter <n_iter> [--overwrite] [b=..] [base=..] [num_nodes=..]
//                                          [radix_increment=..] [dtype=..] [mem=host|device] [k=..]
// Same CLI, CSV name/schema and per-rep protocol as the reference harness: 20 reps,
// correctness AND-reduced over ranks (MPI_Allreduce MIN), time = MAX over ranks
// (Reduce-scatter/main.cpp:34-91); reference collective MPI_Reduce_scatter_block.
#include "harness_common.hpp"

using namespace harness;

static void run_r_b(const Options& o, Ctx& c, std::ofstream& csv, const char* name, int r, int count) {
    const chr_dtype dt = to_chr(o.dtype);
    const size_t es = esize(dt);
    const size_t in_n = (size_t)count * c.nprocs;
    std::vector<char> send, ref(count * es), recv(count * es);
    fill_input(send, in_n, dt, c.rank, in_n, o.pattern);  // seq: rank*(count*nprocs)+i (main.cpp:45-46)
    MPI_Reduce_scatter_block(send.data(), ref.data(), count, dt == CHR_BFLOAT16 ? c.bf16 : mpi_type(dt),
                             dt == CHR_BFLOAT16 ? c.bf16_sum : MPI_SUM, MPI_COMM_WORLD);
    std::vector<double> sumabs(count);
    MPI_Reduce_scatter_block(abs_values(send, in_n, dt).data(), sumabs.data(), count, MPI_DOUBLE, MPI_SUM,
                             MPI_COMM_WORLD);
    const bool dev = o.mem == "device";
    DevBuf dsend(dev ? in_n * es : 0), drecv(dev ? count * es : 0);
    if (dev) {
        (void)hipMemcpy(dsend.p, send.data(), in_n * es, hipMemcpyHostToDevice);
        (void)hipDeviceSynchronize();
    }
    const int reps = o.reps > 0 ? o.reps : 20;
    for (int rep = 0; rep < reps; ++rep) {
        std::fill(recv.begin(), recv.end(), 0);
        if (dev) {
            (void)hipMemset(drecv.p, 0, count * es);
            (void)hipDeviceSynchronize();  // NULL-stream memset vs the comm's non-blocking stream
        }
        MPI_Barrier(MPI_COMM_WORLD);
        const double t0 = MPI_Wtime();
        const int err = chr_reduce_scatter_radix_batch(dev ? dsend.p : send.data(), dev ? drecv.p : recv.data(),
                                                       (size_t)count, dt, CHR_SUM, c.comm, r, o.b);
        MPI_Barrier(MPI_COMM_WORLD);
        const double t1 = MPI_Wtime();
        if (dev) (void)hipMemcpy(recv.data(), drecv.p, count * es, hipMemcpyDeviceToHost);
        const int ok_local = (err == CHR_SUCCESS && check_correctness(recv, ref, sumabs, count, dt, c.nprocs)) ? 1 : 0;
        int ok = 0;
        MPI_Allreduce(&ok_local, &ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
        double el = t1 - t0, el_max = 0;
        MPI_Reduce(&el, &el_max, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
        if (c.rank == 0)
            csv << name << "," << r << "," << o.b << "," << c.nprocs << "," << count << "," << el_max << ","
                << ok << "\n" << std::flush;
    }
}

static void run_standard(const Options& o, Ctx& c, std::ofstream& csv, int count) {
    const chr_dtype dt = to_chr(o.dtype);
    if (dt == CHR_BFLOAT16) return;
    const size_t es = esize(dt);
    const size_t in_n = (size_t)count * c.nprocs;
    std::vector<char> send, recv(count * es), ref(count * es);
    fill_input(send, in_n, dt, c.rank, in_n, o.pattern);
    MPI_Reduce_scatter_block(send.data(), ref.data(), count, mpi_type(dt), MPI_SUM, MPI_COMM_WORLD);
    std::vector<double> sumabs(count);
    MPI_Reduce_scatter_block(abs_values(send, in_n, dt).data(), sumabs.data(), count, MPI_DOUBLE, MPI_SUM,
                             MPI_COMM_WORLD);
    const int reps = o.reps > 0 ? o.reps : 20;
    for (int rep = 0; rep < reps; ++rep) {
        MPI_Barrier(MPI_COMM_WORLD);
        const double t0 = MPI_Wtime();
        const int err = MPI_Reduce_scatter_block(send.data(), recv.data(), count, mpi_type(dt), MPI_SUM, MPI_COMM_WORLD);
        MPI_Barrier(MPI_COMM_WORLD);
        const double t1 = MPI_Wtime();
        const int ok_local = (err == MPI_SUCCESS && check_correctness(recv, ref, sumabs, count, dt, c.nprocs)) ? 1 : 0;
        int ok = 0;
        MPI_Allreduce(&ok_local, &ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
        double el = t1 - t0, el_max = 0;
        MPI_Reduce(&el, &el_max, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
        if (c.rank == 0)
            csv << "reduce_scatter_standard,0,0," << c.nprocs << "," << count << "," << el_max << "," << ok << "\n"
                << std::flush;
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
    for (int i = 0; i < o.n_iter; ++i) {
        const int count = o.base << i;  // NOT x nprocs (Reduce-scatter/main.cpp:241-242)
        if (o.k_only) {
            run_r_b(o, c, csv, "reduce_scatter_radix_batch", o.k_only, count);
        } else {
            for (int r = 2; r < o.b; r += o.radix_increment)
                run_r_b(o, c, csv, "reduce_scatter_radix_batch", r, count);
        }
        run_standard(o, c, csv, count);
    }
    if (c.rank == 0) csv.close();
    chr_comm_destroy(c.comm);
    MPI_Finalize();
    return EXIT_SUCCESS;
}
