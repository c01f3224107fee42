// allgather_main.cpp -- drop-in for Fugaku_experiments/Allgather/main.cpp on MI355X.
//
//   mpiexec -n 8 bin/chiara_allgather <n_iter> [--overwrite] [b=..] [base=..] [num_nodes=..]
//                                     [radix_increment=..] [dtype=..] [mem=host|device] [k=..]
// Same CLI, CSV name/schema and per-rep protocol as the reference harness: 50 reps of
// allgather_radix_batch for k = 2..b-1, then MPI_Allgather ("allgather_standard"); sendbuf
// rank*count + i, exact comparison with MPI_Allgather (Allgather/main.cpp:29-105, 180-193).
#include "harness_common.hpp"

using namespace harness;

static void run_k_b(const Options& o, Ctx& c, std::ofstream& csv, int k, int count) {
    const chr_dtype dt = to_chr(o.dtype);
    const size_t es = esize(dt), out_n = (size_t)count * c.nprocs;
    std::vector<char> send, ref(out_n * es), recv(out_n * es);
    fill_input(send, count, dt, c.rank, count, o.pattern);
    MPI_Allgather(send.data(), count * (int)es, MPI_BYTE, ref.data(), count * (int)es, MPI_BYTE, MPI_COMM_WORLD);
    const bool dev = o.mem == "device";
    DevBuf dsend(dev ? count * es : 0), drecv(dev ? out_n * es : 0);
    if (dev) {
        (void)hipMemcpy(dsend.p, send.data(), count * es, hipMemcpyHostToDevice);
        (void)hipDeviceSynchronize();
    }
    const int reps = o.reps > 0 ? o.reps : 50;
    for (int rep = 0; rep < reps; ++rep) {
        std::fill(recv.begin(), recv.end(), 0);
        if (dev) {
            (void)hipMemset(drecv.p, 0, out_n * es);
            (void)hipDeviceSynchronize();  // NULL-stream memset vs the comm's non-blocking stream
        }
        MPI_Barrier(MPI_COMM_WORLD);
        const double t0 = MPI_Wtime();
        const int err = chr_allgather_radix_batch(dev ? dsend.p : send.data(), (size_t)count, dt,
                                                  dev ? drecv.p : recv.data(), c.comm, k, o.b);
        MPI_Barrier(MPI_COMM_WORLD);
        const double t1 = MPI_Wtime();
        if (dev) (void)hipMemcpy(recv.data(), drecv.p, out_n * es, hipMemcpyDeviceToHost);
        const int ok_local = (err == CHR_SUCCESS && recv == ref) ? 1 : 0;  // data movement: exact
        int ok = 0;
        MPI_Allreduce(&ok_local, &ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
        double el = t1 - t0, el_max = 0;
        MPI_Reduce(&el, &el_max, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
        if (c.rank == 0)
            csv << "allgather_radix_batch," << k << "," << o.b << "," << c.nprocs << "," << count << "," << el_max
                << "," << ok << "\n" << std::flush;
    }
}

static void run_standard(const Options& o, Ctx& c, std::ofstream& csv, int count) {
    const chr_dtype dt = to_chr(o.dtype);
    const size_t es = esize(dt), out_n = (size_t)count * c.nprocs;
    std::vector<char> send, ref(out_n * es), recv(out_n * es);
    fill_input(send, count, dt, c.rank, count, o.pattern);
    MPI_Allgather(send.data(), count * (int)es, MPI_BYTE, ref.data(), count * (int)es, MPI_BYTE, MPI_COMM_WORLD);
    const int reps = o.reps > 0 ? o.reps : 50;
    for (int rep = 0; rep < reps; ++rep) {
        MPI_Barrier(MPI_COMM_WORLD);
        const double t0 = MPI_Wtime();
        const int err = MPI_Allgather(send.data(), count * (int)es, MPI_BYTE, recv.data(), count * (int)es, MPI_BYTE,
                                      MPI_COMM_WORLD);
        MPI_Barrier(MPI_COMM_WORLD);
        const double t1 = MPI_Wtime();
        const int ok_local = (err == MPI_SUCCESS && recv == ref) ? 1 : 0;
        int ok = 0;
        MPI_Allreduce(&ok_local, &ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
        double el = t1 - t0, el_max = 0;
        MPI_Reduce(&el, &el_max, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
        if (c.rank == 0)
            csv << "allgather_standard,0,0," << c.nprocs << "," << count << "," << el_max << "," << ok << "\n"
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
        const int count = o.base << i;
        if (o.k_only) {
            run_k_b(o, c, csv, o.k_only, count);
        } else {
            for (int k = 2; k < o.b; k += o.radix_increment) run_k_b(o, c, csv, k, count);
        }
        run_standard(o, c, csv, count);
    }
    if (c.rank == 0) csv.close();
    chr_comm_destroy(c.comm);
    MPI_Finalize();
    return EXIT_SUCCESS;
}
