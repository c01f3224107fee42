// ref_driver.cpp -- TEST INFRASTRUCTURE ONLY, container-only.
//
// Drives the REAL reference algorithms, compiled unchanged from where they lie:
//   /root/reference/Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp
//   /root/reference/Fugaku_experiments/Reduce-scatter/reduce_scatter_radix_batch.cpp
// against the container's MPICH 3.3.2 (/opt/conda), to produce golden vectors for
// tests/golden/.  Build: `make -C oracle ref`; run: tests/golden/gen_golden.py.
// Nothing from /root/reference is copied; this file only declares the two entry points
// with the signatures at all_reduce_radix_batch.cpp:202-204 and
// reduce_scatter_radix_batch.cpp:200-202.
//
// Usage: mpiexec -n N ref_driver <cases.txt> <outdir>
//   one case per line: id mode k b count dtype op pattern seed inplace
//   mode: ar | rs | ag (radix_batch), ring | rd | rsag | rx | krsag | rm (MPICH baseline allreduces;
//   rx and krsag use b as single_phase_recv), rs_radix | rs_halving | rs_doubling | rs_pairwise
//   (MPICH baseline reduce-scatters, count = recvcount; rs_radix uses k), irs | ilr | isc (CHiArA's
//   phases as stand-alone functions in testing/custom_implementations/work_dir/reduce_scatter/:
//   intra_reduce_scatter_radix_batch, inter_reduce_linear, intra_scatter_radix_batch; count = recvcount)
// For each case rank 0 writes <outdir>/<id>.out (all ranks' outputs, rank-major) and
// <outdir>/<id>.lib (the MPI library collective's result on the same inputs).
#include <mpi.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "chiara_oracle.h"

int all_reduce_radix_batch(char* sendbuf, char* recvbuf, int aCount, MPI_Datatype datatype,
                           MPI_Op op, MPI_Comm comm, int k, int b);
int reduce_scatter_radix_batch(const void* sendbuf, void* recvbuf, MPI_Aint recvcount,
                               MPI_Datatype datatype, MPI_Op op, MPI_Comm comm, int k, int b);
// testing/mpich_implementations/all_reduce/ (the baselines testing/main.cpp drives)
int MPICH_Allreduce_ring(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                         MPI_Comm comm);
int MPICH_Allreduce_recursive_doubling(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                       MPI_Op op, MPI_Comm comm);
int MPICH_Allreduce_reduce_scatter_allgather(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                             MPI_Op op, MPI_Comm comm);
int MPICH_Allreduce_recursive_exchange(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                       MPI_Op op, MPI_Comm comm, int k, int single_phase_recv);
int MPICH_Allreduce_k_reduce_scatter_allgather(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                               MPI_Op op, MPI_Comm comm, int k, int single_phase_recv);
// Fugaku_experiments/Allgather/all_gather_radix_batch_1_0.cpp:37
int allgather_radix_batch(char* sendbuf, int sendcount, MPI_Datatype datatype, char* recvbuf, MPI_Comm comm, int k,
                          int b);
int MPICH_Allreduce_recursive_multiplying(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                          MPI_Op op, MPI_Comm comm, int k);
// testing/mpich_implementations/reduce_scatter/ (the baselines that directory's main.cpp drives)
int MPICH_reduce_scatter_rec_halving(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                                     MPI_Comm comm);
int MPICH_reduce_scatter_rec_doubling(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                                      MPI_Op op, MPI_Comm comm);
int MPICH_reduce_scatter_radix(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                               MPI_Op op, MPI_Comm comm, int k);
int MPICH_reduce_scatter_pairwise(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                                  MPI_Op op, MPI_Comm comm);

// testing/custom_implementations/work_dir/reduce_scatter/ (CHiArA's phases, stand-alone)
int intra_reduce_scatter_radix_batch(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                                     MPI_Op op, MPI_Comm comm, int k, int b);  // intra_reduce_scatter_radix.cpp:208
int inter_reduce_linear(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype, MPI_Op op,
                        MPI_Comm comm, int b);  // inter_linear_reduce.cpp:11
int intra_scatter_radix_batch(char* sendbuf, int recvcount, MPI_Datatype datatype, char* recvbuf, MPI_Comm comm, int k,
                              int b);  // intra_scatter_radix_batch.cpp:10

// orc_reduce_local is the single definition of the bf16 op semantics.
static void bf16_user_op(void* in, void* inout, int* len, MPI_Datatype*) {
    orc_reduce_local(in, inout, (size_t)*len, ORC_BF16, ORC_SUM);
}
static void bf16_user_max(void* in, void* inout, int* len, MPI_Datatype*) {
    orc_reduce_local(in, inout, (size_t)*len, ORC_BF16, ORC_MAX);
}
static void bf16_user_min(void* in, void* inout, int* len, MPI_Datatype*) {
    orc_reduce_local(in, inout, (size_t)*len, ORC_BF16, ORC_MIN);
}
static void bf16_user_prod(void* in, void* inout, int* len, MPI_Datatype*) {
    orc_reduce_local(in, inout, (size_t)*len, ORC_BF16, ORC_PROD);
}

// The user-defined op of the user-op path (chiara_oracle.h ORC_USER_HALFADD), written here independently of the
// oracle: MPI's user-function contract inout[i] = in[i] o inout[i], o = in * 0.5 + inout on MPI_FLOAT / MPI_DOUBLE,
// 3 * in + inout (wrapping) on MPI_INT; created non-commutative (and, as user_halfadd_c, commutative).
template <typename T>
static void halfadd_loop(const void* in, void* inout, int len) {
    const T* a = (const T*)in;
    T* b = (T*)inout;
    for (int i = 0; i < len; ++i) {
        const T h = a[i] * (T)0.5;
        b[i] = h + b[i];
    }
}
static void halfadd_user_op(void* in, void* inout, int* len, MPI_Datatype* dt) {
    if (*dt == MPI_DOUBLE) {
        halfadd_loop<double>(in, inout, *len);
    } else if (*dt == MPI_INT) {
        const uint32_t* a = (const uint32_t*)in;
        uint32_t* b = (uint32_t*)inout;
        for (int i = 0; i < *len; ++i) b[i] = a[i] * 3u + b[i];
    } else {
        halfadd_loop<float>(in, inout, *len);
    }
}

static int parse_dtype(const std::string& s) {
    static const char* names[] = {"f32", "f64", "i32", "bf16", "i8", "u8", "i16", "u16", "u32", "i64", "u64",
                                  "fi",  "di",  "li",  "2i",   "si", "cf", "cd"};
    for (int d = 0; d < (int)(sizeof(names) / sizeof(names[0])); ++d)
        if (s == names[d]) return d;
    return -1;
}
static int parse_op(const std::string& s) {
    static const char* names[] = {"sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor",
                                  "maxloc", "minloc", "user_halfadd", "user_halfadd_c"};
    for (int o = 0; o < (int)(sizeof(names) / sizeof(names[0])); ++o)
        if (s == names[o]) return o;
    return -1;
}
// MPI predefined types for the oracle's dtypes (bf16: the user type below)
static MPI_Datatype mpi_type_of(int dtype) {
    switch (dtype) {
    case ORC_F32: return MPI_FLOAT;
    case ORC_F64: return MPI_DOUBLE;
    case ORC_I32: return MPI_INT;
    case ORC_I8: return MPI_SIGNED_CHAR;
    case ORC_U8: return MPI_UNSIGNED_CHAR;
    case ORC_I16: return MPI_SHORT;
    case ORC_U16: return MPI_UNSIGNED_SHORT;
    case ORC_U32: return MPI_UNSIGNED;
    case ORC_I64: return MPI_INT64_T;
    case ORC_U64: return MPI_UINT64_T;
    case ORC_FI: return MPI_FLOAT_INT;
    case ORC_DI: return MPI_DOUBLE_INT;
    case ORC_LI: return MPI_LONG_INT;
    case ORC_2I: return MPI_2INT;
    case ORC_SI: return MPI_SHORT_INT;
    case ORC_CF: return MPI_C_FLOAT_COMPLEX;
    case ORC_CD: return MPI_C_DOUBLE_COMPLEX;
    default: return MPI_DATATYPE_NULL;
    }
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int rank, nprocs;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &nprocs);
    if (argc != 3) {
        if (rank == 0) fprintf(stderr, "usage: ref_driver cases.txt outdir\n");
        MPI_Finalize();
        return 1;
    }
    MPI_Datatype bf16_t;
    MPI_Type_contiguous(2, MPI_BYTE, &bf16_t);
    MPI_Type_commit(&bf16_t);
    MPI_Op bf16_ops[4];
    MPI_Op_create(bf16_user_op, 1, &bf16_ops[ORC_SUM]);
    MPI_Op_create(bf16_user_prod, 1, &bf16_ops[ORC_PROD]);
    MPI_Op_create(bf16_user_max, 1, &bf16_ops[ORC_MAX]);
    MPI_Op_create(bf16_user_min, 1, &bf16_ops[ORC_MIN]);
    MPI_Op halfadd_op, halfadd_c_op;
    MPI_Op_create(halfadd_user_op, 0, &halfadd_op);    // commute = 0
    MPI_Op_create(halfadd_user_op, 1, &halfadd_c_op);  // the same function declared commutative
    const MPI_Op std_ops[14] = {MPI_SUM,  MPI_PROD, MPI_MAX,  MPI_MIN,    MPI_LAND,   MPI_LOR,    MPI_LXOR,
                                MPI_BAND, MPI_BOR,  MPI_BXOR, MPI_MAXLOC, MPI_MINLOC, halfadd_op, halfadd_c_op};

    std::ifstream cases(argv[1]);
    std::string line;
    while (std::getline(cases, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::istringstream is(line);
        std::string id, mode, dts, ops;
        int k, b, pattern, inplace;
        long long count;
        unsigned long long seed;
        is >> id >> mode >> k >> b >> count >> dts >> ops >> pattern >> seed >> inplace;
        int dtype = parse_dtype(dts), op = parse_op(ops);
        if (dtype < 0 || op < 0 || !orc_valid(dtype, op)) {
            if (rank == 0) fprintf(stderr, "bad case: %s\n", line.c_str());
            continue;
        }
        size_t es = orc_dtype_size(dtype);
        MPI_Datatype mdt = dtype == ORC_BF16 ? bf16_t : mpi_type_of(dtype);
        MPI_Op mop = dtype == ORC_BF16 ? bf16_ops[op] : std_ops[op];

        const bool rs_mode = mode == "rs" || mode.rfind("rs_", 0) == 0;  // rs_lib included
        size_t in_n = rs_mode ? (size_t)count * nprocs : (size_t)count;
        size_t out_n = (mode == "ag") ? (size_t)count * nprocs : (size_t)count;
        const bool phase_mode = mode == "irs" || mode == "ilr" || mode == "isc";
        if (phase_mode) {  // sizes as tests/../oracle/pyoracle.py phase_sizes
            const size_t nnodes = (size_t)nprocs / b, niters = nnodes / b + (nnodes % b ? 1 : 0), irc = (size_t)count * b;
            in_n = mode == "irs" ? (size_t)count * nprocs : mode == "ilr" ? niters * irc : (size_t)b * count;
            out_n = mode == "irs" ? niters * irc : mode == "ilr" ? irc : (size_t)count;
            if (in_n < out_n) in_n = out_n;  // recv is allocated with in_n elements
        }
        std::vector<char> send(in_n * es), recv(in_n * es, 0), lib(out_n * es, 0);
        int ref_rc = 0;  // the MPICH baselines' return code (MPI_ERR_OP where they refuse the op)
        orc_fill(send.data(), in_n, dtype, pattern, seed, rank, in_n);

        if (phase_mode) {
            // no library counterpart: .lib stays zero; recv starts zero, and what a rank does not write stays so
            if (inplace) memcpy(recv.data(), send.data(), in_n * es);
            MPI_Barrier(MPI_COMM_WORLD);
            if (mode == "irs")
                intra_reduce_scatter_radix_batch(inplace ? MPI_IN_PLACE : (const void*)send.data(), recv.data(),
                                                 (MPI_Aint)count, mdt, mop, MPI_COMM_WORLD, k, b);
            else if (mode == "ilr")
                inter_reduce_linear(send.data(), recv.data(), (MPI_Aint)count, mdt, mop, MPI_COMM_WORLD, b);
            else
                intra_scatter_radix_batch(send.data(), (int)count, mdt, recv.data(), MPI_COMM_WORLD, k, b);
        } else if (mode == "ar_lib" || mode == "rs_lib") {
            // MPI's own collective only: the expected output for the pair types whose MPI_Type_size is
            // not their extent (MPI_DOUBLE_INT, MPI_LONG_INT, MPI_SHORT_INT), where the reference's
            // byte arithmetic (all_reduce_radix_batch.cpp:238-256 takes MPI_Type_size as the element
            // stride) does not address the buffer MPI describes
            if (mode == "ar_lib") MPI_Allreduce(send.data(), lib.data(), (int)count, mdt, mop, MPI_COMM_WORLD);
            else MPI_Reduce_scatter_block(send.data(), lib.data(), (int)count, mdt, mop, MPI_COMM_WORLD);
            recv.assign(lib.begin(), lib.end());
        } else if (mode == "ag") {
            MPI_Allgather(send.data(), (int)count, mdt, lib.data(), (int)count, mdt, MPI_COMM_WORLD);
            recv.assign(out_n * es, 0);
            MPI_Barrier(MPI_COMM_WORLD);
            allgather_radix_batch(send.data(), (int)count, mdt, recv.data(), MPI_COMM_WORLD, k, b);
        } else if (mode == "ar") {
            MPI_Allreduce(send.data(), lib.data(), (int)count, mdt, mop, MPI_COMM_WORLD);
            if (inplace) memcpy(recv.data(), send.data(), in_n * es);
            MPI_Barrier(MPI_COMM_WORLD);
            all_reduce_radix_batch(inplace ? (char*)MPI_IN_PLACE : send.data(), recv.data(), (int)count,
                                   mdt, mop, MPI_COMM_WORLD, k, b);
        } else if (mode == "ring" || mode == "rd" || mode == "rsag" || mode == "rx" || mode == "krsag" ||
                   mode == "rm") {
            MPI_Allreduce(send.data(), lib.data(), (int)count, mdt, mop, MPI_COMM_WORLD);
            if (inplace) memcpy(recv.data(), send.data(), in_n * es);
            MPI_Barrier(MPI_COMM_WORLD);
            const char* sb = inplace ? (const char*)MPI_IN_PLACE : send.data();
            if (mode == "ring") ref_rc = MPICH_Allreduce_ring(sb, recv.data(), (int)count, mdt, mop, MPI_COMM_WORLD);
            else if (mode == "rd")
                ref_rc = MPICH_Allreduce_recursive_doubling(sb, recv.data(), (int)count, mdt, mop, MPI_COMM_WORLD);
            else if (mode == "rsag")
                ref_rc = MPICH_Allreduce_reduce_scatter_allgather(sb, recv.data(), (int)count, mdt, mop, MPI_COMM_WORLD);
            else if (mode == "rx")
                ref_rc = MPICH_Allreduce_recursive_exchange(sb, recv.data(), (int)count, mdt, mop, MPI_COMM_WORLD, k, b);
            else if (mode == "krsag")
                ref_rc = MPICH_Allreduce_k_reduce_scatter_allgather(sb, recv.data(), (int)count, mdt, mop,
                                                                    MPI_COMM_WORLD, k, b);
            else ref_rc = MPICH_Allreduce_recursive_multiplying(sb, recv.data(), (int)count, mdt, mop, MPI_COMM_WORLD, k);
        } else if (mode.rfind("rs_", 0) == 0) {
            MPI_Reduce_scatter_block(send.data(), lib.data(), (int)count, mdt, mop, MPI_COMM_WORLD);
            if (inplace) memcpy(recv.data(), send.data(), in_n * es);
            MPI_Barrier(MPI_COMM_WORLD);
            const void* sb = inplace ? MPI_IN_PLACE : (const void*)send.data();
            if (mode == "rs_radix")
                ref_rc = MPICH_reduce_scatter_radix(sb, recv.data(), (MPI_Aint)count, mdt, mop, MPI_COMM_WORLD, k);
            else if (mode == "rs_halving")
                ref_rc = MPICH_reduce_scatter_rec_halving((const char*)sb, recv.data(), (int)count, mdt, mop,
                                                          MPI_COMM_WORLD);
            else if (mode == "rs_doubling")
                ref_rc = MPICH_reduce_scatter_rec_doubling(sb, recv.data(), (MPI_Aint)count, mdt, mop, MPI_COMM_WORLD);
            else
                ref_rc = MPICH_reduce_scatter_pairwise(sb, recv.data(), (MPI_Aint)count, mdt, mop, MPI_COMM_WORLD);
        } else {
            MPI_Reduce_scatter_block(send.data(), lib.data(), (int)count, mdt, mop, MPI_COMM_WORLD);
            if (inplace) memcpy(recv.data(), send.data(), in_n * es);
            MPI_Barrier(MPI_COMM_WORLD);
            reduce_scatter_radix_batch(inplace ? MPI_IN_PLACE : (const void*)send.data(), recv.data(),
                                       (MPI_Aint)count, mdt, mop, MPI_COMM_WORLD, k, b);
        }
        MPI_Barrier(MPI_COMM_WORLD);
        std::vector<char> all(rank == 0 ? out_n * es * nprocs : 1), all_lib(rank == 0 ? out_n * es * nprocs : 1);
        MPI_Gather(recv.data(), (int)(out_n * es), MPI_BYTE, all.data(), (int)(out_n * es), MPI_BYTE, 0,
                   MPI_COMM_WORLD);
        MPI_Gather(lib.data(), (int)(out_n * es), MPI_BYTE, all_lib.data(), (int)(out_n * es), MPI_BYTE, 0,
                   MPI_COMM_WORLD);
        std::vector<int> all_rc(rank == 0 ? nprocs : 1);
        MPI_Gather(&ref_rc, 1, MPI_INT, all_rc.data(), 1, MPI_INT, 0, MPI_COMM_WORLD);
        if (rank == 0) {
            std::string base = std::string(argv[2]) + "/" + id;
            FILE* f = fopen((base + ".out").c_str(), "wb");
            fwrite(all.data(), 1, out_n * es * nprocs, f);
            fclose(f);
            f = fopen((base + ".lib").c_str(), "wb");
            fwrite(all_lib.data(), 1, out_n * es * nprocs, f);
            fclose(f);
            f = fopen((base + ".rc").c_str(), "w");  // every rank's return code, rank order
            for (int r = 0; r < nprocs; ++r) fprintf(f, "%d\n", all_rc[r]);
            fclose(f);
        }
    }
    MPI_Finalize();
    return 0;
}
