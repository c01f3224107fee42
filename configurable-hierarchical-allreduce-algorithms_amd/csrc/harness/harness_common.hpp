// harness_common.hpp -- shared pieces of the MPI harnesses (bin/chiara_allreduce,
// bin/chiara_reduce_scatter) that keep the reference's CLI, CSV schema and is_correct
// surface (Fugaku_experiments/{Allreduce,Reduce-scatter}/main.cpp) while the
// collective runs through libchiara (RCCL over xGMI + HIP bucket-reduction kernels).
// MPI is only the launcher/control plane here: rank discovery, the RCCL unique-id
// broadcast, barriers, MPI_Wtime and the library reference collective for is_correct.
#pragma once

#include <mpi.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "chiara.h"

namespace harness {

struct Options {
    int n_iter = 0;
    bool overwrite = false;
    int b = 16;
    int base = 1;
    int num_nodes = 1;
    int radix_increment = 1;
    // extensions (not in the reference CLI)
    std::string dtype = "i32";   // reference harnesses use MPI_INT
    std::string mem = "host";    // host: the reference's host-memory contract; device: HBM-resident
    int reps = -1;               // default: reference's 50 (allreduce) / 20 (reduce-scatter)
    int k_only = 0;              // run a single k instead of the reference's k sweep
    std::string pattern = "seq"; // seq: the reference's rank*count+i; cancel: sign-alternating ranks
};

inline bool parse(int argc, char** argv, Options* o, int rank) {
    if (argc < 2) {
        if (rank == 0)
            std::fprintf(stderr,
                         "Usage: %s <n_iter> [--overwrite] [b=<value>] [base=<value>] [num_nodes=<value>] "
                         "[radix_increment=<value>] [dtype=i32|f32|f64|bf16] [mem=host|device] [reps=<n>] [k=<k>] "
                         "[pattern=seq|cancel]\n",
                         argv[0]);
        return false;
    }
    o->n_iter = std::atoi(argv[1]);
    for (int i = 2; i < argc; ++i) {
        const char* a = argv[i];
        if (!std::strcmp(a, "--overwrite")) o->overwrite = true;
        else if (!std::strncmp(a, "b=", 2)) o->b = std::atoi(a + 2);
        else if (!std::strncmp(a, "base=", 5)) o->base = std::atoi(a + 5);
        else if (!std::strncmp(a, "num_nodes=", 10)) o->num_nodes = std::atoi(a + 10);
        else if (!std::strncmp(a, "radix_increment=", 16)) o->radix_increment = std::atoi(a + 16);
        else if (!std::strncmp(a, "dtype=", 6)) o->dtype = a + 6;
        else if (!std::strncmp(a, "mem=", 4)) o->mem = a + 4;
        else if (!std::strncmp(a, "reps=", 5)) o->reps = std::atoi(a + 5);
        else if (!std::strncmp(a, "k=", 2)) o->k_only = std::atoi(a + 2);
        else if (!std::strncmp(a, "pattern=", 8)) o->pattern = a + 8;
        else {
            if (rank == 0) std::fprintf(stderr, "Unknown parameter: %s\n", a);
            return false;
        }
    }
    return true;
}

inline chr_dtype to_chr(const std::string& d) {
    if (d == "f32") return CHR_FLOAT32;
    if (d == "f64") return CHR_FLOAT64;
    if (d == "bf16") return CHR_BFLOAT16;
    return CHR_INT32;
}
inline size_t esize(chr_dtype d) { return d == CHR_FLOAT64 ? 8 : d == CHR_BFLOAT16 ? 2 : 4; }

inline float bf2f(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

inline uint16_t f2bf_rne(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Element i of rank r's input.
//  seq:    the reference harness pattern rank*count + i (int32 wraps), converted to the element
//          type (Fugaku_experiments/Allreduce/main.cpp:48-49).
//  cancel: ranks alternate the sign of one common large value per element plus a small per-rank
//          term, so the reduced value is tiny next to sum|x_i|: a different association than MPI's
//          own collective then differs by far more than ulp(|result|), but stays inside the
//          stated tolerance (n-1)*ulp*sum|x_i| (check_correctness).
inline void fill_input(std::vector<char>& buf, size_t n, chr_dtype d, int rank, size_t count_for_seq,
                       const std::string& pattern) {
    buf.assign(n * esize(d), 0);
    const bool cancel = pattern == "cancel";
    for (size_t i = 0; i < n; ++i) {
        if (cancel) {
            const double big = 1.0 + (double)(splitmix64(0xC0FFEEull ^ i) >> 44) / 1024.0;  // [1, 1025)
            const double small = (double)(splitmix64(((uint64_t)rank << 40) ^ i) >> 40) / (double)(1ull << 30);
            const double v = (rank % 2 ? -big : big) + small;
            switch (d) {
            case CHR_INT32: ((int32_t*)buf.data())[i] = (int32_t)(v * 64.0); break;
            case CHR_FLOAT32: ((float*)buf.data())[i] = (float)v; break;
            case CHR_FLOAT64: ((double*)buf.data())[i] = v; break;
            default: ((uint16_t*)buf.data())[i] = f2bf_rne((float)v);
            }
            continue;
        }
        const int32_t v = (int32_t)(uint32_t)((uint64_t)rank * count_for_seq + i);
        switch (d) {
        case CHR_INT32: ((int32_t*)buf.data())[i] = v; break;
        case CHR_FLOAT32: ((float*)buf.data())[i] = (float)(v % 1024) * 0.125f; break;
        case CHR_FLOAT64: ((double*)buf.data())[i] = (double)v; break;
        default: {
            float f = (float)(v % 64) * 0.25f;
            uint32_t u;
            std::memcpy(&u, &f, 4);
            ((uint16_t*)buf.data())[i] = (uint16_t)(u >> 16);  // exact: few significant bits
        }
        }
    }
}

inline double elem(const std::vector<char>& b, size_t i, chr_dtype d) {
    switch (d) {
    case CHR_INT32: return ((const int32_t*)b.data())[i];
    case CHR_FLOAT32: return ((const float*)b.data())[i];
    case CHR_FLOAT64: return ((const double*)b.data())[i];
    default: return bf2f(((const uint16_t*)b.data())[i]);
    }
}

// |x_i| of this rank's input, as doubles: reduced with the same MPI collective as the data
// (MPI_SUM on MPI_DOUBLE), it gives sum over ranks of |x_i| per output element, the scale of the
// float tolerance below.
inline std::vector<double> abs_values(const std::vector<char>& b, size_t n, chr_dtype d) {
    std::vector<double> a(n);
    for (size_t i = 0; i < n; ++i) a[i] = std::fabs(elem(b, i, d));
    return a;
}

// is_correct: exact for integers (the reference's fabs(diff) > 1e-9 test,
// Allreduce/main.cpp:16-24).  Floats: MPI's own collective associates differently, so the
// stated bound is |x - lib| <= (n-1) * ulp * sum_r |x_r[i]| with ulp = 2^-23 (f32), 2^-52 (f64)
// and 2^-8 (bf16, RNE after every step): each of the two sums is within (n-1)*u*sum|x| of the
// exact sum (u = ulp/2).  sumabs[i] = sum_r |x_r[i]| (abs_values reduced over the ranks).
inline bool check_correctness(const std::vector<char>& got, const std::vector<char>& ref,
                              const std::vector<double>& sumabs, size_t n, chr_dtype d, int nranks) {
    const double ulp = d == CHR_FLOAT32 ? std::ldexp(1.0, -23) : d == CHR_BFLOAT16 ? std::ldexp(1.0, -8)
                       : d == CHR_FLOAT64 ? std::ldexp(1.0, -52) : 0.0;
    for (size_t i = 0; i < n; ++i) {
        const double g = elem(got, i, d), r = elem(ref, i, d);
        const double tol = d == CHR_INT32 ? 1e-9 : (nranks - 1) * ulp * sumabs[i] + 1e-300;
        if (!(std::fabs(g - r) <= tol)) return false;
    }
    return true;
}

inline MPI_Datatype mpi_type(chr_dtype d) {
    return d == CHR_INT32 ? MPI_INT : d == CHR_FLOAT32 ? MPI_FLOAT : d == CHR_FLOAT64 ? MPI_DOUBLE : MPI_DATATYPE_NULL;
}

// Host-side reference collective for bf16: f32 add then RNE (an MPI user op).
inline void bf16_sum_op(void* in, void* inout, int* len, MPI_Datatype*) {
    uint16_t* a = (uint16_t*)in;
    uint16_t* b = (uint16_t*)inout;
    for (int i = 0; i < *len; ++i) b[i] = f2bf_rne(bf2f(a[i]) + bf2f(b[i]));
}

struct Ctx {
    int rank = 0, nprocs = 1, device = 0;
    chr_comm* comm = nullptr;
    MPI_Datatype bf16 = MPI_DATATYPE_NULL;
    MPI_Op bf16_sum = MPI_OP_NULL;
};

inline int init(Ctx* c, const Options& o) {
    MPI_Comm_rank(MPI_COMM_WORLD, &c->rank);
    MPI_Comm_size(MPI_COMM_WORLD, &c->nprocs);
    MPI_Comm local;
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, c->rank, MPI_INFO_NULL, &local);
    int lrank = 0;
    MPI_Comm_rank(local, &lrank);
    MPI_Comm_free(&local);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        std::fprintf(stderr, "rank %d: no HIP device\n", c->rank);
        return CHR_ERR_NO_DEVICE;
    }
    c->device = lrank % ndev;
    chr_unique_id id;
    if (c->rank == 0 && chr_get_unique_id(&id) != CHR_SUCCESS) return CHR_ERR_RCCL;
    MPI_Bcast(&id, sizeof(id), MPI_BYTE, 0, MPI_COMM_WORLD);
    int rc = chr_comm_init_rank(&c->comm, c->nprocs, &id, c->rank, c->device);
    // mem=host on every rank (one CLI): pipelined host staging, as the shim does (chiara.h); the
    // device-resident runs keep one collective per call
    if (rc == CHR_SUCCESS && o.mem == "host" && !std::getenv("CHR_HOST_WINDOW_MIB"))
        rc = chr_comm_set_host_pipeline(c->comm, 32);
    MPI_Type_contiguous(2, MPI_BYTE, &c->bf16);
    MPI_Type_commit(&c->bf16);
    MPI_Op_create(bf16_sum_op, 1, &c->bf16_sum);
    return rc;
}

inline std::ofstream open_csv(const Options& o, int rank, int nprocs) {
    std::ofstream csv;
    if (rank == 0) {
        // results<ranks per node>_<num_nodes>_<b>.csv (Allreduce/main.cpp:167-183)
        const std::string fn = "results" + std::to_string(nprocs / o.num_nodes) + "_" + std::to_string(o.num_nodes) +
                               "_" + std::to_string(o.b) + ".csv";
        const bool exists = std::ifstream(fn).good();
        if (o.overwrite || !exists) {
            csv.open(fn, std::ios::out | std::ios::trunc);
            csv << "algorithm_name,k,b,nprocs,send_count,time,is_correct\n";
        } else {
            csv.open(fn, std::ios::out | std::ios::app);
        }
    }
    return csv;
}

// Device buffer helper (mem=device): inputs copied once before the timed reps.
struct DevBuf {
    void* p = nullptr;
    explicit DevBuf(size_t bytes) { (void)hipMalloc(&p, bytes ? bytes : 1); }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace harness
