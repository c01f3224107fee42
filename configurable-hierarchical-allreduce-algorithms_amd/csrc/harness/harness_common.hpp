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
};

inline bool parse(int argc, char** argv, Options* o, int rank) {
    if (argc < 2) {
        if (rank == 0)
            std::fprintf(stderr,
                         "Usage: %s <n_iter> [--overwrite] [b=<value>] [base=<value>] [num_nodes=<value>] "
                         "[radix_increment=<value>] [dtype=i32|f32|f64|bf16] [mem=host|device] [reps=<n>] [k=<k>]\n",
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

// Element i of rank r's input: the reference harness pattern rank*count + i (int32 wraps),
// converted to the element type (Fugaku_experiments/Allreduce/main.cpp:48-49).
inline void fill_seq(std::vector<char>& buf, size_t n, chr_dtype d, int rank, size_t count_for_seq) {
    buf.assign(n * esize(d), 0);
    for (size_t i = 0; i < n; ++i) {
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

// is_correct: exact for integers (the reference's fabs(diff) > 1e-9 test,
// Allreduce/main.cpp:16-24); floats within (n-1) ulps of the reduced magnitude
// (a different association than MPI's own collective).
inline bool check_correctness(const std::vector<char>& got, const std::vector<char>& ref, size_t n, chr_dtype d,
                              int nranks) {
    const double ulp = d == CHR_FLOAT32 ? std::ldexp(1.0, -23) : d == CHR_BFLOAT16 ? std::ldexp(1.0, -8)
                       : d == CHR_FLOAT64 ? std::ldexp(1.0, -52) : 0.0;
    for (size_t i = 0; i < n; ++i) {
        const double g = elem(got, i, d), r = elem(ref, i, d);
        const double tol = d == CHR_INT32 ? 1e-9 : (nranks - 1) * ulp * std::fabs(r) * 2 + 1e-30;
        if (!(std::fabs(g - r) <= tol)) return false;
    }
    return true;
}

inline MPI_Datatype mpi_type(chr_dtype d) {
    return d == CHR_INT32 ? MPI_INT : d == CHR_FLOAT32 ? MPI_FLOAT : d == CHR_FLOAT64 ? MPI_DOUBLE : MPI_DATATYPE_NULL;
}

// Host-side reference collective (bf16 via f32 then RNE; small-integer inputs keep it exact).
inline void bf16_sum_op(void* in, void* inout, int* len, MPI_Datatype*) {
    uint16_t* a = (uint16_t*)in;
    uint16_t* b = (uint16_t*)inout;
    for (int i = 0; i < *len; ++i) {
        float f = bf2f(a[i]) + bf2f(b[i]);
        uint32_t u;
        std::memcpy(&u, &f, 4);
        u += 0x7FFFu + ((u >> 16) & 1u);
        b[i] = (uint16_t)(u >> 16);
    }
}

struct Ctx {
    int rank = 0, nprocs = 1, device = 0;
    chr_comm* comm = nullptr;
    MPI_Datatype bf16 = MPI_DATATYPE_NULL;
    MPI_Op bf16_sum = MPI_OP_NULL;
};

inline int init(Ctx* c) {
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
