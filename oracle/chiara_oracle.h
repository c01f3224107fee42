/*
 * chiara_oracle.h -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of CHiArA's hierarchical radix/batch reduce-scatter and allreduce
 * (reference: /root/reference/Fugaku_experiments/{Allreduce/all_reduce_radix_batch.cpp,
 * Reduce-scatter/reduce_scatter_radix_batch.cpp}) and of the MPICH 3.3.2 predefined
 * reduction loop behind MPI_Reduce_local, which is where the reference does all of its
 * arithmetic.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product (libchiara.so) never links or calls it.
 *
 * Parity pinning: tests/golden/ holds outputs of the REAL reference (its two algorithm
 * files compiled unchanged against the container's MPICH by oracle/Makefile target
 * `ref`, driven by oracle/ref_driver.cpp).  tests/test_oracle_golden.py checks this
 * restatement bit-exactly against them.
 *
 * The synthetic input generator below is shared by the golden driver, the oracle, the
 * numpy test helpers and the product's device fill kernel (same formula everywhere).
 */
#ifndef CHIARA_ORACLE_H
#define CHIARA_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same numbering as include/chiara.h (chr_dtype / chr_op). */
enum {
    ORC_F32 = 0, ORC_F64 = 1, ORC_I32 = 2, ORC_BF16 = 3,
    ORC_I8 = 4, ORC_U8 = 5, ORC_I16 = 6, ORC_U16 = 7, ORC_U32 = 8, ORC_I64 = 9, ORC_U64 = 10,
    /* MPI's pair types for MAXLOC / MINLOC ({value; int index} C structs, element = MPI extent) */
    ORC_FI = 11, ORC_DI = 12, ORC_LI = 13, ORC_2I = 14, ORC_SI = 15,
    /* MPI_C_FLOAT_COMPLEX, MPI_C_DOUBLE_COMPLEX */
    ORC_CF = 16, ORC_CD = 17
};
enum {
    ORC_SUM = 0, ORC_PROD = 1, ORC_MAX = 2, ORC_MIN = 3,
    ORC_LAND = 4, ORC_LOR = 5, ORC_LXOR = 6, ORC_BAND = 7, ORC_BOR = 8, ORC_BXOR = 9,
    ORC_MAXLOC = 10, ORC_MINLOC = 11,
    /* A user-defined, non-commutative MPI op for the user-op path (MPI_Op_create(fn, commute = 0)): MPI's user
     * function computes inout[i] = in[i] o inout[i]; this one is in * 0.5f + inout on MPI_FLOAT (rounded after the
     * multiply: no contraction), in * 0.5 + inout on MPI_DOUBLE and 3 * in + inout (wrapping) on MPI_INT.  Test
     * infrastructure: the same function is the reference's op in oracle/ref_driver.cpp and the device op in
     * tests/userop/halfadd_op.hip. */
    ORC_USER_HALFADD = 12,
    /* The same function created commutative (MPI_Op_create(fn, commute = 1)): identical arithmetic, but the MPICH
     * baselines that branch on MPI_Op_commutative take their commutative paths (allreduce_recursive_doubling.cpp:69,
     * reduce_scatter_recursive_doubling.cpp:134) -- which the non-commutative arithmetic then shows in the bits. */
    ORC_USER_HALFADD_C = 13
};

/* MPI_Op_commutative: every predefined op is commutative; the user ops as created. */
int orc_commutative(int op);

/* MPICH 3.3.2's (type, op) table as MPI_Reduce_local applies it (probed; pairs and complex:
 * oracle/ref_pairs_probe table, tests/golden/pairs_manifest.json); bf16 takes SUM/PROD/MAX/MIN. */
int orc_valid(int dtype, int op);

/* Input patterns for the generator. */
enum {
    ORC_PAT_UNIFORM = 0,  /* f32/f64/bf16: U[-1,1); integers: random bits of the full width */
    ORC_PAT_SEQ = 1,      /* the reference harness pattern: rank*count + i
                             (Fugaku_experiments/Allreduce/main.cpp:48-49) */
    ORC_PAT_TIES = 2,     /* MAX/MIN operand-order probe: each element one of {+0, -0, 1, -1,
                             0.5, NaN with a per-rank payload} (ints: {0, 1, -1, 2, 7}), so
                             ties and unordered compares are frequent and OP(a,b) vs OP(b,a)
                             differ bitwise.  Used with MAX/MIN (and the logical ops) only (NaN
                             payloads through arithmetic are not specified identically on CPU
                             and GPU). */
    ORC_PAT_SPARSE = 3    /* integer types: zero with probability 1/8, else nonzero random bits (the
                             logical ops: LAND results are a mix of 0 and 1 even at 8 ranks) */
};

static inline uint64_t orc_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static inline uint64_t orc_key(uint64_t seed, uint64_t rank, uint64_t i) {
    return orc_splitmix64(seed ^ (rank << 40) ^ i);
}

/* f32 -> bf16 round-to-nearest-even, NaN kept a (quiet) NaN. */
static inline uint16_t orc_f32_to_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return (uint16_t)((u >> 16) | 0x40u);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
static inline float orc_bf16_to_f32(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* Uniform value in [-1, 1) with 24 random bits: exactly representable in f32. */
static inline float orc_gen_f32(uint64_t seed, uint64_t rank, uint64_t i) {
    uint64_t u = orc_key(seed, rank, i);
    return (float)(u >> 40) * (1.0f / 8388608.0f) - 1.0f;
}
static inline double orc_gen_f64(uint64_t seed, uint64_t rank, uint64_t i) {
    uint64_t u = orc_key(seed, rank, i);
    return (double)(u >> 11) * (1.0 / 4503599627370496.0) - 1.0;
}

size_t orc_dtype_size(int dtype);  /* the element stride: MPI's extent for the pair types */

/* Fill `n` elements of rank `rank`'s buffer.  `count_for_seq` is the per-rank element
 * count used by the SEQ pattern (value = rank*count_for_seq + i, wrapping int32). */
void orc_fill(void* buf, size_t n, int dtype, int pattern, uint64_t seed, int rank,
              uint64_t count_for_seq);
/* Elements [start, start + n) of the same input (window of a full-size buffer). */
void orc_fill_at(void* buf, size_t n, int dtype, int pattern, uint64_t seed, int rank,
                 uint64_t count_for_seq, uint64_t start);

/* MPI_Reduce_local restated (MPICH 3.3.2 predefined ops): inout[i] = inout[i] (op) in[i]
 * (MPICH's loop order: MAX/MIN keep inout on ties and NaN compares).
 * int32 arithmetic wraps; bf16 is computed in f32 and rounded to bf16 RNE per call. */
void orc_reduce_local(const void* in, void* inout, size_t n, int dtype, int op);

/* Fused left-to-right form: acc = (((acc op ins[0]) op ins[1]) ... op ins[m-1]). */
void orc_reduce_multi(void* acc, const void* const* ins, int m, size_t n, int dtype, int op);

/* Recexch tables (all_reduce_radix_batch.cpp:11-198) for one group of `nranks` (= b). */
typedef struct {
    int k;               /* possibly clamped (:19-21) */
    int p_of_k, rem, T;
    int step1_sendto;    /* -1 for participants */
    int step1_nrecvs;
    int step1_recvfrom[64];
    int step2_nphases;
    int step2_nbrs[32][64];
} orc_recexch_t;

int orc_recexch_neighbors(int rank, int nranks, int k, orc_recexch_t* out);
void orc_recexch_count_offset(int nranks, int max_phases, int k, int* count, int* offset);

/* Whole-collective simulation of every rank of the communicator in one process.
 * send[r] / recv[r] point at rank r's buffers.  send[r] may be NULL for in-place
 * (then recv[r] holds the input, MPI_IN_PLACE semantics).
 * Return 0 on success, nonzero for the preconditions the reference leaves unchecked. */
int orc_allreduce_radix_batch(int nranks, int k, int b, size_t count, int dtype, int op,
                              const void* const* send, void* const* recv);
int orc_reduce_scatter_radix_batch(int nranks, int k, int b, size_t recvcount, int dtype,
                                   int op, const void* const* send, void* const* recv);

/* MPICH baseline allreduces driven by the reference's testing/main.cpp.
 * send[r] may be NULL (in place: recv[r] holds the input).  They follow MPI_Op_commutative (orc_commutative) where
 * the reference branches on it; 8 = the reference's MPI_ERR_OP (k_reduce_scatter_allgather with a non-commutative
 * op, recursive_multiplying with one at a size that is not a power of k). */
int orc_allreduce_ring(int nranks, size_t count, int dtype, int op, const void* const* send, void* const* recv);
int orc_allreduce_recursive_doubling(int nranks, size_t count, int dtype, int op, const void* const* send,
                                     void* const* recv);
int orc_allreduce_reduce_scatter_allgather(int nranks, size_t count, int dtype, int op, const void* const* send,
                                           void* const* recv);
int orc_allreduce_recexch(int nranks, int k, size_t count, int dtype, int op, const void* const* send,
                          void* const* recv);
int orc_allgather_radix_batch(int nranks, int k, int b, size_t sendcount, int dtype, const void* const* send,
                              void* const* recv);
int orc_allreduce_recursive_multiplying(int nranks, int k, size_t count, int dtype, int op,
                                        const void* const* send, void* const* recv);
int orc_allreduce_k_reduce_scatter_allgather(int nranks, int k, size_t count, int dtype, int op,
                                             const void* const* send, void* const* recv);

/* MPICH baseline reduce-scatters (block) of testing/mpich_implementations/reduce_scatter/: every
 * rank's result (rc elements) into recv[r]; send[r] holds n*rc elements (send[r] == NULL: in place,
 * the input is in recv[r]). */
int orc_reduce_scatter_pairwise(int n, size_t rc, int dtype, int op, const void* const* send, void* const* recv);
int orc_reduce_scatter_rec_halving(int n, size_t rc, int dtype, int op, const void* const* send,
                                   void* const* recv);
int orc_reduce_scatter_rec_doubling(int n, size_t rc, int dtype, int op, const void* const* send,
                                    void* const* recv);
int orc_reduce_scatter_radix(int n, int k, size_t rc, int dtype, int op, const void* const* send,
                             void* const* recv);

/* CHiArA's phases as stand-alone functions (testing/custom_implementations/work_dir/reduce_scatter/).
 * Ranks form n / b groups of b (node = r / b, lane = r % b); IRC = rc * b; nstages = nnodes / b,
 * nu = nnodes % b.  Each writes only what the reference writes into recv[r]; the rest of recv[r] is
 * left as it was.
 *   intra_reduce_scatter: send[r] (NULL: in place, recv[r]) holds rc * n elements; recv[r][s * IRC]
 *     gets chunk s * b + lane reduced over the group (leftover stage: lanes < nu).
 *   inter_reduce_linear: send[r] holds niters chunks of IRC; the root of iteration i (node i * b +
 *     lane) gets its chunk i folded with every other node's chunk i in ascending node order.
 *   intra_scatter: the node root's send (b blocks of rc) scattered, block `lane` to each rank; send[r]
 *     is read on node roots only. */
int orc_intra_reduce_scatter(int n, int k, int b, size_t rc, int dtype, int op, const void* const* send,
                             void* const* recv);
int orc_inter_reduce_linear(int n, int b, size_t rc, int dtype, int op, const void* const* send, void* const* recv);
int orc_intra_scatter(int n, int k, int b, size_t rc, int dtype, const void* const* send, void* const* recv);

#ifdef __cplusplus
}
#endif
#endif
