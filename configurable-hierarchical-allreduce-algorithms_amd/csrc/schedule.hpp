// schedule.hpp -- host-side radix/batch schedule compiler (no device code).
//
// Re-states CHiArA's hierarchical reduce-scatter / allreduce schedule
// (Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp:202-788,
//  Fugaku_experiments/Reduce-scatter/reduce_scatter_radix_batch.cpp:200-653)
// as a per-rank PLAN: a list of steps, each one RCCL group of sends/receives followed by
// local device ops (fused bucket reductions, copies).  Steps are numbered globally, so
// every message is posted by both of its endpoints in the same step and a rank can
// enqueue its whole plan without ever blocking the host (deadlock-free by construction).
//
// HBM layout of the accumulator (ACC): slice-major, then block-major.  The reference keeps
// tmp_results stage-major ([stage][lane block][IRC], :339-400), so each recexch phase
// touches `nstages` (+1 truncated) separate slices.  Here chunk N = stage*b + lane sits
// at position P[lane] + stage, i.e. [lane block][stage][IRC]: the region a phase
// exchanges is ONE contiguous range covering every stage (and exactly the reference's
// truncated leftover-stage region, :422-446), so each neighbour gets one message and
// each phase is one fused kernel.  Element-wise reduction order is unchanged.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace chr {

enum Buf : uint8_t { BUF_SEND = 0, BUF_RECV = 1, BUF_ACC = 2, BUF_STAGE = 3 };

struct Ref {
    uint8_t buf;
    uint64_t off;  // elements
};

struct Xfer {
    int peer;
    Ref ref;
    uint64_t count;  // elements
};

enum LocalKind : uint8_t { L_COPY = 0, L_REDUCE = 1, L_COPY2D = 2, L_TREE = 3 };

// L_REDUCE: dst = (...((acc op ins[0]) op ins[1])...) op ins[m-1]   (dst may equal acc)
// L_COPY:   dst = acc                                    (count elements)
// L_COPY2D: rows x count elements, row r: dst + r*dpitch <- acc + r*spitch
// L_TREE:   dst = one whole expression tree (chr_reduce_tree): leaves acc, ins[0], ins[1], ...
//           in push order; comb[j] combines after leaf j; swaps[c] per combine
constexpr int kTreeMaxLeaves = 8;  // kMaxLeaves, reduce_tree.hip
constexpr int kTreeMaxDepth = 4;   // kTreeDepth
struct LocalOp {
    LocalKind kind;
    Ref dst;
    Ref acc;
    std::vector<Ref> ins;
    uint64_t count;
    int site;  // reference call site this op restates (line in all_reduce_radix_batch.cpp)
    uint64_t rows = 1, dpitch = 0, spitch = 0;
    bool swap = false;  // L_REDUCE: running value is the FIRST operand, OP(acc, in) (MPICH_do_reduce)
    std::vector<uint8_t> comb, swaps;  // L_TREE program
};

// In-place allgather collective (ncclAllGather) over a region of `nranks * count` elements
// at `ref`: rank r contributes [ref + r*count, +count) and receives every other block.
struct Coll {
    Ref ref;
    uint64_t count;  // elements per rank
};

struct Step {
    std::vector<Xfer> sends, recvs;
    std::vector<Coll> allgathers;  // issued after the step's p2p group
    std::vector<LocalOp> post;
    std::string label;
    // Two-stream execution: this step's transfers must wait for the local ops of step
    // `comm_wait` (the latest earlier step whose ops touch what these transfers read or
    // write); -1 = none.  Local ops always wait for their own step's transfers.
    int comm_wait = -1;
    // Every earlier step whose local ops conflict (RAW / WAR / WAW) with this step's transfers,
    // ascending; comm_wait is the last of them.  Local ops run in order on one compute stream, so
    // they need no dependency list of their own.
    std::vector<int> comm_deps;
};

enum Mode : int {
    MODE_ALLREDUCE = 0,        // all_reduce_radix_batch
    MODE_REDUCE_SCATTER = 1,   // reduce_scatter_radix_batch
    MODE_MPICH_RING = 2,       // testing/mpich_implementations/all_reduce/allreduce_ring.cpp
    MODE_MPICH_RD = 3,         // .../allreduce_recursive_doubling.cpp
    MODE_MPICH_RSAG = 4,       // .../allreduce_reduce_scatter_allgather.cpp
    MODE_MPICH_RECEXCH = 5,    // .../allreduce_recexch.cpp (k, single_phase_recv)
    MODE_MPICH_KRSAG = 6,      // .../allreduce_k_reduce_scatter_allgather.cpp (k, single_phase_recv)
    MODE_MPICH_RMULT = 7,      // .../allreduce_recursive_multiplying.cpp (k)
    MODE_ALLGATHER = 8,        // allgather_radix_batch (count = sendcount)
    // MPICH baseline reduce-scatters (block) of testing/mpich_implementations/reduce_scatter/
    // (count = recvcount; driven by that directory's main.cpp)
    MODE_MPICH_RS_RADIX = 9,     // reduce_scatter_radix.cpp:204 (k)
    MODE_MPICH_RS_HALVING = 10,  // reduce_scatter_recursive_halving.cpp:7
    MODE_MPICH_RS_DOUBLING = 11, // reduce_scatter_recursive_doubling.cpp:10
    MODE_MPICH_RS_PAIRWISE = 12, // reduce_scatter_pairwise.cpp:4
    // CHiArA's phases as stand-alone functions (testing/custom_implementations/work_dir/reduce_scatter/;
    // count = recvcount)
    MODE_INTRA_RS = 13,          // intra_reduce_scatter_radix.cpp:208 (k, b)
    MODE_INTER_LINEAR = 14,      // inter_linear_reduce.cpp:11 (b)
    MODE_INTRA_SCATTER = 15      // intra_scatter_radix_batch.cpp:10 (k, b)
};
inline bool is_mpich_rs(int mode) { return mode >= MODE_MPICH_RS_RADIX && mode <= MODE_MPICH_RS_PAIRWISE; }
inline bool is_mpich(int mode) { return (mode >= MODE_MPICH_RING && mode <= MODE_MPICH_RMULT) || is_mpich_rs(mode); }
inline bool is_phase(int mode) { return mode >= MODE_INTRA_RS && mode <= MODE_INTRA_SCATTER; }
// Modes compiled as one unsliced plan (no pipeline depth, no schedule choice).
inline bool is_unpipelined(int mode) { return is_mpich(mode) || mode == MODE_ALLGATHER || is_phase(mode); }

struct Geometry {
    int nranks = 0, b = 0, k = 0, nnodes = 0, nstages = 0, nu = 0, nph = 0;
    uint64_t recvcount = 0, irc = 0, total = 0;
    std::vector<int> S, P;  // chunks per lane block, prefix (P.size() == b+1)
};

struct Plan {
    int error = 0;  // chr_result
    int slices = 1;  // pipeline depth actually used
    bool balanced = false;  // allreduce evaluated piecewise on every rank (see build_plan)
    int sched = 0;          // Sched actually used
    Mode mode = MODE_ALLREDUCE;
    int rank = 0;
    Geometry g;
    uint64_t send_elems = 0, recv_elems = 0, acc_elems = 0, stage_elems = 0;
    std::vector<LocalOp> pre;
    std::vector<Step> steps;
};

// Recexch tables of one group of `nranks` (= b) ranks: all_reduce_radix_batch.cpp:11-198.
struct Recexch {
    int k = 0, p_of_k = 0, rem = 0, T = 0;
    int step1_sendto = -1, step1_nrecvs = 0;
    std::vector<int> step1_recvfrom;
    int step2_nphases = 0;
    std::vector<std::vector<int>> step2_nbrs;
};
int recexch_neighbors(int rank, int nranks, int k, Recexch* out);
void recexch_count_offset(int nranks, int max_phases, int k, std::vector<int>* count,
                          std::vector<int>* offset);

// count = allreduce element count, or reduce-scatter recvcount.  `slices` = pipeline
// depth: every chunk is cut into that many element slices; slice s runs logical step
// t-s in super-step t, so consecutive phases of different slices share an RCCL group.
// The per-element reduction order is unchanged (results are bit-identical for any depth).
// Where the reference's reductions are evaluated (the result bits never depend on it):
//   SCHED_REFERENCE  at the reference's owner lanes / root nodes (its communication pattern)
//   SCHED_BALANCED   single-phase geometries: every rank evaluates 1/n (schedule.cpp S_B*, S_R*)
//   SCHED_FLAT       any geometry: expression trees extracted symbolically, leaves gathered
//                    over the full mesh, evaluated at the piece's rank (build_plan_flat)
//   SCHED_EXACT      the reference's messages end to end, unsliced: REFERENCE's phases 0-2, then
//                    its bcast + k-port Bruck allgather (S_BCAST, S_AG) / k-nomial scatter (S_KSCAT)
//   SCHED_FLAT_AG    SCHED_FLAT with the allgather phase on RCCL's ncclAllGather collective
//                    (pure data movement, so the bits are unchanged) where the pieces are equal
//   SCHED_FLAT_SEQ   SCHED_FLAT with gather and allgather in separate RCCL groups (2P groups per
//                    call instead of P + 2; the ordering before the merged groups)
//   SCHED_FLAT_1SHOT allreduce: every rank gathers the whole buffer from every peer and evaluates
//                    every chunk's tree itself -- one exchange step instead of gather + allgather,
//                    (n-1) S bytes per rank instead of 2 (n-1)/n S: the latency-bound small-message
//                    variant.  Reduce-scatter: SCHED_FLAT (already one step).
//   (6 is CHR_SCHEDULE_AUTO, the executor's measured choice, not a plan.)
enum Sched : int {
    SCHED_REFERENCE = 0, SCHED_BALANCED = 1, SCHED_FLAT = 2, SCHED_EXACT = 3, SCHED_FLAT_AG = 4, SCHED_FLAT_SEQ = 5,
    SCHED_FLAT_1SHOT = 7
};
// A schedule a plan can be built for (every Sched value; not CHR_SCHEDULE_AUTO).
inline bool plan_schedule(int s) { return (s >= SCHED_REFERENCE && s <= SCHED_FLAT_SEQ) || s == SCHED_FLAT_1SHOT; }
// `commutative`: MPI_Op_commutative of the call's op (every predefined op is; a user op as created).  Only the MPICH
// baselines that branch on it read it (build_plan_mpich); CHiArA's own schedules take the reference's operand
// order for any op.
Plan build_plan(Mode mode, int nranks, int rank, int k, int b, uint64_t count, int slices = 1,
                int sched = SCHED_FLAT, bool commutative = true);
int auto_slices(uint64_t irc_bytes);
// MPICH baseline allreduces (count = elements per rank; aux = recexch single_phase_recv) and
// reduce-scatters (count = recvcount).  A non-commutative op takes the reference's rank-ordered branches
// (recursive doubling, reduce-scatter recursive doubling) or its MPI_ERR_OP (error = CHR_ERR_UNSUPPORTED:
// k-reduce-scatter-allgather, recursive multiplying at a size that is not a power of k).
Plan build_plan_mpich(Mode mode, int nranks, int rank, int k, int aux, uint64_t count, bool commutative = true);
Plan build_plan_allgather(int nranks, int rank, int k, int b, uint64_t sendcount);
// The stand-alone phases (MODE_INTRA_RS / MODE_INTER_LINEAR / MODE_INTRA_SCATTER; count = recvcount).
Plan build_plan_phase(Mode mode, int nranks, int rank, int k, int b, uint64_t recvcount);
std::string describe(const Plan& p);
// Phase of a step label for the per-phase timers: slice suffixes and super-step tags dropped,
// distinct phase names joined by '+' ("t3,phase0/s0,lane/s1" -> "phase0+lane").
std::string phase_name(const std::string& label);

}  // namespace chr
