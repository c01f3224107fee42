// executor.cpp -- runs compiled radix/batch plans on MI355X.
//
// Two transports behind one executor:
//  * chr_comm: one rank per process/GPU, messages = RCCL ncclSend/ncclRecv over xGMI.
//    All k-1 neighbour exchanges of a recexch phase (and all nnodes-1 lane messages of
//    the inter-node phase) go into ONE ncclGroupStart/End, so the phase drives several
//    xGMI links at once (the reference serialises them: all_reduce_radix_batch.cpp:343-367),
//    then ONE fused reduction kernel consumes all incoming buckets.
//  * chr_local_group: n virtual ranks on one device, messages = device-to-device copies.
//    Same plans, same kernels; used to check multi-rank schedules on a single MI355X.
// Everything is enqueued on one HIP stream per communicator; scratch (ACC, STAGE) is
// allocated once and reused (the reference mallocs 2x the buffer per call, :296-297).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "chr_internal.hpp"
#include "schedule.hpp"
#include "user_ops.hpp"

namespace {

using chr::Plan;

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    // Grows (never shrinks).  The caller has synchronised the stream before a regrow.
    hipError_t reserve(size_t want, hipStream_t s) {
        if (want <= bytes) return hipSuccess;
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        e = hipMalloc(&p, want);
        if (e == hipSuccess) bytes = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
};

struct Bufs {
    const char* send;
    char* recv;
    char* acc;
    char* stage;
    size_t es;
    char* ptr(const chr::Ref& r) const {
        char* base = r.buf == chr::BUF_SEND   ? const_cast<char*>(send)
                     : r.buf == chr::BUF_RECV ? recv
                     : r.buf == chr::BUF_ACC  ? acc
                                              : stage;
        return base + r.off * es;
    }
};

int hip_code(hipError_t e) {
    if (e == hipSuccess) return CHR_SUCCESS;
    if (e == hipErrorOutOfMemory) return CHR_ERR_OUT_OF_MEMORY;
    if (std::getenv("CHR_DEBUG")) std::fprintf(stderr, "[chiara] HIP error: %s\n", hipGetErrorString(e));
    return CHR_ERR_HIP;
}

int nccl_code(ncclResult_t r) {
    if (r == ncclSuccess) return CHR_SUCCESS;
    if (std::getenv("CHR_DEBUG")) std::fprintf(stderr, "[chiara] RCCL error: %s\n", ncclGetErrorString(r));
    return CHR_ERR_RCCL;
}

// Opt-in timing of the fused reduction launches (chr_comm_profile): HIP events on the
// launch stream around each reduction, summed when read.
struct ReduceProfile {
    bool on = false;
    // span: the caller brackets whole phases with events (record_span) and the launches only add
    // their algorithmic bytes and count -- the local group's mode, whose launches may run on two
    // streams at once
    bool span = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending, spare;
    double ms = 0, bytes = 0;
    long launches = 0;
    // per-phase transfer time (the reference's DEBUG_MODE phase timers, all_reduce_radix_batch.cpp
    // :228-232, :480-489, :542-548, :572-578, :758-764): events around each step's RCCL group on
    // the transfer stream, summed per phase name (the step label without slice suffixes)
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> steps_pending;
    std::map<std::string, double> phase_ms;
    std::pair<hipEvent_t, hipEvent_t> take() {
        if (!spare.empty()) {
            auto e = spare.back();
            spare.pop_back();
            return e;
        }
        std::pair<hipEvent_t, hipEvent_t> e{nullptr, nullptr};
        (void)hipEventCreate(&e.first);
        (void)hipEventCreate(&e.second);
        return e;
    }
    void drain() {
        for (auto& e : pending) {
            float t = 0;
            if (hipEventSynchronize(e.second) == hipSuccess && hipEventElapsedTime(&t, e.first, e.second) == hipSuccess)
                ms += t;
            spare.push_back(e);
        }
        pending.clear();
        for (auto& s : steps_pending) {
            float t = 0;
            if (hipEventSynchronize(s.second.second) == hipSuccess &&
                hipEventElapsedTime(&t, s.second.first, s.second.second) == hipSuccess)
                phase_ms[s.first] += t;
            spare.push_back(s.second);
        }
        steps_pending.clear();
    }
    void release() {
        drain();
        for (auto& e : spare) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
        spare.clear();
    }
};

int run_local(const chr::LocalOp& op, const Bufs& B, int dtype, int rop, hipStream_t s,
              ReduceProfile* prof = nullptr) {
    if (op.count == 0) return CHR_SUCCESS;
    if (op.kind == chr::L_COPY) {
        char* d = B.ptr(op.dst);
        const char* src = B.ptr(op.acc);
        if (d == src) return CHR_SUCCESS;
        return hip_code(hipMemcpyAsync(d, src, op.count * B.es, hipMemcpyDeviceToDevice, s));
    }
    if (op.kind == chr::L_COPY2D)
        return hip_code(hipMemcpy2DAsync(B.ptr(op.dst), op.dpitch * B.es, B.ptr(op.acc), op.spitch * B.es,
                                         op.count * B.es, op.rows, hipMemcpyDeviceToDevice, s));
    const bool tree = op.kind == chr::L_TREE;
    std::vector<const void*> ins;
    if (tree) ins.push_back(B.ptr(op.acc));  // leaf 0
    for (const chr::Ref& r : op.ins) ins.push_back(B.ptr(r));
    const bool counted = prof && prof->on && !ins.empty();
    const bool timed = counted && !prof->span;
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (timed) {
        ev = prof->take();
        (void)hipEventRecord(ev.first, s);
    }
    const int rc =
        tree ? chr::reduce_tree_any(B.ptr(op.dst), ins.data(), (int)ins.size(), op.comb.data(),
                                    op.swaps.empty() ? nullptr : op.swaps.data(), op.count, dtype, rop, s)
             : chr::reduce_any(B.ptr(op.dst), B.ptr(op.acc), ins.data(), (int)ins.size(), op.count, dtype, rop, s,
                               op.swap);
    if (timed) {
        (void)hipEventRecord(ev.second, s);
        prof->pending.push_back(ev);
    }
    if (counted) {
        // algorithmic bytes: every operand read once, the result written once
        prof->bytes += (double)(ins.size() + (tree ? 1 : 2)) * op.count * B.es;
        prof->launches += 1;
    }
    return rc;
}

// Consecutive L_TREE ops of one step (the flat schedule's chunks of one pipeline slice) run as ONE
// batched launch when none writes what another reads or writes (an op's own in-place root over
// its own leaf is element-wise and fine): fewer grid fills and drains per call
// (launch_reduce_tree_multi).  Anything else runs op by op.  Overlap is decided on the resolved
// byte ranges, not on (buffer, offset): under CHR_IN_PLACE the SEND and RECV buffers are one.
bool overlaps(const Bufs& B, const chr::Ref& x, uint64_t xn, const chr::Ref& y, uint64_t yn) {
    const char* px = B.ptr(x);
    const char* py = B.ptr(y);
    return px < py + yn * B.es && py < px + xn * B.es;
}

bool batchable(const std::vector<chr::LocalOp>& ops, size_t i0, size_t i1, const Bufs& B) {
    for (size_t i = i0; i < i1; ++i)
        for (size_t j = i0; j < i1; ++j) {
            if (i == j) continue;
            const chr::LocalOp& w = ops[i];
            const chr::LocalOp& r = ops[j];
            if (overlaps(B, w.dst, w.count, r.dst, r.count) || overlaps(B, w.dst, w.count, r.acc, r.count)) return false;
            for (const chr::Ref& x : r.ins)
                if (overlaps(B, w.dst, w.count, x, r.count)) return false;
        }
    return true;
}

// Trees per batched launch (reduce_tree.hpp kMaxTreeSegs).
constexpr size_t kTreeSegsPerLaunch = 8;

// The tree ops [i0, i1) as resolved jobs for launch_reduce_tree_multi; returns their algorithmic bytes.
double tree_jobs(const std::vector<chr::LocalOp>& ops, size_t i0, size_t i1, const Bufs& B,
                 std::vector<chr::TreeJob>* jobs) {
    double bytes = 0;
    for (size_t i = i0; i < i1; ++i) {
        const chr::LocalOp& op = ops[i];
        if (op.count == 0) continue;
        chr::TreeJob jb{};
        jb.out = B.ptr(op.dst);
        jb.leaves[0] = B.ptr(op.acc);
        for (size_t j = 0; j < op.ins.size(); ++j) jb.leaves[j + 1] = B.ptr(op.ins[j]);
        jb.nl = (int)op.ins.size() + 1;
        jb.comb = op.comb.data();
        jb.swaps = op.swaps.empty() ? nullptr : op.swaps.data();
        jb.n = op.count;
        jobs->push_back(jb);
        bytes += (double)(jb.nl + 1) * op.count * B.es;
    }
    return bytes;
}

int launch_tree_jobs(const std::vector<chr::TreeJob>& jobs, double bytes, int dtype, int rop, hipStream_t s,
                     ReduceProfile* prof) {
    if (jobs.empty()) return CHR_SUCCESS;
    const bool counted = prof && prof->on;
    const bool timed = counted && !prof->span;
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (timed) {
        ev = prof->take();
        (void)hipEventRecord(ev.first, s);
    }
    const int rc = chr::reduce_tree_multi_any(jobs.data(), (int)jobs.size(), dtype, rop, s);
    if (timed) {
        (void)hipEventRecord(ev.second, s);
        prof->pending.push_back(ev);
    }
    if (counted) {
        prof->bytes += bytes;
        // vector launches: launch_reduce_tree_multi packs up to kTreeSegsPerLaunch trees of one leaf count per grid
        prof->launches += (long)((jobs.size() + kTreeSegsPerLaunch - 1) / kTreeSegsPerLaunch);
    }
    return rc;
}

int run_tree_batch(const std::vector<chr::LocalOp>& ops, size_t i0, size_t i1, const Bufs& B, int dtype, int rop,
                   hipStream_t s, ReduceProfile* prof) {
    std::vector<chr::TreeJob> jobs;
    const double bytes = tree_jobs(ops, i0, i1, B, &jobs);
    return launch_tree_jobs(jobs, bytes, dtype, rop, s, prof);
}

// Whether every op of `ops` is a tree of <= 8 leaves and the list is one batchable run (run_locals
// would issue it as a single launch_reduce_tree_multi call).
bool one_tree_run(const std::vector<chr::LocalOp>& ops, const Bufs& B) {
    for (const chr::LocalOp& op : ops)
        if (op.kind != chr::L_TREE || op.ins.size() + 1 > 8) return false;
    return ops.size() < 2 || batchable(ops, 0, ops.size(), B);
}

// Whether job x writes memory job y reads or writes (resolved byte ranges).
bool job_conflict(const chr::TreeJob& x, const chr::TreeJob& y, size_t es) {
    auto hit = [&](const void* a, const void* b) {
        const char* pa = (const char*)a;
        const char* pb = (const char*)b;
        return pa < pb + y.n * es && pb < pa + x.n * es;
    };
    if (hit(x.out, y.out)) return true;
    for (int j = 0; j < y.nl; ++j)
        if (hit(x.out, y.leaves[j])) return true;
    return false;
}

int run_locals(const std::vector<chr::LocalOp>& ops, const Bufs& B, int dtype, int rop, hipStream_t s,
               ReduceProfile* prof = nullptr) {
    for (size_t i = 0; i < ops.size();) {
        size_t j = i;
        while (j < ops.size() && ops[j].kind == chr::L_TREE && ops[j].ins.size() + 1 <= 8) ++j;
        if (j - i >= 2 && batchable(ops, i, j, B)) {
            if (int rc = run_tree_batch(ops, i, j, B, dtype, rop, s, prof)) return rc;
            i = j;
            continue;
        }
        if (int rc = run_local(ops[i], B, dtype, rop, s, prof)) return rc;
        ++i;
    }
    return CHR_SUCCESS;
}

bool is_device_ptr(const void* p) {
    hipPointerAttribute_t attr;
    std::memset(&attr, 0, sizeof(attr));
    hipError_t e = hipPointerGetAttributes(&attr, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

// mode, rank, k, b, count, dtype size, slices, schedule, op commutative (the MPICH baselines branch on it)
using PlanKey = std::tuple<int, int, int, int, uint64_t, int, int, int, bool>;

// CHR_SCHEDULE = reference | balanced | flat | exact | flat_ag | flat_seq | auto (or 0 .. 6); default flat
// CHR_OVERLAP=0: local ops on the transfer stream (no compute/xGMI overlap); default 1
int default_overlap() {
    static const int v = [] {
        const char* e = std::getenv("CHR_OVERLAP");
        return e ? (std::atoi(e) != 0) : 1;
    }();
    return v;
}

// CHR_LG_BATCH=0: a local group launches each virtual rank's trees separately; default 1
int default_lg_batch() {
    static const int v = [] {
        const char* e = std::getenv("CHR_LG_BATCH");
        return e ? (std::atoi(e) != 0) : 1;
    }();
    return v;
}

// CHR_GRAPHS=1: device-resident collectives replay a captured HIP graph per (plan, buffers)
int default_graphs() {
    static const int v = [] {
        const char* e = std::getenv("CHR_GRAPHS");
        return e ? (std::atoi(e) != 0) : 0;
    }();
    return v;
}

// CHR_TIMEOUT_MS: blocking calls give up after this many milliseconds (0 = wait forever, the
// default); see chr_comm_set_timeout
int default_host_window_mib() {
    static const int v = [] {
        const char* e = std::getenv("CHR_HOST_WINDOW_MIB");
        return e ? std::max(0, std::atoi(e)) : 0;
    }();
    return v;
}

int default_timeout_ms() {
    static const int v = [] {
        const char* e = std::getenv("CHR_TIMEOUT_MS");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}

int default_schedule() {
    static const int v = [] {
        const char* e = std::getenv("CHR_SCHEDULE");
        if (!e) return (int)chr::SCHED_FLAT;
        const std::string s(e);
        if (s == "reference" || s == "0") return (int)chr::SCHED_REFERENCE;
        if (s == "balanced" || s == "1") return (int)chr::SCHED_BALANCED;
        if (s == "exact" || s == "3") return (int)chr::SCHED_EXACT;
        if (s == "flat_ag" || s == "4") return (int)chr::SCHED_FLAT_AG;
        if (s == "flat_seq" || s == "5") return (int)chr::SCHED_FLAT_SEQ;
        if (s == "flat_1shot" || s == "7") return (int)chr::SCHED_FLAT_1SHOT;
        if (s == "auto" || s == "6") return CHR_SCHEDULE_AUTO;
        return (int)chr::SCHED_FLAT;
    }();
    return v;
}

// Pipeline depth: explicit setting, else CHR_SLICES, else by chunk size (schedule.cpp auto_slices).
// The flat schedules evaluate one piece per (chunk, rank) per slice -- chunk/n elements (allreduce)
// or the rank's own block (reduce-scatter), divided by the depth -- in batched tree launches whose
// fixed fill/drain cost dominates small pieces (profiles/r02/tree_bench_batched.json, C4's two
// 8-leaf trees per slice: 8 MiB pieces 0.58-0.63 of the HBM peak, 16 MiB 0.68-0.77), so their
// default depth keeps pieces at 16 MiB or more.  CHR_SCHEDULE_AUTO still times every depth from
// the chunk-size one down.
constexpr uint64_t kMinFlatPieceBytes = (uint64_t)16 << 20;

bool flat_family(int sched) {
    return sched == chr::SCHED_FLAT || sched == chr::SCHED_FLAT_AG || sched == chr::SCHED_FLAT_SEQ ||
           sched == chr::SCHED_FLAT_1SHOT;
}

// SCHED_FLAT_1SHOT moves (n-1) S per rank instead of 2 (n-1)/n S: a latency trade for small calls.  AUTO
// times it only up to this many bytes per rank (8 GPUs at ~350 GB/s of xGMI per direction: the
// extra 1.75 S costs one RCCL group's ~15 us of latency near S = 3 MB).
constexpr uint64_t kOneShotMaxBytes = (uint64_t)8 << 20;

int pick_slices(int setting, uint64_t count, int mode, int nranks, int b, size_t es, int sched) {
    if (chr::is_unpipelined(mode)) return 1;  // unpipelined schedules
    if (setting > 0) return setting;
    static const int env = [] {
        const char* v = std::getenv("CHR_SLICES");
        return v ? std::atoi(v) : 0;
    }();
    if (env > 0) return env;
    const uint64_t n = (uint64_t)(nranks > 0 ? nranks : 1);
    const uint64_t recvcount = mode == chr::MODE_ALLREDUCE ? count / n : count;
    const uint64_t irc_bytes = recvcount * (uint64_t)(b > 0 ? b : 1) * es;
    int P = chr::auto_slices(irc_bytes);
    if (flat_family(sched)) {
        const uint64_t piece = mode == chr::MODE_ALLREDUCE && sched != chr::SCHED_FLAT_1SHOT ? irc_bytes / n
                               : mode == chr::MODE_ALLREDUCE                                ? irc_bytes
                                                                                            : recvcount * es;
        const int cap = (int)std::max<uint64_t>(1, piece / kMinFlatPieceBytes);
        P = std::min(P, cap);
    }
    return P;
}

}  // namespace

struct chr_comm {
    int rank = 0, nranks = 0, device = 0;
    int slices = 0;  // 0 = auto
    int sched = default_schedule();
    int overlap = default_overlap();
    ncclComm_t nccl = nullptr;
    hipStream_t stream = nullptr;   // RCCL transfers; the call completes on this stream
    hipStream_t cstream = nullptr;  // local ops (reductions, copies) when overlapping
    std::vector<hipEvent_t> events;  // pool: 2 per step
    hipEvent_t event(size_t i) {
        while (events.size() <= i) {
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
            events.push_back(e);
        }
        return events[i];
    }
    DevBuf acc, stage, hsend, hrecv, flag;  // flag: agree_min's 4-byte exchange
    ReduceProfile prof;
    std::map<PlanKey, std::unique_ptr<Plan>> plans;

    // Pipelined host staging (chr_comm_set_host_pipeline): copy-in and copy-out streams, two
    // device window buffers per direction, and the events that order them against the collective.
    int host_window_mib = default_host_window_mib();
    hipStream_t hin = nullptr, hout = nullptr;
    DevBuf wsend[2], wrecv[2];
    hipEvent_t ev_in[2] = {}, ev_coll[2] = {}, ev_out[2] = {};
    hipError_t host_pipeline_init() {
        if (hin) return hipSuccess;
        hipError_t e = hipStreamCreateWithFlags(&hin, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&hout, hipStreamNonBlocking);
        for (int i = 0; i < 2 && e == hipSuccess; ++i) {
            e = hipEventCreateWithFlags(&ev_in[i], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&ev_coll[i], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&ev_out[i], hipEventDisableTiming);
        }
        return e;
    }
    void host_pipeline_release() {
        if (hin) (void)hipStreamSynchronize(hin);
        if (hout) (void)hipStreamSynchronize(hout);
        for (int i = 0; i < 2; ++i) {
            wsend[i].release();
            wrecv[i].release();
            for (hipEvent_t* e : {&ev_in[i], &ev_coll[i], &ev_out[i]})
                if (*e) (void)hipEventDestroy(*e);
        }
        if (hin) (void)hipStreamDestroy(hin);
        if (hout) (void)hipStreamDestroy(hout);
        hin = hout = nullptr;
    }

    // Failure handling.  A call that fails after it has posted RCCL operations, or that times
    // out, aborts the RCCL communicator (ncclCommAbort: its kernels exit, peers see the closed
    // connections) instead of leaving peers posted; every later call then returns
    // CHR_ERR_ABORTED and chr_comm_destroy skips ncclCommDestroy, which could block on a wedged
    // communicator.  The reference has no such path: under MPI_ERRORS_ARE_FATAL an error aborts
    // the job, and a lost peer is a hang.
    int timeout_ms = default_timeout_ms();
    bool failed = false;
    void abort_comm() {
        if (nccl) (void)ncclCommAbort(nccl);
        nccl = nullptr;
        failed = true;
    }

    // HIP graph replay (chr_comm_set_graphs): one executable graph per (plan, send, recv, dtype, op, overlap),
    // dropped whenever the scratch buffers they point into are reallocated
    int graphs = default_graphs();
    std::map<std::tuple<const Plan*, const void*, void*, int, int, int>, hipGraphExec_t> gexec;
    void drop_graphs() {
        for (auto& kv : gexec) (void)hipGraphExecDestroy(kv.second);
        gexec.clear();
    }
    // The only way scratch grows: whichever path reserves it (eager, graph capture, host-staged,
    // profiled, tuning), a reallocation drops every cached graph, since they point into the old
    // buffers.  reserve() synchronises the stream first, so no replay is still running.
    hipError_t reserve_scratch(size_t acc_bytes, size_t stage_bytes) {
        const void* a0 = acc.p;
        const void* s0 = stage.p;
        hipError_t e = acc.reserve(acc_bytes, stream);
        if (e == hipSuccess) e = stage.reserve(stage_bytes, stream);
        if (acc.p != a0 || stage.p != s0) drop_graphs();
        return e;
    }
    // CHR_SCHEDULE_AUTO: (mode, count, element size, k, b, slices setting, overlap) -> (schedule, depth)
    std::map<std::tuple<int, uint64_t, int, int, int, int, int>, std::pair<int, int>> tuned;

    const Plan& plan(int mode, int k, int b, uint64_t count, size_t es, int sched_, int slices_, bool commutative) {
        const int P = pick_slices(slices_, count, mode, nranks, b, es, sched_);
        PlanKey key{mode, rank, k, b, count, (int)es, P, sched_, commutative};
        auto it = plans.find(key);
        if (it == plans.end())
            it = plans.emplace(key, std::make_unique<Plan>(chr::build_plan((chr::Mode)mode, nranks, rank, k, b, count, P,
                                                                           sched_, commutative)))
                     .first;
        return *it->second;
    }
};

struct chr_local_group {
    int nranks = 0, device = 0;
    // chr_local_group_profile: the fused reductions of every rank, timed as whole phases (from the
    // end of a step's copies to the join of its reductions) with HIP events on the group's stream
    ReduceProfile prof;
    int slices = 0;  // 0 = auto
    // chr_local_group_set_batching: the virtual ranks' tree evaluations of one step share launches
    // (CHR_LG_BATCH=0 turns it off; default on)
    int batch_ranks = default_lg_batch();
    int sched = default_schedule() == CHR_SCHEDULE_AUTO ? (int)chr::SCHED_FLAT : default_schedule();  // no tuning
    hipStream_t stream = nullptr;
    std::vector<DevBuf> acc, stage;
    std::map<std::tuple<int, int, int, uint64_t, int, int, int, bool>, std::vector<Plan>> plans;
};

namespace {

int enqueue_plan(chr_comm* c, const Plan& p, const void* send, void* recv, int dtype, int op, bool* posted);

// Enqueues a whole plan.  A failure after the first RCCL operation was posted aborts the
// communicator: peers may already be waiting on this rank's messages.
int enqueue_rccl(chr_comm* c, const Plan& p, const void* send, void* recv, int dtype, int op) {
    if (c->failed) return CHR_ERR_ABORTED;
    bool posted = false;
    const int rc = enqueue_plan(c, p, send, recv, dtype, op, &posted);
    if (rc && posted) c->abort_comm();
    return rc;
}

int enqueue_plan(chr_comm* c, const Plan& p, const void* send, void* recv, int dtype, int op, bool* posted) {
    const size_t es = chr::dtype_size(dtype);
    hipError_t e = c->reserve_scratch(p.acc_elems * es, p.stage_elems * es);
    if (e != hipSuccess) return hip_code(e);
    Bufs B{(const char*)send, (char*)recv, (char*)c->acc.p, (char*)c->stage.p, es};
    int rc;
    if ((rc = run_locals(p.pre, B, dtype, op, c->stream, &c->prof))) return rc;
    // Transfers on c->stream, local ops on c->cstream.  A step's transfers wait for the local ops of
    // its comm_deps (schedule.cpp analyze_deps), a step's local ops for its own transfers.  The
    // compute stream runs in order, so one wait on the latest dependency (comm_wait) covers every
    // earlier one, and local ops never need to wait for each other.  The call ends with c->stream
    // waiting for the last local ops.
    const bool two = c->overlap && c->cstream;
    int xfer_waited = -1, last_local = -1;
    for (size_t t = 0; t < p.steps.size(); ++t) {
        const chr::Step& s = p.steps[t];
        if (two && s.comm_wait > xfer_waited) {
            hipEvent_t ew = c->event(2 * (size_t)s.comm_wait + 1);
            if (!ew || (rc = hip_code(hipStreamWaitEvent(c->stream, ew, 0)))) return ew ? rc : CHR_ERR_HIP;
            xfer_waited = s.comm_wait;
        }
        const bool xfers = !s.sends.empty() || !s.recvs.empty() || !s.allgathers.empty();
        const bool timed = c->prof.on && xfers;
        std::pair<hipEvent_t, hipEvent_t> sev{nullptr, nullptr};
        if (timed) {
            sev = c->prof.take();
            (void)hipEventRecord(sev.first, c->stream);
        }
        if (xfers) *posted = true;
        if (!s.sends.empty() || !s.recvs.empty()) {
            if ((rc = nccl_code(ncclGroupStart()))) return rc;
            for (const chr::Xfer& x : s.sends)
                if ((rc = nccl_code(ncclSend(B.ptr(x.ref), x.count * es, ncclUint8, x.peer, c->nccl, c->stream)))) {
                    (void)ncclGroupEnd();
                    return rc;
                }
            for (const chr::Xfer& x : s.recvs)
                if ((rc = nccl_code(ncclRecv(B.ptr(x.ref), x.count * es, ncclUint8, x.peer, c->nccl, c->stream)))) {
                    (void)ncclGroupEnd();
                    return rc;
                }
            if ((rc = nccl_code(ncclGroupEnd()))) return rc;
        }
        if (!s.allgathers.empty()) {  // in place: my block already sits at ref + rank*count
            if ((rc = nccl_code(ncclGroupStart()))) return rc;
            for (const chr::Coll& x : s.allgathers) {
                char* base = B.ptr(x.ref);
                if ((rc = nccl_code(ncclAllGather(base + (size_t)c->rank * x.count * es, base, x.count * es, ncclUint8,
                                                  c->nccl, c->stream)))) {
                    (void)ncclGroupEnd();
                    return rc;
                }
            }
            if ((rc = nccl_code(ncclGroupEnd()))) return rc;
        }
        if (timed) {
            (void)hipEventRecord(sev.second, c->stream);
            c->prof.steps_pending.push_back({chr::phase_name(s.label), sev});
        }
        if (s.post.empty()) continue;
        if (!two) {
            if ((rc = run_locals(s.post, B, dtype, op, c->stream, &c->prof))) return rc;
            continue;
        }
        hipEvent_t ec = c->event(2 * t), ed = c->event(2 * t + 1);
        if (!ec || !ed) return CHR_ERR_HIP;
        if ((rc = hip_code(hipEventRecord(ec, c->stream))) || (rc = hip_code(hipStreamWaitEvent(c->cstream, ec, 0))))
            return rc;
        {
            // RCCL's kernels run beside these launches: streaming reductions leave them room on every
            // CU (reduce_common.hpp kCoresidentWgPerCu)
            chr::CoresidentScope beside_rccl(c->nranks > 1);
            if ((rc = run_locals(s.post, B, dtype, op, c->cstream, &c->prof))) return rc;
        }
        if ((rc = hip_code(hipEventRecord(ed, c->cstream)))) return rc;
        last_local = (int)t;
    }
    if (two && last_local > xfer_waited &&
        (rc = hip_code(hipStreamWaitEvent(c->stream, c->event(2 * (size_t)last_local + 1), 0))))
        return rc;
    return CHR_SUCCESS;
}

// Graph replay of a device-resident call.  A plan's whole enqueue -- RCCL groups on the transfer
// stream, reductions and copies forked onto the compute stream and joined back by events -- is
// captured once per (plan, buffers) and replayed with one hipGraphLaunch: the host cost of a call
// drops from the RCCL group calls, launches and event records of every step to one launch, which
// is what bounds small messages.  Scratch is sized before capture (no allocation inside it); if
// that grows a buffer, every cached graph is dropped (they point into the old one).
int launch_graph(chr_comm* c, const Plan& p, const void* send, void* recv, int dtype, int op) {
    const size_t es = chr::dtype_size(dtype);
    hipError_t e = c->reserve_scratch(p.acc_elems * es, p.stage_elems * es);
    if (e != hipSuccess) return hip_code(e);
    auto key = std::make_tuple(&p, send, recv, dtype, op, c->overlap);
    auto it = c->gexec.find(key);
    if (it == c->gexec.end()) {
        if (!c->event(2 * p.steps.size() + 1)) return CHR_ERR_HIP;  // the event pool, created outside the capture
        if ((e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal)) != hipSuccess) return hip_code(e);
        const int rc = enqueue_rccl(c, p, send, recv, dtype, op);
        hipGraph_t g = nullptr;
        e = hipStreamEndCapture(c->stream, &g);
        if (rc || e != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            return rc ? rc : hip_code(e);
        }
        hipGraphExec_t x = nullptr;
        e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (e != hipSuccess) return hip_code(e);
        it = c->gexec.emplace(key, x).first;
    }
    const int rc = hip_code(hipGraphLaunch(it->second, c->stream));
    if (rc) c->abort_comm();  // the replay may have been partly submitted
    return rc;
}

// Blocking completion of a call on the communicator stream.  With a timeout set, the stream is
// polled, and RCCL's asynchronous error state with it (a peer that died or closed its
// connections); on timeout or error the communicator is aborted, so a lost peer becomes an
// error code on every surviving rank instead of a hang.
int wait_call(chr_comm* c) {
    if (c->timeout_ms <= 0) return hip_code(hipStreamSynchronize(c->stream));
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto limit = t0 + std::chrono::milliseconds(c->timeout_ms);
    auto next_check = t0;
    for (int spin = 0;; ++spin) {
        const hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess) return CHR_SUCCESS;
        if (q != hipErrorNotReady) {
            c->abort_comm();
            return hip_code(q);
        }
        const auto now = clk::now();
        if (now >= next_check) {  // RCCL's own error state, every millisecond
            ncclResult_t ae = ncclSuccess;
            if (c->nccl && ncclCommGetAsyncError(c->nccl, &ae) == ncclSuccess && ae != ncclSuccess &&
                ae != ncclInProgress) {
                c->abort_comm();
                (void)hipStreamSynchronize(c->stream);
                return CHR_ERR_RCCL;
            }
            next_check = now + std::chrono::milliseconds(1);
        }
        if (now >= limit) {
            if (std::getenv("CHR_DEBUG"))
                std::fprintf(stderr, "[chiara] rank %d: call timed out after %d ms, aborting the communicator\n",
                             c->rank, c->timeout_ms);
            c->abort_comm();  // RCCL kernels poll the abort flag and exit
            (void)hipStreamSynchronize(c->stream);
            (void)hipStreamSynchronize(c->cstream);
            return CHR_ERR_TIMEOUT;
        }
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// wait_call for one event (the main thread: may abort the communicator).  Used before a copy to or
// from pageable host memory that depends on a collective: such a copy returns only once HIP has
// staged it, so issued first it would block inside HIP -- beyond the timeout -- if a peer is lost.
int wait_event(chr_comm* c, hipEvent_t ev) {
    if (c->timeout_ms <= 0) return CHR_SUCCESS;  // no timeout: let the copy itself wait, as before
    using clk = std::chrono::steady_clock;
    const auto limit = clk::now() + std::chrono::milliseconds(c->timeout_ms);
    for (int spin = 0;; ++spin) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return CHR_SUCCESS;
        if (q != hipErrorNotReady) return hip_code(q);
        ncclResult_t ae = ncclSuccess;
        if (spin % 64 == 0 && c->nccl && ncclCommGetAsyncError(c->nccl, &ae) == ncclSuccess && ae != ncclSuccess &&
            ae != ncclInProgress) {
            c->abort_comm();
            return CHR_ERR_RCCL;
        }
        if (clk::now() >= limit) {
            c->abort_comm();
            return CHR_ERR_TIMEOUT;
        }
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// The copy-out thread's wait for an event under the communicator's timeout.  It never touches the
// RCCL communicator (the issuing thread owns it and does any abort): it reports CHR_ERR_TIMEOUT.
int wait_event_poll(hipEvent_t ev, int timeout_ms) {
    if (timeout_ms <= 0) return CHR_SUCCESS;
    using clk = std::chrono::steady_clock;
    const auto limit = clk::now() + std::chrono::milliseconds(timeout_ms);
    for (int spin = 0;; ++spin) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return CHR_SUCCESS;
        if (q != hipErrorNotReady) return hip_code(q);
        if (clk::now() >= limit) return CHR_ERR_TIMEOUT;
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// Pipelined host staging (chr_comm_set_host_pipeline).  An allreduce/reduce-scatter output element
// depends only on the elements at the same offset of every recvcount block (every reduction is
// element-wise, every message block-granular; pinned by test_block_window_property), so a host
// call splits into collectives over windows [off, off + w) of every block, each with the plan for
// n*w (allreduce) or w (reduce-scatter) elements -- the bits of the whole call.  Window j's H2D
// (2-D copy, one row per block) runs on `hin`, its collective on the communicator's streams, its
// D2H on `hout`; two device buffers per direction let window j+1 come in and j-1 go out while j
// is reduced.
//
// The D2H side is issued from a second host thread.  A copy from or to pageable memory (the
// reference harness mallocs its buffers) returns only when HIP has staged it through its own
// pinned bounce buffers, so from one thread the two directions strictly alternate; from two
// threads they overlap (tools/host_stage_probe: 1 GiB each way, 38.2 ms one after the other,
// 22.5 ms from two threads, the same as pinned memory).  The threads hand windows over through
// two counters: the issuing thread publishes "window j's collective is enqueued" (the D2H may then
// wait on ev_coll), the copy-out thread "window j's D2H is enqueued" (a later collective may then
// wait on ev_out before overwriting that window's device buffer).  Returns -1 when the call is
// not split (one window would cover it).
// One int per rank, the minimum over the ranks, on the communicator stream (blocking, under the
// timeout).  A failure aborts the communicator: the peers are inside the same collective.
// No pageable copy is issued while the exchange may still be pending: such a copy returns only
// once HIP has staged it, i.e. it would wait for the collective inside HIP, past the timeout, if a
// peer never arrives.  The value goes in by a device memset and comes out after wait_call.
int agree_min(chr_comm* c, int mine, int* all) {
    int rc = hip_code(c->flag.reserve(sizeof(int), c->stream));
    int* d = (int*)c->flag.p;
    if (!rc) rc = hip_code(hipMemsetD32Async((hipDeviceptr_t)d, mine, 1, c->stream));
    if (!rc) rc = nccl_code(ncclAllReduce(d, d, 1, ncclInt32, ncclMin, c->nccl, c->stream));
    if (rc) {
        c->abort_comm();
        return rc;
    }
    if ((rc = wait_call(c))) return rc;  // under the timeout; aborts the communicator itself
    rc = hip_code(hipMemcpyAsync(all, d, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (!rc) rc = hip_code(hipStreamSynchronize(c->stream));
    return rc;
}

// Elements per block of one host window, or 0 when the call is not split (one window would cover
// it, or windows are off): a function of the communicator's setting and the arguments only.
size_t host_window_elems(const chr_comm* c, int mode, size_t count, size_t es) {
    if (c->host_window_mib <= 0 || (mode != chr::MODE_ALLREDUCE && mode != chr::MODE_REDUCE_SCATTER)) return 0;
    const size_t n = (size_t)c->nranks;
    const size_t block = mode == chr::MODE_ALLREDUCE ? count / n : count;  // recvcount
    if (mode == chr::MODE_ALLREDUCE && block * n != count) return 0;       // the plan reports the error
    size_t w = ((size_t)c->host_window_mib << 20) / (n * es);
    w -= w % 64;  // windows start 256 B-aligned within each block when the block is
    return w == 0 || w >= block ? 0 : w;
}

int run_host_windows(chr_comm* c, int sched, int slices, int mode, const void* input, void* recv, size_t count,
                     int dtype, int op, int k, int b) {
    const size_t es = chr::dtype_size(dtype), n = (size_t)c->nranks;
    const size_t w = host_window_elems(c, mode, count, es);
    if (w == 0) return -1;
    const size_t block = mode == chr::MODE_ALLREDUCE ? count / n : count;  // recvcount
    hipError_t e = c->host_pipeline_init();
    if (e != hipSuccess) return hip_code(e);
    int rc;
    if ((rc = wait_call(c))) return rc;  // earlier _async work, under the timeout
    const size_t out_rows = mode == chr::MODE_ALLREDUCE ? n : 1;
    for (int i = 0; i < 2; ++i) {
        if ((e = c->wsend[i].reserve(n * w * es, c->stream)) != hipSuccess) return hip_code(e);
        if ((e = c->wrecv[i].reserve(out_rows * w * es, c->stream)) != hipSuccess) return hip_code(e);
    }
    const char* hsrc = (const char*)input;
    char* hdst = (char*)recv;
    const size_t nwin = (block + w - 1) / w;
    const int timeout_ms = c->timeout_ms;

    std::mutex mu;
    std::condition_variable cv;
    size_t coll_enqueued = 0, out_enqueued = 0;  // windows handed over, under mu
    bool stop = false;                           // the issuing thread failed: copy-out ends
    int out_rc = CHR_SUCCESS;                    // the copy-out thread's first error
    auto copy_out_loop = [&] {
        if (hipSetDevice(c->device) != hipSuccess) {
            std::lock_guard<std::mutex> g(mu);
            out_rc = CHR_ERR_HIP;
            cv.notify_all();
            return;
        }
        for (size_t j = 0; j < nwin; ++j) {
            {
                std::unique_lock<std::mutex> g(mu);
                cv.wait(g, [&] { return stop || coll_enqueued > j; });
                if (stop) return;
            }
            const int i = (int)(j & 1);
            const size_t off = j * w, wj = std::min(w, block - off);
            // with a timeout, the collective first: a pageable copy would block inside HIP
            int wrc = wait_event_poll(c->ev_coll[i], timeout_ms);
            hipError_t ee = hipSuccess;
            if (!wrc) ee = hipStreamWaitEvent(c->hout, c->ev_coll[i], 0);
            if (!wrc && ee == hipSuccess)
                ee = hipMemcpy2DAsync(hdst + off * es, block * es, c->wrecv[i].p, wj * es, wj * es, out_rows,
                                      hipMemcpyDefault, c->hout);
            if (!wrc && ee == hipSuccess) ee = hipEventRecord(c->ev_out[i], c->hout);
            std::lock_guard<std::mutex> g(mu);
            if (wrc || ee != hipSuccess) {
                out_rc = wrc ? wrc : hip_code(ee);
                cv.notify_all();
                return;
            }
            out_enqueued = j + 1;
            cv.notify_all();
        }
    };
    // The copy-out side runs on a second host thread; if one cannot be started, the issuing loop
    // copies each window out itself right after its collective (no overlap of the two PCIe
    // directions, same bits) -- no exception crosses the C ABI.
    std::thread copy_out;
    try {
        copy_out = std::thread(copy_out_loop);
    } catch (const std::exception&) {
        copy_out = std::thread();
    }
    const bool threaded = copy_out.joinable();
    auto issue = [&]() -> int {
        for (size_t j = 0; j < nwin; ++j) {
            const int i = (int)(j & 1);
            const size_t off = j * w, wj = std::min(w, block - off);
            // window j reuses window j-2's buffers: its copy-in waits for j-2's collective, and
            // the collective for j-2's copy-out, once the copy-out thread has enqueued it
            if (j >= 2) {
                int r2;
                if ((r2 = wait_event(c, c->ev_coll[i]))) return r2;  // with a timeout: before the pageable copy
                if ((e = hipStreamWaitEvent(c->hin, c->ev_coll[i], 0)) != hipSuccess) return hip_code(e);
            }
            if ((e = hipMemcpy2DAsync(c->wsend[i].p, wj * es, hsrc + off * es, block * es, wj * es, n, hipMemcpyDefault,
                                      c->hin)) != hipSuccess)
                return hip_code(e);
            if ((e = hipEventRecord(c->ev_in[i], c->hin)) != hipSuccess) return hip_code(e);
            if ((e = hipStreamWaitEvent(c->stream, c->ev_in[i], 0)) != hipSuccess) return hip_code(e);
            if (j >= 2) {
                if (threaded) {
                    std::unique_lock<std::mutex> g(mu);
                    auto ready = [&] { return out_rc != CHR_SUCCESS || out_enqueued >= j - 1; };
                    if (timeout_ms > 0) {
                        // the copy-out thread gives up after the same timeout; this is the backstop
                        if (!cv.wait_for(g, std::chrono::milliseconds(2 * (int64_t)timeout_ms + 1000), ready))
                            return CHR_ERR_TIMEOUT;
                    } else {
                        cv.wait(g, ready);
                    }
                    if (out_rc != CHR_SUCCESS) return out_rc;
                }
                if ((e = hipStreamWaitEvent(c->stream, c->ev_out[i], 0)) != hipSuccess) return hip_code(e);
            }
            const Plan& p = c->plan(mode, k, b, mode == chr::MODE_ALLREDUCE ? n * wj : wj, es, sched, slices,
                                    chr::op_commutative(op));
            if (p.error) return p.error;
            int r = enqueue_rccl(c, p, c->wsend[i].p, c->wrecv[i].p, dtype, op);
            if (r) return r;
            if ((e = hipEventRecord(c->ev_coll[i], c->stream)) != hipSuccess) return hip_code(e);
            if (!threaded) {  // this thread copies window j out itself
                if ((r = wait_event(c, c->ev_coll[i]))) return r;
                if ((e = hipStreamWaitEvent(c->hout, c->ev_coll[i], 0)) != hipSuccess ||
                    (e = hipMemcpy2DAsync(hdst + off * es, block * es, c->wrecv[i].p, wj * es, wj * es, out_rows,
                                          hipMemcpyDefault, c->hout)) != hipSuccess ||
                    (e = hipEventRecord(c->ev_out[i], c->hout)) != hipSuccess)
                    return hip_code(e);
                continue;
            }
            std::lock_guard<std::mutex> g(mu);
            coll_enqueued = j + 1;
            cv.notify_all();
        }
        return CHR_SUCCESS;
    };
    rc = issue();
    if (rc) {
        if (!c->failed && (rc == CHR_ERR_TIMEOUT || rc == CHR_ERR_RCCL)) c->abort_comm();  // peers may be posted
        std::lock_guard<std::mutex> g(mu);
        stop = true;
        cv.notify_all();
    }
    if (!rc) rc = wait_call(c);  // the last collective, under the communicator's timeout
    if (threaded) copy_out.join();
    const int rc_out = hip_code(hipStreamSynchronize(c->hout));
    if (rc) return rc;
    if (out_rc && !c->failed) c->abort_comm();  // the copy-out side timed out: peers may still be posted
    return out_rc ? out_rc : rc_out;
}

// The (dtype, op) pairs a mode accepts: the data-movement collectives (allgather, the stand-alone
// intra scatter) move elements of any type and ignore op.
bool valid_args(int mode, int dtype, int op) {
    if (mode == chr::MODE_ALLGATHER || mode == chr::MODE_INTRA_SCATTER) return chr::dtype_size(dtype) != 0;
    return chr::valid_any(dtype, op);
}

int run_collective(chr_comm* c, int sched, int slices, int mode, const void* send, void* recv, size_t count, int dtype,
                   int op, int k, int b, bool sync) {
    const Plan& p = c->plan(mode, k, b, count, chr::dtype_size(dtype), sched, slices, chr::op_commutative(op));
    if (p.error) return p.error;
    if (p.g.total == 0) return CHR_SUCCESS;
    if (!recv && p.recv_elems) return CHR_ERR_INVALID_ARG;  // a rank whose plan writes no output may pass NULL
    const size_t es = chr::dtype_size(dtype);
    const bool inplace = send == CHR_IN_PLACE;
    if (inplace && (mode == chr::MODE_INTER_LINEAR || mode == chr::MODE_INTRA_SCATTER)) return CHR_ERR_INVALID_ARG;
    const void* input = !inplace ? send
                        : mode == chr::MODE_ALLGATHER ? (const void*)((char*)recv + (size_t)c->rank * count * es)
                                                      : (const void*)recv;
    if (!input && p.send_elems) return CHR_ERR_INVALID_ARG;  // a rank whose plan reads no input may pass NULL
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return hip_code(e);
    const bool dev_out = is_device_ptr(recv), dev_in = p.send_elems ? is_device_ptr(input) : dev_out;
    // Pipelined staging splits a call into window collectives.  Every rank must issue the same
    // collectives, so whether a call is split cannot depend on where this rank's buffers live alone:
    // a call large enough to split (host_window_elems) first agrees with one 4-byte
    // ncclAllReduce(min) whether every rank is device-resident.  If so, no rank windows (the direct,
    // graph-capable path, which the AUTO tuner also times); otherwise every rank does, a device
    // buffer then being staged device to device.  The exchange costs one small collective on calls of
    // at least one window (32 MiB per rank by default).
    if (sync && host_window_elems(c, mode, count, es)) {
        if (c->failed) return CHR_ERR_ABORTED;
        int all_dev = 0;
        int rc = agree_min(c, dev_in && dev_out, &all_dev);
        if (rc) return rc;
        if (!all_dev && (rc = run_host_windows(c, sched, slices, mode, input, recv, count, dtype, op, k, b)) >= 0)
            return rc;
    }
    if (dev_in && dev_out) {
        // a user op's launcher may allocate stream-ordered scratch: never captured (chiara.h chr_op_create)
        int rc = c->graphs && !c->prof.on && !chr::is_user_op(op) ? launch_graph(c, p, input, recv, dtype, op)
                                                                  : enqueue_rccl(c, p, input, recv, dtype, op);
        if (rc || !sync) return rc;
        return wait_call(c);
    }
    if (!sync) return CHR_ERR_UNSUPPORTED;  // async needs device-resident buffers
    // Host-memory contract of the reference: stage through HBM (PCIe H2D / D2H).  With a timeout
    // set, every copy to or from pageable memory is issued only after what it depends on has
    // completed (wait_call), since such a copy blocks inside HIP until it is staged.
    const void* dsend = input;
    void* drecv = recv;
    int rc;
    if ((rc = wait_call(c))) return rc;  // earlier _async work
    if (!dev_in && p.send_elems) {
        if ((e = c->hsend.reserve(p.send_elems * es, c->stream)) != hipSuccess) return hip_code(e);
        if ((e = hipMemcpyAsync(c->hsend.p, input, p.send_elems * es, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
            return hip_code(e);
        dsend = c->hsend.p;
    }
    if (!dev_out) {
        if ((e = c->hrecv.reserve(p.recv_elems * es, c->stream)) != hipSuccess) return hip_code(e);
        drecv = c->hrecv.p;
    }
    rc = enqueue_rccl(c, p, dsend, drecv, dtype, op);
    if (rc) return rc;
    if (!dev_out && p.recv_elems) {
        if (c->timeout_ms > 0 && (rc = wait_call(c))) return rc;  // the collective, under the timeout
        if ((e = hipMemcpyAsync(recv, drecv, p.recv_elems * es, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
            return hip_code(e);
    }
    return wait_call(c);
}

// CHR_SCHEDULE_AUTO.  The single-node schedules FLAT, FLAT_SEQ and FLAT_AG move the same bits
// over the same full-mesh traffic (2S/n per link) but differ in how RCCL groups and collectives
// share the links, and the pipeline depth trades overlap against per-group latency; which is
// fastest is a property of the machine, so on the first device-resident call for a given
// (collective, count, dtype, k, b) every candidate runs TUNE_REPS timed calls, the ranks agree on
// the slowest rank's time per candidate (one ncclAllReduce(max), so every rank picks the same
// one) and the fastest is kept for every later call.  Each tuning call is a complete collective;
// an in-place call is tuned on temporary copies so the caller's data is reduced exactly once.
//
// Tuning is collective, so every decision that could differ between ranks is agreed on first:
// whether this call can be tuned (device-resident buffers, the temporaries allocated) is one
// ncclAllReduce(min) over the ranks, and a call no rank can tune runs FLAT untuned on every rank.
// The cache is then identical on every rank, and a cached choice applies to later calls of the
// same arguments whatever memory their buffers are in.  A candidate that fails after posting
// RCCL operations aborts the communicator (enqueue_rccl); peers with a timeout (chr_comm_set_timeout)
// then return an error instead of waiting.
constexpr int TUNE_REPS = 3;

int tune_schedule(chr_comm* c, int mode, const void* send, void* recv, size_t count, int dtype, int op, int k, int b,
                  int* sched_out, int* slices_out) {
    *sched_out = chr::SCHED_FLAT;
    *slices_out = c->slices;
    if (chr::is_unpipelined(mode) || c->nranks < 2) return CHR_SUCCESS;
    if (c->failed) return CHR_ERR_ABORTED;
    const size_t es = chr::dtype_size(dtype);
    auto key = std::make_tuple(mode, (uint64_t)count, (int)es, k, b, c->slices, c->overlap);
    auto it = c->tuned.find(key);
    if (it != c->tuned.end()) {
        *sched_out = it->second.first;
        *slices_out = it->second.second;
        return CHR_SUCCESS;
    }
    const Plan& p0 = c->plan(mode, k, b, count, es, chr::SCHED_FLAT, c->slices, chr::op_commutative(op));
    if (p0.error) return p0.error;  // a function of the arguments only: the same on every rank
    if (p0.g.total == 0) return CHR_SUCCESS;
    const bool inplace = send == CHR_IN_PLACE;
    const void* input = inplace ? (const void*)recv : send;
    // in place: tune on copies (the collective would otherwise reduce the caller's data again)
    void* tsend = nullptr;
    void* trecv = nullptr;
    const void* s_arg = send;
    void* r_arg = recv;
    int ok = input && recv && is_device_ptr(input) && is_device_ptr(recv);
    if (ok && inplace) {
        ok = hipMalloc(&tsend, p0.send_elems * es) == hipSuccess && hipMalloc(&trecv, p0.recv_elems * es) == hipSuccess &&
             hipMemcpyAsync(tsend, recv, p0.send_elems * es, hipMemcpyDeviceToDevice, c->stream) == hipSuccess;
        (void)hipGetLastError();
        s_arg = tsend;
        r_arg = trecv;
    }
    auto release = [&]() {
        if (tsend || trecv) (void)hipStreamSynchronize(c->stream);
        (void)hipFree(tsend);
        (void)hipFree(trecv);
    };
    int all = 0;
    int rc = agree_min(c, ok, &all);
    if (rc || !all) {  // host-staged somewhere, or an allocation failed somewhere: FLAT, untuned
        release();
        return rc;
    }
    std::vector<std::pair<int, int>> cand;
    std::vector<int> depths;
    const int pa = pick_slices(c->slices, count, mode, c->nranks, b, es, chr::SCHED_REFERENCE);  // chunk-size depth
    for (int d = pa; d >= 1; d /= 2) {
        depths.push_back(d);
        if (c->slices > 0) break;  // an explicit depth is kept
    }
    for (int sc : {(int)chr::SCHED_FLAT, (int)chr::SCHED_FLAT_SEQ, (int)chr::SCHED_FLAT_AG})
        for (int d : depths) cand.push_back({sc, d});
    if (mode == chr::MODE_ALLREDUCE && (uint64_t)count * es <= kOneShotMaxBytes)
        for (int d : depths) cand.push_back({(int)chr::SCHED_FLAT_1SHOT, d});
    std::vector<float> ms(cand.size(), 0.f);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipSuccess;
    if ((e = hipEventCreate(&e0)) != hipSuccess || (e = hipEventCreate(&e1)) != hipSuccess) {
        rc = hip_code(e);
        c->abort_comm();  // the peers are about to start the candidates
    }
    for (size_t i = 0; i < cand.size() && !rc; ++i) {
        const int sc = cand[i].first, d = cand[i].second;
        // untimed first call: plan compile, scratch growth, RCCL connection setup
        if ((rc = run_collective(c, sc, d, mode, s_arg, r_arg, count, dtype, op, k, b, true))) break;
        if ((rc = hip_code(hipEventRecord(e0, c->stream)))) break;
        for (int r = 0; r < TUNE_REPS && !rc; ++r)
            rc = run_collective(c, sc, d, mode, s_arg, r_arg, count, dtype, op, k, b, false);
        if (rc || (rc = hip_code(hipEventRecord(e1, c->stream))) || (rc = wait_call(c))) break;
        rc = hip_code(hipEventElapsedTime(&ms[i], e0, e1));
    }
    if (rc && !c->failed) c->abort_comm();  // a local failure mid-tuning: the peers are still in it
    float* dms = nullptr;
    if (!rc && (rc = hip_code(hipMalloc(&dms, ms.size() * sizeof(float)))) == CHR_SUCCESS) {
        if (!(rc = hip_code(hipMemcpyAsync(dms, ms.data(), ms.size() * sizeof(float), hipMemcpyHostToDevice,
                                           c->stream))) &&
            !(rc = nccl_code(ncclAllReduce(dms, dms, ms.size(), ncclFloat32, ncclMax, c->nccl, c->stream))) &&
            !(rc = hip_code(hipMemcpyAsync(ms.data(), dms, ms.size() * sizeof(float), hipMemcpyDeviceToHost,
                                           c->stream))))
            rc = wait_call(c);
        if (rc && !c->failed) c->abort_comm();
    } else if (rc == CHR_ERR_OUT_OF_MEMORY && !c->failed) {
        c->abort_comm();
    }
    (void)hipFree(dms);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    release();
    if (rc) return rc;
    size_t best = 0;
    for (size_t i = 1; i < cand.size(); ++i)
        if (ms[i] < ms[best]) best = i;
    if (std::getenv("CHR_TUNE_VERBOSE") && c->rank == 0)
        for (size_t i = 0; i < cand.size(); ++i)
            std::fprintf(stderr, "[chiara] tune mode %d count %zu: schedule %d slices %d  %.3f ms%s\n", mode, count,
                         cand[i].first, cand[i].second, ms[i] / TUNE_REPS, i == best ? "  <- kept" : "");
    c->tuned[key] = cand[best];
    *sched_out = cand[best].first;
    *slices_out = cand[best].second;
    return CHR_SUCCESS;
}

int collective(chr_comm* c, int mode, const void* send, void* recv, size_t count, int dtype, int op, int k, int b,
               bool sync) {
    // allgather moves elements of any type (its op is unused)
    if (!c || !valid_args(mode, dtype, op)) return CHR_ERR_INVALID_ARG;
    if (c->failed) return CHR_ERR_ABORTED;
    int sched = c->sched, slices = c->slices;
    if (sched == CHR_SCHEDULE_AUTO) {
        if (hipSetDevice(c->device) != hipSuccess) return CHR_ERR_HIP;
        int rc = tune_schedule(c, mode, send, recv, count, dtype, op, k, b, &sched, &slices);
        if (rc) return rc;
    }
    return run_collective(c, sched, slices, mode, send, recv, count, dtype, op, k, b, sync);
}

int local_collective(chr_local_group* g, int mode, const void* const* sends, void* const* recvs, size_t count,
                     int dtype, int op, int k, int b) {
    if (!g || !sends || !recvs || !valid_args(mode, dtype, op)) return CHR_ERR_INVALID_ARG;
    const int n = g->nranks;
    // the MPICH baselines branch on MPI_Op_commutative (build_plan_mpich); CHiArA's own collectives take any op
    const bool commutative = chr::op_commutative(op);
    const int depth = pick_slices(g->slices, count, mode, n, b, chr::dtype_size(dtype), g->sched);
    auto key = std::make_tuple(mode, k, b, (uint64_t)count, (int)chr::dtype_size(dtype), depth, g->sched, commutative);
    auto it = g->plans.find(key);
    if (it == g->plans.end()) {
        std::vector<Plan> v;
        for (int r = 0; r < n; ++r)
            v.push_back(chr::build_plan((chr::Mode)mode, n, r, k, b, count, depth, g->sched, commutative));
        it = g->plans.emplace(key, std::move(v)).first;
    }
    const std::vector<Plan>& P = it->second;
    if (P[0].error) return P[0].error;
    if (P[0].g.total == 0) return CHR_SUCCESS;
    const size_t es = chr::dtype_size(dtype);
    hipError_t e = hipSetDevice(g->device);
    if (e != hipSuccess) return hip_code(e);
    std::vector<Bufs> B(n);
    for (int r = 0; r < n; ++r) {
        if (!recvs[r] && P[r].recv_elems) return CHR_ERR_INVALID_ARG;
        if ((e = g->acc[r].reserve(P[r].acc_elems * es, g->stream)) != hipSuccess) return hip_code(e);
        if ((e = g->stage[r].reserve(P[r].stage_elems * es, g->stream)) != hipSuccess) return hip_code(e);
        if (sends[r] == CHR_IN_PLACE && (mode == chr::MODE_INTER_LINEAR || mode == chr::MODE_INTRA_SCATTER))
            return CHR_ERR_INVALID_ARG;
        const void* in = sends[r] != CHR_IN_PLACE ? sends[r]
                         : mode == chr::MODE_ALLGATHER ? (const void*)((char*)recvs[r] + (size_t)r * count * es)
                                                       : (const void*)recvs[r];
        if ((P[r].send_elems && (!in || !is_device_ptr(in))) || (P[r].recv_elems && !is_device_ptr(recvs[r])))
            return CHR_ERR_INVALID_ARG;
        B[r] = Bufs{(const char*)in, (char*)recvs[r], (char*)g->acc[r].p, (char*)g->stage[r].p, es};
    }
    int rc;
    // One phase of local ops of all ranks, on the group's stream; while profiling, bracketed by events
    // on that stream.
    auto phase = [&](auto&& ops_of) -> int {
        bool any = false, reduces = false;
        for (int r = 0; r < n; ++r) {
            any = any || !ops_of(r).empty();
            for (const chr::LocalOp& op : ops_of(r)) reduces = reduces || op.kind == chr::L_REDUCE || op.kind == chr::L_TREE;
        }
        if (!any) return CHR_SUCCESS;
        // a phase of copies only (re-layouts, the stand-alone phases' copy-outs) is not a reduction span
        const bool span = g->prof.on && reduces;
        std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
        if (span) {
            ev = g->prof.take();
            if ((rc = hip_code(hipEventRecord(ev.first, g->stream)))) return rc;
        }
        // The virtual ranks' local ops of one step touch only their own buffers.  When every rank's
        // ops are one batchable run of trees (the flat schedules' slice evaluations), all ranks'
        // trees go to one launch_reduce_tree_multi call: one grid per 8 trees instead of one per
        // rank, so the step pays the fixed cost of a launch -- ~4.5 us between back-to-back grids
        // on one stream plus ~3-4 us of fill and drain (tools/reduce_microbench focus22/23,
        // profiles/r03/launch_timeline/) -- once per 8 trees.  A real node has one rank per GPU
        // and so one launch per rank per slice; rows measured there are the rank-alone replays of
        // bench.py --collective-kernels.
        std::vector<chr::TreeJob> jobs;
        double bytes = 0;
        bool merged = g->batch_ranks && n > 1;
        for (int r = 0; r < n && merged; ++r) {
            const std::vector<chr::LocalOp>& ops = ops_of(r);
            if (!one_tree_run(ops, B[r])) {
                merged = false;
                break;
            }
            const size_t j0 = jobs.size();
            bytes += tree_jobs(ops, 0, ops.size(), B[r], &jobs);
            for (size_t x = 0; x < j0 && merged; ++x)  // earlier ranks' trees vs this rank's
                for (size_t y = j0; y < jobs.size() && merged; ++y)
                    merged = !job_conflict(jobs[x], jobs[y], es) && !job_conflict(jobs[y], jobs[x], es);
        }
        if (merged) {
            if ((rc = launch_tree_jobs(jobs, bytes, dtype, op, g->stream, &g->prof))) return rc;
        } else {
            for (int r = 0; r < n; ++r)
                if ((rc = run_locals(ops_of(r), B[r], dtype, op, g->stream, &g->prof))) return rc;
        }
        if (span) {
            if ((rc = hip_code(hipEventRecord(ev.second, g->stream)))) return rc;
            g->prof.pending.push_back(ev);
        }
        return CHR_SUCCESS;
    };
    if ((rc = phase([&](int r) -> const std::vector<chr::LocalOp>& { return P[r].pre; }))) return rc;
    const size_t nsteps = P[0].steps.size();
    for (size_t si = 0; si < nsteps; ++si) {
        // Loopback transport: each receive takes the next unmatched send of its peer to
        // this rank in the same step (RCCL's per-pair ordering).
        std::vector<std::vector<char>> used(n);
        for (int r = 0; r < n; ++r) used[r].assign(P[r].steps[si].sends.size(), 0);
        for (int r = 0; r < n; ++r) {
            for (const chr::Xfer& rv : P[r].steps[si].recvs) {
                const int q = rv.peer;
                const auto& qs = P[q].steps[si].sends;
                size_t j = 0;
                while (j < qs.size() && (used[q][j] || qs[j].peer != r)) ++j;
                if (j == qs.size() || qs[j].count != rv.count) {
                    std::fprintf(stderr, "[chiara] plan mismatch: step %zu rank %d <- %d\n", si, r, q);
                    return CHR_ERR_UNSUPPORTED;
                }
                used[q][j] = 1;
                if ((e = hipMemcpyAsync(B[r].ptr(rv.ref), B[q].ptr(qs[j].ref), rv.count * es, hipMemcpyDeviceToDevice,
                                        g->stream)) != hipSuccess)
                    return hip_code(e);
            }
        }
        for (int r = 0; r < n; ++r)
            for (size_t j = 0; j < used[r].size(); ++j)
                if (!used[r][j]) {
                    std::fprintf(stderr, "[chiara] plan mismatch: unmatched send step %zu rank %d\n", si, r);
                    return CHR_ERR_UNSUPPORTED;
                }
        // allgather collectives: every rank's block r to every other rank, same region
        for (size_t ci = 0; ci < P[0].steps[si].allgathers.size(); ++ci)
            for (int r = 0; r < n; ++r)
                for (int q = 0; q < n; ++q) {
                    if (q == r) continue;
                    const chr::Coll& x = P[r].steps[si].allgathers[ci];
                    const size_t off = (size_t)q * x.count * es;
                    if ((e = hipMemcpyAsync(B[r].ptr(x.ref) + off, B[q].ptr(P[q].steps[si].allgathers[ci].ref) + off,
                                            x.count * es, hipMemcpyDeviceToDevice, g->stream)) != hipSuccess)
                        return hip_code(e);
                }
        if ((rc = phase([&](int r) -> const std::vector<chr::LocalOp>& { return P[r].steps[si].post; })))
            return rc;
    }
    return hip_code(hipStreamSynchronize(g->stream));
}

}  // namespace

extern "C" {

int chr_get_unique_id(chr_unique_id* id) {
    static_assert(sizeof(chr_unique_id) == sizeof(ncclUniqueId), "unique id size");
    if (!id) return CHR_ERR_INVALID_ARG;
    ncclUniqueId u;
    int rc = nccl_code(ncclGetUniqueId(&u));
    if (!rc) std::memcpy(id, &u, sizeof(u));
    return rc;
}

int chr_comm_init_rank(chr_comm** out, int nranks, const chr_unique_id* id, int rank, int device) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return CHR_ERR_INVALID_ARG;
    {  // the entry paths set the default (api.cpp); a multi-rank communicator without it is worth a warning
        static bool warned = false;
        const char* ipc = std::getenv("HSA_ENABLE_IPC_MODE_LEGACY");
        if (!warned && nranks > 1 && (!ipc || std::strcmp(ipc, "0") != 0)) {
            std::fprintf(stderr,
                         "[chiara] HSA_ENABLE_IPC_MODE_LEGACY=%s: RCCL's IPC transport needs 0 (dmabuf) on this "
                         "driver; expect hipIpcGetMemHandle failures\n",
                         ipc ? ipc : "(unset)");
            warned = true;
        }
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return CHR_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return CHR_ERR_INVALID_ARG;
    auto c = std::make_unique<chr_comm>();
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamDefault);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->cstream, hipStreamDefault);
    if (e != hipSuccess) return hip_code(e);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    int rc = nccl_code(ncclCommInitRank(&c->nccl, nranks, u, rank));
    if (rc) {
        (void)hipStreamDestroy(c->stream);
        (void)hipStreamDestroy(c->cstream);
        return rc;
    }
    *out = c.release();
    return CHR_SUCCESS;
}

int chr_comm_destroy(chr_comm* c) {
    if (!c) return CHR_SUCCESS;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->drop_graphs();
    c->prof.release();
    if (c->nccl) (void)ncclCommDestroy(c->nccl);  // an aborted communicator was released by ncclCommAbort
    c->acc.release();
    c->stage.release();
    c->hsend.release();
    c->hrecv.release();
    c->flag.release();
    c->host_pipeline_release();
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    for (hipEvent_t e : c->events) (void)hipEventDestroy(e);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return CHR_SUCCESS;
}

int chr_comm_rank(const chr_comm* c, int* rank) {
    if (!c || !rank) return CHR_ERR_INVALID_ARG;
    *rank = c->rank;
    return CHR_SUCCESS;
}

int chr_comm_size(const chr_comm* c, int* n) {
    if (!c || !n) return CHR_ERR_INVALID_ARG;
    *n = c->nranks;
    return CHR_SUCCESS;
}

int chr_comm_info(const chr_comm* c, int* rccl_nranks, int* rccl_rank, int* rccl_device, char* pci_bus_id,
                  int len) {
    if (!c || !rccl_nranks || !rccl_rank || !rccl_device || (!pci_bus_id && len > 0) || len < 0)
        return CHR_ERR_INVALID_ARG;
    if (c->failed || !c->nccl) return CHR_ERR_ABORTED;
    // what RCCL's communicator itself holds, not this struct's copy of the init arguments
    int rc = nccl_code(ncclCommCount(c->nccl, rccl_nranks));
    if (!rc) rc = nccl_code(ncclCommUserRank(c->nccl, rccl_rank));
    if (!rc) rc = nccl_code(ncclCommCuDevice(c->nccl, rccl_device));
    if (rc) return rc;
    if (len > 0) {
        pci_bus_id[0] = '\0';
        const hipError_t e = hipDeviceGetPCIBusId(pci_bus_id, len, *rccl_device);
        if (e != hipSuccess) return hip_code(e);
    }
    return CHR_SUCCESS;
}

int chr_comm_set_timeout(chr_comm* c, int timeout_ms) {
    if (!c || timeout_ms < 0) return CHR_ERR_INVALID_ARG;
    c->timeout_ms = timeout_ms;
    return CHR_SUCCESS;
}

int chr_comm_abort(chr_comm* c) {
    if (!c) return CHR_ERR_INVALID_ARG;
    (void)hipSetDevice(c->device);
    c->abort_comm();
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    return CHR_SUCCESS;
}

int chr_comm_synchronize(chr_comm* c) {
    if (!c) return CHR_ERR_INVALID_ARG;
    if (c->failed) return CHR_ERR_ABORTED;
    if (hipSetDevice(c->device) != hipSuccess) return CHR_ERR_HIP;
    return wait_call(c);
}

int chr_comm_is_aborted(const chr_comm* c) { return c && c->failed ? 1 : 0; }

int chr_comm_set_slices(chr_comm* c, int slices) {
    if (!c || slices < 0) return CHR_ERR_INVALID_ARG;
    c->slices = slices;
    return CHR_SUCCESS;
}

int chr_comm_profile(chr_comm* c, int enable) {
    if (!c) return CHR_ERR_INVALID_ARG;
    c->prof.on = enable != 0;
    return CHR_SUCCESS;
}

int chr_comm_profile_read(chr_comm* c, double* reduce_ms, double* reduce_bytes, long* launches, int reset) {
    if (!c) return CHR_ERR_INVALID_ARG;
    (void)hipSetDevice(c->device);
    c->prof.drain();
    if (reduce_ms) *reduce_ms = c->prof.ms;
    if (reduce_bytes) *reduce_bytes = c->prof.bytes;
    if (launches) *launches = c->prof.launches;
    if (reset) {
        c->prof.ms = 0;
        c->prof.bytes = 0;
        c->prof.launches = 0;
    }
    return CHR_SUCCESS;
}

long chr_comm_profile_phases(chr_comm* c, char* buf, size_t len, int reset) {
    if (!c) return -1;
    (void)hipSetDevice(c->device);
    c->prof.drain();
    std::string s;
    char line[160];
    for (const auto& kv : c->prof.phase_ms) {
        std::snprintf(line, sizeof line, "%s %.6f\n", kv.first.c_str(), kv.second);
        s += line;
    }
    if (buf && len) {
        const size_t n = s.size() < len - 1 ? s.size() : len - 1;
        std::memcpy(buf, s.data(), n);
        buf[n] = '\0';
    }
    if (reset) c->prof.phase_ms.clear();
    return (long)s.size();
}

int chr_comm_set_overlap(chr_comm* c, int enable) {
    if (!c) return CHR_ERR_INVALID_ARG;
    c->overlap = enable != 0;
    return CHR_SUCCESS;
}

int chr_comm_get_overlap(const chr_comm* c, int* enable) {
    if (!c || !enable) return CHR_ERR_INVALID_ARG;
    *enable = c->overlap ? 1 : 0;
    return CHR_SUCCESS;
}

int chr_comm_set_schedule(chr_comm* c, int schedule) {
    if (!c || !(chr::plan_schedule(schedule) || schedule == CHR_SCHEDULE_AUTO)) return CHR_ERR_INVALID_ARG;
    c->sched = schedule;
    return CHR_SUCCESS;
}

int chr_comm_set_host_pipeline(chr_comm* c, int window_mib) {
    if (!c || window_mib < 0) return CHR_ERR_INVALID_ARG;
    c->host_window_mib = window_mib;
    return CHR_SUCCESS;
}

int chr_comm_set_graphs(chr_comm* c, int enable) {
    if (!c) return CHR_ERR_INVALID_ARG;
    if (!enable && c->stream) {
        (void)hipStreamSynchronize(c->stream);
        c->drop_graphs();
    }
    c->graphs = enable != 0;
    return CHR_SUCCESS;
}

int chr_comm_tuned_schedule(const chr_comm* c, int mode, size_t count, chr_dtype dtype, int k, int b, int* schedule,
                            int* slices) {
    if (!c || !schedule || !slices || !chr::dtype_size(dtype)) return CHR_ERR_INVALID_ARG;
    if (mode != chr::MODE_ALLREDUCE && mode != chr::MODE_REDUCE_SCATTER) return CHR_ERR_INVALID_ARG;
    if (c->failed) return CHR_ERR_ABORTED;
    if (c->sched != CHR_SCHEDULE_AUTO) {  // a fixed schedule: it, at the depth such a call runs
        const int P = pick_slices(c->slices, (uint64_t)count, mode, c->nranks, b, chr::dtype_size(dtype), c->sched);
        // the arguments a call would reject (k < 2, nranks % b, count % nranks) are rejected here too
        const chr::Plan p = chr::build_plan((chr::Mode)mode, c->nranks, c->rank, k, b, (uint64_t)count, P, c->sched);
        if (p.error) return p.error;
        *schedule = c->sched;
        *slices = P;
        return CHR_SUCCESS;
    }
    auto it = c->tuned.find(std::make_tuple(mode, (uint64_t)count, (int)chr::dtype_size(dtype), k, b, c->slices,
                                            c->overlap));
    if (it == c->tuned.end()) return CHR_ERR_INVALID_ARG;
    *schedule = it->second.first;
    *slices = it->second.second;
    return CHR_SUCCESS;
}

int chr_local_group_set_schedule(chr_local_group* g, int schedule) {
    if (!g || !chr::plan_schedule(schedule)) return CHR_ERR_INVALID_ARG;
    g->sched = schedule;
    return CHR_SUCCESS;
}

int chr_local_group_set_batching(chr_local_group* g, int enable) {
    if (!g) return CHR_ERR_INVALID_ARG;
    g->batch_ranks = enable != 0;
    return CHR_SUCCESS;
}

int chr_local_group_set_slices(chr_local_group* g, int slices) {
    if (!g || slices < 0) return CHR_ERR_INVALID_ARG;
    g->slices = slices;
    return CHR_SUCCESS;
}

int chr_comm_stream(const chr_comm* c, hipStream_t* s) {
    if (!c || !s) return CHR_ERR_INVALID_ARG;
    *s = c->stream;
    return CHR_SUCCESS;
}

int chr_allreduce_radix_batch(const void* send, void* recv, size_t count, chr_dtype dtype, chr_op op, chr_comm* comm,
                              int k, int b) {
    return collective(comm, chr::MODE_ALLREDUCE, send, recv, count, dtype, op, k, b, true);
}

int chr_reduce_scatter_radix_batch(const void* send, void* recv, size_t recvcount, chr_dtype dtype, chr_op op,
                                   chr_comm* comm, int k, int b) {
    return collective(comm, chr::MODE_REDUCE_SCATTER, send, recv, recvcount, dtype, op, k, b, true);
}

int chr_allreduce_radix_batch_async(const void* send, void* recv, size_t count, chr_dtype dtype, chr_op op,
                                    chr_comm* comm, int k, int b) {
    return collective(comm, chr::MODE_ALLREDUCE, send, recv, count, dtype, op, k, b, false);
}

int chr_reduce_scatter_radix_batch_async(const void* send, void* recv, size_t recvcount, chr_dtype dtype, chr_op op,
                                         chr_comm* comm, int k, int b) {
    return collective(comm, chr::MODE_REDUCE_SCATTER, send, recv, recvcount, dtype, op, k, b, false);
}

int chr_local_group_create(chr_local_group** out, int nranks, int device) {
    if (!out || nranks < 1) return CHR_ERR_INVALID_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return CHR_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return CHR_ERR_INVALID_ARG;
    auto g = std::make_unique<chr_local_group>();
    g->nranks = nranks;
    g->device = device;
    g->acc.resize(nranks);
    g->stage.resize(nranks);
    g->prof.span = true;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->stream, hipStreamDefault);
    if (e != hipSuccess) {
        chr_local_group_destroy(g.release());
        return hip_code(e);
    }
    *out = g.release();
    return CHR_SUCCESS;
}

int chr_local_group_profile(chr_local_group* g, int enable) {
    if (!g) return CHR_ERR_INVALID_ARG;
    g->prof.on = enable != 0;
    return CHR_SUCCESS;
}

int chr_local_group_profile_read(chr_local_group* g, double* reduce_ms, double* reduce_bytes, long* launches,
                                 int reset) {
    if (!g) return CHR_ERR_INVALID_ARG;
    (void)hipSetDevice(g->device);
    g->prof.drain();
    if (reduce_ms) *reduce_ms = g->prof.ms;
    if (reduce_bytes) *reduce_bytes = g->prof.bytes;
    if (launches) *launches = g->prof.launches;
    if (reset) {
        g->prof.ms = 0;
        g->prof.bytes = 0;
        g->prof.launches = 0;
    }
    return CHR_SUCCESS;
}

int chr_local_group_destroy(chr_local_group* g) {
    if (!g) return CHR_SUCCESS;
    (void)hipSetDevice(g->device);
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    g->prof.release();
    for (auto& d : g->acc) d.release();
    for (auto& d : g->stage) d.release();
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
    return CHR_SUCCESS;
}

int chr_local_group_stream(const chr_local_group* g, hipStream_t* s) {
    if (!g || !s) return CHR_ERR_INVALID_ARG;
    *s = g->stream;
    return CHR_SUCCESS;
}

int chr_local_allreduce_radix_batch(chr_local_group* g, const void* const* sends, void* const* recvs, size_t count,
                                    chr_dtype dtype, chr_op op, int k, int b) {
    return local_collective(g, chr::MODE_ALLREDUCE, sends, recvs, count, dtype, op, k, b);
}

int chr_local_reduce_scatter_radix_batch(chr_local_group* g, const void* const* sends, void* const* recvs,
                                         size_t recvcount, chr_dtype dtype, chr_op op, int k, int b) {
    return local_collective(g, chr::MODE_REDUCE_SCATTER, sends, recvs, recvcount, dtype, op, k, b);
}

static bool valid_mpich_mode(chr_mode m) {
    return m >= CHR_MODE_MPICH_RING && m <= CHR_MODE_MPICH_RMULT;
}

static bool valid_mpich_rs_mode(chr_mode m) {
    return m >= CHR_MODE_MPICH_RS_RADIX && m <= CHR_MODE_MPICH_RS_PAIRWISE;
}

int chr_allreduce_mpich(const void* send, void* recv, size_t count, chr_dtype dtype, chr_op op, chr_comm* comm,
                        chr_mode algo, int k, int single_phase_recv) {
    if (!valid_mpich_mode(algo)) return CHR_ERR_INVALID_ARG;
    return collective(comm, algo, send, recv, count, dtype, op, k, single_phase_recv, true);
}

int chr_allreduce_mpich_async(const void* send, void* recv, size_t count, chr_dtype dtype, chr_op op, chr_comm* comm,
                              chr_mode algo, int k, int single_phase_recv) {
    if (!valid_mpich_mode(algo)) return CHR_ERR_INVALID_ARG;
    return collective(comm, algo, send, recv, count, dtype, op, k, single_phase_recv, false);
}

int chr_local_allreduce_mpich(chr_local_group* g, const void* const* sends, void* const* recvs, size_t count,
                              chr_dtype dtype, chr_op op, chr_mode algo, int k, int single_phase_recv) {
    if (!valid_mpich_mode(algo)) return CHR_ERR_INVALID_ARG;
    return local_collective(g, algo, sends, recvs, count, dtype, op, k, single_phase_recv);
}

int chr_reduce_scatter_mpich(const void* send, void* recv, size_t recvcount, chr_dtype dtype, chr_op op,
                             chr_comm* comm, chr_mode algo, int k) {
    if (!valid_mpich_rs_mode(algo)) return CHR_ERR_INVALID_ARG;
    return collective(comm, algo, send, recv, recvcount, dtype, op, k, 0, true);
}

int chr_reduce_scatter_mpich_async(const void* send, void* recv, size_t recvcount, chr_dtype dtype, chr_op op,
                                   chr_comm* comm, chr_mode algo, int k) {
    if (!valid_mpich_rs_mode(algo)) return CHR_ERR_INVALID_ARG;
    return collective(comm, algo, send, recv, recvcount, dtype, op, k, 0, false);
}

int chr_local_reduce_scatter_mpich(chr_local_group* g, const void* const* sends, void* const* recvs, size_t recvcount,
                                   chr_dtype dtype, chr_op op, chr_mode algo, int k) {
    if (!valid_mpich_rs_mode(algo)) return CHR_ERR_INVALID_ARG;
    return local_collective(g, algo, sends, recvs, recvcount, dtype, op, k, 0);
}

int chr_allgather_radix_batch(const void* send, size_t sendcount, chr_dtype dtype, void* recv, chr_comm* comm, int k,
                              int b) {
    return collective(comm, chr::MODE_ALLGATHER, send, recv, sendcount, dtype, CHR_SUM, k, b, true);
}

int chr_allgather_radix_batch_async(const void* send, size_t sendcount, chr_dtype dtype, void* recv, chr_comm* comm,
                                    int k, int b) {
    return collective(comm, chr::MODE_ALLGATHER, send, recv, sendcount, dtype, CHR_SUM, k, b, false);
}

int chr_local_allgather_radix_batch(chr_local_group* g, const void* const* sends, void* const* recvs, size_t sendcount,
                                    chr_dtype dtype, int k, int b) {
    return local_collective(g, chr::MODE_ALLGATHER, sends, recvs, sendcount, dtype, CHR_SUM, k, b);
}

int chr_intra_reduce_scatter_radix_batch(const void* send, void* recv, size_t recvcount, chr_dtype dtype, chr_op op,
                                         chr_comm* comm, int k, int b) {
    return collective(comm, chr::MODE_INTRA_RS, send, recv, recvcount, dtype, op, k, b, true);
}

int chr_inter_reduce_linear(const void* send, void* recv, size_t recvcount, chr_dtype dtype, chr_op op, chr_comm* comm,
                            int b) {
    return collective(comm, chr::MODE_INTER_LINEAR, send, recv, recvcount, dtype, op, 2, b, true);
}

int chr_intra_scatter_radix_batch(const void* send, size_t recvcount, chr_dtype dtype, void* recv, chr_comm* comm,
                                  int k, int b) {
    return collective(comm, chr::MODE_INTRA_SCATTER, send, recv, recvcount, dtype, CHR_SUM, k, b, true);
}

int chr_local_phase_collective(chr_local_group* g, chr_mode mode, const void* const* sends, void* const* recvs,
                               size_t recvcount, chr_dtype dtype, chr_op op, int k, int b) {
    if (!chr::is_phase(mode)) return CHR_ERR_INVALID_ARG;
    return local_collective(g, mode, sends, recvs, recvcount, dtype, mode == CHR_MODE_INTRA_SCATTER ? CHR_SUM : op,
                            mode == CHR_MODE_INTER_REDUCE_LINEAR ? 2 : k, b);
}

}  // extern "C"
