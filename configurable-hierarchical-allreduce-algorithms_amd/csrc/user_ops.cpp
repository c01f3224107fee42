// user_ops.cpp -- user-defined reduction ops: MPI_Op_create's analogue on MI355X.
//
// The reference is generic over MPI_Op (all_reduce_radix_batch.cpp:202-204), user-defined ops included: each of its
// MPI_Reduce_local calls (:332, :364, :446, :529) hands the op's function the host buffers.  Here a user op's
// arithmetic is the caller's own device code: chr_op_create registers a host launcher that enqueues it on the stream
// the library passes (include/chiara.h chr_user_reduce_fn; include/chiara_user_op.hpp builds one from a device
// functor).  Folds go to the launcher as they are; an expression tree (the flat schedules' one-pass evaluation,
// k_reduce_tree for the predefined ops) is evaluated fold by fold in its post-order program, intermediate values in
// stream-ordered scratch.  Nothing runs on the host.
#include "user_ops.hpp"

#include <mutex>
#include <vector>

#include "chiara.h"

namespace chr {

namespace {

struct UserOp {
    chr_user_reduce_fn fn = nullptr;
    void* ctx = nullptr;
    int commute = 0;
    bool live = false;
};

std::mutex g_mu;
UserOp g_ops[kMaxUserOps];

bool lookup(int op, UserOp* out) {
    if (!is_user_op(op)) return false;
    std::lock_guard<std::mutex> lk(g_mu);
    const UserOp& u = g_ops[op - kUserOpBase];
    if (!u.live) return false;
    *out = u;
    return true;
}

int hip_status(hipError_t e) {
    if (e == hipSuccess) return CHR_SUCCESS;
    return e == hipErrorOutOfMemory ? CHR_ERR_OUT_OF_MEMORY : CHR_ERR_HIP;
}

// The launcher's verdict: 0 = enqueued; anything else = the op refused the call (e.g. a type it does not implement).
int call(const UserOp& u, void* out, const void* acc, const void* const* ins, int m, size_t n, int dtype, bool rf,
         hipStream_t s) {
    if (u.fn(out, acc, ins, m, n, (chr_dtype)dtype, rf ? 1 : 0, s, u.ctx) != 0) return CHR_ERR_UNSUPPORTED;
    return hip_status(hipGetLastError());
}

// One post-order program (launch_reduce_tree's contract): push leaf j, then comb[j] combines, each popping the top
// `in` and folding it into the value below -- MPI_Reduce_local(in, below), or with the combine's swap bit
// MPI_Reduce_local(below, in) (MPICH_do_reduce's order), the running-value-first form of the launcher.  Consecutive
// combines that fold leaves into the same running value in the same order are one chain -- one launcher call with
// m inputs, as chr_reduce_multi_ex would make it -- so C4's tree ((l0 l1 l2 l3)(l4 l5 l6 l7)) is three calls, not
// seven.  A chain's result goes to scratch slot p (its stack position; it may read slot p itself as the running
// value, never as an input), the last one straight to `out` unless `out` is one of its inputs.
int user_tree(const UserOp& u, void* out, const void* const* leaves, int nl, const uint8_t* comb,
              const uint8_t* swaps, size_t n, int dtype, hipStream_t s) {
    const size_t bytes = n * dtype_size(dtype);
    void* slot[8] = {};  // stack positions: at most 8 leaves (tree_program_ok)
    struct Val {
        const void* p;
        bool leaf;
    };
    struct Chain {
        int pos = -1;  // stack position of the running value; -1: none pending
        const void* acc = nullptr;
        std::vector<const void*> ins;
        bool rf = false;
    } ch;
    std::vector<Val> st;
    int rc = CHR_SUCCESS;
    auto flush = [&](bool last) -> int {
        if (ch.pos < 0) return CHR_SUCCESS;
        void* dst = nullptr;
        if (last) {
            bool out_is_input = false;
            for (const void* q : ch.ins) out_is_input |= q == out;
            if (!out_is_input) dst = out;
        }
        if (!dst) {
            if (!slot[ch.pos])
                if (int e = hip_status(hipMallocAsync(&slot[ch.pos], bytes, s))) return e;
            dst = slot[ch.pos];
        }
        const int e = call(u, dst, ch.acc, ch.ins.data(), (int)ch.ins.size(), n, dtype, ch.rf, s);
        st[ch.pos] = {dst, false};
        ch.pos = -1;
        ch.ins.clear();
        return e;
    };
    int ci = 0;
    for (int j = 0; j < nl && !rc; ++j) {
        st.push_back({leaves[j], true});
        for (int c = 0; c < comb[j] && !rc; ++c, ++ci) {
            const int p = (int)st.size() - 2;  // the running value's position; the top is at p + 1
            const bool rf = swaps && swaps[ci];
            if (ch.pos == p && ch.rf == rf && st.back().leaf) {  // a leaf into the pending chain's running value
                ch.ins.push_back(st.back().p);
                st.pop_back();
                continue;
            }
            if ((rc = flush(false))) break;  // the pending chain's value lands in st[] before it is read
            ch.pos = p;
            ch.acc = st[p].p;
            ch.ins.assign(1, st.back().p);
            ch.rf = rf;
            st.pop_back();
        }
    }
    if (!rc) rc = flush(true);
    if (!rc && st.size() == 1 && st[0].p != out)
        rc = hip_status(hipMemcpyAsync(out, st[0].p, bytes, hipMemcpyDeviceToDevice, s));
    for (void* q : slot)
        if (q) (void)hipFreeAsync(q, s);
    return rc;
}

}  // namespace

bool is_user_op(int op) { return op >= kUserOpBase && op < kUserOpBase + kMaxUserOps; }

bool op_commutative(int op) {
    UserOp u;
    return !is_user_op(op) || (lookup(op, &u) && u.commute);
}

bool valid_any(int dtype, int op) {
    if (!is_user_op(op)) return valid_dtype_op(dtype, op);
    UserOp u;
    return dtype_size(dtype) != 0 && lookup(op, &u);
}

int reduce_any(void* out, const void* acc, const void* const* ins, int m, size_t n, int dtype, int op, hipStream_t s,
               bool running_first) {
    UserOp u;
    if (!is_user_op(op)) return hip_status(launch_reduce(out, acc, ins, m, n, dtype, op, s, running_first));
    if (!lookup(op, &u)) return CHR_ERR_INVALID_ARG;
    if (n == 0) return CHR_SUCCESS;
    return call(u, out, acc, ins, m, n, dtype, running_first, s);
}

int reduce_tree_any(void* out, const void* const* leaves, int nl, const uint8_t* comb, const uint8_t* swaps, size_t n,
                    int dtype, int op, hipStream_t s) {
    UserOp u;
    if (!is_user_op(op)) return hip_status(launch_reduce_tree(out, leaves, nl, comb, swaps, n, dtype, op, s));
    if (!lookup(op, &u)) return CHR_ERR_INVALID_ARG;
    if (n == 0) return CHR_SUCCESS;
    return user_tree(u, out, leaves, nl, comb, swaps, n, dtype, s);
}

int reduce_tree_multi_any(const TreeJob* jobs, int njobs, int dtype, int op, hipStream_t s) {
    UserOp u;
    if (!is_user_op(op)) return hip_status(launch_reduce_tree_multi(jobs, njobs, dtype, op, s));
    if (!lookup(op, &u)) return CHR_ERR_INVALID_ARG;
    for (int t = 0; t < njobs; ++t)
        if (jobs[t].n)
            if (int rc = user_tree(u, jobs[t].out, jobs[t].leaves, jobs[t].nl, jobs[t].comb, jobs[t].swaps, jobs[t].n,
                                   dtype, s))
                return rc;
    return CHR_SUCCESS;
}

}  // namespace chr

extern "C" {

int chr_op_create(chr_user_reduce_fn fn, void* ctx, int commute, chr_op* op) {
    if (!fn || !op) return CHR_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(chr::g_mu);
    for (int i = 0; i < chr::kMaxUserOps; ++i) {
        chr::UserOp& u = chr::g_ops[i];
        if (u.live) continue;
        u.fn = fn;
        u.ctx = ctx;
        u.commute = commute != 0;
        u.live = true;
        *op = (chr_op)(chr::kUserOpBase + i);
        return CHR_SUCCESS;
    }
    return CHR_ERR_UNSUPPORTED;  // every slot taken
}

int chr_op_free(chr_op op) {
    if (!chr::is_user_op((int)op)) return CHR_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(chr::g_mu);
    chr::UserOp& u = chr::g_ops[(int)op - chr::kUserOpBase];
    if (!u.live) return CHR_ERR_INVALID_ARG;
    u = chr::UserOp{};
    return CHR_SUCCESS;
}

}  // extern "C"
