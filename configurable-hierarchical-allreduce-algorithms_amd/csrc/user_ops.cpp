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
// MPI_Reduce_local(below, in) (MPICH_do_reduce's order), the running-value-first form of the launcher.  A combine
// at stack position p writes scratch slot p: it reads the value below (a leaf, or slot p itself) and the top (a leaf
// or slot p + 1), so no input is ever written.  The root is copied to `out` after the last fold.
int user_tree(const UserOp& u, void* out, const void* const* leaves, int nl, const uint8_t* comb,
              const uint8_t* swaps, size_t n, int dtype, hipStream_t s) {
    const size_t bytes = n * dtype_size(dtype);
    void* slot[8] = {};  // stack positions: at most 8 leaves (tree_program_ok)
    std::vector<const void*> st;
    int ci = 0, rc = CHR_SUCCESS;
    for (int j = 0; j < nl && !rc; ++j) {
        st.push_back(leaves[j]);
        for (int c = 0; c < comb[j] && !rc; ++c, ++ci) {
            const void* top = st.back();
            st.pop_back();
            const size_t p = st.size() - 1;
            if (!slot[p] && (rc = hip_status(hipMallocAsync(&slot[p], bytes, s)))) break;
            rc = call(u, slot[p], st.back(), &top, 1, n, dtype, swaps && swaps[ci], s);
            st.back() = slot[p];
        }
    }
    if (!rc && st.size() == 1 && st[0] != out)
        rc = hip_status(hipMemcpyAsync(out, st[0], bytes, hipMemcpyDeviceToDevice, s));
    for (void* p : slot)
        if (p) (void)hipFreeAsync(p, s);
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
