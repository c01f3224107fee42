// plan_fuzz.cpp -- host-only sweep of the schedule compiler under AddressSanitizer / UBSan.
// Builds every rank's plan for every (mode, n, k, b, count, slices, schedule) in a wide grid,
// checks the plans pair up (every send has a matching receive in the same step with the same
// size) and that every buffer reference stays inside its declared buffer, and describes each
// plan (exercising the printer).  Run by tests/test_plan_fuzz.py:
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all \
//       -Iinclude -I<pkg>/csrc tools/plan_fuzz.cpp <pkg>/csrc/schedule.cpp -o /tmp/plan_fuzz
#include <cstdio>
#include <cstdlib>
#include <map>
#include <tuple>
#include <vector>

#include "schedule.hpp"

using namespace chr;

static int g_bad = 0;
static void fail(const char* what, int mode, int n, int k, int b, unsigned long long count, int sched) {
    if (g_bad++ < 20)
        std::fprintf(stderr, "FAIL %s mode=%d n=%d k=%d b=%d count=%llu sched=%d\n", what, mode, n, k, b, count, sched);
}

static bool in_bounds(const Plan& p, const Ref& r, uint64_t cnt) {
    const uint64_t lim = r.buf == BUF_SEND ? p.send_elems : r.buf == BUF_RECV ? p.recv_elems
                         : r.buf == BUF_ACC ? p.acc_elems : p.stage_elems;
    return r.off + cnt <= lim;
}

static bool op_in_bounds(const Plan& p, const LocalOp& op) {
    const uint64_t rows = op.kind == L_COPY2D ? op.rows : 1;
    for (uint64_t row = 0; row < rows; ++row) {
        Ref d = op.dst, a = op.acc;
        d.off += row * op.dpitch;
        a.off += row * op.spitch;
        if (!in_bounds(p, d, op.count) || !in_bounds(p, a, op.count)) return false;
    }
    for (const Ref& x : op.ins)
        if (!in_bounds(p, x, op.count)) return false;
    return true;
}

int main(int argc, char** argv) {
    const int max_n = argc > 1 ? std::atoi(argv[1]) : 16;  // the CPU test runs a reduced grid
    // per-phase timer names (chr_comm_profile_phases): whole-token de-duplication
    const std::pair<const char*, const char*> names[] = {
        {"t3,phase0/s0,lane/s1", "phase0+lane"}, {"gather/s2", "gather"}, {"allgather/s0,gather/s1", "allgather+gather"},
        {"phase01/s0,phase0/s1", "phase01+phase0"}, {"t12", "step"}, {"bruck1,bruck1/s3", "bruck1"}};
    for (const auto& nm : names)
        if (phase_name(nm.first) != nm.second) {
            std::fprintf(stderr, "FAIL phase_name(%s) = %s, want %s\n", nm.first, phase_name(nm.first).c_str(), nm.second);
            ++g_bad;
        }
    long plans = 0;
    const int modes[] = {MODE_ALLREDUCE,         MODE_REDUCE_SCATTER,    MODE_ALLGATHER,        MODE_MPICH_RING,
                         MODE_MPICH_RD,          MODE_MPICH_RSAG,        MODE_MPICH_RECEXCH,    MODE_MPICH_KRSAG,
                         MODE_MPICH_RMULT,       MODE_MPICH_RS_RADIX,    MODE_MPICH_RS_HALVING, MODE_MPICH_RS_DOUBLING,
                         MODE_MPICH_RS_PAIRWISE, MODE_INTRA_RS,          MODE_INTER_LINEAR,     MODE_INTRA_SCATTER};
    for (int mode : modes)
        for (int n = 1; n <= max_n; ++n)
            for (int b = 1; b <= n; ++b) {
                if (n % b && (mode <= MODE_REDUCE_SCATTER || is_phase(mode))) continue;
                for (int k = 2; k <= 9; ++k)
                    for (unsigned long long per : {1ull, 3ull, 64ull, 1000ull})
                        for (int slices : {1, 3, 8})
                            for (int sched : {0, 1, 2, 3, 4, 5, (int)SCHED_FLAT_1SHOT}) {
                                if (is_unpipelined(mode) && (sched != SCHED_FLAT || slices != 1))
                                    continue;
                                const unsigned long long count =
                                    mode == MODE_ALLREDUCE || is_mpich(mode) ? per * (unsigned long long)n : per;
                                const int aux = is_mpich(mode) ? (b % 2) : b;  // single_phase_recv for MPICH modes
                                std::vector<Plan> P;
                                for (int r = 0; r < n; ++r)
                                    P.push_back(is_mpich(mode) ? build_plan_mpich((Mode)mode, n, r, k, aux, count)
                                                               : build_plan((Mode)mode, n, r, k, b, count, slices, sched));
                                ++plans;
                                if (P[0].error) continue;
                                for (const Plan& p : P) (void)describe(p);
                                const size_t ns = P[0].steps.size();
                                for (const Plan& p : P)
                                    if (p.steps.size() != ns) fail("step count", mode, n, k, b, count, sched);
                                for (size_t s = 0; s < ns && !g_bad; ++s) {
                                    // sends r->q and receives at q from r: same sizes, same order
                                    std::map<std::pair<int, int>, std::vector<uint64_t>> snd, rcv;
                                    for (int r = 0; r < n; ++r) {
                                        const Step& st = P[r].steps[s];
                                        for (const Xfer& x : st.sends) {
                                            snd[{r, x.peer}].push_back(x.count);
                                            if (!in_bounds(P[r], x.ref, x.count)) fail("send bounds", mode, n, k, b, count, sched);
                                        }
                                        for (const Xfer& x : st.recvs) {
                                            rcv[{x.peer, r}].push_back(x.count);
                                            if (!in_bounds(P[r], x.ref, x.count)) fail("recv bounds", mode, n, k, b, count, sched);
                                        }
                                        for (const Coll& c : st.allgathers)
                                            if (!in_bounds(P[r], c.ref, c.count * (uint64_t)n))
                                                fail("allgather bounds", mode, n, k, b, count, sched);
                                        for (const LocalOp& op : st.post)
                                            if (!op_in_bounds(P[r], op)) fail("local op bounds", mode, n, k, b, count, sched);
                                    }
                                    if (snd != rcv) fail("unmatched messages", mode, n, k, b, count, sched);
                                }
                                for (const Plan& p : P)
                                    for (const LocalOp& op : p.pre)
                                        if (!op_in_bounds(p, op)) fail("pre op bounds", mode, n, k, b, count, sched);
                            }
            }
    std::printf("{\"plans\": %ld, \"failures\": %d}\n", plans, g_bad);
    return g_bad ? 1 : 0;
}
