// schedule.cpp -- radix/batch schedule compiler.  See schedule.hpp for the plan model
// and the block-major ACC layout.  Line citations are to
// Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp (the reduce-scatter file is
// line-for-line identical through phase 2).
#include "schedule.hpp"

#include <functional>
#include <tuple>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <sstream>

namespace chr {

int recexch_neighbors(int rank, int nranks, int k, Recexch* o) {
    *o = Recexch();
    if (k < 2 || nranks < 1) return 1;
    if (nranks < k) k = nranks > 2 ? nranks : 2;  // :19-21 (k is clamped, silently)
    o->k = k;
    int p_of_k = 1, log_p = 0;
    while (p_of_k <= nranks) {  // :23-28 largest power of k <= nranks
        p_of_k *= k;
        ++log_p;
    }
    p_of_k /= k;
    --log_p;
    o->p_of_k = p_of_k;
    o->step2_nphases = log_p;
    o->rem = nranks - p_of_k;
    o->T = (o->rem * k) / (k - 1);  // :47-49
    const int rem = o->rem, T = o->T;
    int newrank;
    if (rank < T) {  // :56-70: every k-th rank below T participates, the others fold into it
        if (rank % k != k - 1) {
            o->step1_sendto = std::min(rank + (k - 1 - rank % k), T);
            newrank = -1;
        } else {
            for (int i = 0; i < k - 1; ++i) o->step1_recvfrom.push_back(rank - i - 1);
            o->step1_nrecvs = k - 1;
            newrank = rank / k;
        }
    } else {  // :71-82: rank T absorbs the incomplete last group of non-participants
        newrank = rank - rem;
        if (rank == T && T >= 1 && (T - 1) % k != k - 1) {
            const int nsenders = (T - 1) % k + 1;
            for (int j = nsenders - 1; j >= 0; --j) o->step1_recvfrom.push_back(T - nsenders + j);
            o->step1_nrecvs = nsenders;
        }
    }
    if (o->step1_sendto != -1) return 0;
    // :84-134: phase-p neighbours flip base-k digit p of the step-2 rank.
    std::vector<int> digit(std::max(log_p, 1), 0);
    for (int t = newrank, d = 0; t != 0; t /= k) digit[d++] = t % k;
    o->step2_nbrs.assign(log_p, std::vector<int>());
    for (int phase = 0; phase < log_p; ++phase) {
        const int own = digit[phase];
        for (int v = 0; v < k; ++v) {
            if (v == own) continue;
            digit[phase] = v;
            int nbr = 0;
            for (int j = log_p - 1; j >= 0; --j) nbr = nbr * k + digit[j];
            o->step2_nbrs[phase].push_back(nbr < rem / (k - 1) ? nbr * k + (k - 1) : nbr + rem);
        }
        digit[phase] = own;
    }
    return 0;
}

static inline int step2_to_orig(int r, int rem, int k) {  // :152-161
    return r < rem / (k - 1) ? r * k + (k - 1) : r + rem;
}

void recexch_count_offset(int nranks, int max_phases, int k, std::vector<int>* count,
                          std::vector<int>* offset) {  // :163-198
    int p_of_k = 1;
    while (p_of_k <= nranks) p_of_k *= k;
    p_of_k /= k;
    const int rem = nranks - p_of_k, T = (rem * k) / (k - 1);
    count->assign((size_t)max_phases * nranks, 0);
    offset->assign((size_t)max_phases * nranks, 0);
    for (int phase = 0, kpp = 1; phase < max_phases; ++phase, kpp *= k) {
        for (int r = 0; r < nranks; ++r) {
            const int s2 = r < T ? r / k : r - rem;  // :140-149
            const int lo = (s2 / kpp) * kpp - 1, hi = lo + kpp;  // (lo, hi] in step-2 ranks
            const int olo = lo >= 0 ? step2_to_orig(lo, rem, k) : lo;
            const int ohi = step2_to_orig(hi, rem, k);
            (*count)[(size_t)phase * nranks + r] = ohi - olo;
            (*offset)[(size_t)phase * nranks + r] = olo + 1;
        }
    }
}

namespace {

LocalOp make_reduce(Ref dst, Ref acc, std::vector<Ref> ins, uint64_t n, int site) {
    LocalOp op;
    op.kind = L_REDUCE;
    op.dst = dst;
    op.acc = acc;
    op.ins = std::move(ins);
    op.count = n;
    op.site = site;
    return op;
}
LocalOp make_copy(Ref dst, Ref src, uint64_t n, int site) {
    LocalOp op;
    op.kind = L_COPY;
    op.dst = dst;
    op.acc = src;
    op.count = n;
    op.site = site;
    return op;
}
// rows x width elements, row r from src + r*spitch to dst + r*dpitch.
LocalOp make_copy2d(Ref dst, Ref src, uint64_t width, uint64_t rows, uint64_t dpitch, uint64_t spitch, int site) {
    if (rows <= 1 || (dpitch == width && spitch == width)) return make_copy(dst, src, width * rows, site);
    LocalOp op = make_copy(dst, src, width, site);
    op.kind = L_COPY2D;
    op.rows = rows;
    op.dpitch = dpitch;
    op.spitch = spitch;
    return op;
}

enum Logical { S_FOLD, S_PHASE, S_RETURN, S_LANE, S_DIST1, S_DIST2, S_SCATTER, S_BPHASE, S_BLANE, S_BDIST,
               S_RPHASE, S_RLANE, S_BCAST, S_AG, S_KSCAT };

// One element-slice [lo, lo+len) of every chunk, laid out slice-major in ACC:
// chunk position `pos` of slice p lives at acc_base + pos*len.
struct SliceCtx {
    uint64_t lo, len, acc_base, stage_base;
};

struct Builder {
    Plan& p;
    const Geometry& g;
    Mode mode;
    int n, me, node, lane;
    std::vector<Recexch> rx;
    std::vector<int> cnt, off;
    uint64_t stage_per_elem = 0;  // STAGE elements needed per element of slice length
    // SCHED_EXACT (unsliced): the reference's own phases 3-4 message for message.
    bool exact = false;
    int k_in = 0;            // k as passed: the reference sizes its allgather / scatter loops with it
    uint64_t ex_bc = 0;      // STAGE: bcast landing, one IRC per stage (tmp_results, :552-568)
    uint64_t ex_tmp = 0;     // STAGE: Bruck buffers (tmp_recvbuf, :582-756) / RS scatter buffer (:572-627)
    int nph_ag = 0;          // allgather / scatter phases (:274-277; RS :271-275), unclamped k
    // left-over k-Bruck (nu_count != 0, :645-756): my receives / sends per phase, in IRC units
    struct LeftMsg {
        bool send;
        int peer_lane;
        uint64_t off, cnt;
    };
    std::vector<std::vector<LeftMsg>> left;

    // Restatement of the left-over Bruck's bookkeeping (all_reduce_radix_batch.cpp:645-742):
    // active[] / send_sizes[][] evolve identically on every rank; each rank's receives land at
    // its running `received` offset, its sends always start at offset 0.
    void plan_left() {
        const int b = g.b, k = g.k, nu = g.nu;
        left.assign(nph_ag, {});
        if (!nu) return;
        std::vector<int> active(b);
        std::vector<std::vector<long long>> ss(nph_ag + 1, std::vector<long long>(b, 0));
        for (int l = 0; l < b; ++l) {
            active[l] = l < nu ? 0 : -1;
            ss[0][l] = l < nu ? 1 : 0;
        }
        long long delta = 1;
        for (int i = 0; i < nph_ag; ++i) {
            long long received = ss[i][lane];
            for (int j = 1; j < k; ++j) {
                if (delta * j >= b) {
                    for (int l = 0; l < b; ++l) {
                        if (active[l] == i) active[l] = i + 1;
                        ss[i + 1][l] += ss[i][l];
                    }
                    break;
                }
                const int isrc = (int)((lane + delta * j) % b);
                const int idst = (int)((b + (lane - delta * j) % b) % b);
                long long sz = std::min(ss[i][isrc], (long long)nu - received);
                if (active[isrc] == i && sz > 0) {
                    left[i].push_back({false, isrc, (uint64_t)received, (uint64_t)sz});
                    received += sz;
                }
                sz = std::min(ss[i][lane], (long long)nu - (ss[i][idst] + ss[i + 1][idst]));
                if (active[lane] == i && sz > 0) left[i].push_back({true, idst, 0, (uint64_t)sz});
                for (int l = 0; l < b; ++l) {
                    if (active[l] == i) {
                        const int t = (int)((b + (l - delta * j) % b) % b);
                        active[t] = active[t] != i ? i + 1 : i;
                        ss[i + 1][t] += ss[i][l];
                        if (j == k - 1) active[l] = i + 1;
                    }
                    if (j == k - 1) ss[i + 1][l] += ss[i][l];
                }
            }
            delta *= k;
        }
    }
    Ref tmp_stage(int stg) const {  // Bruck buffer of stage stg (stg == nstages: the left-over part)
        if (lane == 0 || (stg == g.nstages && lane >= g.nu)) return {BUF_RECV, (uint64_t)stg * g.b * g.irc};
        return {BUF_STAGE, ex_tmp + (uint64_t)stg * g.b * g.irc};
    }

    uint64_t chunk_pos(int N) const { return (uint64_t)g.P[N % g.b] + (uint64_t)(N / g.b); }
    // Region of lane blocks [o, o+c) of one slice, in elements.
    void region(const SliceCtx& c, int ph, int l, uint64_t* start, uint64_t* len) const {
        const int o = off[(size_t)ph * g.b + l], cn = cnt[(size_t)ph * g.b + l];
        const int e = std::min(o + cn, g.b);
        *start = c.acc_base + (uint64_t)g.P[o] * c.len;
        *len = o < e ? (uint64_t)(g.P[e] - g.P[o]) * c.len : 0;
    }
    const Recexch& x() const { return rx[lane]; }
    bool b1() const { return g.b == 1; }
    bool participant() const { return rx[lane].step1_sendto == -1; }

    // Pieces of the distribute scatter: [lo, lo+len) cut into n-1 pieces, 64-element aligned.
    void piece(const SliceCtx& c, int i, uint64_t* a, uint64_t* l) const {
        const uint64_t np = (uint64_t)(n - 1);
        auto cut = [&](uint64_t j) { return j == np ? c.len : (c.len * j / np) / 64 * 64; };
        *a = c.lo + cut((uint64_t)i);
        *l = cut((uint64_t)i + 1) - cut((uint64_t)i);
    }

    // Balanced evaluation (single-phase geometries): the slice of every chunk is cut into n
    // pieces, piece (j, Y) = index j*nnodes + Y, 64-element aligned; rank Y*b + j evaluates
    // piece (j, Y) of every chunk.  Lane j's sub-piece = pieces (j, 0..nnodes-1), contiguous.
    uint64_t bcut(const SliceCtx& c, uint64_t i) const {
        const uint64_t np = (uint64_t)n;
        return i >= np ? c.len : (c.len * i / np) / 64 * 64;
    }
    void bpiece(const SliceCtx& c, int j, int Y, uint64_t* a, uint64_t* l) const {
        const uint64_t i = (uint64_t)j * g.nnodes + (uint64_t)Y;
        *a = bcut(c, i);
        *l = bcut(c, i + 1) - *a;
    }
    void bsub(const SliceCtx& c, int j, uint64_t* a, uint64_t* l) const {
        *a = bcut(c, (uint64_t)j * g.nnodes);
        *l = bcut(c, (uint64_t)(j + 1) * g.nnodes) - *a;
    }
    uint64_t acc_of(const SliceCtx& c, int N) const { return c.acc_base + chunk_pos(N) * c.len; }

    void emit(Logical kind, int ph, const SliceCtx& c, Step& s) {
        const uint64_t irc = g.irc, recvcount = g.recvcount;
        const uint64_t slice_total = (uint64_t)g.nnodes * c.len;  // this slice of every chunk
        switch (kind) {
        case S_FOLD: {  // :315-335
            if (!participant()) {
                s.sends.push_back({x().step1_sendto + g.b * node, {BUF_ACC, c.acc_base}, slice_total});
            } else if (x().step1_nrecvs > 0) {
                std::vector<Ref> ins;
                for (int i = 0; i < x().step1_nrecvs; ++i) {
                    const Ref slot{BUF_STAGE, c.stage_base + (uint64_t)i * slice_total};
                    s.recvs.push_back({x().step1_recvfrom[i] + g.b * node, slot, slice_total});
                    ins.push_back(slot);
                }
                s.post.push_back(make_reduce({BUF_ACC, c.acc_base}, {BUF_ACC, c.acc_base}, ins, slice_total, 332));
            }
            break;
        }
        case S_PHASE: {  // :339-478
            if (!participant()) break;
            uint64_t my_start, my_len;
            region(c, ph, lane, &my_start, &my_len);
            std::vector<Ref> ins;
            for (int i = 0; i < g.k - 1; ++i) {
                const int dst = x().step2_nbrs[ph][i];
                uint64_t st, len;
                region(c, ph, dst, &st, &len);
                if (len) s.sends.push_back({dst + g.b * node, {BUF_ACC, st}, len});  // :353 / :425
                if (my_len) {
                    const Ref slot{BUF_STAGE, c.stage_base + (uint64_t)i * my_len};
                    s.recvs.push_back({dst + g.b * node, slot, my_len});  // :360 / :442
                    ins.push_back(slot);
                }
            }
            if (my_len) s.post.push_back(make_reduce({BUF_ACC, my_start}, {BUF_ACC, my_start}, ins, my_len, 364));
            break;
        }
        case S_RETURN: {  // :378-385, :465-473
            if (!participant()) {
                const uint64_t len = (uint64_t)g.S[lane] * c.len;
                if (len)
                    s.recvs.push_back({x().step1_sendto + g.b * node, {BUF_ACC, c.acc_base + (uint64_t)g.P[lane] * c.len}, len});
            } else {
                for (int i = 0; i < x().step1_nrecvs; ++i) {
                    const int q = x().step1_recvfrom[i];
                    const uint64_t len = (uint64_t)g.S[q] * c.len;
                    if (len) s.sends.push_back({q + g.b * node, {BUF_ACC, c.acc_base + (uint64_t)g.P[q] * c.len}, len});
                }
            }
            break;
        }
        case S_LANE: {  // :498-539
            for (int i = 0; i < g.S[lane]; ++i) {
                const int R = i * g.b + lane;  // root node of iteration i (:502)
                const uint64_t mine = c.acc_base + ((uint64_t)g.P[lane] + i) * c.len;
                if (node != R) {
                    s.sends.push_back({R * g.b + lane, {BUF_ACC, mine}, c.len});  // :534
                    continue;
                }
                std::vector<Ref> ins;
                for (int X = 0, slot = 0; X < g.nnodes; ++X) {  // stage order (:523-530)
                    if (X == R) continue;
                    const Ref r{BUF_STAGE, c.stage_base + (uint64_t)slot * c.len};
                    s.recvs.push_back({X * g.b + lane, r, c.len});  // :517
                    ins.push_back(r);
                    ++slot;
                }
                if (mode == MODE_ALLREDUCE) {
                    // reduce straight into the chunk's final place in recvbuf
                    s.post.push_back(make_reduce({BUF_RECV, (uint64_t)R * irc + c.lo}, {BUF_ACC, mine}, ins, c.len, 529));
                } else if (exact) {
                    s.post.push_back(make_reduce({BUF_ACC, mine}, {BUF_ACC, mine}, ins, c.len, 552));
                    // root re-layout (reduce_scatter_radix_batch.cpp:572-579): block real_slot of the
                    // chunk to normalized slot (real_slot - root_local) mod b; root_local == lane here
                    const uint64_t rc = recvcount;
                    const Ref t{BUF_STAGE, ex_tmp};
                    s.post.push_back(make_copy(t, {BUF_ACC, mine + (uint64_t)lane * rc}, (uint64_t)(g.b - lane) * rc, 575));
                    if (lane)
                        s.post.push_back(make_copy({BUF_STAGE, ex_tmp + (uint64_t)(g.b - lane) * rc}, {BUF_ACC, mine},
                                                   (uint64_t)lane * rc, 575));
                    if (nph_ag == 0) s.post.push_back(make_copy({BUF_RECV, 0}, t, rc, 625));  // b == 1: shift 0
                } else {
                    s.post.push_back(make_reduce({BUF_ACC, mine}, {BUF_ACC, mine}, ins, c.len, 552));
                    // own sub-block (reduce_scatter_radix_batch.cpp:572-579, :625-627)
                    const uint64_t a = std::max(c.lo, (uint64_t)lane * recvcount);
                    const uint64_t e = std::min(c.lo + c.len, (uint64_t)(lane + 1) * recvcount);
                    if (a < e)
                        s.post.push_back(make_copy({BUF_RECV, a - (uint64_t)lane * recvcount}, {BUF_ACC, mine + (a - c.lo)},
                                                   e - a, 625));
                }
            }
            break;
        }
        case S_DIST1:  // allreduce phases 3-4 (:552-756) as a link-balanced scatter ...
        case S_DIST2: {  // ... + forward: every ordered pair of GPUs carries ~1/(n-1) of each chunk
            for (int N = 0; N < g.nnodes; ++N) {
                const int owner = N * g.b + N % g.b;
                const uint64_t base = (uint64_t)N * irc;
                if (n == 2) {  // one peer: the whole slice, single hop
                    if (kind == S_DIST2) continue;
                    if (me == owner) s.sends.push_back({1 - me, {BUF_RECV, base + c.lo}, c.len});
                    else s.recvs.push_back({owner, {BUF_RECV, base + c.lo}, c.len});
                    continue;
                }
                for (int Y = 0; Y < n; ++Y) {
                    if (Y == owner) continue;
                    uint64_t a, l;
                    piece(c, Y < owner ? Y : Y - 1, &a, &l);
                    if (!l) continue;
                    if (kind == S_DIST1) {
                        if (me == owner) s.sends.push_back({Y, {BUF_RECV, base + a}, l});
                        else if (me == Y) s.recvs.push_back({owner, {BUF_RECV, base + a}, l});
                    } else {
                        for (int Z = 0; Z < n; ++Z) {
                            if (Z == owner || Z == Y) continue;
                            if (me == Y) s.sends.push_back({Z, {BUF_RECV, base + a}, l});
                            else if (me == Z) s.recvs.push_back({Y, {BUF_RECV, base + a}, l});
                        }
                    }
                }
            }
            break;
        }
        case S_BPHASE: {
            // Phase 1 of chunk N is, in the reference, evaluated at lane L = N % b of every node:
            // acc = L's data, then step2_nbrs[0][0..k-2] of L in order (:343-364).  Here lane j
            // evaluates that same expression on its sub-piece of the chunk: it receives the
            // other members' sub-piece j and reduces in L's operand order.
            uint64_t a, len;
            bsub(c, lane, &a, &len);
            if (b1()) break;
            for (int m = 0; m < g.b; ++m) {  // my sub-piece of m's lane to member m
                if (m == lane) continue;
                uint64_t ma, ml;
                bsub(c, m, &ma, &ml);
                for (int N = 0; N < g.nnodes && ml; ++N)
                    s.sends.push_back({node * g.b + m, {BUF_ACC, acc_of(c, N) + ma}, ml});
            }
            if (!len) break;
            for (int N = 0; N < g.nnodes; ++N) {
                auto src = [&](int m) -> Ref {  // member m's sub-piece `lane` of chunk N, here
                    if (m == lane) return {BUF_ACC, acc_of(c, N) + a};
                    const int slot = (m < lane ? m : m - 1) * g.nnodes + N;
                    return {BUF_STAGE, c.stage_base + (uint64_t)slot * c.len + a};
                };
                for (int m = 0; m < g.b; ++m)
                    if (m != lane) s.recvs.push_back({node * g.b + m, src(m), len});
                const int L = N % g.b;
                std::vector<Ref> ins;
                for (int i = 0; i < g.k - 1; ++i) ins.push_back(src(rx[L].step2_nbrs[0][i]));
                s.post.push_back(make_reduce({BUF_ACC, acc_of(c, N) + a}, src(L), ins, len, 364));
            }
            break;
        }
        case S_BLANE: {
            // Phase 2 of chunk N is evaluated at root node N in the reference: acc = node N's
            // phase-1 value, then the other nodes' in stage order (:498-539).  Rank (Y, j)
            // evaluates it on piece (j, Y), writing straight into recvbuf.
            uint64_t a, len;
            bpiece(c, lane, node, &a, &len);
            for (int X = 0; X < g.nnodes; ++X) {  // my piece (lane, X) of every chunk to node X
                if (X == node) continue;
                uint64_t xa, xl;
                bpiece(c, lane, X, &xa, &xl);
                for (int N = 0; N < g.nnodes && xl; ++N)
                    s.sends.push_back({X * g.b + lane, {BUF_ACC, acc_of(c, N) + xa}, xl});
            }
            if (!len) break;
            for (int N = 0; N < g.nnodes; ++N) {
                auto src = [&](int X) -> Ref {
                    if (X == node) return {BUF_ACC, acc_of(c, N) + a};
                    const int slot = (X < node ? X : X - 1) * g.nnodes + N;
                    return {BUF_STAGE, c.stage_base + (uint64_t)slot * c.len + a};
                };
                for (int X = 0; X < g.nnodes; ++X)
                    if (X != node) s.recvs.push_back({X * g.b + lane, src(X), len});
                std::vector<Ref> ins;
                for (int X = 0; X < g.nnodes; ++X)
                    if (X != N) ins.push_back(src(X));
                s.post.push_back(make_reduce({BUF_RECV, (uint64_t)N * irc + c.lo + a}, src(N), ins, len, 529));
            }
            break;
        }
        case S_BDIST: {  // allgather of the pieces: every rank's piece of every chunk to every rank
            uint64_t a, len;
            bpiece(c, lane, node, &a, &len);
            for (int q = 0; q < n; ++q) {
                if (q == me) continue;
                uint64_t qa, ql;
                bpiece(c, q % g.b, q / g.b, &qa, &ql);
                for (int N = 0; N < g.nnodes; ++N) {
                    const uint64_t base = (uint64_t)N * irc + c.lo;
                    if (len) s.sends.push_back({q, {BUF_RECV, base + a}, len});
                    if (ql) s.recvs.push_back({q, {BUF_RECV, base + qa}, ql});
                }
            }
            break;
        }
        case S_RPHASE: {
            // Balanced reduce-scatter: the output block of rank (Y, j) is sub-block j (recvcount
            // elements of the IRC chunk) of chunk Y.  Phase 1 of every chunk N: lane j evaluates
            // sub-block j in the owner lane's order (as S_BPHASE, pieces = recvcount blocks).
            const uint64_t a = std::max(c.lo, (uint64_t)lane * recvcount);
            const uint64_t e = std::min(c.lo + c.len, (uint64_t)(lane + 1) * recvcount);
            for (int m = 0; m < g.b; ++m) {
                if (m == lane) continue;
                const uint64_t ma = std::max(c.lo, (uint64_t)m * recvcount);
                const uint64_t me_ = std::min(c.lo + c.len, (uint64_t)(m + 1) * recvcount);
                for (int N = 0; N < g.nnodes && ma < me_; ++N)
                    s.sends.push_back({node * g.b + m, {BUF_ACC, acc_of(c, N) + (ma - c.lo)}, me_ - ma});
            }
            if (a >= e) break;
            const uint64_t off = a - c.lo, len = e - a;
            for (int N = 0; N < g.nnodes; ++N) {
                auto src = [&](int m) -> Ref {
                    if (m == lane) return {BUF_ACC, acc_of(c, N) + off};
                    const int slot = (m < lane ? m : m - 1) * g.nnodes + N;
                    return {BUF_STAGE, c.stage_base + (uint64_t)slot * c.len + off};
                };
                for (int m = 0; m < g.b; ++m)
                    if (m != lane) s.recvs.push_back({node * g.b + m, src(m), len});
                const int L = N % g.b;
                std::vector<Ref> ins;
                for (int i = 0; i < g.k - 1; ++i) ins.push_back(src(rx[L].step2_nbrs[0][i]));
                s.post.push_back(make_reduce({BUF_ACC, acc_of(c, N) + off}, src(L), ins, len, 366));
            }
            break;
        }
        case S_RLANE: {
            // Phase 2 of chunk N, sub-block j: at rank (N, j), root-node order (:498-552), written
            // straight into recvbuf; every other node sends its sub-block j of chunk N there.
            const uint64_t a = std::max(c.lo, (uint64_t)lane * recvcount);
            const uint64_t e = std::min(c.lo + c.len, (uint64_t)(lane + 1) * recvcount);
            if (a >= e) break;
            const uint64_t off = a - c.lo, len = e - a;
            for (int N = 0; N < g.nnodes; ++N)
                if (N != node) s.sends.push_back({N * g.b + lane, {BUF_ACC, acc_of(c, N) + off}, len});
            auto src = [&](int X) -> Ref {  // node X's phase-1 value of chunk `node`, sub-block lane
                if (X == node) return {BUF_ACC, acc_of(c, node) + off};
                const int slot = X < node ? X : X - 1;
                return {BUF_STAGE, c.stage_base + (uint64_t)slot * c.len + off};
            };
            std::vector<Ref> ins;
            for (int X = 0; X < g.nnodes; ++X) {
                if (X == node) continue;
                s.recvs.push_back({X * g.b + lane, src(X), len});
                ins.push_back(src(X));
            }
            s.post.push_back(make_reduce({BUF_RECV, a - (uint64_t)lane * recvcount}, src(node), ins, len, 552));
            break;
        }
        case S_BCAST: {  // allreduce allgather phase 1 (:552-568): lane root -> same lane of every node
            for (int stg = 0; stg * g.b < g.nnodes; ++stg) {
                const int N = stg * g.b + lane;  // chunk of my lane in this stage
                if (N >= g.nnodes) continue;
                const Ref bc{BUF_STAGE, ex_bc + (uint64_t)stg * irc};
                if (node == N) {
                    s.post.push_back(make_copy(bc, {BUF_RECV, (uint64_t)N * irc}, irc, 558));
                    for (int j = 0; j < g.nnodes; ++j)
                        if (j != node) s.sends.push_back({j * g.b + lane, {BUF_RECV, (uint64_t)N * irc}, irc});  // :564
                } else {
                    s.recvs.push_back({N * g.b + lane, bc, irc});  // :555
                }
            }
            // each stage's own chunk to slot 0 of its Bruck buffer (:591, :645-647)
            for (int stg = 0; stg < g.nstages; ++stg)
                s.post.push_back(make_copy(tmp_stage(stg), {BUF_STAGE, ex_bc + (uint64_t)stg * irc}, irc, 591));
            if (g.nu && lane < g.nu)
                s.post.push_back(make_copy(tmp_stage(g.nstages), {BUF_STAGE, ex_bc + (uint64_t)g.nstages * irc}, irc, 646));
            break;
        }
        case S_AG: {  // allreduce allgather phase 2 (:587-756): k-port Bruck inside the node, phase ph
            const int b = g.b, k = g.k;
            long long delta = 1;
            for (int i = 0; i < ph; ++i) delta *= k;
            const bool last = ph == nph_ag - 1;
            const int p_of_k = x().p_of_k;
            for (int stg = 0; stg < g.nstages; ++stg) {  // full stages (:587-640)
                const Ref t = tmp_stage(stg);
                for (int j = 1; j < k; ++j) {
                    if (delta * j >= b) break;
                    const int dst = (int)((b + (lane - delta * j) % b) % b) + node * b;
                    const int src = (int)((lane + delta * j) % b) + node * b;
                    long long cnt = delta;  // in IRC units (:604-617)
                    if (last && p_of_k != b) {
                        const long long left_cnt = b - delta * j;
                        cnt = j == k - 1 ? left_cnt : std::min(cnt, left_cnt);
                    }
                    s.recvs.push_back({src, {t.buf, t.off + (uint64_t)(j * delta) * irc}, (uint64_t)cnt * irc});  // :620
                    s.sends.push_back({dst, t, (uint64_t)cnt * irc});                                           // :623
                }
                if (last && lane != 0) {  // rotation into recvbuf (:627-637)
                    const uint64_t base = (uint64_t)stg * b * irc;
                    s.post.push_back(make_copy({BUF_RECV, base}, {t.buf, t.off + (uint64_t)(b - lane) * irc},
                                               (uint64_t)lane * irc, 629));
                    s.post.push_back(make_copy({BUF_RECV, base + (uint64_t)lane * irc}, t, (uint64_t)(b - lane) * irc, 633));
                }
            }
            if (g.nu) {  // left-over chunks (:645-756)
                const Ref t = tmp_stage(g.nstages);
                for (const LeftMsg& m : left[ph]) {
                    if (m.send) s.sends.push_back({node * b + m.peer_lane, {t.buf, t.off + m.off * irc}, m.cnt * irc});
                    else s.recvs.push_back({node * b + m.peer_lane, {t.buf, t.off + m.off * irc}, m.cnt * irc});
                }
                if (last && lane != 0 && lane < g.nu) {  // :745-754
                    const uint64_t base = (uint64_t)g.nstages * b * irc;
                    s.post.push_back(make_copy({BUF_RECV, base}, {t.buf, t.off + (uint64_t)(g.nu - lane) * irc},
                                               (uint64_t)lane * irc, 747));
                    s.post.push_back(make_copy({BUF_RECV, base + (uint64_t)lane * irc}, t, (uint64_t)(g.nu - lane) * irc,
                                               751));
                }
            }
            break;
        }
        case S_KSCAT: {  // reduce-scatter k-nomial scatter inside the node (:584-627), phase ph
            const int b = g.b, k = g.k;
            const uint64_t rc = recvcount;
            const int root_local = node % b, shift = (lane - root_local + b) % b;
            // delta: k_in^(nph-1) in the first phase, then divided by the clamped k (:271-275, :621)
            long long delta = 1;
            for (int i = 0; i < nph_ag; ++i) delta *= k_in;
            delta /= k_in;
            for (int q = nph_ag - 1; q > ph; --q) delta = q > 0 ? delta / k : delta;
            const long long group = delta * k, gstart = (shift / group) * group;
            const long long bend = std::min<long long>(gstart + group, b), offs = shift - gstart;
            if (offs == 0) {
                for (int j = 1; j < k; ++j) {
                    const long long child = gstart + j * delta;
                    if (child >= bend) break;
                    const long long sub = std::min(delta, bend - child);
                    const int dst = node * b + (int)((child + root_local) % b);
                    s.sends.push_back({dst, {BUF_STAGE, ex_tmp + (uint64_t)child * rc}, (uint64_t)sub * rc});  // :603
                }
            } else if (offs % delta == 0 && offs < group) {
                const int src = node * b + (int)((gstart + root_local) % b);
                const long long sub = std::min<long long>(delta, bend - shift);
                s.recvs.push_back({src, {BUF_STAGE, ex_tmp + (uint64_t)shift * rc}, (uint64_t)sub * rc});  // :615
            }
            if (ph == 0) s.post.push_back(make_copy({BUF_RECV, 0}, {BUF_STAGE, ex_tmp + (uint64_t)shift * rc}, rc, 625));
            break;
        }
        case S_SCATTER: {  // reduce-scatter phase 3 (:572-627): owner -> every lane, direct
            const int owner = node * g.b + node % g.b;
            if (me == owner) {
                const uint64_t mine = c.acc_base + ((uint64_t)g.P[lane] + node / g.b) * c.len;
                for (int j = 0; j < g.b; ++j) {
                    if (j == lane) continue;
                    const uint64_t a = std::max(c.lo, (uint64_t)j * recvcount);
                    const uint64_t e = std::min(c.lo + c.len, (uint64_t)(j + 1) * recvcount);
                    if (a < e) s.sends.push_back({node * g.b + j, {BUF_ACC, mine + (a - c.lo)}, e - a});
                }
            } else {
                const uint64_t a = std::max(c.lo, (uint64_t)lane * recvcount);
                const uint64_t e = std::min(c.lo + c.len, (uint64_t)(lane + 1) * recvcount);
                if (a < e) s.recvs.push_back({owner, {BUF_RECV, a - (uint64_t)lane * recvcount}, e - a});
            }
            break;
        }
        }
    }
};

}  // namespace

int auto_slices(uint64_t irc_bytes) {
    // Pipeline depth: ~64 MiB per slice message, at most 8 slices, none below 32 MiB.
    const uint64_t s = irc_bytes / ((uint64_t)64 << 20);
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(8, s));
}

Plan build_plan_flat(Mode mode, int n, int me, int k, int b, const Geometry& g, int slices, bool coll_ag = false,
                     bool merge = true, bool oneshot = false);
static Plan build_plan_impl(Mode mode, int n, int me, int k_in, int b, uint64_t count, int slices, int sched);

// The fused kernel takes at most kPlanFanIn inputs per pass (kMaxFanIn, reduce_kernels.hip)
// and chains longer folds through `dst`.  A later input that aliases `dst` -- the own leaf
// read in place from SEND (== RECV under MPI_IN_PLACE), or recvbuf itself in MPICH's
// running-value chains -- would then be read after it was overwritten.  Such reductions are
// split: the leading inputs fold into a STAGE scratch region, the last <= kPlanFanIn inputs
// are folded from there into `dst` in one pass.  Same association, same bits.
static constexpr int kPlanFanIn = 8;

static bool may_alias(const Ref& a, uint64_t na, const Ref& b, uint64_t nb) {
    const bool io = (a.buf == BUF_SEND && b.buf == BUF_RECV) || (a.buf == BUF_RECV && b.buf == BUF_SEND);
    if (io) return true;  // in place: SEND is RECV (offsets differ for allgather / reduce-scatter)
    return a.buf == b.buf && a.off < b.off + nb && b.off < a.off + na;
}

static void split_wide_reductions(Plan& p) {
    const uint64_t scratch = p.stage_elems;
    uint64_t need = 0;
    auto fix = [&](std::vector<LocalOp>& ops) {
        std::vector<LocalOp> out;
        for (LocalOp& op : ops) {
            const size_t m = op.ins.size();
            bool alias = false;
            if (op.kind == L_REDUCE && m > (size_t)kPlanFanIn)
                for (size_t j = kPlanFanIn; j < m; ++j) alias = alias || may_alias(op.ins[j], op.count, op.dst, op.count);
            if (!alias) {
                out.push_back(std::move(op));
                continue;
            }
            const size_t r = (m - 1) % kPlanFanIn + 1;  // inputs of the final pass
            LocalOp a = op, z = op;
            a.dst = {BUF_STAGE, scratch};
            a.ins.assign(op.ins.begin(), op.ins.end() - (long)r);
            z.acc = {BUF_STAGE, scratch};
            z.ins.assign(op.ins.end() - (long)r, op.ins.end());
            need = std::max(need, op.count);
            out.push_back(std::move(a));
            out.push_back(std::move(z));
        }
        ops.swap(out);
    };
    fix(p.pre);
    for (Step& st : p.steps) fix(st.post);
    p.stage_elems += need;
}

// Dependencies for two-stream execution (transfers on the comm stream, local ops on the
// compute stream).  Regions are compared in one address space for SEND and RECV (they are the
// same memory under MPI_IN_PLACE; a false conflict only costs overlap, never correctness).
struct Region {
    uint8_t buf;
    uint64_t lo, hi;
};
static uint8_t space(uint8_t b) { return b == BUF_SEND ? (uint8_t)BUF_RECV : b; }
static bool overlap(const Region& a, const Region& b) {
    return space(a.buf) == space(b.buf) && a.lo < b.hi && b.lo < a.hi;
}
static void op_regions(const LocalOp& op, std::vector<Region>* rd, std::vector<Region>* wr) {
    if (op.kind == L_COPY2D) {
        for (uint64_t r = 0; r < op.rows; ++r) {
            rd->push_back({op.acc.buf, op.acc.off + r * op.spitch, op.acc.off + r * op.spitch + op.count});
            wr->push_back({op.dst.buf, op.dst.off + r * op.dpitch, op.dst.off + r * op.dpitch + op.count});
        }
        return;
    }
    rd->push_back({op.acc.buf, op.acc.off, op.acc.off + op.count});
    for (const Ref& x : op.ins) rd->push_back({x.buf, x.off, x.off + op.count});
    wr->push_back({op.dst.buf, op.dst.off, op.dst.off + op.count});
}
static bool conflict(const std::vector<Region>& wr_a, const std::vector<Region>& rd_a, const std::vector<Region>& rd_b,
                     const std::vector<Region>& wr_b) {
    for (const Region& a : wr_a) {
        for (const Region& b : rd_b)
            if (overlap(a, b)) return true;  // RAW
        for (const Region& b : wr_b)
            if (overlap(a, b)) return true;  // WAW
    }
    for (const Region& a : rd_a)
        for (const Region& b : wr_b)
            if (overlap(a, b)) return true;  // WAR
    return false;
}

static void analyze_deps(Plan& p) {
    const size_t ns = p.steps.size();
    std::vector<std::vector<Region>> prd(ns), pwr(ns);
    for (size_t u = 0; u < ns; ++u)
        for (const LocalOp& op : p.steps[u].post) op_regions(op, &prd[u], &pwr[u]);
    for (size_t t = 0; t < ns; ++t) {
        std::vector<Region> crd, cwr;  // transfers: sends read, receives write
        for (const Xfer& x : p.steps[t].sends) crd.push_back({x.ref.buf, x.ref.off, x.ref.off + x.count});
        for (const Xfer& x : p.steps[t].recvs) cwr.push_back({x.ref.buf, x.ref.off, x.ref.off + x.count});
        for (const Coll& x : p.steps[t].allgathers) {
            crd.push_back({x.ref.buf, x.ref.off + (uint64_t)p.rank * x.count, x.ref.off + (uint64_t)(p.rank + 1) * x.count});
            cwr.push_back({x.ref.buf, x.ref.off, x.ref.off + (uint64_t)p.g.nranks * x.count});
        }
        Step& st = p.steps[t];
        st.comm_deps.clear();
        for (size_t u = 0; u < t; ++u) {
            if (pwr[u].empty() && prd[u].empty()) continue;
            if (conflict(pwr[u], prd[u], crd, cwr)) st.comm_deps.push_back((int)u);
        }
        st.comm_wait = st.comm_deps.empty() ? -1 : st.comm_deps.back();
    }
}

Plan build_plan(Mode mode, int n, int me, int k_in, int b, uint64_t count, int slices, int sched, bool commutative) {
    Plan p = is_mpich(mode) ? build_plan_mpich(mode, n, me, k_in, b, count, commutative)
                            : build_plan_impl(mode, n, me, k_in, b, count, slices, sched);
    if (!p.error) {
        split_wide_reductions(p);
        analyze_deps(p);
    }
    return p;
}

static Plan build_plan_impl(Mode mode, int n, int me, int k_in, int b, uint64_t count, int slices, int sched) {
    const bool balance = sched == SCHED_BALANCED;
    if (is_mpich(mode)) return build_plan_mpich(mode, n, me, k_in, b, count);
    if (mode == MODE_ALLGATHER) return build_plan_allgather(n, me, k_in, b, count);
    if (is_phase(mode)) return build_plan_phase(mode, n, me, k_in, b, count);
    Plan p;
    p.mode = mode;
    p.rank = me;
    if (n < 1 || b < 1 || k_in < 2 || me < 0 || me >= n || b > n || slices < 1) {
        p.error = 1;  // CHR_ERR_INVALID_ARG
        return p;
    }
    if (n % b != 0) {
        p.error = 3;  // CHR_ERR_BATCH_NOT_DIVISOR (reference: MPI_Irecv invalid-rank abort)
        return p;
    }
    uint64_t recvcount = count;
    if (mode == MODE_ALLREDUCE) {
        if (count % (uint64_t)n != 0) {
            p.error = 2;  // CHR_ERR_COUNT_NOT_DIVISIBLE (reference: silent wrong tail, :239)
            return p;
        }
        recvcount = count / (uint64_t)n;
    }
    Geometry& g = p.g;
    g.nranks = n;
    g.b = b;
    g.nnodes = n / b;  // :241-244
    g.nstages = g.nnodes / b;
    g.nu = g.nnodes % b;  // :258
    g.recvcount = recvcount;
    g.irc = recvcount * (uint64_t)b;  // :249
    g.total = recvcount * (uint64_t)n;  // :254
    g.S.assign(b, 0);
    g.P.assign(b + 1, 0);
    for (int j = 0; j < b; ++j) {
        g.S[j] = g.nstages + (j < g.nu ? 1 : 0);
        g.P[j + 1] = g.P[j] + g.S[j];
    }
    Builder B{p, g, mode, n, me, me / b, me % b, {}, {}, {}};
    B.rx.resize(b);
    for (int l = 0; l < b; ++l)
        if (recexch_neighbors(l, b, k_in, &B.rx[l])) {
            p.error = 1;
            return p;
        }
    g.k = B.rx[0].k;
    g.nph = B.rx[0].step2_nphases;
    recexch_count_offset(b, g.nph, g.k, &B.cnt, &B.off);

    p.send_elems = g.total;
    p.recv_elems = mode == MODE_ALLREDUCE ? g.total : recvcount;
    p.acc_elems = g.total;
    if (g.total == 0) return p;
    if ((sched == SCHED_FLAT || sched == SCHED_FLAT_AG || sched == SCHED_FLAT_SEQ || sched == SCHED_FLAT_1SHOT) &&
        n > 1) {
        Plan f = build_plan_flat(mode, n, me, k_in, b, g, slices, sched == SCHED_FLAT_AG, sched != SCHED_FLAT_SEQ,
                                 sched == SCHED_FLAT_1SHOT && mode == MODE_ALLREDUCE);
        if (!f.error) return f;
    }

    // Logical steps, identical on every rank (so super-step numbering agrees globally).
    std::vector<std::pair<Logical, int>> L;
    const bool folds = B.rx[0].rem > 0;  // non-participants exist in every group
    // Balanced evaluation: one recexch phase (k == b after clamping) or none (b == 1), no
    // fold.  Same expressions, evaluated on 1/n of every chunk at every rank (allreduce), or
    // on exactly the rank's own output block (reduce-scatter).
    p.balanced = balance && n > 1 && !folds && g.nph <= 1;
    p.sched = p.balanced ? SCHED_BALANCED : sched == SCHED_EXACT ? SCHED_EXACT : SCHED_REFERENCE;
    B.exact = sched == SCHED_EXACT;
    if (B.exact) {
        B.k_in = k_in;
        for (int t = b - 1; t > 0; t /= k_in) ++B.nph_ag;  // :274-277 / RS :271-275 (k before clamping)
        slices = 1;  // the reference's messages are whole chunks
        if (mode == MODE_ALLREDUCE) B.plan_left();
    }
    if (p.balanced && mode == MODE_ALLREDUCE) {
        if (g.nph == 1) L.push_back({S_BPHASE, 0});
        L.push_back({S_BLANE, 0});
        L.push_back({S_BDIST, 0});
    } else if (p.balanced) {  // reduce-scatter: each rank evaluates exactly its own block
        if (g.nph == 1) L.push_back({S_RPHASE, 0});
        L.push_back({S_RLANE, 0});
    }
    if (folds) L.push_back({S_FOLD, 0});
    if (!p.balanced) {
        for (int ph = g.nph - 1; ph >= 0; --ph) L.push_back({S_PHASE, ph});
        if (folds) L.push_back({S_RETURN, 0});
        L.push_back({S_LANE, 0});
        if (B.exact && mode == MODE_ALLREDUCE) {  // bcast + k-port Bruck (:552-756)
            if (n > 1) {
                L.push_back({S_BCAST, 0});
                for (int ph = 0; ph < B.nph_ag; ++ph) L.push_back({S_AG, ph});
            }
        } else if (B.exact) {  // k-nomial scatter, highest phase first (:584-622)
            for (int ph = B.nph_ag - 1; ph >= 0; --ph) L.push_back({S_KSCAT, ph});
        } else if (mode == MODE_ALLREDUCE) {
            if (n > 1) L.push_back({S_DIST1, 0});
            if (n > 2) L.push_back({S_DIST2, 0});
        } else if (b > 1) {
            L.push_back({S_SCATTER, 0});
        }
    }

    // STAGE per element of slice length (max over the steps this rank can receive in).
    uint64_t max_region_chunks = 0;
    for (int ph = 0; ph < g.nph; ++ph)
        for (int l = 0; l < b; ++l) {
            const int o = B.off[(size_t)ph * b + l], e = std::min(o + B.cnt[(size_t)ph * b + l], b);
            if (o < e) max_region_chunks = std::max<uint64_t>(max_region_chunks, (uint64_t)(g.P[e] - g.P[o]));
        }
    int max_nrecvs = 0;
    for (int l = 0; l < b; ++l) max_nrecvs = std::max(max_nrecvs, B.rx[l].step1_nrecvs);
    B.stage_per_elem = std::max<uint64_t>({(uint64_t)max_nrecvs * g.nnodes, (uint64_t)(g.k - 1) * max_region_chunks,
                                           (uint64_t)(g.nnodes - 1), 1});
    if (p.balanced)  // (b-1) members' or (nnodes-1) nodes' pieces of every chunk
        B.stage_per_elem = std::max<uint64_t>({(uint64_t)(b - 1) * g.nnodes, (uint64_t)(g.nnodes - 1) * g.nnodes, 1});

    // Element slices of every chunk (pipeline depth), 256-element aligned bounds.
    const uint64_t G = 256;
    int P = slices;
    if ((uint64_t)P > g.irc / G) P = (int)std::max<uint64_t>(1, g.irc / G);
    p.slices = P;
    std::vector<SliceCtx> sl(P);
    for (int s = 0; s < P; ++s) {
        const uint64_t lo = s == 0 ? 0 : (g.irc * s / P) / G * G;
        const uint64_t hi = s == P - 1 ? g.irc : (g.irc * (s + 1) / P) / G * G;
        sl[s] = {lo, hi - lo, lo * (uint64_t)g.nnodes, lo * B.stage_per_elem};
    }
    p.stage_elems = g.irc * B.stage_per_elem;
    if (B.exact) {  // bcast landing + Bruck buffers (allreduce) / scatter buffer (reduce-scatter)
        B.ex_bc = p.stage_elems;
        B.ex_tmp = B.ex_bc + (mode == MODE_ALLREDUCE ? (uint64_t)(g.nstages + 1) * g.irc : 0);
        p.stage_elems = B.ex_tmp + (mode == MODE_ALLREDUCE ? g.total : g.irc);
    }

    // pre: SEND -> ACC, slice-major and block-major (:306-312 copy, re-laid out)
    for (const SliceCtx& c : sl) {
        int N = 0;
        while (N < g.nnodes) {
            int e = N + 1;
            while (e < g.nnodes && B.chunk_pos(e) == B.chunk_pos(e - 1) + 1) ++e;
            p.pre.push_back(make_copy2d({BUF_ACC, c.acc_base + B.chunk_pos(N) * c.len}, {BUF_SEND, (uint64_t)N * g.irc + c.lo},
                                        c.len, (uint64_t)(e - N), c.len, g.irc, 308));
            N = e;
        }
    }

    // Super-steps: slice s runs logical step t - s in super-step t (a wavefront), so the
    // phases of consecutive slices share one RCCL group and use different links at once.
    const int S = (int)L.size();
    p.steps.resize((size_t)(P + S - 1));
    for (int t = 0; t < P + S - 1; ++t) {
        Step& st = p.steps[t];
        for (int s = 0; s < P; ++s) {
            const int ls = t - s;
            if (ls < 0 || ls >= S) continue;
            if (st.label.empty()) st.label = "t" + std::to_string(t);
            static const char* names[] = {"fold", "phase", "return", "lane", "dist1", "dist2", "scatter",
                                          "bphase", "blane", "bdist", "rphase", "rlane", "bcast", "bruck", "kscat"};
            const Logical lk = L[ls].first;
            st.label += std::string(st.label.size() > 0 ? "," : "") + names[lk] +
                        (lk == S_PHASE || lk == S_AG || lk == S_KSCAT ? std::to_string(L[ls].second) : "") + "/s" +
                        std::to_string(s);
            B.emit(L[ls].first, L[ls].second, sl[s], st);
        }
    }
    return p;
}

static const char* buf_name(uint8_t b) {
    switch (b) {
    case BUF_SEND: return "SEND";
    case BUF_RECV: return "RECV";
    case BUF_ACC: return "ACC";
    default: return "STAGE";
    }
}

// "t3,phase0/s0,lane/s1" -> "phase0+lane"; "gather/s2" -> "gather".  Names are compared as
// whole tokens ("gather" after "allgather" is a phase of its own).
std::string phase_name(const std::string& label) {
    std::vector<std::string> names;
    std::string tok;
    auto flush = [&]() {
        const std::string name = tok.substr(0, tok.find('/'));
        tok.clear();
        if (name.empty() || (name[0] == 't' && name.size() > 1 && std::isdigit((unsigned char)name[1]))) return;
        for (const auto& n : names)
            if (n == name) return;
        names.push_back(name);
    };
    for (char ch : label) {
        if (ch == ',') flush();
        else tok += ch;
    }
    flush();
    std::string out;
    for (const auto& n : names) out += (out.empty() ? "" : "+") + n;
    return out.empty() ? "step" : out;
}

std::string describe(const Plan& p) {
    std::ostringstream o;
    const Geometry& g = p.g;
    o << "plan mode=" << (int)p.mode << " error=" << p.error << " nranks=" << g.nranks << " rank=" << p.rank
      << " k=" << g.k << " b=" << g.b << " recvcount=" << g.recvcount << " irc=" << g.irc << " send=" << p.send_elems
      << " recv=" << p.recv_elems << " acc=" << p.acc_elems << " stage=" << p.stage_elems
      << " slices=" << p.slices << " balanced=" << (p.balanced ? 1 : 0) << " schedule=" << p.sched
      << " steps=" << p.steps.size() << "\n";
    auto local = [&](const LocalOp& op) {
        if (op.kind == L_COPY) {
            o << "copy " << buf_name(op.dst.buf) << " " << op.dst.off << " " << buf_name(op.acc.buf) << " "
              << op.acc.off << " " << op.count << "\n";
        } else if (op.kind == L_COPY2D) {
            o << "copy2d " << buf_name(op.dst.buf) << " " << op.dst.off << " " << buf_name(op.acc.buf) << " "
              << op.acc.off << " " << op.count << " " << op.rows << " " << op.dpitch << " " << op.spitch << "\n";
        } else if (op.kind == L_TREE) {
            o << "tree " << buf_name(op.dst.buf) << " " << op.dst.off << " " << buf_name(op.acc.buf) << " "
              << op.acc.off << " " << op.count << " " << op.ins.size();
            for (const Ref& r : op.ins) o << " " << buf_name(r.buf) << " " << r.off;
            o << " c";
            for (uint8_t c : op.comb) o << " " << (int)c;
            o << " s";
            for (uint8_t w : op.swaps) o << " " << (int)w;
            o << "\n";
        } else {
            o << (op.swap ? "reduce_sw " : "reduce ") << buf_name(op.dst.buf) << " " << op.dst.off << " " << buf_name(op.acc.buf) << " "
              << op.acc.off << " " << op.count << " " << op.ins.size();
            for (const Ref& r : op.ins) o << " " << buf_name(r.buf) << " " << r.off;
            o << "\n";
        }
    };
    for (const LocalOp& op : p.pre) {
        o << "pre ";
        local(op);
    }
    for (size_t i = 0; i < p.steps.size(); ++i) {
        const Step& s = p.steps[i];
        o << "step " << i << " " << (s.label.empty() ? "-" : s.label) << " wait=" << s.comm_wait;
        o << " deps=";
        for (size_t j = 0; j < s.comm_deps.size(); ++j) o << (j ? "," : "") << s.comm_deps[j];
        if (s.comm_deps.empty()) o << "-";
        o << "\n";
        for (const Xfer& x : s.sends)
            o << "send " << x.peer << " " << buf_name(x.ref.buf) << " " << x.ref.off << " " << x.count << "\n";
        for (const Xfer& x : s.recvs)
            o << "recv " << x.peer << " " << buf_name(x.ref.buf) << " " << x.ref.off << " " << x.count << "\n";
        for (const Coll& x : s.allgathers)
            o << "allgather " << buf_name(x.ref.buf) << " " << x.ref.off << " " << x.count << "\n";
        for (const LocalOp& op : s.post) local(op);
    }
    return o.str();
}

}  // namespace chr

// ==== MPICH baseline allreduces driven by the reference's testing/main.cpp ==================
// (testing/mpich_implementations/all_reduce/*.cpp).  They work in
// recvbuf; STAGE holds incoming blocks; every reduction goes through the same fused kernel.
namespace chr {
namespace {

struct MB {
    Plan& p;
    int n, me;
    uint64_t count;
    bool commutative;
    Step& add(const char* label) {
        p.steps.emplace_back();
        p.steps.back().label = label;
        return p.steps.back();
    }
    void need(uint64_t e) { p.stage_elems = std::max(p.stage_elems, e); }
    // recvbuf[off, +len) = OP(STAGE[soff], recvbuf)  (MPI_Reduce_local(tmp, recvbuf + off))
    void reduce_in(Step& s, uint64_t off, uint64_t soff, uint64_t len, int site) {
        if (len) s.post.push_back(make_reduce({BUF_RECV, off}, {BUF_RECV, off}, {{BUF_STAGE, soff}}, len, site));
    }
};

// Fold of the non-power-of-two ranks (recursive doubling :35-55, reduce_scatter_allgather :28-52):
// even r < 2*rem sends its whole buffer to r+1, which reduces it.
void mb_fold(MB& b, int rem, int site) {
    Step& s = b.add("fold");
    if (b.me < 2 * rem) {
        if (b.me % 2 == 0) {
            s.sends.push_back({b.me + 1, {BUF_RECV, 0}, b.count});
        } else {
            s.recvs.push_back({b.me - 1, {BUF_STAGE, 0}, b.count});
            b.need(b.count);
            b.reduce_in(s, 0, 0, b.count, site);
        }
    }
}
void mb_unfold(MB& b, int rem) {  // :88-97 / :161-171
    Step& s = b.add("unfold");
    if (b.me < 2 * rem) {
        if (b.me % 2) s.sends.push_back({b.me - 1, {BUF_RECV, 0}, b.count});
        else s.recvs.push_back({b.me + 1, {BUF_RECV, 0}, b.count});
    }
}

void build_ring(MB& b) {  // allreduce_ring.cpp:3-104
    const int n = b.n, me = b.me;
    std::vector<uint64_t> cnts(n, 0), displs(n, 0);
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) {  // :31-38
        cnts[i] = (b.count + n - 1) / n;
        if (total + cnts[i] > b.count) {
            cnts[i] = b.count - total;
            break;
        }
        total += cnts[i];
    }
    for (int i = 1; i < n; ++i) displs[i] = displs[i - 1] + cnts[i - 1];
    const int src = (n + me - 1) % n, dst = (me + 1) % n;
    for (int i = 0; i < n - 1; ++i) {  // :56-84
        Step& s = b.add("ring-rs");
        const int recv_rank = (2 * n + me - 2 - i) % n, send_rank = (2 * n + me - 1 - i) % n;
        if (cnts[send_rank]) s.sends.push_back({dst, {BUF_RECV, displs[send_rank]}, cnts[send_rank]});
        if (cnts[recv_rank]) {
            s.recvs.push_back({src, {BUF_STAGE, 0}, cnts[recv_rank]});
            b.need(cnts[recv_rank]);
            b.reduce_in(s, displs[recv_rank], 0, cnts[recv_rank], 80);
        }
    }
    Step& s = b.add("allgatherv");  // MPI_Allgatherv (:86): block j is final on rank j
    for (int j = 0; j < n; ++j) {
        if (j == me) continue;
        if (cnts[me]) s.sends.push_back({j, {BUF_RECV, displs[me]}, cnts[me]});
        if (cnts[j]) s.recvs.push_back({j, {BUF_RECV, displs[j]}, cnts[j]});
    }
}

// allreduce_recursive_doubling.cpp:4-101.  A non-commutative op keeps rank order (:69-80): the partner's buffer is
// the left operand when the partner is the lower rank, else the running value is (reduced into tmp_buf, copied back:
// the running-value-first combine).
void build_rd(MB& b) {
    int pof2 = 1;
    while (pof2 <= b.n) pof2 <<= 1;
    pof2 >>= 1;
    const int rem = b.n - pof2;
    mb_fold(b, rem, 48);
    const int newrank = b.me < 2 * rem ? (b.me % 2 ? b.me / 2 : -1) : b.me - rem;
    for (int mask = 1; mask < pof2; mask <<= 1) {
        Step& s = b.add("rd");
        if (newrank < 0) continue;
        const int newdst = newrank ^ mask, dst = newdst < rem ? newdst * 2 + 1 : newdst + rem;
        s.sends.push_back({dst, {BUF_RECV, 0}, b.count});
        s.recvs.push_back({dst, {BUF_STAGE, 0}, b.count});
        b.need(b.count);
        b.reduce_in(s, 0, 0, b.count, 70);
        if (!b.commutative && dst > b.me) s.post.back().swap = true;  // :75-79
    }
    mb_unfold(b, rem);
}

void build_rsag(MB& b) {  // allreduce_reduce_scatter_allgather.cpp:3-173
    int pof2 = 1;
    while (pof2 <= b.n) pof2 *= 2;
    pof2 /= 2;
    const int rem = b.n - pof2;
    mb_fold(b, rem, 43);
    const int newrank = b.me < 2 * rem ? (b.me % 2 ? b.me / 2 : -1) : b.me - rem;
    std::vector<uint64_t> cnts(pof2), disps(pof2, 0);
    for (int i = 0; i < pof2; ++i) cnts[i] = b.count / pof2 + ((uint64_t)i < b.count % pof2 ? 1 : 0);
    for (int i = 1; i < pof2; ++i) disps[i] = disps[i - 1] + cnts[i - 1];
    auto sum = [&](int a, int e) {
        uint64_t t = 0;
        for (int i = a; i < e; ++i) t += cnts[i];
        return t;
    };
    int send_idx = 0, recv_idx = 0, last_idx = pof2;
    int mask = 1;
    for (; mask < pof2; mask <<= 1) {  // reduce-scatter (:76-117)
        Step& s = b.add("rsag-rs");
        if (newrank < 0) continue;
        const int newdst = newrank ^ mask, dst = newdst < rem ? newdst * 2 + 1 : newdst + rem;
        uint64_t send_cnt, recv_cnt;
        if (newrank < newdst) {
            send_idx = recv_idx + pof2 / (mask * 2);
            send_cnt = sum(send_idx, last_idx);
            recv_cnt = sum(recv_idx, send_idx);
        } else {
            recv_idx = send_idx + pof2 / (mask * 2);
            send_cnt = sum(send_idx, recv_idx);
            recv_cnt = sum(recv_idx, last_idx);
        }
        if (send_cnt) s.sends.push_back({dst, {BUF_RECV, disps[send_idx]}, send_cnt});
        if (recv_cnt) {
            s.recvs.push_back({dst, {BUF_STAGE, disps[recv_idx]}, recv_cnt});
            b.need(b.count);
            b.reduce_in(s, disps[recv_idx], disps[recv_idx], recv_cnt, 104);
        }
        send_idx = recv_idx;
        if ((mask << 1) < pof2) last_idx = recv_idx + pof2 / (mask << 1);
    }
    for (mask >>= 1; mask > 0; mask >>= 1) {  // allgather (:119-160)
        Step& s = b.add("rsag-ag");
        if (newrank < 0) continue;
        const int newdst = newrank ^ mask, dst = newdst < rem ? newdst * 2 + 1 : newdst + rem;
        uint64_t send_cnt, recv_cnt;
        if (newrank < newdst) {
            if (mask != pof2 / 2) last_idx = last_idx + pof2 / (mask * 2);
            recv_idx = send_idx + pof2 / (mask * 2);
            send_cnt = sum(send_idx, recv_idx);
            recv_cnt = sum(recv_idx, last_idx);
        } else {
            recv_idx = send_idx - pof2 / (mask * 2);
            send_cnt = sum(send_idx, last_idx);
            recv_cnt = sum(recv_idx, send_idx);
        }
        if (send_cnt) s.sends.push_back({dst, {BUF_RECV, disps[send_idx]}, send_cnt});
        if (recv_cnt) s.recvs.push_back({dst, {BUF_RECV, disps[recv_idx]}, recv_cnt});
        if (newrank > newdst) send_idx = recv_idx;
    }
    mb_unfold(b, rem);
}

void build_recexch(MB& b, int k_in) {  // allreduce_recexch.cpp:188-440 (float path)
    if (b.n == 1) return;
    Recexch x;
    if (recexch_neighbors(b.me, b.n, k_in, &x)) {
        b.p.error = 1;
        return;
    }
    const int k = x.k;
    const uint64_t cnt = b.count;
    {  // step 1 (:267-296): non-participants send, participants reduce in recvfrom order
        Step& s = b.add("rx-step1");
        if (x.step1_sendto != -1) {
            s.sends.push_back({x.step1_sendto, {BUF_RECV, 0}, cnt});
        } else if (x.step1_nrecvs) {
            std::vector<Ref> ins;
            for (int i = 0; i < x.step1_nrecvs; ++i) {
                s.recvs.push_back({x.step1_recvfrom[i], {BUF_STAGE, (uint64_t)i * cnt}, cnt});
                ins.push_back({BUF_STAGE, (uint64_t)i * cnt});
            }
            b.need((uint64_t)x.step1_nrecvs * cnt);
            s.post.push_back(make_reduce({BUF_RECV, 0}, {BUF_RECV, 0}, ins, cnt, 298));
        }
    }
    for (int ph = 0; ph < x.step2_nphases; ++ph) {  // step 2 (:298-365)
        Step& s = b.add("rx-phase");
        if (x.step1_sendto != -1) continue;
        for (int i = 0; i < k - 1; ++i) {
            s.sends.push_back({x.step2_nbrs[ph][i], {BUF_RECV, 0}, cnt});
            s.recvs.push_back({x.step2_nbrs[ph][i], {BUF_STAGE, (uint64_t)i * cnt}, cnt});
        }
        b.need((uint64_t)(k - 1) * cnt);
        // MPICH_do_reduce (:147-186): fold [b_0..b_{idx-1}, recv, b_idx..b_{k-2}] left to right
        // with the running value as the FIRST operand; MPICH_find_myidx (:137-145) picks idx.
        int idx = k - 1;
        for (int i = 0; i < k - 1; ++i)
            if (x.step2_nbrs[ph][i] > b.me) {
                idx = i;
                break;
            }
        std::vector<Ref> seq;
        for (int i = 0; i < idx; ++i) seq.push_back({BUF_STAGE, (uint64_t)i * cnt});
        seq.push_back({BUF_RECV, 0});
        for (int i = idx; i < k - 1; ++i) seq.push_back({BUF_STAGE, (uint64_t)i * cnt});
        LocalOp op = make_reduce({BUF_RECV, 0}, seq[0], std::vector<Ref>(seq.begin() + 1, seq.end()), cnt, 153);
        op.swap = true;
        s.post.push_back(op);
    }
    {  // step 3 (:367-386)
        Step& s = b.add("rx-step3");
        if (x.step1_sendto != -1) s.recvs.push_back({x.step1_sendto, {BUF_RECV, 0}, cnt});
        else
            for (int i = 0; i < x.step1_nrecvs; ++i) s.sends.push_back({x.step1_recvfrom[i], {BUF_RECV, 0}, cnt});
    }
}

// allreduce_recursive_multiplying.cpp:3-176.  Every k-way combine (the pre-fold :58-84 and
// each level :110-145) folds the members' buffers left to right with the running value as
// the first operand -- the same chain as MPICH_do_reduce.
void build_rmult(MB& b, int k) {
    const int n = b.n, me = b.me;
    const uint64_t cnt = b.count;
    int pofk = 1;
    while (pofk * k <= n) pofk *= k;
    auto chain = [&](Step& s, const std::vector<Ref>& seq) {
        LocalOp op = make_reduce({BUF_RECV, 0}, seq[0], std::vector<Ref>(seq.begin() + 1, seq.end()), cnt, 123);
        op.swap = true;
        s.post.push_back(op);
    };
    if (pofk < n) {
        Step& s = b.add("rm-pre");
        if (me >= pofk) {
            s.sends.push_back({me % pofk, {BUF_RECV, 0}, cnt});
        } else {
            std::vector<Ref> seq;
            for (int src = me + pofk; src < n; src += pofk) {
                const uint64_t slot = (uint64_t)seq.size() * cnt;
                s.recvs.push_back({src, {BUF_STAGE, slot}, cnt});
                seq.push_back({BUF_STAGE, slot});
            }
            if (!seq.empty()) {
                b.need((uint64_t)seq.size() * cnt);
                seq.push_back({BUF_RECV, 0});
                chain(s, seq);
            }
        }
    }
    for (int distance = 1, next = k; distance < pofk; distance = next, next *= k) {
        Step& s = b.add("rm-level");
        if (me >= pofk) continue;
        const int start = me / next * next;
        std::vector<Ref> seq;
        uint64_t e = 0;
        for (int dst = start + me % distance; dst < start + next; dst += distance) {
            if (dst == me) {
                seq.push_back({BUF_RECV, 0});
                continue;
            }
            s.sends.push_back({dst, {BUF_RECV, 0}, cnt});
            s.recvs.push_back({dst, {BUF_STAGE, e * cnt}, cnt});
            seq.push_back({BUF_STAGE, e * cnt});
            ++e;
        }
        b.need(e * cnt);
        chain(s, seq);
    }
    if (pofk < n) {
        Step& s = b.add("rm-post");
        if (me >= pofk) s.recvs.push_back({me % pofk, {BUF_RECV, 0}, cnt});
        else
            for (int dst = me + pofk; dst < n; dst += pofk) s.sends.push_back({dst, {BUF_RECV, 0}, cnt});
    }
}

// allreduce_k_reduce_scatter_allgather.cpp:257-533: recexch step 1, a k-ary reduce-scatter
// over the base-k digit-reversed blocks, the mirror allgather, step 3.  The reference runs
// each neighbour of a phase as its own blocking exchange; the blocks involved are disjoint,
// so one group per phase with a fused (k-1)-way reduce in neighbour order is the same data
// flow and the same per-element reduction order.
struct KrsagGeom {
    int n, k, pofk, rem, T, log_pofk;
    std::vector<uint64_t> cnts, displs;
    int reverse_digits(int rank) const {  // :66-120
        int s2 = rank < T ? rank / k : rank - rem;
        std::vector<int> digit(std::max(log_pofk, 1), 0);
        for (int i = 0; s2 != 0; ++i) {
            digit[i] = s2 % k;
            s2 /= k;
        }
        int rev = 0, power = 1;
        for (int i = 0; i < log_pofk; ++i) {
            rev += digit[log_pofk - 1 - i] * power;
            power *= k;
        }
        return step2_to_orig(rev, rem, k);
    }
    void block(int rank, int level, uint64_t* off, uint64_t* cnt) const {  // :25-63
        const int rr = reverse_digits(rank);
        int kpp = 1;
        while (level-- > 0) kpp *= k;
        const int s2 = rr < T ? rr / k : rr - rem;
        const int mn = (s2 / kpp) * kpp - 1, mx = mn + kpp;
        const int omn = mn >= 0 ? step2_to_orig(mn, rem, k) : mn, omx = step2_to_orig(mx, rem, k);
        *off = displs[omn + 1];
        *cnt = 0;
        for (int x = omn + 1; x <= omx; ++x) *cnt += cnts[x];
    }
};

void build_krsag(MB& b, int k_in) {
    const int n = b.n, me = b.me;
    const uint64_t cnt = b.count;
    if (k_in <= 1) k_in = 2;  // :273-275
    Recexch x;
    if (recexch_neighbors(me, n, k_in, &x)) {
        b.p.error = 1;
        return;
    }
    const int k = x.k, nph = x.step2_nphases;
    const bool part = x.step1_sendto == -1;
    {  // step 1 (:313-333): sequential receive + reduce, recvfrom order
        Step& s = b.add("krsag-step1");
        if (!part) {
            s.sends.push_back({x.step1_sendto, {BUF_RECV, 0}, cnt});
        } else if (x.step1_nrecvs) {
            std::vector<Ref> ins;
            for (int i = 0; i < x.step1_nrecvs; ++i) {
                s.recvs.push_back({x.step1_recvfrom[i], {BUF_STAGE, (uint64_t)i * cnt}, cnt});
                ins.push_back({BUF_STAGE, (uint64_t)i * cnt});
            }
            b.need((uint64_t)x.step1_nrecvs * cnt);
            s.post.push_back(make_reduce({BUF_RECV, 0}, {BUF_RECV, 0}, ins, cnt, 327));
        }
    }
    KrsagGeom g{n, k, x.p_of_k, n - x.p_of_k, x.T, nph, {}, {}};
    g.cnts.assign(n + 1, 0);
    g.displs.assign(n + 1, 0);
    for (int i = 0; i < g.pofk - 1; ++i) g.cnts[step2_to_orig(i, g.rem, k)] = cnt / (uint64_t)g.pofk;  // :341-345
    g.cnts[n - 1] = cnt - (cnt / (uint64_t)g.pofk) * (uint64_t)(g.pofk - 1);  // :346-347 (always rank n-1)
    for (int i = 1; i < n; ++i) g.displs[i] = g.displs[i - 1] + g.cnts[i - 1];
    for (int p = 0; p < nph; ++p) {  // reduce-scatter (:353-401)
        Step& s = b.add("krsag-rs");
        if (!part) continue;
        const int j = nph - 1 - p;
        uint64_t off, len;
        g.block(me, j, &off, &len);
        std::vector<Ref> ins;
        for (int i = 0; i < k - 1; ++i) {
            const int dst = x.step2_nbrs[p][i];
            uint64_t soff, slen;
            g.block(dst, j, &soff, &slen);
            if (slen) s.sends.push_back({dst, {BUF_RECV, soff}, slen});
            if (len) {
                s.recvs.push_back({dst, {BUF_STAGE, (uint64_t)i * cnt + off}, len});
                ins.push_back({BUF_STAGE, (uint64_t)i * cnt + off});
            }
        }
        if (len) {
            b.need((uint64_t)(k - 1) * cnt);
            s.post.push_back(make_reduce({BUF_RECV, off}, {BUF_RECV, off}, ins, len, 395));
        }
    }
    for (int p = 0; p < nph; ++p) {  // allgather (:403-493): level p, phase nph-1-p neighbours
        Step& s = b.add("krsag-ag");
        if (!part) continue;
        const int ph = nph - 1 - p;
        uint64_t off, len;
        g.block(me, p, &off, &len);
        for (int i = 0; i < k - 1; ++i) {
            const int nbr = x.step2_nbrs[ph][i];
            uint64_t roff, rlen;
            g.block(nbr, p, &roff, &rlen);
            if (len) s.sends.push_back({nbr, {BUF_RECV, off}, len});
            if (rlen) s.recvs.push_back({nbr, {BUF_RECV, roff}, rlen});
        }
    }
    {  // step 3 (:496-520)
        Step& s = b.add("krsag-step3");
        if (!part) s.recvs.push_back({x.step1_sendto, {BUF_RECV, 0}, cnt});
        else
            for (int i = 0; i < x.step1_nrecvs; ++i) s.sends.push_back({x.step1_recvfrom[i], {BUF_RECV, 0}, cnt});
    }
}

// ---- MPICH baseline reduce-scatters (block) ------------------------------------------------
// testing/mpich_implementations/reduce_scatter/*.cpp, driven by that directory's main.cpp
// (MPI_Reduce_scatter_block semantics: rank r gets block r of the reduced n*rc buffer).  SEND holds
// the n*rc input (RECV under MPI_IN_PLACE), RECV the rc-element result, ACC the reference's
// tmp_results, STAGE its tmp_recvbuf.
struct RB {
    Plan& p;
    int n, me;
    uint64_t rc, total;
    bool commutative;
    Step& add(const char* label) {
        p.steps.emplace_back();
        p.steps.back().label = label;
        return p.steps.back();
    }
    void need(uint64_t e) { p.stage_elems = std::max(p.stage_elems, e); }
};

// reduce_scatter_pairwise.cpp:4-74: n-1 Sendrecv rounds, round i sends block (me+i) to me+i and
// receives my block from me-i, each folded into the result in round order (:54 / :56).  The
// blocks sent are never written, so all rounds share one group and one fused reduction.
void build_rs_pairwise(RB& b) {
    const uint64_t rc = b.rc;
    if (b.n == 1) {
        b.p.pre.push_back(make_copy({BUF_RECV, 0}, {BUF_SEND, 0}, rc, 32));
        return;
    }
    Step& s = b.add("pw");
    std::vector<Ref> ins;
    for (int i = 1; i < b.n; ++i) {
        const int src = (b.me - i + b.n) % b.n, dst = (b.me + i) % b.n;
        s.sends.push_back({dst, {BUF_SEND, (uint64_t)dst * rc}, rc});
        s.recvs.push_back({src, {BUF_STAGE, (uint64_t)(i - 1) * rc}, rc});
        ins.push_back({BUF_STAGE, (uint64_t)(i - 1) * rc});
    }
    b.need((uint64_t)(b.n - 1) * rc);
    // in place the result lands in block 0 of recvbuf (:64-66); its input is sent in this step
    s.post.push_back(make_reduce({BUF_RECV, 0}, {BUF_SEND, (uint64_t)b.me * rc}, ins, rc, 54));
}

// reduce_scatter_recursive_halving.cpp:7-153: the 2*rem lowest ranks fold pairwise (even -> odd,
// whole buffer, :50-66), the pof2 survivors halve the live range log2(pof2) times (:88-128) over
// blocks of 1 or 2 ranks (newcnts), then odd fold ranks return their partner's block (:137-143).
void build_rs_halving(RB& b) {
    const int n = b.n, me = b.me;
    const uint64_t rc = b.rc, total = b.total;
    int pof2 = 1;
    while (pof2 <= n) pof2 *= 2;
    pof2 = pof2 == n ? pof2 : pof2 / 2;  // :40-46
    const int rem = n - pof2;
    const int newrank = me < 2 * rem ? (me % 2 ? me / 2 : -1) : me - rem;
    if (newrank >= 0) {
        b.p.pre.push_back(make_copy({BUF_ACC, 0}, {BUF_SEND, 0}, total, 35));
        b.p.acc_elems = total;
    }
    {
        Step& s = b.add("rh-fold");
        if (me < 2 * rem) {
            if (me % 2 == 0) {
                s.sends.push_back({me + 1, {BUF_SEND, 0}, total});
            } else {
                s.recvs.push_back({me - 1, {BUF_STAGE, 0}, total});
                b.need(total);
                s.post.push_back(make_reduce({BUF_ACC, 0}, {BUF_ACC, 0}, {{BUF_STAGE, 0}}, total, 59));
            }
        }
    }
    std::vector<uint64_t> cnts(pof2), disps(pof2, 0);
    for (int i = 0; i < pof2; ++i) {  // :74-86
        const int old_i = i < rem ? i * 2 + 1 : i + rem;
        cnts[i] = old_i < 2 * rem ? 2 * rc : rc;
    }
    for (int i = 1; i < pof2; ++i) disps[i] = disps[i - 1] + cnts[i - 1];
    auto sum = [&](int a, int e) {
        uint64_t t = 0;
        for (int i = a; i < e; ++i) t += cnts[i];
        return t;
    };
    int send_idx = 0, recv_idx = 0, last_idx = pof2;
    for (int mask = pof2 >> 1; mask > 0; mask >>= 1) {  // :91-128
        Step& s = b.add("rh");
        if (newrank < 0) continue;
        const int newdst = newrank ^ mask, dst = newdst < rem ? newdst * 2 + 1 : newdst + rem;
        uint64_t send_cnt, recv_cnt;
        if (newrank < newdst) {
            send_idx = recv_idx + mask;
            send_cnt = sum(send_idx, last_idx);
            recv_cnt = sum(recv_idx, send_idx);
        } else {
            recv_idx = send_idx + mask;
            send_cnt = sum(send_idx, recv_idx);
            recv_cnt = sum(recv_idx, last_idx);
        }
        if (send_cnt) s.sends.push_back({dst, {BUF_ACC, disps[send_idx]}, send_cnt});
        if (recv_cnt) {
            s.recvs.push_back({dst, {BUF_STAGE, disps[recv_idx]}, recv_cnt});
            b.need(total);
            s.post.push_back(make_reduce({BUF_ACC, disps[recv_idx]}, {BUF_ACC, disps[recv_idx]},
                                         {{BUF_STAGE, disps[recv_idx]}}, recv_cnt, 121));
        }
        send_idx = recv_idx;
        last_idx = recv_idx + mask;
    }
    Step& s = b.add("rh-unfold");
    if (me < 2 * rem) {
        if (me % 2) s.sends.push_back({me - 1, {BUF_ACC, (uint64_t)(me - 1) * rc}, rc});
        else s.recvs.push_back({me + 1, {BUF_RECV, 0}, rc});
    }
    if (newrank >= 0) s.post.push_back(make_copy({BUF_RECV, 0}, {BUF_ACC, (uint64_t)me * rc}, rc, 130));
}

// reduce_scatter_recursive_doubling.cpp:10-177: at distance `mask` each rank exchanges every block outside its
// own and its partner's subtree of `mask` ranks (two hindexed blocks each way, :58-104); for a
// non-power-of-two size the ranks without a partner get the data relayed down the subtree
// (:106-130); the received blocks are folded into tmp_results (:132-155) -- as the left operand for a commutative
// op or when the partner's subtree is the lower one, else with tmp_results as the left operand (reduced into
// tmp_recvbuf and copied back, :158: the running-value-first combine).
void build_rs_doubling(RB& b) {
    const int P = b.n, me = b.me;
    const uint64_t rc = b.rc, total = b.total;
    b.p.pre.push_back(make_copy({BUF_ACC, 0}, {BUF_SEND, 0}, total, 39));
    b.p.acc_elems = total;
    b.need(total);
    const bool pof2 = (P & (P - 1)) == 0;
    int stage = 0;
    for (int mask = 1; mask < P; mask <<= 1, ++stage) {
        const int dst = me ^ mask;
        const int dtr = (dst >> stage) << stage, mtr = (me >> stage) << stage;
        // (offset, length) in elements of the two send and receive blocks
        const uint64_t s0 = (uint64_t)mtr * rc;
        const uint64_t s1 = P - (mtr + mask) > 0 ? (uint64_t)(P - (mtr + mask)) * rc : 0;
        const uint64_t s1off = s0 + rc * (uint64_t)(std::min(mtr + mask, P) - mtr);
        const uint64_t r0 = rc * (uint64_t)std::min(dtr, P);
        const uint64_t r1 = P - (dtr + mask) > 0 ? (uint64_t)(P - (dtr + mask)) * rc : 0;
        const uint64_t r1off = r0 + rc * (uint64_t)(std::min(dtr + mask, P) - dtr);
        bool received = false;
        Step* last = &b.add("rd");
        if (dst < P) {
            if (s0) last->sends.push_back({dst, {BUF_ACC, 0}, s0});
            if (s1) last->sends.push_back({dst, {BUF_ACC, s1off}, s1});
            if (r0) last->recvs.push_back({dst, {BUF_STAGE, 0}, r0});
            if (r1) last->recvs.push_back({dst, {BUF_STAGE, r1off}, r1});
            received = true;
        }
        if (!pof2) {  // relays: one step per level for every rank, so the steps line up
            const bool tail = dtr + mask > P;
            const int npc = P - mtr - mask;
            int k = 0;
            for (int j = mask; j >>= 1;) ++k;  // log2(mask)
            for (int tmp_mask = mask >> 1; tmp_mask; tmp_mask >>= 1, --k) {
                Step& s = b.add("rd-relay");
                last = &s;
                if (!tail) continue;
                const int sd = me ^ tmp_mask, tree_root = (me >> k) << k;
                if (sd > me && me < tree_root + npc && sd >= tree_root + npc) {
                    if (r0) s.sends.push_back({sd, {BUF_STAGE, 0}, r0});
                    if (r1) s.sends.push_back({sd, {BUF_STAGE, r1off}, r1});
                } else if (sd < me && sd < tree_root + npc && me >= tree_root + npc) {
                    if (r0) s.recvs.push_back({sd, {BUF_STAGE, 0}, r0});
                    if (r1) s.recvs.push_back({sd, {BUF_STAGE, r1off}, r1});
                    received = true;
                }
            }
        }
        if (received) {
            const bool run_first = !b.commutative && !(dtr < mtr);
            if (r0) {
                last->post.push_back(make_reduce({BUF_ACC, 0}, {BUF_ACC, 0}, {{BUF_STAGE, 0}}, r0, 141));
                last->post.back().swap = run_first;
            }
            if (r1) {
                last->post.push_back(make_reduce({BUF_ACC, r1off}, {BUF_ACC, r1off}, {{BUF_STAGE, r1off}}, r1, 151));
                last->post.back().swap = run_first;
            }
        }
    }
    Step& s = b.add("rd-out");  // :171-174
    s.post.push_back(make_copy({BUF_RECV, 0}, {BUF_ACC, (uint64_t)me * rc}, rc, 173));
}

// reduce_scatter_radix.cpp:204-377: the single-level ancestor of CHiArA's phase 1.  Recexch
// step 1 folds the non-participants' whole buffers (:247-273), step 2 exchanges, per phase from
// the highest digit down, with the k-1 neighbours the regions count/offset name in units of
// recvcount blocks, folding each into the own region in neighbour order (:279-318), step 3 returns
// the non-participants' blocks (:321-347).  The k-1 exchanges of a phase touch disjoint regions,
// so they share one group and one fused reduction.
void build_rs_radix(RB& b, int k_in) {
    const int n = b.n, me = b.me;
    const uint64_t rc = b.rc, total = b.total;
    Recexch x;
    if (recexch_neighbors(me, n, k_in, &x)) {
        b.p.error = 1;
        return;
    }
    const int k = x.k, nph = x.step2_nphases;
    const bool part = x.step1_sendto == -1;
    std::vector<int> cnt, off;
    recexch_count_offset(n, std::max(nph, 1), k, &cnt, &off);
    if (part) {
        b.p.pre.push_back(make_copy({BUF_ACC, 0}, {BUF_SEND, 0}, total, 240));
        b.p.acc_elems = total;
    }
    {
        Step& s = b.add("rr-step1");
        if (!part) {
            s.sends.push_back({x.step1_sendto, {BUF_SEND, 0}, total});
        } else if (x.step1_nrecvs) {
            std::vector<Ref> ins;
            for (int i = 0; i < x.step1_nrecvs; ++i) {
                s.recvs.push_back({x.step1_recvfrom[i], {BUF_STAGE, (uint64_t)i * total}, total});
                ins.push_back({BUF_STAGE, (uint64_t)i * total});
            }
            b.need((uint64_t)x.step1_nrecvs * total);
            s.post.push_back(make_reduce({BUF_ACC, 0}, {BUF_ACC, 0}, ins, total, 266));
        }
    }
    for (int ph = nph - 1; ph >= 0; --ph) {
        Step& s = b.add("rr-phase");
        if (!part) continue;
        const uint64_t moff = (uint64_t)off[ph * n + me] * rc, mlen = (uint64_t)cnt[ph * n + me] * rc;
        std::vector<Ref> ins;
        for (int i = 0; i < k - 1; ++i) {
            const int dst = x.step2_nbrs[ph][i];
            const uint64_t soff = (uint64_t)off[ph * n + dst] * rc, slen = (uint64_t)cnt[ph * n + dst] * rc;
            if (slen) s.sends.push_back({dst, {BUF_ACC, soff}, slen});
            if (mlen) {
                s.recvs.push_back({dst, {BUF_STAGE, (uint64_t)i * total}, mlen});
                ins.push_back({BUF_STAGE, (uint64_t)i * total});
            }
        }
        if (mlen) {
            b.need((uint64_t)(k - 1) * total);
            s.post.push_back(make_reduce({BUF_ACC, moff}, {BUF_ACC, moff}, ins, mlen, 310));
        }
    }
    Step& s = b.add("rr-step3");
    if (!part) {
        s.recvs.push_back({x.step1_sendto, {BUF_RECV, 0}, rc});
    } else {
        for (int i = 0; i < x.step1_nrecvs; ++i)
            s.sends.push_back({x.step1_recvfrom[i], {BUF_ACC, (uint64_t)x.step1_recvfrom[i] * rc}, rc});
        s.post.push_back(make_copy({BUF_RECV, 0}, {BUF_ACC, (uint64_t)me * rc}, rc, 322));
    }
}

}  // namespace

Plan build_plan_mpich(Mode mode, int n, int me, int k, int aux, uint64_t count, bool commutative) {
    (void)aux;  // recexch single_phase_recv: buffering only, same data flow
    Plan p;
    p.mode = mode;
    p.rank = me;
    if (n < 1 || me < 0 || me >= n || ((mode == MODE_MPICH_RECEXCH || mode == MODE_MPICH_RMULT) && k < 2)) {
        p.error = 1;
        return p;
    }
    if (!commutative) {  // the reference's MPI_ERR_OP, before any data moves
        int pofk = 1;
        while (mode == MODE_MPICH_RMULT && pofk * k <= n) pofk *= k;
        if (mode == MODE_MPICH_KRSAG ||                     // allreduce_k_reduce_scatter_allgather.cpp:278-283
            (mode == MODE_MPICH_RMULT && pofk < n)) {       // allreduce_recursive_multiplying.cpp:43-49
            p.error = 8;                                    // CHR_ERR_UNSUPPORTED
            return p;
        }
    }
    p.g.nranks = n;
    p.g.k = k;
    if (is_mpich_rs(mode)) {
        if (mode == MODE_MPICH_RS_RADIX && k < 2) {
            p.error = 1;
            return p;
        }
        p.g.recvcount = count;
        p.g.total = count * (uint64_t)n;
        p.send_elems = p.g.total;
        p.recv_elems = count;
        if (count == 0) return p;
        RB rb{p, n, me, count, p.g.total, commutative};
        switch (mode) {
        case MODE_MPICH_RS_RADIX: build_rs_radix(rb, k); break;
        case MODE_MPICH_RS_HALVING: build_rs_halving(rb); break;
        case MODE_MPICH_RS_DOUBLING: build_rs_doubling(rb); break;
        default: build_rs_pairwise(rb); break;
        }
        return p;
    }
    p.g.total = count;
    p.send_elems = p.recv_elems = count;
    if (count == 0) return p;
    // pre: recvbuf <- sendbuf (every algorithm starts with this memcpy; no-op in place)
    p.pre.push_back(make_copy({BUF_RECV, 0}, {BUF_SEND, 0}, count, 0));
    MB b{p, n, me, count, commutative};
    switch (mode) {
    case MODE_MPICH_RING: build_ring(b); break;
    case MODE_MPICH_RD: build_rd(b); break;
    case MODE_MPICH_RSAG: build_rsag(b); break;
    case MODE_MPICH_RECEXCH: build_recexch(b, k); break;
    case MODE_MPICH_KRSAG: build_krsag(b, k); break;
    case MODE_MPICH_RMULT: build_rmult(b, k); break;
    default: p.error = 1;
    }
    return p;
}

}  // namespace chr

// ==== allgather_radix_batch (Fugaku_experiments/Allgather/all_gather_radix_batch_1_0.cpp) ====
// The reference gathers each group of b ranks to a root with a k-nomial tree (:55-133),
// exchanges the group blocks between roots linearly (:137-163) and spreads them inside every
// group with a k-port Bruck allgather (:168-360).  Its output is the rank-major concatenation
// (checked against MPI_Allgather for every geometry of tests/golden).  On one node every pair
// of GPUs has its own xGMI link, so relaying blocks through roots only adds hops: here each
// rank sends its block straight to every peer, k-1 peers per step (k ports, as the Bruck
// phase), peers of its own group of b first and then the other groups.  Every link carries
// each block exactly once; no local copies besides placing the own block.
namespace chr {

Plan build_plan_allgather(int n, int me, int k, int b, uint64_t count) {
    Plan p;
    p.mode = MODE_ALLGATHER;
    p.rank = me;
    if (n < 1 || me < 0 || me >= n || k < 2 || b < 1) {
        p.error = 1;
        return p;
    }
    if (n % b) {
        p.error = 3;  // CHR_ERR_BATCH_NOT_DIVISOR
        return p;
    }
    p.g.nranks = n;
    p.g.k = k;
    p.g.b = b;
    p.g.nnodes = n / b;
    p.g.total = count;
    p.send_elems = count;
    p.recv_elems = count * (uint64_t)n;
    if (count == 0) return p;
    const Ref mine{BUF_RECV, (uint64_t)me * count};
    p.pre.push_back(make_copy(mine, {BUF_SEND, 0}, count, 0));
    // (to, from) pairs: offset d inside the group, then group offset D with in-group rotation e.
    // For every pair, `to` receives from this rank in the same step (same offset list).
    const int g = me / b, lr = me % b, nn = n / b;
    std::vector<std::pair<int, int>> peers;
    for (int d = 1; d < b; ++d) peers.push_back({g * b + (lr + d) % b, g * b + (lr - d + b) % b});
    for (int D = 1; D < nn; ++D)
        for (int e = 0; e < b; ++e)
            peers.push_back({((g + D) % nn) * b + (lr + e) % b, ((g - D + nn) % nn) * b + (lr - e + b) % b});
    for (size_t i = 0; i < peers.size(); i += (size_t)(k - 1)) {
        p.steps.emplace_back();
        Step& s = p.steps.back();
        s.label = i < (size_t)(b - 1) ? "ag-intra" : "ag-inter";
        for (size_t j = i; j < peers.size() && j < i + (size_t)(k - 1); ++j) {
            s.sends.push_back({peers[j].first, mine, count});
            s.recvs.push_back({peers[j].second, {BUF_RECV, (uint64_t)peers[j].second * count}, count});
        }
    }
    return p;
}

}  // namespace chr

// ==== CHiArA's phases as stand-alone collectives ==============================================
// testing/custom_implementations/work_dir/reduce_scatter/ keeps each phase of the hierarchical
// reduce-scatter as its own function (each with a DEBUG_MODE self-test main).  Ranks form nnodes =
// n / b groups of b: node = rank / b, lane = rank % b, IRC = recvcount * b, nstages = nnodes / b,
// nu = nnodes % b.  The plans keep the reference's buffers: ACC is tmp_results (stage-major, as the
// reference lays it out), STAGE its tmp_recvbuf / tmp.
namespace chr {
namespace {

// intra_reduce_scatter_radix.cpp:208-541.  Recexch over the group's b lanes (tables of lane, b):
// step 1 folds the non-participants' whole buffers once (:274-311); then, per stage, step 2 runs
// the phases from the highest digit down, exchanging with the k-1 neighbours the count/offset
// regions in units of IRC and folding each received region into the own one in neighbour order
// (:314-356), and step 3 copies the lane's chunk out and returns the non-participants' (:359-386).
// The leftover stage (nu != 0) does the same on regions clipped to its nu chunks (:400-500).  A
// phase's k-1 exchanges read the neighbours' regions and write the own one, which are disjoint, so
// they share one group and one fused reduction, in the reference's operand order.
void build_intra_rs(Plan& p, int n, int me, int k_in, int b, uint64_t rc) {
    const int node = me / b, lane = me % b, base = node * b, nnodes = n / b, nstages = nnodes / b, nu = nnodes % b;
    const uint64_t irc = rc * (uint64_t)b, total = rc * (uint64_t)n, blk = irc * (uint64_t)b;
    p.send_elems = total;
    p.recv_elems = (uint64_t)(nstages + (lane < nu ? 1 : 0)) * irc;
    Recexch x;
    if (recexch_neighbors(lane, b, k_in, &x)) {
        p.error = 1;
        return;
    }
    const int k = x.k, nph = x.step2_nphases;
    const bool part = x.step1_sendto == -1;
    std::vector<int> cnt, off;
    recexch_count_offset(b, std::max(nph, 1), k, &cnt, &off);
    auto need = [&](uint64_t e) { p.stage_elems = std::max(p.stage_elems, e); };
    auto add = [&](const char* label) -> Step& {
        p.steps.emplace_back();
        p.steps.back().label = label;
        return p.steps.back();
    };
    if (part) {
        p.pre.push_back(make_copy({BUF_ACC, 0}, {BUF_SEND, 0}, total, 277));  // :274-280
        p.acc_elems = total;
    }
    {
        Step& s = add("irs-step1");
        if (!part) {
            s.sends.push_back({base + x.step1_sendto, {BUF_SEND, 0}, total});  // :290
        } else if (x.step1_nrecvs) {
            std::vector<Ref> ins;
            for (int i = 0; i < x.step1_nrecvs; ++i) {
                s.recvs.push_back({base + x.step1_recvfrom[i], {BUF_STAGE, (uint64_t)i * total}, total});
                ins.push_back({BUF_STAGE, (uint64_t)i * total});
            }
            need((uint64_t)x.step1_nrecvs * total);
            s.post.push_back(make_reduce({BUF_ACC, 0}, {BUF_ACC, 0}, ins, total, 303));
        }
    }
    // one stage's phases and return; `lim` clips every region to the leftover stage's nu chunks
    auto stage = [&](uint64_t sb, uint64_t lim, uint64_t out_off, bool left) {
        auto clip = [&](int c, int o, uint64_t* len) {  // (offset, length) of a count/offset region
            const uint64_t ro = (uint64_t)o * irc, rl = (uint64_t)c * irc;
            *len = ro < lim ? std::min(rl, lim - ro) : 0;
            return ro;
        };
        for (int ph = nph - 1; ph >= 0; --ph) {
            Step& s = add(left ? "irs-phase-left" : "irs-phase");
            if (!part) continue;
            uint64_t mlen = 0;
            const uint64_t moff = clip(cnt[ph * b + lane], off[ph * b + lane], &mlen);
            std::vector<Ref> ins;
            for (int i = 0; i < k - 1; ++i) {
                const int dst = x.step2_nbrs[ph][i];
                uint64_t slen = 0;
                const uint64_t soff = clip(cnt[ph * b + dst], off[ph * b + dst], &slen);
                if (slen) s.sends.push_back({base + dst, {BUF_ACC, sb + soff}, slen});
                if (mlen) {
                    s.recvs.push_back({base + dst, {BUF_STAGE, (uint64_t)i * blk}, mlen});
                    ins.push_back({BUF_STAGE, (uint64_t)i * blk});
                }
            }
            if (mlen) {
                need((uint64_t)(k - 1) * blk);
                s.post.push_back(make_reduce({BUF_ACC, sb + moff}, {BUF_ACC, sb + moff}, ins, mlen, left ? 464 : 348));
            }
        }
        Step& s = add(left ? "irs-step3-left" : "irs-step3");
        const bool mine = (uint64_t)lane * irc < lim;  // the leftover stage's chunk exists for lanes < nu
        if (!part) {
            if (mine) s.recvs.push_back({base + x.step1_sendto, {BUF_RECV, out_off}, irc});  // :370 / :488
        } else {
            for (int i = 0; i < x.step1_nrecvs; ++i)
                if ((uint64_t)x.step1_recvfrom[i] * irc < lim)
                    s.sends.push_back({base + x.step1_recvfrom[i], {BUF_ACC, sb + (uint64_t)x.step1_recvfrom[i] * irc}, irc});
            if (mine) s.post.push_back(make_copy({BUF_RECV, out_off}, {BUF_ACC, sb + (uint64_t)lane * irc}, irc, 360));
        }
    };
    for (int st = 0; st < nstages; ++st) stage((uint64_t)st * blk, blk, (uint64_t)st * irc, false);
    if (nu) stage((uint64_t)nstages * blk, (uint64_t)nu * irc, (uint64_t)nstages * irc, true);
}

// inter_linear_reduce.cpp:11-73.  For iteration i the lane's root is node i * b + lane: it starts
// from its own chunk i and folds the other nodes' chunk i in ascending node order (MPI_Recv +
// MPI_Reduce_local, :55-63); the others send it theirs (:67).  A rank is the root of at most
// one iteration and all messages of all iterations are independent, so they share one group and
// the root's folds are one fused reduction.
void build_inter_linear(Plan& p, int n, int me, int b, uint64_t rc) {
    const int node = me / b, lane = me % b, nnodes = n / b, niters = nnodes / b + (nnodes % b ? 1 : 0);
    const uint64_t irc = rc * (uint64_t)b;
    // the send buffer this rank reads: up to the last chunk it sends or folds (0 for a lane that is
    // the root of no iteration, :48, whose send buffer may be NULL)
    p.send_elems = 0;
    Step& s = p.steps.emplace_back();
    s.label = "ilr";
    for (int i = 0; i < niters; ++i) {
        const int root_node = i * b + lane;
        if (root_node >= nnodes) continue;  // :48
        const Ref chunk{BUF_SEND, (uint64_t)i * irc};
        p.send_elems = (uint64_t)(i + 1) * irc;
        if (node != root_node) {
            s.sends.push_back({root_node * b + lane, chunk, irc});
            continue;
        }
        p.recv_elems = irc;
        std::vector<Ref> ins;
        for (int j = 0; j < nnodes; ++j) {
            if (j == node) continue;
            const Ref slot{BUF_STAGE, (uint64_t)ins.size() * irc};
            s.recvs.push_back({j * b + lane, slot, irc});
            ins.push_back(slot);
        }
        p.stage_elems = (uint64_t)ins.size() * irc;
        if (ins.empty()) s.post.push_back(make_copy({BUF_RECV, 0}, chunk, irc, 53));  // :53
        else s.post.push_back(make_reduce({BUF_RECV, 0}, chunk, ins, irc, 63));
    }
}

// intra_scatter_radix_batch.cpp:10-110.  The node root (lane node % b) lays its b blocks out in
// normalised order (slot (lane - root) mod b, :40-46); from the largest delta = k^(nphases-1) down,
// every group leader sends each child subgroup's blocks to the child's leader (:65-83) and the
// child leaders receive them (:84-97); each rank copies its block out at the end (:103-105).
void build_intra_scatter(Plan& p, int n, int me, int k, int b, uint64_t rc) {
    (void)n;
    const int node = me / b, lane = me % b, root = node % b, shift = (lane - root + b) % b;
    p.send_elems = lane == root ? (uint64_t)b * rc : 0;
    p.recv_elems = rc;
    p.stage_elems = (uint64_t)b * rc;
    if (lane == root) {  // real slot j -> normalised slot (j - root) mod b: two runs
        p.pre.push_back(make_copy({BUF_STAGE, 0}, {BUF_SEND, (uint64_t)root * rc}, (uint64_t)(b - root) * rc, 44));
        if (root) p.pre.push_back(make_copy({BUF_STAGE, (uint64_t)(b - root) * rc}, {BUF_SEND, 0}, (uint64_t)root * rc, 44));
    }
    int nphases = 0;
    for (int t = b - 1; t > 0; t /= k) ++nphases;  // ceil(log_k b), :31-32
    int delta = 1;
    for (int i = 1; i < nphases; ++i) delta *= k;
    auto peer = [&](int norm) { return node * b + (norm + root) % b; };
    for (int ph = nphases - 1; ph >= 0; --ph) {
        Step& s = p.steps.emplace_back();
        s.label = "isc";
        const int group = delta * k, gstart = (shift / group) * group, gend = std::min(gstart + group, b);
        const int offset = shift - gstart;
        if (offset == 0) {
            for (int j = 1; j < k; ++j) {
                const int child = gstart + j * delta;
                if (child >= gend) break;
                const int subtree = std::min(delta, gend - child);
                s.sends.push_back({peer(child), {BUF_STAGE, (uint64_t)child * rc}, (uint64_t)subtree * rc});
            }
        } else if (offset % delta == 0 && offset < group) {
            const int subtree = std::min(delta, gend - shift);
            s.recvs.push_back({peer(gstart), {BUF_STAGE, (uint64_t)shift * rc}, (uint64_t)subtree * rc});
        }
        delta = ph > 0 ? delta / k : delta;
    }
    Step& s = p.steps.emplace_back();
    s.label = "isc-out";
    s.post.push_back(make_copy({BUF_RECV, 0}, {BUF_STAGE, (uint64_t)shift * rc}, rc, 103));
}

}  // namespace

Plan build_plan_phase(Mode mode, int n, int me, int k, int b, uint64_t rc) {
    Plan p;
    p.mode = mode;
    p.rank = me;
    if (!is_phase(mode) || n < 1 || me < 0 || me >= n || b < 1 || b > n || (mode != MODE_INTER_LINEAR && k < 2)) {
        p.error = 1;  // CHR_ERR_INVALID_ARG
        return p;
    }
    if (n % b) {
        p.error = 3;  // CHR_ERR_BATCH_NOT_DIVISOR
        return p;
    }
    Geometry& g = p.g;
    g.nranks = n;
    g.k = k;
    g.b = b;
    g.nnodes = n / b;
    g.nstages = g.nnodes / b;
    g.nu = g.nnodes % b;
    g.recvcount = rc;
    g.irc = rc * (uint64_t)b;
    g.total = rc;  // zero: nothing to do
    if (rc == 0) return p;
    if (mode == MODE_INTRA_RS) build_intra_rs(p, n, me, k, b, rc);
    else if (mode == MODE_INTER_LINEAR) build_inter_linear(p, n, me, b, rc);
    else build_intra_scatter(p, n, me, k, b, rc);
    return p;
}

}  // namespace chr

// ==== flat schedule: the reference's arithmetic, the full xGMI mesh's communication ==========
//
// The radix/batch hierarchy fixes, for every element, an expression tree over the n ranks'
// inputs (recexch phases in neighbour order, step-1 folds, lane reduction in stage order);
// that tree is what makes the result bits.  Where it is evaluated is free.  build_plan_flat
// extracts the tree of every chunk by executing the reference-order plans of all ranks
// symbolically (expression ids instead of numbers, recvcount = 1), then emits:
//   gather    every rank sends piece q of every chunk (allreduce) / block q (reduce-scatter)
//             straight to rank q: all n-1 links at once, S/n per directed pair;
//   evaluate  rank q evaluates the chunk's tree on its piece with the fused kernel, one launch
//             per reference reduction op, operands in the reference's order;
//   allgather (allreduce) the n result pieces to everyone, S/n per pair.
// Every link carries 2S/n in all, the full-mesh optimum, for any (k, b).  Inputs are read in
// place from SEND: no re-layout copy.
namespace chr {
namespace {

struct SymNode {
    int leaf = -1;  // >= 0: rank r's input element
    int acc = -1;
    std::vector<int> ins;
    bool swap = false;
};

struct SymExec {
    std::vector<SymNode> nodes;
    std::vector<std::vector<std::vector<int>>> buf;  // [rank][Buf][elem] -> node id
    const std::vector<Plan>& P;
    explicit SymExec(const std::vector<Plan>& plans) : P(plans) {
        const int n = (int)P.size();
        for (int r = 0; r < n; ++r) nodes.push_back({r, -1, {}, false});
        buf.resize(n);
        for (int r = 0; r < n; ++r) {
            buf[r].resize(4);
            buf[r][BUF_SEND].assign(P[r].send_elems, r);
            buf[r][BUF_RECV].assign(P[r].recv_elems, -1);
            buf[r][BUF_ACC].assign(P[r].acc_elems, -1);
            buf[r][BUF_STAGE].assign(P[r].stage_elems, -1);
        }
    }
    int* at(int r, const Ref& x, uint64_t i) { return &buf[r][x.buf].at(x.off + i); }
    void local(int r, const LocalOp& op) {
        if (op.kind == L_COPY || op.kind == L_COPY2D) {
            const uint64_t rows = op.kind == L_COPY2D ? op.rows : 1;
            std::vector<int> tmp;
            for (uint64_t row = 0; row < rows; ++row)
                for (uint64_t i = 0; i < op.count; ++i) tmp.push_back(*at(r, op.acc, row * op.spitch + i));
            size_t t = 0;
            for (uint64_t row = 0; row < rows; ++row)
                for (uint64_t i = 0; i < op.count; ++i) *at(r, op.dst, row * op.dpitch + i) = tmp[t++];
            return;
        }
        std::vector<int> out(op.count);
        for (uint64_t i = 0; i < op.count; ++i) {
            const int a = *at(r, op.acc, i);
            if (op.ins.empty()) {
                out[i] = a;
                continue;
            }
            SymNode nd;
            nd.acc = a;
            nd.swap = op.swap;
            for (const Ref& x : op.ins) nd.ins.push_back(*at(r, x, i));
            nodes.push_back(nd);
            out[i] = (int)nodes.size() - 1;
        }
        for (uint64_t i = 0; i < op.count; ++i) *at(r, op.dst, i) = out[i];
    }
    bool run() {
        const int n = (int)P.size();
        for (int r = 0; r < n; ++r)
            for (const LocalOp& op : P[r].pre) local(r, op);
        const size_t ns = P[0].steps.size();
        for (size_t si = 0; si < ns; ++si) {
            std::vector<std::vector<char>> used(n);
            for (int r = 0; r < n; ++r) used[r].assign(P[r].steps[si].sends.size(), 0);
            std::vector<std::tuple<int, Ref, std::vector<int>>> land;
            for (int r = 0; r < n; ++r)
                for (const Xfer& rv : P[r].steps[si].recvs) {
                    const auto& qs = P[rv.peer].steps[si].sends;
                    size_t j = 0;
                    while (j < qs.size() && (used[rv.peer][j] || qs[j].peer != r)) ++j;
                    if (j == qs.size() || qs[j].count != rv.count) return false;
                    used[rv.peer][j] = 1;
                    std::vector<int> data(rv.count);
                    for (uint64_t i = 0; i < rv.count; ++i) data[i] = *at(rv.peer, qs[j].ref, i);
                    land.emplace_back(r, rv.ref, std::move(data));
                }
            for (auto& [r, ref, data] : land)
                for (uint64_t i = 0; i < data.size(); ++i) *at(r, ref, i) = data[i];
            for (int r = 0; r < n; ++r)
                for (const LocalOp& op : P[r].steps[si].post) local(r, op);
        }
        return true;
    }
};

// Evaluation program of one expression: internal nodes in dependency order.  Operand codes:
// >= 0 leaf rank, < 0 temp ~t (result of program entry t).
struct EvalOp {
    int acc;
    std::vector<int> ins;
    bool swap;
};

bool eval_program(const std::vector<SymNode>& nodes, int root, int n, std::vector<EvalOp>* prog) {
    std::vector<int> memo(nodes.size(), INT32_MIN);
    std::vector<char> seen_leaf(n, 0);
    bool ok = true;
    std::function<int(int)> visit = [&](int id) -> int {
        if (id < 0 || (size_t)id >= nodes.size()) {
            ok = false;
            return 0;
        }
        if (memo[id] != INT32_MIN) return memo[id];
        const SymNode& nd = nodes[id];
        if (nd.leaf >= 0) {
            if (seen_leaf[nd.leaf]++) ok = false;  // every input exactly once
            return memo[id] = nd.leaf;
        }
        EvalOp e;
        e.acc = visit(nd.acc);
        for (int c : nd.ins) e.ins.push_back(visit(c));
        e.swap = nd.swap;
        prog->push_back(e);
        return memo[id] = ~(int)(prog->size() - 1);
    };
    const int top = visit(root);
    for (int r = 0; r < n; ++r) ok = ok && seen_leaf[r] == 1;
    return ok && top < 0;
}

// Post-order stack program of one expression for the fused tree kernel (chr_reduce_tree):
// leaves in push order, comb[j] = combines right after leaf j, swaps per combine.  Every fold
// acc (op) in_0 (op) in_1 ... becomes: program(acc), then per input program(in_i) + combine.
bool tree_program(const std::vector<EvalOp>& pr, std::vector<int>* leaves, std::vector<uint8_t>* comb,
                  std::vector<uint8_t>* swaps) {
    if (pr.size() < 2) return false;  // a single fold is already one launch of k_reduce_vec
    int depth = 0, maxd = 0;
    bool ok = true;
    std::function<void(int)> emit = [&](int code) {
        if (code >= 0) {
            leaves->push_back(code);
            comb->push_back(0);
            maxd = std::max(maxd, ++depth);
            return;
        }
        const EvalOp& e = pr[~code];
        emit(e.acc);
        for (int x : e.ins) {
            emit(x);
            if (comb->back() >= 3) ok = false;
            comb->back()++;
            swaps->push_back(e.swap ? 1 : 0);
            --depth;
        }
    };
    emit(~(int)(pr.size() - 1));
    return ok && depth == 1 && (int)leaves->size() <= kTreeMaxLeaves && maxd <= kTreeMaxDepth;
}

// CHR_TREE=0 evaluates flat expressions op by op (one k_reduce_vec launch per reference fold).
bool tree_enabled() {
    const char* e = std::getenv("CHR_TREE");
    return !e || std::atoi(e) != 0;
}

}  // namespace

// oneshot (allreduce): every rank's "piece" is the whole slice -- it receives every peer's whole
// slice of every chunk and evaluates all of it, so no allgather follows (SCHED_FLAT_1SHOT).
Plan build_plan_flat(Mode mode, int n, int me, int k, int b, const Geometry& g, int slices, bool coll_ag, bool merge,
                     bool oneshot) {
    Plan p;
    p.mode = mode;
    p.rank = me;
    p.g = g;
    p.sched = oneshot ? SCHED_FLAT_1SHOT : coll_ag ? SCHED_FLAT_AG : merge ? SCHED_FLAT : SCHED_FLAT_SEQ;
    // 1. the reference-order plans of every rank at recvcount = 1, executed symbolically
    const uint64_t cnt1 = mode == MODE_ALLREDUCE ? (uint64_t)n : 1;
    std::vector<Plan> ref;
    for (int r = 0; r < n; ++r) ref.push_back(build_plan_impl(mode, n, r, k, b, cnt1, 1, SCHED_REFERENCE));
    if (ref[0].error) {
        p.error = ref[0].error;
        return p;
    }
    SymExec X(ref);
    if (!X.run()) {
        p.error = 8;
        return p;
    }
    const uint64_t irc1 = (uint64_t)b;  // IRC at recvcount 1
    std::vector<std::vector<EvalOp>> progs;
    if (mode == MODE_ALLREDUCE) {
        for (int N = 0; N < g.nnodes; ++N) {
            std::vector<EvalOp> pr;
            for (int r = 0; r < n; ++r) {  // every rank holds the same expression for chunk N
                std::vector<EvalOp> q;
                if (!eval_program(X.nodes, X.buf[r][BUF_RECV][(uint64_t)N * irc1], n, &q)) {
                    p.error = 8;
                    return p;
                }
                if (r == 0) pr = q;
            }
            progs.push_back(pr);
        }
    } else {
        std::vector<EvalOp> pr;
        if (!eval_program(X.nodes, X.buf[me][BUF_RECV][0], n, &pr)) {
            p.error = 8;
            return p;
        }
        progs.push_back(pr);
    }
    // whole-tree programs (one fused launch per chunk) where the kernel's limits allow
    struct TreeProg {
        bool on = false;
        std::vector<int> leaves;
        std::vector<uint8_t> comb, swaps;
    };
    std::vector<TreeProg> tprog(progs.size());
    const bool use_tree = tree_enabled();
    size_t temps = 1;
    for (size_t i = 0; i < progs.size(); ++i) {
        TreeProg& t = tprog[i];
        t.on = use_tree && tree_program(progs[i], &t.leaves, &t.comb, &t.swaps);
        if (!t.on) temps = std::max(temps, progs[i].size());
    }

    // 2. slices and pieces
    const uint64_t span = mode == MODE_ALLREDUCE ? g.irc : g.recvcount;  // sliced range
    const uint64_t G = 256;
    int P = slices;
    if ((uint64_t)P > span / G) P = (int)std::max<uint64_t>(1, span / G);
    p.slices = P;
    p.send_elems = g.total;
    p.recv_elems = mode == MODE_ALLREDUCE ? g.total : g.recvcount;
    p.acc_elems = 0;
    const int nchunks = mode == MODE_ALLREDUCE ? g.nnodes : 1;
    const uint64_t slots = (uint64_t)(n - 1 + (int)temps) * (uint64_t)nchunks;
    struct Sl {
        uint64_t lo, len, stage, stride;
    };
    std::vector<Sl> sl(P);
    uint64_t stage = 0;
    for (int s2 = 0; s2 < P; ++s2) {
        const uint64_t lo = s2 == 0 ? 0 : (span * s2 / P) / G * G;
        const uint64_t hi = s2 == P - 1 ? span : (span * (s2 + 1) / P) / G * G;
        const uint64_t len = hi - lo;
        // slots: 64-element multiples, +64 for the per-chunk phase shift below
        const uint64_t stride = ((mode == MODE_ALLREDUCE && !oneshot ? len / (uint64_t)n + 64 : len) + 127) / 64 * 64;
        sl[s2] = {lo, len, stage, stride};
        stage += slots * stride;
    }
    p.stage_elems = stage;
    // piece q of a slice (allreduce): 64-element aligned cut into n
    auto cut = [&](const Sl& c, uint64_t i) { return i >= (uint64_t)n ? c.len : (c.len * i / (uint64_t)n) / 64 * 64; };
    auto piece = [&](const Sl& c, int q, uint64_t* a, uint64_t* l) {
        if (oneshot) {  // every rank evaluates the whole slice
            *a = 0;
            *l = c.len;
            return;
        }
        *a = cut(c, (uint64_t)q);
        *l = cut(c, (uint64_t)q + 1) - *a;
    };
    // position of my operand data for chunk N / my block, in the slice
    auto own = [&](const Sl& c, int N, uint64_t a) -> Ref {  // my input, in place
        if (mode == MODE_ALLREDUCE) return {BUF_SEND, (uint64_t)N * g.irc + c.lo + a};
        return {BUF_SEND, (uint64_t)me * g.recvcount + c.lo};
    };
    // every operand of one evaluation congruent mod 64 elements with the in-place data, so the
    // fused kernel takes its 16-B vector path whatever irc is
    auto phase = [&](int N) -> uint64_t {
        return mode == MODE_ALLREDUCE ? ((uint64_t)N * g.irc) % 64 : ((uint64_t)me * g.recvcount) % 64;
    };
    auto leaf_slot = [&](const Sl& c, int r, int N, uint64_t a) -> Ref {
        const uint64_t idx = (uint64_t)(r < me ? r : r - 1) * (uint64_t)nchunks + (uint64_t)N;
        (void)a;
        return {BUF_STAGE, c.stage + idx * c.stride + phase(N)};
    };
    auto temp_slot = [&](const Sl& c, int t, int N) -> Ref {
        const uint64_t idx = (uint64_t)(n - 1 + t) * (uint64_t)nchunks + (uint64_t)N;
        return {BUF_STAGE, c.stage + idx * c.stride + phase(N)};
    };

    enum { F_GATHER, F_EVAL, F_DIST };
    auto emit = [&](int kind, const Sl& c, Step& st) {
        uint64_t a = 0, len = c.len;
        if (mode == MODE_ALLREDUCE) piece(c, me, &a, &len);
        if (kind == F_GATHER) {
            for (int q = 0; q < n; ++q) {
                if (q == me) continue;
                if (mode == MODE_ALLREDUCE) {
                    uint64_t qa, ql;
                    piece(c, q, &qa, &ql);
                    for (int N = 0; N < nchunks && ql; ++N)
                        st.sends.push_back({q, {BUF_SEND, (uint64_t)N * g.irc + c.lo + qa}, ql});
                } else if (c.len) {
                    st.sends.push_back({q, {BUF_SEND, (uint64_t)q * g.recvcount + c.lo}, c.len});
                }
                for (int N = 0; N < nchunks && len; ++N) st.recvs.push_back({q, leaf_slot(c, q, N, a), len});
            }
            if (!len) return;
            for (int N = 0; N < nchunks; ++N) {
                const auto& pr = progs[mode == MODE_ALLREDUCE ? N : 0];
                const TreeProg& tp = tprog[mode == MODE_ALLREDUCE ? N : 0];
                auto opnd = [&](int code) -> Ref {
                    if (code >= 0) return code == me ? own(c, N, a) : leaf_slot(c, code, N, a);
                    return temp_slot(c, ~code, N);
                };
                if (tp.on) {
                    LocalOp op;
                    op.kind = L_TREE;
                    op.dst = mode == MODE_ALLREDUCE ? Ref{BUF_RECV, (uint64_t)N * g.irc + c.lo + a} : Ref{BUF_RECV, c.lo};
                    op.acc = opnd(tp.leaves[0]);
                    for (size_t j = 1; j < tp.leaves.size(); ++j) op.ins.push_back(opnd(tp.leaves[j]));
                    op.count = len;
                    op.comb = tp.comb;
                    op.swaps = tp.swaps;
                    st.post.push_back(op);
                    continue;
                }
                for (size_t t = 0; t < pr.size(); ++t) {
                    const bool last = t + 1 == pr.size();
                    Ref dst = last ? (mode == MODE_ALLREDUCE ? Ref{BUF_RECV, (uint64_t)N * g.irc + c.lo + a}
                                                             : Ref{BUF_RECV, c.lo})
                                   : temp_slot(c, (int)t, N);
                    std::vector<Ref> ins;
                    for (int x : pr[t].ins) ins.push_back(opnd(x));
                    LocalOp op = make_reduce(dst, opnd(pr[t].acc), ins, len, 0);
                    op.swap = pr[t].swap;
                    st.post.push_back(op);
                }
            }
        } else if (kind == F_DIST) {
            // equal pieces (every BASELINE size): one in-place ncclAllGather per chunk
            bool equal = coll_ag;
            for (int q = 1; q < n && equal; ++q) {
                uint64_t qa, ql;
                piece(c, q, &qa, &ql);
                equal = ql == len && qa == (uint64_t)q * len;
            }
            if (equal && len) {
                for (int N = 0; N < nchunks; ++N) st.allgathers.push_back({{BUF_RECV, (uint64_t)N * g.irc + c.lo}, len});
                return;
            }
            for (int q = 0; q < n; ++q) {
                if (q == me) continue;
                uint64_t qa, ql;
                piece(c, q, &qa, &ql);
                for (int N = 0; N < nchunks; ++N) {
                    const uint64_t base = (uint64_t)N * g.irc + c.lo;
                    if (len) st.sends.push_back({q, {BUF_RECV, base + a}, len});
                    if (ql) st.recvs.push_back({q, {BUF_RECV, base + qa}, ql});
                }
            }
        }
    };
    auto add = [&](int kind, int s2) {
        p.steps.emplace_back();
        Step& st = p.steps.back();
        st.label = std::string(kind == F_GATHER ? "gather" : "fdist") + "/s" + std::to_string(s2);
        emit(kind, sl[s2], st);
    };
    if (oneshot) {  // P gather steps, each followed by the whole slice's evaluation; nothing to distribute
        for (int s2 = 0; s2 < P; ++s2) add(F_GATHER, s2);
        return p;
    }
    if (merge && mode == MODE_ALLREDUCE) {
        // One RCCL group per step t: gather of slice t together with the allgather of slice t-2.
        // Slice t-2 was reduced (compute stream) while step t-1's group was on the links, so the
        // group rarely waits; the two flows share every link at once, and a call has P + 2
        // groups instead of 2P (fewer launch / drain bubbles).
        for (int t = 0; t < P + 2; ++t) {
            p.steps.emplace_back();
            Step& st = p.steps.back();
            if (t < P) {
                st.label = "gather/s" + std::to_string(t);
                emit(F_GATHER, sl[t], st);
            }
            if (t >= 2 && t - 2 < P) {
                st.label += std::string(st.label.empty() ? "" : ",") + "fdist/s" + std::to_string(t - 2);
                emit(F_DIST, sl[t - 2], st);
            }
            if (st.label.empty()) p.steps.pop_back();
        }
        return p;
    }
    // Step order G0, G1, D0, G2, D1, ..., D(P-1): gather s+1 needs nothing from the evaluation
    // of slice s, so with two streams it runs while slice s is reduced; allgather s follows it.
    for (int s2 = 0; s2 < P; ++s2) {
        add(F_GATHER, s2);
        if (mode == MODE_ALLREDUCE && s2 > 0) add(F_DIST, s2 - 1);
    }
    if (mode == MODE_ALLREDUCE) add(F_DIST, P - 1);
    return p;
}

}  // namespace chr
