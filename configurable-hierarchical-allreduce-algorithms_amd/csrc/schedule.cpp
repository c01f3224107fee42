// schedule.cpp -- radix/batch schedule compiler.  See schedule.hpp for the plan model
// and the block-major ACC layout.  Line citations are to
// Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp (the reduce-scatter file is
// line-for-line identical through phase 2).
#include "schedule.hpp"

#include <algorithm>
#include <cstdio>
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

enum Logical { S_FOLD, S_PHASE, S_RETURN, S_LANE, S_DIST1, S_DIST2, S_SCATTER };

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

    uint64_t chunk_pos(int N) const { return (uint64_t)g.P[N % g.b] + (uint64_t)(N / g.b); }
    // Region of lane blocks [o, o+c) of one slice, in elements.
    void region(const SliceCtx& c, int ph, int l, uint64_t* start, uint64_t* len) const {
        const int o = off[(size_t)ph * g.b + l], cn = cnt[(size_t)ph * g.b + l];
        const int e = std::min(o + cn, g.b);
        *start = c.acc_base + (uint64_t)g.P[o] * c.len;
        *len = o < e ? (uint64_t)(g.P[e] - g.P[o]) * c.len : 0;
    }
    const Recexch& x() const { return rx[lane]; }
    bool participant() const { return rx[lane].step1_sendto == -1; }

    // Pieces of the distribute scatter: [lo, lo+len) cut into n-1 pieces, 64-element aligned.
    void piece(const SliceCtx& c, int i, uint64_t* a, uint64_t* l) const {
        const uint64_t np = (uint64_t)(n - 1);
        auto cut = [&](uint64_t j) { return j == np ? c.len : (c.len * j / np) / 64 * 64; };
        *a = c.lo + cut((uint64_t)i);
        *l = cut((uint64_t)i + 1) - cut((uint64_t)i);
    }

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

Plan build_plan(Mode mode, int n, int me, int k_in, int b, uint64_t count, int slices) {
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

    // Logical steps, identical on every rank (so super-step numbering agrees globally).
    std::vector<std::pair<Logical, int>> L;
    const bool folds = B.rx[0].rem > 0;  // non-participants exist in every group
    if (folds) L.push_back({S_FOLD, 0});
    for (int ph = g.nph - 1; ph >= 0; --ph) L.push_back({S_PHASE, ph});
    if (folds) L.push_back({S_RETURN, 0});
    L.push_back({S_LANE, 0});
    if (mode == MODE_ALLREDUCE) {
        if (n > 1) L.push_back({S_DIST1, 0});
        if (n > 2) L.push_back({S_DIST2, 0});
    } else if (b > 1) {
        L.push_back({S_SCATTER, 0});
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
            static const char* names[] = {"fold", "phase", "return", "lane", "dist1", "dist2", "scatter"};
            st.label += std::string(st.label.size() > 0 ? "," : "") + names[L[ls].first] +
                        (L[ls].first == S_PHASE ? std::to_string(L[ls].second) : "") + "/s" + std::to_string(s);
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

std::string describe(const Plan& p) {
    std::ostringstream o;
    const Geometry& g = p.g;
    o << "plan mode=" << (int)p.mode << " error=" << p.error << " nranks=" << g.nranks << " rank=" << p.rank
      << " k=" << g.k << " b=" << g.b << " recvcount=" << g.recvcount << " irc=" << g.irc << " send=" << p.send_elems
      << " recv=" << p.recv_elems << " acc=" << p.acc_elems << " stage=" << p.stage_elems
      << " slices=" << p.slices << " steps=" << p.steps.size() << "\n";
    auto local = [&](const LocalOp& op) {
        if (op.kind == L_COPY) {
            o << "copy " << buf_name(op.dst.buf) << " " << op.dst.off << " " << buf_name(op.acc.buf) << " "
              << op.acc.off << " " << op.count << "\n";
        } else if (op.kind == L_COPY2D) {
            o << "copy2d " << buf_name(op.dst.buf) << " " << op.dst.off << " " << buf_name(op.acc.buf) << " "
              << op.acc.off << " " << op.count << " " << op.rows << " " << op.dpitch << " " << op.spitch << "\n";
        } else {
            o << "reduce " << buf_name(op.dst.buf) << " " << op.dst.off << " " << buf_name(op.acc.buf) << " "
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
        o << "step " << i << " " << (s.label.empty() ? "-" : s.label) << "\n";
        for (const Xfer& x : s.sends)
            o << "send " << x.peer << " " << buf_name(x.ref.buf) << " " << x.ref.off << " " << x.count << "\n";
        for (const Xfer& x : s.recvs)
            o << "recv " << x.peer << " " << buf_name(x.ref.buf) << " " << x.ref.off << " " << x.count << "\n";
        for (const LocalOp& op : s.post) local(op);
    }
    return o.str();
}

}  // namespace chr
