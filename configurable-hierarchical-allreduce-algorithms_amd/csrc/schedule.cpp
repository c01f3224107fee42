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

struct Builder {
    Plan& p;
    const Geometry& g;
    std::vector<Recexch> rx;
    std::vector<int> cnt, off;

    uint64_t chunk_pos(int N) const { return (uint64_t)g.P[N % g.b] + (uint64_t)(N / g.b); }
    // Region of lane blocks [o, o+c) in the block-major ACC, in elements.
    void region(int ph, int lane, uint64_t* start, uint64_t* len) const {
        const int o = off[(size_t)ph * g.b + lane], c = cnt[(size_t)ph * g.b + lane];
        const int e = std::min(o + c, g.b);
        *start = (uint64_t)g.P[o] * g.irc;
        *len = o < e ? (uint64_t)(g.P[e] - g.P[o]) * g.irc : 0;
    }
    void need_stage(uint64_t e) { p.stage_elems = std::max(p.stage_elems, e); }
};

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

}  // namespace

Plan build_plan(Mode mode, int n, int me, int k_in, int b, uint64_t count) {
    Plan p;
    p.mode = mode;
    p.rank = me;
    if (n < 1 || b < 1 || k_in < 2 || me < 0 || me >= n || b > n) {
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
    Builder B{p, g, {}, {}, {}};
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
    p.steps.resize(4 + g.nph);
    for (auto& s : p.steps) s.label.clear();
    if (g.total == 0) {
        p.steps.clear();
        return p;
    }
    const int node = me / b, lane = me % b;
    const Recexch& x = B.rx[lane];
    const bool participant = x.step1_sendto == -1;
    const uint64_t irc = g.irc, total = g.total;

    // ---- pre: SEND -> ACC in block-major order (:306-312 copy, re-laid out) ------------
    {
        std::vector<std::pair<uint64_t, uint64_t>> runs;  // (dst chunk, src chunk) starts
        std::vector<uint64_t> lens;
        for (int N = 0; N < g.nnodes; ++N) {
            const uint64_t d = B.chunk_pos(N), s = (uint64_t)N;
            if (!runs.empty() && runs.back().first + lens.back() == d && runs.back().second + lens.back() == s)
                ++lens.back();
            else {
                runs.push_back({d, s});
                lens.push_back(1);
            }
        }
        for (size_t i = 0; i < runs.size(); ++i)
            p.pre.push_back(make_copy({BUF_ACC, runs[i].first * irc}, {BUF_SEND, runs[i].second * irc},
                                      lens[i] * irc, 308));
    }

    // ---- step 0: step-1 fold (:315-335) -------------------------------------------------
    {
        Step& s = p.steps[0];
        s.label = "step1-fold";
        if (!participant) {
            s.sends.push_back({x.step1_sendto + b * node, {BUF_ACC, 0}, total});
        } else if (x.step1_nrecvs > 0) {
            std::vector<Ref> ins;
            for (int i = 0; i < x.step1_nrecvs; ++i) {
                s.recvs.push_back({x.step1_recvfrom[i] + b * node, {BUF_STAGE, (uint64_t)i * total}, total});
                ins.push_back({BUF_STAGE, (uint64_t)i * total});
            }
            B.need_stage((uint64_t)x.step1_nrecvs * total);
            s.post.push_back(make_reduce({BUF_ACC, 0}, {BUF_ACC, 0}, ins, total, 332));
        }
    }

    // ---- steps 1..nph: recexch reduce-scatter phases, highest digit first (:339-478) -----
    for (int ph = g.nph - 1, si = 1; ph >= 0; --ph, ++si) {
        Step& s = p.steps[si];
        s.label = "recexch-phase-" + std::to_string(ph);
        if (!participant) continue;
        uint64_t my_start, my_len;
        B.region(ph, lane, &my_start, &my_len);
        std::vector<Ref> ins;
        for (int i = 0; i < g.k - 1; ++i) {
            const int dst = x.step2_nbrs[ph][i];
            uint64_t st, len;
            B.region(ph, dst, &st, &len);
            if (len) s.sends.push_back({dst + b * node, {BUF_ACC, st}, len});  // :353 / :425
            if (my_len) {
                s.recvs.push_back({dst + b * node, {BUF_STAGE, (uint64_t)i * my_len}, my_len});  // :360 / :442
                ins.push_back({BUF_STAGE, (uint64_t)i * my_len});
            }
        }
        if (my_len) {
            B.need_stage((uint64_t)(g.k - 1) * my_len);
            s.post.push_back(make_reduce({BUF_ACC, my_start}, {BUF_ACC, my_start}, ins, my_len, 364));
        }
    }

    // ---- step nph+1: participants return the folded ranks' blocks (:378-385, :465-473) ---
    {
        Step& s = p.steps[1 + g.nph];
        s.label = "step1-return";
        if (!participant) {
            const uint64_t len = (uint64_t)g.S[lane] * irc;
            if (len) s.recvs.push_back({x.step1_sendto + b * node, {BUF_ACC, (uint64_t)g.P[lane] * irc}, len});
        } else {
            for (int i = 0; i < x.step1_nrecvs; ++i) {
                const int q = x.step1_recvfrom[i];
                const uint64_t len = (uint64_t)g.S[q] * irc;
                if (len) s.sends.push_back({q + b * node, {BUF_ACC, (uint64_t)g.P[q] * irc}, len});
            }
        }
    }

    // ---- step nph+2: inter-node linear reduce to the rotating lane roots (:498-539) ------
    {
        Step& s = p.steps[2 + g.nph];
        s.label = "inter-lane-reduce";
        for (int i = 0; i < g.S[lane]; ++i) {
            const int R = i * b + lane;  // root node of iteration i (:502)
            const uint64_t mine = ((uint64_t)g.P[lane] + i) * irc;
            if (node != R) {
                s.sends.push_back({R * b + lane, {BUF_ACC, mine}, irc});  // :534
                continue;
            }
            std::vector<Ref> ins;
            for (int X = 0, slot = 0; X < g.nnodes; ++X) {  // stage order (:523-530)
                if (X == R) continue;
                s.recvs.push_back({X * b + lane, {BUF_STAGE, (uint64_t)slot * irc}, irc});  // :517
                ins.push_back({BUF_STAGE, (uint64_t)slot * irc});
                ++slot;
            }
            B.need_stage((uint64_t)(g.nnodes - 1) * irc);
            if (mode == MODE_ALLREDUCE) {
                // Reduce straight into the chunk's final place in recvbuf.
                s.post.push_back(make_reduce({BUF_RECV, (uint64_t)R * irc}, {BUF_ACC, mine}, ins, irc, 529));
            } else {
                s.post.push_back(make_reduce({BUF_ACC, mine}, {BUF_ACC, mine}, ins, irc, 552));
                // own sub-block (reduce_scatter_radix_batch.cpp:572-579, :625-627)
                s.post.push_back(make_copy({BUF_RECV, 0}, {BUF_ACC, mine + (uint64_t)lane * recvcount}, recvcount, 625));
            }
        }
    }

    // ---- step nph+3: distribution.  Allreduce: phases 3-4 (:552-756) replaced by a direct
    //      owner->all copy of each reduced chunk over the xGMI mesh (pure data movement).
    //      Reduce-scatter: the intra k-nomial scatter (:572-627) as direct owner->lane sends.
    {
        Step& s = p.steps[3 + g.nph];
        s.label = "distribute";
        if (mode == MODE_ALLREDUCE) {
            for (int N = 0; N < g.nnodes; ++N) {
                const int owner = N * b + N % b;
                if (me == owner) {
                    for (int Y = 0; Y < n; ++Y)
                        if (Y != me) s.sends.push_back({Y, {BUF_RECV, (uint64_t)N * irc}, irc});
                } else {
                    s.recvs.push_back({owner, {BUF_RECV, (uint64_t)N * irc}, irc});
                }
            }
        } else {
            const int owner = node * b + node % b;
            if (me == owner) {
                const uint64_t mine = ((uint64_t)g.P[lane] + node / b) * irc;
                for (int j = 0; j < b; ++j)
                    if (j != lane) s.sends.push_back({node * b + j, {BUF_ACC, mine + (uint64_t)j * recvcount}, recvcount});
            } else {
                s.recvs.push_back({owner, {BUF_RECV, 0}, recvcount});
            }
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
      << " steps=" << p.steps.size() << "\n";
    auto local = [&](const LocalOp& op) {
        if (op.kind == L_COPY) {
            o << "copy " << buf_name(op.dst.buf) << " " << op.dst.off << " " << buf_name(op.acc.buf) << " "
              << op.acc.off << " " << op.count << "\n";
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
