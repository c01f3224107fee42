"""Test-side interpreter of libchiara plans (host only, no GPU).

Executes every rank's compiled plan (chr_plan_describe) with numpy buffers: messages
are matched exactly as the loopback/RCCL transports match them (same step, per-pair
order), local reductions go through the oracle's MPI_Reduce_local restatement.  This
checks the schedule compiler's data movement and reduction order on CPU.
"""
import numpy as np

import chiara_amd as ca
import pyoracle as po
import tree_util


def load_plans(mode, n, k, b, count, slices=1, schedule=None, commutative=True):
    return [ca.parse_plan(ca.describe_plan(mode, n, r, k, b, count, slices, schedule, commutative)) for r in range(n)]


def commutative(op):
    """MPI_Op_commutative of an oracle op name: every predefined op is; the test user op user_halfadd is created
    non-commutative, user_halfadd_c commutative (chiara_oracle.c orc_commutative)."""
    return op != "user_halfadd"


class RankState:
    def __init__(self, plan, send, recv_init, dtype):
        h = plan["header"]
        npdt = po.NP_DTYPES[dtype]
        self.buf = {
            "SEND": send,
            "RECV": recv_init if recv_init is not None else np.zeros(h["recv"], dtype=npdt),
            "ACC": np.zeros(h["acc"], dtype=npdt),
            "STAGE": np.zeros(max(h["stage"], 1), dtype=npdt),
        }

    def view(self, ref, n):
        name, off = ref
        return self.buf[name][off:off + n]


def run_local(st, op, dtype, rop):
    kind, dst, acc, n, ins = op[:5]
    if n == 0:
        return
    if kind == "tree":  # chr_reduce_tree: post-order stack program over the leaves
        comb, swaps = op[5]
        leaves = [st.view(ref, n) for ref in [acc] + list(ins)]
        st.view(dst, n)[:] = tree_util.tree_ref(leaves, comb, swaps, dtype, rop)
        return
    if kind == "copy2d":
        rows, dp, sp = ins
        for r in range(rows):
            st.view((dst[0], dst[1] + r * dp), n)[:] = st.view((acc[0], acc[1] + r * sp), n).copy()
        return
    if kind == "copy":
        st.view(dst, n)[:] = st.view(acc, n).copy()
        return
    # Model of the device launcher: at most FAN_IN inputs per pass; each pass reads its inputs
    # and writes dst before the next pass reads (launch_reduce chains through dst).
    cur = acc
    for g0 in range(0, max(len(ins), 1), FAN_IN):
        a = st.view(cur, n).copy()
        grp = [st.view(r, n).copy() for r in ins[g0:g0 + FAN_IN]]
        if kind == "reduce_sw":  # running value first: a = MPI_Reduce_local(a -> in, x -> inout)
            for x in grp:
                po.reduce_local(a, x, dtype, rop)
                a = x
        elif grp:
            po.reduce_multi(a, grp, dtype, rop)
        st.view(dst, n)[:] = a
        cur = dst


FAN_IN = 8  # kMaxFanIn in csrc/reduce_kernels.hip


def execute(plans, sends, dtype, rop, inplace=False, recv_init=None):
    """recv_init: optional initial RECV buffer per rank (its size may exceed what the plan writes)."""
    n = len(plans)
    states = []
    for r in range(n):
        if recv_init is not None and not inplace:
            st = RankState(plans[r], sends[r], recv_init[r], dtype)
        elif inplace and plans[r]["header"]["mode"] == ca.MODE_ALLGATHER:
            # MPI_IN_PLACE allgather: the own block already sits at recv + r*sendcount
            c = sends[r].size
            buf = np.zeros(plans[r]["header"]["recv"], dtype=sends[r].dtype)
            buf[r * c:(r + 1) * c] = sends[r]
            st = RankState(plans[r], buf[r * c:(r + 1) * c], buf, dtype)
        elif inplace:
            buf = sends[r].copy()
            st = RankState(plans[r], buf, buf, dtype)
        else:
            st = RankState(plans[r], sends[r], None, dtype)
        states.append(st)
    for r in range(n):
        for op in plans[r]["pre"]:
            run_local(states[r], op, dtype, rop)
    nsteps = len(plans[0]["steps"])
    assert all(len(p["steps"]) == nsteps for p in plans)
    for si in range(nsteps):
        used = [[False] * len(plans[r]["steps"][si]["sends"]) for r in range(n)]
        payload = []
        for r in range(n):
            for peer, ref, cnt in plans[r]["steps"][si]["recvs"]:
                qs = plans[peer]["steps"][si]["sends"]
                j = next(j for j, s in enumerate(qs) if not used[peer][j] and s[0] == r)
                assert qs[j][2] == cnt, "send/recv size mismatch"
                used[peer][j] = True
                payload.append((r, ref, states[peer].view(qs[j][1], cnt).copy()))
        assert all(all(u) for u in used), f"unmatched send in step {si}"
        for r, ref, data in payload:
            states[r].view(ref, data.size)[:] = data
        for ci in range(len(plans[0]["steps"][si].get("allgathers", []))):  # in-place allgather collectives
            blocks = []
            for r in range(n):
                (buf, off), cnt = plans[r]["steps"][si]["allgathers"][ci]
                blocks.append(states[r].view((buf, off + r * cnt), cnt).copy())
            for r in range(n):
                (buf, off), cnt = plans[r]["steps"][si]["allgathers"][ci]
                for q in range(n):
                    states[r].view((buf, off + q * cnt), cnt)[:] = blocks[q]
        for r in range(n):
            for op in plans[r]["steps"][si]["post"]:
                run_local(states[r], op, dtype, rop)
    return [st.buf["RECV"] for st in states]


def simulate(mode, sends, k, b, dtype, op, inplace=False, slices=1, schedule=None):
    n = len(sends)
    rs = mode in ca.RS_MODES
    count = sends[0].size // n if rs else sends[0].size
    plans = load_plans(mode, n, k, b, count, slices, schedule, commutative(op))
    if plans[0]["header"]["error"]:
        raise ValueError(f"plan error {plans[0]['header']['error']}", plans[0]["header"]["error"])
    outs = execute(plans, sends, dtype, op, inplace)
    if rs:
        outs = [o[:count] for o in outs]
    return outs
