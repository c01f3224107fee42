"""The XCD-run workgroup map (reduce_common.hpp xcd_trip, xcd_trip_w) must cover every trip exactly once.

Streaming (nt) launches place each workgroup's trip by xcd_trip: runs of 2^cs consecutive trips per
XCD, identity for the blocks past the last whole 8 * 2^cs group.  A wrong map shows up as elements
never written or written twice.  The policy only engages on >= 40 MiB calls (bucket) / 64 MiB (trees), so these tests run in
a child process with CHR_REDUCE_NT=1 (nt at any size) and small runs (CHR_XCD_RUN_KIB) so that
ragged trip counts, partial groups and the tail trip all occur at oracle-sized inputs.  Bit-exact
against the oracle, for the bucket kernel (m = 1, 3, 7) and for batched trees (segments whose first
block sits anywhere in the XCD rotation)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

CHILD = r"""
import json, sys
import numpy as np
sys.path[:0] = [{here!r}, {oracle!r}, {pkg!r}]
import chiara_amd as ca
import gpu_util as gu
import pyoracle as po

bad = []
def same(got, ref, what):
    if not np.array_equal(got.view(np.uint32), ref.view(np.uint32)):
        bad.append(what)

# bucket kernel: m = 1 (U = 4, 4 KiB trips) and m = 3, 7 (U = 2, 2 KiB trips)
for m in (1, 3, 7):
    for n in (4096 * 8 * 3 + 17, 100003, (1 << 20) + 4 * 64 * 3 + 4, 1 << 21):
        acc = po.fill(n, "f32", 0, 11, 0)
        ins = [po.fill(n, "f32", 0, 11, r + 1) for r in range(m)]
        d_acc = gu.to_dev(acc)
        d_ins = [gu.to_dev(x) for x in ins]
        rc = ca.reduce_multi(d_acc, d_acc, d_ins, n, ca.FLOAT32, ca.SUM, gu.stream())
        gu.sync()
        if rc:
            bad.append(("rc", m, n, rc))
            continue
        same(gu.from_dev(d_acc, np.float32, n), po.reduce_multi(acc.copy(), ins, "f32", "sum"), ("vec", m, n))

# batched trees: 3 trees of 8 leaves (left folds) and of 3 leaves, ragged lengths
for nl in (3, 8):
    for n in (100003, (1 << 19) + 7):
        trees = [[po.fill(n, "f32", 0, 23 + t, j) for j in range(nl)] for t in range(3)]
        d_leaves = [[gu.to_dev(x) for x in tr] for tr in trees]
        d_outs = [gu.empty_dev(n * 4) for _ in trees]
        comb = [[0] + [1] * (nl - 1)] * 3
        rc = ca.reduce_tree_batch(d_outs, d_leaves, comb, None, n, ca.FLOAT32, ca.SUM, gu.stream())
        gu.sync()
        if rc:
            bad.append(("rc-tree", nl, n, rc))
            continue
        for t, tr in enumerate(trees):
            ref = po.reduce_multi(tr[0].copy(), tr[1:], "f32", "sum")
            same(gu.from_dev(d_outs[t], np.float32, n), ref, ("tree", nl, n, t))
print(json.dumps({{"bad": [str(b) for b in bad]}}))
"""


XCD_CONFIGS = [(4, 0, -1), (8, 0, -1), (64, 0, -1), (8, 3000, -1), (8, 0, 1), (0, 0, 2), (4, 3000, 3)]


def test_xcd_run_map_covers_every_trip():
    """Every (run_kib, max_vec, hand_shift) configuration in its own child process (the tuning variables are read
    once per process), the seven children at once: each is a second of small launches behind a second or two of
    start-up (the suite's time).  max_vec > 0 also caps the vectors per launch / tree segment
    (CHR_REDUCE_MAX_LAUNCH_VEC), so the paths that split > 32 GiB buckets into several launches and > 1 GiB trees
    into several segments (and several flushes of 8 segments) run at these sizes, with partial trips inside a call.
    hand_shift: the odd-XCD handover (xcd_trip_w) -- the policy's shift 6 engages at the 2^21-element bucket here;
    shifts 1-3 hand up to half of every odd XCD's share over, on run and identity maps."""
    code = CHILD.format(here=HERE, oracle=os.path.join(REPO, "oracle"),
                        pkg=os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd"))
    procs = []
    for run_kib, max_vec, hand_shift in XCD_CONFIGS:
        env = dict(os.environ, CHR_REDUCE_NT="1", CHR_XCD_RUN_KIB=str(run_kib),
                   CHR_REDUCE_MAX_LAUNCH_VEC=str(max_vec))
        if hand_shift >= 0:
            env["CHR_XCD_HAND_SHIFT"] = str(hand_shift)
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    failures = []
    for cfg, p in zip(XCD_CONFIGS, procs):
        try:
            out, err = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            p.kill()
            out, err = p.communicate()
            failures.append((cfg, "timeout"))
            continue
        if p.returncode != 0:
            failures.append((cfg, err[-3000:]))
            continue
        res = json.loads(out.strip().splitlines()[-1])
        if res["bad"]:
            failures.append((cfg, res["bad"][:10]))
    assert not failures, failures
