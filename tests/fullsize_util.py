"""Bit-exact checks of BASELINE-size collectives against the C oracle, window by window.

A full-size call (C4: 8 ranks x 1 GiB fp32; C5: 8 ranks x 1 GiB bf16) is checked over its WHOLE
output, but the oracle runs on block windows (pyoracle.window_inputs): the outputs restricted to
the window [off, off + w) of every recvcount block equal the collective on the inputs restricted
to the same windows (the block-window property, pinned by
tests/test_oracle_golden.py::test_block_window_property).  Windows tile [0, recvcount), run in a
thread pool (ctypes releases the GIL inside liboracle), so host memory stays bounded and the
oracle's single-threaded C runs on several host cores.  Test infrastructure only.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import pyoracle as po


def windows(recvcount, width):
    return [(off, min(width, recvcount - off)) for off in range(0, recvcount, width)]


def check_allreduce(out_window, n, k, b, dtype, count, seed, pattern=po.PAT_UNIFORM, width=1 << 21, threads=16,
                    ranks=None, part=None):
    """out_window(r, off, w) -> numpy array of rank r's output at block_window(n, count // n, off, w).
    Returns the list of (rank, off) windows that differ from the oracle (empty = bit-exact).  part = (i, p): only
    every p-th window from the i-th (p processes checking one output together).  16 threads: the GPU box's CPU share
    (one process checking alone)."""
    rc = count // n
    check = list(range(n)) if ranks is None else list(ranks)

    def one(win):
        off, w = win
        ins = po.window_inputs(n, count, off, w, dtype, pattern, seed)
        want = po.allreduce_radix_batch(ins, k, b, dtype, "sum")
        del ins
        bad = []
        for r in check:
            got = out_window(r, off, w)
            if not np.array_equal(got.view(np.uint8), want[r].view(np.uint8)):
                bad.append((r, off))
        return bad

    wins = windows(rc, width)
    if part is not None:
        wins = wins[part[0]::part[1]]
    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(one, wins))
    return [x for bad in res for x in bad]


def check_reduce_scatter(out_window, n, k, b, dtype, recvcount, seed, pattern=po.PAT_UNIFORM, width=1 << 21,
                         threads=16):
    """out_window(r, off, w) -> rank r's output elements [off, off + w)."""
    count = recvcount * n

    def one(win):
        off, w = win
        ins = po.window_inputs(n, count, off, w, dtype, pattern, seed)
        want = po.reduce_scatter_radix_batch(ins, k, b, dtype, "sum")
        return [(r, off) for r in range(n)
                if not np.array_equal(out_window(r, off, w).view(np.uint8), want[r].view(np.uint8))]

    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(one, windows(recvcount, width)))
    return [x for bad in res for x in bad]
