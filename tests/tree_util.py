"""Test-side helpers for the fused expression-tree op (chr_reduce_tree): a CPU evaluator of
the post-order stack program over the oracle's MPI_Reduce_local restatement, and a random
valid-program generator."""
import numpy as np

import pyoracle as po


def tree_ref(leaves, comb, swaps, dtype, op):
    """Evaluate the program: push leaf j, then comb[j] combines; a combine pops `in` and
    folds it into the running value below it: MPI_Reduce_local(in, run) -> run, or with the
    swap bit MPI_Reduce_local(run, in) -> in (MPICH_do_reduce order)."""
    stack, ci = [], 0
    for j, leaf in enumerate(leaves):
        stack.append(leaf.view(np.uint8).copy().view(leaf.dtype))  # keeps padding bytes (pair types)
        for _ in range(comb[j]):
            x = stack.pop()
            run = stack.pop()
            if swaps[ci]:
                po.reduce_local(run, x, dtype, op)
                stack.append(x)
            else:
                po.reduce_local(x, run, dtype, op)
                stack.append(run)
            ci += 1
    assert len(stack) == 1
    return stack[0]


def random_program(rng, nl, max_depth=4):
    """A random valid program with nl leaves and stack depth <= max_depth."""
    while True:
        comb, depth, ok = [], 0, True
        for j in range(nl):
            depth += 1
            if depth > max_depth:
                ok = False
                break
            left = nl - 1 - j  # leaves still to push
            lo = max(0, depth - 1 - left) if left == 0 else 0
            hi = min(3, depth - 1)
            c = depth - 1 if left == 0 else int(rng.integers(lo, hi + 1))
            if c > 3:
                ok = False
                break
            comb.append(c)
            depth -= c
        if ok and depth == 1:
            swaps = [int(x) for x in rng.integers(0, 2, nl - 1)]
            return comb, swaps
