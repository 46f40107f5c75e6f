"""Env sharding across ranks.

Env ``i`` of a job with ``total`` envs lives on rank ``i // (total / world)``
(contiguous blocks).  Each rank creates its handle with ``env_base`` = the
global index of its first env, so every Philox stream (reset noise, task
draws, teleport destinations, invalid-action draws, expert noise) is counted
by the GLOBAL env index under one shared seed, and a G-rank job reproduces the
single-GPU job of the same ``total`` bit for bit.  There is no per-step
exchange; the only collective is the eval all-gather
(``evaluation.gather_counters``).

Bit-identity does not depend on how envs are grouped into wavefronts: every
contact-solver choice of the maze step is made per lane (round 3,
``tests/test_locomaze_gpu.py::test_results_do_not_depend_on_wavefront_composition``).
Blocks are still kept multiples of 64 envs (``align``) so that every rank's
wavefronts are full.
"""

from __future__ import annotations


def shard(total, world, rank, align=64):
    """(env_base, num_envs) of `rank` for `total` envs over `world` ranks.

    Blocks are contiguous and, except possibly the last, multiples of `align`
    envs (full 64-lane wavefronts; results do not depend on the grouping).
    """
    total, world, rank = int(total), int(world), int(rank)
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f'rank {rank} out of range for world size {world}')
    if total < world:
        raise ValueError(f'cannot shard {total} envs over {world} ranks')
    per = -(-total // world)  # ceil
    per = -(-per // align) * align
    base = min(rank * per, total)
    n = max(0, min(per, total - base))
    if n == 0:
        raise ValueError(f'{total} envs leave rank {rank} of {world} empty at alignment {align}')
    return base, n


def rank_of_env(i, total, world, align=64):
    """Rank holding global env `i` (inverse of `shard`)."""
    base0, per = shard(total, world, 0, align)
    return int(i) // per
