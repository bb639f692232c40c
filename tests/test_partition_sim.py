"""tools/s42_partition_sim.py (the quotient's cache / partition simulation
behind DESIGN.md section 3.4, round 6): its Belady cache with bypass gives the
optimal miss count of a k-slot cache on small read streams (checked against
an exhaustive search over cache states), and the contiguous cut keeps program
order and covers every instruction once.  CPU only."""
import itertools
import os
import random
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import s42_partition_sim as sim  # noqa: E402


def optimal_misses(stream, slots):
    """minimum misses over every policy (any subset of the seen values may be
    held, a value enters only when it is read)"""
    states = {frozenset(): 0}
    for key in stream:
        nxt = {}
        for held, miss in states.items():
            m = miss + (key not in held)
            pool = sorted(held | {key})  # after the read: keep any subset (bypass or evict)
            for size in range(min(slots, len(pool)) + 1):
                for keep in itertools.combinations(pool, size):
                    s = frozenset(keep)
                    nxt[s] = min(nxt.get(s, 1 << 30), m)
        states = nxt
    return min(states.values())


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("slots", [1, 2, 3])
def test_belady_is_optimal(seed, slots):
    rng = random.Random(seed * 7 + slots)
    stream = [rng.randrange(5) for _ in range(9)]
    assert sim.belady(stream, slots) == optimal_misses(stream, slots)


def test_belady_known_cases():
    assert sim.belady(list("abab"), 1) == 3
    assert sim.belady(list("abab"), 2) == 2
    assert sim.belady(list("aaaa"), 1) == 1
    assert sim.belady([], 4) == 0


def test_contiguous_cut_covers_program_in_order():
    cost = [3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5, 8, 9, 7, 9]
    segs = sim.contiguous(len(cost), cost, 4)
    flat = [k for s in segs for k in s]
    assert flat == list(range(len(cost))) and 1 <= len(segs) <= 4
