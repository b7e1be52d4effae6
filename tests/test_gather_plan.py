"""CPU: the RCCL gather's protocol arithmetic (sbe_gather_plan, include/sbecodec.h), which
sbe_gather_encoded runs on every rank after the all-gather of {bytes, records, root capacities}:
prefix bases at world 1..8, roots other than 0, zero-record shards, and the ENOSPC decision on
both root capacities (bytes and offset entries) — identical on every rank, so no rank posts a
transfer the root refused."""
import random

import pytest

import sbecodec as C

ENOSPC = -3


def expect(ranks, root):
    bb, rb, b, m = [], [], 0, 0
    for r in ranks:
        bb.append(b)
        rb.append(m)
        b += r[0]
        m += r[1]
    bb.append(b)
    rb.append(m)
    cap, off_cap = ranks[root][2], ranks[root][3]
    rc = 0 if (b <= cap and m + 1 <= off_cap) else ENOSPC
    return rc, bb, rb, (b, m)


@pytest.mark.parametrize("world", range(1, 9))
def test_plan_matches_prefix_sums_every_root(world):
    rng = random.Random(world)
    for trial in range(40):
        shards = []
        for r in range(world):
            m = 0 if rng.random() < 0.25 else rng.randrange(1, 5000)  # zero-record shards included
            shards.append((256 * m if rng.random() < 0.5 else rng.randrange(34 * m, 600 * m + 1), m))
        total_b = sum(b for b, _ in shards)
        total_m = sum(m for _, m in shards)
        for root in range(world):
            # the root's capacities: exact, one short (bytes), one short (offsets), generous
            for cap, off_cap in ((total_b, total_m + 1), (total_b - 1, total_m + 1), (total_b, total_m),
                                 (total_b + 4096, total_m + 99)):
                if cap < 0:
                    continue
                ranks = [(b, m, cap if r == root else 0, off_cap if r == root else 0)
                         for r, (b, m) in enumerate(shards)]
                got = C.gather_plan(ranks, root)
                assert got == expect(ranks, root), (world, root, ranks)


def test_plan_is_the_same_on_every_rank():
    # every rank computes the plan from the same all-gathered array: the decision cannot differ
    ranks = [(2560, 10, 0, 0), (0, 0, 0, 0), (256, 1, 2816, 11), (0, 0, 0, 0)]
    outs = [C.gather_plan(ranks, 2) for _ in range(4)]
    assert all(o == outs[0] for o in outs)
    rc, bb, rb, tot = outs[0]
    assert rc == ENOSPC and tot == (2816, 11)  # 11 records need 12 offset entries
    ranks[2] = (256, 1, 2816, 12)
    assert C.gather_plan(ranks, 2) == (0, [0, 2560, 2560, 2816, 2816], [0, 10, 10, 11, 11], (2816, 11))


def test_plan_rejects_bad_arguments():
    assert C.gather_plan([(1, 1, 9, 9)], 1)[0] == -1
    assert C.gather_plan([(1, 1, 9, 9)], -1)[0] == -1
    assert C.gather_plan([], 0)[0] == -1


def test_empty_gather_fits_an_empty_root():
    # no records anywhere: the root still writes the closing offset (1 entry)
    ranks = [(0, 0, 0, 1), (0, 0, 0, 0)]
    assert C.gather_plan(ranks, 0) == (0, [0, 0, 0], [0, 0, 0], (0, 0))
    ranks[0] = (0, 0, 0, 0)
    assert C.gather_plan(ranks, 0)[0] == ENOSPC
