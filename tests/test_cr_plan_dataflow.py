"""CPU check of the cyclic-reduction schedule the C ABI builds (no device):
dwh_debug_cr_plan_check builds the plan dwh_create would and verifies its
dataflow -- every block a launch reads was written by an earlier launch (or
is a level-0 / static block), no launch reads a block it writes (other than a
task's own accumulate input or an in-place inversion), no two tasks of one
launch write the same block, and the force / E_f gathers read written blocks.
This is what the side-work placement (products run inside later inversion
launches) must respect; a schedule that read U'/L' in the launch producing
them would fail here before it could race on the GPU."""
import ctypes as C

import numpy as np
import pytest

LATTICES = [(4, 1), (4, 2), (3, 3), (5, 7), (8, 8), (6, 9), (17, 4), (20, 6), (32, 2), (32, 3), (32, 5),
            (32, 16), (32, 31), (32, 32), (32, 33), (40, 3), (48, 12), (64, 2), (64, 9)]


def check(lib, Lx, Ly, nbatch, side, inv0):
    stats = np.zeros(6, dtype=np.int64)
    rc = lib.dwh_debug_cr_plan_check(Lx, Ly, nbatch, side, inv0, stats.ctypes.data_as(C.c_void_p))
    return rc, stats, lib.dwh_last_error(None).decode()


@pytest.mark.parametrize("Lx,Ly", LATTICES)
@pytest.mark.parametrize("nbatch", [14, 56])
@pytest.mark.parametrize("sparse0", ["1", "0"])
@pytest.mark.parametrize("merge", ["8", "0"])
def test_cr_schedule_dataflow(dwhmc, monkeypatch, Lx, Ly, nbatch, sparse0, merge):
    monkeypatch.setenv("DWHMC_CR_SPARSE0", sparse0)
    monkeypatch.setenv("DWHMC_CR_MERGE", merge)
    lib = dwhmc.load_library()
    for side in (0, 1):
        for inv0 in (0, 1):
            rc, stats, err = check(lib, Lx, Ly, nbatch, side, inv0)
            assert rc == 0, (Lx, Ly, nbatch, side, inv0, err)
            assert stats[0] == stats[1] + stats[3] and stats[1] >= 1


def test_cr_schedule_c3_shape(dwhmc, monkeypatch):
    """The C3 plan (L = 32, 14 poles): 6 inversion launches, 4 of them with
    side work, 19 product launches, two of them the sparse level-0 stages
    (level 0 makes no U'/L' side work for the level-1
    inversion): the backward merge (round 6) runs the G_ee stage of the m = 2
    level inside the m = 4 level's first stage, 25 launches instead of 26
    (DWHMC_CR_MERGE=0), 24 with DWHMC_CR_MERGE=8 (the m = 4 one too); without
    side work the merge products sit in the top level's D' stage only while
    they stay small (BP = 64: none); the dense level 0 (DWHMC_CR_SPARSE0=0)
    puts side work on 5."""
    lib = dwhmc.load_library()
    monkeypatch.delenv("DWHMC_CR_SPARSE0", raising=False)
    monkeypatch.delenv("DWHMC_CR_MERGE", raising=False)
    rc, stats, err = check(lib, 32, 32, 14, 1, 1)
    assert rc == 0, err
    assert list(stats[:4]) == [25, 6, 4, 19]
    monkeypatch.setenv("DWHMC_CR_MERGE", "8")
    rc, stats, err = check(lib, 32, 32, 14, 1, 1)
    assert rc == 0, err
    assert list(stats[:4]) == [24, 6, 4, 18]
    monkeypatch.delenv("DWHMC_CR_MERGE", raising=False)
    rc, stats, err = check(lib, 32, 32, 14, 0, 1)
    assert rc == 0, err
    assert list(stats[:4]) == [26, 6, 0, 20]
    # four chains (56 batch items): one merge fits the idle CUs
    rc, stats, err = check(lib, 32, 32, 56, 1, 1)
    assert rc == 0, err
    assert list(stats[:4]) == [25, 6, 3, 19]
    monkeypatch.setenv("DWHMC_CR_MERGE", "0")
    rc, stats, err = check(lib, 32, 32, 14, 1, 1)
    assert rc == 0, err
    assert list(stats[:4]) == [26, 6, 4, 20]
    monkeypatch.setenv("DWHMC_CR_SPARSE0", "0")
    rc, stats, err = check(lib, 32, 32, 14, 1, 1)
    assert rc == 0, err
    assert list(stats[:4]) == [26, 6, 5, 20]
    monkeypatch.setenv("DWHMC_CR_MERGE", "8")
    rc, stats, err = check(lib, 32, 32, 14, 1, 1)
    assert rc == 0, err
    assert list(stats[:4]) == [24, 6, 5, 18]


def test_cr_schedule_rejects_wide_rows(dwhmc):
    lib = dwhmc.load_library()
    rc, _, err = check(lib, 65, 4, 14, 1, 1)
    assert rc != 0 and "too wide" in err


def default_rows(Lx, Ly):
    """Lattice rows per CR block the context picks (cr_rows_per_block): as many
    as fill a 16-site block half, lowered to a divisor of Ly."""
    r = max(1, 16 // Lx)
    while r > 1 and Ly % r:
        r -= 1
    return r


def plan_flops(lib, Lx, Ly, nbatch, side, inv0):
    out = np.zeros(3)
    rc = lib.dwh_debug_cr_plan_flops(Lx, Ly, nbatch, side, inv0, out.ctypes.data_as(C.c_void_p))
    assert rc == 0, lib.dwh_last_error(None).decode()
    return out


@pytest.mark.parametrize("Lx,Ly", [(4, 1), (4, 2), (3, 3), (8, 8), (17, 4), (20, 6), (24, 24), (32, 5),
                                   (32, 32), (32, 33), (48, 48), (64, 9)])
@pytest.mark.parametrize("nbatch", [13, 52])
@pytest.mark.parametrize("sparse0", ["1", "0"])
def test_cr_plan_flops_independent_count(dwhmc, monkeypatch, Lx, Ly, nbatch, sparse0):
    """The plan's per-stage algorithmic flops (what the cr_* timers, bench.py's
    alg_flops_per_step and the roofline use) against tools/cr_model.py's count
    of the recursion: moving products into inversion launches (side work)
    must move their flops with them, never drop them.
    With the sparse level 0 (default for even block rows >= 4) the count of
    its sparse products comes from the nonzeros of an oracle-assembled BdG
    matrix, not from the library's tables."""
    from tools.cr_model import cr_flop_count
    monkeypatch.setenv("DWHMC_CR_SPARSE0", sparse0)
    lib = dwhmc.load_library()
    for side in (0, 1):
        # the backward merge's products depend on where they can run (side work or not)
        inv_ref, prod_ref = cr_flop_count(Lx, Ly, default_rows(Lx, Ly), sparse0=sparse0 == "1", nbatch=nbatch,
                                          side=bool(side))
        for inv0 in (0, 1):
            inv, prod, side_f = plan_flops(lib, Lx, Ly, nbatch, side, inv0)
            assert inv == pytest.approx(inv_ref, rel=1e-12), (side, inv0)
            assert prod + side_f == pytest.approx(prod_ref, rel=1e-12), (side, inv0, prod, side_f)
            if not side:
                assert side_f == 0.0


def test_cr_plan_flops_c3_side_work(dwhmc):
    """At C3 (L = 32, 13 poles) the side work carries real products (the W
    products of levels 1 and 2 and U'/L' of levels 1-3: 16 % of the product
    flops with the sparse level 0, which leaves no level-0 side work)."""
    lib = dwhmc.load_library()
    inv, prod, side_f = plan_flops(lib, 32, 32, 13, 1, 1)
    assert side_f > 0.12 * (prod + side_f)


@pytest.mark.parametrize("Lx,Ly,rows,blocks", [(8, 8, 2, 4), (4, 4, 4, 1), (4, 6, 3, 2), (6, 9, 1, 9), (5, 7, 1, 7),
                                               (3, 3, 3, 1), (16, 16, 1, 16), (8, 5, 1, 5), (2, 10, 5, 2)])
def test_cr_default_rows_per_block(dwhmc, monkeypatch, Lx, Ly, rows, blocks):
    """Narrow lattices (Lx <= 8) group rows into 16-site blocks by default
    (cr_rows_per_block): 8 x 8 (C1) runs 4 two-row blocks, one CR level less
    than 8 half-empty one-row blocks; the inversion count of the plan shows the
    block count."""
    assert default_rows(Lx, Ly) == rows
    lib = dwhmc.load_library()
    rc, st, err = check(lib, Lx, Ly, 10, 1, 1)
    assert rc == 0, err
    m, ninv = blocks, 0
    while m > 1:
        ninv += 1
        m = (m + 1) // 2
    assert st[1] == ninv + 1
