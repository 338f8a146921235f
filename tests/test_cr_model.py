"""CPU check of the block cyclic-reduction algorithm the CR device path runs
(tools/cr_model.py restates the planner of csrc/dwhmc_api.cpp build_cr_plan):
ln|det| and the block-tridiagonal part of G = (H_BdG - i y)^-1 against dense
numpy for every chain shape the planner distinguishes (Ly = 1, 2, odd levels,
even levels, non-square)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import cr_model  # noqa: E402


@pytest.mark.parametrize("Lx,Ly", [(4, 1), (4, 2), (3, 3), (4, 4), (6, 5), (4, 6), (2, 7), (5, 8),
                                   (3, 12), (4, 16), (2, 2), (8, 3), (3, 24)])
def test_cr_selected_inverse_matches_dense(Lx, Ly):
    dl, err = cr_model.check(Lx, Ly, seed=Lx * 7 + Ly, y=0.4)
    assert dl <= 1e-11 * Lx * Ly
    assert err <= 1e-12


@pytest.mark.parametrize("Lx,Ly", [(4, 4), (3, 6), (2, 8), (3, 12), (2, 16), (3, 5), (2, 24), (4, 7)])
def test_cr_backward_merge_matches_dense(Lx, Ly):
    """The backward merge (build_cr_plan, round 6): with every level that may
    merge (depth >= 1, m <= 8) reading the G_ee of the level above through its
    expansion W G_ee = W Dinv + (W W1) G_ae + (W W2) G_ce, G_ee V = Dinv V +
    G_ea (V1 V) + G_ec (V2 V), the top-half recursion still gives the
    block-tridiagonal part of the dense inverse (odd and even level sizes)."""
    levels = []
    m = Ly
    while m > 1:
        levels.append(m)
        m = (m + 1) // 2
    merge = frozenset(d for d in range(1, len(levels) - 1) if levels[d] <= 8)
    assert merge or Ly <= 4
    err = cr_model.check_top_cr(Lx, Ly, seed=Lx + 3 * Ly, y=0.5, merge=merge)
    assert err <= 1e-11, err


def test_merge_depths_c3():
    """The C3 policy: L = 32 blocks at BP = 64, 12 poles with side work: the
    m = 4 level (depth 3) takes the G_ee stage above it (m = 8 too at
    DWHMC_CR_MERGE=8); four chains (48 items): depth 3; BP = 96 without side
    work: none; C2 (BP = 32, no side work): depths 1 and 2."""
    assert cr_model.merge_depths(32, 64, 12, True, True) == {3}
    assert cr_model.merge_depths(32, 64, 12, True, True, merge=8) == {2, 3}
    assert cr_model.merge_depths(32, 64, 48, True, True) == {3}
    assert cr_model.merge_depths(48, 96, 68, False, True) == set()
    assert cr_model.merge_depths(16, 32, 10, False, False) == {1, 2}
    assert cr_model.merge_depths(32, 64, 12, True, True, merge=False) == set()
