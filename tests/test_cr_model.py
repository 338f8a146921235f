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
