"""bench.py's command line and step schedule (CPU only): the driver's fixed
command `bench.py --gpus 1 --steps 20 --warmup 5` must parse and time
exactly --steps leapfrog steps whatever Nt the thermalisation ends with."""
import pytest

import bench


def test_driver_argv_parses():
    a = bench.parse(["--gpus", "1", "--steps", "20", "--warmup", "5"])
    assert (a.gpus, a.steps, a.warmup, a.Nt) == (1, 20, 5, 10)


@pytest.mark.parametrize("argv", [["--steps", "0"], ["--warmup", "-1"], ["--Nt", "0"]])
def test_bad_counts_rejected(argv):
    with pytest.raises(SystemExit):
        bench.parse(argv)


@pytest.mark.parametrize("steps", [1, 5, 9, 10, 20, 23, 50, 101])
@pytest.mark.parametrize("Nt", [1, 4, 10, 12, 17, 40])
def test_schedule_is_exact(steps, Nt):
    pieces = bench.schedule(3, steps, Nt)
    assert sum(n * nt for _, n, nt in pieces) == steps
    # draw indices are consecutive from `first`, every trajectory but the last has Nt steps
    first = 3
    for f, n, nt in pieces:
        assert f == first
        first += n
    assert all(nt == Nt for _, _, nt in pieces[:-1])
    assert bench.n_draws(pieces) == -(-steps // Nt)


def test_warmup_rounds_up_to_sweeps():
    Nt = 10
    warm = bench.schedule(0, -(-5 // Nt) * Nt, Nt)
    assert warm == [(0, 1, 10)]
