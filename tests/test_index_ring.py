"""Host logic of the row-index ring tracking (engine.TrainEngine._mark_built / _covered /
prefetch_index's range arithmetic) -- no GPU: a bare engine object with the ring's fields."""
import pytest

from rae.engine import TrainEngine


class _Ev:
    pass


def _eng(iw=8):
    e = TrainEngine.__new__(TrainEngine)
    e.index_window = iw
    e.index_overlap = True
    e._win = iw // 2
    e._ready = None
    e._neg_version = 0
    return e


def test_contiguous_builds_extend_the_range():
    e = _eng()
    e._mark_built(0, 4)
    assert e._covered(0, 4) and not e._covered(0, 5)
    ev = _Ev()
    e._mark_built(4, 8, ev)
    assert e._ready == (0, 8, 0, ev) and e._covered(2, 7)
    e._mark_built(8, 12)                 # ring of 8: batches 0..3 overwritten
    assert e._ready[:2] == (4, 12) and e._ready[3] is ev
    assert not e._covered(3, 5) and e._covered(4, 12)


def test_gap_or_new_negatives_start_a_new_range():
    e = _eng()
    e._mark_built(0, 4)
    e._mark_built(6, 9)
    assert e._ready[:2] == (6, 9)
    e._neg_version += 1                  # set_epoch_negatives / train_call
    assert not e._covered(6, 9)
    e._mark_built(9, 12)
    assert e._ready[:3] == (9, 12, 1)


def test_run_windows_are_half_the_ring():
    e = _eng(8)
    assert e.windows(0, 11) == [(0, 4), (4, 4), (8, 3)]
    e.index_overlap, e._win = False, 8
    assert e.windows(0, 11) == [(0, 8), (8, 3)]


@pytest.mark.parametrize("iw", [2, 8, 256, 2048])
def test_prefetch_never_overwrites_the_window_in_flight(iw):
    """run() prefetches the next window [b+n, b+n+n') while window [b, b+n) runs: the slots it
    writes (batch % iw) must not be the running window's."""
    win = iw // 2
    for n in range(1, win + 1):
        for n2 in range(1, win + 1):
            b = 5 * iw + 3
            running = {x % iw for x in range(b, b + n)}
            written = {x % iw for x in range(b + n, b + n + n2)}
            assert not running & written

