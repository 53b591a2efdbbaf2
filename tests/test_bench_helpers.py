"""bench.py's reporting helpers on CPU: the step-interval medians from out-of-order lane completions and the gathered
value_proj's algorithmic byte model."""
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


class _Ev:
    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


def test_completion_intervals_are_the_step_time_with_lanes_out_of_order():
    """Three lanes, a step every 10 ms, lanes finishing out of issue order (and in bursts): the windowed intervals
    over the sorted completions are all 10 ms, never negative (the round-3 median was -0.18 ms)."""
    b = _bench()
    start = _Ev(0.0)
    ends = [30.0, 20.0, 40.0, 60.0, 50.0, 70.0, 90.0, 80.0, 100.0, 120.0, 110.0, 130.0]  # issue order
    marks = [(None, _Ev(t)) for t in ends]
    iv = b.completion_intervals(start, marks, 3)
    assert len(iv) == len(ends) - 3 and min(iv) > 0
    assert np.allclose(iv, 10.0)
    # bursts: pairs finishing together every 20 ms -> still 10 ms per step over a window of the lanes
    burst = [10.0, 10.0, 30.0, 30.0, 50.0, 50.0, 70.0, 70.0]
    iv2 = b.completion_intervals(start, [(None, _Ev(t)) for t in burst], 2)
    assert np.allclose(iv2, 10.0)
    # one lane: consecutive differences
    assert b.completion_intervals(start, [(None, _Ev(t)) for t in (5.0, 9.0, 14.0)], 1) == [4.0, 5.0]


def test_value_proj_algo_bytes_counts_each_neighbourhood_pixel_once():
    """Scene 0: pixels (0,0), (1,1), (63,63) -> their in-map 3x3 neighbourhoods overlap: 4 + 9 - 4 + 4 = 13 distinct
    pixels; scene 1: two horizontally adjacent interior pixels -> 12. Bytes = (25 + 5 live rows) x 1 KB + the
    2304 x 256 x 4 B weight image."""
    b = _bench()
    taps = np.zeros(8, np.int32)
    taps[:3] = [0, 65, 4095]
    taps[4:6] = [4096 + 64 * 10 + 10, 4096 + 64 * 10 + 11]
    got = b.value_proj_algo_bytes(taps, np.array([3, 2], np.int32), 2)
    assert got == (25 + 5) * 1024 + 9 * 256 * 256 * 4


def test_gather_slices_ok_detects_a_wrong_slice():
    """bench.gather_slices_ok on one rank: the rank's own slice of the gathered rows against its local output."""
    import torch
    b = _bench()
    local = torch.full((4, 8, 3), 1.0)
    gathered = torch.cat([torch.zeros(4, 8, 3), local, torch.full((4, 8, 3), 2.0)])
    assert b.gather_slices_ok(gathered, local, 1, 4)
    assert not b.gather_slices_ok(gathered, local, 0, 4)
