"""oracle.reconcile_parallel (the full-size GPU checks' oracle): disjoint topology ranges
reconciled concurrently and concatenated equal one reconcile() call bit for bit."""
import numpy as np
import pytest

import oracle as O
from helpers import random_epoch_input
from kdtn import synth


@pytest.mark.parametrize("seed", [3, 11])
def test_parallel_equals_serial_random(seed):
    _, inp = random_epoch_input(seed, T=300, big=2)
    want = O.reconcile(inp)
    for th in (1, 3, 7):
        got = O.reconcile_parallel(inp, threads=th)
        assert not got.mismatches(want), th


@pytest.mark.parametrize("cfg,pods", [(2, 3000), (3, 3000), (4, 2000)])
def test_parallel_equals_serial_synthetic(cfg, pods):
    inp = synth.make(cfg, pods_per_shard=pods)
    want = O.reconcile(inp)
    got = O.reconcile_parallel(inp, threads=5)
    assert not got.mismatches(want)
    a, b = pods // 3, pods // 2                       # a sub-range, as the windows use it
    w = O.reconcile(inp, t_begin=a, t_end=b)
    g = O.reconcile_parallel(inp, t_begin=a, t_end=b, threads=4)
    assert not g.mismatches(w)
    assert np.array_equal(g.add_off, w.add_off)
