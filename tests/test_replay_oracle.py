"""CPU checks of the replay oracle (oracle/replay.py) on hand-built trees: the SumTree invariant,
stratified sampling of a known priority vector, the policy switch at passes >= 1, batch_update's
clipping / epsilon / max bookkeeping."""
import numpy as np
import pytest

from oracle.replay import Memory, SumTree


def test_sumtree_layout_and_invariant():
    t = SumTree(5, 2, "sequential")
    assert t.num_of_nodes == 7 and len(t.tree) == 12
    for i, p in enumerate([1., 2., 3., 4., 5.]):
        t.add(p, np.full(2, i, np.float32), None)
    assert t.total_p == 15.
    for node in range(t.num_of_nodes):
        l, r = 2 * node + 1, 2 * node + 2
        exp = (t.tree[l] if l < len(t.tree) else 0.) + (t.tree[r] if r < len(t.tree) else 0.)
        assert t.tree[node] == exp


def test_get_leaf_picks_by_cumulative_priority():
    t = SumTree(4, 1, "sequential")
    for i, p in enumerate([1., 0., 2., 1.]):
        t.add(p, np.array([i], np.float32), None)
    # cumulative [1, 1, 3, 4]: v in (0,1] -> slot 0, (1,3] -> slot 2, (3,4] -> slot 3
    assert t.get_leaf(0.5)[2][0] == 0 and t.get_leaf(1.0)[2][0] == 0
    assert t.get_leaf(1.5)[2][0] == 2 and t.get_leaf(3.5)[2][0] == 3


def test_policy_switch_and_wrap():
    m = Memory(10, 1, "random", passes_before_random=0.2, seed=3)
    # sequential while passes < 1, passes accumulating 1/capacity in floating point: -0.2 + 12 x 0.1
    # lands just below 1, so the reference makes 13 sequential adds (wrapping once) before going random
    passes, n_seq = -0.2, 0
    while passes < 1.:
        passes += 0.1
        n_seq += 1
    assert n_seq == 13
    for i in range(n_seq):
        m.store(np.array([i], np.float32))
    assert len(m) == 10 and m.tree.data_pointer == 3 and m.rand_ctr == 0
    assert list(m.tree.data[:, 0]) == [10, 11, 12, 3, 4, 5, 6, 7, 8, 9]
    m.store(np.array([99], np.float32))
    assert m.rand_ctr == 1 and 99 in m.tree.data[:, 0]


def test_batch_update_bookkeeping():
    m = Memory(8, 1, "sequential")
    for i in range(8):
        m.store(np.array([i], np.float32))
    idx = np.array([7, 8, 9], dtype=np.int32)      # leaves of slots 0, 1, 2
    m.batch_update(idx, np.array([0.5, 3.0, 1e-3], np.float32))
    assert m.max == pytest.approx(0.95)          # max(clipped) = 1 (3.0 clipped)
    assert m.tree.tree[8] == 1.0 and m.tree.tree[7] == pytest.approx(0.5 ** 0.2, rel=1e-6)
    # the next update adds epsilon = 1e-5 * max
    m.batch_update(np.array([10], np.int32), np.array([0.0], np.float32))
    assert m.tree.tree[10] == pytest.approx((1e-5 * 0.95) ** 0.2, rel=1e-5)


def test_sampling_is_stratified():
    m = Memory(16, 1, "sequential")
    for i in range(16):
        m.store(np.array([i], np.float32))
    idx, w, rows = m.obtain_sample(4, np.full(4, 0.5))
    assert list(rows[:, 0]) == [1, 5, 9, 13]   # v = 2, 6, 10, 14 on unit priorities; ties go left
    assert np.allclose(w, 1.0)
