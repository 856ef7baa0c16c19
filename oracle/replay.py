"""Pure-Python restatement of the reference's prioritized replay (SumTree + Memory).

TEST INFRASTRUCTURE ONLY: the checker of the device replay (csrc/qcart_replay.hip), imported by tests/.
Follows inverted harmonic oscillator/RL.py line for line:
  SumTree.__init__ :241-265, add :273-288, compiled_update :303-310, compiled_recalculate_structure
  :312-331, compiled_get_leaf :334-364; Memory.store :417-420, obtain_sample :423-432,
  batch_update :438-446, compiled_sampling :448-469, compiled_batch_update :471-475.
Substitutions (the reference's streams are not reproducible): np.random.rand(n) in
compiled_sampling -> injected uniforms; random.randrange(capacity) -> the Philox4x32-10 draw the device
uses (u = ((w0 << 32 | w1) >> 11) 2^-53 of counter (ctr, 0, 0, 0x200), slot = floor(u capacity)).
numpy 1.x scalar promotion is written out (float(...)) where numpy 2 would keep float32.
An out-of-range sibling (the last leaf as a left child when capacity is not a power of two) reads 0
here; the reference's numba code reads past the array there.
"""
from __future__ import annotations

import numpy as np

from . import oracle as O


def philox_u53(seed: int, ctr: int, i: int, tag: int) -> float:
    w = O.philox([ctr & 0xFFFFFFFF, ctr >> 32, i, tag], [seed & 0xFFFFFFFF, seed >> 32])
    return float(((int(w[0]) << 32 | int(w[1])) >> 11) * 2.0 ** -53)


class SumTree:
    def __init__(self, capacity: int, data_size: int, policy: str = "random", passes_before_random: float = 0.):
        self.capacity = capacity
        width = 1
        self.num_of_nodes = 0
        while width < capacity:
            self.num_of_nodes += width
            width *= 2
        self.tree = np.zeros(self.num_of_nodes + capacity, dtype=np.float64)
        self.data = np.zeros((capacity, data_size), dtype=np.float32)
        self.data_size = data_size
        self.len = 0
        self.passes = -passes_before_random
        self.sequential = policy == "sequential"
        self.data_pointer = 0

    def add(self, p, data, randrange):
        if self.sequential or self.passes < 1.:
            tree_idx = self.data_pointer + self.num_of_nodes
            self.data[self.data_pointer] = data
            self.update(tree_idx, p)
            self.data_pointer += 1
            self.passes += 1. / self.capacity
            if self.len != self.capacity:
                self.len += 1
            if self.data_pointer >= self.capacity:
                self.data_pointer = 0
        else:
            self.data_pointer = randrange(self.capacity)
            tree_idx = self.data_pointer + self.num_of_nodes
            self.data[self.data_pointer] = data
            self.update(tree_idx, p)

    def update(self, tree_idx, p):
        tree = self.tree
        tree[tree_idx] = p
        while tree_idx != 0:
            sib = tree_idx + 1 if tree_idx % 2 else tree_idx - 1
            s = tree[tree_idx] + (tree[sib] if sib < len(tree) else 0.)
            tree_idx = (tree_idx - 1) // 2
            tree[tree_idx] = s

    def get_leaf(self, v):
        tree = self.tree
        parent = 0
        while True:
            cl = 2 * parent + 1
            cr = cl + 1
            if cl >= len(tree):
                leaf = parent
                break
            if v <= tree[cl]:
                parent = cl
            else:
                v -= tree[cl]
                parent = cr
        data_idx = leaf - (len(tree) - self.capacity)
        if data_idx >= self.capacity:
            data_idx = self.capacity - 1
        return leaf, tree[leaf], self.data[data_idx]

    @property
    def total_p(self):
        return self.tree[0]


class Memory:
    alpha = 0.2
    beta = 0.2
    beta_increment_per_sampling = 0.001
    abs_err_upper = 1.

    def __init__(self, capacity, data_size, policy="sequential", passes_before_random=0., seed=0):
        self.tree = SumTree(capacity, data_size, policy, passes_before_random)
        self.max = 0.
        self.seed = seed
        self.rand_ctr = 0

    def _randrange(self, capacity):
        u = philox_u53(self.seed, self.rand_ctr, 0, 0x200)
        self.rand_ctr += 1
        return min(int(u * capacity), capacity - 1)

    def __len__(self):
        return self.tree.len

    def store(self, transition):
        p = self.abs_err_upper if self.max == 0. else self.max
        self.tree.add(p, transition, self._randrange)

    def obtain_sample(self, n, v_rand):
        self.beta = float(np.min([1., self.beta + self.beta_increment_per_sampling]))
        total_p, length = self.tree.total_p, len(self)
        pri_seg = total_p / n
        b_idx, isw = np.empty((n,), dtype=np.int32), np.empty((n,), dtype=np.float32)
        out = np.empty((n, self.tree.data_size), dtype=np.float32)
        for i in range(n):
            v = (i + v_rand[i]) * pri_seg
            idx, p, data = self.tree.get_leaf(v)
            assert p != 0.
            isw[i] = np.power(p / (total_p / length), -self.beta)
            b_idx[i], out[i] = idx, data
        return b_idx, isw, out

    def batch_update(self, tree_idx, abs_errors):
        epsilon = 0.00001 * self.max
        abs_errors = np.asarray(abs_errors, dtype=np.float32) + np.float32(epsilon)
        clipped = np.minimum(abs_errors, np.float32(self.abs_err_upper))
        ps = np.power(clipped, np.float32(self.alpha))
        for ti, p in zip(tree_idx, ps):
            self.tree.update(int(ti), float(p))
        self.max = 0.95 * max(self.max, float(np.max(clipped)))
