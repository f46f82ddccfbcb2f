"""Mixing-matrix (topology) builders -- host-side setup for the gossip / mixing kernels.

Reference: python/fedml/core/distributed/topology/topo_utils.py:6-94 and
symmetric_topology_manager.py:8-104.  Every builder returns the same float32 matrix as the
reference (pinned by tests/golden/topologies.npz), including its quirks:

* ``overlay_2d_torus`` keeps the reference's diagonal slip (it writes ``W[i, i]`` where it means
  ``W[idx, idx]``, topo_utils.py:16), so rows are not stochastic;
* ``SymmetricTopologyManager.generate_topology`` = ring plus ``neighbor_num`` nearest-neighbour
  links (Watts-Strogatz with no rewiring), self loop, each row scaled by 1 / (row count);
* ``overlay_random`` draws its graph with networkx's G(n, p) generator from Python's global
  ``random`` state, as the reference does.

The reference needed networkx < 3 (``nx.to_numpy_matrix``); nothing here does.
"""
from __future__ import annotations

import math

import numpy as np


def _ring_adjacency(n: int, half_width: int) -> np.ndarray:
    """0/1 adjacency of a ring lattice linking every node to its `half_width` nearest neighbours on
    each side (networkx.watts_strogatz_graph(n, 2 * half_width, p=0) without rewiring)."""
    a = np.zeros((n, n), dtype=np.float32)
    for i in range(n):
        for d in range(1, half_width + 1):
            j = (i + d) % n
            if j != i:
                a[i, j] = a[j, i] = 1.0
    return a


def overlay_2d_torus(node_num: int) -> np.ndarray:
    side = math.isqrt(node_num)
    assert side * side == node_num, "2d torus needs a square node count"
    w = np.zeros((node_num, node_num), dtype=np.float32)
    fifth = 1 / 5
    for r in range(side):
        for c in range(side):
            row = r * side + c
            w[r, r] = fifth  # reference quirk: the diagonal of row r, not of row `row`
            for nr, nc in (((r + 1) % side, c), ((r - 1) % side, c), (r, (c + 1) % side), (r, (c - 1) % side)):
                w[row, nr * side + nc] = fifth
    return w


def overlay_star(node_num: int) -> np.ndarray:
    w = np.zeros((node_num, node_num), dtype=np.float32)
    w[0, 0] = 1 / node_num
    for i in range(1, node_num):
        w[0, i] = w[i, 0] = 1 / node_num
        w[i, i] = 1 - 1 / node_num
    return w


def overlay_complete(node_num: int) -> np.ndarray:
    w = np.ones((node_num, node_num), dtype=np.float32)
    w /= node_num
    return w


def overlay_isolated(node_num: int) -> np.ndarray:
    return np.eye(node_num, dtype=np.float32)


def overlay_balanced_tree(node_num: int, degree: int = 2) -> np.ndarray:
    """Children of node i are 2i+1 .. 2i+degree (the reference's indexing, whatever the degree)."""
    w = np.zeros((node_num, node_num), dtype=np.float32)
    for i in range(node_num):
        for j in range(1, degree + 1):
            child = 2 * i + j
            if child >= node_num:
                break
            w[i, child] = 1 / (degree + 1)
    for i in range(node_num):
        w[i, i] = 1 - w[i, :].sum()
    return w


def overlay_random(node_num: int, probability: float = 0.5) -> np.ndarray:
    import networkx as nx
    g = nx.fast_gnp_random_graph(node_num, probability)
    w = np.asarray(nx.to_numpy_array(g), dtype=np.float32)
    deg = w.sum(1)
    for i in range(node_num):
        for j in range(node_num):
            if i != j and w[i, j] > 0:
                w[i, j] = 1 / (1 + max(deg[i], deg[j]))
        w[i, i] = 1 - w[i].sum()
    return w


class SymmetricTopologyManager:
    """Reference symmetric_topology_manager.py:8-104 (same constructor / methods)."""

    def __init__(self, n, neighbor_num=2):
        self.n = n
        self.neighbor_num = neighbor_num
        self.topology = []

    def generate_custom_topology(self, args):
        name = args.topo_name
        builders = {
            "2d_torus": lambda: overlay_2d_torus(self.n),
            "star": lambda: overlay_star(self.n),
            "complete": lambda: overlay_complete(self.n),
            "isolated": lambda: overlay_isolated(self.n),
            "balanced_tree": lambda: overlay_balanced_tree(self.n, self.neighbor_num),
            "random": lambda: overlay_random(self.n, args.topo_edge_probability),
        }
        if name == "ring":
            self.neighbor_num = 2
            self.generate_topology()
        elif name in builders:
            self.topology = builders[name]()
        else:
            raise Exception(name)

    def generate_topology(self):
        k = int(self.neighbor_num)
        if k > self.n:
            raise ValueError("neighbor_num > n")
        a = _ring_adjacency(self.n, 1)
        extra = np.ones((self.n, self.n), dtype=np.float32) - np.eye(self.n, dtype=np.float32) \
            if k == self.n else _ring_adjacency(self.n, k // 2)
        a = np.maximum(a, extra)
        np.fill_diagonal(a, 1)
        for i in range(self.n):
            a[i] = a[i] / int(np.count_nonzero(a[i] == 1))
        self.topology = a

    def get_in_neighbor_weights(self, node_index):
        return [] if node_index >= self.n else self.topology[node_index]

    def get_out_neighbor_weights(self, node_index):
        return [] if node_index >= self.n else self.topology[node_index]

    def get_in_neighbor_idx_list(self, node_index):
        w = self.get_in_neighbor_weights(node_index)
        return [j for j, v in enumerate(w) if v > 0 and j != node_index]

    def get_out_neighbor_idx_list(self, node_index):
        w = self.get_out_neighbor_weights(node_index)
        return [j for j, v in enumerate(w) if v > 0 and j != node_index]


def dense_rows(W: np.ndarray):
    """CSR of a dense mixing matrix, every column in ascending order, zeros included -- the
    reference's _pfedavg_mixing_ loop order (HierFedAvgCloudAggregator.py:182-193)."""
    n = W.shape[0]
    row_ptr = [i * W.shape[1] for i in range(n + 1)]
    cols = [j for _ in range(n) for j in range(W.shape[1])]
    vals = [float(W[i, j]) for i in range(n) for j in range(W.shape[1])]
    return row_ptr, cols, vals


def gossip_rows(W: np.ndarray, rows=None):
    """CSR of one DSGD/PushSum gossip step for the given receiver rows: [self (W_ii), then every
    in-neighbour j != i with W_ji != 0 in ascending j (the send order, decentralized_fl_api.py:
    115-120), weight W_ji] (client_dsgd.py:92-116)."""
    n = W.shape[0]
    rows = range(n) if rows is None else rows
    row_ptr, cols, vals = [0], [], []
    for i in rows:
        cols.append(i)
        vals.append(float(W[i, i]))
        for j in range(n):
            if j != i and W[j, i] != 0:
                cols.append(j)
                vals.append(float(W[j, i]))
        row_ptr.append(len(cols))
    return row_ptr, cols, vals
