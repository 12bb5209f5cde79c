"""Skeleton priors for the spatial DSTDGC (constant tables).

Restates what ``Graph(layout).get_all_adjacency()`` returns in the reference
(model/layers/graph.py:4-348): per layout a stack of two 0/1 matrices
``[connect, part]`` of shape (2, V, V), where ``connect`` = identity + bone
edges (:313-319) and ``part`` = the hand-picked mirror / arm-leg edges without
self loops (:320-324).  Edges are stored here already mapped to the used-joint
index space; tests/test_tables.py checks the result against the reference's
own output captured in tests/golden/graphs.npz.
"""
import numpy as np

# (num_joints, bone edges, part edges) in used-joint indices
_LAYOUTS = {
    "h36m": (22,
             [(0, 1), (0, 8), (1, 2), (2, 3), (4, 5), (4, 8), (5, 6), (6, 7), (8, 9), (8, 10), (9, 10), (9, 12),
              (9, 17), (10, 11), (12, 13), (13, 14), (14, 15), (14, 16), (17, 18), (18, 19), (19, 20), (19, 21)],
             [(0, 4), (0, 13), (0, 18), (1, 5), (1, 14), (1, 19), (2, 6), (3, 7), (4, 13), (4, 18), (5, 14),
              (5, 19), (12, 17), (13, 18), (14, 19), (15, 20), (16, 21)]),
    "cmu": (25,
            [(0, 1), (0, 8), (1, 2), (2, 3), (4, 5), (4, 8), (5, 6), (6, 7), (8, 9), (9, 10), (9, 13), (9, 19),
             (10, 11), (11, 12), (13, 14), (14, 15), (15, 16), (15, 18), (16, 17), (19, 20), (20, 21), (21, 22),
             (21, 24), (22, 23)],
            [(0, 2), (0, 3), (0, 4), (0, 5), (0, 14), (0, 15), (0, 20), (0, 21), (1, 3), (1, 4), (1, 5), (1, 7),
             (1, 15), (1, 20), (2, 6), (4, 6), (4, 7), (4, 15), (4, 20), (4, 21), (5, 7), (5, 14), (5, 21),
             (13, 15), (13, 16), (13, 17), (13, 18), (13, 19), (13, 20), (14, 19), (14, 20), (14, 21), (15, 20),
             (15, 21), (16, 18), (16, 22), (17, 18), (17, 23), (18, 24), (19, 21), (19, 22), (19, 23), (19, 24),
             (22, 24), (23, 24)]),
    "3dpw": (23,
             [(0, 2), (0, 3), (1, 2), (1, 4), (2, 5), (3, 6), (4, 7), (5, 8), (6, 9), (7, 10), (8, 11), (8, 12),
              (8, 13), (11, 12), (11, 13), (11, 14), (12, 15), (13, 16), (15, 17), (16, 18), (17, 19), (18, 20),
              (19, 21), (20, 22)],
             [(0, 1), (0, 13), (0, 15), (1, 13), (1, 15), (3, 4), (3, 17), (3, 18), (4, 17), (4, 18), (6, 7),
              (6, 19), (6, 20), (7, 19), (7, 20), (9, 10), (12, 13), (15, 16), (17, 18), (19, 20), (21, 22)]),
}


def _symmetric(n, edges, self_loops):
    m = np.eye(n) if self_loops else np.zeros((n, n))
    for i, j in edges:
        m[i, j] = m[j, i] = 1.0
    return m


class Graph:
    """Same constructor / methods as the reference Graph used on the hot path."""

    def __init__(self, layout="h36m"):
        if layout not in _LAYOUTS:
            raise ValueError(f"Invalid layout {layout}")
        self.layout = layout
        self.num_joint, self._bones, self._parts = _LAYOUTS[layout]

    def get_adjacency_type(self, type="self"):
        if type == "self":
            return np.eye(self.num_joint)
        if type == "connect":
            return _symmetric(self.num_joint, self._bones, True)
        if type == "part":
            return _symmetric(self.num_joint, self._parts, False)
        if type == "all":
            return _symmetric(self.num_joint, self._bones + self._parts, True)
        raise ValueError(f"Invalid graph type {type}")

    def get_adjacency(self):
        return self.get_adjacency_type("all")

    def get_all_adjacency(self):
        return np.stack([self.get_adjacency_type("connect"), self.get_adjacency_type("part")], axis=0)
