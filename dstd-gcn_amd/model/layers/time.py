"""Temporal prior for the temporal DSTDGC (constant table).

Restates ``Time(T).get_all_adjacency()`` (reference model/layers/time.py:37-41),
which stacks the "neighboor" matrix of :19-22.  That recipe is NOT a plain
tridiagonal band: it writes ``eye(T-1)`` into the [:-1, 1:] and [1:, :-1]
sub-blocks, overwriting the diagonal of the identity it started from, so the
result is asymmetric with only the corner diagonal entries left.
We reproduce it in closed form; tests/test_tables.py pins it to the
reference output for T in {6, 35, 40, 75}.
"""
import numpy as np


class Time:

    def __init__(self, seq_length):
        self.seq_length = seq_length
        self.input_length = 10  # hard-coded in the reference (:7); used only by unused types
        self.output_length = seq_length - self.input_length

    def _band(self):
        # Closed form of the reference's two overlapping block writes: the
        # sub-diagonal is complete, the super-diagonal and the diagonal keep
        # only their first / last entries.
        T = self.seq_length
        m = np.zeros((T, T))
        idx = np.arange(T - 1)
        m[idx + 1, idx] = 1.0
        m[0, 0] = m[0, 1] = 1.0
        m[T - 2, T - 1] = m[T - 1, T - 1] = 1.0
        return m

    def get_adjacency(self):
        return self._band()

    def get_adjacency_type(self, type="self"):
        T, k = self.seq_length, self.input_length
        if type == "self":
            return np.eye(T)
        if type == "neighboor":
            return self._band()
        if type == "inout":
            m = np.zeros((T, T))
            m[:k, k:] = 1
            m[k:, :k] = 1
            return m
        if type == "all":
            m = self._band()
            m[:k, k:] = 1
            m[k:, :k] = 1
            return m
        raise ValueError(f"Invalid graph type {type}")

    def get_all_adjacency(self):
        return self.get_adjacency_type("neighboor")[None]
