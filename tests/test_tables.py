"""Graph / time priors vs the reference's own output (tests/golden/graphs.npz)."""
import numpy as np
import pytest

from conftest import load_npz
from model.layers.graph import Graph
from model.layers.time import Time


@pytest.mark.parametrize("layout", ["h36m", "cmu", "3dpw"])
def test_graph_tables(layout):
    d = load_npz("graphs.npz")
    np.testing.assert_array_equal(Graph(layout).get_all_adjacency(), d[f"graph_{layout}"])


@pytest.mark.parametrize("T", [6, 35, 40, 75])
def test_time_tables(T):
    d = load_npz("graphs.npz")
    np.testing.assert_array_equal(Time(T).get_all_adjacency(), d[f"time_{T}"])


def test_bad_layout():
    with pytest.raises(ValueError):
        Graph("nope")
