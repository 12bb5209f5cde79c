"""Oracle package -- test infrastructure only (see dstdgcn_oracle.py header).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything from here; the product path under ``dstd-gcn_amd/``
never does.
"""
