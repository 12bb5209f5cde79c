"""CPU checks of bench.py's roofline bookkeeping (no GPU): the compulsory
bytes SURVEY §8(d) defines, the one-launch-per-block family merge, the kernel
instance the roofline's measured traffic is looked up under, and that lookup
against the committed profiles/pmc_traffic.json."""
import json
import os

import numpy as np
import pytest

import bench
import dstd_native as native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _opts(cfg):
    d = np.load(os.path.join(ROOT, "tests", "golden", bench.CONFIGS[cfg][0]), allow_pickle=False)
    return {k[4:]: d[k].item() for k in d.files if k.startswith("opt/")}


def test_compulsory_bytes_match_survey():
    assert bench.op_compulsory_bytes(64, 64, 35, 22) == 394_240  # one 64->64 DSTDGC / DSTDGCB, per sequence
    assert bench.model_compulsory_bytes(_opts("h36m")) == 2_393_160  # the whole H36M forward


@pytest.mark.parametrize("cfg", ["h36m", "cmu", "3dpw"])
def test_block_merge_is_one_family_per_block(cfg):
    o = _opts(cfg)
    blocks = bench.model_block_bytes(o, True)
    merged = bench.merge_blocks(blocks, True)
    assert len(merged) == len(blocks) == o["num_layers"] + 2
    for b, m in zip(blocks, merged):
        assert native.KIND_BLOCK in m
        for k in (native.KIND_SPATIAL, native.KIND_TEMPORAL, native.KIND_ADJ_T, native.KIND_ADJ_S):
            assert k not in m
        assert m[native.KIND_BLOCK] == sum(b.values())  # nothing lost, nothing counted twice
    # phase 3: every block after the first gets its spatial planes from the previous launch
    assert all(b[native.KIND_ADJ_S] == 0 for b in blocks[1:]) and blocks[0][native.KIND_ADJ_S] > 0


def test_block_roofline_instance_and_traffic_lookup():
    inst = bench.split_instance(native.KIND_BLOCK, 35, 22)
    assert inst == "k_block_fused<35, 22, 64, 64, 1>"
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        d = json.load(f)
    assert bench.load_traffic("block_split", inst) == d["by_kernel"][inst]["hbm_bytes_per_launch"]
    # the block launch moves at least its compulsory bytes
    assert bench.load_traffic("block_split", inst) >= bench.op_compulsory_bytes(64, 64, 35, 22) * 256
