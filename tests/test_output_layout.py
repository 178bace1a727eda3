"""CPU: argument rules of stage_set_output_layout (no device call)."""
import pytest

import stage


def test_output_layout_arguments():
    t = stage.Table(key_width=8)
    t.load_ycsb(0, 1000, 8)
    assert t.stride == 1024
    t.set_output_layout(1008, 16)
    assert t.stride == 1008
    for bad in [(1000, 32), (1012, 32), (1008, 24)]:
        with pytest.raises(RuntimeError):
            t.set_output_layout(*bad)
    t.set_output_layout(0, 32)
    assert t.stride == 1024
    v = stage.Table(payload_size=8, leaf_node_size=4096, split_threshold=3072, merge_threshold=1024, key_width=0)
    with pytest.raises(RuntimeError):  # 16-B records: fixed-width keys in 64-slot leaves only
        v.set_output_layout(0, 16)
    v.set_output_layout(16, 32)
