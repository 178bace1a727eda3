"""GPU: bench.py's C3 leg (YCSB-B epochs) on a small table with both write paths -- the device
write path (stage_update_batch_device, adopted by the host in the background) and the host one
(stage_update_batch + incremental publish) -- each read checked against the oracle replaying
the same epochs."""
import numpy as np
import pytest

import bench
import oracle_lib as O
import stage

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("write_path", ["device", "host"])
def test_c3_leg_write_paths(gpu, write_path):
    rows = 400_000
    args = bench.parse(["--config", "c3", "--rows", str(rows), "--batch", str(1 << 15), "--write-path", write_path,
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline"])
    tab = stage.Table(key_width=8)
    tab.load_ycsb(0, rows, 8, mode=0)
    tab.sync()
    stream = stage.Stream()
    d, rec = bench.c3_leg(tab, args, stream, 4, args.steps, args.warmup)
    cfg = d["config"]
    assert d["self_check"] and d["value"] > 0 and d["ops_per_s_incl_writes"] == d["value"] and d["reads_per_s"] > 0
    assert cfg["write_path"] == write_path and 0 < cfg["updates_applied"] <= cfg["update_ops"]
    rcs = cfg["update_rc_counts"]
    assert sum(rcs.values()) == cfg["update_ops"] and rcs["ok"] == cfg["updates_applied"]
    # RunMixed's stream: each update's byte is a fresh next_char(), so an update finds its own
    # value already there only by chance (1/256 per update), not on every repeat of a hot key
    assert rcs.get("not_needed_update", 0) < 0.05 * cfg["update_ops"]
    # the oracle replays every epoch and answers the last epoch's sampled reads at their read ids
    orc = O.OracleTree()
    orc.load_ycsb(0, rows, 8, 0)
    applied = 0
    for ep in rec["record"]:
        deltas = np.repeat(ep["colb"][:, None], 100, 1)
        _, ok = orc.update_batch(ep["keys"], 8, 0, deltas, ep["rid"], ep["cid"])
        applied += ok
    keys, rids, st, got_rows = rec["check"]
    o_out, o_rec = orc.read_batch(keys, 8, rids)
    assert (o_out["status"] == st).all()
    assert (got_rows[:, :orc.row] == o_rec).all()
    assert cfg["updates_applied"] <= applied
