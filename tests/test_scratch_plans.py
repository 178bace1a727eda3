"""CPU: the multi-table operations' device scratch plans (no device work).

Each table's per-call scratch is one buffer handed out from offset 0, so within one CH-Q2 or
stock-level call it may have one user.  Round 5 faulted on exactly that (781d36d: CH-Q2's batch
buffers were carved from NATION's scratch while it held the NATION scan rows, so the mirrored
supp_stock_map offsets were overwritten and q2_gather read out of range).  The library's plans
pass stage_scratch_plan_check; the round-5 layout is refused; and a CH-Q2 call given one table
for two roles whose scratch users collide is refused before anything reaches the device."""
import ctypes

import numpy as np
import pytest

import stage

E_ARG, E_STATE = -1, -4
REGION, NATION, SUPPLIER, ITEM, STOCK = range(5)


def plan_check(op, roles=None):
    L = stage.lib()
    if roles is None:
        return L.stage_scratch_plan_check(op, None, 0), ""
    r = np.ascontiguousarray(roles, np.int32)
    rc = L.stage_scratch_plan_check(op, r.ctypes.data, r.size)
    return rc, L.stage_last_error().decode()


def test_library_plans_are_disjoint():
    assert plan_check(0)[0] == 0  # CH-Q2: batch buffers (SUPPLIER), REGION / NATION scan rows, staging (ITEM)
    assert plan_check(1)[0] == 0  # stock-level: its batch buffers (DISTRICT)
    assert plan_check(0, [SUPPLIER, REGION, NATION, ITEM])[0] == 0  # the same plan spelled out


def test_round5_fault_layout_is_refused():
    """the layout before 781d36d: the batch buffers in NATION's scratch"""
    rc, msg = plan_check(0, [NATION, REGION, NATION, ITEM])
    assert rc == E_ARG
    assert "batch buffers" in msg and "NATION scan rows" in msg
    rc, msg = plan_check(0, [REGION, REGION, NATION, ITEM])  # ... or REGION's
    assert rc == E_ARG and "REGION scan rows" in msg
    assert plan_check(0, [SUPPLIER, REGION])[0] == E_ARG  # one role per user of the plan
    assert plan_check(7)[0] == E_ARG


def _ch_tables():
    t = {"region": stage.Table(key_width=8, payload_size=64), "nation": stage.Table(key_width=8, payload_size=64),
         "supplier": stage.Table(key_width=8, payload_size=64), "item": stage.Table(key_width=8, payload_size=128),
         "stock": stage.Table(key_width=16, payload_size=64)}
    return t


def _q2(t, roles):
    map_off = np.zeros(10001, np.uint32)
    rids = np.array([5], np.uint32)
    out = np.zeros((1, 16), stage.Q2_REC_DTYPE)
    n = ctypes.c_uint64()
    ab = np.zeros(1, np.int32)
    L = stage.lib()
    rc = L.stage_ch_query2_batch(*[t[r].h for r in roles], map_off.ctypes.data, None, 3, rids.ctypes.data, 1,
                                 out.ctypes.data, 16, ctypes.byref(n), ab.ctypes.data, None)
    return rc, L.stage_last_error().decode()


def test_ch_query2_refuses_aliased_tables_before_device_work():
    t = _ch_tables()  # host tables only: nothing is published to a device
    order = ["region", "nation", "supplier", "item", "stock"]
    rc, msg = _q2(t, order)
    assert rc == E_STATE  # the plan check passed; the tables are simply not on a device
    for aliased in (["region", "nation", "nation", "item", "stock"],     # supplier := nation
                    ["region", "region", "supplier", "item", "stock"],   # nation := region
                    ["region", "nation", "supplier", "supplier", "stock"]):  # item := supplier
        rc, msg = _q2(t, aliased)
        assert rc == E_ARG and "scratch alias" in msg, (aliased, rc, msg)
    # one table for two roles whose users do not collide (stock has no scratch user) is allowed
    rc, _ = _q2(t, ["region", "nation", "supplier", "item", "item"])
    assert rc == E_STATE
