"""CPU: the dispatch rule C3's overlap rests on, checked on the built library.

Beside the read probe, whose 256-thread workgroups fill every CU, another kernel's workgroup is
dispatched only into the slot one retired probe workgroup frees: one wave per SIMD and that
wave's registers.  The device write path's kernels that run before an epoch's publish (its
(slot, op) sort on 64-bit keys included) therefore keep to workgroups of at most 256 threads
and at most the probe's VGPR count -- a kernel that outgrows either waits for the probe's last
dispatch, and the epoch's write tail is exposed again (the round-5 C3 tail).

The gfx950 code objects are read from libstage_hip.so's offload bundles and their kernel
metadata (llvm-readelf --notes): no GPU needed."""
import os
import re
import struct
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "stage-indexorganized_amd", "lib", "libstage_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# the write path's kernels enqueued before an epoch's publish (write_path.hip)
WRITE_CHAIN = ("wp_set_bases", "wp_keys", "wp_heads", "wp_classify", "wp_speculate", "wp_finish_groups", "wp_jump_links",
               "wp_jump_chain", "wp_jump_codes", "wp_flags", "wp_totals", "wp_headers", "wp_write")
READ_PROBE = "_ZN5stage12probe_kernelILb0ELi1ELi8ELi1ELi1ELi64ELi32ELb0ELb0EEE"  # the C2 / C3 read probe
VGPR_GRANULE = 8  # gfx950 allocates a wave's VGPRs in blocks of 8: the slot a probe wave frees


def gfx950_code_objects(path):
    data = open(path, "rb").read()
    sec = None
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "fatbin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={out}", path],
                       check=True, capture_output=True)
        sec = open(out, "rb").read()
    del data
    cos = []
    i = sec.find(MAGIC)
    while i != -1:
        p = i + len(MAGIC)
        (n,) = struct.unpack_from("<Q", sec, p)
        p += 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", sec, p)
            p += 24
            triple = sec[p:p + tl].decode()
            p += tl
            if "gfx950" in triple:
                cos.append(sec[i + off:i + off + size])
        i = sec.find(MAGIC, i + 1)
    return cos


def kernels(co):
    """name -> {vgpr_count, agpr_count, max_flat_workgroup_size, group_segment_fixed_size}"""
    with tempfile.NamedTemporaryFile(suffix=".o") as f:
        f.write(co)
        f.flush()
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], check=True,
                               capture_output=True, text=True).stdout
    out, cur = {}, {}
    for line in notes.splitlines():
        if re.match(r"\s+- \.agpr_count:", line):  # a kernel's entry starts with its first key
            cur = {}
        m = re.match(r"\s+-?\s*\.(name|vgpr_count|agpr_count|max_flat_workgroup_size|group_segment_fixed_size):\s+(\S+)", line)
        if m:
            k, v = m.group(1), m.group(2)
            cur[k] = v if k == "name" else int(v)
            if k == "name":
                out[v] = cur
    return out


@pytest.fixture(scope="module")
def table():
    if not os.path.exists(LIB) or not os.path.exists(os.path.join(LLVM, "llvm-readelf")):
        pytest.skip("libstage_hip.so or the ROCm LLVM tools are missing")
    ks = {}
    for co in gfx950_code_objects(LIB):
        ks.update(kernels(co))
    return ks


def probe_budget(table):
    """the VGPRs (arch + acc) one retired probe wave leaves free"""
    probe = [v for k, v in table.items() if k.startswith(READ_PROBE)]
    assert len(probe) == 1, "the read probe instance is missing"
    assert probe[0]["max_flat_workgroup_size"] == 256
    used = probe[0]["vgpr_count"] + probe[0].get("agpr_count", 0)
    return -(-used // VGPR_GRANULE) * VGPR_GRANULE


def test_write_chain_fits_beside_the_read_probe(table):
    budget = probe_budget(table)
    seen = set()
    for name, v in table.items():
        short = next((w for w in WRITE_CHAIN if f"{len(w)}{w}E" in name), None)
        if short is None:
            continue
        seen.add(short)
        assert v["max_flat_workgroup_size"] <= 256, (short, v)
        assert v["vgpr_count"] + v.get("agpr_count", 0) <= budget, (short, v, budget)
    assert seen == set(WRITE_CHAIN), set(WRITE_CHAIN) - seen


def test_write_path_sort_fits_beside_the_read_probe(table):
    """the (slot, op) sort: rocprim's onesweep kernels for 64-bit keys with 32-bit values
    (radix_sort.hpp's SortConfig<uint64_t>: 256-thread kernel_configs; rocprim instantiates the
    kernel body for gfx950 only -- the other target_arch instances are empty stubs)"""
    budget = probe_budget(table)
    sort = {k: v for k, v in table.items()
            if "onesweep_iteration" in k and "EmjEE" in k and "kernel_configILj256E" in k
            and "target_archE950" in k}
    assert sort, "the write path's onesweep kernels were not found"
    for name, v in sort.items():
        assert v["max_flat_workgroup_size"] <= 256, (name[:120], v)
        assert v["vgpr_count"] + v.get("agpr_count", 0) <= budget, (name[:120], v, budget)
