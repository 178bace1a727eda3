"""CPU: the host table and the oracle under AddressSanitizer + UndefinedBehaviorSanitizer.

`make -C stage-indexorganized_amd/csrc check_host` builds tools/host_table_check.cpp with
host_table.cpp (g++, -fsanitize=address,undefined; no HIP) and runs a randomized single-writer
workload -- inserts with leaf splits, updates with commit / abort / finalize, deletes, aborted
inserts, batched epochs with repeated keys, location export/resolve and a leaf-image round trip --
over variable-length, 8-byte and 32-byte key geometries against a model of the present keys.
Any sanitizer report or model mismatch fails the run.  `make -C oracle check` does the same for
the C restatement (oracle/oracle_check.c: loads, threaded reads and scans, random writes with
commit / abort / finalize, deletes, aborted inserts, batched epochs, transactions, leaf images,
locations).  `make -C oracle check_tsan` runs the threaded update and read paths under
ThreadSanitizer (oracle/oracle_tsan.c).
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "stage-indexorganized_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_host_table_under_asan_ubsan():
    env = dict(os.environ, UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run(["make", "-s", "-C", CSRC, "check_host"], capture_output=True, text=True, timeout=900,
                       env=env)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "host_table_check: ok" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no host compiler")
def test_oracle_under_asan_ubsan():
    env = dict(os.environ, UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "check"], capture_output=True, text=True,
                       timeout=900, env=env)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert ": ok" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no host compiler")
def test_oracle_threaded_paths_under_tsan():
    """`make -C oracle check_tsan`: the C3 CPU leg's concurrent writers (orc_update_batch_mt, 8
    writers over hot keys, uncommitted updates and absent keys, three epochs) equal the single
    writer's replay on a twin table, and ThreadSanitizer reports no race -- the writers' leaf
    searches read other writers' slot meta words, which are relaxed atomics as the reference's
    CASed words are (round 6: the first TSan run flagged plain loads and stores there)."""
    p = subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "check_tsan"], capture_output=True,
                       text=True, timeout=900)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "oracle_tsan: ok" in p.stdout
    assert "ThreadSanitizer" not in p.stderr
