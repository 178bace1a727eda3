"""Regenerates tests/golden/murmur64a_kat.json from the REFERENCE's own MurmurHash64A.

The reference's misc/murmur/MurmurHash2.cpp compiles unmodified from its own source file;
`make -C oracle ref` builds it into oracle/_ref/libref_murmur.so (never committed).  This
script feeds it fixed inputs and records the outputs as known-answer vectors.  Run it in a
container that has /root/reference (the GPU box does not; the committed JSON travels).
"""
import ctypes
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SO = os.path.join(REPO, "oracle", "_ref", "libref_murmur.so")


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    L = ctypes.CDLL(SO)
    L.ref_murmur64a.restype = ctypes.c_uint64
    L.ref_murmur64a.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64]
    vectors = []
    # every tail length 0..16 over a fixed byte pattern, three seeds
    pattern = bytes((i * 37 + 11) & 0xFF for i in range(64))
    for seed in (0, 1, 0x9747B28C):
        for ln in range(0, 17):
            data = pattern[:ln]
            vectors.append({"hex": data.hex(), "seed": seed, "hash": L.ref_murmur64a(data, ln, seed)})
    # the shard router's inputs: 8-byte little-endian keys, seed 0
    for k in [0, 1, 2, 3, 255, 256, 65535, 65536, 999999, 10**8 - 1, 2**32 - 1, 2**63, 2**64 - 1]:
        data = k.to_bytes(8, "little")
        vectors.append({"hex": data.hex(), "seed": 0, "hash": L.ref_murmur64a(data, 8, 0)})
    out = {"source": "reference misc/murmur/MurmurHash2.cpp:99-147 built by oracle/Makefile `ref`",
           "generator": "tests/golden/make_golden.py", "vectors": vectors}
    with open(os.path.join(HERE, "murmur64a_kat.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(len(vectors), "vectors")


if __name__ == "__main__":
    main()
