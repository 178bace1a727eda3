"""Regenerates tests/golden/zipf_kat.json from the REFERENCE's own FastRandom / ZipfDistribution.

benchmark/benchmark_common.h is header-only; `make -C oracle ref` compiles it (unmodified,
included where it lies) with oracle/ref_zipf_kat.cpp into oracle/_ref/ref_zipf_kat (never
committed).  The reference seeds its Zipf generator with rand(); the driver replaces it by
FastRandom(seed) after construction, which is what the harness's stage_zipf_draws(n, theta,
seed, ...) takes.  The key ranges are the drivers' own: ZipfDistribution(scale_factor - 1,
theta) (ycsb_workload.cpp:88) for C1 (1000 rows), 1M rows and C2/C3 (100M rows).
Run it in a container that has /root/reference; the committed JSON travels.
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
BIN = os.path.join(REPO, "oracle", "_ref", "ref_zipf_kat")

FAST = [(0, 64), (1, 64), (0x5EED, 64), ((1 << 47) + 3, 64)]
ZIPF = [(999, 0.9, 1, 512), (999, 0.99, 7, 512), (999_999, 0.9, 0x5EED, 512), (999_999, 0.99, 0x5EED + 1, 512),
        (99_999_999, 0.9, 0x5EED, 512), (99_999_999, 0.99, 0x5EED + 1000, 512)]
# RunMixed op streams (ycsb_mixed.cpp:26-44): (seed, count, update_ratio); -1 = read, else the delta byte
OPS = [(1, 2048, 0.05), (0x5EED + 77, 2048, 0.05), (3, 1024, 0.5), (9, 256, 1.0)]


def run(*args):
    return json.loads(subprocess.run([BIN] + [str(a) for a in args], check=True, capture_output=True,
                                     text=True).stdout)


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"], check=True)
    out = {"source": "reference benchmark/benchmark_common.h:10-98 built by oracle/Makefile `ref`",
           "generator": "tests/golden/make_zipf_kat.py", "fastrandom": [], "zipf": []}
    for seed, count in FAST:
        out["fastrandom"].append({"seed": seed, "next": run("fast", seed, count)["next"]})
    for n, theta, seed, count in ZIPF:
        r = run("zipf", n, repr(theta), seed, count)
        out["zipf"].append(dict(n=n, theta=theta, seed=seed, **r))
        print(n, theta, r["zeta_n_bits"])
    out["ops"] = [dict(seed=seed, count=count, update_ratio=ratio, ops=run("ops", seed, count, repr(ratio))["ops"])
                  for seed, count, ratio in OPS]
    with open(os.path.join(HERE, "zipf_kat.json"), "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
