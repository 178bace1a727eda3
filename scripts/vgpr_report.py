"""Register report of the kernels in a device assembly file:
    hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -I include -o k.s csrc/kernels.hip
    python scripts/vgpr_report.py k.s [name-substring]
prints VGPRs, SGPRs, SGPR spills into VGPR lanes (v_writelane) and scratch use per kernel --
the probe's occupancy hinges on it (5 waves/SIMD up to 96 VGPRs, 3 at 154)."""
import re
import sys

src = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\S+):\s*;\s*@", src, re.M):
    name = m.group(1)
    if pat not in name:
        continue
    end = src.find(".Lfunc_end", m.end())
    body = src[m.end():end]
    def meta(key):
        r = re.search(r"\.set " + re.escape(name) + r"\." + key + r", (\d+)", src)
        return r.group(1) if r else "?"
    print(f"{name[:70]:70s} vgpr {meta('num_vgpr'):>4s} sgpr {meta('numbered_sgpr'):>4s} "
          f"writelane {body.count('v_writelane_b32'):4d} scratch {meta('private_seg_size'):>4s}")
