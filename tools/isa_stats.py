#!/usr/bin/env python3
"""Per-kernel ISA statistics of trace.hip (instruction count, scratch ops, resources).

  python tools/isa_stats.py [-D...]     (compiles the device half with hipcc -S)
"""
import re
import subprocess
import sys
from collections import Counter
from pathlib import Path

CSRC = Path(__file__).resolve().parents[1] / "distraytracer_old_amd" / "csrc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "--cuda-device-only"]


def main():
    extra = sys.argv[1:]
    out = "/tmp/isa_stats.s"
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-S", str(CSRC / "trace.hip"), "-o", out],
                       capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-3000:]); sys.exit(1)
    s = open(out).read()
    for m in re.finditer(r"^(_ZN2rt2dv\w+):", s, re.M):
        name = m.group(1)
        j = s.find(".amdhsa_kernel " + name, m.end())
        if j < 0:
            continue
        body = s[m.end():j].split("\n")
        ins = [l.strip().split()[0] for l in body if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
        c = Counter(ins)
        # resource lines from the kernel descriptor
        kd = s.index(".amdhsa_kernel " + name)
        kde = s.index(".end_amdhsa_kernel", kd)
        desc = s[kd:kde]
        def g(k):
            mm = re.search(r"\.%s\s+(\d+)" % k, desc)
            return int(mm.group(1)) if mm else -1
        scr = sum(v for k, v in c.items() if k.startswith("scratch_"))
        print(f"{name[:60]:60s} ins={len(ins):6d} scratch_ops={scr:4d} div={c['v_div_scale_f64']//2:4d} "
              f"private={g('amdhsa_private_segment_fixed_size')} "
              f"nvgpr={g('amdhsa_next_free_vgpr')} accum_off={g('amdhsa_accum_offset')}")


if __name__ == "__main__":
    main()
