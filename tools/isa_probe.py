#!/usr/bin/env python3
"""Fast ISA check of ONE render-kernel variant (register-pressure experiments): compiles a
stub that instantiates only render_kernel<false, F> from trace_kernels.h (device only) and
prints instructions, scratch ops (total and inside loops of depth >= 2), private bytes, VGPRs.

  python tools/isa_probe.py [F=0] [-DNAME=...]
"""
import re
import subprocess
import sys
import tempfile
from collections import Counter
from pathlib import Path

CSRC = Path(__file__).resolve().parents[1] / "distraytracer_old_amd" / "csrc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "--cuda-device-only"]


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 0
    extra = [a for a in sys.argv[1:] if a.startswith("-") and a != "--lines"]
    lines = "--lines" in sys.argv
    src = ('#include <hip/hip_runtime.h>\n#include "rt_internal.h"\n#include "trace_kernels.h"\n'
           f"template __global__ void rt::dv::render_kernel<false, {F}u>(rt::SceneD, rt::ParamsD, float*, int*, unsigned long long*);\n")
    with tempfile.TemporaryDirectory() as td:
        p = Path(td) / "probe.hip"
        p.write_text(src)
        out = Path(td) / "probe.s"
        r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *(["-gline-tables-only"] if lines else []), "-I", str(CSRC), *extra, "-S",
                            str(p), "-o", str(out)],
                           capture_output=True, text=True)
        if r.returncode:
            print(r.stderr[-3000:]); sys.exit(1)
        s = out.read_text()
    m = [mm for mm in re.finditer(r"^(_ZN2rt2dv13render_kernel\w+):", s, re.M)][0]
    j = s.index(".amdhsa_kernel " + m.group(1))
    body = s[m.end():j].split("\n")
    files = dict(re.findall(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s, re.M))
    depth, c, deep, where, loc, bydepth = 0, Counter(), Counter(), Counter(), "?", Counter()
    for l in body:
        t = l.strip()
        ml = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if ml:
            loc = files.get(ml.group(1), "?").split("/")[-1] + ":" + ml.group(2)
        if re.match(r"^\.LBB|^; %bb", t):
            d = re.search(r"Depth=(\d+)", l)
            depth = int(d.group(1)) if d else 0
        if t and not t.startswith((".", ";")) and l.startswith("\t"):
            op = t.split()[0]
            c[op] += 1
            if op.startswith(("scratch_", "buffer_")):  # private memory: arrays and spills
                c["_priv"] += 1
                bydepth[min(depth, 6)] += 1
                if depth >= 2:
                    deep["st" if "store" in op else "ld"] += 1
                where[(depth, "st" if "store" in op else "ld", loc)] += 1
    desc = s[s.index(".amdhsa_kernel " + m.group(1)):]
    g = lambda k: int(re.search(r"\.%s\s+(\d+)" % k, desc).group(1))
    priv = c.pop("_priv", 0)
    ins = sum(c.values())
    scr = priv
    print(f"F={F} ins={ins} scratch={scr} deep_st={deep['st']} deep_ld={deep['ld']} "
          f"private={g('amdhsa_private_segment_fixed_size')} vgpr_next={g('amdhsa_next_free_vgpr')} "
          f"sgpr_next={g('amdhsa_next_free_sgpr')} by_depth={dict(sorted(bydepth.items()))}")
    if lines:  # -g changes scheduling slightly: counts are indicative
        for (dp, kind, lc), v in sorted(where.items(), key=lambda x: (-x[0][0], -x[1]))[:60]:
            print(f"  depth {dp} {kind} {lc}: {v}")


if __name__ == "__main__":
    main()
