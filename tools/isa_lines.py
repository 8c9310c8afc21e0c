#!/usr/bin/env python3
"""Map instructions of one kernel to source lines (hipcc -g): counts per (file:line) for
instructions matching a prefix, e.g. scratch_ (spills / private arrays).

  python tools/isa_lines.py <kernel-substring> <insn-prefix> [-D...]
"""
import re
import subprocess
import sys
from collections import Counter
from pathlib import Path

CSRC = Path(__file__).resolve().parents[1] / "distraytracer_old_amd" / "csrc"
FLAGS = ["-O3", "-g", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "--cuda-device-only"]


def main():
    kern, pref, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
    out = "/tmp/isa_lines.s"
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-S", str(CSRC / "trace.hip"), "-o", out], capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-3000:]); sys.exit(1)
    s = open(out).read()
    files = dict(re.findall(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s, re.M))
    m = [mm for mm in re.finditer(r"^(_ZN2rt2dv\w+):", s, re.M) if kern in mm.group(1)][0]
    j = s.index(".amdhsa_kernel " + m.group(1))
    cur = "?"
    c = Counter()
    for l in s[m.end():j].split("\n"):
        t = l.strip()
        if t.startswith(".loc"):
            f = t.split()
            cur = f"{Path(files.get(f[1], f[1])).name}:{f[2]}"
        elif t and not t.startswith((".", ";")) and t.split()[0].startswith(pref):
            c[cur] += 1
    for k, v in c.most_common(40):
        print(f"{v:5d} {k}")


if __name__ == "__main__":
    main()
