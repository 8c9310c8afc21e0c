#!/usr/bin/env python3
"""VALU issue model of a render-kernel variant (VERDICT r05 Weak #4): how much of the SIMDs' VALU
issue capacity the kernel's instructions fill, from MEASURED issue costs instead of an assumed
4 cycles per instruction.

  python tools/valu_model.py [F=0] --probe profiles/r06_valu_issue.json --out profiles/r06_c3_valu_static.json

* issue costs: tools/valu_issue.hip's event-timed throughput per instruction class (wave64
  instructions per ns per SIMD at 8 waves per SIMD, independent instructions);
* the kernel's dynamic counts per class come from rocprofv3 PMC (SQ_INSTS_VALU_{ADD,MUL,FMA}_F64,
  TRANS_F64, {ADD,MUL,FMA,TRANS}_F32, INT32, INT64, CVT and the total SQ_INSTS_VALU): bench.py
  multiplies them by the per-class cost written here;
* the instructions no PMC class counts (moves, compares, selects, min / max, lane ops: the "rest")
  and the INT32 class mix several costs; their mean cost is taken from this variant's ISA -- the
  static mix of those mnemonics inside loops (depth >= 1), each priced by the probe (the mnemonic
  itself, or the nearest measured one of its encoding / width, else the fp64-add rate). That mean
  is an estimate (static, not dynamic, weights); the PMC classes themselves are exact.
Writes {class: ns per wave instruction per SIMD} for bench.py's roofline.valu.
"""
from __future__ import annotations

import json
import re
import subprocess
import sys
import tempfile
from collections import Counter
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
CSRC = REPO / "distraytracer_old_amd" / "csrc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "--cuda-device-only"]
MINREG = ["-mllvm=--amdgpu-sched-strategy=iterative-minreg", "-mllvm=--amdgpu-use-amdgpu-trackers=1"]

# probe class -> mnemonics priced by it (the mnemonic after stripping _e32 / _e64 / _dpp / _sdwa)
PRICE_AS = {
    "v_mov_b32": ["v_mov_b32"],
    "v_add_u32": ["v_add_u32", "v_subrev_u32"],
    "v_sub_u32": ["v_sub_u32"],
    "v_and_b32": ["v_and_b32"],
    "v_or_b32": ["v_or_b32", "v_xor_b32", "v_not_b32"],
    "v_lshrrev_b32(vgpr)": ["v_lshrrev_b32", "v_ashrrev_i32"],
    "v_lshlrev_b32": ["v_lshlrev_b32"],
    "v_add_f32": ["v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32"],
    "v_fma_f32": ["v_fma_f32", "v_fmac_f32"],
    "v_max3_f32": ["v_max3_f32", "v_min3_f32", "v_med3_f32"],
    "v_add_f64": ["v_add_f64"],
    "v_mul_f64": ["v_mul_f64"],
    "v_fma_f64": ["v_fma_f64", "v_fmac_f64"],
    "v_min_f64": ["v_min_f64"],
    "v_max_f64": ["v_max_f64"],
    "v_cmp_lt_f64(vcc)": [],          # v_cmp_* / v_cmpx_*: by width below
    "v_cndmask_b32_e64": ["v_cndmask_b32"],
    "v_mov_b64": ["v_mov_b64"],
    "v_lshlrev_b64": ["v_lshlrev_b64", "v_lshrrev_b64", "v_ashrrev_i64"],
    "v_add_co_u32": ["v_add_co_u32", "v_addc_co_u32", "v_sub_co_u32", "v_subb_co_u32", "v_subrev_co_u32"],
    "v_mbcnt_lo_u32_b32": ["v_mbcnt_lo_u32_b32", "v_mbcnt_hi_u32_b32"],
    "v_readfirstlane_b32": ["v_readfirstlane_b32", "v_readlane_b32"],
    "v_writelane_b32": ["v_writelane_b32"],
    "v_bfe_u32": ["v_bfe_u32", "v_bfe_i32", "v_bfi_b32", "v_alignbit_b32", "v_lshl_add_u32", "v_lshl_or_b32",
                  "v_add3_u32", "v_and_or_b32", "v_or3_b32", "v_add_lshl_u32", "v_perm_b32"],
    "v_mul_lo_u32": ["v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24", "v_mul_u32_u24", "v_mad_u64_u32"],
    "v_max_i32": ["v_max_i32", "v_min_i32", "v_max_u32", "v_min_u32"],
    "v_cvt_f32_f64": ["v_cvt_f32_f64", "v_cvt_f64_f32", "v_cvt_i32_f64", "v_cvt_u32_f32", "v_cvt_f32_u32",
                      "v_cvt_f32_i32", "v_cvt_i32_f32"],
    "v_cvt_f64_i32": ["v_cvt_f64_i32", "v_cvt_f64_u32"],
    "v_rcp_f64": ["v_rcp_f64", "v_rsq_f64", "v_sqrt_f64"],
    "v_fract_f64": ["v_fract_f64", "v_frexp_mant_f64", "v_frexp_exp_i32_f64", "v_trig_preop_f64"],
    "v_ldexp_f64": ["v_ldexp_f64", "v_div_scale_f64", "v_div_fmas_f64", "v_div_fixup_f64"],
    "v_mov_b32_dpp": [],
}
FP64_PMC = {"v_add_f64": "SQ_INSTS_VALU_ADD_F64", "v_mul_f64": "SQ_INSTS_VALU_MUL_F64", "v_fma_f64": "SQ_INSTS_VALU_FMA_F64",
            "v_fmac_f64": "SQ_INSTS_VALU_FMA_F64"}
TRANS64 = {"v_rcp_f64", "v_rsq_f64", "v_sqrt_f64"}
F32_PMC = {"v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32"}
CVT = set(PRICE_AS["v_cvt_f32_f64"] + PRICE_AS["v_cvt_f64_i32"])
INT64 = set(PRICE_AS["v_lshlrev_b64"]) | {"v_mad_u64_u32"}
INT32 = (set(PRICE_AS["v_add_u32"] + PRICE_AS["v_sub_u32"] + PRICE_AS["v_and_b32"] + PRICE_AS["v_or_b32"] +
             PRICE_AS["v_lshrrev_b32(vgpr)"] + PRICE_AS["v_lshlrev_b32"] + PRICE_AS["v_bfe_u32"] +
             PRICE_AS["v_mul_lo_u32"] + PRICE_AS["v_max_i32"] + PRICE_AS["v_add_co_u32"]) - {"v_mad_u64_u32"})


def kernel_isa(F: int) -> str:
    src = ('#include <hip/hip_runtime.h>\n#include "rt_internal.h"\n#include "trace_kernels.h"\n'
           f"template __global__ void rt::dv::render_kernel<false, {F}u>(rt::SceneD, rt::ParamsD, float*, int*, unsigned long long*);\n")
    with tempfile.TemporaryDirectory() as td:
        p = Path(td) / "probe.hip"
        p.write_text(src)
        out = Path(td) / "probe.s"
        extra = MINREG if F in (0,) else []
        r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-I", str(CSRC), "-S", str(p), "-o", str(out)],
                           capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr[-3000:])
        return out.read_text()


def static_mix(s: str) -> Counter:
    m = [mm for mm in re.finditer(r"^(_ZN2rt2dv13render_kernel\w+):", s, re.M)][0]
    body = s[m.end():s.index(".amdhsa_kernel " + m.group(1))].split("\n")
    depth, c = 0, Counter()
    for ln in body:
        t = ln.strip()
        if re.match(r"^\.LBB|^; %bb", t):
            d = re.search(r"Depth=(\d+)", ln)
            depth = int(d.group(1)) if d else 0
        if depth >= 1 and ln.startswith("\t") and t.startswith("v_"):
            op = re.sub(r"_(e32|e64|dpp|sdwa)$", "", t.split()[0])
            c[op] += 1
    return c


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 0
    probe = json.loads(Path(sys.argv[sys.argv.index("--probe") + 1]).read_text())["classes"]
    out = Path(sys.argv[sys.argv.index("--out") + 1]) if "--out" in sys.argv else None
    rate = {k: v["winst_per_ns_per_simd"] for k, v in probe.items()}
    base = rate["v_add_f64"]
    ns = {}  # mnemonic -> ns per wave instruction per SIMD
    for cls, ops in PRICE_AS.items():
        for op in ops:
            ns[op] = 1.0 / rate[cls]

    def price(op: str) -> tuple[float, str]:
        if op in ns:
            return ns[op], "measured"
        if op.startswith(("v_cmp", "v_cmpx")):
            return 1.0 / rate["v_cmp_lt_f64(vcc)"], "v_cmp_*"
        return 1.0 / base, "default (fp64-add rate)"

    mix = static_mix(kernel_isa(F))
    groups = {"rest": Counter(), "int32": Counter()}
    for op, n in mix.items():
        if op in FP64_PMC or op in TRANS64 or op in F32_PMC or op in CVT or op in INT64:
            continue
        groups["int32" if op in INT32 else "rest"][op] += n
    cost = {
        "add_f64": 1.0 / rate["v_add_f64"], "mul_f64": 1.0 / rate["v_mul_f64"], "fma_f64": 1.0 / rate["v_fma_f64"],
        "trans_f64": 1.0 / rate["v_rcp_f64"], "add_f32": 1.0 / rate["v_add_f32"], "mul_f32": 1.0 / rate["v_add_f32"],
        "fma_f32": 1.0 / rate["v_fma_f32"], "trans_f32": 1.0 / rate["v_rcp_f64"] / 2, "cvt": 1.0 / rate["v_cvt_f32_f64"],
        "int64": 1.0 / rate["v_lshlrev_b64"],
    }
    detail = {}
    for g, cnt in groups.items():
        tot = sum(cnt.values()) or 1
        cost[g] = sum(price(op)[0] * n for op, n in cnt.items()) / tot
        detail[g] = {"static_instructions_in_loops": tot,
                     "top": [[op, n, round(price(op)[0] * base * 4, 2), price(op)[1]] for op, n in cnt.most_common(25)]}
    res = {"variant_F": F, "probe": "tools/valu_issue.hip (event-timed, 8 waves / SIMD)",
           "unit": "ns per wave64 instruction per SIMD at the probe's clock (4 x fp64-add rate = the '4-cycle' unit)",
           "fp64_add_rate_winst_per_ns_per_simd": base,
           "cost_ns": cost,
           "cost_in_fp64_add_cycles": {k: round(v * base * 4, 3) for k, v in cost.items()},
           "static_mix": detail}
    txt = json.dumps(res, indent=1)
    if out:
        out.write_text(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
