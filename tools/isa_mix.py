"""VALU instruction mix of a kernel's hot loop from the ISA (make -C ransac_amd isa) and its issue
cost in SIMD cycles, two ways:

  guide     MI355X_MICROARCH.md 'Per-instruction cycle constants': a wave64 VALU op issues over 2
            SIMD cycles, a packed one (v_pk_*) and a transcendental over 4;
  measured  profiles/r4/valu_issue_costs.json (tools/ubench/valu_issue_bench.hip on an MI355X,
            8 waves per SIMD on every CU, wall time x 2.4 GHz per wave-instruction): only
            v_fma/v_add/v_sub/v_mul_f32, v_mov_b32 and the 32-bit integer add / bitwise ops with
            VGPR operands and no |.| / neg modifiers sustain ~2.3-2.6 cycles; a plain op with an
            SGPR source, |.| modifier (v_fma_f32 |a| 3.9), v_max / v_max3 / v_cmp_*_e64 /
            v_cndmask (4.2-4.5), v_pk_fma_f32 (4.3 with an SGPR-pair source, 4.5 all-VGPR) and
            v_fma_f64 (4.7) take about twice that; v_rcp_f32 8.2, v_rcp_f64 16.3.

The hot loop = the innermost backward-branching block range holding the most instructions of
the chosen kind (default: the one with the most v_pk_fma_f32; KIND=v_mfma for the matrix-core
scorer).  MFMA instructions are counted apart (mix "mfma"), not as VALU issue.
  [KIND=<opcode prefix>] python3 tools/isa_mix.py <file.s> <mangled-name-substring> [json-out]
"""
import json
import os
import re
import sys

TRANS = ("v_rcp_", "v_sqrt_", "v_rsq_", "v_exp_", "v_log_", "v_sin_", "v_cos_")
FAST = ("v_fma_f32", "v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_mov_b32", "v_add_u32",
        "v_sub_u32", "v_and_b32", "v_or_b32", "v_xor_b32")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COSTS = os.path.join(ROOT, "profiles", "r4", "valu_issue_costs.json")


def measured_table():
    """instr name -> SIMD cycles per wave-instruction at 8 waves per SIMD"""
    d = json.load(open(COSTS))
    return {r["instr"]: r["simd_cycles_per_wave_instr"] for r in d["rows"] if r["waves_per_simd"] == 8}


def function_body(lines, name):
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r"^_Z\S*%s\S*:" % re.escape(name), ln):
            start = i
        elif start is not None and ln.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit("function %s not found" % name)


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_pk_"):
        return "valu_packed"
    if op.startswith(TRANS):
        return "valu_trans"
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "valu_lane"
    if op.startswith("v_"):
        return "valu_plain"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def measured_cost(ins, t):
    """one VALU instruction's measured issue cycles (see the module doc)"""
    parts = ins.split(None, 1)
    op, args = parts[0], (parts[1] if len(parts) > 1 else "")
    srcs = args.split(",")[1:] if "," in args else []
    sgpr_src = any(re.match(r"\s*s\[|\s*s\d", a) for a in srcs)
    if op.startswith("v_pk_"):
        return t["v_pk_fma_f32 (sgpr pair src)"] if sgpr_src else t["v_pk_fma_f32"]
    if op.startswith("v_rcp_f64") or op.startswith(("v_sqrt_f64", "v_rsq_f64")):
        return t["v_rcp_f64"]
    if op.startswith(TRANS):
        return t["v_rcp_f32"]
    if op.endswith("_f64") or "_f64_" in op:
        return t["v_fma_f64"]
    base = re.sub(r"_e(32|64)$", "", op)
    if base in FAST and not sgpr_src and "|" not in args and "neg(" not in args and "neg_" not in args:
        return t["v_fma_f32"]
    if base == "v_fma_f32" and "|" in args:
        return t["v_fma_f32 |a|"]
    if base.startswith("v_cmp"):
        return t["v_cmp_ngt_f32_e64 (sgpr dst)"]
    if base.startswith("v_cndmask"):
        return t["v_cndmask_b32_e64 (sgpr pair)"]
    return t["v_max_f32_e64 |a|,|b|"]  # the ~4.2-cycle class


def loops(body):
    """(label, first line, last line) of every block range closed by a backward branch."""
    labels = {}
    out = []
    for i, ln in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            labels[m.group(1)] = i
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\S+)", ln)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            out.append((m.group(1), labels[m.group(1)], i))
    return out


def mix(lines):
    c = {}
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        k = classify(s)
        c[k] = c.get(k, 0) + 1
    return c


def main():
    path, name = sys.argv[1], sys.argv[2]
    body = function_body(open(path).read().splitlines(), name)
    best = None
    for lab, a, b in loops(body):
        seg = body[a:b + 1]
        npk = sum(1 for ln in seg if ln.strip().startswith(os.environ.get("KIND", "v_pk_fma_f32")))
        if best is None or npk > best[0] or (npk == best[0] and b - a < best[2] - best[1]):
            best = (npk, a, b, lab)
    _, a, b, lab = best
    seg = body[a:b + 1]
    m = mix(seg)
    valu = m.get("valu_packed", 0) + m.get("valu_plain", 0) + m.get("valu_trans", 0) + m.get("valu_lane", 0)
    issue = 4 * m.get("valu_packed", 0) + 2 * m.get("valu_plain", 0) + 4 * m.get("valu_trans", 0) + \
        2 * m.get("valu_lane", 0)
    t = measured_table()
    meas, by_op = 0.0, {}
    for ln in seg:
        s = ln.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":") or not classify(s).startswith("valu"):
            continue
        c = measured_cost(s, t)
        meas += c
        key = s.split()[0] + (" (sgpr src)" if re.search(r",\s*s[\[\d]", s) else "") + (" |.|" if "|" in s else "")
        e = by_op.setdefault(key, [0, c])
        e[0] += 1
    out = {"function": name, "loop": lab, "lines": [a, b], "mix": m, "valu_instructions": valu,
           "issue_cycles_per_iteration": issue, "issue_cycles_per_valu_instruction": issue / max(valu, 1),
           "measured_cycles_per_iteration": meas, "measured_cycles_per_valu_instruction": meas / max(valu, 1),
           "measured_by_opcode": {k: {"count": v[0], "cycles_each": v[1]} for k, v in sorted(by_op.items())},
           "measured_source": os.path.relpath(COSTS, ROOT),
           "note": "guide issue cycles per SIMD: plain wave64 VALU 2, packed (v_pk_*) 4, transcendental 4; "
                   "measured: the per-opcode costs of valu_issue_costs.json (8 waves/SIMD, wall time x 2.4 GHz); "
                   "the PMC x4 model (SQ_ACTIVE_INST_VALU x 4) charges 4 per instruction"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
