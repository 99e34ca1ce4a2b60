"""VALU instruction mix of a kernel's hot loop from the ISA (make -C ransac_amd isa): packed
(v_pk_*) vs plain VALU vs transcendental, the loop's SALU / SMEM / waits, and the issue cycles the
guide prices them at (MI355X_MICROARCH.md 'Per-instruction cycle constants': a wave64 VALU op
issues over 2 SIMD cycles, a packed one over 4 -- two FMAs per lane -- and a transcendental over 4
at throughput).  The hot loop = the innermost backward-branching block range holding the most
instructions of the chosen kind (default: the one with the most v_pk_fma_f32).
  python3 tools/isa_mix.py <file.s> <mangled-name-substring> [json-out]
"""
import json
import re
import sys

TRANS = ("v_rcp_", "v_sqrt_", "v_rsq_", "v_exp_", "v_log_", "v_sin_", "v_cos_")


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
        npk = sum(1 for ln in seg if ln.strip().startswith("v_pk_fma_f32"))
        if best is None or npk > best[0] or (npk == best[0] and b - a < best[2] - best[1]):
            best = (npk, a, b, lab)
    _, a, b, lab = best
    m = mix(body[a:b + 1])
    valu = m.get("valu_packed", 0) + m.get("valu_plain", 0) + m.get("valu_trans", 0) + m.get("valu_lane", 0)
    issue = 4 * m.get("valu_packed", 0) + 2 * m.get("valu_plain", 0) + 4 * m.get("valu_trans", 0) + \
        2 * m.get("valu_lane", 0)
    out = {"function": name, "loop": lab, "lines": [a, b], "mix": m, "valu_instructions": valu,
           "issue_cycles_per_iteration": issue, "issue_cycles_per_valu_instruction": issue / max(valu, 1),
           "note": "issue cycles per SIMD: plain wave64 VALU 2, packed (v_pk_*) 4, transcendental 4; the "
                   "PMC x4 model (SQ_ACTIVE_INST_VALU x 4) charges 4 per instruction"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
