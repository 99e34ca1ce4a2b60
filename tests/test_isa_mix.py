"""tools/isa_mix.py prices a kernel's hot loop with the per-opcode VALU costs measured on the
MI355X (profiles/r4/valu_issue_costs.json) -- the issue model behind the cfg2 line's roofline
`frac`.  CPU: the classification rules on a synthetic loop, and the committed cfg2 mix file
agreeing with a fresh pricing of its own opcode counts."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_mix  # noqa: E402

LOOP = """_Z3fooPf:
.LBB0_1:
	s_load_dwordx16 s[36:51], s[28:29], 0x0
	s_waitcnt lgkmcnt(0)
	v_pk_fma_f32 v[38:39], v[10:11], s[36:37], v[12:13]
	v_pk_fma_f32 v[40:41], v[26:27], v[28:29], v[30:31]
	v_fma_f32 v1, v2, v3, v4
	v_fma_f32 v40, |v42|, v50, v51
	v_fma_f32 v5, s4, v6, v7
	v_add_f32_e32 v8, v9, v10
	v_max_f32_e64 v38, |v38|, |v40|
	v_cmp_ngt_f32_e64 s[0:1], v38, v40
	v_cndmask_b32_e64 v3, v4, v5, s[2:3]
	v_fma_f64 v[2:3], v[4:5], v[6:7], v[8:9]
	v_rcp_f32_e32 v9, v9
	v_rcp_f64_e32 v[2:3], v[2:3]
	s_or_b64 vcc, s[0:1], s[6:7]
	s_cbranch_vccnz .LBB0_1
.Lfunc_end0:
"""


def test_measured_costs_per_opcode_class():
    t = isa_mix.measured_table()
    assert t["v_fma_f32"] < 3.0 < t["v_max_f32_e64 |a|,|b|"]  # the fast plain family vs the rest
    expect = [
        ("v_pk_fma_f32 v[38:39], v[10:11], s[36:37], v[12:13]", t["v_pk_fma_f32 (sgpr pair src)"]),
        ("v_pk_fma_f32 v[40:41], v[26:27], v[28:29], v[30:31]", t["v_pk_fma_f32"]),
        ("v_fma_f32 v1, v2, v3, v4", t["v_fma_f32"]),
        ("v_fma_f32 v40, |v42|, v50, v51", t["v_fma_f32 |a|"]),
        ("v_fma_f32 v5, s4, v6, v7", t["v_max_f32_e64 |a|,|b|"]),  # SGPR source: the ~4.2 class
        ("v_add_f32_e32 v8, v9, v10", t["v_fma_f32"]),
        ("v_max_f32_e64 v38, |v38|, |v40|", t["v_max_f32_e64 |a|,|b|"]),
        ("v_cmp_ngt_f32_e64 s[0:1], v38, v40", t["v_cmp_ngt_f32_e64 (sgpr dst)"]),
        ("v_cndmask_b32_e64 v3, v4, v5, s[2:3]", t["v_cndmask_b32_e64 (sgpr pair)"]),
        ("v_fma_f64 v[2:3], v[4:5], v[6:7], v[8:9]", t["v_fma_f64"]),
        ("v_rcp_f32_e32 v9, v9", t["v_rcp_f32"]),
        ("v_rcp_f64_e32 v[2:3], v[2:3]", t["v_rcp_f64"]),
    ]
    for ins, cyc in expect:
        assert isa_mix.measured_cost(ins, t) == cyc, ins


def test_loop_pricing(tmp_path):
    f = tmp_path / "k.s"
    f.write_text(LOOP)
    out = tmp_path / "k.json"
    sys.argv = ["isa_mix.py", str(f), "3foo", str(out)]
    isa_mix.main()
    d = json.loads(out.read_text())
    assert d["valu_instructions"] == 12 and d["mix"]["smem"] == 1 and d["mix"]["salu"] == 1
    t = isa_mix.measured_table()
    want = sum(isa_mix.measured_cost(ln.strip(), t) for ln in LOOP.splitlines() if ln.strip().startswith("v_"))
    assert abs(d["measured_cycles_per_iteration"] - want) < 1e-9
    # the guide's model: plain 2, packed / transcendental 4
    assert d["issue_cycles_per_iteration"] == 2 * 4 + 8 * 2 + 2 * 4


def test_committed_cfg2_mix_consistent():
    d = json.load(open(os.path.join(ROOT, "profiles", "r4", "isa_k_score_hf_8_false.json")))
    total = sum(v["count"] * v["cycles_each"] for v in d["measured_by_opcode"].values())
    assert abs(total - d["measured_cycles_per_iteration"]) < 1e-6
    assert d["valu_instructions"] == sum(v["count"] for v in d["measured_by_opcode"].values()) == 56
