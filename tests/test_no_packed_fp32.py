"""The library issues no packed fp32 VALU instruction (usac_pk.hpp): on gfx950
v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 return wrong values in lanes 48-63 while another kernel's
waves execute MFMAs on the same CU (tools/mfma_interference.cpp).  CPU test: every gfx950 code object
in ransac_amd/libransac_amd.so is disassembled and searched."""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def test_no_packed_fp32_in_code_objects(tmp_path):
    so = os.path.join(ROOT, "ransac_amd", "libransac_amd.so")
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    assert os.path.exists(so), "libransac_amd.so not built (make -C ransac_amd)"
    local = tmp_path / "lib.so"
    shutil.copy(so, local)
    subprocess.run([OBJDUMP, "--offloading", str(local)], cwd=tmp_path, check=True, capture_output=True)
    objs = glob.glob(str(tmp_path / "lib.so.*gfx950*"))
    assert objs, "no gfx950 code object in the library"
    pat = re.compile(r"\bv_pk_((fma|mul|add)_f32|mov_b32)\b")  # the packed-fp32 family (Makefile: -packed-fp32-ops)
    n_instr = 0
    for o in objs:
        dis = subprocess.run([OBJDUMP, "-d", o], check=True, capture_output=True, text=True).stdout
        n_instr += dis.count("\n")
        hits = [l for l in dis.splitlines() if pat.search(l)]
        assert not hits, "%s: %d packed fp32 instructions, e.g. %s" % (os.path.basename(o), len(hits), hits[0])
    assert n_instr > 10000
