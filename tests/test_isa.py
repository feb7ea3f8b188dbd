"""Machine-code guard on the built gfx950 code objects (no GPU needed).

A subtraction with a DPP-permuted operand folded into one instruction
(v_sub*_dpp / v_subrev*_dpp) came back from the MI355X without the
permutation: the quad pipeline's column passes (hl_quad.h) were wrong in every
odd row until their DPP reads were kept as separate moves (hl_quad.h dpp_x).
This test disassembles the product library and the GPU unit library and fails
if any such instruction is present, so a code change that re-enables the fold
is caught on the CPU before it reaches the GPU.
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
LIBS = [os.path.join(ROOT, "hartallo_amd", "libhartallo_amd.so"), os.path.join(ROOT, "tests", "gpu_unit", "libhl_unit.so")]


def _disassemble(lib, td):
    fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "co.elf")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib], check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--output={co}"], check=True, capture_output=True)
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True, text=True).stdout


@pytest.mark.parametrize("lib", LIBS, ids=["product", "gpu_unit"])
def test_no_folded_dpp_subtraction(lib):
    if not os.path.exists(lib) or not os.path.exists(f"{LLVM}/llvm-objdump"):
        pytest.skip("library or LLVM tools not present")
    with tempfile.TemporaryDirectory() as td:
        dis = _disassemble(lib, td)
    assert "v_mov_b32_dpp" in dis  # the disassembly really holds the kernels
    bad = sorted(set(re.findall(r"\bv_sub(?:rev)?_(?:co_)?[iu]32_dpp\b", dis)))
    assert not bad, f"{os.path.basename(lib)} contains DPP-folded subtractions: {bad}"
