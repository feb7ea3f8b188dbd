"""Digest of the gfx950 device code of a library: the disassembly of every
kernel, addresses stripped (a source change that leaves the machine code
alone gives the same digest).  Development tool.
    python tools/isa_digest.py [lib.so]    (default: the in-tree product)"""
import hashlib
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _disassemble_all(lib, td):
    """Every code object of the library's .hip_fatbin (one bundle per HIP
    translation unit: hl_encoder.hip and hl_encoder_fam3.hip)."""
    fat = os.path.join(td, "fat.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib], check=True, capture_output=True)
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    text = []
    for k, a in enumerate(starts):
        b = starts[k + 1] if k + 1 < len(starts) else len(data)
        part, co = os.path.join(td, f"b{k}.bin"), os.path.join(td, f"co{k}.elf")
        open(part, "wb").write(data[a:b])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        text.append(subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True, capture_output=True, text=True).stdout)
    return "\n".join(text), len(starts)


def digest(lib):
    with tempfile.TemporaryDirectory() as td:
        text, nb = _disassemble_all(lib, td)
    lines = []
    for ln in text.splitlines():
        ln = re.sub(r"//.*$", "", ln).strip()
        ln = re.sub(r"^[0-9a-f]+:\s*", "", ln)
        ln = re.sub(r"<[^>]*\+0x[0-9a-f]+>", "", ln)
        if ln and not ln.startswith("Disassembly") and not ln.endswith("file format elf64-amdgpu"):
            lines.append(ln)
    return hashlib.sha256("\n".join(lines).encode()).hexdigest()[:16], len(lines), f"{nb} code objects"


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "hartallo_amd", "libhartallo_amd.so")
    print(lib, *digest(lib))
