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
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_isa import _disassemble  # noqa: E402


def digest(lib):
    with tempfile.TemporaryDirectory() as td:
        text = _disassemble(lib, td)
    lines = []
    for ln in text.splitlines():
        ln = re.sub(r"//.*$", "", ln).strip()
        ln = re.sub(r"^[0-9a-f]+:\s*", "", ln)
        ln = re.sub(r"<[^>]*\+0x[0-9a-f]+>", "", ln)
        if ln and not ln.startswith("Disassembly") and not ln.endswith("file format elf64-amdgpu"):
            lines.append(ln)
    return hashlib.sha256("\n".join(lines).encode()).hexdigest()[:16], len(lines)


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "hartallo_amd", "libhartallo_amd.so")
    print(lib, *digest(lib))
