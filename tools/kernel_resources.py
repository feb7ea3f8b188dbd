"""Register, spill and LDS figures of the gfx950 kernels in a built library
(read from the code object's metadata notes; no GPU needed).

  python tools/kernel_resources.py [lib.so] [kernel-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
KEYS = (".vgpr_count", ".vgpr_spill_count", ".sgpr_count", ".sgpr_spill_count", ".agpr_count", ".group_segment_fixed_size",
        ".private_segment_fixed_size")


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def resources(lib):
    """Every code object of the library's .hip_fatbin (one bundle per HIP
    translation unit: hl_encoder.hip and hl_encoder_fam3.hip)."""
    notes = ""
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib], check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for k, a in enumerate(starts):
            b = starts[k + 1] if k + 1 < len(starts) else len(data)
            part, co = os.path.join(td, f"b{k}.bin"), os.path.join(td, f"co{k}.elf")
            open(part, "wb").write(data[a:b])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
            notes += subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
    # one YAML list item per kernel: keys before and after .name belong to it
    out, item = {}, {}
    def flush():
        if "name" in item:
            out[item.pop("name")] = dict(item)
    for line in notes.splitlines():
        if re.match(r"\s*- \.", line) and re.match(r"\s*- \.(agpr_count|args)", line):
            flush()
            item = {}
        m = re.match(r"\s*-?\s*\.name:\s+(\S+)", line)
        if m:
            item["name"] = m.group(1)
        for k in KEYS:
            m = re.match(r"\s*-?\s*" + re.escape(k) + r":\s+(\d+)", line)
            if m:
                item[k[1:]] = int(m.group(1))
    flush()
    return out


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1].endswith(".so") else os.path.join(ROOT, "hartallo_amd", "libhartallo_amd.so")
    pats = [a for a in sys.argv[1:] if not a.endswith(".so")] or ["k_pipeline", "k_mb_diag"]
    for name, r in sorted(resources(lib).items()):
        if any(p in name for p in pats):
            print(name, " ".join(f"{k}={v}" for k, v in r.items() if k != "name"))


if __name__ == "__main__":
    main()
