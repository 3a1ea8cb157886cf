"""isa_mix.py OBJ KERNEL_PATTERN: instruction mix (mnemonic counts) of one
gfx950 kernel in a hipcc object file, from its disassembly (no GPU)."""
import collections
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def disasm(obj):
    with tempfile.TemporaryDirectory() as tmp:
        fat, co = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "k.co")
        subprocess.run([f"{B}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{B}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True,
                              text=True).stdout


def mix(text, pat):
    counts, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            cur = m.group(1) if re.search(pat, m.group(1)) else None
            if cur:
                counts[cur] = collections.Counter()
            continue
        if cur:
            m = re.match(r"^\s+([a-z_0-9]+)\s", line)
            if m:
                counts[cur][m.group(1)] += 1
    return counts


if __name__ == "__main__":
    for name, c in mix(disasm(sys.argv[1]), sys.argv[2]).items():
        total = sum(c.values())
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print(f"{name[:70]}: {total} instructions, {valu} VALU")
        for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 14):
            print(f"   {k:28s} {v}")
