"""kernel_resources.py OBJ [PATTERN]: VGPR / SGPR / spills / LDS / code
size of the gfx950 kernels in a hipcc object file (its .hip_fatbin), read
from the code object's metadata -- no GPU needed."""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def main():
    obj = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    with tempfile.TemporaryDirectory() as tmp:
        fat, co = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "k.co")
        subprocess.run([f"{B}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fat], check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{B}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
        sizes = {}
        syms = subprocess.run([f"{B}/llvm-readelf", "-sW", co], capture_output=True, text=True).stdout
        for line in syms.splitlines():
            f = line.split()
            if len(f) >= 8 and f[3] == "FUNC":
                sizes[f[7]] = int(f[2])
    for blk in notes.split("- .agpr_count")[1:]:
        def get(key):
            m = re.search(r"\.%s:\s+(\S+)" % key, blk)
            return m.group(1) if m else "?"
        name = get("name")
        if not pat.search(name):
            continue
        print(f"{name[:64]:64s} vgpr {get('vgpr_count'):>4} sgpr {get('sgpr_count'):>4} "
              f"vspill {get('vgpr_spill_count'):>3} lds {get('group_segment_fixed_size'):>6} "
              f"scratch {get('private_segment_fixed_size'):>4} code {sizes.get(name, 0)} B")


if __name__ == "__main__":
    main()
