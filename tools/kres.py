"""Register / scratch / LDS use of the kernels in a class object: python tools/kres.py <obj.o> ..."""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")


def notes(obj: Path, tmp: Path) -> str:
    fat, co = tmp / (obj.stem + ".fatbin"), tmp / (obj.stem + ".co")
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(obj), str(tmp / "x.o")],
                   check=True, capture_output=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
    return subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True, capture_output=True,
                          text=True).stdout


if __name__ == "__main__":
    keys = ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size",
            "group_segment_fixed_size")
    for o in sys.argv[1:]:
        with tempfile.TemporaryDirectory() as t:
            n = notes(Path(o), Path(t))
        for block in n.split("  - .")[1:]:
            m = re.search(r"\.name:\s+(\S+)", block)
            if m and not m.group(1).endswith(".kd"):
                vals = dict(re.findall(r"\.(" + "|".join(keys) + r"):\s+(\d+)", block))
                print(m.group(1), " ".join(f"{k}={vals.get(k)}" for k in keys))
