"""Register / scratch budget of the replay kernels (CPU: reads the gfx950 code objects built
by __graft_entry__.build()).

The replay engine keeps every document's per-op control in registers; the class kernels run
one wavefront per document, and each class's kernel may use the registers its LDS residency leaves
(16 documents per CU in the start class: 4 waves per SIMD, at most 128 VGPRs) and must not spill
to scratch.  A change that pushes a replay kernel past its budget silently cuts residency
(measured: 22.3 ms -> 35 ms per config-2 launch at 147 VGPRs in the 16-per-CU class), so it is
pinned here."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
OBJ = ROOT / "fluidframework_amd" / "build" / "release"
LLVM = Path("/opt/rocm/lib/llvm/bin")


def _notes(obj: Path, tmp: Path) -> str:
    fat, co = tmp / (obj.stem + ".fatbin"), tmp / (obj.stem + ".co")
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(obj), str(tmp / "x.o")],
                   check=True, capture_output=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
    return subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True, capture_output=True,
                          text=True).stdout


def _kernels(notes: str) -> dict:
    out = {}
    for block in notes.split("  - .")[1:]:
        m = re.search(r"\.name:\s+(\S+)", block)
        if not m:
            continue
        out[m.group(1)] = {k: int(v) for k, v in re.findall(r"\.(vgpr_count|private_segment_fixed_size):\s+(\d+)", block)}
    return out


# VGPR budget of each class's replay kernel: 512 / the waves per SIMD its LDS layout allows
# (mt_device.h class_waves_per_eu: 16 documents per CU in class 464 -> 4 waves -> 128 VGPRs; 5 in
# class 2046 -> 2 -> 256; 4 in class 2688 -> 1 -> 512)
BUDGET = {464: 128, 563: 128, 1400: 256, 2046: 256, 2688: 512}


@pytest.mark.skipif(not (LLVM / "llvm-readelf").exists() or not OBJ.exists(), reason="no build / ROCm llvm tools")
@pytest.mark.parametrize("seg", sorted(BUDGET))
def test_replay_kernel_fits_its_class_residency(seg, tmp_path):
    obj, obj2 = OBJ / f"k{seg}_1.o", OBJ / f"k{seg}_2.o"
    if not obj.exists() or not obj2.exists():
        pytest.skip("class object not built")
    k = _kernels(_notes(obj, tmp_path))
    r = k[f"mt_replay_kernel_{seg}"]
    assert r["vgpr_count"] <= BUDGET[seg], r
    # no spill traffic: a real VGPR overflow spills hundreds of bytes and shows up as scratch
    # instructions; a few dwords of reserved (unused) private segment are tolerated
    assert r["private_segment_fixed_size"] <= 64, r
    assert _scratch_insts(tmp_path / (obj.stem + ".co"), f"mt_replay_kernel_{seg}") == 0
    assert not any(n.startswith("mt_follow_kernel_") for n in k)  # the follow-on path was removed
    # the writer replay (local-client path) keeps the 4-waves-per-SIMD residency; its extra state
    # spills a few dwords (bounded here so growth is noticed); so does the bigprops replay (property
    # sets of any size), which takes the replay's register budget
    k2 = _kernels(_notes(obj2, tmp_path))
    assert not any(n.startswith("mt_follow_kernel_") for n in k2)
    for name in (f"mt_writer_kernel_{seg}", f"mt_bigprops_kernel_{seg}"):
        w = k2[name]
        assert w["vgpr_count"] <= BUDGET[seg], w
        assert w["private_segment_fixed_size"] <= 512, w


def _scratch_insts(co: Path, kernel: str) -> int:
    """scratch loads / stores in `kernel`'s code (llvm-objdump of the code object _notes unbundled)"""
    dis = subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], check=True, capture_output=True,
                         text=True).stdout
    body = dis.split(f"<{kernel}>:", 1)[1].split("\n\n", 1)[0]
    return len(re.findall(r"\bscratch_(?:load|store)", body))
