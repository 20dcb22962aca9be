"""Experiment builds: recompile only some capacity classes with extra flags and link them with the
release objects of the others into fluidframework_amd/libmtreplay_<name>.so (loaded through
FLUIDFRAMEWORK_AMD_LIB, which skips the source-stamp check).
python tools/quick_variant.py NAME "CLASS,CLASS,..." [-DFLAG ...]"""
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as g  # noqa: E402

name, classes, flags = sys.argv[1], [int(c) for c in sys.argv[2].split(",") if c], sys.argv[3:]
rel = g.PKG / "build" / "release"
out = g.PKG / "build" / f"q_{name}"
out.mkdir(parents=True, exist_ok=True)
base = [g._hipcc(), "-x", "hip", "-O3", "-std=c++17", f"--offload-arch={g.ARCH}", "-fPIC", "-fvisibility=hidden", *flags]
# QV_SCHED: the machine scheduler of the rebuilt classes (default max-ilp, as the release build;
# "default": the compiler's own)
sched = os.environ.get("QV_SCHED", "max-ilp")
sflags = [] if sched == "default" else ["-mllvm", f"-amdgpu-sched-strategy={sched}"]
procs = [subprocess.Popen(base + sflags + ["-c", f"-DMT_SEG={seg}", "-DMT_PART=1",
                                  "-o", str(out / f"k{seg}_1.o"), str(g.PKG / "csrc" / "mt_kernels.hip")], cwd=ROOT)
         for seg in classes]
host_flags = [f for f in flags if f == "-DMT_PROF"]
if host_flags:  # the host object sees the same switches (MT_PROF: its report)
    procs.append(subprocess.Popen(base + ["-c", '-DMT_BUILD_ID="MTBUILDID:variant000000000"', "-o", str(out / "host.o"),
                                          str(g.PKG / "csrc" / "mt_host.cpp")], cwd=ROOT))
for p in procs:
    if p.wait() != 0:
        sys.exit(1)
objs = []
for seg in g.CLASSES:  # (the observer replay objects of `classes` rebuilt; the rest from the release build)
    objs.append(str(out / f"k{seg}_1.o") if seg in classes else str(rel / f"k{seg}_1.o"))
    objs.append(str(rel / f"k{seg}_2.o"))
for o in ("host", "digest", "snapshot", "json", "json_gpu", "values"):
    objs.append(str(out / f"{o}.o") if (out / f"{o}.o").exists() and o == "host" and host_flags else str(rel / f"{o}.o"))
lib = g.PKG / f"libmtreplay_{name}.so"
subprocess.run([g._hipcc(), f"--offload-arch={g.ARCH}", "-shared", "-fPIC", "-o", str(lib), *objs], check=True, cwd=ROOT)
print(lib)
