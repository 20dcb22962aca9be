"""Rewrite the capacity-class ladder everywhere it is spelled out (mt_device.h kClassSegs, the
kernel table in mt_host.cpp, __graft_entry__.CLASSES).  usage: python tools/set_classes.py 128 376 ..."""
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
NEW = [int(x) for x in sys.argv[1:]]
assert len(NEW) == 16 and NEW[-1] > 65000, "16 classes, the last the HBM class (> 65,000 slots)"

p = ROOT / "fluidframework_amd/csrc/mt_device.h"
s = p.read_text()
s = re.sub(r"constexpr int kClassSegs\[\] = \{[0-9, ]+\};", "constexpr int kClassSegs[] = {" + ", ".join(map(str, NEW)) + "};", s)
p.write_text(s)

p = ROOT / "fluidframework_amd/csrc/mt_host.cpp"
s = p.read_text()
a = s.index("MT_DECLARE_CLASS(", s.index("#define MT_DECLARE_CLASS(S)") + 10)
e = s.index('extern "C" __global__ void mt_digest_kernel')
s = s[:a] + "".join(f"MT_DECLARE_CLASS({x})\n" for x in NEW) + s[e:]
a = s.index("static const KernelClass kKernels[mt::kNumClasses] = {")
e = s.index("};", a) + 2
ents = ",\n".join(f"    {{{x}, (const void *)mt_replay_kernel_{x}, (const void *)mt_generate_kernel_{x}, "
                  f"(const void *)mt_load_kernel_{x},\n     (const void *)mt_follow_kernel_{x}}}" for x in NEW)
s = s[:a] + "static const KernelClass kKernels[mt::kNumClasses] = {\n" + ents + ",\n};" + s[e:]
p.write_text(s)

p = ROOT / "__graft_entry__.py"
s = p.read_text()
s = re.sub(r"CLASSES = \([0-9, ]+\)", "CLASSES = (" + ", ".join(map(str, NEW)) + ")", s)
p.write_text(s)
print("classes:", NEW)
