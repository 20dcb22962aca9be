"""The GPU JSON parser's lane parser (mt_json_gpu.hip: parse_msg and below, host-callable) on the
CPU under AddressSanitizer (tests/native/jg_parse_asan.cpp): valid logs and thousands of mutated
copies, count and write passes into exactly-sized buffers — no read or write leaves its buffer and
both passes agree.  Needs hipcc (cross-compiles here without a GPU)."""
import json
import random
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if Path("/opt/rocm/bin/hipcc").exists() else None)


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_lane_parser_is_memory_safe_on_valid_and_mutated_logs(tmp_path):
    import test_gpu_json as t
    from combine_logs import RELPOS_DOCS
    from test_json_ingest import EDGE_DOCS, _farm_messages

    exe = tmp_path / "jg_asan"
    subprocess.run([HIPCC, "-x", "hip", "-std=c++17", "--offload-arch=gfx950", "-O1", "-g", "-Xarch_host",
                    "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer", "-o", str(exe),
                    str(ROOT / "tests" / "native" / "jg_parse_asan.cpp")], check=True, cwd=tmp_path)
    rng = random.Random(7)
    docs = [json.dumps(_farm_messages()[:800])] + [json.dumps(d) for d in t.FAST_DOCS + EDGE_DOCS + RELPOS_DOCS]
    docs += [t._fuzz_doc(rng, 100).replace("\n", " ").replace("\r", " ") for _ in range(20)]
    docs += [t._marker_doc(rng, 150) for _ in range(5)]
    corpus = tmp_path / "corpus.txt"
    corpus.write_text("".join(d + "\n" for d in docs))
    r = subprocess.run([str(exe), str(corpus), "100", "11"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    _, msgs, parsed = r.stdout.split()
    assert int(msgs) > 100000 and int(parsed) > 0.5 * int(msgs)
