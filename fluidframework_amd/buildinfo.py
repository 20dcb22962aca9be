"""Source identity of libmtreplay.so: the build stamps a hash of its sources into the library
(mt_build_id, include/mtreplay.h) and the loader compares it with the sources in the tree, so a
library that was not built from the checked-out sources is refused instead of silently run."""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
SRC = [PKG / "csrc" / "mt_host.cpp", PKG / "csrc" / "mt_engine.hip", PKG / "csrc" / "mt_kernels.hip",
       PKG / "csrc" / "mt_device.h", PKG / "csrc" / "mt_digest.hip", PKG / "csrc" / "mt_snapshot.hip",
       PKG / "csrc" / "mt_json.cpp", PKG / "csrc" / "mt_values.cpp", PKG / "csrc" / "mt_json_gpu.hip",
       PKG / "csrc" / "mt_json_gpu.h", ROOT / "include" / "mtreplay.h",
       ROOT / "include" / "mt_oplog.h", ROOT / "include" / "mt_gen.h"]
MARKER = b"MTBUILDID:"


def src_hash(flags: str = "") -> str:
    """sha256 over the sources (name + contents, in SRC order) and the compile flags; 16 hex digits."""
    h = hashlib.sha256()
    for p in SRC:
        if p.exists():
            h.update(p.name.encode() + b"\0" + p.read_bytes() + b"\0")
    h.update(flags.encode())
    return h.hexdigest()[:16]


def stamped_hash(lib: Path) -> str | None:
    """The build id stamped into a built library (None: absent or unstamped)."""
    try:
        data = lib.read_bytes()
    except OSError:
        return None
    i = data.find(MARKER)
    if i < 0:
        return None
    return data[i + len(MARKER): i + len(MARKER) + 16].decode("ascii", "replace")


def sources_present() -> bool:
    return all(p.exists() for p in SRC)
