"""numpy restatement of the per-document SnapshotV1 bytes digest (test checker)."""
import numpy as np


def _mix64(x):
    x = x ^ (x >> np.uint64(30))
    x = x * np.uint64(0xBF58476D1CE4E5B9)
    x = x ^ (x >> np.uint64(27))
    x = x * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def bytes_digest(data: bytes) -> int:
    """numpy restatement of mt_bytes_digest_kernel (mt_digest.hip)."""
    with np.errstate(over="ignore"):
        pad = data + b"\0" * (-len(data) % 8)
        w = np.frombuffer(pad, "<u8")
        k = np.arange(1, len(w) + 1, dtype=np.uint64)
        acc = _mix64(w + np.uint64(0x9E3779B97F4A7C15) * k).sum(dtype=np.uint64) if len(w) else np.uint64(0)
        h = _mix64(np.uint64(len(data)) ^ np.uint64(0x736E617073686F74))
        return int(_mix64(h ^ acc))

