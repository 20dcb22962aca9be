"""tests/golden/kats.json with every scenario's "messages" materialised (see make_kats.py: an
`append_digits` scenario is that many single-character appends, MT/test/snapshot.spec.ts:188-202)."""
import json
from pathlib import Path

KATS_PATH = Path(__file__).resolve().parent / "golden" / "kats.json"


def expand(kat: dict) -> dict:
    if "messages" in kat:
        return kat
    a = kat["append_digits"]
    msgs = []
    for i in range(a["n"]):
        msgs.append({"clientId": a["client"], "sequenceNumber": i + 1, "referenceSequenceNumber": i,
                     "minimumSequenceNumber": i + 1 if a["increase_msn"] else 0, "type": "op",
                     "contents": {"type": 0, "pos1": i, "seg": str(i % 10)}})
    return dict(kat, messages=msgs)


def load_kats() -> list:
    return [expand(k) for k in json.loads(KATS_PATH.read_text())]
