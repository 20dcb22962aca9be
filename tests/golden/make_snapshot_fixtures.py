"""Extract the reference's golden SnapshotV1 blobs into a compact fixture.

Source (data files held by the reference's own tests, byte-checked there by
packages/dds/sequence/src/test/snapshotVersion.spec.ts:86-105):
    /root/reference/packages/dds/sequence/src/test/snapshots/v1/<name>.json
Each file is JSON.stringify(sharedString.snapshot(), undefined, 1); we keep only the
data this build must reproduce: the interval-collection "header" blob and the
merge-tree "content" tree's blob contents (header, body_0, ...), plus the recipe that
produced them (generateSharedStrings.ts:24-97, restated as data below).

Run from the repo root:  python tests/golden/make_snapshot_fixtures.py
"""
import json
import sys
from pathlib import Path

REF = Path("/root/reference/packages/dds/sequence/src/test/snapshots/v1")
OUT = Path(__file__).with_name("snapshot_v1.json")

MARKER_PROPS = '{"ItemType":"Paragraph","Properties":{"Bold":false},"markerId":"marker%d","referenceTileLabels":["Eop"]}'

# generateSharedStrings.ts:24-97 (Snapshot.sizeOfFirstChunk = 10000, insertText = "text")
RECIPES = {
    "headerOnly": {"inserts": 1250, "fmt": "text%d"},
    "headerAndBody": {"inserts": 5000, "fmt": "text%d"},
    "largeBody": {"inserts": 10000, "fmt": "text-%d"},
    "withMarkers": {"inserts": 5000, "fmt": "text%d", "markers_every": 70, "marker_ref_type": 1,
                    "marker_props": MARKER_PROPS},
    "withAnnotations": {"inserts": 5000, "fmt": "text%d", "annotate_every": 70, "annotate_len": 10,
                        "annotate_props": '{"bold":true}'},
}


def main():
    fixtures = {}
    for name, recipe in RECIPES.items():
        tree = json.loads((REF / f"{name}.json").read_text())
        interval_header = next(e for e in tree["entries"] if e["path"] == "header")["value"]["contents"]
        content = next(e for e in tree["entries"] if e["path"] == "content")["value"]
        blobs = [[e["path"], e["value"]["contents"]] for e in content["entries"]]
        fixtures[name] = {"recipe": recipe, "interval_header": interval_header, "blobs": blobs}
    OUT.write_text(json.dumps(fixtures, indent=0, sort_keys=True))
    print(f"wrote {OUT} ({OUT.stat().st_size} bytes)")


if __name__ == "__main__":
    sys.exit(main())
