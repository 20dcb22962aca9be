"""Pin the oracle (CPU restatement) against the reference's own fixtures.

* SnapshotV1 golden files (sequence/src/test/snapshots/v1/*.json, byte-checked by the
  reference in snapshotVersion.spec.ts:86-105), regenerated with the recipe of
  generateSharedStrings.ts:24-97 through the non-collaborating local edit path.
* Known-answer observer scenarios (tests/golden/kats.json, see make_kats.py for sources).
"""
import json
from pathlib import Path

import pytest

import oracle_ffi as O
from kat_util import load_kats

GOLDEN = Path(__file__).with_name("golden")
SNAP = json.loads((GOLDEN / "snapshot_v1.json").read_text())
KATS = load_kats()


def build_recipe(r) -> O.Doc:
    d = O.Doc()
    for i in range(r["inserts"]):
        assert d.insert_local(0, json.dumps(r["fmt"] % i)) == 0, d.error
    if "markers_every" in r:
        i = 0
        while i < d.length():
            seg = '{"marker":{"refType":%d},"props":%s}' % (r["marker_ref_type"], r["marker_props"] % i)
            assert d.insert_local(i, seg) == 0, d.error
            i += r["markers_every"]
    if "annotate_every" in r:
        i = 0
        while i < d.length():
            assert d.annotate_local(i, i + r["annotate_len"], r["annotate_props"]) == 0, d.error
            i += r["annotate_every"]
    return d


@pytest.mark.parametrize("name", sorted(SNAP))
def test_snapshot_v1_golden_bytes(name):
    fx = SNAP[name]
    d = build_recipe(fx["recipe"])
    blobs = d.snapshot_v1()
    assert list(blobs) == [p for p, _ in fx["blobs"]]
    for path, contents in fx["blobs"]:
        assert blobs[path] == contents, f"{name}/{path} differs from the reference golden file"


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_observer_kats(kat):
    d = O.Doc()
    d.start_collab("readonly")
    msgs = kat["messages"]
    cut = kat.get("reload_after", len(msgs))
    for m in msgs[:cut]:
        assert d.apply_msg(json.dumps(m)) == 0, d.error
    if "reload_after" in kat:
        # TestString.checkSnapshot (MT/test/snapshot.spec.ts:59-79): SnapshotV1 round trip into a
        # new client with the same text and length, which then takes the remaining ops
        d2 = O.Doc()
        assert d2.load_snapshot(d.snapshot_v1(), "readonly") == 0, d2.error
        assert d2.text() == d.text() and d2.length() == d.length()
        d = d2
    for m in msgs[cut:]:
        assert d.apply_msg(json.dumps(m)) == 0, d.error
    assert d.text() == kat["text"]
    if "props_runs" in kat:
        assert json.loads(d.props_runs()) == kat["props_runs"]


def _inserting_walk_tree(shape):
    """The spec's trees built exactly as MT/test/mergeTree.insertingWalk.spec.ts:26-157 does: local
    edits of a non-collaborating tree (UniversalSequenceNumber segments), then collaboration."""
    d = O.Doc()
    if shape == "single_segment":
        assert d.insert_local(0, json.dumps("hello world")) == 0
    else:
        n = 7 if shape == "full_single_layer" else 32
        for i in range(n):
            assert d.insert_local(d.length(), json.dumps(str(i))) == 0
        if shape == "with_removes":
            r = int(d.length() / 4 + 0.5)
            assert d.remove_local(0, r) == 0
            assert d.remove_local(d.length() - r, d.length()) == 0
    return d


@pytest.mark.parametrize("shape", ["single_segment", "full_single_layer", "with_removes"])
def test_inserting_walk_spec_trees(shape):
    """The insertingWalk KATs on the spec's own tree shapes: the full single layer is one block of
    MaxNodesInBlock - 1 leaves (:80-91), and an insert at the beginning / end / middle gives the
    spec's text (:187-253) — here as a remote insert of a client that has seen the whole tree."""
    for where in ("beginning", "end", "middle"):
        kat = next(k for k in KATS if k["name"] == f"inserting_walk_{shape}_{where}")
        d = _inserting_walk_tree(shape)
        if shape == "full_single_layer":
            assert d.shape() == "D1:7", d.shape()
        assert d.start_collab("readonly") == 0
        ins = dict(kat["messages"][-1], sequenceNumber=1, referenceSequenceNumber=0)
        assert d.apply_msg(json.dumps(ins)) == 0, d.error
        assert d.text() == kat["text"], (shape, where)


def test_snapshot_chunking_and_merge_info():
    """SnapshotV1 with a collaborating tree: merge info for segments above the MSN,
    elision of removals at/below it, 10000-char chunking (snapshotV1.ts:57-79,151-247)."""
    d = O.Doc()
    d.start_collab("readonly")
    seq = 0
    for i in range(1200):
        seq += 1
        m = {"clientId": "A" if i % 2 else "B", "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
             "minimumSequenceNumber": max(0, seq - 30), "type": "op",
             "contents": {"type": 0, "pos1": 0, "seg": "abcdefghij"}}
        assert d.apply_msg(json.dumps(m)) == 0, d.error
    seq += 1
    rm = {"clientId": "B", "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
          "minimumSequenceNumber": seq - 30, "type": "op", "contents": {"type": 1, "pos1": 5, "pos2": 25}}
    assert d.apply_msg(json.dumps(rm)) == 0
    blobs = d.snapshot_v1()
    hdr = json.loads(blobs["header"])
    assert hdr["headerMetadata"]["minSequenceNumber"] == seq - 30
    assert hdr["headerMetadata"]["sequenceNumber"] == seq
    assert hdr["headerMetadata"]["totalLength"] == 12000
    assert [c["id"] for c in hdr["headerMetadata"]["orderedChunkMetadata"]] == list(blobs)
    seg0 = hdr["segments"][0]
    assert seg0["json"] == "abcde" and seg0["seq"] == seq - 1 and seg0["client"] == "A"
    assert hdr["segments"][1]["removedSeq"] == seq and hdr["segments"][1]["removedClient"] == "B"
    total = 0
    for name, blob in blobs.items():
        c = json.loads(blob)
        assert c["length"] == sum(len(s["json"] if isinstance(s, dict) else s) for s in c["segments"])
        total += c["length"]
    assert total == hdr["headerMetadata"]["totalLength"]


def test_invalid_insert_position_status():
    d = O.Doc()
    d.start_collab("readonly")
    m = {"clientId": "A", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
         "type": "op", "contents": {"type": 0, "pos1": 5, "seg": "x"}}
    assert d.apply_msg(json.dumps(m)) == 1  # MergeTree insert failed
    assert "MergeTree insert failed" in d.error


def test_sequence_order_violation_status():
    d = O.Doc()
    d.start_collab("readonly")
    mk = lambda s, ms=0: json.dumps({"clientId": "A", "sequenceNumber": s, "referenceSequenceNumber": 0,
                                     "minimumSequenceNumber": ms, "type": "op",
                                     "contents": {"type": 0, "pos1": 0, "seg": "x"}})
    assert d.apply_msg(mk(2)) == 0
    assert d.apply_msg(mk(2)) == 2


def test_msn_backwards_status():
    d = O.Doc()
    d.start_collab("readonly")
    mk = lambda s, ms: json.dumps({"clientId": "A", "sequenceNumber": s, "referenceSequenceNumber": s - 1,
                                   "minimumSequenceNumber": ms, "type": "op",
                                   "contents": {"type": 0, "pos1": 0, "seg": "x"}})
    assert d.apply_msg(mk(1, 0)) == 0
    assert d.apply_msg(mk(2, 1)) == 0
    assert d.apply_msg(mk(3, 0)) == 3


@pytest.mark.parametrize("name", sorted(SNAP))
def test_snapshot_loader_rebuilds_golden_files(name):
    """SnapshotLoader (snapshotLoader.ts:36-205) on the reference's golden files: the reference's
    rebuild test (snapshotVersion.spec.ts:29-58) checks text, length and properties against the
    generated string; re-serializing the loaded tree must give the golden bytes again."""
    fx = SNAP[name]
    want = build_recipe(fx["recipe"])
    blobs = {p: c for p, c in fx["blobs"]}
    d = O.Doc()
    assert d.load_snapshot(blobs, "snapshot") == 0, d.error
    assert d.length() == want.length()
    assert d.text() == want.text()
    assert json.loads(d.props_runs()) == json.loads(want.props_runs())
    assert d.snapshot_v1() == blobs


_FARMS = [  # (n_ops, docs, kwargs) — text-only, config-3 mix, wide collab windows, markers-free farms
    (1500, 6, dict(seed=0xC0FFEE)),
    (1500, 6, dict(pct_insert=55, pct_remove=35, seed=0xBADC0DE)),
    (1200, 6, dict(n_clients=24, max_lag=200, pct_insert=50, pct_remove=40, min_len=0, max_insert=3, seed=77)),
    (3000, 3, dict(pct_insert=50, pct_remove=15, seed=2024)),
]


def _farm_digests():
    out = []
    for n, docs, kw in _FARMS:
        p = O.gen_params(n, **kw)
        ops, text, props, off = O.gen_batch(p, docs)
        _, dig, st = O.replay_batch(ops, off, text, props, O.gen_tables(), O.gen_client_names(p.n_clients), n_threads=2)
        out += [int(x) for x in dig] + [int(x) for x in st]
    return out


def test_oracle_subtree_shortcut_is_exact():
    """The oracle's block lengths skip subtrees whose seqs are all at or below refSeq (their view
    length is cachedLength); with MTO_SLOW_LENGTHS=1 every block length is the full recursive leaf
    sum.  Both give identical final states on conflict farms, including wide collab windows."""
    import json
    import os
    import subprocess
    import sys

    code = ("import json, sys; sys.path.insert(0, %r); import test_oracle_golden as T; "
            "print(json.dumps(T._farm_digests()))") % str(Path(__file__).resolve().parent)
    env = dict(os.environ, MTO_SLOW_LENGTHS="1")
    slow = json.loads(subprocess.run([sys.executable, "-c", code], env=env, check=True, capture_output=True,
                                     text=True, cwd=str(Path(__file__).resolve().parents[1])).stdout)
    assert slow == _farm_digests()
