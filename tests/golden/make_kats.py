"""Build tests/golden/kats.json: observer-replay known-answer scenarios.

Each scenario is a list of ISequencedDocumentMessage JSON objects (protocol.ts:132-172)
applied by a passive observer ("readonly", MT/test/mergeTreeOperationRunner.ts:107-108)
plus the expected final text / properties.  `source` names where the expectation comes
from:
  * "reference:<file>:<lines>" — a literal expectation asserted by the reference's own
    merge-tree test suite for the same message sequence (every client converges on it,
    so the observer must produce it too);
  * "derived:<file>:<lines>" — the reference test checks convergence only; the expected
    observer value was derived by hand from the cited rules and is NOT reference-pinned.

Run from the repo root:  python tests/golden/make_kats.py
"""
import json
from pathlib import Path

OUT = Path(__file__).with_name("kats.json")


def msg(client, seq, ref, contents, msn=0):
    return {"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": msn, "type": "op", "contents": contents}


def ins(pos, seg):
    return {"type": 0, "pos1": pos, "seg": seg}


def rem(a, b):
    return {"type": 1, "pos1": a, "pos2": b}


def ann(a, b, props, combining=None):
    op = {"type": 2, "pos1": a, "pos2": b, "props": props}
    if combining:
        op["combiningOp"] = combining
    return op


def hello_world():
    # MT/test/mergeTree.markRangeRemoved.spec.ts:13-22: client "local" inserts each char of
    # "hello world" at the end, each op sequenced as currentSeq + 1 with refSeq currentSeq.
    return [msg("local", i + 1, i, ins(i, ch)) for i, ch in enumerate("hello world")]


def inserting_walk_kats():
    """MT/test/mergeTree.insertingWalk.spec.ts:26-257: three tree shapes — one segment "hello world";
    a full single layer (MaxNodesInBlock - 1 = 7 leaves "0".."6"); 32 leaves "0".."31" with the first
    and last quarter of the text removed — and an insert of "a" at the beginning, the end and
    Math.round(...) "middle" of each; expected text `a${t}`, `${t}a`, t[:m] + "a" + t[m:]
    (:206, :225, :244-248).  The spec builds the trees with local edits at
    UniversalSequenceNumber; here the same edits arrive as sequenced ops of a "builder" client (MSN
    0: no zamboni, every segment stays a leaf) and the insert is a remote op of a "writer" that has
    seen them all.  tests/test_oracle_golden.py also rebuilds the spec's exact trees through the
    oracle's local path and checks the same answers."""
    out = []
    shapes = []
    # single segment tree (:27-50)
    t = "hello world"
    shapes.append(("single_segment", [ins(0, t)], t, int(len(t) / 2 + 0.5)))
    # full single layer tree (:51-102): "0" then appends "1".."6"
    edits, t = [], ""
    for i in range(7):
        edits.append(ins(len(t), str(i)))
        t += str(i)
    shapes.append(("full_single_layer", edits, t, 4))  # Math.round(MaxNodesInBlock / 2)
    # tree with remove segments (:103-156): "0".."31" appended, remove = Math.round(len / 4) from the
    # start, then the same count from the end of what is left
    edits, t = [], ""
    for i in range(32):
        edits.append(ins(len(t), str(i)))
        t += str(i)
    r = int(len(t) / 4 + 0.5)
    edits.append(rem(0, r))
    t = t[r:]
    edits.append(rem(len(t) - r, len(t)))
    t = t[:len(t) - r]
    shapes.append(("with_removes", edits, t, int(len(t) / 2 + 0.5)))
    for name, edits, t, mid in shapes:
        base = [msg("builder", i + 1, i, e) for i, e in enumerate(edits)]
        n = len(base)
        for where, pos, want in (("beginning", 0, "a" + t), ("end", len(t), t + "a"),
                                 ("middle", mid, t[:mid] + "a" + t[mid:])):
            out.append({"name": f"inserting_walk_{name}_{where}",
                        "source": "reference:MT/test/mergeTree.insertingWalk.spec.ts:26-257",
                        "messages": base + [msg("writer", n + 1, n, ins(pos, "a"))], "text": want})
    return out


def snapshot_kats():
    """MT/test/snapshot.spec.ts:136-202 through a passive observer: TestString.queue (:96-106) sends
    each op with refSeq = the previous seq and minSeq = seq when increaseMsn, else the last minSeq.
    `reload_after` = messages applied before TestString.expect / checkSnapshot round-trips the
    replica through SnapshotV1 (:59-79): the rest is applied to the client loaded from the
    snapshot.  `append_digits` expands to that many appends of `${i % 10}` (:188-202)."""
    w = "fakeId"
    out = []

    def seq_msgs(edits):
        res, msn = [], 0
        for i, (e, inc) in enumerate(edits):
            if inc:
                msn = i + 1
            res.append(msg(w, i + 1, i, e, msn=msn))
        return res

    src = "reference:MT/test/snapshot.spec.ts"
    out.append({"name": "snapshot_segments_below_msn", "source": f"{src}:136-139",
                "messages": seq_msgs([(ins(0, "0"), True)]), "reload_after": 1, "text": "0"})
    out.append({"name": "snapshot_acked_segments_above_msn", "source": f"{src}:141-144",
                "messages": seq_msgs([(ins(0, "0"), False)]), "reload_after": 1, "text": "0"})
    out.append({"name": "snapshot_removal_above_msn", "source": f"{src}:146-150",
                "messages": seq_msgs([(ins(0, "0x"), False), (rem(1, 2), False)]), "reload_after": 2, "text": "0"})
    out.append({"name": "snapshot_removal_above_msn_of_segment_below_msn", "source": f"{src}:152-156",
                "messages": seq_msgs([(ins(0, "0x"), True), (rem(1, 2), False)]), "reload_after": 2, "text": "0"})
    out.append({"name": "snapshot_insert_after_loading_removed_segment", "source": f"{src}:158-164",
                "messages": seq_msgs([(ins(0, "0x"), True), (rem(1, 2), False), (ins(1, "1"), False)]),
                "reload_after": 2, "text": "01"})
    out.append({"name": "snapshot_insert_relative_to_removed_segment_loaded", "source": f"{src}:175-186",
                "messages": seq_msgs([(ins(0, "0x"), False), (ins(2, "2"), False), (rem(1, 2), False),
                                      (ins(1, "1"), False), (ins(3, "3"), False)]),
                "reload_after": 3, "text": "0123"})
    n = 10000 + 10  # SnapshotV1.chunkSize + 10
    for inc, lines in ((True, "188-194"), (False, "196-202")):
        out.append({"name": f"snapshot_body_chunk_{'below' if inc else 'above'}_msn", "source": f"{src}:{lines}",
                    "append_digits": {"client": w, "n": n, "increase_msn": inc}, "reload_after": n,
                    "text": "".join(str(i % 10) for i in range(n))})
    return out


def main():
    kats = []
    base = hello_world()
    kats.append({"name": "hello_world", "source": "reference:MT/test/mergeTree.markRangeRemoved.spec.ts:21",
                 "messages": base, "text": "hello world"})
    kats.append({"name": "remote_remove_then_remote_insert",
                 "source": "reference:MT/test/mergeTree.markRangeRemoved.spec.ts:69-89",
                 "messages": base + [msg("remote2", 12, 11, rem(0, 11)), msg("remote", 13, 11, ins(0, "text"))],
                 "text": "text"})
    kats.append({"name": "remote_insert_then_remote_remove",
                 "source": "reference:MT/test/mergeTree.markRangeRemoved.spec.ts:91-107",
                 "messages": base + [msg("remote", 12, 11, ins(0, "text")), msg("remote2", 13, 11, rem(0, 11))],
                 "text": "text"})
    # issue #1213 observer run (MT/test/mergeTree.markRangeRemoved.spec.ts:111-135): the test only
    # compares observer and writer; "cX" follows from breakTie (mergeTree.ts:2248-2277).
    kats.append({"name": "issue1213_observer", "source": "derived:MT/test/mergeTree.markRangeRemoved.spec.ts:111-135",
                 "messages": [msg("1", 1, 0, ins(0, "a")), msg("1", 2, 0, rem(0, 1)), msg("2", 3, 0, ins(0, "X")),
                              msg("1", 4, 2, ins(0, "c"))],
                 "text": "cX"})
    # MT/test/snapshot.spec.ts:160-167 "can insert segments relative to removed segment"
    w = "writer"
    kats.append({"name": "insert_relative_to_removed", "source": "reference:MT/test/snapshot.spec.ts:160-167",
                 "messages": [msg(w, 1, 0, ins(0, "0x")), msg(w, 2, 1, ins(2, "2")), msg(w, 3, 2, rem(1, 2)),
                              msg(w, 4, 3, ins(1, "1")), msg(w, 5, 4, ins(3, "3"))],
                 "text": "0123"})
    # MT/test/snapshot.spec.ts:146-151 with MSN advancing (zamboni unlinks the tombstone)
    kats.append({"name": "removal_above_msn_of_segment_below_msn", "source": "reference:MT/test/snapshot.spec.ts:146-151",
                 "messages": [msg(w, 1, 0, ins(0, "0x"), msn=1), msg(w, 2, 1, rem(1, 2), msn=1),
                              msg(w, 3, 2, ins(1, "1"), msn=3)],
                 "text": "01"})
    # MT/test/mergeTree.annotate.spec.ts:485-509 "remote first" / "remote only" / "split remote"
    kats.append({"name": "remote_annotate", "source": "reference:MT/test/mergeTree.annotate.spec.ts:485-519",
                 "messages": [msg("remote", 1, 0, ins(0, "hello world")),
                              msg("remote", 2, 1, ann(3, 7, {"propertySource": "remote", "remoteProperty": 1}))],
                 "text": "hello world",
                 "props_runs": [[0, 3, None], [3, 4, '{"propertySource":"remote","remoteProperty":1}'],
                                [7, 4, None]]})
    # JS key order: integer-like keys first, delete + re-add moves a string key last
    # (MT/properties.ts:95-116 via Object.keys order); null deletes.
    kats.append({"name": "annotate_key_order", "source": "derived:MT/properties.ts:95-116",
                 "messages": [msg("A", 1, 0, ins(0, "abcdef")),
                              msg("A", 2, 1, ann(0, 6, {"b": 1, "a": 2, "2": 3})),
                              msg("B", 3, 2, ann(2, 4, {"b": None, "1": 4})),
                              msg("A", 4, 3, ann(3, 6, {"b": 5}))],
                 "text": "abcdef",
                 "props_runs": [[0, 2, '{"2":3,"b":1,"a":2}'], [2, 1, '{"1":4,"2":3,"a":2}'],
                                [3, 1, '{"1":4,"2":3,"a":2,"b":5}'], [4, 2, '{"2":3,"b":5,"a":2}']]})
    # overlapping removes (MT/test/client.applyMsg.spec.ts:201-231): both clients remove [0,5)
    kats.append({"name": "overlapping_removes", "source": "reference:MT/test/client.applyMsg.spec.ts:201-231",
                 "messages": [msg("A", 1, 0, ins(0, "0123456789")), msg("B", 2, 1, rem(0, 5)),
                              msg("A", 3, 1, rem(0, 5))],
                 "text": "56789"})
    # MT/test/mergeTree.annotate.spec.ts:504-521 "remote first": "remote only" reads the annotated
    # segment's props, "split remote" splits it (splitAt(1)) and the right part carries the same
    # props.  DERIVED: the reference asserts only the split-off half's two props (:512-519); here a
    # concurrent remote insert performs the split, and the text and full props runs are derived.
    kats.append({"name": "split_remote_annotate", "source": "derived:MT/test/mergeTree.annotate.spec.ts:504-521",
                 "messages": [msg("remote", 1, 0, ins(0, "hello world")),
                              msg("remote", 2, 1, ann(3, 7, {"propertySource": "remote", "remoteProperty": 1})),
                              msg("other", 3, 2, ins(4, "X"))],
                 "text": "hellXo world",
                 "props_runs": [[0, 3, None], [3, 1, '{"propertySource":"remote","remoteProperty":1}'],
                                [4, 1, None], [5, 3, '{"propertySource":"remote","remoteProperty":1}'],
                                [8, 4, None]]})
    # The spec's own tree (:27-45): "hello world!", a Tile marker at annotateStart + 2 = 3 by the
    # remote client; "remote first" (:486-502) annotates [1, 5) remotely; the segment at
    # annotateStart is then "el" and splitAt(1) leaves "l" (here: split by a remote insert at 2).
    # The literal assertion (:512-519): the split-off half has propertySource "remote" and
    # remoteProperty 1 — props_runs' entry at position 3 (that "l"; the run also covers the marker at 4
    # and the "l" at 5).  The other
    # runs are derived.
    kats.append({"name": "split_remote_annotate_spec_tree",
                 "source": "reference:MT/test/mergeTree.annotate.spec.ts:27-45,486-519 (split-off half's props)",
                 "messages": [msg("remote", 1, 0, ins(0, "hello world!")),
                              msg("remote", 2, 1, ins(3, {"marker": {"refType": 1}})),
                              msg("remote", 3, 2, ann(1, 5, {"propertySource": "remote", "remoteProperty": 1})),
                              msg("other", 4, 3, ins(2, "X"))],
                 "text": "heXllo world!",
                 "props_runs": [[0, 1, None], [1, 1, '{"propertySource":"remote","remoteProperty":1}'],
                                [2, 1, None], [3, 3, '{"propertySource":"remote","remoteProperty":1}'],
                                [6, 8, None]]})
    kats.extend(inserting_walk_kats())
    kats.extend(snapshot_kats())
    OUT.write_text(json.dumps(kats, indent=1))
    print(f"wrote {OUT} ({len(kats)} scenarios)")


if __name__ == "__main__":
    main()
