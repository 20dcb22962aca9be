"""Op logs with combiningOp annotates (properties.ts:26-60, segmentPropertiesManager.ts:96-101),
shared by the CPU packer / oracle tests and the GPU parity tests."""
import json
import random

import oracle_ffi as O


def _msg(c, s, r, contents, msn=0):
    return {"clientId": c, "sequenceNumber": s, "referenceSequenceNumber": r, "minimumSequenceNumber": msn,
            "type": "op", "contents": contents}


def combine_farm(n_ops, seed, n_clients=6, lag=16):
    """A valid conflict-farm log whose annotates use combiningOps (properties.ts:26-60) next to plain
    and "rewrite" annotates: "incr" (numeric defaults, keys holding numbers -> NaN), "consensus"
    (absent keys -> {value: undefined, seq} or the defaultValue with seq -1 updated), any other
    name (keeps the value, absent -> defaultValue).  Keys are typed so that every combine stays on
    the device's path (incr never meets a string)."""
    rnd = random.Random(seed)
    names = [f"w{i}" for i in range(n_clients)]
    model = O.Doc()
    model.start_collab("readonly")
    short, last_ref, msgs = {}, {}, []
    for k in range(1, n_ops + 1):
        c = names[rnd.randrange(n_clients)]
        ref = max(last_ref.get(c, 0), k - 1 - rnd.randrange(lag + 1))
        last_ref[c] = ref
        msn = min(last_ref.values()) if len(last_ref) == n_clients else 0
        sid = short.get(c, len(short) + 1)
        n = model.view_length(ref, sid)
        u = rnd.randrange(100)
        if n < 4 or u < 45:
            seg = "".join(rnd.choice("abcdef\n") for _ in range(rnd.randint(1, 5)))
            if rnd.random() < 0.2:
                seg = {"text": seg, "props": {"n": rnd.randrange(3)}}
            contents = {"type": 0, "pos1": rnd.randrange(n + 1), "seg": seg}
        else:
            a = rnd.randrange(n)
            b = min(n, a + 1 + rnd.randrange(6))
            if u < 70:
                contents = {"type": 1, "pos1": a, "pos2": b}
            else:
                v = rnd.randrange(8)
                if v == 0:
                    contents = {"type": 2, "pos1": a, "pos2": b, "props": {"n": rnd.randrange(3), "k": "x"}}
                elif v == 1:
                    cop = {"name": "incr"}
                    if rnd.random() < 0.5:
                        cop["defaultValue"] = rnd.randrange(-2, 3)
                    if rnd.random() < 0.3:
                        cop["minValue"] = 1
                    contents = {"type": 2, "pos1": a, "pos2": b, "props": {"n": 1}, "combiningOp": cop}
                elif v == 2:
                    cop = {"name": "consensus"}
                    r = rnd.random()
                    if r < 0.3:
                        cop["defaultValue"] = {"value": rnd.randrange(3), "seq": -1}
                    elif r < 0.5:
                        cop["defaultValue"] = rnd.choice(["d", 7, True])
                    contents = {"type": 2, "pos1": a, "pos2": b, "props": {"c": 0}, "combiningOp": cop}
                elif v == 3:
                    contents = {"type": 2, "pos1": a, "pos2": b, "props": {"o": None},
                                "combiningOp": {"name": "keep", "defaultValue": rnd.choice(["p", 2, None])}}
                elif v == 4:
                    contents = {"type": 2, "pos1": a, "pos2": b, "props": {"k": rnd.choice(["x", "y"])},
                                "combiningOp": {"name": "rewrite"}}
                else:
                    contents = {"type": 2, "pos1": a, "pos2": b, "props": {"k": rnd.choice(["x", "y", None])}}
        m = _msg(c, k, ref, contents, msn)
        assert model.apply_msg(json.dumps(m)) == 0, model.error()
        short.setdefault(c, len(short) + 1)
        msgs.append(m)
    return msgs


COMBINE_DOCS = [
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "hello world", "props": {"n": 5, "s": "ab"}}}),
     _msg("B", 2, 1, {"type": 2, "pos1": 0, "pos2": 5, "props": {"n": 1, "z": None},
                      "combiningOp": {"name": "incr", "defaultValue": 2, "minValue": 3}}),
     _msg("A", 3, 2, {"type": 2, "pos1": 3, "pos2": 8, "props": {"c": 1, "d": 1},
                      "combiningOp": {"name": "consensus", "defaultValue": {"value": 7, "seq": -1}}}, 1),
     _msg("B", 4, 3, {"type": 2, "pos1": 6, "pos2": 11, "props": {"e": 1}, "combiningOp": {"name": "consensus"}}, 2),
     _msg("A", 5, 4, {"type": 2, "pos1": 0, "pos2": 11, "props": {"q": 1}, "combiningOp": {"name": "zzz", "defaultValue": "dv"}}, 3),
     _msg("A", 6, 5, {"type": 0, "pos1": 11, "seg": "!"}, 5)],
    # incr of an absent key with a string default: "<default>undefined", clamped to a larger string minValue
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abcdef"}),
     _msg("A", 2, 1, {"type": 2, "pos1": 0, "pos2": 3, "props": {"s": 0},
                      "combiningOp": {"name": "incr", "defaultValue": "a", "minValue": "b"}}),
     _msg("A", 3, 2, {"type": 2, "pos1": 3, "pos2": 6, "props": {"s": 0},
                      "combiningOp": {"name": "incr", "defaultValue": "c", "minValue": "b"}}, 2)],
    # NaN never matches, not even itself: the halves of a split stay apart after zamboni
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "abcdefgh", "props": {"n": 1}}}),
     _msg("A", 2, 1, {"type": 2, "pos1": 2, "pos2": 5, "props": {"n": 0}, "combiningOp": {"name": "incr"}}),
     _msg("A", 3, 2, {"type": 2, "pos1": 0, "pos2": 8, "props": {"n": 0}, "combiningOp": {"name": "incr"}}, 2),
     _msg("A", 4, 3, {"type": 0, "pos1": 8, "seg": "z"}, 3),
     _msg("A", 5, 4, {"type": 0, "pos1": 9, "seg": "y"}, 4)],
]



def _probe_ok(msgs):
    """True when the oracle replays `msgs` without an error status."""
    d = O.Doc()
    d.start_collab("readonly")
    for m in msgs:
        if d.apply_msg(json.dumps(m)) != 0:
            return False
    return True


def _live_ids(doc):
    """ids of the markers the oracle's segment table holds and has not removed (mto_dump lines;
    a marker zamboni unlinked is gone from the table)"""
    out = set()
    for ln in doc.dump().splitlines():
        if '"markerId"' in ln and " rseq=none " in ln:
            out.add(json.loads(ln[ln.index("{"):])["markerId"])
    return out


def relpos_farm(n_ops, seed, n_clients=5, lag=12, rel_pct=20, live_ids_only=False):
    """A valid conflict-farm log with markers carrying ids (props.markerId) and ops addressed by
    relative positions (relativePos1 / relativePos2: a marker id, before, offset — client.ts:485-502,
    mergeTree.ts:1942-1966).  Every relative op is checked by replaying the log with the oracle;
    one that would fail is replaced by a positional insert.  live_ids_only: relative ops name only
    markers not removed so far (a SnapshotV1 reload maps only those: snapshotLoader via
    reloadFromSegments' addNodeReferences, mergeTree.ts:270-285)."""
    rnd = random.Random(seed)
    names = [f"r{i}" for i in range(n_clients)]
    model = O.Doc()
    model.start_collab("readonly")
    short, last_ref, msgs, ids = {}, {}, [], []
    for k in range(1, n_ops + 1):
        c = names[rnd.randrange(n_clients)]
        ref = max(last_ref.get(c, 0), k - 1 - rnd.randrange(lag + 1))
        last_ref[c] = ref
        msn = min(last_ref.values()) if len(last_ref) == n_clients else 0
        sid = short.get(c, len(short) + 1)
        n = model.view_length(ref, sid)
        u = rnd.randrange(100)
        contents = None
        cands = ids
        if live_ids_only and ids and u < rel_pct:
            live = _live_ids(model)
            cands = [i for i in ids if i in live]
        if cands and u < rel_pct:
            rel = {"id": rnd.choice(cands)}
            if rnd.random() < 0.5:
                rel["before"] = True  # (an offset before a marker can reach below 0: not on the device)
            elif rnd.random() < 0.4:
                rel["offset"] = rnd.randrange(0, 3)
            kind = rnd.randrange(3)
            if kind == 0:
                contents = {"type": 0, "relativePos1": rel, "seg": rnd.choice(["x", "yz", "\n"])}
            elif kind == 1 and n > 0:
                contents = {"type": 1, "pos1": rnd.randrange(n), "relativePos2": rel}
            else:
                contents = {"type": 2, "relativePos1": rel, "pos2": n, "props": {"r": rnd.randrange(3)}}
            if not _probe_ok(msgs + [_msg(c, k, ref, contents, msn)]):
                contents = None
        if contents is None:
            if n < 4 or u < 60:
                if rnd.random() < 0.25:
                    mid = f"m{k}"
                    ids.append(mid)
                    seg = {"marker": {"refType": 1}, "props": {"markerId": mid}}
                else:
                    seg = "".join(rnd.choice("abcde") for _ in range(rnd.randint(1, 4)))
                contents = {"type": 0, "pos1": rnd.randrange(n + 1), "seg": seg}
            else:
                a = rnd.randrange(n)
                b = min(n, a + 1 + rnd.randrange(4))
                contents = {"type": 1, "pos1": a, "pos2": b} if u < 85 else \
                    {"type": 2, "pos1": a, "pos2": b, "props": {"k": rnd.randrange(3)}}
        m = _msg(c, k, ref, contents, msn)
        assert model.apply_msg(json.dumps(m)) == 0, model.error
        short.setdefault(c, len(short) + 1)
        msgs.append(m)
    return msgs


RELPOS_DOCS = [
    # insert before / after a marker, with offsets; a range ending at a marker
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "hello world"}),
     _msg("A", 2, 1, {"type": 0, "pos1": 5, "seg": {"marker": {"refType": 1}, "props": {"markerId": "p1"}}}),
     _msg("B", 3, 2, {"type": 0, "relativePos1": {"id": "p1"}, "seg": "A"}),
     _msg("B", 4, 3, {"type": 0, "relativePos1": {"id": "p1", "before": True}, "seg": "B"}),
     _msg("A", 5, 3, {"type": 0, "relativePos1": {"id": "p1", "offset": 2}, "seg": "C"}),
     _msg("B", 6, 5, {"type": 1, "pos1": 0, "relativePos2": {"id": "p1", "before": True, "offset": 1}}),
     _msg("A", 7, 6, {"type": 2, "relativePos1": {"id": "p1"}, "pos2": 9, "props": {"x": 1}})],
    # numeric id (idToSegment keys are strings: 7 and "7" are the same key), ids in a group
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abcdef"}),
     _msg("A", 2, 1, {"type": 3, "ops": [
         {"type": 0, "pos1": 3, "seg": {"marker": {"refType": 2}, "props": {"markerId": 7}}},
         {"type": 0, "relativePos1": {"id": "7", "before": True}, "seg": "Q"}]}),
     _msg("B", 3, 1, {"type": 0, "relativePos1": {"id": 7}, "seg": "R"})],
    # a removed marker unlinked by zamboni: the reference's map keeps the detached marker
    # (getPosition 0), so "after" it is position 1
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abcdef"}),
     _msg("A", 2, 1, {"type": 0, "pos1": 2, "seg": {"marker": {"refType": 1}, "props": {"markerId": "gone"}}}, 1),
     _msg("A", 3, 2, {"type": 1, "pos1": 2, "pos2": 3}, 2),
     _msg("A", 4, 3, {"type": 0, "pos1": 0, "seg": "zz"}, 4),
     _msg("A", 5, 4, {"type": 0, "relativePos1": {"id": "gone"}, "seg": "!"}, 5)],
]


def big_prop_docs():
    """Property sets of any size (properties.ts:95 copies every key; textSegment.ts:23-28): an insert
    of 500 props, a 130-prop insert (past the 126 a record's flags hold: MT_OPF_NPROPS_EXT), an
    annotate chain that grows a set past 300 keys over concurrent, splitting annotates of two
    clients (zamboni then merges neighbours whose big sets match), deletions, a rewrite with 80
    keys, a 200-prop marker, and combiningOps over a 100-key set.  Every message is valid for its
    view (positions within the refSeq view's length)."""
    docs = []
    big = {f"k{i}": i for i in range(500)}
    d0 = [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "abcdef", "props": big}}),
          _msg("B", 2, 1, {"type": 2, "pos1": 1, "pos2": 4, "props": {f"b{i}": "x" for i in range(20)}}),
          _msg("A", 3, 2, {"type": 1, "pos1": 2, "pos2": 3}, msn=1),
          _msg("B", 4, 3, {"type": 0, "pos1": 0, "seg": {"text": "XYZ", "props": {f"z{i}": True for i in range(130)}}}, msn=2),
          _msg("A", 5, 4, {"type": 2, "pos1": 0, "pos2": 8, "props": {"k7": None, "k8": None, "q": 1}}, msn=3),
          _msg("B", 6, 5, {"type": 0, "pos1": 8, "seg": "tail"}, msn=5),
          _msg("A", 7, 6, {"type": 2, "pos1": 0, "pos2": 12, "props": {"last": [1, 2]}}, msn=6)]
    docs.append(d0)
    rnd = random.Random(11)
    d1 = [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "0123456789", "props": {f"s{i}": i for i in range(40)}}})]
    seq, length = 1, 10
    for i in range(320):
        seq += 1
        c = "A" if i % 2 else "B"
        msn = max(0, seq - 3)
        if i == 150:
            props = {f"s{j}": j for j in range(0, 80)}
            d1.append(_msg(c, seq, seq - 1, {"type": 2, "pos1": 0, "pos2": length, "props": props,
                                               "combiningOp": {"name": "rewrite"}}, msn=msn))
            continue
        if i == 200:
            d1.append(_msg(c, seq, seq - 1, {"type": 0, "pos1": 5, "seg": {"marker": {"refType": 1},
                                                                          "props": {f"mk{j}": j for j in range(200)}}}, msn=msn))
            length += 1
            continue
        if i % 40 == 7:
            d1.append(_msg(c, seq, seq - 1, {"type": 0, "pos1": rnd.randrange(length + 1), "seg": "ab"}, msn=msn))
            length += 2
            continue
        a = rnd.randrange(0, 3)
        b = length - rnd.randrange(0, 3)
        props = {f"m{i}": i % 5}
        if i % 7 == 0 and i >= 5:
            props[f"m{i - 5}"] = None
        if i % 11 == 0:
            props.update({f"w{i}_{j}": "v" for j in range(70)})  # one op past 64 keys
        d1.append(_msg(c, seq, seq - 2 if seq > 2 else 0, {"type": 2, "pos1": a, "pos2": b, "props": props}, msn=msn))
    docs.append(d1)
    d2 = [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "numbers", "props": {f"n{i}": i for i in range(100)}}}),
          _msg("B", 2, 1, {"type": 2, "pos1": 0, "pos2": 4, "props": {"n1": 5, "n2": 5, "fresh": 5},
                           "combiningOp": {"name": "incr", "defaultValue": 1}}),
          _msg("A", 3, 2, {"type": 2, "pos1": 2, "pos2": 7, "props": {"n3": 9, "other": 2},
                           "combiningOp": {"name": "keep", "defaultValue": 7}}, msn=1),
          _msg("B", 4, 3, {"type": 0, "pos1": 7, "seg": "!"}, msn=3)]
    docs.append(d2)
    return docs
