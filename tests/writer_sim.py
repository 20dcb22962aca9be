"""Writer-replica logs for the local-client path (TEST INFRASTRUCTURE).

A writer replica sees two kinds of events (client.ts:797-819, testClient.ts:213-234):
  * its own local ops, applied at once with UnassignedSequenceNumber — here an unsequenced message
    {"clientId": <replica>, "sequenceNumber": -1, "referenceSequenceNumber": <its currentSeq>, ...}
    (what TestClient.makeOpMessage(op) builds), and
  * the sequenced stream, in which its own messages ack its pending segment groups.

Two sources:
  * `farm`: a conflict farm in the oracle (client.conflictFarm.spec.ts's shape): writer replicas
    issue ops from their own local views, a server sequences them as they arrive (msn = the
    lowest sequence number every replica has processed, the deli rule), replicas process the
    stream at their own pace.  Every replica's event stream is recorded.
  * `writer_log`: the stream a writer `w` of a generated observer log saw.  Its op k (sequenced at
    s_k with refSeq r_k) was issued right after it processed message r_k; its position is the same
    in both views (the observer's view (r_k, w) and w's local view hold the same segments), so the
    log is rearranged, not re-derived.
"""
from __future__ import annotations

import json
import random

import numpy as np

import oracle_ffi as O

UNASSIGNED = -1


def local_message(client: str, op: dict, ref: int) -> dict:
    return {"clientId": client, "sequenceNumber": UNASSIGNED, "referenceSequenceNumber": ref,
            "minimumSequenceNumber": 0, "type": "op", "contents": op}


TILE_LABELS = ("pg", "EOP", "cell")
RANGE_LABELS = ("row", "box", "cell")


def random_op(rng: random.Random, length: int, n_keys: int = 4, p_annotate: int = 15, p_remove: int = 30,
              max_insert: int = 6, rewrite: int = 0, markers: int = 0, ranges: int = 0, label_annot: int = 0) -> dict:
    """An op drawn from a replica's local view (length = its getLength()).  markers: percentage of
    inserts that are Tile / plain markers carrying referenceTileLabels; ranges: percentage that are
    NestBegin / NestEnd markers carrying referenceRangeLabels; label_annot: percentage of annotates
    that set (or delete) referenceTileLabels / referenceRangeLabels (the block maps go stale)."""
    u = rng.randrange(100)
    if ranges and (length == 0 or u >= p_annotate + p_remove) and rng.randrange(100) < ranges:
        labels = rng.sample(RANGE_LABELS, 1 + rng.randrange(2))
        return {"type": 0, "pos1": rng.randrange(length + 1),
                "seg": {"marker": {"refType": rng.choice((2, 2, 4, 4, 3, 5, 6))},
                        "props": {"referenceRangeLabels": labels}}}
    if markers and (length == 0 or u >= p_annotate + p_remove) and rng.randrange(100) < markers:
        labels = rng.sample(TILE_LABELS, 1 + rng.randrange(2))
        return {"type": 0, "pos1": rng.randrange(length + 1),
                "seg": {"marker": {"refType": rng.choice((1, 1, 1, 0, 3))}, "props": {"referenceTileLabels": labels}}}
    if length == 0 or u >= p_annotate + p_remove:
        n = 1 + rng.randrange(max_insert)
        text = "".join(rng.choice("abcdefgh \n" if rng.randrange(10) == 0 else "abcdefgh ") for _ in range(n))
        seg = text if rng.randrange(4) else {"text": text, "props": {"k0": rng.randrange(3)}}
        return {"type": 0, "pos1": rng.randrange(length + 1), "seg": seg}
    start = rng.randrange(length)
    end = min(length, start + 1 + rng.randrange(8))
    if u < p_remove:
        return {"type": 1, "pos1": start, "pos2": end}
    props = {}
    if label_annot and rng.randrange(100) < label_annot:
        key, pool = (("referenceTileLabels", TILE_LABELS) if rng.randrange(2) else ("referenceRangeLabels", RANGE_LABELS))
        props[key] = None if rng.randrange(6) == 0 else rng.sample(pool, 1 + rng.randrange(2))
    else:
        for _ in range(1 + rng.randrange(2)):
            props[f"k{rng.randrange(n_keys)}"] = None if rng.randrange(8) == 0 else rng.randrange(4)
    op = {"type": 2, "pos1": start, "pos2": end, "props": props}
    if rewrite and rng.randrange(100) < rewrite:
        op["combiningOp"] = {"name": "rewrite"}
    return op


def id_op(rng: random.Random, ids: list, registered: set, live=None) -> tuple:
    """An op addressed by a marker id (ids: markerIds inserted so far anywhere; registered: the ids
    this replica's annotateMarkerNotifyConsensus calls registered): (op, notify).
      * Client.annotateMarkerNotifyConsensus (client.ts:113-134): createAnnotateMarkerOp's shape
        with combiningOp {name: "consensus"} (notify = True);
      * annotateMarker with consensus on an id already registered (its ack re-combines too);
      * local ops with relativePos1 / relativePos2 (client.ts:485-502): inserts, removes and
        annotates at a marker, before / after it, with offsets.
    live(id): the marker is present in the issuer's local view; only those are addressed.  (A
    removed marker's position is its detached position once zamboni dropped it — 0 — so replicas
    that zambonied at different times resolve it differently, and annotateMarkerNotifyConsensus on
    it names the next segment: its { seq: -1 } object would land on text that may split later.)"""
    u = rng.randrange(100)
    cand = [i for i in (ids if u < 35 or u >= 45 else sorted(registered)) if live is None or live(i)]
    if not cand:
        return None, False
    mid = rng.choice(cand)
    cons = {"type": 2, "props": {f"v{rng.randrange(3)}": rng.randrange(5)}, "combiningOp": {"name": "consensus"},
            "relativePos1": {"id": mid, "before": True}, "relativePos2": {"id": mid}}
    if u < 35:
        return cons, True
    if u < 45:
        return cons, False

    def rel():
        r = {"id": mid}
        if rng.randrange(2):
            r["before"] = True
        if rng.randrange(3) == 0:
            r["offset"] = rng.randrange(4)
        return r

    if u < 65:
        return {"type": 0, "relativePos1": rel(), "seg": rng.choice(["x", "yz", "\n", "abc"])}, False
    end = {"relativePos2": rel()} if rng.randrange(2) else {"pos2": 1 + rng.randrange(12)}
    if u < 80:
        return dict({"type": 1, "relativePos1": rel()}, **end), False
    return dict({"type": 2, "relativePos1": rel(), "props": {"r": rng.randrange(3)}}, **end), False


class Farm:
    """Writer replicas + an observer over one sequenced stream (all in the oracle)."""

    def __init__(self, n_clients: int, seed: int, initial: str = ""):
        self.rng = random.Random(seed)
        self.names = [chr(ord("A") + i) for i in range(n_clients)]
        self.docs = {}
        self.events = {n: [] for n in self.names}
        for n in self.names:
            d = O.Doc()
            if initial:
                assert d.insert_local(0, json.dumps(initial)) == 0
            d.start_collab(n)
            self.docs[n] = d
        self.observer = O.Doc()
        if initial:
            assert self.observer.insert_local(0, json.dumps(initial)) == 0
        self.observer.start_collab("readonly")
        self.log = []        # sequenced messages
        self.cursor = {n: 0 for n in self.names}
        self.ids = []        # markerIds inserted (step(consensus=...))
        self.registered = {n: set() for n in self.names}

    def msn(self) -> int:
        live = [c for c in self.cursor.values() if c <= len(self.log)]
        return min(live) if live else len(self.log)

    def local(self, name: str, op: dict, notify: bool = False):
        d = self.docs[name]
        if d.status != 0:
            return
        ref = d.L.mto_current_seq(d.h)
        before = d.pending_groups()
        assert d.local_op(op, notify) == 0, d.error
        msg = local_message(name, op, ref)
        if notify:  # the op came from annotateMarkerNotifyConsensus (a repo-defined stream field)
            msg["notifyConsensus"] = True
        self.events[name].append(msg)
        if d.pending_groups() == before:  # not applied (empty): nothing is submitted
            return
        if notify:
            self.registered[name].add(op["relativePos1"]["id"])
        seq = len(self.log) + 1
        self.log.append({"clientId": name, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                         "minimumSequenceNumber": self.msn(), "type": "op", "contents": op})

    def deliver(self, name: str, k: int = 1):
        d = self.docs[name]
        for _ in range(k):
            c = self.cursor[name]
            if c >= len(self.log):
                return
            m = self.log[c]
            self.events[name].append(m)
            self.cursor[name] = c + 1
            if d.apply_msg(json.dumps(m)) != 0:
                # a replica whose order diverged (the #1213 family: a remote insert beside locally
                # removed, unacked segments) can be handed a position it does not have: the
                # reference throws "MergeTree insert failed"; the replica stops here
                self.cursor[name] = len(self.log) + 10 ** 9
                return

    def issue(self, name: str, consensus=0, **op_kw):
        """One random local op of replica `name`.  consensus: percentage of local ops addressed
        by marker ids (id_op) once markers with ids exist; marker inserts then carry a markerId."""
        d = self.docs[name]
        if consensus and self.ids and self.rng.randrange(100) < consensus:
            op, notify = id_op(self.rng, self.ids, self.registered[name], lambda i: d.local_marker_pos(i) >= 0)
            if op is not None:
                self.local(name, op, notify)
            return
        op = random_op(self.rng, d.length(), **op_kw)
        seg = op.get("seg")
        if consensus and isinstance(seg, dict) and "marker" in seg:
            mid = f"{name}{len(self.ids)}"
            seg.setdefault("props", {})["markerId"] = mid
            self.ids.append(mid)
        self.local(name, op)

    def step(self, p_op=45, **op_kw):
        name = self.rng.choice(self.names)
        if self.rng.randrange(100) < p_op:
            self.issue(name, **op_kw)
        else:
            self.deliver(name, 1 + self.rng.randrange(4))

    def finish(self):
        for n in self.names:
            self.deliver(n, len(self.log))
        for m in self.log:
            if self.observer.apply_msg(json.dumps(m)) != 0:
                break


def farm(n_clients: int, n_steps: int, seed: int, initial: str = "", **kw) -> Farm:
    """Free-running farm: replicas issue ops and process the stream at their own pace, so a
    replica may have acked its own ops while another's concurrent ops are still unseen — the
    race of issue #1213 (mergeTree.markRangeRemoved.spec.ts:111-164, a skipped test: the
    reference's replicas can diverge from the observer there).  For GPU == oracle parity."""
    f = Farm(n_clients, seed, initial)
    for _ in range(n_steps):
        f.step(**kw)
    f.finish()
    return f


def round_farm(n_clients: int, n_rounds: int, seed: int, initial: str = "", max_ops: int = 24, **kw) -> Farm:
    """The reference's conflict farm schedule (client.conflictFarm.spec.ts:60-99,
    mergeTreeOperationRunner.ts:95-176): each round every replica starts caught up at seq S with
    minSeq S, random replicas issue local ops (refSeq S, each seeing its own pending ops), the
    round's messages are sequenced in issue order with msn S and every replica applies all of them.
    The reference asserts convergence for this schedule."""
    f = Farm(n_clients, seed, initial)
    for _ in range(n_rounds):
        s0 = len(f.log)
        ops = 1 + f.rng.randrange(max_ops)
        for _ in range(ops):
            f.issue(f.rng.choice(f.names), **kw)
        for m in f.log[s0:]:
            m["minimumSequenceNumber"] = s0
        for n in f.names:
            f.deliver(n, len(f.log))
    f.finish()
    return f


def writer_messages(msgs: list, w: str) -> list:
    """The event stream writer `w` saw, rebuilt from a sequenced message list (seq order)."""
    issued = {}
    for m in msgs:
        if m["clientId"] == w and m.get("type") == "op":
            issued.setdefault(m["referenceSequenceNumber"], []).append(
                local_message(w, m["contents"], m["referenceSequenceNumber"]))
    out = list(issued.get(0, []))
    for m in msgs:
        out.append(m)
        out.extend(issued.get(m["sequenceNumber"], []))
    return out


def writer_log(ops: np.ndarray, names: list, w: int):
    """writer_messages on a packed log (one document, generator / packer records): records of
    client `w` are issued as local copies (seq -1, client 0) after the last record of the message
    numbered by their refSeq, and ack as client 0; every other client keeps its name.  Returns
    (records, client names with w's name first)."""
    ops = np.asarray(ops)
    # group the records into messages (a GROUP's members share one message: GROUP_CONT chains)
    msgs, cur = [], []
    for i in range(len(ops)):
        cur.append(i)
        if not (int(ops[i]["flags"]) & 1):
            msgs.append(cur)
            cur = []
    if cur:
        msgs.append(cur)
    issued = {}
    for m in msgs:
        r0 = ops[m[0]]
        if int(r0["tc"]) >> 4 == w and int(r0["tc"]) & 0xF != 15:
            local = ops[m].copy()
            local["seq"] = UNASSIGNED
            local["tc"] = local["tc"] & 0xF  # client 0
            local["msn"] = 0
            issued.setdefault(int(r0["ref_seq"]), []).append(local)
    # short ids: w first, the others keep their order (the packed client field indexes `names`)
    order = [w] + [c for c in range(len(names)) if c != w]
    remap = np.zeros(4096, np.int64)
    for new, old in enumerate(order):
        remap[old] = new
    out = list(issued.get(0, []))
    for m in msgs:
        rec = ops[m].copy()
        rec["tc"] = (rec["tc"] & 0xF) | (remap[(rec["tc"] >> 4).astype(np.int64)] << 4).astype(np.uint16)
        out.append(rec)
        out.extend(issued.get(int(ops[m[0]]["seq"]), []))
    recs = np.concatenate(out) if out else ops[:0].copy()
    return recs, [names[c] for c in order]


def writer_batch(ops: np.ndarray, off: np.ndarray, names: list, writer_of) -> tuple:
    """writer_log over every document of a packed batch; writer_of(d) picks the writer's short id.
    Returns (ops, off, per-document client names)."""
    out, offs, docs_names = [], [0], []
    for d in range(len(off) - 1):
        recs, nm = writer_log(ops[off[d]:off[d + 1]], names, writer_of(d))
        out.append(recs)
        offs.append(offs[-1] + len(recs))
        docs_names.append(nm)
    return np.concatenate(out), np.array(offs, np.int64), docs_names
