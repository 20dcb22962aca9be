"""regeneratePendingOp on the oracle (client.ts:674-766, 855-893), pinned by the reference's
resetPendingSegmentsToOp.spec.ts (literal pending-group counts) and the reconnect farm's
convergence (client.reconnectFarm.spec.ts: one replica's ops are held back, regenerated after the
others' ops and resubmitted; every replica converges)."""
import json
import random

import pytest

import oracle_ffi as O
from writer_sim import random_op

INSERTS = 5
EXPECTED_SEGMENTS = INSERTS * 2 - 1


class Spec:
    """resetPendingSegmentsToOp.spec.ts:11-39: 'local user' inserts "hello" at 0..4 locally."""

    def __init__(self):
        self.c = O.Doc()
        self.c.start_collab("local user")
        self.ops = []
        self.seq = 0
        for i in range(INSERTS):
            op = {"pos1": i, "seg": "hello", "type": 0}
            assert self.c.local_op(op) == 0
            self.ops.append(op)
            assert self.c.pending_groups() == i + 1

    def apply_op_list(self):
        while self.ops:
            op = self.ops.pop(0)
            if op:
                self.seq += 1
                msg = {"clientId": "local user", "sequenceNumber": self.seq, "referenceSequenceNumber": 0,
                       "minimumSequenceNumber": 0, "type": "op", "contents": op}
                assert self.c.apply_msg(json.dumps(msg)) == 0, self.c.error


def test_acked_insert_segment():  # :41-44
    s = Spec()
    s.apply_op_list()
    assert s.c.pending_groups() == 0


def test_nacked_insert_segment():  # :46-55
    s = Spec()
    s.ops = [s.c.regenerate(op) for op in s.ops]
    assert s.c.pending_groups() == EXPECTED_SEGMENTS
    s.apply_op_list()
    assert s.c.pending_groups() == 0


def test_nacked_remove_range():  # :66-78
    s = Spec()
    s.apply_op_list()
    s.ops.append({"pos1": 0, "pos2": s.c.length(), "type": 1})
    assert s.c.local_op(s.ops[-1]) == 0
    s.ops.append(s.c.regenerate(s.ops.pop(0)))
    assert s.c.pending_groups() == EXPECTED_SEGMENTS
    s.apply_op_list()
    assert s.c.pending_groups() == 0
    assert s.c.text() == ""


def test_nacked_insert_and_remove():  # :80-90
    s = Spec()
    op = {"pos1": 0, "pos2": s.c.length(), "type": 1}
    assert s.c.local_op(op) == 0
    s.ops.append(op)
    s.ops = [s.c.regenerate(o) for o in s.ops]
    assert s.c.pending_groups() == EXPECTED_SEGMENTS * 2
    s.apply_op_list()
    assert s.c.pending_groups() == 0


def test_nacked_annotate_range():  # :101-113
    s = Spec()
    s.apply_op_list()
    op = {"pos1": 0, "pos2": s.c.length(), "props": {"foo": "bar"}, "type": 2}
    assert s.c.local_op(op) == 0
    s.ops.append(op)
    s.ops.append(s.c.regenerate(s.ops.pop(0)))
    assert s.c.pending_groups() == EXPECTED_SEGMENTS
    s.apply_op_list()
    assert s.c.pending_groups() == 0
    assert json.loads(s.c.props_runs()) == [[0, 25, json.dumps({"foo": "bar"}, separators=(",", ":"))]]


def test_nacked_insert_and_annotate():  # :115-125
    s = Spec()
    op = {"pos1": 0, "pos2": s.c.length(), "props": {"foo": "bar"}, "type": 2}
    assert s.c.local_op(op) == 0
    s.ops.append(op)
    s.ops = [s.c.regenerate(o) for o in s.ops]
    assert s.c.pending_groups() == EXPECTED_SEGMENTS * 2
    s.apply_op_list()
    assert s.c.pending_groups() == 0


def reconnect_farm(n_clients, rounds, seed, ops_per_round=(4, 40)):
    """client.reconnectFarm.spec.ts's schedule: each round every replica is caught up at S; random
    replicas issue local ops; replica 1's messages are held back while the others' are sequenced
    and applied; then replica 1 regenerates each held op (regeneratePendingOp) and the resubmitted
    ops are sequenced and applied."""
    rng = random.Random(seed)
    names = [chr(ord("A") + i) for i in range(n_clients)]
    docs = {}
    for n in names:
        d = O.Doc()
        d.start_collab(n)
        docs[n] = d
    obs = O.Doc()
    obs.start_collab("readonly")
    seq = 0
    msn = 0
    events = {n: [] for n in names}
    for _ in range(rounds):
        s0 = seq
        pending = []
        for _ in range(rng.randrange(*ops_per_round)):
            n = rng.choice(names)
            op = random_op(rng, docs[n].length(), p_annotate=30, p_remove=30)
            if docs[n].length() < 16:
                op = random_op(rng, docs[n].length(), p_annotate=0, p_remove=0)
            assert docs[n].local_op(op) == 0
            events[n].append({"clientId": n, "sequenceNumber": -1, "referenceSequenceNumber": s0,
                              "minimumSequenceNumber": 0, "type": "op", "contents": op})
            pending.append((n, op, s0))
        held = [(n, op) for n, op, _ in pending if n == names[1]]
        msgs = []
        for n, op, ref in pending:
            if n == names[1]:
                continue
            seq += 1
            msgs.append({"clientId": n, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                         "minimumSequenceNumber": s0, "type": "op", "contents": op})
        for m in msgs:
            for n in names:
                events[n].append(m)
                assert docs[n].apply_msg(json.dumps(m)) == 0, docs[n].error
            assert obs.apply_msg(json.dumps(m)) == 0
        r = docs[names[1]]
        regen = []
        for n, op in held:
            new = r.regenerate(op)
            events[names[1]].append({"clientId": names[1], "sequenceNumber": -1, "type": "regenerate",
                                     "contents": op})
            regen.append({"clientId": names[1], "sequenceNumber": 0,
                          "referenceSequenceNumber": r.L.mto_current_seq(r.h), "minimumSequenceNumber": s0,
                          "type": "op", "contents": new})
        for m in regen:
            seq += 1
            m["sequenceNumber"] = seq
            for n in names:
                events[n].append(m)
                assert docs[n].apply_msg(json.dumps(m)) == 0, docs[n].error
            assert obs.apply_msg(json.dumps(m)) == 0
    return names, docs, obs, events


@pytest.mark.parametrize("n_clients,seed", [(2, 1), (4, 2), (8, 3)])
def test_reconnect_farm_converges(n_clients, seed):
    names, docs, obs, _ = reconnect_farm(n_clients, 3, seed)
    for n in names:
        assert docs[n].pending_groups() == 0
        assert docs[n].text() == obs.text(), n


def test_packed_reconnect_streams_replay_like_the_json_ones():
    """A reconnecting writer's stream packed by oplog (MT_OP_REGENERATE records) rebuilds the same
    replica and the same regenerated ops on the oracle's packed path."""
    from fluidframework_amd import oplog

    names, docs, _, events = reconnect_farm(4, 3, 7)
    r = names[1]
    assert any(e.get("type") == "regenerate" for e in events[r])
    p = oplog.Packer()
    for n in names:
        p.add_document(events[n], n)
    pb = p.finish()
    t = O.Tables(pb.keys or ["_"], pb.values)
    for i, n in enumerate(names):
        recs = pb.ops[pb.doc_op_off[i]:pb.doc_op_off[i + 1]].copy()
        d = O.replay_doc(recs, pb.text, pb.props, t, pb.clients[i])
        assert d.status == 0, d.error
        assert d.digest() == docs[n].digest() and d.dump() == docs[n].dump()
        assert d.regenerated_ops() == docs[n].regenerated_ops()
    assert len(docs[r].regenerated_ops()) > 0
