"""The oracle's local-client path (pending segment groups, acks), pinned by the reference's own tests.

* client.applyMsg.spec.ts (MT/test, 15-381): every scenario restated on the oracle — the literal
  assertions (seq / removedSeq of the segment at 0 before and after the ack, pending group counts,
  getText) and the multi-client ones' convergence (TestClientLogger.validate: every replica's
  getText() equal), with an observer replaying the same sequenced stream as an extra replica.
* client.conflictFarm.spec.ts's property: random multi-writer farms converge — every writer and
  the observer end with the same text and property runs, with no pending groups left.
* Writer streams rebuilt from generated observer logs converge to the observer's result.
"""
import json

import numpy as np
import pytest

import oracle_ffi as O
from writer_sim import farm, round_farm, writer_log, writer_messages

LOCAL = "localUser"


def props_by_char(runs_json: str) -> list:
    """Per-character property maps (key order dropped: replicas that applied concurrent annotates
    in different orders hold the same keys and values in different insertion orders)."""
    out = []
    for start, n, pj in json.loads(runs_json):
        out.extend([None if pj is None else json.loads(pj)] * n)
    return out


def seg_lines(d):
    return [ln.strip() for ln in d.dump().splitlines() if ln.strip().startswith("S ")]


def field(line, name):
    return line.split(f"{name}=")[1].split()[0]


def op_msg(op, seq, client=LOCAL, ref=0, msn=0):
    return json.dumps({"clientId": client, "sequenceNumber": seq, "referenceSequenceNumber": ref,
                       "minimumSequenceNumber": msn, "type": "op", "contents": op})


@pytest.fixture
def client():
    """beforeEach (client.applyMsg.spec.ts:17-21): 'hello world' inserted before collaborating."""
    d = O.Doc()
    assert d.insert_local(0, json.dumps("hello world")) == 0
    d.start_collab(LOCAL)
    return d


def test_insert_text_local(client):  # spec :91-101
    op = {"type": 0, "pos1": 0, "seg": "abc"}
    assert client.local_op(op) == 0
    assert field(seg_lines(client)[0], "seq") == "-1" and "'abc'" in seg_lines(client)[0]
    assert client.apply_msg(op_msg(op, 17)) == 0
    assert field(seg_lines(client)[0], "seq") == "17"
    assert client.text() == "abchello world"


def test_remove_range_local(client):  # spec :103-113
    op = {"type": 1, "pos1": 0, "pos2": 1}
    assert client.local_op(op) == 0
    assert field(seg_lines(client)[0], "rseq") == "-1"
    assert client.apply_msg(op_msg(op, 17)) == 0
    assert field(seg_lines(client)[0], "rseq") == "17"
    assert client.text() == "ello world"


def test_annotate_segment_local(client):  # spec :115-132
    op = {"type": 2, "pos1": 0, "pos2": 1, "props": {"foo": "bar"}}
    assert client.local_op(op) == 0
    assert client.pending_groups() == 1
    assert client.apply_msg(op_msg(op, 17)) == 0
    assert client.pending_groups() == 0


def test_annotate_then_remove_local(client):  # spec :134-168
    end = len(client.text())
    ann = {"type": 2, "pos1": 0, "pos2": end, "props": {"foo": "bar"}}
    rem = {"type": 1, "pos1": 0, "pos2": end}
    assert client.local_op(ann) == 0
    assert client.pending_groups() == 1
    assert client.local_op(rem) == 0
    assert field(seg_lines(client)[0], "rseq") == "-1"
    assert client.pending_groups() == 2
    assert client.apply_msg(op_msg(ann, 17)) == 0
    assert field(seg_lines(client)[0], "rseq") == "-1"
    assert client.pending_groups() == 1
    assert client.apply_msg(op_msg(rem, 18)) == 0
    assert field(seg_lines(client)[0], "rseq") == "18"
    assert client.pending_groups() == 0


def test_multiple_interleaved_annotate_local(client):  # spec :170-198
    end = len(client.text())
    msgs = []
    seq = 0
    while end > 0:
        op = {"type": 2, "pos1": 0, "pos2": end, "props": {"end": end, "foo": "bar"}}
        assert client.local_op(op) == 0
        seq += 1
        msgs.append(op_msg(op, seq))
        end //= 2
    assert client.pending_groups() == len(msgs)
    for m in msgs:
        assert client.apply_msg(m) == 0
    assert client.pending_groups() == 0


def test_overlapping_deletes(client):  # spec :200-229
    initial = client.text()
    op = {"type": 1, "pos1": 0, "pos2": 5}
    assert client.local_op(op) == 0
    first = seg_lines(client)[0]
    assert field(first, "rseq") == "-1" and field(first, "grp") == "1"
    assert client.apply_msg(op_msg(op, 17, client="remoteClient")) == 0
    first = seg_lines(client)[0]
    assert field(first, "rseq") == "17" and field(first, "grp") == "1"
    assert client.apply_msg(op_msg(op, 18)) == 0
    first = seg_lines(client)[0]
    assert field(first, "rseq") == "17" and "grp=" not in first
    assert client.length() == len(initial) - 5
    assert client.text() == initial[5:]


def test_interleaved_inserts_annotates_and_deletes(client):  # spec :23-89
    changes = []
    for i in range(100):
        n = client.length()
        pos1 = n // 2
        imod6 = i % 6
        if imod6 in (0, 5):
            op = {"type": 1, "pos1": pos1, "pos2": max((n - pos1) // 4 - imod6 + pos1, pos1 + 1)}
        elif imod6 in (1, 4):
            op = {"type": 0, "pos1": pos1, "seg": str(i) * (imod6 + 5)}
        else:
            op = {"type": 2, "pos1": pos1, "pos2": max((n - pos1) // 3 - imod6 + pos1, pos1 + 1),
                  "props": {"foo": str(i)}}
        assert client.local_op(op) == 0
        changes.append(op_msg(op, i + 1))
    assert client.pending_groups() == 100
    observer = O.Doc()
    observer.insert_local(0, json.dumps("hello world"))
    observer.start_collab("readonly")
    for i, m in enumerate(changes):
        assert client.apply_msg(m) == 0, client.error
        assert client.pending_groups() == 99 - i
        assert observer.apply_msg(m) == 0, observer.error
    # every segment acked, no outstanding groups (spec :81-88)
    for ln in seg_lines(client):
        assert field(ln, "seq") != "-1" and "grp=" not in ln
    assert client.text() == observer.text()
    assert props_by_char(client.props_runs()) == props_by_char(observer.props_runs())


def _converge(clients_init, script):
    """Replicas named by clients_init {name: initial text}; script: (issuer, op) in order, each
    made into a message with the issuer's currentSeq as refSeq and sequenced in that order (the
    spec's makeOpMessage(op, ++seq) list), then every replica applies every message."""
    docs = {}
    for name, init in clients_init.items():
        d = O.Doc()
        if init:
            d.insert_local(0, json.dumps(init))
        d.start_collab(name)
        docs[name] = d
    obs = O.Doc()
    init0 = next(iter(clients_init.values()))
    if init0:
        obs.insert_local(0, json.dumps(init0))
    obs.start_collab("readonly")
    msgs = []
    for seq, (who, op) in enumerate(script, 1):
        d = docs[who]
        ref = d.L.mto_current_seq(d.h)
        assert d.local_op(op) == 0
        msgs.append(op_msg(op, seq, client=who, ref=ref))
    for m in msgs:
        for d in list(docs.values()) + [obs]:
            assert d.apply_msg(m) == 0, d.error
    texts = {n: d.text() for n, d in docs.items()}
    assert len(set(texts.values())) == 1, texts
    assert obs.text() == next(iter(texts.values()))
    for d in docs.values():
        assert d.pending_groups() == 0
    return obs.text()


def test_overlapping_insert_and_delete():  # spec :231-258
    # the spec's first message is applied by both before the rest are made
    docs = {"localUser": O.Doc(), "remoteUser": O.Doc()}
    for n, d in docs.items():
        d.insert_local(0, json.dumps("hello world"))
        d.start_collab(n)
    obs = O.Doc()
    obs.insert_local(0, json.dumps("hello world"))
    obs.start_collab("readonly")
    first = {"type": 0, "pos1": 0, "seg": "-"}
    docs["localUser"].local_op(first)
    m1 = op_msg(first, 1, client="localUser", ref=0)
    for d in list(docs.values()) + [obs]:
        assert d.apply_msg(m1) == 0
    script = [("localUser", {"type": 0, "pos1": 0, "seg": "L"}), ("localUser", {"type": 1, "pos1": 1, "pos2": 2}),
              ("remoteUser", {"type": 0, "pos1": 0, "seg": "R"}), ("remoteUser", {"type": 1, "pos1": 1, "pos2": 2})]
    msgs = []
    for seq, (who, op) in enumerate(script, 2):
        d = docs[who]
        ref = d.L.mto_current_seq(d.h)
        assert d.local_op(op) == 0
        msgs.append(op_msg(op, seq, client=who, ref=ref))
    for m in msgs:
        for d in list(docs.values()) + [obs]:
            assert d.apply_msg(m) == 0
    assert docs["localUser"].text() == docs["remoteUser"].text() == obs.text()


def test_intersecting_insert_after_local_delete():  # spec :260-288
    _converge({"A": "", "B": "", "C": ""},
              [("C", {"type": 0, "pos1": 0, "seg": "c"}), ("C", {"type": 1, "pos1": 0, "pos2": 1}),
               ("B", {"type": 0, "pos1": 0, "seg": "b"}), ("C", {"type": 0, "pos1": 0, "seg": "c"})])


def test_conflicting_insert_after_shared_delete():  # spec :290-318
    _converge({"A": "a", "B": "a", "C": "a"},
              [("B", {"type": 0, "pos1": 0, "seg": "b"}), ("C", {"type": 1, "pos1": 0, "pos2": 1}),
               ("C", {"type": 0, "pos1": 0, "seg": "c"})])


def test_local_remove_followed_by_conflicting_insert():  # spec :320-346
    _converge({"A": "", "B": "", "C": ""},
              [("C", {"type": 0, "pos1": 0, "seg": "c"}), ("B", {"type": 0, "pos1": 0, "seg": "b"}),
               ("C", {"type": 1, "pos1": 0, "pos2": 1}), ("C", {"type": 0, "pos1": 0, "seg": "c"})])


def test_intersecting_insert_with_unack_insert_and_delete():  # spec :348-380
    _converge({"A": "", "B": "", "C": ""},
              [("C", {"type": 0, "pos1": 0, "seg": "c"}), ("B", {"type": 0, "pos1": 0, "seg": "bb"}),
               ("B", {"type": 1, "pos1": 0, "pos2": 1})])


def test_local_op_with_invalid_range_is_not_applied(client):
    # getValidOpRange's local check (client.ts:504-543): logged, not applied, nothing pending
    n = client.length()
    for op in ({"type": 1, "pos1": n, "pos2": n + 1}, {"type": 2, "pos1": 2, "pos2": 2, "props": {"a": 1}},
               {"type": 0, "pos1": n + 1, "seg": "x"}):
        assert client.local_op(op) == 0
    assert client.pending_groups() == 0 and client.text() == "hello world"


def test_issue_1213_writer_diverges_from_the_observer():
    """mergeTree.markRangeRemoved.spec.ts:111-164 (it.skip: the reference's writer replica and its
    observer disagree when a replica that acked its insert + remove of "a" inserts "c" while
    another's concurrent "X" is unseen).  The observer block is the expected text "cX"; the writer
    ends with "Xc" — the divergence the skipped test records."""
    obs = O.Doc()
    obs.start_collab("3")
    for m in (op_msg({"type": 0, "pos1": 0, "seg": "a"}, 1, client="1", ref=0),
              op_msg({"type": 1, "pos1": 0, "pos2": 1}, 2, client="1", ref=0),
              op_msg({"type": 0, "pos1": 0, "seg": "X"}, 3, client="2", ref=0),
              op_msg({"type": 0, "pos1": 0, "seg": "c"}, 4, client="1", ref=2)):
        assert obs.apply_msg(m) == 0
    assert obs.text() == "cX"
    act = O.Doc()
    act.start_collab("1")
    op1, op2, op4 = ({"type": 0, "pos1": 0, "seg": "a"}, {"type": 1, "pos1": 0, "pos2": 1},
                     {"type": 0, "pos1": 0, "seg": "c"})
    assert act.local_op(op1) == 0 and act.local_op(op2) == 0
    assert act.apply_msg(op_msg(op1, 1, client="1", ref=0)) == 0
    assert act.apply_msg(op_msg(op2, 2, client="1", ref=0)) == 0
    assert act.local_op(op4) == 0
    assert act.apply_msg(op_msg({"type": 0, "pos1": 0, "seg": "X"}, 3, client="2", ref=0)) == 0
    assert act.apply_msg(op_msg(op4, 4, client="1", ref=2)) == 0
    assert act.text() == "Xc" != obs.text()


@pytest.mark.parametrize("seed,n_clients,rounds,rewrite", [(1, 3, 40, 0), (2, 5, 40, 0), (3, 8, 30, 20),
                                                          (4, 2, 60, 30)])
def test_conflict_farm_converges(seed, n_clients, rounds, rewrite):
    """client.conflictFarm.spec.ts's property on the oracle's writer replicas (its round schedule)."""
    f = round_farm(n_clients, rounds, seed, initial="hello world" if seed % 2 else "", rewrite=rewrite)
    steps = rounds
    obs_text, obs_runs = f.observer.text(), props_by_char(f.observer.props_runs())
    assert len(f.log) > steps // 4
    for n, d in f.docs.items():
        assert d.status == 0, d.error
        assert d.pending_groups() == 0
        assert d.text() == obs_text, n
        assert props_by_char(d.props_runs()) == obs_runs, n


@pytest.mark.parametrize("mk", [lambda: farm(4, 500, 11, rewrite=10), lambda: round_farm(4, 30, 12, rewrite=10)])
def test_farm_event_streams_replay_to_the_same_replica(mk):
    """A recorded writer stream, replayed by a fresh replica (local ops + acks), rebuilds the
    writer's exact state — the stream is what the GPU path ingests."""
    f = mk()
    for n, d in f.docs.items():
        r = O.Doc()
        r.start_collab(n)
        for m in f.events[n]:
            if m["sequenceNumber"] == -1:
                assert r.local_op(m["contents"]) == 0
            else:
                assert r.apply_msg(json.dumps(m)) == 0
        assert r.digest() == d.digest() and r.dump() == d.dump()


def test_writer_streams_of_generated_logs_replay():
    """Every writer's stream rebuilt from a generated observer log (writer_log) replays with every
    op acked.  Generated logs run clients at different refSeqs, so a writer can diverge from the
    observer where the #1213 race occurs (test_issue_1213_...; later ops then resolve against the
    diverged order): no convergence is asserted here — the GPU must equal this oracle replica
    exactly (tests/test_gpu_writer.py)."""
    p = O.gen_params(1200, pct_insert=55, pct_remove=35, seed=0x5EED)
    ops, text, props, off = O.gen_batch(p, 4)
    t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
    for d in range(4):
        doc_ops = ops[off[d]:off[d + 1]].copy()
        obs = O.replay_doc(doc_ops, text, props, t, names)
        assert obs.status == 0
        for w in (1 + d % p.n_clients, 1 + (d + 3) % p.n_clients):
            recs, wn = writer_log(doc_ops, names, w)
            assert (recs["seq"] == -1).sum() == ((doc_ops["tc"] >> 4) == w).sum()
            wd = O.replay_doc(recs, text, props, t, wn)
            assert wd.status == 0, wd.error
            assert wd.pending_groups() == 0
            assert wd.L.mto_current_seq(wd.h) == obs.L.mto_current_seq(obs.h)


def test_writer_messages_of_a_farm_log_converge():
    """writer_messages rebuilds each writer's stream from the farm's sequenced log alone."""
    f = round_farm(3, 30, 5)
    for n in f.names:
        msgs = writer_messages(f.log, n)
        r = O.Doc()
        r.start_collab(n)
        for m in msgs:
            if m["sequenceNumber"] == -1:
                assert r.local_op(m["contents"]) == 0
            else:
                assert r.apply_msg(json.dumps(m)) == 0
        assert r.text() == f.observer.text()
        assert r.pending_groups() == 0


def test_packed_writer_streams_replay_like_the_json_ones():
    """fluidframework_amd.oplog packs a writer's stream (local ops as seq -1 records of client 0,
    own messages as client-0 acks); the oracle's packed path rebuilds the same replica."""
    from fluidframework_amd import oplog

    f = farm(4, 600, 17, rewrite=15)
    p = oplog.Packer()
    for n in f.names:
        p.add_document(f.events[n], n)
    pb = p.finish()
    t = O.Tables(pb.keys or ["_"], pb.values)
    for i, n in enumerate(f.names):
        recs = pb.ops[pb.doc_op_off[i]:pb.doc_op_off[i + 1]].copy()
        assert (recs["seq"] == -1).any() and (((recs["tc"] >> 4) == 0) & (recs["seq"] > 0)).any()
        d = O.replay_doc(recs, pb.text, pb.props, t, pb.clients[i])
        assert d.status == 0, d.error
        assert d.digest() == f.docs[n].digest() and d.dump() == f.docs[n].dump()


def test_vectorized_writer_records_equal_writer_log():
    """oplog.writer_records (the bench's batch transform) == writer_log, record for record."""
    from fluidframework_amd import oplog

    p = O.gen_params(600, pct_insert=55, pct_remove=35, seed=0xAB)
    ops, text, props, off = O.gen_batch(p, 6)
    names = O.gen_client_names(p.n_clients)
    wof = np.array([1 + d % p.n_clients for d in range(6)])
    got, goff = oplog.writer_records(ops, off, wof)
    for d in range(6):
        recs, _ = writer_log(ops[off[d]:off[d + 1]], names, int(wof[d]))
        mine = got[goff[d]:goff[d + 1]]
        # writer_log keeps client names by remapping; writer_records swaps 0 and w
        w = int(wof[d])
        exp = recs.copy()
        order = [w] + [c for c in range(len(names)) if c != w]
        back = {new: old for new, old in enumerate(order)}
        exp_client = np.array([0 if back[int(c)] == w else (w if back[int(c)] == 0 else back[int(c)]) for c in exp["tc"] >> 4])
        oplog.set_client(exp, exp_client)
        assert mine.tobytes() == exp.tobytes(), d
