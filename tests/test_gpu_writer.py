"""GPU parity of the local-client path (writer replicas) through the C ABI (mt_writer_kernel_<SEG>).

A writer replica's log interleaves its own local ops (unsequenced, UnassignedSequenceNumber) with
the sequenced stream, in which its own messages ack them (client.ts:797-819, mergeTree.ts:
1893-1929).  The HIP replay must equal the oracle's replica bit for bit: state digest (segment table
incl. pending seqs, tombstones, leaf-block membership), tree shape, text, property runs and
SnapshotV1 (which elides unacked segments, snapshotV1.ts:184-186).
"""
import json

import numpy as np
import pytest

import oracle_ffi as O
import fluidframework_amd as fa
from writer_sim import farm, round_farm, writer_batch
from test_gpu_parity import oracle_docs_from_messages

pytestmark = pytest.mark.gpu

GEN_KEYS = [O.lib().mto_gen_key_name(k).decode() for k in range(4)]
ST_BAD_INPUT = 5  # mt_device.h: an assert of the reference (here: in the ack path)
GEN_VALUES = [O.lib().mto_gen_value_json(v).decode() for v in range(22)]


def assert_same(dv, od, what=""):
    assert dv.status == od.status, (what, fa.status_string(dv.status), od.error)
    if od.status != 0:
        return
    assert dv.digest() == od.digest(), f"{what}: digest\nGPU {dv.shape()}\nCPU {od.shape()}"
    assert dv.shape() == od.shape(), what
    assert dv.get_text() == od.text(), what
    assert dv.props_runs() == json.loads(od.props_runs()), what
    assert dv.snapshot_v1() == od.snapshot_v1(), what


def oracle_replica(name, events, initial=""):
    d = O.Doc()
    if initial:
        d.insert_local(0, json.dumps(initial))
    d.start_collab(name)
    for m in events:
        if m.get("type") == "regenerate":
            d.regenerate(m["contents"])
        elif m["sequenceNumber"] == -1:
            assert d.local_op(m["contents"], bool(m.get("notifyConsensus"))) == 0
        elif d.apply_msg(json.dumps(m)) != 0:
            break
    return d


def max_pending(name, events):
    """The most unacked local ops the oracle replica held at once before it stopped."""
    d = O.Doc()
    d.start_collab(name)
    mx = 0
    for m in events:
        if m.get("type") == "regenerate":
            d.regenerate(m["contents"])
        elif m["sequenceNumber"] == -1:
            d.local_op(m["contents"])
        elif d.apply_msg(json.dumps(m)) != 0:
            break
        mx = max(mx, d.pending_groups())
    return mx


def _farm_parity(f, **opts):
    names = list(f.names)
    docs = [f.events[n] for n in names]
    with fa.ReplayBatch(len(docs), **opts) as b:
        b.ingest_messages(docs, observer=names)
        b.run()
        for i, n in enumerate(names):
            assert_same(b.doc(i), f.docs[n], n)
        return b.stats()


@pytest.mark.parametrize("opts", [{}, {"seg_cap": 64, "max_retries": 24}], ids=["plain", "escalating"])
def test_consensus_writers_and_local_relative_positions(opts):
    """Writers calling annotateMarkerNotifyConsensus (client.ts:113-134) and issuing local ops
    addressed by marker ids (client.ts:485-543) on free-running farms, plus the hand-worked cases
    of tests/test_consensus.py: every replica on the GPU equals the oracle's — state, and the
    consensus callbacks (updateConsensusProperty's re-combine at the ack, the min-seq listener
    calls, client.ts:980-987) in call order."""
    from test_consensus import _kat_registered, _kat_remote_first, _kat_unregistered, consensus_farms

    farms = consensus_farms() + [round_farm(5, 50, 63, markers=35, consensus=45, rewrite=10)]
    docs, names, want = [], [], []
    for f in farms:
        for n in f.names:
            docs.append(f.events[n])
            names.append(n)
            want.append(f.docs[n])
    kats = [_kat_registered()[0], _kat_remote_first()[0]] + list(_kat_unregistered())
    for ev in kats:
        docs.append(ev)
        names.append("W")
        want.append(oracle_replica("W", ev))
    calls = 0
    with fa.ReplayBatch(len(docs), **opts) as b:
        b.ingest_messages(docs, observer=names)
        b.run()
        cnt = b.counters()
        for i, od in enumerate(want):
            dv = b.doc(i)
            if dv.status != od.status:  # name the record the device stopped at
                from fluidframework_amd import oplog
                p = oplog.Packer()
                p.add_document(docs[i], names[i])
                rec = p.finish().ops[int(cnt.fail_op[i])] if cnt.fail_op[i] >= 0 else None
                assert False, (i, names[i], fa.status_string(dv.status), int(cnt.fail_op[i]), rec)
            assert_same(dv, od, f"{i} {names[i]}")
            if od.status == 0:
                assert dv.consensus_events() == od.consensus_events(), i
                calls += len(od.consensus_events())
    assert want[-1].status != 0 and calls > 40


@pytest.mark.parametrize("seg_cap", [0, 64])
def test_writer_with_hundreds_of_pending_ops(seg_cap):
    """An offline burst / reconnect storm: writer A issues 300 local ops (inserts, removes,
    annotates, rewrites; splits of pending segments) before its first ack while B and C edit and
    sequence concurrently, then A catches up.  Beyond 64 pending groups the segments' mask bits are
    shared by groups 32 apart (mt_device.h pend_groups) and the entry lists decide membership:
    every replica equals the oracle's, also through checkpoint / resume with the groups in flight."""
    from writer_sim import Farm, random_op

    f = Farm(3, 77)
    for i in range(300):
        f.local("A", random_op(f.rng, f.docs["A"].length(), rewrite=10))
        if i % 4 == 0:
            o = f.rng.choice(["B", "C"])
            f.local(o, random_op(f.rng, f.docs[o].length()))
            f.deliver(o, 1 + f.rng.randrange(3))
    f.finish()
    assert max_pending("A", f.events["A"]) > 250
    _farm_parity(f, **({"seg_cap": seg_cap, "max_retries": 24} if seg_cap else {}))


def test_writer_beyond_1024_pending_ops():
    """More unacked local ops than round 5's fixed 1,024-group region: writer A issues 1,500 local
    ops before its first ack while B and C edit concurrently.  The host sizes the pending-group
    region from the log (mt_host.cpp writer_regions: the replica's peak of local records less acks,
    mt_device.h pend_groups) and the replica equals the oracle's."""
    from writer_sim import Farm, random_op

    f = Farm(3, 1501)
    for i in range(1500):
        f.local("A", random_op(f.rng, f.docs["A"].length()))
        if i % 10 == 0:
            o = f.rng.choice(["B", "C"])
            f.local(o, random_op(f.rng, f.docs[o].length()))
            f.deliver(o, 1 + f.rng.randrange(3))
    f.finish()
    assert max_pending("A", f.events["A"]) > 1024
    assert all(f.docs[n].status == 0 for n in f.names)  # (assert_same compares states only then)
    _farm_parity(f)


@pytest.mark.parametrize("seed,n_clients,steps,rewrite", [(1, 3, 400, 0), (2, 6, 900, 10), (3, 8, 1500, 25)])
def test_free_running_farm_writers(seed, n_clients, steps, rewrite):
    """Writers at their own pace (deep pending windows, remote ops on pending segments, the #1213
    race): every writer's replica on the GPU equals the oracle's.  (Pre-collaboration text starts
    from a snapshot: test_writer_replicas_starting_from_a_snapshot.)"""
    _farm_parity(farm(n_clients, steps, seed, rewrite=rewrite))


def test_writer_replicas_starting_from_a_snapshot():
    """Pre-collaboration text (what commit afa32c4 took out of the free-running farms): every replica
    of a farm held "hello world" before collaborating.  Each writer's GPU replica starts from the
    SnapshotV1 of that state (snapshotLoader.ts:36-205, the host JSON parser's {"snapshot",
    "messages"} form) and replays its own stream — local ops, acks, remote ops, rewrites — equal to
    the oracle replica loaded the same way, whose text and digest equal the farm replica's (that
    one inserted the text locally before startOrUpdateCollaboration)."""
    d = O.Doc()
    d.insert_local(0, json.dumps("hello world"))
    blobs = d.snapshot_v1()
    for f in (farm(4, 700, 31, initial="hello world", rewrite=10), round_farm(3, 25, 32, initial="hello world")):
        for n in f.names:
            od = O.Doc()
            assert od.load_snapshot(blobs, n) == 0
            for m in f.events[n]:
                if m["sequenceNumber"] == -1:
                    assert od.local_op(m["contents"]) == 0
                elif od.apply_msg(json.dumps(m)) != 0:
                    break
            if f.docs[n].status == 0:
                assert od.text() == f.docs[n].text() and od.digest() == f.docs[n].digest(), n
            with fa.ReplayBatch(1) as b:
                assert b.ingest_json([json.dumps({"snapshot": blobs, "messages": f.events[n]})], observer=n,
                                     device="host")["path"] == "host"
                b.run()
                assert_same(b.doc(0), od, n)


@pytest.mark.parametrize("seed,n_clients,rounds", [(5, 4, 40), (6, 8, 30)])
def test_conflict_farm_rounds_writers(seed, n_clients, rounds):
    """The reference's conflict-farm schedule: writers converge (checked on the oracle) and the GPU
    equals every writer exactly."""
    f = round_farm(n_clients, rounds, seed, rewrite=15)
    _farm_parity(f)
    assert len({f.docs[n].text() for n in f.names}) == 1


def test_writer_farm_with_forced_escalation():
    """Checkpoint / resume through several capacity classes with pending groups in flight (the
    pending-group region persists across launches)."""
    f = farm(5, 1500, 9, rewrite=10)
    stats = _farm_parity(f, seg_cap=64, max_retries=24)
    assert stats["launches"] >= 2


def test_issue_1213_writer_on_gpu():
    """mergeTree.markRangeRemoved.spec.ts:111-164: the writer ends with "Xc" (its observer "cX")."""
    m = lambda op, seq, c, ref: {"clientId": c, "sequenceNumber": seq, "referenceSequenceNumber": ref,  # noqa
                                 "minimumSequenceNumber": 0, "type": "op", "contents": op}
    op1, op2, op4 = ({"type": 0, "pos1": 0, "seg": "a"}, {"type": 1, "pos1": 0, "pos2": 1},
                     {"type": 0, "pos1": 0, "seg": "c"})
    events = [m(op1, -1, "1", 0), m(op2, -1, "1", 0), m(op1, 1, "1", 0), m(op2, 2, "1", 0), m(op4, -1, "1", 2),
              m({"type": 0, "pos1": 0, "seg": "X"}, 3, "2", 0), m(op4, 4, "1", 2)]
    with fa.ReplayBatch(1) as b:
        b.ingest_messages([events], observer=["1"])
        b.run()
        assert b.doc(0).get_text() == "Xc"
        assert_same(b.doc(0), oracle_replica("1", events))


def _diverged_writer_log(kind):
    """Hand-built writer-"1" logs whose local order diverged from the sequenced one: local ops with
    an invalid range are dropped (getValidOpRange, client.ts:504-543: no segment group), so the
    acks of the sequenced copies dequeue the *next* op's group and BaseSegment.ack runs the
    incoming op's rules on it (mergeTree.ts:487-522, 1893-1920).  Returns the messages and the
    index of the message the reference throws on (None: it never throws)."""
    m = lambda op, seq, c, ref, msn=0: {"clientId": c, "sequenceNumber": seq, "referenceSequenceNumber": ref,  # noqa
                                        "minimumSequenceNumber": msn, "type": "op", "contents": op}
    rm_bad, rm_bad2 = {"type": 1, "pos1": 5, "pos2": 6}, {"type": 1, "pos1": 7, "pos2": 8}
    an_bad = {"type": 2, "pos1": 5, "pos2": 6, "props": {"color": "red"}}
    ins, rem = {"type": 0, "pos1": 0, "seg": "abc"}, {"type": 1, "pos1": 0, "pos2": 3}
    ins_p = {"type": 0, "pos1": 0, "seg": {"text": "abc", "props": {"bold": True}}}
    tail = [m({"type": 0, "pos1": 0, "seg": "zz"}, 5, "2", 4, 4), m({"type": 0, "pos1": 1, "seg": "y"}, 6, "2", 5, 5),
            m({"type": 0, "pos1": 0, "seg": "q"}, 7, "2", 6, 6)]
    if kind in ("orphan_removed_unlinked", "orphan_removed_held"):
        # two dropped removes: their acks run the remove rules on the insert's and the remove's
        # groups; "abc" ends with seq -1, removedSeq 1 and no group, and scourNode unlinks it
        # once minSeq reaches 1 (held while minSeq is 0)
        ev = [m(rm_bad, -1, "1", 0), m(rm_bad2, -1, "1", 0), m(ins, -1, "1", 0), m(rem, -1, "1", 0),
              m(rm_bad, 1, "1", 0), m(rm_bad2, 2, "1", 0), m(ins, 3, "1", 0), m(rem, 4, "1", 0)]
        return (ev + tail if kind == "orphan_removed_unlinked" else ev), None
    if kind == "insert_rules_on_remove_group":
        # the dropped remove's ack removes "abc" at seq 1; the insert's ack gives it seq 2 via its
        # remove group; the remove's ack finds no group
        ev = [m(rm_bad, -1, "1", 0), m(ins, -1, "1", 0), m(rem, -1, "1", 0),
              m(rm_bad, 1, "1", 0), m(ins, 2, "1", 0), m(rem, 3, "1", 0), m({"type": 0, "pos1": 0, "seg": "k"}, 4, "2", 3, 3)]
        return ev + tail, None
    if kind == "throws_later":
        # ... and the remove's ack meets the later insert's group: assert(removalInfo) throws
        ev = [m(rm_bad, -1, "1", 0), m(ins, -1, "1", 0), m(rem, -1, "1", 0), m({"type": 0, "pos1": 0, "seg": "de"}, -1, "1", 0),
              m(rm_bad, 1, "1", 0), m(ins, 2, "1", 0), m(rem, 3, "1", 0), m({"type": 0, "pos1": 0, "seg": "de"}, 4, "1", 0)]
        return ev + tail, 6
    if kind == "annotate_without_property_manager":
        ev = [m(an_bad, -1, "1", 0), m(ins, -1, "1", 0), m(an_bad, 1, "1", 0), m(ins, 2, "1", 0)]
        return ev + tail, 2
    if kind == "unassigned_insert_orphan":
        # the annotate's ack acks the insert's group (the segment has props): "abc" keeps seq -1
        # with no group — a state the device does not model (MT_UNSUPPORTED)
        ev = [m(an_bad, -1, "1", 0), m(ins_p, -1, "1", 0), m(an_bad, 1, "1", 0), m(ins_p, 2, "1", 0)]
        return ev + tail, None
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["orphan_removed_unlinked", "orphan_removed_held", "insert_rules_on_remove_group",
                                  "throws_later", "annotate_without_property_manager", "unassigned_insert_orphan"])
def test_acks_follow_the_incoming_op_type(kind):
    """A diverged replica keeps going where the reference's does: the GPU runs every ack with the
    incoming op's rules on whatever group is oldest, stops (MT_BAD_INPUT) on the record whose assert
    throws in the reference, and equals the oracle's replica before it and at the end."""
    ev, throws_at = _diverged_writer_log(kind)
    od = oracle_replica("1", ev)
    with fa.ReplayBatch(1) as b:
        b.ingest_messages([ev], observer=["1"])
        b.run()
        dv = b.doc(0)
        if kind == "unassigned_insert_orphan":
            assert od.status == 0 and dv.status == fa.MT_UNSUPPORTED, (od.error, fa.status_string(dv.status))
            return
        if throws_at is None:
            assert od.status == 0, od.error
            assert_same(dv, od, kind)
            if kind == "orphan_removed_unlinked":
                assert "abc" not in od.dump() and dv.get_text() == "qzyz"
            return
        assert od.status == ST_BAD_INPUT and dv.status == ST_BAD_INPUT, (od.error, fa.status_string(dv.status))
        assert int(b.counters()["fail_op"][0]) == throws_at
    before = ev[:throws_at]
    od = oracle_replica("1", before)
    with fa.ReplayBatch(1) as b:
        b.ingest_messages([before], observer=["1"])
        b.run()
        assert od.status == 0
        assert_same(b.doc(0), od, kind + " before the throw")


def test_pending_segments_in_snapshot_and_text():
    """A writer stopped with ops still pending: getText holds its unacked inserts, SnapshotV1 elides
    them and its pending removes (snapshotV1.ts:184-186)."""
    f = farm(3, 300, 21)
    names = list(f.names)
    docs = []
    for n in names:
        ev = list(f.events[n])
        # drop the acks of the last few local ops: they stay pending
        own = [i for i, e in enumerate(ev) if e["clientId"] == n and e["sequenceNumber"] > 0]
        cut = own[-3] if len(own) >= 3 else len(ev)
        docs.append(ev[:cut])
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs, observer=names)
        b.run()
        for i, n in enumerate(names):
            od = oracle_replica(n, docs[i])
            assert od.pending_groups() > 0
            assert_same(b.doc(i), od, n)


def _gen_writer_parity(p, n_docs, full_every=4, doc_params=None, launches=None, **opts):
    ops, text, props, off = O.gen_batch(p, n_docs, doc_params=doc_params)
    t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
    wops, woff, wnames = writer_batch(ops, off, names, lambda d: 1 + d % p.n_clients)
    stopped = []  # (doc, failing record)
    with fa.ReplayBatch(n_docs, **opts) as b:
        b.set_tables(GEN_KEYS, GEN_VALUES)
        for d in range(n_docs):
            b.set_clients(wnames[d], d)
        b.ingest(wops, woff, text, props)
        b.run()
        fail_op = b.counters()["fail_op"]
        for d in range(n_docs):
            od = O.replay_doc(wops[woff[d]:woff[d + 1]].copy(), text, props, t, wnames[d])
            dv = b.doc(d)
            assert dv.status == od.status, (d, fa.status_string(dv.status), od.error)
            if od.status == ST_BAD_INPUT:
                # a reference assert inside ackPendingSegment (the writer's local order diverged
                # from the sequenced one, the #1213 family): both sides stop at the same record,
                # and the states just before it are compared below
                stopped.append((d, int(fail_op[d])))
                continue
            assert dv.digest() == od.digest(), f"doc {d}"
            if d % full_every == 0:
                assert_same(dv, od, f"doc {d}")
        stats = b.stats()
        if launches is not None:
            launches.extend(b.launches())
    if stopped:
        _stopped_writer_parity(wops, woff, wnames, text, props, t, stopped, **opts)
    return stats


def _stopped_writer_parity(wops, woff, wnames, text, props, t, stopped, **opts):
    """A replica stopped by a reference assert: the oracle stops at the GPU's failing record — it
    applies every record before it without an error and throws on it (an ack of a pending group is
    run with the incoming op's BaseSegment.ack rules whatever op made the group, mergeTree.ts:
    487-522, 1893-1920, on both sides) — and the GPU replay of the log cut before that record
    equals the oracle's state there (digest, shape, text, props, SnapshotV1): the state immediately
    before the throw."""
    logs = []
    for d, k in stopped:
        log = wops[woff[d]:woff[d + 1]]
        assert 0 <= k < len(log), (d, k)
        od = O.replay_doc(log[:k + 1].copy(), text, props, t, wnames[d])
        assert od.status == ST_BAD_INPUT, (d, k, od.status, od.error)
        logs.append(log[:k].copy())
    off = np.zeros(len(logs) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in logs])
    with fa.ReplayBatch(len(logs), **opts) as b:
        b.set_tables(GEN_KEYS, GEN_VALUES)
        for i, (d, _) in enumerate(stopped):
            b.set_clients(wnames[d], i)
        b.ingest(np.concatenate(logs) if len(logs) else wops[:0], off, text, props)
        b.run()
        for i, (d, k) in enumerate(stopped):
            od = O.replay_doc(logs[i], text, props, t, wnames[d])
            assert od.status == 0 and b.doc(i).status == 0, (d, k, od.error)
            assert b.doc(i).digest() == od.digest(), f"doc {d} before record {k}"
            assert_same(b.doc(i), od, f"doc {d} before record {k}")


def test_generated_writer_logs_config2_shape():
    """Writers of BASELINE configs[1]-shaped logs (8 clients, lag <= 32, insert 60 / remove 40)."""
    _gen_writer_parity(O.gen_params(2000, seed=0xC0FFEE), 24)


def test_generated_writer_logs_config3_mix():
    """Writers of configs[2]-mix logs (annotate 10 %: remote annotates meet pending local keys)."""
    _gen_writer_parity(O.gen_params(1500, pct_insert=55, pct_remove=35, seed=0xBADC0DE), 24)


def test_generated_writer_logs_wide_windows():
    """24 clients, lag 200: up to ~60 pending groups per writer, deep continuation walks.  Wide
    windows make writer-order divergence common: about half of these writers stop where the
    reference's replica would (insert failed / an ack assert), the GPU at the same record."""
    _gen_writer_parity(O.gen_params(1200, n_clients=24, max_lag=200, pct_insert=50, pct_remove=40, min_len=0,
                                    max_insert=3, seed=77), 16)


def test_generated_writer_logs_early_escalation():
    """1,024 writers of config-2-shaped logs that fit class 464 and 4 whose collab window (lag up to
    400) outgrows its overlay list within a few hundred records: the first launch reports those
    while it runs and their next class starts beside it (mt_host.cpp poll_notices; writer waves of
    such launches raise their priority); every replica equals the oracle's."""
    small = O.gen_params(1500, seed=0xEA53)
    wide = O.gen_params(1500, max_lag=400, seed=0xEA54)
    n, wide_at = 1024, (3, 300, 700, 1023)
    launches = []
    _gen_writer_parity(small, n, full_every=64, doc_params=[wide if d in wide_at else small for d in range(n)],
                       launches=launches)
    first = launches[0]
    assert first["seg_class"] == 464 and first["n_docs"] == n, launches
    print([(li["seg_class"], li["n_docs"], round(li["start_ms"], 2), round(li["ms"], 2)) for li in launches])
    assert any(li["start_ms"] < first["start_ms"] + first["ms"] for li in launches[1:]), launches


def test_observer_logs_still_run_the_observer_kernel():
    """A log without local ops / own acks is an observer batch (mt_replay_kernel_<SEG>)."""
    p = O.gen_params(500, seed=4)
    ops, text, props, off = O.gen_batch(p, 4)
    t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
    _, dig, st = O.replay_batch(ops, off, text, props, t, names)
    with fa.ReplayBatch(4) as b:
        b.set_tables(GEN_KEYS, GEN_VALUES)
        b.set_clients(names)
        b.ingest(ops, off, text, props)
        b.run()
        for d in range(4):
            assert b.doc(d).digest() == int(dig[d])


def test_find_tile_kats_on_gpu():
    """client.spec.ts:29-231 (findTile literal positions) on GPU replicas of local-only logs."""
    def mk(label="EOP"):
        return {"marker": {"refType": 1}, "props": {"referenceTileLabels": [label], "markerId": "some-id"}}

    def local(ops):
        return [{"clientId": "localUser", "sequenceNumber": -1, "referenceSequenceNumber": 0,
                 "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 0, "pos1": p, "seg": s}}
                for p, s in ops]

    three = [(0, mk()), (0, "abc d"), (0, mk()), (7, "ef"), (8, mk())]
    cases = [  # (ops, [(startPos, preceding, expected pos or None)])
        ([(0, mk()), (0, "abc")], [(0, False, 3), (5, True, 3), (5, False, None)]),
        ([(0, "abc d"), (0, mk())], [(0, False, 0)]),
        (three, [(5, True, 0), (5, False, 6)]),
        ([(0, mk())], [(0, True, 0), (0, False, 0)]),
        ([(0, "abc")], [(1, True, None), (1, False, None)]),
        ([(0, "x")], []),
    ]
    docs = [local(ops) for ops, _ in cases] + [[]]
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs, observer="localUser")
        b.run()
        for i, (_, queries) in enumerate(cases):
            for start, prec, want in queries:
                got = b.doc(i).find_tile(start, "EOP", prec)
                assert (None if got is None else got["pos"]) == want, (i, start, prec)
        empty = b.doc(len(docs) - 1)
        assert empty.find_tile(1, "EOP") is None and empty.find_tile(1, "EOP", False) is None


@pytest.mark.parametrize("mk", [lambda: round_farm(4, 30, 31, markers=30), lambda: farm(5, 600, 32, markers=25),
                                lambda: round_farm(4, 40, 33, markers=35, label_annot=40),
                                lambda: farm(5, 700, 34, markers=30, ranges=10, label_annot=45)])
def test_find_tile_matches_oracle(mk):
    """Every replica (writers and observer) of farms with Tile markers: the GPU table's findTile
    equals the oracle's block-map search at every position, both directions, every label.  With
    label_annot, annotates rewrite referenceTileLabels: the reference rebuilds the block maps only in
    blockUpdate (mergeTree.ts:2748-2767), so they keep older labels — the device tracks, per marker,
    the prop set its leaf block's last blockUpdate read (parity beyond the oracle's literal maps is
    unpinned: no reference fixture holds stale maps)."""
    from writer_sim import TILE_LABELS

    f = mk()
    names = list(f.names)
    docs = [f.events[n] for n in names]
    obs_msgs = list(f.log)
    with fa.ReplayBatch(len(docs) + 1) as b:
        b.ingest_messages(docs + [obs_msgs], observer=names + ["readonly"])
        b.run()
        for i, od in enumerate([f.docs[n] for n in names] + [f.observer]):
            dv = b.doc(i)
            assert dv.digest() == od.digest()
            n = od.length()
            for label in TILE_LABELS:
                for pos in range(0, n + 2):
                    for prec in (True, False):
                        assert dv.find_tile(pos, label, prec) == od.find_tile(pos, label, prec), (i, label, pos, prec)


RANGE_QUERIES = (["row"], ["box", "row"], ["cell", "box", "row"], [])


@pytest.mark.parametrize("mk", [lambda: round_farm(4, 30, 41, ranges=35), lambda: farm(5, 600, 42, ranges=30, markers=10),
                                lambda: round_farm(4, 40, 43, ranges=35, label_annot=40),
                                lambda: farm(5, 700, 44, ranges=30, markers=10, label_annot=45)])
def test_stack_context_matches_oracle(mk):
    """Client.getStackContext (client.ts:946-948, mergeTree.ts:1750-1760) on every replica (writers
    and observer) of farms with NestBegin / NestEnd markers carrying referenceRangeLabels: the
    stacks the library rebuilds from the final table (leaves + the interior blocks each leaf block
    closes) equal the oracle's block rangeStacks search at every position, for several label sets
    (parity beyond beastTest's nesting check is unpinned: tests/test_oracle_ranges.py)."""
    f = mk()
    names = list(f.names)
    docs = [f.events[n] for n in names]
    with fa.ReplayBatch(len(docs) + 1) as b:
        b.ingest_messages(docs + [list(f.log)], observer=names + ["readonly"])
        b.run()
        for i, od in enumerate([f.docs[n] for n in names] + [f.observer]):
            dv = b.doc(i)
            assert dv.digest() == od.digest()
            for labels in RANGE_QUERIES:
                for pos in range(0, od.length() + 2):
                    assert dv.get_stack_context(pos, labels) == od.stack_context(pos, labels), (i, labels, pos)


def test_stack_context_document_trees():
    """beastTest.ts DocumentTree documents (rows / boxes / paragraphs, NestBegin / NestEnd markers):
    replayed by an observer from the writer's sequenced messages, the GPU's getStackContext gives
    the document's nesting at every text position (checkStacksAllPositions) and equals the
    oracle everywhere; after an annotate of referenceRangeLabels (stale block maps) it still equals
    the oracle."""
    import random

    from test_oracle_ranges import DocTree, add_to_tree, check_stacks_all_positions, gen_content

    class Rec:  # an oracle doc that records its local ops as sequenced messages of client "W"
        def __init__(self):
            self.d = O.Doc()
            self.d.start_collab("W")
            self.msgs = []

        def local_op(self, op):
            self.msgs.append({"clientId": "W", "sequenceNumber": len(self.msgs) + 1,
                              "referenceSequenceNumber": len(self.msgs), "minimumSequenceNumber": len(self.msgs),
                              "type": "op", "contents": op})
            return self.d.local_op(op)

        def __getattr__(self, k):
            return getattr(self.d, k)

    trees, logs = [], []
    for seed in range(4):
        rng = random.Random(100 + seed)
        children = gen_content(rng, 0.6)
        r = Rec()
        st = {"pos": 0, "ids": {"box": 0, "row": 0}}
        for c in children:
            add_to_tree(r, c, st)
        trees.append(children)
        logs.append(r.msgs)
    logs.append(logs[0] + [{"clientId": "W", "sequenceNumber": len(logs[0]) + 1, "referenceSequenceNumber": len(logs[0]),
                            "minimumSequenceNumber": len(logs[0]), "type": "op",
                            "contents": {"type": 2, "pos1": 0, "pos2": 1, "props": {"referenceRangeLabels": ["x"]}}}])
    oracle = oracle_docs_from_messages(logs)
    with fa.ReplayBatch(len(logs)) as b:
        b.ingest_messages(logs)
        b.run()
        for i, children in enumerate(trees):
            dv, od = b.doc(i), oracle[i]
            assert dv.digest() == od.digest()
            assert check_stacks_all_positions(_StackView(dv), children) == []
            for labels in RANGE_QUERIES:
                for pos in range(0, od.length() + 2):
                    assert dv.get_stack_context(pos, labels) == od.stack_context(pos, labels), (i, labels, pos)
        # the annotated document: its block maps keep the labels of their last blockUpdate
        dv, od = b.doc(len(trees)), oracle[len(trees)]
        for labels in RANGE_QUERIES + (["x"], ["x", "row"]):
            for pos in range(0, od.length() + 2):
                assert dv.get_stack_context(pos, labels) == od.stack_context(pos, labels), (labels, pos)


def test_stack_context_derived_kats_on_gpu():
    """The hand-worked getStackContext cases (tests/test_oracle_ranges.py STACK_KATS, marked
    derived) on a read-only GPU replica of each case's sequenced inserts."""
    from test_oracle_ranges import STACK_KATS, stack_kat_messages

    logs = [stack_kat_messages(k) for k in STACK_KATS]
    with fa.ReplayBatch(len(logs)) as b:
        b.ingest_messages(logs)
        b.run()
        for i, kat in enumerate(STACK_KATS):
            dv = b.doc(i)
            for pos, labels, want in kat["queries"]:
                got = dv.get_stack_context(pos, labels)
                assert got == want and list(got) == list(want), (kat["name"], pos, labels, got)


class _StackView:
    def __init__(self, dv):
        self.dv = dv

    def stack_context(self, pos, labels):
        return self.dv.get_stack_context(pos, labels)


def test_regenerate_pending_ops_on_gpu():
    """Reconnecting writers (client.reconnectFarm.spec.ts's schedule): each regeneratePendingOp on
    the GPU gives the oracle's regenerated ops, and every replica (incl. the one that regenerated
    and was then acked through its new groups) equals the oracle's."""
    from test_oracle_regenerate import reconnect_farm

    for n_clients, seed in ((2, 1), (4, 2), (8, 3)):
        names, docs, _, events = reconnect_farm(n_clients, 3, seed)
        with fa.ReplayBatch(len(names)) as b:
            b.ingest_messages([events[n] for n in names], observer=names)
            b.run()
            for i, n in enumerate(names):
                assert_same(b.doc(i), docs[n], n)
                assert b.doc(i).regenerated_ops() == docs[n].regenerated_ops(), n


def test_regenerate_with_more_than_64_pending_groups():
    """regeneratePendingOp over 130 pending local ops (reconnect with a deep queue): 110 inserts at
    random places, removes and annotates over them, every one regenerated (each regenerated op a new
    group with the original localSeq) and then acked — GPU == oracle on the regenerated ops and the
    final state."""
    import random

    rng = random.Random(5)

    def local(op):
        return {"clientId": "W", "sequenceNumber": -1, "referenceSequenceNumber": 0,
                "minimumSequenceNumber": 0, "type": "op", "contents": op}

    def regen(op):
        return {"clientId": "W", "sequenceNumber": -1, "type": "regenerate", "contents": op}

    ops, length = [], 0
    for i in range(130):
        if i < 110 or length < 4:
            op = {"type": 0, "pos1": rng.randrange(length + 1), "seg": "ab"[: 1 + rng.randrange(2)]}
            length += len(op["seg"])
        else:
            a = rng.randrange(length - 1)
            op = {"type": 1 + (i % 2), "pos1": a, "pos2": a + 1 + rng.randrange(3)}
            if op["type"] == 2:
                op["props"] = {"k": i}
            else:
                length -= op["pos2"] - a
        ops.append(op)
    ev = [local(o) for o in ops] + [regen(o) for o in ops]
    od = oracle_replica("W", ev)
    assert od.status == 0 and od.pending_groups() > 100
    acks = [{"clientId": "W", "sequenceNumber": k + 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
             "type": "op", "contents": op} for k, op in enumerate(od.regenerated_ops())]
    full = ev + acks
    od2 = oracle_replica("W", full)
    with fa.ReplayBatch(1) as b:
        b.ingest_messages([full], observer=["W"])
        b.run()
        assert b.doc(0).regenerated_ops() == od.regenerated_ops()
        assert_same(b.doc(0), od2, "regenerate")


def test_reset_pending_segments_to_op_kats_on_gpu():
    """resetPendingSegmentsToOp.spec.ts:46-125 as writer streams: regenerated inserts / removes /
    annotates, acked through the new groups (pending counts pinned on the oracle)."""
    def local(op):
        return {"clientId": "local user", "sequenceNumber": -1, "referenceSequenceNumber": 0,
                "minimumSequenceNumber": 0, "type": "op", "contents": op}

    def regen(op):
        return {"clientId": "local user", "sequenceNumber": -1, "type": "regenerate", "contents": op}

    inserts = [{"pos1": i, "seg": "hello", "type": 0} for i in range(5)]
    streams = []
    # nacked insertSegment: every insert regenerated, then the regenerated ops acked
    ev = [local(o) for o in inserts] + [regen(o) for o in inserts]
    streams.append(ev)
    # nacked insertSegment and removeRange / annotateRange
    for extra in ({"pos1": 0, "pos2": 25, "type": 1}, {"pos1": 0, "pos2": 25, "props": {"foo": "bar"}, "type": 2}):
        streams.append([local(o) for o in inserts] + [local(extra)] + [regen(o) for o in inserts + [extra]])
    # replay each stream on the oracle to learn the regenerated ops, then ack them in order
    full = []
    for ev in streams:
        od = oracle_replica("local user", ev)
        seq = 0
        acks = []
        for op in od.regenerated_ops():
            seq += 1
            acks.append({"clientId": "local user", "sequenceNumber": seq, "referenceSequenceNumber": 0,
                         "minimumSequenceNumber": 0, "type": "op", "contents": op})
        full.append(ev + acks)
    with fa.ReplayBatch(len(full)) as b:
        b.ingest_messages(full, observer="local user")
        b.run()
        for i, ev in enumerate(full):
            od = O.Doc()
            od.start_collab("local user")
            for e in ev:
                if e.get("type") == "regenerate":
                    od.regenerate(e["contents"])
                elif e["sequenceNumber"] == -1:
                    assert od.local_op(e["contents"]) == 0
                else:
                    assert od.apply_msg(json.dumps(e)) == 0, od.error
            assert od.pending_groups() == 0
            assert_same(b.doc(i), od, f"stream {i}")
            assert b.doc(i).regenerated_ops() == od.regenerated_ops()
