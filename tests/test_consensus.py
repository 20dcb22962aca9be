"""Writer consensus path and relative positions in local ops (the oracle and the packers, on CPU).

Client.annotateMarkerNotifyConsensus (client.ts:113-134) annotates a marker through its id
(createAnnotateMarkerOp, opBuilder.ts:25-39: relativePos1 {id, before: true}, relativePos2 {id},
combiningOp {name: "consensus"}) and registers the marker in pendingConsensus; the ack runs
updateConsensusProperty (client.ts:980-987: the marker re-combines the op's keys with the sequenced
seq, updating the { value: undefined, seq: -1 } its local op made in place) and queues a min-seq
listener that calls the callback once minSeq reaches the seq (mergeTree.ts:1701-1736).  A writer's
stream marks such a local message with "notifyConsensus": true (a repo-defined field: the stream
records what the client API was called with).  Local ops may address positions by marker id
(getValidOpRange, client.ts:485-543: posFromRelativePos in the local view; -1 for an unknown id,
which the local range check then drops).

The reference's tests hold no fixture for these paths (its consensus callers are in the sequence /
server packages), so the known answers below are worked by hand from the cited code and marked
derived; the farm tests compare the oracle's JSON and packed paths and the three packers."""
import json
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_ffi as O
from fluidframework_amd import oplog
from writer_sim import farm, local_message, round_farm

ROOT = Path(__file__).resolve().parents[1]
MTO_UNSUPPORTED = 4


def _msg(c, s, r, contents, msn=0):
    return {"clientId": c, "sequenceNumber": s, "referenceSequenceNumber": r, "minimumSequenceNumber": msn,
            "type": "op", "contents": contents}


def _notify(mid, props):
    return {"type": 2, "props": props, "combiningOp": {"name": "consensus"},
            "relativePos1": {"id": mid, "before": True}, "relativePos2": {"id": mid}}


MARKER = {"type": 0, "pos1": 0, "seg": {"marker": {"refType": 0}, "props": {"markerId": "m"}}}


def _local(op, ref, notify=False):
    m = local_message("W", op, ref)
    if notify:
        m["notifyConsensus"] = True
    return m


# (events of writer "W", expected text, expected props_runs of the marker, expected callbacks, status)
def _kat_registered():
    """notify -> ack re-combines {seq:-1} in place to the ack's seq -> msn 3 calls the callback;
    local inserts / removes at the marker; an unknown id drops the local op"""
    n = _notify("m", {"v": 1})
    ins = {"type": 0, "relativePos1": {"id": "m"}, "seg": "X"}                      # after m: pos 1
    rem = {"type": 1, "relativePos1": {"id": "m", "offset": 2}, "pos2": 5}        # 0 + 1 + 2 = 3 .. 5
    gone = {"type": 0, "relativePos1": {"id": "nope"}, "seg": "Q"}                # -1: not applied
    ev = [_msg("B", 1, 0, MARKER), _msg("B", 2, 1, {"type": 0, "pos1": 1, "seg": "abc"}),
          _local(n, 2, True), _local(ins, 2), _local(rem, 2), _local(gone, 2),
          _msg("W", 3, 2, n, 1), _msg("W", 4, 2, ins, 2), _msg("W", 5, 2, rem, 2),
          _msg("B", 6, 5, {"type": 0, "pos1": 0, "seg": "Z"}, 3)]
    return ev, "ZXa", {"markerId": "m", "v": {"seq": 3}}, [{"markerId": "m", "seq": 3, "minSeq": 3}], 0


def _kat_remote_first():
    """B's consensus on the marker lands while W's is pending: it sets the seq of W's {seq:-1} in
    place (segmentPropertiesManager.ts:56-63: a combining op modifies pending keys), so W's ack
    finds seq 4 !== -1 and keeps it; the callback still fires for W's seq 5"""
    n = _notify("m", {"v": 1})
    ev = [_msg("B", 1, 0, MARKER), _local(n, 1, True), _msg("B", 2, 1, {"type": 0, "pos1": 1, "seg": "ab"}, 1),
          _msg("B", 3, 1, {"type": 0, "pos1": 1, "seg": "c"}, 1),
          _msg("B", 4, 3, dict(_notify("m", {"v": 7})), 1),
          _msg("W", 5, 1, n, 1), _msg("B", 6, 5, {"type": 0, "pos1": 0, "seg": "Z"}, 5)]
    return ev, "Zcab", {"markerId": "m", "v": {"seq": 4}}, [{"markerId": "m", "seq": 5, "minSeq": 5}], 0


def _kat_unregistered():
    """annotateMarker with consensus but no notify: the ack finds no pendingConsensus entry (no
    re-combine: {seq:-1} stays), and its listener's callback is undefined — a TypeError once msn
    reaches the seq"""
    n = _notify("m", {"v": 1})
    ev = [_msg("B", 1, 0, MARKER), _local(n, 1), _msg("W", 2, 1, n, 1), _msg("B", 3, 2, {"type": 0, "pos1": 0, "seg": "Z"}, 1)]
    ev_fire = ev + [_msg("B", 4, 3, {"type": 0, "pos1": 0, "seg": "Y"}, 2)]
    return ev, ev_fire


def oracle_writer(events, name="W"):
    d = O.Doc()
    d.start_collab(name)
    for m in events:
        if m["sequenceNumber"] == -1:
            assert d.local_op(m["contents"], bool(m.get("notifyConsensus"))) == 0, d.error
        elif d.apply_msg(json.dumps(m)) != 0:
            break
    return d


def _marker_props(d):
    runs = [json.loads(r[2]) for r in json.loads(d.props_runs()) if r[2] and "markerId" in r[2]]
    assert len(runs) == 1
    return runs[0]


@pytest.mark.parametrize("kat", [_kat_registered, _kat_remote_first], ids=["registered", "remote_first"])
def test_consensus_derived_kats(kat):
    """derived (hand-worked from client.ts / properties.ts / mergeTree.ts, not reference fixtures)"""
    ev, text, props, calls, st = kat()
    d = oracle_writer(ev)
    assert d.status == st, d.error
    assert d.text() == text
    assert _marker_props(d) == props
    assert d.consensus_events() == calls


def test_consensus_unregistered_id_throws_when_the_listener_fires():
    ev, ev_fire = _kat_unregistered()
    d = oracle_writer(ev)
    assert d.status == 0 and _marker_props(d) == {"markerId": "m", "v": {"seq": -1}} and d.consensus_events() == []
    d = oracle_writer(ev_fire)
    assert d.status == MTO_UNSUPPORTED


def consensus_farms():
    """Round farms (client.conflictFarm.spec.ts's converging schedule) with consensus and marker-id
    ops.  (Free-running farms diverge — the #1213 family — and a replica can then call
    annotateMarkerNotifyConsensus on a marker another replica already removed, which puts the
    { seq: -1 } object on text there: a shared-object case the GPU flags MT_UNSUPPORTED;
    test_oracle_packed_consensus_matches_json_replay still runs one on the oracle.)"""
    return [round_farm(4, 40, 61, markers=30, consensus=40), round_farm(3, 30, 62, markers=40, consensus=50, rewrite=10)]


def _packed_writer(events, name):
    p = oplog.Packer()
    p.add_document(events, name)
    pb = p.finish()
    t = O.Tables(pb.keys or ["_"], pb.values)
    d = O.replay_doc(pb.ops.copy(), pb.text, pb.props, t, pb.clients[0])
    d._t = t
    return d, pb


def test_oracle_packed_consensus_matches_json_replay():
    """The packed records (MT_RELF_NOTIFY RELPOS, ack pos1 = relativePos1.id) replay on the
    oracle exactly like the JSON events, callbacks included."""
    n_notify = n_calls = 0
    for f in consensus_farms() + [farm(4, 700, 61, markers=30, consensus=40), None]:
        streams = {"W": _kat_registered()[0], "W2": _kat_remote_first()[0]} if f is None else \
            {n: f.events[n] for n in f.names}
        for name, ev in streams.items():
            ref = f.docs[name] if f is not None else oracle_writer(ev, "W")
            got, pb = _packed_writer(ev, name if f is not None else "W")
            assert got.status == ref.status, (name, got.error, ref.error)
            if ref.status:
                continue
            assert got.digest() == ref.digest() and got.props_runs() == ref.props_runs() and got.text() == ref.text()
            assert got.consensus_events() == ref.consensus_events()
            n_calls += len(ref.consensus_events())
            n_notify += int(((oplog.rec_type(pb.ops) == oplog.OP_RELPOS) & ((pb.ops["flags"] & oplog.RELF_NOTIFY) != 0)).sum())
    assert n_notify > 20 and n_calls > 20


def test_consensus_streams_pack_identically():
    """The native ingest == the Python packer on consensus / relative-position writer streams."""
    from fluidframework_amd.mtreplay import PackedJson

    f = consensus_farms()[0]
    p = oplog.Packer()
    for n in f.names:
        p.add_document(f.events[n], n)
    want = p.finish()
    pj = PackedJson([json.dumps({"replica": n, "messages": f.events[n]}) for n in f.names], n_threads=2)
    got = pj.arrays()
    pj.close()
    assert (got.doc_op_off == want.doc_op_off).all()
    assert (got.ops == want.ops).all()
    assert (got.text == want.text).all()
    assert len(got.props) == len(want.props) and (got.props == want.props).all()
    assert got.keys == want.keys and got.values == want.values and got.clients == want.clients


NODE = shutil.which("node")


@pytest.mark.skipif(NODE is None, reason="node not available")
def test_consensus_streams_node_packer_byte_identical(tmp_path):
    f = consensus_farms()[1]
    src = tmp_path / "ev.json"
    src.write_text(json.dumps([[n, f.events[n]] for n in f.names]))
    code = ("const {Packer}=require('./fluidframework_amd/js');const fs=require('fs');"
            f"const docs=JSON.parse(fs.readFileSync({json.dumps(str(src))},'utf8'));const p=new Packer();"
            "for(const [n,d] of docs)p.addDocument(d,n);const r=p.finish();"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'ops.bin'))},r.ops);"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'meta.json'))},JSON.stringify({{values:r.values}}));")
    r = subprocess.run([NODE, "-e", code], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    p = oplog.Packer()
    for n in f.names:
        p.add_document(f.events[n], n)
    want = p.finish()
    assert np.frombuffer((tmp_path / "ops.bin").read_bytes(), oplog.OP_DTYPE).tobytes() == want.ops.tobytes()
    assert json.loads((tmp_path / "meta.json").read_text())["values"] == want.values


def test_notify_on_another_op_shape_is_unsupported():
    bad = _notify("m", {"v": 1})
    bad["relativePos1"]["offset"] = 1
    ev = [_msg("B", 1, 0, MARKER), _local(bad, 1, True)]
    with pytest.raises(oplog.UnsupportedOp):
        oplog.pack_documents([ev], observer="W")
    no_rel = {"type": 2, "pos1": 0, "pos2": 1, "props": {"v": 1}, "combiningOp": {"name": "consensus"}}
    with pytest.raises(oplog.UnsupportedOp):  # updateConsensusProperty reads relativePos1.id: a TypeError
        oplog.pack_documents([[_msg("B", 1, 0, MARKER), _local(no_rel, 1), _msg("W", 2, 1, no_rel, 1)]], observer="W")
