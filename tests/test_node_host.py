"""The Node host layer (fluidframework_amd/js: N-API addon + index.js) over the C ABI.

CPU: the addon builds, loads and exports its functions; without a GPU it fails loudly.
GPU: replaying the KATs and mixed-op logs through Node gives the oracle's text, property
runs, SnapshotV1 blobs and digests (the JS packer is an independent restatement of
fluidframework_amd/oplog.py, so this also cross-checks the two packers)."""
import json
import shutil
import subprocess
from pathlib import Path

import pytest

import oracle_ffi as O
from kat_util import load_kats

ROOT = Path(__file__).resolve().parents[1]
NODE = shutil.which("node")
ADDON = ROOT / "fluidframework_amd" / "js" / "mtreplay.node"
pytestmark = pytest.mark.skipif(NODE is None or not ADDON.exists(), reason="node / N-API addon not available")

FUNCS = {"createBatch", "setTables", "setClients", "ingest", "generate", "run", "runAsync", "docStatus", "docText",
         "docPropsRuns", "docSnapshotV1", "docDigest", "deviceDigests", "stats", "statusString", "ingestJson",
         "docFindTile", "docRegeneratedOps", "docStackContext", "docConsensusEvents"}


def _node(code):
    return subprocess.run([NODE, "-e", code], capture_output=True, text=True, cwd=ROOT, timeout=60)


def test_addon_loads_and_exports():
    r = _node("const m=require('./fluidframework_amd/js/mtreplay.node');console.log(JSON.stringify(Object.keys(m)))")
    assert r.returncode == 0, r.stderr
    assert set(json.loads(r.stdout)) == FUNCS


def test_addon_fails_loudly_without_device():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    r = _node("const {ReplayBatch}=require('./fluidframework_amd/js');"
              "try{new ReplayBatch(2);console.log('created')}catch(e){console.log(e.code)}")
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "103"  # MT_ERR_NO_DEVICE


def _msg(c, s, r, contents, msn=0):
    return {"clientId": c, "sequenceNumber": s, "referenceSequenceNumber": r, "minimumSequenceNumber": msn,
            "type": "op", "contents": contents}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["applyMsg", "json"])
def test_node_replay_matches_oracle(tmp_path, mode):
    kats = load_kats()
    docs = [k["messages"] for k in kats]
    docs.append([_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "héllo wörld", "props": {"b": 1, "10": "x", "2": None}}}),
                 _msg("B", 2, 0, {"type": 0, "pos1": 0, "seg": {"marker": {"refType": 1}, "props": {"id": "m1"}}}),
                 _msg("A", 3, 1, {"type": 3, "ops": [{"type": 0, "pos1": 2, "seg": "XY"},
                                                     {"type": 2, "pos1": 0, "pos2": 4, "props": {"c": {"n": [1, 2]}}}]}),
                 _msg("B", 4, 3, {"type": 2, "pos1": 1, "pos2": 6, "props": {"c": None, "b": 2},
                                  "combiningOp": {"name": "rewrite"}}, msn=1),
                 _msg("A", 5, 4, {"type": 1, "pos1": 0, "pos2": 2}, msn=3)])
    path = tmp_path / "logs.json"
    path.write_text(json.dumps(docs))
    r = subprocess.run([NODE, str(ROOT / "tests" / "node_replay.js"), str(path), mode], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    for msgs, g in zip(docs, got):
        od = O.Doc()
        od.start_collab("readonly")
        for m in msgs:
            if od.apply_msg(json.dumps(m)) != 0:
                break
        assert g["status"] == od.status
        if od.status:
            continue
        assert g["text"] == od.text()
        assert g["runs"] == json.loads(od.props_runs())
        assert g["snapshot"] == od.snapshot_v1()
        assert int(g["digest"]) == od.digest()


@pytest.mark.gpu
def test_node_writer_replica_and_find_tile():
    """The JS Client's local methods (insertTextLocal / insertMarkerLocal / removeRangeLocal) +
    applyMsg acks, and findTile: client.spec.ts:75-151's three-tile document (preceding tile of 5 at
    0, following at 6) and the issue-1213 writer ("Xc"), equal to the oracle's replicas."""
    code = r"""
const { ReplayBatch } = require('./fluidframework_amd/js');
(async () => {
  const b = new ReplayBatch(2);
  const c = b.client(0);
  c.startOrUpdateCollaboration('localUser');
  const m = { referenceTileLabels: ['EOP'], markerId: 'some-id' };
  c.insertMarkerLocal(0, 1, m); c.insertTextLocal(0, 'abc d'); c.insertMarkerLocal(0, 1, m);
  c.insertTextLocal(7, 'ef'); c.insertMarkerLocal(8, 1, m);
  const w = b.client(1);
  w.startOrUpdateCollaboration('1');
  const msg = (op, seq, cid, ref) => ({ clientId: cid, sequenceNumber: seq, referenceSequenceNumber: ref,
                                        minimumSequenceNumber: 0, type: 'op', contents: op });
  const op1 = w.insertTextLocal(0, 'a'), op2 = w.removeRangeLocal(0, 1);
  w.applyMsg(msg(op1, 1, '1', 0)); w.applyMsg(msg(op2, 2, '1', 0));
  const op4 = w.insertTextLocal(0, 'c');
  w.applyMsg(msg({ type: 0, pos1: 0, seg: 'X' }, 3, '2', 0)); w.applyMsg(msg(op4, 4, '1', 2));
  await b.runAsync();
  process.stdout.write(JSON.stringify({
    len: c.getText().length, prec: c.findTile(5, 'EOP'), next: c.findTile(5, 'EOP', false),
    none: c.findTile(5, 'pg') === undefined, wtext: w.getText(), wdigest: w.digest().toString(),
    cdigest: c.digest().toString() }));
})().catch((e) => { console.error(e); process.exit(1); });
"""
    r = _node(code)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    # getText() holds the text segments only; each marker is length 1 in positions
    assert got["len"] == 7 and got["prec"]["pos"] == 0 and got["next"]["pos"] == 6 and got["none"]
    assert got["prec"]["props"] == {"referenceTileLabels": ["EOP"], "markerId": "some-id"}
    assert got["wtext"] == "Xc"
    od = O.Doc()
    od.start_collab("localUser")
    mk = {"marker": {"refType": 1}, "props": {"referenceTileLabels": ["EOP"], "markerId": "some-id"}}
    for pos, seg in ((0, mk), (0, "abc d"), (0, mk), (7, "ef"), (8, mk)):
        od.local_op({"type": 0, "pos1": pos, "seg": seg})
    assert int(got["cdigest"]) == od.digest()


@pytest.mark.gpu
def test_node_consensus_callbacks():
    """Client.annotateMarkerNotifyConsensus through the JS client (client.ts:113-134): the
    callback runs once minSeq reaches the ack's seq, and the marker holds the re-combined value —
    the derived case of tests/test_consensus.py, equal to the oracle."""
    from test_consensus import _kat_registered

    ev, text, props, calls, _ = _kat_registered()
    code = r"""
const { ReplayBatch } = require('./fluidframework_amd/js');
const ev = JSON.parse(process.argv[1]);
(async () => {
  const b = new ReplayBatch(1);
  const w = b.client(0);
  w.startOrUpdateCollaboration('W');
  const seen = [];
  for (const m of ev) {
    if (m.sequenceNumber !== -1) w.applyMsg(m);
    else if (m.notifyConsensus) w.annotateMarkerNotifyConsensus(m.contents.relativePos1.id, m.contents.props, (e) => seen.push(e));
    else w.localOp(m.contents);
  }
  await b.runAsync();
  w.runConsensusCallbacks();
  process.stdout.write(JSON.stringify({ text: w.getText(), seen, props: w.propertyRuns() }));
})().catch((e) => { console.error(e); process.exit(1); });
"""
    r = subprocess.run([NODE, "-e", code, json.dumps(ev)], capture_output=True, text=True, cwd=ROOT, timeout=60)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    assert got["text"] == text and got["seen"] == calls
    assert [json.loads(x[2]) for x in got["props"] if x[2] and "markerId" in x[2]] == [props]


@pytest.mark.gpu
def test_node_ingest_json_on_the_gpu():
    """ReplayBatch.ingestJson parses on the GPU (mt_batch_ingest_json_gpu) and replays exactly like
    the host parser's batch; a batch outside the GPU fast path falls back to the host parser."""
    code = r"""
const { ReplayBatch } = require('./fluidframework_amd/js');
const msg = (c, s, r, op) => ({ clientId: c, sequenceNumber: s, referenceSequenceNumber: r,
                                minimumSequenceNumber: 0, type: 'op', contents: op });
const docs = [[msg('A', 1, 0, { type: 0, pos1: 0, seg: 'hello world' }),
               msg('B', 2, 1, { type: 2, pos1: 0, pos2: 5, props: { bold: true } }),
               msg('A', 3, 2, { type: 1, pos1: 5, pos2: 6 })],
              [msg('C', 1, 0, { type: 0, pos1: 0, seg: { text: 'xyz', props: { k: 'v' } } })]];
const g = new ReplayBatch(2), h = new ReplayBatch(2), f = new ReplayBatch(1);
const pg = g.ingestJson(docs, 0, 'gpu'), ph = h.ingestJson(docs, 0, 'host');
const pf = f.ingestJson([[msg('A', 1, 0, { type: 0, pos1: 0, seg: { text: 'a', props: { '1': 1 } } })]]);  // an array-index key: JS key order, the host parser
g.run(); h.run(); f.run();
const dg = g.deviceDigests(), dh = h.deviceDigests();
// a document count that differs from the batch's is refused by the wrapper and by the C ABI
// (mt_batch_ingest_json_gpu's n_docs), never read past the caller's arrays
const codes = [];
for (const dev of ['gpu', 'host']) {
  try { new ReplayBatch(3).ingestJson(docs, 0, dev); codes.push('ok'); } catch (e) { codes.push(e.code); }
}
const raw = new ReplayBatch(3);
try { require('./fluidframework_amd/js').native().ingestJson(raw.h, docs.map((d) => JSON.stringify(d)), 'readonly', 0, 'gpu');
      codes.push('ok'); } catch (e) { codes.push(e.code); }
process.stdout.write(JSON.stringify({ pg, ph, pf, same: dg[0] === dh[0] && dg[1] === dh[1],
                                      text: g.client(0).getText(), codes }));
"""
    r = _node(code)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    assert got == {"pg": "gpu", "ph": "host", "pf": "host", "same": True, "text": "helloworld",
                   "codes": [101, 101, 101]}
