"""BASELINE configs[0]: one SharedString, 4 clients, 10k insert/remove ops, on the CPU (no GPU).

The generated log is turned back into ISequencedDocumentMessage JSON and replayed three ways:
the oracle's applyMsg(JSON) path (the reference's entry point), the Python packer + packed
replay, and the Node packer (fluidframework_amd/js/index.js) + packed replay.  All three must
agree on text, property runs, SnapshotV1 and the state digest, and the two packers must emit
byte-identical records."""
import json
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_ffi as O
from fluidframework_amd import oplog

ROOT = Path(__file__).resolve().parents[1]
NAMES = O.gen_client_names(4)


def _messages(ops, text, props):
    keys = [O.lib().mto_gen_key_name(k).decode() for k in range(4)]
    vals = [json.loads(O.lib().mto_gen_value_json(v).decode()) for v in range(22)]
    out = []
    for o in ops:
        t = int(o["tc"]) & 0xF
        if t == 0:
            s = text[o["payload"]:o["payload"] + o["payload_len"]]
            c = {"type": 0, "pos1": int(o["pos1"]), "seg": s.tobytes().decode("utf-16-le")}
        elif t == 1:
            c = {"type": 1, "pos1": int(o["pos1"]), "pos2": int(o["pos2"])}
        else:
            pr = props[o["payload"]:o["payload"] + o["payload_len"]]
            c = {"type": 2, "pos1": int(o["pos1"]), "pos2": int(o["pos2"]),
                 "props": {keys[int(p["key"])]: vals[int(p["value"])] for p in pr}}
        out.append({"clientId": NAMES[int(o["tc"]) >> 4], "sequenceNumber": int(o["seq"]),
                    "referenceSequenceNumber": int(o["ref_seq"]), "minimumSequenceNumber": int(o["msn"]),
                    "type": "op", "contents": c})
    return out


@pytest.fixture(scope="module")
def farm():
    p = O.gen_params(10000, n_clients=4, max_lag=8, pct_insert=60, pct_remove=40, seed=0x1F00D)
    ops, text, props = O.gen_doc(p, 0)
    msgs = _messages(ops, text, props)
    ref = O.Doc()
    ref.start_collab("readonly")
    for m in msgs:
        assert ref.apply_msg(json.dumps(m)) == 0, ref.error
    return msgs, ref


def _replay_packed(pb):
    t = O.Tables(pb.keys or ["_"], pb.values)
    d = O.replay_doc(pb.ops.copy(), pb.text, pb.props, t, pb.clients[0])
    d._t = t
    return d


def test_config1_python_packer_matches_applymsg(farm):
    msgs, ref = farm
    got = _replay_packed(oplog.pack_documents([msgs]))
    assert got.status == 0, got.error
    assert got.text() == ref.text() and len(ref.text()) > 1000
    assert got.props_runs() == ref.props_runs()
    assert got.snapshot_v1() == ref.snapshot_v1()
    assert got.digest() == ref.digest()


NODE = shutil.which("node")


@pytest.mark.skipif(NODE is None, reason="node not available")
def test_config1_node_packer_is_byte_identical(farm, tmp_path):
    msgs, ref = farm
    src = tmp_path / "msgs.json"
    src.write_text(json.dumps([msgs]))
    code = ("const {Packer}=require('./fluidframework_amd/js');const fs=require('fs');"
            f"const docs=JSON.parse(fs.readFileSync({json.dumps(str(src))},'utf8'));const p=new Packer();"
            "for(const d of docs)p.addDocument(d);const r=p.finish();"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'ops.bin'))},r.ops);"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'text.bin'))},Buffer.from(r.text.buffer,0,2*r.nText));"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'meta.json'))},JSON.stringify({{keys:r.keys,values:r.values,clients:r.clients,off:Array.from(r.docOpOff,Number)}}));")
    r = subprocess.run([NODE, "-e", code], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    pb = oplog.pack_documents([msgs])
    ops = np.frombuffer((tmp_path / "ops.bin").read_bytes(), oplog.OP_DTYPE)
    meta = json.loads((tmp_path / "meta.json").read_text())
    assert ops.tobytes() == pb.ops.tobytes()
    assert np.frombuffer((tmp_path / "text.bin").read_bytes(), np.uint16).tobytes() == pb.text.tobytes()
    assert meta["keys"] == pb.keys and meta["values"] == pb.values and meta["clients"] == pb.clients
    assert meta["off"] == pb.doc_op_off.tolist()
    node = _replay_packed(pb)
    assert node.digest() == ref.digest()


@pytest.mark.skipif(NODE is None, reason="node not available")
def test_node_packer_combining_ops_byte_identical(tmp_path):
    """The Node packer's combiningOp and MT_OP_RELPOS records equal the Python packer's (include/mt_oplog.h)."""
    from combine_logs import COMBINE_DOCS, RELPOS_DOCS, combine_farm, relpos_farm

    docs = COMBINE_DOCS + [combine_farm(300, seed=3)] + RELPOS_DOCS + [relpos_farm(150, seed=3)]
    src = tmp_path / "msgs.json"
    src.write_text(json.dumps(docs))
    code = ("const {Packer}=require('./fluidframework_amd/js');const fs=require('fs');"
            f"const docs=JSON.parse(fs.readFileSync({json.dumps(str(src))},'utf8'));const p=new Packer();"
            "for(const d of docs)p.addDocument(d);const r=p.finish();"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'ops.bin'))},r.ops);"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'props.bin'))},Buffer.from(r.props.buffer));"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'meta.json'))},JSON.stringify({{values:r.values}}));")
    r = subprocess.run([NODE, "-e", code], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    pb = oplog.pack_documents(docs)
    assert np.frombuffer((tmp_path / "ops.bin").read_bytes(), oplog.OP_DTYPE).tobytes() == pb.ops.tobytes()
    assert np.frombuffer((tmp_path / "props.bin").read_bytes(), oplog.PROP_DTYPE).tobytes() == pb.props.tobytes()
    assert json.loads((tmp_path / "meta.json").read_text())["values"] == pb.values



@pytest.mark.skipif(NODE is None, reason="node not available")
def test_node_packer_large_prop_sets_byte_identical(tmp_path):
    """Inserts past 126 props (the extended count record, include/mt_oplog.h MT_OPF_NPROPS_EXT) and
    annotates past 64 keys: the Node packer == the Python packer."""
    from combine_logs import big_prop_docs

    docs = big_prop_docs()
    src = tmp_path / "msgs.json"
    src.write_text(json.dumps(docs))
    code = ("const {Packer}=require('./fluidframework_amd/js');const fs=require('fs');"
            f"const docs=JSON.parse(fs.readFileSync({json.dumps(str(src))},'utf8'));const p=new Packer();"
            "for(const d of docs)p.addDocument(d);const r=p.finish();"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'ops.bin'))},r.ops);"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'props.bin'))},Buffer.from(r.props.buffer));")
    r = subprocess.run([NODE, "-e", code], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    pb = oplog.pack_documents(docs)
    assert np.frombuffer((tmp_path / "ops.bin").read_bytes(), oplog.OP_DTYPE).tobytes() == pb.ops.tobytes()
    assert np.frombuffer((tmp_path / "props.bin").read_bytes(), oplog.PROP_DTYPE).tobytes() == pb.props.tobytes()


@pytest.mark.skipif(NODE is None, reason="node not available")
def test_node_packer_writer_streams_byte_identical(tmp_path):
    """Writer replicas' streams (local ops, acks): the Node packer == the Python packer."""
    from writer_sim import farm as writer_farm

    f = writer_farm(4, 400, 8, rewrite=20, markers=10)
    docs = [[n, f.events[n]] for n in f.names]
    src = tmp_path / "msgs.json"
    src.write_text(json.dumps(docs))
    code = ("const {Packer}=require('./fluidframework_amd/js');const fs=require('fs');"
            f"const docs=JSON.parse(fs.readFileSync({json.dumps(str(src))},'utf8'));const p=new Packer();"
            "for(const [n,d] of docs)p.addDocument(d,n);const r=p.finish();"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'ops.bin'))},r.ops);"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'props.bin'))},Buffer.from(r.props.buffer));"
            f"fs.writeFileSync({json.dumps(str(tmp_path / 'meta.json'))},JSON.stringify({{values:r.values,clients:r.clients}}));")
    r = subprocess.run([NODE, "-e", code], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    p = oplog.Packer()
    for n, d in docs:
        p.add_document(d, n)
    pb = p.finish()
    assert np.frombuffer((tmp_path / "ops.bin").read_bytes(), oplog.OP_DTYPE).tobytes() == pb.ops.tobytes()
    assert np.frombuffer((tmp_path / "props.bin").read_bytes(), oplog.PROP_DTYPE).tobytes() == pb.props.tobytes()
    meta = json.loads((tmp_path / "meta.json").read_text())
    assert meta["values"] == pb.values and meta["clients"] == pb.clients
