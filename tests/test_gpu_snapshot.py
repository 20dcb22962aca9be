"""GPU SnapshotV1 (mt_snapshot.hip via mt_batch_snapshots) vs the host serializer and the oracle.

The host serializer (mt_doc_snapshot_v1) is itself pinned to the oracle by test_gpu_parity.py;
here every document's GPU-serialized blobs must be byte-identical to both, across coalescing
(runs, '\\n' ends, the 256-unit granularity rule, property matching), markers, standalone
segments with seq / client / removedSeq / removedClient, chunking (small chunk sizes, more
chunks than the device meta holds), unicode escaping (surrogate pairs split across coalesced
records, lone surrogates, control characters) and capacity escalation across launches.
"""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle_ffi as O
from kat_util import load_kats
from snapdigest import bytes_digest
import fluidframework_amd as fa

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
KATS = load_kats()
GEN_KEYS = [O.lib().mto_gen_key_name(k).decode() for k in range(4)]
GEN_VALUES = [O.lib().mto_gen_value_json(v).decode() for v in range(22)]


def _msg(c, s, r, contents, msn=0):
    return {"clientId": c, "sequenceNumber": s, "referenceSequenceNumber": r, "minimumSequenceNumber": msn,
            "type": "op", "contents": contents}


def _oracle(msgs):
    d = O.Doc()
    d.start_collab("readonly")
    for m in msgs:
        if d.apply_msg(json.dumps(m)) != 0:
            break
    return d


UNICODE_DOCS = [
    # a surrogate pair split across two coalesced records, a lone low surrogate, escapes
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "a\ud83d"}),
     _msg("A", 2, 1, {"type": 0, "pos1": 2, "seg": "\ude00b\"\\\n\x01\x1fé€\t\r\b\f/"}),
     _msg("B", 3, 2, {"type": 0, "pos1": 1, "seg": "\udc00"}, msn=2),
     _msg("B", 4, 3, {"type": 0, "pos1": 0, "seg": "z"}, msn=3)],
    # lone high surrogate at the end of a run, and at the end of the document
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "x\ud800"}),
     _msg("B", 2, 1, {"type": 0, "pos1": 2, "seg": "\ud800"}, msn=1),
     _msg("A", 3, 2, {"type": 0, "pos1": 0, "seg": {"text": "𐏿", "props": {"kéy\"": "v\n"}}}, msn=3)],
    # markers with and without props, text with props that coalesce and that do not
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"marker": {"refType": 2}}}),
     _msg("A", 2, 1, {"type": 0, "pos1": 1, "seg": {"text": "ab", "props": {"2": 1, "b": [1, {"q": None}], "0": "z"}}}),
     _msg("A", 3, 2, {"type": 0, "pos1": 3, "seg": {"text": "cd", "props": {"b": [1, {"q": None}], "0": "z", "2": 1}}}),
     _msg("A", 4, 3, {"type": 0, "pos1": 5, "seg": {"marker": {"refType": 0}, "props": {"id": "m "}}}),
     _msg("A", 5, 4, {"type": 0, "pos1": 6, "seg": {"text": "ef", "props": {"b": 2}}}, msn=5),
     _msg("B", 6, 4, {"type": 1, "pos1": 1, "pos2": 2}, msn=5),
     _msg("B", 7, 6, {"type": 0, "pos1": 0, "seg": "tail"}, msn=5)],
    # '\n' ends a run; granularity rule (both sides > 256 do not coalesce)
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "line\n"}),
     _msg("A", 2, 1, {"type": 0, "pos1": 5, "seg": "next"}),
     _msg("A", 3, 2, {"type": 0, "pos1": 9, "seg": "L" * 300}),
     _msg("A", 4, 3, {"type": 0, "pos1": 309, "seg": "M" * 300}),
     _msg("A", 5, 4, {"type": 0, "pos1": 609, "seg": "s"}, msn=5)],
    [],
]


def _check_batch(b, oracle=None, docs=None):
    info = b.snapshots()
    assert info["bytes"] >= 0 and info["device_ms"] >= 0
    buf, off, meta = b.snapshot_buffer()
    for i in docs if docs is not None else range(b.n_docs):
        dv = b.doc(i)
        gpu = dv.snapshot_v1(device=True)
        host = dv.snapshot_v1()
        assert gpu == host, f"doc {i}: GPU SnapshotV1 differs from the host serializer"
        if oracle is not None and oracle[i] is not None:
            assert gpu == oracle[i].snapshot_v1(), f"doc {i}: GPU SnapshotV1 differs from the oracle"
        n = meta[i, 0]
        assert n == len(host), f"doc {i}: every blob on the GPU"
        # the bulk buffer holds the same blobs back to back; the meta row the first SNAP_MAX_BLOBS
        assert buf[off[i]:off[i + 1]] == "".join(host.values()).encode("utf-8")
        m = min(n, fa.mtreplay.SNAP_MAX_BLOBS)
        sizes = [len(v.encode("utf-8")) for v in host.values()]
        assert list(meta[i, 3:3 + 3 * m:3]) == sizes[:m]


def test_snapshot_kats_unicode_markers():
    docs = [k["messages"] for k in KATS] + UNICODE_DOCS
    oracle = [_oracle(m) for m in docs]
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        for i in range(len(docs)):
            assert b.doc(i).status == oracle[i].status
        _check_batch(b, oracle)


@pytest.mark.parametrize("chunk_size", [1, 7, 64, 10000])
def test_snapshot_chunking(chunk_size):
    docs = UNICODE_DOCS + [k["messages"] for k in KATS]
    with fa.ReplayBatch(len(docs), chunk_size=chunk_size) as b:
        b.ingest_messages(docs)
        b.run()
        _check_batch(b)


def _gen(p, n_docs, **opts):
    ops, text, props, off = O.gen_batch(p, n_docs)
    names = O.gen_client_names(p.n_clients)
    b = fa.ReplayBatch(n_docs, **opts)
    b.set_tables(GEN_KEYS, GEN_VALUES)
    b.set_clients(names)
    b.ingest(ops, off, text, props)
    b.run()
    return b, (ops, text, props, off, names)


def test_snapshot_config2_shape():
    b, _ = _gen(O.gen_params(2000, n_clients=8, max_lag=32, pct_insert=60, pct_remove=40, seed=11), 256)
    with b:
        _check_batch(b)


def test_snapshot_config3_shape_with_oracle():
    b, (ops, text, props, off, names) = _gen(O.gen_params(3000, n_clients=8, max_lag=32, pct_insert=55,
                                                           pct_remove=35, seed=12), 64)
    t = O.gen_tables()
    with b:
        oracle = [None] * 64
        for d in range(0, 64, 8):
            oracle[d] = O.replay_doc(ops[off[d]:off[d + 1]].copy(), text, props, t, names)
        _check_batch(b, oracle)


def test_snapshot_more_blobs_than_the_meta_row():
    # chunk_size 16 on 1500-op documents: hundreds of blobs, beyond MT_SNAP_MAX_BLOBS, stay on the GPU
    b, _ = _gen(O.gen_params(1500, n_clients=4, max_lag=8, pct_insert=70, pct_remove=20, seed=13), 32, chunk_size=16)
    with b:
        _check_batch(b)
        _, meta = b.snapshot_index()
        assert (meta[:, 0] > fa.mtreplay.SNAP_MAX_BLOBS).all()


def test_snapshot_after_capacity_escalation():
    b, _ = _gen(O.gen_params(4000, n_clients=8, max_lag=32, pct_insert=70, pct_remove=20, seed=14), 48, seg_cap=64)
    with b:
        assert b.stats()["launches"] > 1
        _check_batch(b)


def test_snapshot_digests_cover_all_blobs():
    b, _ = _gen(O.gen_params(1500, n_clients=8, max_lag=32, pct_insert=55, pct_remove=35, seed=15), 96)
    with b:
        b.snapshots()
        dig = b.snapshot_digests()
        for i in range(b.n_docs):
            blobs = b.doc(i).snapshot_v1()
            assert int(dig[i]) == bytes_digest("".join(blobs.values()).encode("utf-8")), i
        assert len(set(dig.tolist())) == b.n_docs
