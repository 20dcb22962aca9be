"""GPU parity: the HIP replay (through the C ABI) vs the oracle on the same inputs.

Bit-exact on everything the path produces: final text, property runs, SnapshotV1 blobs
and the state digest (full segment table incl. tombstones, leaf-block membership, tree
depth, collab window).  Sizes are chosen so the oracle finishes in seconds.
"""
import dataclasses
import json
from pathlib import Path

import numpy as np
import pytest

import oracle_ffi as O
from kat_util import load_kats
import fluidframework_amd as fa
from fluidframework_amd import oplog
from combine_logs import COMBINE_DOCS, RELPOS_DOCS, combine_farm, relpos_farm

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]
KATS = load_kats()
GIANT, HBM = 2000000, 2097152  # mt_device.h kGiantSeg, kHbmSeg
GEN_KEYS = [O.lib().mto_gen_key_name(k).decode() for k in range(4)]
GEN_VALUES = [O.lib().mto_gen_value_json(v).decode() for v in range(22)]


def oracle_docs_from_messages(docs):
    out = []
    for msgs in docs:
        d = O.Doc()
        d.start_collab("readonly")
        for m in msgs:
            if d.apply_msg(json.dumps(m)) != 0:
                break
        out.append(d)
    return out


def assert_doc_parity(dv, od, full=True):
    assert dv.status == od.status, (fa.status_string(dv.status), od.error)
    if od.status != 0:
        return
    assert dv.digest() == od.digest(), f"state digest differs\nGPU shape {dv.shape()}\nCPU shape {od.shape()}"
    if full:
        assert dv.shape() == od.shape()
        assert dv.get_text() == od.text()
        assert dv.props_runs() == json.loads(od.props_runs())
        assert dv.snapshot_v1() == od.snapshot_v1()


def test_kats_on_gpu():
    docs = [k["messages"] for k in KATS]
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        for i, k in enumerate(KATS):
            dv = b.doc(i)
            assert dv.get_text() == k["text"], k["name"]
            if "props_runs" in k:
                assert dv.props_runs() == k["props_runs"], k["name"]
            assert_doc_parity(dv, oracle[i])


def _gen_batch_parity(p, n_docs, full_every=8, **opts):
    ops, text, props, off = O.gen_batch(p, n_docs)
    t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
    _, dig, st = O.replay_batch(ops, off, text, props, t, names)
    with fa.ReplayBatch(n_docs, **opts) as b:
        b.set_tables(GEN_KEYS, GEN_VALUES)
        b.set_clients(names)
        b.ingest(ops, off, text, props)
        b.run()
        stats = b.stats()
        assert stats["docs_failed"] == int((st != 0).sum())
        for d in range(n_docs):
            dv = b.doc(d)
            assert dv.status == st[d]
            assert dv.digest() == int(dig[d]), f"doc {d} digest differs"
            if d % full_every == 0:
                a, e = off[d], off[d + 1]
                od = O.replay_doc(ops[a:e].copy(), text, props, t, names)
                assert_doc_parity(dv, od)
        return stats


def test_text_only_config2_shape():
    """BASELINE configs[1] shape (8 clients, refSeq lag <= 32, insert 60 / remove 40), 2k ops."""
    _gen_batch_parity(O.gen_params(2000, seed=0xC0FFEE), 48)


def test_annotate_and_zamboni_config3_shape():
    """BASELINE configs[2] op mix (insert 55 / remove 35 / annotate 10) at 1.5k ops."""
    _gen_batch_parity(O.gen_params(1500, pct_insert=55, pct_remove=35, seed=0xBADC0DE), 32)


def test_high_concurrency_tie_breaks():
    """Wide collab windows stress breakTie / overlapping removes / pack."""
    _gen_batch_parity(O.gen_params(1200, n_clients=24, max_lag=200, pct_insert=50, pct_remove=40,
                                   min_len=0, max_insert=3, seed=77), 32)


def test_small_capacity_escalation():
    """Force the smallest LDS class so documents overflow and are re-run in larger classes."""
    stats = _gen_batch_parity(O.gen_params(800, seed=3), 16, full_every=4, seg_cap=64, max_retries=6)
    assert stats["launches"] >= 2


def test_gpu_generator_matches_oracle_generator():
    p = O.gen_params(700, pct_insert=55, pct_remove=35, seed=12345)
    n = 12
    with fa.ReplayBatch(n) as b:
        b.generate(fa.gen_params(700, pct_insert=55, pct_remove=35, seed=12345))
        ops, off, text, props = b.download_log()
        b.run()
        for d in range(n):
            o_ops, o_text, o_props = O.gen_doc(p, d)
            g_ops = ops[off[d]:off[d + 1]]
            for f in ("tc", "seq", "ref_seq", "msn", "pos1", "pos2", "payload_len"):
                assert (g_ops[f] == o_ops[f]).all(), (d, f)
            ins = (g_ops["tc"] & 0xF) == 0
            g_txt = np.concatenate([text[o["payload"]:o["payload"] + o["payload_len"]] for o in g_ops[ins]])
            assert (g_txt == o_text).all()
            od = O.replay_doc(o_ops, o_text, o_props, O.gen_tables(), O.gen_client_names(8))
            assert b.doc(d).digest() == od.digest()


def _msg(c, s, r, contents, msn=0):
    return {"clientId": c, "sequenceNumber": s, "referenceSequenceNumber": r, "minimumSequenceNumber": msn,
            "type": "op", "contents": contents}


def test_markers_props_groups_rewrite():
    docs = [
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "hello", "props": {"b": 1, "3": "x"}}}),
         _msg("B", 2, 0, {"type": 0, "pos1": 0, "seg": {"marker": {"refType": 1}, "props": {"id": "m1"}}}),
         _msg("A", 3, 1, {"type": 3, "ops": [{"type": 0, "pos1": 2, "seg": "XY"},
                                             {"type": 2, "pos1": 0, "pos2": 4, "props": {"c": True}}]}),
         _msg("B", 4, 3, {"type": 2, "pos1": 1, "pos2": 6, "props": {"c": None, "b": 2},
                          "combiningOp": {"name": "rewrite"}}, msn=1),
         _msg("A", 5, 4, {"type": 0, "pos1": 3, "seg": {"text": "e", "props": {}}}, msn=3),
         _msg("B", 6, 5, {"type": 1, "pos1": 0, "pos2": 2}, msn=5)],
        # removes racing an insert at the same position (issue #1213 family)
        [_msg("1", 1, 0, {"type": 0, "pos1": 0, "seg": "abc"}),
         _msg("2", 2, 0, {"type": 0, "pos1": 0, "seg": "XYZ"}),
         _msg("1", 3, 1, {"type": 1, "pos1": 1, "pos2": 3}),
         _msg("3", 4, 1, {"type": 1, "pos1": 0, "pos2": 3}),
         _msg("2", 5, 2, {"type": 0, "pos1": 3, "seg": "q"}),
         _msg("3", 6, 4, {"type": 0, "pos1": 0, "seg": "r"}, msn=1)],
        # a no-op message advances the MSN (zamboni on setMinSeq)
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "aaaa"}),
         _msg("A", 2, 1, {"type": 0, "pos1": 4, "seg": "bbbb"}),
         {"clientId": "A", "sequenceNumber": 3, "referenceSequenceNumber": 2, "minimumSequenceNumber": 2,
          "type": "noop", "contents": None}],
    ]
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        for i in range(len(docs)):
            assert_doc_parity(b.doc(i), oracle[i])


def test_error_statuses_match_oracle():
    docs = [
        [_msg("A", 1, 0, {"type": 0, "pos1": 3, "seg": "x"})],  # insert beyond the end
        [_msg("A", 2, 0, {"type": 0, "pos1": 0, "seg": "x"}), _msg("A", 2, 0, {"type": 0, "pos1": 0, "seg": "y"})],
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "x"}), _msg("A", 2, 1, {"type": 0, "pos1": 0, "seg": "y"}, 1),
         _msg("A", 3, 2, {"type": 0, "pos1": 0, "seg": "z"}, 0)],
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "fine"})],
    ]
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        got = [b.doc(i).status for i in range(len(docs))]
        assert got == [od.status for od in oracle] == [fa.MT_INVALID_POS, fa.MT_SEQ_ORDER, fa.MT_MSN_ORDER, 0]
        assert b.doc(3).get_text() == "fine"


def _many_client_farm(n_clients, n_ops, seed, lag=24, hot=12, active=0):
    """A valid conflict-farm log of n_clients writers, generated against the oracle as the replica
    model (each op is drawn from its issuer's view getLength(refSeq, client), then applied):
    removes and annotates favour the first `hot` positions, so concurrent removes of the same
    segments by many clients (removedClientOverlap with clients beyond the 31st) are common.
    active > 0: sessions — at most `active` clients are connected at once, each leaves after a few
    ops and a new client id joins in its place (a reconnect is a new clientId in a real
    messages.json), the MSN is the minimum over the connected ones; n_clients ids in all."""
    import random

    rnd = random.Random(seed)
    names = [f"client-{i:04d}" for i in range(n_clients)]
    model = O.Doc()
    model.start_collab("readonly")
    short, last_ref, msgs = {}, {}, []
    live, joined, floor = [], 0, 0
    for k in range(1, n_ops + 1):
        if active:
            while len(live) < active and joined < n_clients:
                live.append(names[joined])
                last_ref[names[joined]] = max(floor, k - 1)
                joined += 1
            c = live[rnd.randrange(len(live))]
        else:
            c = names[rnd.randrange(n_clients)] if k > 1 else names[0]
        ref = max(last_ref.get(c, 0), k - 1 - rnd.randrange(lag + 1))
        last_ref[c] = ref
        msn = max(floor, min(last_ref[x] for x in live)) if active else min(last_ref.values())
        floor = msn
        sid = short.get(c, len(short) + 1)
        n = model.view_length(ref, sid)
        u = rnd.randrange(100)
        if n < 4 or u < 45:
            pos = rnd.randrange(n + 1)
            contents = {"type": 0, "pos1": pos, "seg": "".join(rnd.choice("abcdefgh\n") for _ in range(rnd.randint(1, 6)))}
        else:
            a = rnd.randrange(min(n, hot)) if rnd.random() < 0.7 else rnd.randrange(n)
            b = min(n, a + 1 + rnd.randrange(4))
            if u < 85:
                contents = {"type": 1, "pos1": a, "pos2": b}
            else:
                contents = {"type": 2, "pos1": a, "pos2": b, "props": {"k": rnd.randrange(3)}}
        m = _msg(c, k, ref, contents, msn)
        assert model.apply_msg(json.dumps(m)) == 0, model.error()
        short.setdefault(c, len(short) + 1)
        msgs.append(m)
        if active and rnd.random() < 0.15 and joined < n_clients:  # the client leaves: a new id joins
            live.remove(c)
            del last_ref[c]
    return msgs


def test_many_clients_with_overlapping_removes():
    """Short client ids are 15-bit (up to 32,765 writers per document; client.ts:636-660 assigns them
    in first-appearance order and a long-lived document's log names a new clientId on every
    reconnect; the op record keeps the id's high bits in flags 11-13, mt_oplog.h): 5,000 and 1,000
    session ids over a 16-client window with overlapping removes, and 300 writers with concurrent
    overlapping removes (overlap sets beyond 31 clients are pool lists, mergeTree.ts:2544-2563)
    replay bit-exact, also through checkpoint / resume; more than 32,765 are flagged, not wrong."""
    docs = [_many_client_farm(1000, 7000, seed=13, active=16, hot=8),
            _many_client_farm(300, 2500, seed=11), _many_client_farm(200, 1500, seed=12, lag=60, hot=6),
            _many_client_farm(5000, 36000, seed=14, active=16, hot=8)]
    assert len({m["clientId"] for m in docs[0]}) == 1000
    assert len({m["clientId"] for m in docs[3]}) == 5000
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        for i in range(len(docs)):
            assert_doc_parity(b.doc(i), oracle[i])
        b.snapshots()
        for i in range(len(docs)):
            assert b.doc(i).snapshot_v1(device=True) == oracle[i].snapshot_v1()
        d0 = b.device_digests()
    with fa.ReplayBatch(len(docs), seg_cap=64) as b:  # through checkpoint / resume: same digests
        b.ingest_messages(docs)
        b.run()
        assert (b.device_digests() == d0).all()
    js = [json.dumps(d) for d in docs]
    with fa.ReplayBatch(len(docs)) as b:  # the native JSON parsers (host threads, and the GPU's)
        assert b.ingest_json(js, device="host")["path"] == "host"
        b.run()
        assert (b.device_digests() == d0).all()
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_json(js, device="gpu")
        b.run()
        assert (b.device_digests() == d0).all()
    msgs = [_msg(f"c{i}", i + 1, i, {"type": 0, "pos1": 0, "seg": "x"}) for i in range(32770)]
    with fa.ReplayBatch(1) as b:
        with pytest.raises(oplog.UnsupportedOp):
            b.ingest_messages([msgs])


def test_collab_window_beyond_16_bit_seqs():
    """The LDS classes keep the overlay entries' sequence numbers relative to minSeq in 16 bits
    (DESIGN §2): a document whose collab window (currentSeq - minSeq, held open by a client that never
    advances its refSeq) reaches 65,520 ops re-runs from scratch in the giant class, whose relative
    seqs are 32-bit (MergeTree keeps JS numbers, mergeTree.ts:1718-1736: no window limit), and from
    there in the HBM class when its overlay list outgrows the giant class's LDS.  Windows below and
    far beyond the 16-bit limit, with concurrent inserts spread through them, replay bit-exact."""
    def doc(n_noops, every=0):
        msgs = [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abc"})]
        for k in range(2, 2 + n_noops):
            if every and k % every == 0:  # C keeps up and inserts; B holds minSeq at 0
                msgs.append(_msg("C", k, k - 1, {"type": 0, "pos1": 0, "seg": "q" + str(k % 7)}))
            else:
                msgs.append({"clientId": "B", "sequenceNumber": k, "referenceSequenceNumber": 1,
                             "minimumSequenceNumber": 0, "type": "noop", "contents": None})
        msgs.append(_msg("B", 2 + n_noops, 1, {"type": 0, "pos1": 1, "seg": "X"}))
        msgs.append(_msg("A", 3 + n_noops, 1, {"type": 1, "pos1": 0, "pos2": 2}))
        return msgs
    docs = [doc(65400), doc(65600), doc(65600, every=997), doc(140000, every=131)]
    oracle = oracle_docs_from_messages(docs)
    assert all(o.status == 0 for o in oracle)
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        for d in range(len(docs)):
            assert_doc_parity(b.doc(d), oracle[d])
        classes = {li["seg_class"] for li in b.launches()}
        assert max(classes) >= 2000000, classes  # the wide windows ran in a spill class


def test_empty_documents_and_empty_inserts():
    docs = [[], [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": ""}), _msg("A", 2, 1, {"type": 0, "pos1": 0, "seg": "k"})]]
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(2) as b:
        b.ingest_messages(docs)
        b.run()
        assert b.doc(0).get_text() == "" and b.doc(0).snapshot_v1() == oracle[0].snapshot_v1()
        assert_doc_parity(b.doc(1), oracle[1])


def test_device_digests_are_placement_independent():
    """The 8-byte device digest (gathered to rank 0 by bench.py) depends only on a document's
    log: the same global document replayed in another batch, shard or capacity class (with
    checkpoint/resume) gets the same digest; different documents get different ones."""
    p = fa.gen_params(600, pct_insert=55, pct_remove=35, seed=99)
    with fa.ReplayBatch(12) as a:
        a.generate(p, 0)
        a.run()
        da = a.device_digests()
    with fa.ReplayBatch(6) as b:
        b.generate(p, 6)
        b.run()
        db = b.device_digests()
    with fa.ReplayBatch(12, seg_cap=64, max_retries=8) as c:
        c.generate(p, 0)
        c.run()
        assert c.stats()["launches"] >= 2
        dc = c.device_digests()
    assert (da[6:] == db).all()
    assert (da == dc).all()
    assert len(set(da.tolist())) == 12


def test_hbm_class_spills_documents_beyond_lds():
    """A document that outgrows the largest LDS class (4,096 slots) is checkpointed and resumed
    in the HBM class (tables in global memory, same engine code) and stays bit-exact."""
    p = O.gen_params(12000, pct_insert=50, pct_remove=15, seed=2024)  # 35% annotate: props keep segments apart
    n = 1
    ops, text, props, off = O.gen_batch(p, n)
    t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
    _, dig, st = O.replay_batch(ops, off, text, props, t, names)
    with fa.ReplayBatch(n) as b:
        b.set_tables(GEN_KEYS, GEN_VALUES)
        b.set_clients(names)
        b.ingest(ops, off, text, props)
        b.run()
        c = b.counters()
        assert (c["max_slots"] > 4096).any(), c["max_slots"]
        for d in range(n):
            assert b.doc(d).status == st[d] == 0, {k: int(c[k][d]) for k in c.dtype.names}
            assert b.doc(d).digest() == int(dig[d])
        od = O.replay_doc(ops[off[0]:off[1]].copy(), text, props, t, names)
        assert b.doc(0).snapshot_v1() == od.snapshot_v1()


def test_mixed_size_batch_generate_docs_and_concurrent_classes():
    """Config 4 machinery on a small scale: per-document sizes and global ids
    (mt_batch_generate_docs == the oracle generator), first launches grouped by capacity class
    and run concurrently (largest documents first), LPT order, parity of every document."""
    from fluidframework_amd import shard

    sizes = shard.zipf_sizes(64, 200, 12000, 1.1)
    parts, _ = shard.lpt(sizes, 2)
    ids = parts[1]  # rank 1's documents, in decreasing size
    ops_n = sizes[ids]
    p = O.gen_params(0, pct_insert=70, pct_remove=20, seed=0x21BF)
    ops, text, props, off = O.gen_batch(p, len(ids), doc_ids=ids, doc_ops=ops_n)
    t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
    _, dig, st = O.replay_batch(ops, off, text, props, t, names)
    with fa.ReplayBatch(len(ids)) as b:
        b.generate_docs(fa.gen_params(0, pct_insert=70, pct_remove=20, seed=0x21BF), ids, ops_n)
        gops, goff, gtext, gprops = b.download_log()
        assert (goff == off).all()
        for f in ("tc", "seq", "ref_seq", "msn", "pos1", "pos2", "payload_len"):
            assert (gops[f] == ops[f]).all(), f
        ins = (gops["tc"] & 0xF) == 0
        g_txt = np.concatenate([gtext[o["payload"]:o["payload"] + o["payload_len"]] for o in gops[ins]])
        o_txt = np.concatenate([text[o["payload"]:o["payload"] + o["payload_len"]] for o in ops[ins]])
        assert (g_txt == o_txt).all()
        b.run()
        launches = b.launches()
        assert len({li["seg_class"] for li in launches}) >= 3
        for d in range(len(ids)):
            assert b.doc(d).status == st[d]
            assert b.doc(d).digest() == int(dig[d]), f"doc {d} ({ops_n[d]} ops) digest differs"
        b.snapshots()
        for d in range(0, len(ids), 5):
            assert b.doc(d).snapshot_v1(device=True) == b.doc(d).snapshot_v1()


def test_native_json_ingest_replays_like_the_packer():
    """mt_pack_json + mt_batch_ingest_packed (host threads) replays every document exactly like
    the Python packer's ingest; both equal the oracle's applyMsg(JSON) replay."""
    import sys as _sys
    _sys.path.insert(0, str(ROOT / "tests"))
    from test_json_ingest import EDGE_DOCS, _farm_messages

    # the oracle's JSON entry point takes string client ids only: the system message gets one
    edge = [[dict(m, clientId=m["clientId"] or "A") for m in d] for d in EDGE_DOCS[:2]]
    docs = [k["messages"] for k in KATS] + edge + [_farm_messages()]
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(len(docs)) as a, fa.ReplayBatch(len(docs)) as b:
        a.ingest_messages(docs)
        b.ingest_json([json.dumps(d) for d in docs], n_threads=4)
        a.run()
        b.run()
        for i in range(len(docs)):
            assert b.doc(i).status == a.doc(i).status == oracle[i].status
            assert b.doc(i).digest() == a.doc(i).digest()
            assert_doc_parity(b.doc(i), oracle[i])


def test_config3_documents_at_full_size():
    """The north-star workload's documents at their own size: config-3 mix (55/35/10), 10k ops,
    no seg_cap forcing, so documents run the natural capacity chain (class 464 -> 563 -> ... ->
    1,679 -> 2,046) through checkpoint / resume.  Every digest equals the oracle's; every 8th
    document also text, property runs and SnapshotV1 (host and GPU serializers)."""
    n = 32
    p = O.gen_params(10000, pct_insert=55, pct_remove=35, seed=0xDEADBEEF)
    ops, text, props, off = O.gen_batch(p, n)
    t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
    _, dig, st = O.replay_batch(ops, off, text, props, t, names)
    with fa.ReplayBatch(n) as b:
        b.set_tables(GEN_KEYS, GEN_VALUES)
        b.set_clients(names)
        b.ingest(ops, off, text, props)
        b.run()
        launches = b.launches()
        assert len({li["seg_class"] for li in launches}) >= 3, launches  # the escalation chain ran
        assert int(b.counters()["max_slots"].max()) > 1376
        for d in range(n):
            assert b.doc(d).status == st[d] == 0
            assert b.doc(d).digest() == int(dig[d]), f"doc {d} digest differs"
        b.snapshots()
        for d in range(0, n, 8):
            od = O.replay_doc(ops[off[d]:off[d + 1]].copy(), text, props, t, names)
            assert_doc_parity(b.doc(d), od)
            assert b.doc(d).snapshot_v1(device=True) == od.snapshot_v1()


def _settle(msgs, seq):
    """a no-op message moving the MSN to `seq` (zamboni scours the settled segments)"""
    return msgs + [{"clientId": "A", "sequenceNumber": seq + 1, "referenceSequenceNumber": seq,
                    "minimumSequenceNumber": seq, "type": "noop", "contents": None}]


def _props_run(values, key="k"):
    """adjacent inserts carrying {key: value} for each value, then the MSN passes them all"""
    msgs, pos = [], 0
    for i, v in enumerate(values):
        msgs.append(_msg("A", i + 1, i, {"type": 0, "pos1": pos, "seg": {"text": "ab", "props": {key: v}}}))
        pos += 2
    return _settle(msgs, len(values))


NESTED_PROPS_DOCS = [
    _props_run([{"x": 1, "y": 2}, {"y": 2, "x": 1}]),              # nested key order: match
    _props_run([[1, 2], {"0": 1, "1": 2}]),                        # array == index-keyed object
    _props_run([5, {}]),                                           # for-in over a number: no keys
    _props_run([{}, 5]),                                           # ... but not the other way round
    _props_run([{"a": 0}, {"a": None}]),                           # falsy vs nested null: match
    _props_run([{"a": None}, {"a": 0}]),                           # ... not reversed
    _props_run(["ab", ["a", "b"]]),                                # for-in over a string: its indices
    _props_run([5, {}, 5]),                                        # intransitive: the chain head decides
    _props_run([{"p": [1, {"q": "r"}]}, {"p": {"1": {"q": "r"}, "0": 1}}, {"p": [1, {"q": "s"}]}]),
    _props_run([{"x": 1}, {"x": 1, "y": 2}]),                      # different key sets
    _props_run([0, False]),                                        # strict equality of primitives
]


def test_nested_property_values_match_structurally():
    """matchProperties (properties.ts:62-93) decides zamboni merges and SnapshotV1 coalescing: nested
    values compare structurally and key-order-free, arrays equal index-keyed objects, and the
    asymmetric / intransitive cases follow the reference's loop order.  GPU == oracle on the
    segment table, text, property runs and SnapshotV1 (host and GPU serializers)."""
    docs = NESTED_PROPS_DOCS
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        b.snapshots()
        for i in range(len(docs)):
            assert b.doc(i).status == 0, i
            assert_doc_parity(b.doc(i), oracle[i])
            assert b.doc(i).snapshot_v1(device=True) == oracle[i].snapshot_v1(), i
        merged = [json.loads(b.doc(i).snapshot_v1()["header"])["segmentCount"] for i in range(len(docs))]
        # the reference's answers (one coalesced segment where matchProperties holds along the chain)
        assert merged == [1, 1, 1, 2, 1, 2, 1, 1, 2, 2, 2], merged


def test_terminal_capacity_digests_are_defined():
    """A document that stops for good with MT_CAPACITY (no larger class allowed) still gets a
    device digest from its final launch: deterministic across runs and batches."""
    p = fa.gen_params(3000, pct_insert=55, pct_remove=35, seed=4242)
    got = []
    for _ in range(2):
        with fa.ReplayBatch(8, seg_cap=64, max_retries=-1) as b:
            b.generate(p, 0)
            b.run()
            st = b.statuses()
            assert (st == fa.MT_CAPACITY).any(), st
            got.append(b.device_digests())
            assert (b.device_digests() == got[-1]).all()
    assert (got[0] == got[1]).all()
    assert len(set(got[0].tolist())) == 8


def test_segments_beyond_16_bit_lengths_move_to_the_giant_class():
    """LDS classes keep segment lengths in 16 bits; a longer segment (one large insert, or zamboni
    appending short inserts to a 65,530-unit run) re-runs the document from scratch in the giant
    class with 32-bit lengths, bit-exact with the oracle."""
    big = "x" * 70000
    near = "y" * 65530
    docs = [
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": big}), _msg("B", 2, 1, {"type": 1, "pos1": 10, "pos2": 20}, 1)],
        _settle([_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": near})] +
                [_msg("B", k, k - 1, {"type": 0, "pos1": 65530 + 2 * (k - 2), "seg": "ab"}) for k in range(2, 12)], 11),
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "short"})],
    ]
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        classes = {li["seg_class"] for li in b.launches()}
        assert GIANT in classes, b.launches()
        for i in range(len(docs)):
            assert_doc_parity(b.doc(i), oracle[i])
        assert len(json.loads(b.doc(1).snapshot_v1()["header"])["segments"]) == 1  # merged past 65,535


def test_one_launch_escalating_into_several_classes():
    """One first launch whose documents escalate into different classes at once — checkpoints into
    the next LDS class, a long segment into the giant class, a large property set into the bigprops
    kernel — so the host submits several launches while scheduling that launch's escalations
    (mt_host.cpp mt_batch_sync: every target group gets its own launch); all equal the oracle."""
    from combine_logs import big_prop_docs

    p = O.gen_params(900, pct_insert=55, pct_remove=35, seed=0xE5C)
    docs = [[_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "x" * 70000})],
            big_prop_docs()[0]]
    # generated logs as messages (growing documents that checkpoint out of the small first class)
    keys = [O.lib().mto_gen_key_name(k).decode() for k in range(4)]
    vals = [json.loads(O.lib().mto_gen_value_json(v).decode()) for v in range(22)]
    names = O.gen_client_names(p.n_clients)
    for d in range(6):
        o_ops, o_text, o_props = O.gen_doc(p, d)
        msgs = []
        for o in o_ops:
            t = int(o["tc"]) & 0xF
            c = {"type": t, "pos1": int(o["pos1"])}
            if t == 0:
                c["seg"] = "".join(chr(x) for x in o_text[int(o["payload"]):int(o["payload"]) + int(o["payload_len"])])
            else:
                c["pos2"] = int(o["pos2"])
            if t == 2:
                c["props"] = {keys[int(q["key"])]: vals[int(q["value"])]
                              for q in o_props[int(o["payload"]):int(o["payload"]) + int(o["payload_len"])]}
            msgs.append(_msg(names[int(o["tc"]) >> 4], int(o["seq"]), int(o["ref_seq"]), c, int(o["msn"])))
        docs.append(msgs)
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(len(docs), seg_cap=128, max_retries=24) as b:
        b.ingest_messages(docs)
        b.run()
        launches = b.launches()
        classes = [li["seg_class"] for li in launches]
        assert GIANT in classes and len(set(classes)) >= 3, launches
        for i in range(len(docs)):
            assert_doc_parity(b.doc(i), oracle[i])


def test_early_escalation_while_the_first_launch_runs():
    """A batch whose first launch fits nearly every document (2,048 of 1,500 ops in class 464) and a
    few wide-window documents (refSeq lag up to 1,500: the overlay list outgrows the class within
    a few hundred ops).  Those append an early-escalation notice (mt_engine.hip escalation_notice)
    and the host starts their next launch while the first one still runs (mt_host.cpp
    poll_notices); every document equals the oracle, and the first launch's ops exclude the
    escalated documents' resumed part exactly once."""
    n_small, wide_at = 2048, (5, 700, 1400, 2047)
    small = O.gen_params(1500, pct_insert=55, pct_remove=35, seed=0xEA51)
    wide = O.gen_params(1500, max_lag=1500, pct_insert=55, pct_remove=35, seed=0xEA52)
    params = [wide if d in wide_at else small for d in range(n_small)]
    ops, text, props, off = O.gen_batch(small, n_small, doc_params=params)
    t, names = O.gen_tables(), O.gen_client_names(small.n_clients)
    _, dig, st = O.replay_batch(ops, off, text, props, t, names)
    with fa.ReplayBatch(n_small) as b:
        b.set_tables(GEN_KEYS, GEN_VALUES)
        b.set_clients(names)
        b.ingest(ops, off, text, props)
        b.run()
        launches = b.launches()
        first = launches[0]
        assert first["seg_class"] == 464 and first["n_docs"] == n_small, launches
        early = [li for li in launches[1:] if li["start_ms"] < first["start_ms"] + first["ms"]]
        assert early, launches
        # (a document re-run from scratch counts its first partial replay too)
        if all(li["resumed"] == li["n_docs"] for li in launches[1:]):
            assert sum(li["ops"] for li in launches) == len(ops), launches
        for d in range(n_small):
            dv = b.doc(d)
            assert dv.status == st[d] == 0, d
            assert dv.digest() == int(dig[d]), d


def test_giant_document_beyond_65k_segments():
    """A document far beyond the LDS classes and 16-bit ids (>= 100k live segments; SURVEY §8d
    config 4's tail) escalates through the ladder into the giant class (2M slots, 32-bit slot and
    block ids, the top of the tree / overlay list / heap in the CU's LDS, the rest in HBM) and
    stays bit-exact with the oracle."""
    p = O.gen_params(360000, pct_insert=50, pct_remove=15, seed=4096)  # 35% annotate: props keep segments apart
    ops, text, props, off = O.gen_batch(p, 1)
    t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
    _, dig, st = O.replay_batch(ops, off, text, props, t, names)
    with fa.ReplayBatch(1) as b:
        b.set_tables(GEN_KEYS, GEN_VALUES)
        b.set_clients(names)
        b.ingest(ops, off, text, props)
        b.run()
        c = b.counters()
        hbm = [li for li in b.launches() if li["seg_class"] == GIANT]
        print(f"max slots {int(c['max_slots'][0])}; giant class: {hbm[0]['ops']} ops in {hbm[0]['ms']:.1f} ms = "
              f"{1e3 * hbm[0]['ms'] / max(1, hbm[0]['ops']):.2f} us/op")
        assert b.doc(0).status == st[0] == 0
        assert b.doc(0).digest() == int(dig[0])
        assert hbm and hbm[0]["ops"] > 0
        assert int(c["max_slots"][0]) >= 100000, int(c["max_slots"][0])
        od = O.replay_doc(ops.copy(), text, props, t, names)
        assert b.doc(0).get_text() == od.text()
        assert b.doc(0).snapshot_v1() == od.snapshot_v1()


def test_config4_largest_document_beyond_a_million_segments():
    """BASELINE configs[3]'s largest Zipf document at full size: 2M ops of the config-4 mix (insert 50 /
    remove 15 / annotate 35, so props keep neighbouring segments apart), generated on the GPU, grows
    past 1,000,000 segment slots (about a million live segments at the end), escalates through the
    LDS ladder into the giant class and replays bit-exact with the oracle on the downloaded log:
    state digest, text and SnapshotV1.  Prints the giant class's microseconds per op."""
    n_ops = 2000000
    with fa.ReplayBatch(1) as b:
        b.generate(fa.gen_params(n_ops, pct_insert=50, pct_remove=15, seed=4096), 0)
        ops, off, text, props = b.download_log()
        print("generated", flush=True)
        b.run()
        print("replayed", flush=True)
        c = b.counters()
        giant = [li for li in b.launches() if li["seg_class"] == GIANT]
        print(f"max slots {int(c['max_slots'][0])}, out entries {int(c['n_entries'][0])}, depth {int(c['depth'][0])}; "
              f"giant class: {giant[0]['ops']} ops in {giant[0]['ms']:.1f} ms = "
              f"{1e3 * giant[0]['ms'] / max(1, giant[0]['ops']):.2f} us/op; launches "
              f"{[(li['seg_class'], round(li['ms'], 1)) for li in b.launches()]}", flush=True)
        assert b.doc(0).status == 0
        assert giant and giant[0]["ops"] > n_ops // 2
        assert int(c["max_slots"][0]) >= 1000000, int(c["max_slots"][0])
        od = O.replay_doc(ops.copy(), text, props, O.gen_tables(), O.gen_client_names(8))
        assert od.status == 0
        dv = b.doc(0)
        assert dv.digest() == od.digest()
        assert dv.get_text() == od.text()
        assert dv.snapshot_v1() == od.snapshot_v1()


def test_wide_collab_window_passes_through_the_giant_class_to_the_hbm_class():
    """A client that never advances its refSeq holds minSeq at 0, so every segment stays in the
    overlay list: the list outgrows the LDS classes and the giant class's LDS list (kGiantUlist), and
    the document continues in the HBM class (every table in HBM) — the checkpoint passes through
    the giant class unchanged — bit-exact with the oracle."""
    import random

    rng = random.Random(11)
    msgs = [_msg("B", 1, 0, {"type": 0, "pos1": 0, "seg": "start"})]
    length = 5
    for k in range(2, 3200):
        pos = rng.randrange(length + 1)
        msgs.append(_msg("A", k, k - 1, {"type": 0, "pos1": pos, "seg": "ab"}))
        length += 2
    docs = [msgs]
    oracle = oracle_docs_from_messages(docs)
    assert oracle[0].status == 0, oracle[0].error
    with fa.ReplayBatch(1) as b:
        b.ingest_messages(docs)
        b.run()
        classes = [li["seg_class"] for li in b.launches()]
        assert GIANT in classes and HBM in classes, b.launches()
        assert int(b.counters()["max_unsettled"][0]) > 2048
        assert_doc_parity(b.doc(0), oracle[0])


def test_combining_ops_match_oracle():
    """combiningOp "incr" / "consensus" / other names with the reference's quirk (segmentPropertiesManager.ts:98
    passes the still-undefined local `newValue` to combine, so the op's values are ignored; incr of a
    number is NaN, serialized as null and matching nothing).  GPU == oracle on text, property runs, the
    segment table (zamboni merges) and SnapshotV1 (host and GPU serializers)."""
    docs = COMBINE_DOCS + [combine_farm(1500, seed=s) for s in (1, 2, 3)]
    oracle = oracle_docs_from_messages(docs)
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        b.snapshots()
        for i in range(len(docs)):
            assert b.doc(i).status == 0, (i, fa.status_string(b.doc(i).status))
            assert_doc_parity(b.doc(i), oracle[i])
            assert b.doc(i).snapshot_v1(device=True) == oracle[i].snapshot_v1(), i
        nan_doc = json.loads(b.doc(2).snapshot_v1()["header"])
        assert nan_doc["segmentCount"] >= 3, nan_doc  # NaN-valued halves are never coalesced
    with fa.ReplayBatch(len(docs), seg_cap=64) as b:  # through checkpoint / resume
        b.ingest_messages(docs)
        b.run()
        for i in range(len(docs)):
            assert_doc_parity(b.doc(i), oracle[i], full=False)


def test_combining_ops_outside_the_device_path_are_flagged():
    """Combines the device does not model are MT_UNSUPPORTED, never silently different: incr of a key
    holding a string (string concatenation), consensus over an object with seq -1 set by a plain
    annotate (the reference updates that shared object in place), an "other" combiningOp without a
    defaultValue on an absent key (a key holding undefined).  consensus of an absent key with a null
    defaultValue throws in the reference (the oracle fails too)."""
    docs = [
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "abc", "props": {"n": "s"}}}),
         _msg("A", 2, 1, {"type": 2, "pos1": 0, "pos2": 3, "props": {"n": 1}, "combiningOp": {"name": "incr"}})],
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abc"}),
         _msg("A", 2, 1, {"type": 2, "pos1": 0, "pos2": 3, "props": {"c": {"seq": -1}}}),
         _msg("A", 3, 2, {"type": 2, "pos1": 1, "pos2": 2, "props": {"c": 0}, "combiningOp": {"name": "consensus"}})],
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abc"}),
         _msg("A", 2, 1, {"type": 2, "pos1": 0, "pos2": 3, "props": {"c": 0}, "combiningOp": {"name": "other"}})],
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abc"}),
         _msg("A", 2, 1, {"type": 2, "pos1": 0, "pos2": 3, "props": {"c": 0},
                          "combiningOp": {"name": "consensus", "defaultValue": None}})],
    ]
    oracle = oracle_docs_from_messages(docs)
    assert [od.status for od in oracle] == [0, 0, 0, fa.MT_UNSUPPORTED]
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        assert [b.doc(i).status for i in range(len(docs))] == [fa.MT_UNSUPPORTED] * len(docs)


def test_relative_positions_match_oracle():
    """Ops addressed by marker ids (relativePos1 / relativePos2 with before / offset:
    Client.getValidOpRange client.ts:485-502, MergeTree.posFromRelativePos mergeTree.ts:1942-1966,
    getPosition :1586-1603): numeric and string ids, ids inside a GROUP, a marker unlinked by
    zamboni (the reference's map keeps the detached marker: position 0), random farms.  GPU == oracle
    on digest / text / props / SnapshotV1, also through checkpoint / resume."""
    docs = RELPOS_DOCS + [relpos_farm(400, seed=s) for s in (1, 2, 3, 4)]
    oracle = oracle_docs_from_messages(docs)
    for od in oracle:
        assert od.status == 0, od.error
    for opts in ({}, {"seg_cap": 64}):
        with fa.ReplayBatch(len(docs), **opts) as b:
            pb = b.ingest_messages(docs)
            b.run()
            for i in range(len(docs)):
                assert b.doc(i).status == 0, (i, fa.status_string(b.doc(i).status))
                assert_doc_parity(b.doc(i), oracle[i], full=not opts)
            if not opts:
                # the downloaded log holds value ids again (the device's marker keys mapped back),
                # so it re-ingests to the same replay
                ops, off, text, props = b.download_log()
                with fa.ReplayBatch(len(docs)) as b2:
                    b2.ingest_packed(dataclasses.replace(pb, ops=ops, doc_op_off=off, text=text, props=props))
                    b2.run()
                    for i in range(len(docs)):
                        assert b2.doc(i).digest() == b.doc(i).digest(), i
    for dev in ("gpu", "host"):  # the native JSON ingests pack them the same way
        with fa.ReplayBatch(len(docs)) as b:
            b.ingest_json([json.dumps(d) for d in docs], device=dev)
            b.run()
            for i in range(len(docs)):
                assert_doc_parity(b.doc(i), oracle[i], full=False)


def test_relative_positions_outside_the_device_path_are_flagged():
    """An id that names no marker (the reference passes position -1 on), an id two markers carry
    (the reference's map follows its blockUpdate order) and ids re-annotated on markers are
    MT_UNSUPPORTED on the device, never silently different."""
    mk = lambda i: {"marker": {"refType": 1}, "props": {"markerId": i}}
    docs = [
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abc"}),
         _msg("A", 2, 1, {"type": 0, "relativePos1": {"id": "nope"}, "seg": "x"})],
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abc"}),
         _msg("A", 2, 1, {"type": 0, "pos1": 1, "seg": mk("d")}),
         _msg("A", 3, 2, {"type": 0, "pos1": 3, "seg": mk("d")}),
         _msg("A", 4, 3, {"type": 0, "relativePos1": {"id": "d"}, "seg": "x"})],
        [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "abc"}),
         _msg("A", 2, 1, {"type": 0, "pos1": 1, "seg": mk("e")}),
         _msg("A", 3, 2, {"type": 2, "pos1": 1, "pos2": 2, "props": {"markerId": "f"}}),
         _msg("A", 4, 3, {"type": 0, "relativePos1": {"id": "e"}, "seg": "x"})],
    ]
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs)
        b.run()
        assert [b.doc(i).status for i in range(len(docs))] == [fa.MT_UNSUPPORTED] * len(docs)


@pytest.mark.parametrize("path", ["packer", "json_host", "json_auto", "escalating"])
def test_prop_sets_of_any_size(path):
    """Property sets of any size (properties.ts:95, textSegment.ts:23-28): inserts of 500 and 130
    props (the extended count record, include/mt_oplog.h MT_OPF_NPROPS_EXT), an annotate chain that
    grows sets past 300 keys with concurrent splitting annotates of two clients (zamboni merges
    neighbours whose large sets match), deletions, a rewrite with 80 keys, a 200-prop marker, and
    combiningOps over a 100-key set.  Sets past one pair per lane are built in the pool
    (mt_engine.hip props_extend_big).  Ingested by the Python packer, the host JSON parser, and the
    automatic GPU / host choice (the GPU parser's fast path takes objects of up to 16 keys, so these
    documents go to the host parser); "escalating" starts them in the smallest class, so they
    re-run in the bigprops kernel (cap_kind 11) and escalate through checkpoints with their large
    sets.  GPU == oracle on digest, text, props runs and SnapshotV1 (GPU and host serializers)."""
    from combine_logs import big_prop_docs

    docs = big_prop_docs()
    opts = {"seg_cap": 64, "max_retries": 24} if path == "escalating" else {}
    with fa.ReplayBatch(len(docs), **opts) as b:
        if path in ("packer", "escalating"):
            b.ingest_messages(docs)
        else:
            info = b.ingest_json([json.dumps(d) for d in docs], device="host" if path == "json_host" else "auto")
            assert info["path"] == "host"
        b.run()
        b.snapshots()
        for i, msgs in enumerate(docs):
            ref = O.Doc()
            ref.start_collab("readonly")
            for m in msgs:
                assert ref.apply_msg(json.dumps(m)) == 0, ref.error
            dv = b.doc(i)
            assert dv.status == 0, (i, fa.status_string(dv.status), int(b.counters()["cap_kind"][i]))
            assert dv.digest() == ref.digest(), i
            assert dv.get_text() == ref.text(), i
            assert dv.props_runs() == json.loads(ref.props_runs()), i
            assert dv.snapshot_v1() == ref.snapshot_v1(), i
            assert dv.snapshot_v1(device=True) == ref.snapshot_v1(), i
        # the largest set the replay built
        assert max(len(json.loads(x[2])) for i in range(len(docs)) for x in b.doc(i).props_runs()
                   if isinstance(x[2], str)) > 300
