"""GPU JSON op-log ingest (mt_json_gpu.hip) == the host parser (mt_pack_json), on the MI355X.

The GPU parser must produce the host parser's packed records, text, prop records and interned key /
value / client tables byte for byte on every log of its fast path (mt_json_gpu.h), report the first
document outside it (never a silently different result), and a batch ingested through it must
replay exactly like the host-ingested batch (the host parser is itself pinned to the Python / JS
packers by tests/test_json_ingest.py)."""
import json
import random

import numpy as np
import pytest

import fluidframework_amd as fa
import oracle_ffi as O
from fluidframework_amd.mtreplay import NotOnGpuPath, PackedJson, PackedJsonGpu
from kat_util import load_kats
from test_json_ingest import _farm_messages, _msg

pytestmark = pytest.mark.gpu


def _same(docs, observer="readonly"):
    want = PackedJson(docs, observer).arrays()
    pg = PackedJsonGpu(docs, observer)
    got = pg.arrays()
    assert (got.doc_op_off == want.doc_op_off).all()
    assert len(got.ops) == len(want.ops)
    for i in np.nonzero(got.ops != want.ops)[0][:3]:
        raise AssertionError(f"record {i}: GPU {got.ops[i]} host {want.ops[i]}")
    assert (got.text == want.text).all()
    assert len(got.props) == len(want.props) and (got.props == want.props).all()
    assert got.keys == want.keys
    assert got.values == want.values
    assert got.clients == want.clients
    return pg.stats


FAST_DOCS = [
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"text": "hello", "props": {"b": 1, "c": "x", "d": None}}}),
     _msg("B", 2, 0, {"type": 3, "ops": [{"type": 0, "pos1": 2, "seg": "XY"},
                                         {"type": 2, "pos1": 0, "pos2": 4, "props": {"c": True, "e": False}}]}),
     _msg("A", 3, 1, {"type": 0, "pos1": 3, "seg": {"text": "e", "props": {}}}, msn=1),
     _msg(None, 4, 3, None, msn=1, type_="join"),
     _msg("readonly", 5, 3, {"anything": [1, 2.5, {"x": "y"}]}, msn=1, type_="noop"),
     _msg("B", 6, 5, {"type": 1, "pos1": 0, "pos2": 2}, msn=3),
     _msg("C", 7, 6, {"type": 3, "ops": []}, msn=5),
     _msg("A", 8, 7, {"type": 2, "pos1": 0, "pos2": 1, "props": {}, "combiningOp": None}, msn=5),
     _msg("null", 9, 8, {"type": 1, "pos1": 0, "pos2": 1}, msn=5),
     _msg("A", 10, 9, {"type": 0, "pos1": 0, "seg": {"text": "p", "props": None}, "register": None}, msn=5),
     _msg("B", 11, 10, {"type": 2, "pos1": 0, "pos2": 3, "props": {"b": 2, "c": None},
                        "combiningOp": {"name": "rewrite"}}, msn=5),
     _msg("B", 12, 11, {"type": 2, "pos1": 0, "pos2": 1, "props": {"e": 1}, "combiningOp": False}, msn=5)],
    [_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "a\ud83d"}),
     _msg("A", 2, 1, {"type": 0, "pos1": 2, "seg": "\ude00b\"\\\n\x01é€😀\t/"}),
     _msg("B", 3, 2, {"type": 2, "pos1": 0, "pos2": 3, "props": {"k": -12, "n": 0, "s": "a b~", "big": 123456789012345}}),
     _msg("B", 4, 3, {"type": 0, "pos1": 1, "seg": "x\n"})],
    [],
]


def _extra_fields(doc, rng):
    """The same messages with the fields real logs carry around the op (timestamps, traces,
    metadata) and a shuffled key order."""
    out = []
    for m in doc:
        m = dict(m)
        m["timestamp"] = 1.6e12 + rng.random()
        m["traces"] = [{"service": "alfred", "action": "start", "timestamp": 1.5e3}]
        m["term"] = 1
        m["metadata"] = {"batch": rng.random() < 0.5}
        items = list(m.items())
        rng.shuffle(items)
        out.append(dict(items))
    return out


def test_fast_path_shapes_parse_identically():
    _same([json.dumps(d) for d in FAST_DOCS] + [json.dumps(FAST_DOCS[1], ensure_ascii=False)])


def test_kats_parse_identically():
    """Every reference KAT log on the fast path parses identically; the others (markers,
    rewrite annotates) are reported."""
    on_path = 0
    for k in load_kats():
        try:
            _same([json.dumps(k["messages"])])
            on_path += 1
        except NotOnGpuPath:
            pass
    assert on_path >= 3


def test_generated_logs_parse_identically():
    farm = _farm_messages()
    rng = random.Random(5)
    docs = [farm, farm[:3000], _extra_fields(farm[:2000], rng), FAST_DOCS[0]] * 3
    texts = [json.dumps(d) for d in docs]
    # whitespace and indentation variants
    texts.append("[\n  " + ",\n  ".join(json.dumps(m, indent=1) for m in farm[:500]) + "\n]\n")
    texts.append(" \t[ " + " , ".join(json.dumps(m, separators=(",", ":")) for m in farm[:500]) + " ] \r\n")
    st = _same(texts)
    assert st["n_msgs"] == sum(len(d) for d in docs) + 1000


def test_observer_and_many_clients():
    docs = [[_msg(f"client-{i % 250}", i + 1, i, {"type": 0, "pos1": 0, "seg": "a"}) for i in range(600)],
            [_msg("me", 1, 0, None, type_="join"), _msg("X", 2, 0, {"type": 0, "pos1": 0, "seg": "a"})]]
    _same([json.dumps(d) for d in docs], observer="me")


# property values outside JSON.stringify form: parsed on the GPU, formatted by the host
# (JSON.stringify(JSON.parse(text)): Number::toString, JS key order, duplicate keys), equal tables
_ANN = '{"clientId":"A","sequenceNumber":%d,"referenceSequenceNumber":0,"minimumSequenceNumber":0,' \
       '"type":"op","contents":{"type":2,"pos1":0,"pos2":1,"props":{"a":%s}}}'
CANON_VALUES = ["1.5", "1.50", "1.5e0", "15E-1", "1.0", "-0.0", "-0", "1e21", "1e-7", "5e-7", "123456789012345678",
                "1.7976931348623157e308", "1e400", "-1e400", "0.1", "[[1]]", "[1, [2, {\"z\": 0.1}]]", '{"b": 1}',
                '{"2": 1, "b": 2, "1": 3}', '{"x": 1, "y": 0, "x": 2}', '{ }', '[ ]', '"\\/"', '"\\u0041\\u00e9"',
                '"\\ud83d\\ude00"', '"\\ud800"', '[true, null, "a"]', '{"k": {"n": [1.25e2, {"0": 0}]}}']
CANON_DOC = "[" + ",".join(_ANN % (i + 1, v) for i, v in enumerate(CANON_VALUES)) + "]"


def test_values_outside_stringify_form_parse_identically():
    """floats / exponents / long integers, objects (key order, duplicate keys, whitespace), nested
    arrays and other string escapes stay on the GPU path: the host formats the few unique value
    texts, and the batch tables equal the host parser's (first-appearance order included)."""
    st = _same([CANON_DOC, json.dumps([_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {
        "marker": {"refType": 1}, "props": {"referenceTileLabels": ["a", "b"], "x": {"y": [1.5]}}}}),
        _msg("B", 2, 1, {"type": 2, "pos1": 0, "pos2": 1, "props": {"a": "é", "b": 2.5}})]), CANON_DOC])
    assert st["n_msgs"] == 2 * len(CANON_VALUES) + 2


OUTSIDE = [  # (message, reason) — every one must be reported, never parsed differently
    (_msg("A", 1, 0, {"type": 2, "pos1": 0, "pos2": 1, "props": {"1": 1}}), "array-index key"),
    (_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": {"marker": {"refType": 1.5}}}), "float refType"),
    (_msg("A", 1, 0, {"type": 2, "pos1": 0, "pos2": 1, "props": {"a": 1},
                      "combiningOp": {"name": "incr"}}), "combiningOp incr"),
    (_msg("A", 1, 0, {"type": 2, "pos1": 0, "pos2": 1, "props": {"a": 1},
                      "combiningOp": {"defaultValue": 1}}), "combiningOp without a name"),
    (_msg("A", 1, 0, {"type": 1, "relativePos1": {"id": "m", "offset": 1.5}, "pos2": 1}), "float offset"),
    (_msg("A", 1, 0, {"type": 1, "relativePos1": {"id": {"x": 1}}, "pos2": 1}), "object id"),
    (_msg("A", -1, 0, {"type": 0, "pos1": 0, "seg": "a"}), "local op of another client"),
    (_msg("readonly", -1, 0, {"type": 0, "pos1": 0, "pos2": 1, "seg": "a"}), "local insert with an end"),
    (_msg("readonly", -1, 0, [{"type": 1, "pos1": 0, "pos2": 1}], type_="regenerate"), "regenerate"),
    (dict(_msg("readonly", -1, 0, {"type": 2, "pos1": 0, "pos2": 1, "props": {"a": 1}}), notifyConsensus=True),
     "notifyConsensus"),
    (_msg("readonly", 1, 0, {"type": 1, "relativePos1": {"id": "m"}, "pos2": 1}), "ack with a relative position"),
    (_msg("A", 1, 0, {"type": 3, "ops": [{"type": 3, "ops": []}]}), "nested group"),
    (_msg("A", 1, 0, {"type": 0, "pos1": 0, "seg": "a", "register": "r"}), "register"),
    (_msg("A", 2 ** 31, 0, {"type": 1, "pos1": 0, "pos2": 1}), "seq beyond int32"),
]


@pytest.mark.parametrize("msg,why", OUTSIDE, ids=[w for _, w in OUTSIDE])
def test_outside_the_fast_path_is_reported(msg, why):
    docs = [json.dumps(FAST_DOCS[0]), json.dumps([msg])]
    with pytest.raises(NotOnGpuPath) as e:
        PackedJsonGpu(docs)
    assert e.value.bad_doc == 1, why


@pytest.mark.parametrize("text", ['[{"clientId": "A", "sequenceNumber": 1,', '[{"a":1}', '{"messages": []}',
                                  '[{"sequenceNumber":1,"referenceSequenceNumber":0,"minimumSequenceNumber":0},]',
                                  '[,{"sequenceNumber":1,"referenceSequenceNumber":0,"minimumSequenceNumber":0}]',
                                  '[1]', '[] x', '', '[{"clientId":"A","clientId":"B","sequenceNumber":1,'
                                  '"referenceSequenceNumber":0,"minimumSequenceNumber":0}]',
                                  '[{"sequenceNumber":01,"referenceSequenceNumber":0,"minimumSequenceNumber":0}]'])
def test_malformed_or_unusual_json_is_reported(text):
    with pytest.raises(NotOnGpuPath) as e:
        PackedJsonGpu(["[]", text])
    assert e.value.bad_doc == 1


def _replay_equal(b1, b2, n):
    for d in range(n):
        x, y = b1.doc(d), b2.doc(d)
        assert x.status == y.status, d
        assert x.digest() == y.digest(), d
        if d % 3 == 0 and x.status == 0:
            assert x.get_text() == y.get_text()
            assert x.props_runs() == y.props_runs()
            assert x.snapshot_v1() == y.snapshot_v1()


def test_gpu_ingest_replays_like_host_ingest():
    farm = _farm_messages()
    docs = [farm, farm[:4000], FAST_DOCS[0], FAST_DOCS[1], [], farm[:7000]]
    texts = [json.dumps(d) for d in docs]
    with fa.ReplayBatch(len(docs)) as g, fa.ReplayBatch(len(docs)) as h:
        info = g.ingest_json(texts, device="gpu")
        assert info["path"] == "gpu" and info["n_msgs"] == sum(len(d) for d in docs)
        h.ingest_json(texts, device="host")
        g.run()
        h.run()
        _replay_equal(g, h, len(docs))


def test_gpu_ingest_replays_canonicalized_values_and_many_clients():
    """Annotates whose values the host canonicalizes (floats, objects, escapes) and a document of
    700 writers (client ids beyond 8 bits) replay on the GPU-ingested batch exactly like the
    host-ingested one: same digests, text, property runs and snapshots."""
    ins = ('{"clientId":"Z","sequenceNumber":1,"referenceSequenceNumber":0,"minimumSequenceNumber":0,'
           '"type":"op","contents":{"type":0,"pos1":0,"seg":"abcdef"}}')
    canon_msgs = [ins] + [_ANN.replace('"referenceSequenceNumber":0', '"referenceSequenceNumber":1') % (i + 2, v)
                          for i, v in enumerate(CANON_VALUES)]
    canon = "[" + ",".join(canon_msgs) + "]"
    crowd = [_msg(f"writer-{i}", i + 1, i, {"type": 0, "pos1": i % (i + 1), "seg": chr(65 + i % 26)})
             for i in range(700)]
    crowd += [_msg(f"writer-{i}", 701 + k, 700 + k, {"type": 2, "pos1": i, "pos2": i + 2, "props": {"w": i * 0.5}})
              for k, i in enumerate(range(0, 600, 7))]
    texts = [canon, json.dumps(crowd), canon]
    want = []
    for msgs in (canon_msgs, [json.dumps(m) for m in crowd], canon_msgs):  # the oracle's JSON path
        ref = O.Doc()
        ref.start_collab("readonly")
        for m in msgs:
            assert ref.apply_msg(m) == 0, ref.error
        want.append((ref.digest(), json.loads(ref.props_runs())))
    with fa.ReplayBatch(len(texts)) as g, fa.ReplayBatch(len(texts)) as h:
        assert g.ingest_json(texts, device="gpu")["path"] == "gpu"
        h.ingest_json(texts, device="host")
        g.run()
        h.run()
        for d in range(len(texts)):
            x, y = g.doc(d), h.doc(d)
            assert x.status == y.status == 0, d
            assert x.digest() == y.digest() == want[d][0]
            assert x.get_text() == y.get_text()
            assert x.props_runs() == y.props_runs() == want[d][1]
            assert x.snapshot_v1() == y.snapshot_v1()


def test_gpu_ingest_from_device_resident_json():
    """The parse reads JSON already in HBM (a buffer of the library's own HIP runtime)."""
    import ctypes as C

    hip = C.CDLL("libamdhip64.so.7")
    farm = _farm_messages()
    docs = [farm[:5000], farm[:3000], FAST_DOCS[0]]
    buf, off = fa.json_concat(docs)
    ptr = C.c_void_p()
    assert hip.hipMalloc(C.byref(ptr), C.c_size_t(len(buf) + 64)) == 0
    try:
        assert hip.hipMemset(ptr, 0, C.c_size_t(len(buf) + 64)) == 0
        assert hip.hipMemcpy(ptr, buf, C.c_size_t(len(buf)), 1) == 0  # hipMemcpyHostToDevice
        with fa.ReplayBatch(len(docs)) as g, fa.ReplayBatch(len(docs)) as h:
            g.ingest_json_gpu(buf, off, d_json=ptr)
            h.ingest_json([json.dumps(d) for d in docs], device="host")
            g.run()
            h.run()
            _replay_equal(g, h, len(docs))
    finally:
        hip.hipFree(ptr)


def test_auto_falls_back_to_the_host_parser():
    docs = [json.dumps(FAST_DOCS[0]), json.dumps([OUTSIDE[0][0]])]
    with fa.ReplayBatch(2) as g, fa.ReplayBatch(2) as h:
        info = g.ingest_json(docs)
        assert info["path"] == "host" and info["bad_doc"] == 1
        h.ingest_json(docs, device="host")
        g.run()
        h.run()
        _replay_equal(g, h, 2)


def _fuzz_doc(rng: random.Random, n: int) -> str:
    """A random observer log on (and sometimes just off) the fast path, as JSON text with random
    whitespace, key order, escapes and extra fields."""
    alphabet = "ab c\n\t\"\\/é€😀 \x01\x1f" + "xyz" * 5
    names = [f"client-{i}" for i in range(rng.randrange(1, 6))] + [None, "readonly"]

    def ws():
        return rng.choice(["", "", " ", "\n", "\t ", "\r\n  "])

    def dump(v):
        if isinstance(v, dict):
            items = list(v.items())
            rng.shuffle(items)
            return "{" + ws() + ("," + ws()).join(f"{json.dumps(k)}{ws()}:{ws()}{dump(x)}" for k, x in items) + ws() + "}"
        if isinstance(v, list):
            return "[" + ws() + ("," + ws()).join(dump(x) for x in v) + ws() + "]"
        return json.dumps(v, ensure_ascii=rng.random() < 0.5)

    def text():
        return "".join(rng.choice(alphabet) for _ in range(1 + rng.randrange(6)))

    def props():
        return {f"k{rng.randrange(5)}": rng.choice([None, True, False, 0, -7, 123456789012345, "red", "a b", ""])
                for _ in range(rng.randrange(4))}

    def op():
        t = rng.randrange(3)
        if t == 0:
            seg = text() if rng.random() < 0.6 else {"text": text(), **({"props": props()} if rng.random() < 0.7 else {})}
            return {"type": 0, "pos1": rng.randrange(50), "seg": seg}
        if t == 1:
            return {"type": 1, "pos1": rng.randrange(50), "pos2": rng.randrange(50)}
        return {"type": 2, "pos1": rng.randrange(50), "pos2": rng.randrange(50), "props": props()}

    msgs = []
    for s in range(1, n + 1):
        cid = rng.choice(names)
        m = {"clientId": cid, "sequenceNumber": s, "referenceSequenceNumber": rng.randrange(s),
             "minimumSequenceNumber": 0}
        if cid == "readonly" or rng.random() < 0.1:
            m["type"] = rng.choice(["join", "leave", "noop"])
            m["contents"] = rng.choice([None, {"x": [1.5, {"y": "z"}]}, "s"])
        else:
            m["type"] = "op"
            u = rng.random()
            m["contents"] = {"type": 3, "ops": [op() for _ in range(rng.randrange(4))]} if u < 0.15 else op()
        if rng.random() < 0.3:
            m["timestamp"] = rng.random() * 1e12
            m["traces"] = [{"a": rng.random(), "b": [None, True]}]
        msgs.append(m)
    return "[" + ws() + ("," + ws()).join(dump(m) for m in msgs) + ws() + "]" + ws()


def test_fuzzed_logs_parse_identically_or_are_reported():
    """Random logs (unicode / escapes / whitespace / key order / extra fields / groups / noops): the
    GPU parser equals the host parser on every batch it accepts, and the batches it reports name a
    document the host parser also handles or rejects by itself."""
    rng = random.Random(1234)
    accepted = 0
    for trial in range(40):
        docs = [_fuzz_doc(rng, 1 + rng.randrange(300)) for _ in range(1 + rng.randrange(6))]
        try:
            _same(docs)
            accepted += 1
        except NotOnGpuPath as e:
            assert 0 <= e.bad_doc < len(docs)
    assert accepted >= 20


def _marker_doc(rng: random.Random, n: int, compact=(",", ":")):
    """A text + Tile-marker log as JSON.stringify writes it (compact): paragraph markers with
    referenceTileLabels and markerIds, annotates, removes."""
    msgs, length = [], 0
    for s in range(1, n + 1):
        u = rng.random()
        if length == 0 or u < 0.25:
            seg = {"marker": {"refType": rng.choice([0, 1, 2])},
                   "props": {"referenceTileLabels": rng.sample(["pg", "EOP", "cell"], 1 + rng.randrange(2)),
                             **({"markerId": f"m{s}"} if rng.random() < 0.5 else {})}}
            op, dl = {"type": 0, "pos1": rng.randrange(length + 1), "seg": seg}, 1
        elif u < 0.6:
            t = "".join(rng.choice("abc de") for _ in range(1 + rng.randrange(5)))
            op, dl = {"type": 0, "pos1": rng.randrange(length + 1), "seg": t}, len(t)
        elif u < 0.8:
            a = rng.randrange(length)
            b = min(length, a + 1 + rng.randrange(3))
            op, dl = {"type": 1, "pos1": a, "pos2": b}, a - b
        else:
            a = rng.randrange(length)
            op, dl = {"type": 2, "pos1": a, "pos2": min(length, a + 2), "props": {"bold": rng.random() < 0.5}}, 0
        length += dl
        msgs.append(_msg(f"c{rng.randrange(3)}", s, s - 1, op, msn=max(0, s - 4)))
    return json.dumps(msgs, separators=compact)


def test_markers_and_tile_labels_on_the_gpu_path():
    """Tile markers (refType, referenceTileLabels arrays, markerIds) parse on the GPU exactly as on
    the host, and the GPU-ingested batch replays to the same state and findTile answers."""
    rng = random.Random(99)
    docs = [_marker_doc(rng, 200 + 50 * i) for i in range(6)]
    _same(docs)
    with fa.ReplayBatch(len(docs)) as g, fa.ReplayBatch(len(docs)) as h:
        assert g.ingest_json(docs, device="gpu")["path"] == "gpu"
        h.ingest_json(docs, device="host")
        g.run()
        h.run()
        _replay_equal(g, h, len(docs))
        for d in range(len(docs)):
            n = len(g.doc(d).get_text()) + 8
            for pos in range(0, n, 3):
                for label in ("pg", "EOP"):
                    for prec in (True, False):
                        assert g.doc(d).find_tile(pos, label, prec) == h.doc(d).find_tile(pos, label, prec)


def test_relative_positions_on_the_gpu_path():
    """Ops addressed by marker ids (relativePos1 / relativePos2 with id / before / offset): the GPU
    packs the same MT_OP_RELPOS records and value table as the host (ids are interned in the host
    packer's value() order: a relative position's id before the op's props), and the GPU-ingested
    batch replays like the host-ingested one."""
    from combine_logs import RELPOS_DOCS, relpos_farm

    docs = [json.dumps(d, separators=(",", ":")) for d in RELPOS_DOCS + [relpos_farm(300, seed=5), relpos_farm(500, seed=6)]]
    on_path = []
    for d in docs:
        try:
            _same([d])
            on_path.append(d)
        except NotOnGpuPath:
            pass
    assert len(on_path) >= 2
    _same(on_path)
    with fa.ReplayBatch(len(on_path)) as g, fa.ReplayBatch(len(on_path)) as h:
        assert g.ingest_json(on_path, device="gpu")["path"] == "gpu"
        h.ingest_json(on_path, device="host")
        g.run()
        h.run()
        _replay_equal(g, h, len(on_path))


def test_string_values_with_escapes_and_unicode():
    """String prop values already in JSON.stringify form (escaped quotes / backslashes / control
    characters, raw non-ASCII as json.dumps(ensure_ascii=False) writes them) parse on the GPU like
    on the host; other spellings of the same strings (\\u escapes of printable characters, \\/,
    uppercase hex) too, formatted by the host (JSON.stringify(JSON.parse(text)))."""
    vals = ["say \"hi\"", "back\\slash", "tab\tnl\nret\r", "ctl\x01\x1f", "é€😀 café", "ß\u2028x", "a/b", "del\x7f"]
    msgs = [_msg("A", i + 1, i, {"type": 0, "pos1": 0, "seg": {"text": "x", "props": {"k": v}}}) for i, v in enumerate(vals)]
    msgs.append(_msg("B", len(vals) + 1, len(vals), {"type": 2, "pos1": 0, "pos2": 2, "props": {"tags": ["ü", "a\"b"]}}))
    _same([json.dumps(msgs, ensure_ascii=False, separators=(",", ":"))])
    for raw in ['"\\u0041"', '"a\\/b"', '"\\u001F"', '"\\u00e9"']:
        doc = ('[{"clientId":"A","sequenceNumber":1,"referenceSequenceNumber":0,"minimumSequenceNumber":0,'
               '"type":"op","contents":{"type":2,"pos1":0,"pos2":1,"props":{"k":' + raw + '}}}]')
        _same(["[]", doc])


def _writer_streams(n_docs=6, steps=400):
    """Writer replica "A"'s stream of several conflict farms (local ops as sequenceNumber -1, its own
    sequenced messages as acks; rewrites and markers included): one document per farm."""
    from writer_sim import farm

    return [farm(4, steps, 11 + k, rewrite=20, markers=10).events["A"] for k in range(n_docs)]


def test_writer_streams_parse_identically():
    """A writer replica's log stays on the GPU fast path: records (seq -1 local ops, acks), text,
    props and tables equal the host parser's byte for byte."""
    docs = _writer_streams()
    assert any(m["sequenceNumber"] == -1 for m in docs[0])
    st = _same([json.dumps(d) for d in docs], observer="A")
    assert st["n_msgs"] == sum(len(d) for d in docs)
    got = PackedJsonGpu([json.dumps(d) for d in docs], "A").arrays()
    assert (got.ops["seq"] == -1).any()


def test_gpu_ingested_writer_streams_replay_like_host_and_oracle():
    """mt_batch_ingest_json_gpu of writer streams sets up the writer regions (pending groups) and
    replays in the writer kernel exactly like the host-ingested batch and the oracle's replica."""
    from test_gpu_writer import oracle_replica

    docs = _writer_streams()
    texts = [json.dumps(d) for d in docs]
    with fa.ReplayBatch(len(docs)) as g, fa.ReplayBatch(len(docs)) as h:
        assert g.ingest_json(texts, observer="A", device="gpu")["path"] == "gpu"
        h.ingest_json(texts, observer="A", device="host")
        g.run()
        h.run()
        _replay_equal(g, h, len(docs))
        for d, ev in enumerate(docs):
            ref = oracle_replica("A", ev)
            assert g.doc(d).status == 0 and g.doc(d).digest() == ref.digest(), d
            assert g.doc(d).get_text() == ref.text()


def test_gpu_ingested_writer_beyond_1024_pending_ops():
    """A writer stream with 1,500 unacked local ops parsed on the GPU: the device counts the
    replica's peak of pending groups (mt_json_gpu.hip jg_pending_peak_kernel) and the pending
    region is sized from it, so the replica equals the host-ingested batch and the oracle's."""
    from test_gpu_writer import max_pending, oracle_replica
    from writer_sim import Farm, random_op

    f = Farm(3, 1501)
    for i in range(1500):
        f.local("A", random_op(f.rng, f.docs["A"].length()))
        if i % 10 == 0:
            o = f.rng.choice(["B", "C"])
            f.local(o, random_op(f.rng, f.docs[o].length()))
            f.deliver(o, 1 + f.rng.randrange(3))
    f.finish()
    ev = f.events["A"]
    assert max_pending("A", ev) > 1024
    texts = [json.dumps(ev)]
    with fa.ReplayBatch(1) as g, fa.ReplayBatch(1) as h:
        assert g.ingest_json(texts, observer="A", device="gpu")["path"] == "gpu"
        h.ingest_json(texts, observer="A", device="host")
        g.run()
        h.run()
        _replay_equal(g, h, 1)
        ref = oracle_replica("A", ev)
        assert g.doc(0).status == ref.status == 0, (g.doc(0).status, ref.status)
        assert g.doc(0).digest() == ref.digest()
        assert g.doc(0).get_text() == ref.text()
