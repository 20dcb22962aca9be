"""Pack ISequencedDocumentMessage streams into the device op-log format (include/mt_oplog.h).

The reference consumes messages one at a time through ``Client.applyMsg(msg)``
(packages/dds/merge-tree/src/client.ts:797-819).  A message is

    {"clientId": str, "sequenceNumber": int, "referenceSequenceNumber": int,
     "minimumSequenceNumber": int, "type": "op", "contents": IMergeTreeOp}

(server/routerlicious/packages/protocol-definitions/src/protocol.ts:132-172) with
IMergeTreeOp one of insert {type:0,pos1,seg}, remove {type:1,pos1,pos2},
annotate {type:2,pos1,pos2,props,combiningOp?} or group {type:3,ops:[...]}
(merge-tree/src/ops.ts:29-110).  This module turns a batch of such streams into
the flat arrays that ``mt_batch_ingest`` takes: fixed 32-byte records, a UTF-16 text
arena, interned property keys/values and per-document client tables.

Short client ids are assigned per document in first-appearance order with the
observer first, exactly as ``Client.getOrAddShortClientId`` does (client.ts:636-660).

Writer replicas (the local-client path): a document's stream may also hold the replica's own
*unsequenced* messages — ``{"clientId": <replica>, "sequenceNumber": -1, "contents": op, ...}``,
what ``TestClient.makeOpMessage(op)`` builds for a local op (testClient.ts:213-234) — which the
replica applies locally (insertSegmentLocal / removeRangeLocal / annotateRangeLocal) and keeps
pending until its own *sequenced* message arrives and acks it (client.ts:797-819).  They pack as
records with seq -1 and client 0; the acks as ordinary records of client 0.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field

import numpy as np

# "tc": the record type (bits 0-3) and the 12-bit short client id (bits 4-15), mt_op's bit-fields
OP_DTYPE = np.dtype(
    [("tc", "<u2"), ("flags", "<u2"), ("seq", "<i4"), ("ref_seq", "<i4"),
     ("msn", "<i4"), ("pos1", "<i4"), ("pos2", "<i4"), ("payload", "<u4"), ("payload_len", "<u4")]
)
PROP_DTYPE = np.dtype([("key", "<u4"), ("value", "<u4")])
assert OP_DTYPE.itemsize == 32

OP_INSERT, OP_REMOVE, OP_ANNOTATE, OP_RELPOS, OP_REGENERATE, OP_NOOP = 0, 1, 2, 6, 7, 15
UNASSIGNED_SEQ = -1  # UnassignedSequenceNumber (merge-tree/src/constants.ts:11): a local, unacked op
# MT_OP_RELPOS flags (include/mt_oplog.h mt_relpos_flags)
RELF_POS1, RELF_POS2, RELF_BEFORE1, RELF_BEFORE2, RELF_OFF1, RELF_OFF2 = 0x10, 0x20, 0x40, 0x80, 0x100, 0x200
RELF_NOTIFY = 0x2  # a local RELPOS of Client.annotateMarkerNotifyConsensus (include/mt_oplog.h)
OPF_GROUP_CONT, OPF_MARKER, OPF_HAS_PROPS, OPF_REWRITE = 1, 2, 4, 8
# an insert's prop count: flags bits 4-10 up to NPROPS_INLINE; beyond, NPROPS_EXT there and a first
# record {KEY_NPROPS, count} (include/mt_oplog.h MT_OPF_NPROPS_EXT)
NPROPS_INLINE, NPROPS_EXT, KEY_NPROPS = 126, 127, 0xFFFFFFFE
# combiningOp other than "rewrite" (include/mt_oplog.h mt_combine_kind): annotate flags bits 4-5,
# then three records {KEY_COMBINE, defaultValue}, {KEY_COMBINE, minValue}, {KEY_COMBINE, result slot}
COMBINE_INCR, COMBINE_CONSENSUS, COMBINE_OTHER = 1, 2, 3
KEY_COMBINE = VALUE_UNDEFINED = 0xFFFFFFFF


MAX_CLIENTS = 0x7FFE  # short ids 0..32765 (include/mt_oplog.h MT_MAX_CLIENTS; 0x7FFE / 0x7FFF are sentinels)
CLIENT_NONCOLLAB, CLIENT_NONE = 0x7FFE, 0x7FFF
OPF_CLIENT_HI_MASK = 0x3800  # the short id's high 3 bits live in flags bits 11-13 (mt_oplog.h)


def rec_type(a):
    """record type(s) of an mt_op record / array (the low 4 bits of "tc")"""
    return a["tc"] & 0xF


def rec_client(a):
    """short client id(s) of an mt_op record / array: the high 12 bits of "tc", and flags bits 11-13
    above them (include/mt_oplog.h MT_OP_CLIENT)"""
    return (np.asarray(a["tc"], np.uint32) >> 4) | (((np.asarray(a["flags"], np.uint32) >> 11) & 7) << 12)


def make_tc(t, c):
    """the "tc" word of type t and short client id c (scalars or integer arrays)"""
    return (np.asarray(t, np.uint32) & 0xF) | (np.asarray(c, np.uint32) << 4)


def set_client(a, c):
    """replace the short client id(s) of records, keeping their types and other flags"""
    c = np.asarray(c, np.uint32)
    a["tc"] = make_tc(a["tc"] & 0xF, c & 0xFFF).astype(np.uint16)
    a["flags"] = ((np.asarray(a["flags"], np.uint32) & ~np.uint32(OPF_CLIENT_HI_MASK)) |
                  (((c >> 12) & 7) << 11)).astype(np.uint16)


class UnsupportedOp(ValueError):
    """An op shape outside the device's replay path (registers, relative positions or
    combiningOps in local ops, ...)."""


def js_truthy(v) -> bool:
    """JS ToBoolean of a JSON-parsed value."""
    if v is None or isinstance(v, bool):
        return bool(v)
    if isinstance(v, (int, float)):
        return v == v and v != 0
    if isinstance(v, str):
        return len(v) > 0
    return True


def js_stringify(value) -> str:
    """JSON.stringify for JSON-parsed values: integer-index keys first (ascending), then
    insertion order; no whitespace.  Python's json keeps insertion order, so only the
    integer-key hoisting needs doing."""
    if isinstance(value, dict):
        items = list(value.items())
        idx = [(int(k), k, v) for k, v in items if _is_array_index(k)]
        rest = [(k, v) for k, v in items if not _is_array_index(k)]
        ordered = [(k, v) for _, k, v in sorted(idx)] + rest
        return "{" + ",".join(_js_quote(k) + ":" + js_stringify(v) for k, v in ordered) + "}"
    if isinstance(value, list):
        return "[" + ",".join(js_stringify(v) for v in value) + "]"
    if isinstance(value, bool) or value is None:
        return json.dumps(value)
    if isinstance(value, (int, float)):
        return js_number(value)
    return _js_quote(value)


_LONE = re.compile("[\ud800-\udfff]")


def _js_quote(s: str) -> str:
    """JSON.stringify(string): like json.dumps(ensure_ascii=False), lone surrogates escaped
    (well-formed JSON.stringify); paired surrogates arrive as one code point from json.loads."""
    return _LONE.sub(lambda m: "\\u%04x" % ord(m.group()), json.dumps(s, ensure_ascii=False))


def js_number(v) -> str:
    """Number.prototype.toString (ECMA-262 Number::toString, radix 10) as JSON.stringify writes
    it: shortest round-trip digits, fixed notation for 1e-7 < |v| < 1e21, else d.ddde±x;
    NaN / Infinity -> null; integers beyond 2**53 are doubles first, as in JS."""
    from decimal import Decimal

    v = float(v) if not isinstance(v, int) or abs(v) >= 2 ** 53 else v
    if isinstance(v, int):
        return str(v)
    if v != v or v in (float("inf"), float("-inf")):
        return "null"
    if v == 0:
        return "0"
    sign = "-" if v < 0 else ""
    v = abs(v)
    if v < 2 ** 53 and v == int(v):
        return sign + str(int(v))
    t = Decimal(repr(v)).as_tuple()
    digits = "".join(map(str, t.digits))
    exp = t.exponent
    stripped = digits.rstrip("0")
    exp += len(digits) - len(stripped)
    digits = stripped or "0"
    k = len(digits)
    n = k + exp  # v = 0.d1..dk x 10**n
    if k <= n <= 21:
        out = digits + "0" * (n - k)
    elif 0 < n <= 21:
        out = digits[:n] + "." + digits[n:]
    elif -6 < n <= 0:
        out = "0." + "0" * (-n) + digits
    else:
        e = n - 1
        out = digits[0] + ("." + digits[1:] if k > 1 else "") + "e" + ("+" if e >= 0 else "-") + str(abs(e))
    return sign + out


def _is_array_index(k: str) -> bool:
    if not k or len(k) > 10 or not k.isdigit() or (k[0] == "0" and len(k) > 1):
        return False
    return int(k) <= 4294967294


def _utf16(s: str) -> np.ndarray:
    return np.frombuffer(s.encode("utf-16-le", "surrogatepass"), dtype="<u2")


def _js_keys(obj: dict) -> list:
    """Object.keys order of a JSON-parsed object."""
    ks = list(obj.keys())
    idx = sorted((k for k in ks if _is_array_index(k)), key=int)
    return idx + [k for k in ks if not _is_array_index(k)]


@dataclass
class PackedBatch:
    ops: np.ndarray
    doc_op_off: np.ndarray
    text: np.ndarray
    props: np.ndarray
    keys: list
    values: list
    clients: list  # per-document list of long client ids (index = short id)


@dataclass
class Packer:
    """Incrementally packs documents.  ``observer`` is the replica's own long id
    (``startOrUpdateCollaboration(observer)``), short id 0 in every document."""

    observer: str = "readonly"
    keys: list = field(default_factory=list)
    values: list = field(default_factory=lambda: ["null"])
    _key_ids: dict = field(default_factory=dict)
    _value_ids: dict = field(default_factory=lambda: {"null": 0})
    _ops: list = field(default_factory=list)
    _text: list = field(default_factory=list)
    _text_len: int = 0
    _props: list = field(default_factory=list)
    _off: list = field(default_factory=lambda: [0])
    _clients: list = field(default_factory=list)

    def _key(self, k: str) -> int:
        i = self._key_ids.get(k)
        if i is None:
            i = self._key_ids[k] = len(self.keys)
            self.keys.append(k)
        return i

    def _value(self, v) -> int:
        if v is None:
            return 0
        s = js_stringify(v)
        i = self._value_ids.get(s)
        if i is None:
            i = self._value_ids[s] = len(self.values)
            self.values.append(s)
        return i

    def _prop_records(self, props: dict) -> tuple[int, int]:
        if not isinstance(props, dict):
            raise UnsupportedOp("props must be an object")
        off = len(self._props)
        for k in _js_keys(props):
            self._props.append((self._key(k), self._value(props[k])))
        return off, len(self._props) - off

    def add_document(self, messages, replica: str | None = None) -> int:
        """Append one document's message stream; returns its index.  ``replica`` (default: the
        packer's ``observer``) is the document's own long id: its unsequenced messages
        (sequenceNumber -1) are local ops, its sequenced ones ack them (a writer replica)."""
        me = self.observer if replica is None else replica
        names = [me]
        short = {me: 0}
        recs = []
        for msg in messages:
            if isinstance(msg, str):
                msg = json.loads(msg)
            cid = msg["clientId"]
            if cid is None:  # system messages: one short id for all of them (mt_json.cpp does the same)
                cid = "null"
            if cid not in short:  # getOrAddShortClientId (client.ts:636-641)
                if len(names) >= MAX_CLIENTS:
                    raise UnsupportedOp(f"more than {MAX_CLIENTS - 1} clients (short ids are 15-bit)")
                short[cid] = len(names)
                names.append(cid)
            c = short[cid]
            seq = msg["sequenceNumber"]
            # a local op of this replica: an unsequenced message (TestClient.makeOpMessage's default
            # seq, UnassignedSequenceNumber = -1), applied with the replica's local view and kept
            # pending until the replica's own sequenced message (client 0) acks it
            local = seq == UNASSIGNED_SEQ
            if local and c != 0:
                raise UnsupportedOp("an unsequenced message of another client")
            base = dict(client=c, seq=seq, ref_seq=msg.get("referenceSequenceNumber", 0),
                        msn=0 if local else msg["minimumSequenceNumber"])
            if local and msg.get("type") == "regenerate":
                # Client.regeneratePendingOp(contents, oldest pending group) on reconnect: one
                # MT_OP_REGENERATE record per member of the reset op (include/mt_oplog.h)
                members = self._flatten(msg["contents"])
                for j, op in enumerate(members):
                    t = op.get("type")
                    r = dict(base, type=OP_REGENERATE, ref_seq=t, flags=0, pos1=0, pos2=0, payload=0, payload_len=0)
                    if t == 2:
                        cop = op.get("combiningOp")
                        if js_truthy(cop):
                            if not (isinstance(cop, dict) and cop.get("name") == "rewrite"):
                                raise UnsupportedOp("local combiningOp other than rewrite")
                            r["flags"] |= OPF_REWRITE
                        r["payload"], r["payload_len"] = self._prop_records(op.get("props"))
                    elif t not in (0, 1):
                        raise UnsupportedOp(f"regenerate of op type {t}")
                    if j + 1 < len(members):
                        r["flags"] |= OPF_GROUP_CONT
                    recs.append(r)
                continue
            if msg.get("type") != "op":
                if local:
                    raise UnsupportedOp("a local message that is not an op")
                recs.append(dict(base, type=OP_NOOP, flags=0, pos1=0, pos2=0, payload=0, payload_len=0))
                continue
            ack = c == 0 and not local  # Client.applyMsg -> ackPendingSegment (client.ts:810-812)
            members = self._flatten(msg["contents"])
            # {"notifyConsensus": true} on a local message: the op came from
            # Client.annotateMarkerNotifyConsensus (a repo-defined field of the writer stream)
            notify = local and js_truthy(msg.get("notifyConsensus"))
            notify_raw = 0
            if notify:
                notify_raw = self._notify_id(members)
            for j, op in enumerate(members):
                rel = self._relpos(op, base)
                if rel is not None:
                    if notify:
                        rel["flags"] |= RELF_NOTIFY
                        rel["payload"] = notify_raw
                    if not ack:  # an ack reads no positions
                        recs.append(rel)
                if local and op.get("type") == 0 and ("pos2" in op or js_truthy(op.get("relativePos2"))):
                    # getValidOpRange validates an insert's end when one is given (client.ts:520-524)
                    raise UnsupportedOp("a local insert with an end position")
                r = self._pack_op(op, base)
                if ack and op.get("type") == 2 and isinstance(op.get("combiningOp"), dict) and \
                        op["combiningOp"].get("name") == "consensus":
                    # updateConsensusProperty reads op.relativePos1.id (client.ts:981): a missing
                    # relativePos1 throws; an id a Map lookup cannot match (none, an object) is 0
                    rp = op.get("relativePos1")
                    if rp is None:
                        raise UnsupportedOp("ack of a consensus annotate without relativePos1 (a TypeError)")
                    rid = rp.get("id") if isinstance(rp, dict) else None
                    r["pos1"] = self._value(rid) if rid is not None and not isinstance(rid, (dict, list)) else 0
                if j + 1 < len(members):
                    r["flags"] |= OPF_GROUP_CONT
                recs.append(r)
            if not members:  # empty group: updateSeqNumbers only
                recs.append(dict(base, type=OP_NOOP, flags=0, pos1=0, pos2=0, payload=0, payload_len=0))
        self._ops.extend(recs)
        self._off.append(self._off[-1] + len(recs))
        self._clients.append(names)
        return len(self._clients) - 1

    def _notify_id(self, members: list) -> int:
        """The marker id a Client.annotateMarkerNotifyConsensus op registers (client.ts:113-134): the
        op createAnnotateMarkerOp makes (opBuilder.ts:25-39) with combiningOp {name: "consensus"}."""
        op = members[0] if len(members) == 1 else None
        ok = isinstance(op, dict) and op.get("type") == 2 and "pos1" not in op and "pos2" not in op and \
            op.get("combiningOp") == {"name": "consensus"}
        r1, r2 = (op.get("relativePos1"), op.get("relativePos2")) if ok else (None, None)
        ok = ok and isinstance(r1, dict) and isinstance(r2, dict) and "offset" not in r1 and "offset" not in r2
        mid = r1.get("id") if ok else None
        ok = ok and js_truthy(mid) and not isinstance(mid, (dict, list)) and r2.get("id") == mid and \
            type(r2.get("id")) is type(mid) and js_truthy(r1.get("before")) and not js_truthy(r2.get("before"))
        if not ok:
            raise UnsupportedOp("notifyConsensus on an op annotateMarkerNotifyConsensus does not make")
        return self._value(mid)

    @staticmethod
    def _flatten(op) -> list:
        if op.get("type") == 3:
            out = []
            for m in op.get("ops", []):
                out.extend(Packer._flatten(m))
            return out
        return [op]

    def _relpos(self, op: dict, base: dict):
        """The MT_OP_RELPOS record of an op whose pos1 (pos2) is undefined and relativePos1
        (relativePos2) truthy (Client.getValidOpRange, client.ts:485-502), else None."""
        t = op.get("type")
        r = dict(base, type=OP_RELPOS, flags=OPF_GROUP_CONT, pos1=0, pos2=0, payload=0, payload_len=0)
        for k in (1, 2):
            rp = op.get(f"relativePos{k}")
            if f"pos{k}" in op or not js_truthy(rp) or (k == 2 and t not in (1, 2)):
                continue
            r["flags"] |= RELF_POS1 if k == 1 else RELF_POS2
            rp = rp if isinstance(rp, dict) else {}
            if js_truthy(rp.get("id")):
                r[f"pos{k}"] = self._value(rp["id"])
            if js_truthy(rp.get("before")):
                r["flags"] |= RELF_BEFORE1 if k == 1 else RELF_BEFORE2
            if "offset" in rp:  # `offset !== undefined`; null adds 0
                off = rp["offset"] if rp["offset"] is not None else 0
                if isinstance(off, bool) or not isinstance(off, int):
                    raise UnsupportedOp("relative position offset must be an integer")
                r["flags"] |= RELF_OFF1 if k == 1 else RELF_OFF2
                r["payload" if k == 1 else "payload_len"] = off & 0xFFFFFFFF
        return r if r["flags"] & (RELF_POS1 | RELF_POS2) else None

    def _pack_op(self, op: dict, base: dict) -> dict:
        t = op.get("type")
        if "pos1" not in op and not js_truthy(op.get("relativePos1")):
            raise UnsupportedOp("op without a position")
        if op.get("register") is not None:
            raise UnsupportedOp("registers are not on the observer fast path")
        r = dict(base, type=t, flags=0, pos1=int(op["pos1"]) if "pos1" in op else 0, pos2=0, payload=0,
                 payload_len=0)
        if t == 0:
            seg = op.get("seg")
            props = None
            if isinstance(seg, str):
                text = seg
            elif isinstance(seg, dict) and "text" in seg:
                text, props = seg["text"], seg.get("props")
            elif isinstance(seg, dict) and "marker" in seg:
                r["flags"] |= OPF_MARKER
                r["payload"] = int(seg["marker"].get("refType", 0))
                r["payload_len"] = 1
                props = seg.get("props")
                text = None
            else:
                raise UnsupportedOp("unknown segment spec")
            if text is not None:
                u = _utf16(text)
                r["payload"] = self._text_len
                r["payload_len"] = len(u)
                self._text.append(u)
                self._text_len += len(u)
            if isinstance(props, list):
                raise UnsupportedOp("array props")
            if props:  # TextSegment.make: `if (props) addProperties(props)`
                off, n = self._prop_records(props)
                if n > NPROPS_INLINE:  # any number of props: the count leads the records
                    self._props.insert(off, (KEY_NPROPS, n))
                    n = NPROPS_EXT
                r["flags"] |= OPF_HAS_PROPS | (n << 4)
                r["pos2"] = off
            elif isinstance(props, dict):  # {} is truthy: an empty map is created
                r["flags"] |= OPF_HAS_PROPS
                r["pos2"] = len(self._props)
        elif t in (1, 2):
            r["pos2"] = int(op["pos2"]) if op.get("pos2") is not None else 0
            if t == 2:
                # addProperties (segmentPropertiesManager.ts:53-54): "rewrite" when op.name is
                # "rewrite", else any truthy combiningOp goes through Properties.combine
                cop = op.get("combiningOp")
                kind = 0
                if js_truthy(cop):
                    name = cop.get("name") if isinstance(cop, dict) else None
                    if isinstance(name, str) and name == "rewrite":
                        r["flags"] |= OPF_REWRITE
                    else:
                        kind = {"incr": COMBINE_INCR, "consensus": COMBINE_CONSENSUS}.get(
                            name if isinstance(name, str) else None, COMBINE_OTHER)
                # annotateRange -> addProperties(op.props) iterates its keys: an object is required
                r["payload"], r["payload_len"] = self._prop_records(op.get("props"))
                if kind:
                    r["flags"] |= kind << 4
                    c = cop if isinstance(cop, dict) else {}
                    for f in ("defaultValue", "minValue"):
                        self._props.append((KEY_COMBINE, self._value(c[f]) if f in c else VALUE_UNDEFINED))
                    self._props.append((KEY_COMBINE, VALUE_UNDEFINED))  # result slot (library)
        else:
            raise UnsupportedOp(f"op type {t}")
        return r

    def finish(self) -> PackedBatch:
        ops = np.zeros(len(self._ops), OP_DTYPE)
        for name in OP_DTYPE.names:
            if name == "tc":
                ops[name] = [r["type"] | ((r["client"] & 0xFFF) << 4) for r in self._ops] if self._ops else []
            elif name == "flags":  # the short id's high bits in flags 11-13
                ops[name] = [r["flags"] | (((r["client"] >> 12) & 7) << 11) for r in self._ops] if self._ops else []
            else:
                ops[name] = [r[name] for r in self._ops] if self._ops else []
        text = np.concatenate(self._text) if self._text else np.zeros(0, np.uint16)
        props = np.array(self._props, PROP_DTYPE) if self._props else np.zeros(0, PROP_DTYPE)
        return PackedBatch(ops=ops, doc_op_off=np.array(self._off, np.int64), text=text.astype(np.uint16),
                           props=props, keys=list(self.keys), values=list(self.values), clients=self._clients)


def pack_documents(docs, observer: str = "readonly") -> PackedBatch:
    p = Packer(observer=observer)
    for msgs in docs:
        p.add_document(msgs)
    return p.finish()


def writer_records(ops: np.ndarray, off: np.ndarray, writer_of: np.ndarray):
    """Writer replicas of observer logs whose messages are single records with contiguous seqs
    1..N per document (the generator's, include/mt_gen.h): document d is replayed as its client
    writer_of[d] (>= 1) saw it.  That writer's op k (seq s_k, refSeq r_k) was issued right after it
    processed message r_k, in the view (r_k, writer) — the same segments its local view held — so
    each of its records gets a local copy (seq -1, client 0, the writer's own unsequenced message)
    placed after record r_k, and the original stays as the ack.  Short ids: the writer becomes 0,
    the observer (0, which sends nothing) takes the writer's old id.  Vectorized over the batch;
    returns (ops, off): per-document client tables are the observer's with 0 and writer_of[d]
    swapped."""
    ops = np.asarray(ops)
    off = np.asarray(off, np.int64)
    D = len(off) - 1
    counts = np.diff(off)
    doc = np.repeat(np.arange(D, dtype=np.int64), counts)
    idx = np.arange(len(ops), dtype=np.int64) - off[doc]
    w = np.asarray(writer_of, np.int64)[doc]
    client = rec_client(ops).astype(np.int64)
    mine = client == w
    orig = ops.copy()
    set_client(orig, np.where(mine, 0, np.where(client == 0, w, client)))
    loc = ops[mine].copy()
    loc["seq"] = -1
    set_client(loc, 0)
    loc["msn"] = 0
    # order inside a document: original record i at 2i, a local copy with refSeq r at 2r - 1 (right
    # after the record with seq r, i.e. index r - 1); copies with the same refSeq in issue order
    key = np.concatenate([2 * idx, 2 * ops["ref_seq"][mine].astype(np.int64) - 1])
    tie = np.concatenate([idx, idx[mine]])
    dd = np.concatenate([doc, doc[mine]])
    allr = np.concatenate([orig, loc])
    order = np.lexsort((tie, key, dd))
    new_counts = counts + np.bincount(doc[mine], minlength=D)
    new_off = np.zeros(D + 1, np.int64)
    np.cumsum(new_counts, out=new_off[1:])
    return allr[order], new_off


def records_to_json(ops: np.ndarray, off: np.ndarray, text: np.ndarray, props: np.ndarray, keys: list,
                    values: list, clients) -> list:
    """The inverse of packing for observer logs: per document the JSON text of its
    ISequencedDocumentMessage array (single-record insert / remove / annotate messages and noops;
    text segments, annotate props; GROUP_CONT members become one group message).  clients: the
    long ids (one list for every document, or one per document).  Used to build JSON workloads
    from generated logs (tools/bench_json.py)."""
    ops = np.asarray(ops)
    off = np.asarray(off, np.int64)
    t16 = np.asarray(text, np.uint16)
    kq = [json.dumps(k) for k in keys]
    out = []
    shared = clients and isinstance(clients[0], str)
    typ = rec_type(ops).tolist()
    cli = rec_client(ops).tolist()
    flg = ops["flags"].tolist()
    seq = ops["seq"].tolist()
    ref = ops["ref_seq"].tolist()
    msn = ops["msn"].tolist()
    p1 = ops["pos1"].tolist()
    p2 = ops["pos2"].tolist()
    pay = ops["payload"].tolist()
    plen = ops["payload_len"].tolist()
    pk = props["key"].tolist() if len(props) else []
    pv = props["value"].tolist() if len(props) else []
    for d in range(len(off) - 1):
        names = [json.dumps(c) for c in (clients if shared else clients[d])]
        msgs, members = [], []
        for i in range(int(off[d]), int(off[d + 1])):
            t = typ[i]
            if t == OP_NOOP:
                c = None
            elif t == 0:
                s = t16[pay[i]:pay[i] + plen[i]].tobytes().decode("utf-16-le", "surrogatepass")
                c = f'{{"type":0,"pos1":{p1[i]},"seg":{json.dumps(s)}}}'
            elif t == 1:
                c = f'{{"type":1,"pos1":{p1[i]},"pos2":{p2[i]}}}'
            elif t == 2:
                pr = ",".join(f"{kq[pk[q]]}:{values[pv[q]]}" for q in range(pay[i], pay[i] + plen[i]))
                c = f'{{"type":2,"pos1":{p1[i]},"pos2":{p2[i]},"props":{{{pr}}}}}'
            else:
                raise UnsupportedOp(f"record type {t}")
            if c is not None:
                members.append(c)
            if flg[i] & OPF_GROUP_CONT:
                continue
            head = (f'{{"clientId":{names[cli[i]]},"sequenceNumber":{seq[i]},"referenceSequenceNumber":{ref[i]},'
                    f'"minimumSequenceNumber":{msn[i]},')
            if not members:
                msgs.append(head + '"type":"noop","contents":null}')
            elif len(members) == 1:
                msgs.append(head + f'"type":"op","contents":{members[0]}}}')
            else:
                msgs.append(head + f'"type":"op","contents":{{"type":3,"ops":[{",".join(members)}]}}}}')
            members = []
        out.append("[" + ",".join(msgs) + "]")
    return out
