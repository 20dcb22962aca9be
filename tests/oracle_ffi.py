"""ctypes binding of the test oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the CPU restatement of the reference's
merge-tree replay (see oracle/mt_oracle.h).  Product code never imports this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"
LIB_PATH = ORACLE_DIR / "build" / "liboracle.so"

OP_DTYPE = np.dtype(
    [
        ("tc", "<u2"),  # type (bits 0-3) | short client id << 4 (include/mt_oplog.h bit-fields)
        ("flags", "<u2"),
        ("seq", "<i4"),
        ("ref_seq", "<i4"),
        ("msn", "<i4"),
        ("pos1", "<i4"),
        ("pos2", "<i4"),
        ("payload", "<u4"),
        ("payload_len", "<u4"),
    ]
)
assert OP_DTYPE.itemsize == 32
PROP_DTYPE = np.dtype([("key", "<u4"), ("value", "<u4")])


class GenParams(C.Structure):
    _fields_ = [
        ("n_ops", C.c_int32),
        ("n_clients", C.c_int32),
        ("max_lag", C.c_int32),
        ("pct_insert", C.c_int32),
        ("pct_remove", C.c_int32),
        ("min_len", C.c_int32),
        ("max_insert", C.c_int32),
        ("pct_newline", C.c_int32),
        ("seed", C.c_uint64),
    ]


_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        build()
    L = C.CDLL(str(LIB_PATH))
    vp, cp, i, l, d = C.c_void_p, C.c_char_p, C.c_int, C.c_long, C.c_double
    L.mto_new.restype = vp
    L.mto_free.argtypes = [vp]
    L.mto_status.argtypes = [vp]
    L.mto_error.argtypes = [vp]
    L.mto_error.restype = cp
    L.mto_start_collab.argtypes = [vp, cp, i, i]
    L.mto_apply_msg_json.argtypes = [vp, cp]
    L.mto_load_snapshot_v1.argtypes = [vp, C.POINTER(cp), vp, i, cp]
    L.mto_insert_local_json.argtypes = [vp, i, cp]
    L.mto_annotate_local_json.argtypes = [vp, i, i, cp]
    L.mto_remove_local.argtypes = [vp, i, i]
    L.mto_local_op_json.argtypes = [vp, cp]
    L.mto_local_op_notify_json.argtypes = [vp, cp, i]
    L.mto_consensus_events.argtypes = [vp]
    L.mto_consensus_events.restype = C.c_void_p
    L.mto_local_marker_pos.argtypes = [vp, cp]
    L.mto_pending_groups.argtypes = [vp]
    L.mto_find_tile.argtypes = [vp, i, cp, i, C.POINTER(C.c_void_p)]
    L.mto_find_tile.restype = l
    L.mto_free_string.argtypes = [vp]
    L.mto_stack_context.argtypes = [vp, i, C.POINTER(cp), i, C.POINTER(i)]
    L.mto_stack_context.restype = C.c_void_p
    L.mto_regenerate_pending_op_json.argtypes = [vp, cp, C.POINTER(C.c_void_p)]
    L.mto_regenerated_ops.argtypes = [vp, C.c_char_p, l]
    L.mto_regenerated_ops.restype = l
    L.mto_get_length.argtypes = [vp]
    L.mto_view_length.argtypes = [vp, i, i]
    L.mto_current_seq.argtypes = [vp]
    L.mto_min_seq.argtypes = [vp]
    for fn in ("mto_get_text", "mto_props_runs", "mto_shape", "mto_dump"):
        getattr(L, fn).argtypes = [vp, C.c_char_p, l]
        getattr(L, fn).restype = l
    L.mto_snapshot_v1.argtypes = [vp, i]
    L.mto_snapshot_blob.argtypes = [vp, i, C.c_char_p, l, C.c_char_p, l]
    L.mto_snapshot_blob.restype = l
    L.mto_state_digest.argtypes = [vp]
    L.mto_state_digest.restype = C.c_uint64
    L.mto_tables_new.argtypes = [C.POINTER(cp), i, C.POINTER(cp), i]
    L.mto_tables_new.restype = vp
    L.mto_tables_free.argtypes = [vp]
    L.mto_apply_packed.argtypes = [vp, vp, l, vp, vp, vp, C.POINTER(cp), i]
    L.mto_gen_doc.argtypes = [C.POINTER(GenParams), l, vp, vp, l, C.POINTER(l), vp, l, C.POINTER(l)]
    L.mto_gen_key_name.argtypes = [i]
    L.mto_gen_key_name.restype = cp
    L.mto_gen_value_json.argtypes = [i]
    L.mto_gen_value_json.restype = cp
    L.mto_gen_client_name.argtypes = [i]
    L.mto_gen_client_name.restype = cp
    L.mto_replay_batch.argtypes = [vp, vp, l, vp, vp, vp, C.POINTER(cp), i, i, vp, vp]
    L.mto_replay_batch.restype = d
    _lib = L
    return L


def _read(fn, doc) -> str:
    n = fn(doc, None, 0)
    buf = C.create_string_buffer(n + 1)
    fn(doc, buf, n + 1)
    return buf.raw[:n].decode("utf-8")


class Doc:
    """One SharedString replica in the oracle (a merge-tree Client)."""

    def __init__(self):
        self.L = lib()
        self.h = self.L.mto_new()

    def close(self):
        if self.h:
            self.L.mto_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    @property
    def status(self) -> int:
        return self.L.mto_status(self.h)

    @property
    def error(self) -> str:
        return self.L.mto_error(self.h).decode()

    def start_collab(self, long_id: str, min_seq=0, cur_seq=0) -> int:
        return self.L.mto_start_collab(self.h, long_id.encode(), min_seq, cur_seq)

    def load_snapshot(self, blobs, long_id: str = "readonly") -> int:
        """SnapshotLoader: blobs = {"header": .., "body_0": ..} (emit order) or a list."""
        import numpy as np

        vals = list(blobs.values()) if isinstance(blobs, dict) else list(blobs)
        bufs = [v.encode("utf-8", "surrogatepass") if isinstance(v, str) else v for v in vals]
        arr = (C.c_char_p * len(bufs))(*bufs)
        lens = np.array([len(b) for b in bufs], np.int64)
        self._keep = (arr, lens, bufs)
        return self.L.mto_load_snapshot_v1(self.h, arr, lens.ctypes.data, len(bufs), long_id.encode())

    def apply_msg(self, msg_json: str) -> int:
        return self.L.mto_apply_msg_json(self.h, msg_json.encode())

    def insert_local(self, pos: int, seg_json: str) -> int:
        return self.L.mto_insert_local_json(self.h, pos, seg_json.encode())

    def annotate_local(self, start: int, end: int, props_json: str) -> int:
        return self.L.mto_annotate_local_json(self.h, start, end, props_json.encode())

    def remove_local(self, start: int, end: int) -> int:
        return self.L.mto_remove_local(self.h, start, end)

    def local_op(self, op, notify: bool = False) -> int:
        """A local IMergeTreeOp of a collaborating replica (pending until its own message acks it);
        notify: the op came from Client.annotateMarkerNotifyConsensus (registers its marker id)."""
        import json as _json

        return self.L.mto_local_op_notify_json(self.h, (op if isinstance(op, str) else _json.dumps(op)).encode(),
                                               1 if notify else 0)

    def local_marker_pos(self, marker_id) -> int:
        """The local position of the marker `marker_id` names (-1: none, or removed locally)."""
        import json as _json

        return self.L.mto_local_marker_pos(self.h, _json.dumps(marker_id).encode())

    def consensus_events(self) -> list:
        """The consensus callbacks made so far, in call order: [{"markerId", "seq", "minSeq"}]."""
        import json as _json

        p = self.L.mto_consensus_events(self.h)
        try:
            return _json.loads(C.string_at(p).decode())
        finally:
            self.L.mto_free_string(p)

    def pending_groups(self) -> int:
        return self.L.mto_pending_groups(self.h)

    def regenerate(self, op):
        """Client.regeneratePendingOp(op, oldest pending group): the regenerated op (a dict)."""
        import json as _json

        out = C.c_void_p()
        rc = self.L.mto_regenerate_pending_op_json(self.h, (op if isinstance(op, str) else _json.dumps(op)).encode(),
                                                   C.byref(out))
        if rc != 0:
            raise RuntimeError(self.error)
        r = _json.loads(C.string_at(out.value).decode())
        self.L.mto_free_string(out)
        return r

    def regenerated_ops(self) -> list:
        import json as _json

        return _json.loads(_read(self.L.mto_regenerated_ops, self.h))

    def find_tile(self, start_pos: int, label: str, preceding: bool = True):
        """MergeTree.findTile for the local client: None, or {"pos", "props"}; raises on a label
        list the reference could not iterate."""
        import json as _json

        pj = C.c_void_p()
        pos = self.L.mto_find_tile(self.h, start_pos, label.encode(), 1 if preceding else 0, C.byref(pj))
        props = None
        if pj.value:
            props = _json.loads(C.string_at(pj.value).decode())
            self.L.mto_free_string(pj)
        if pos == -2:
            raise ValueError("unsupported tile labels")
        return None if pos < 0 else {"pos": pos, "props": props}

    def stack_context(self, start_pos: int, labels) -> dict:
        """MergeTree.getStackContext for the local client (client.ts:946-948): {label: [{"pos",
        "refType"[, "props"]}, ...]} in JS key order; raises on a range label list the reference
        could not iterate."""
        import json as _json

        arr = (C.c_char_p * max(1, len(labels)))(*[l.encode() for l in labels])
        st = C.c_int(0)
        p = self.L.mto_stack_context(self.h, start_pos, arr, len(labels), C.byref(st))
        if not p:
            raise ValueError("unsupported range labels")
        try:
            return _json.loads(C.string_at(p).decode(), object_pairs_hook=lambda kv: dict(kv))
        finally:
            self.L.mto_free_string(p)

    def length(self) -> int:
        return self.L.mto_get_length(self.h)

    def view_length(self, ref_seq: int, short_client: int) -> int:
        return self.L.mto_view_length(self.h, ref_seq, short_client)

    def text(self) -> str:
        return _read(self.L.mto_get_text, self.h)

    def props_runs(self) -> str:
        return _read(self.L.mto_props_runs, self.h)

    def shape(self) -> str:
        return _read(self.L.mto_shape, self.h)

    def dump(self) -> str:
        return _read(self.L.mto_dump, self.h)

    def digest(self) -> int:
        return int(self.L.mto_state_digest(self.h))

    def snapshot_v1(self, chunk_size: int = 0) -> dict[str, str]:
        n = self.L.mto_snapshot_v1(self.h, chunk_size)
        out = {}
        for i in range(n):
            name = C.create_string_buffer(64)
            size = self.L.mto_snapshot_blob(self.h, i, name, 64, None, 0)
            buf = C.create_string_buffer(size + 1)
            self.L.mto_snapshot_blob(self.h, i, name, 64, buf, size + 1)
            out[name.value.decode()] = buf.raw[:size].decode("utf-8")
        return out


def _cstr_array(strs):
    arr = (C.c_char_p * max(1, len(strs)))()
    for k, s in enumerate(strs):
        arr[k] = None if s is None else s.encode()
    return arr


class Tables:
    def __init__(self, keys, values):
        self.L = lib()
        self._k = _cstr_array(keys)
        self._v = _cstr_array(values)
        self.h = self.L.mto_tables_new(self._k, len(keys), self._v, len(values))

    def __del__(self):
        if self.h:
            self.L.mto_tables_free(self.h)
            self.h = None


def gen_tables() -> Tables:
    L = lib()
    keys = [L.mto_gen_key_name(k).decode() for k in range(4)]
    values = [L.mto_gen_value_json(v).decode() for v in range(22)]
    return Tables(keys, values)


def gen_client_names(n_clients: int) -> list[str]:
    L = lib()
    return [L.mto_gen_client_name(i).decode() for i in range(n_clients + 1)]


def gen_params(n_ops, n_clients=8, max_lag=32, pct_insert=60, pct_remove=40, min_len=4, max_insert=8,
               pct_newline=2, seed=0xDEADBEEF):
    return GenParams(n_ops, n_clients, max_lag, pct_insert, pct_remove, min_len, max_insert, pct_newline, seed)


def gen_doc(p: GenParams, doc: int):
    """Generate one document's log with the oracle generator.  Returns (ops, text u16, props)."""
    L = lib()
    ops = np.zeros(p.n_ops, OP_DTYPE)
    text_cap = p.n_ops * max(1, p.max_insert) + 16
    text = np.zeros(text_cap, np.uint16)
    props = np.zeros(2 * p.n_ops + 16, PROP_DTYPE)
    tl, npr = C.c_long(0), C.c_long(0)
    st = L.mto_gen_doc(C.byref(p), doc, ops.ctypes.data, text.ctypes.data, text_cap, C.byref(tl),
                       props.ctypes.data, len(props), C.byref(npr))
    if st != 0:
        raise RuntimeError(f"oracle generator failed with status {st}")
    return ops, text[: tl.value].copy(), props[: npr.value].copy()


def gen_batch(p: GenParams, n_docs: int, first_doc: int = 0, doc_ids=None, doc_ops=None, doc_params=None):
    """Concatenate generated docs with absolute offsets (the C-ABI batch layout).  doc_ids /
    doc_ops: per-document global indices and op counts (mt_batch_generate_docs); doc_params:
    per-document GenParams (mixed batches)."""
    all_ops, all_text, all_props, off = [], [], [], [0]
    t_base = p_base = 0
    ids = list(doc_ids) if doc_ids is not None else list(range(first_doc, first_doc + n_docs))
    for j, dd in enumerate(ids):
        pj = p
        if doc_ops is not None:
            pj = GenParams(*[getattr(p, f) for f, _ in GenParams._fields_])
            pj.n_ops = int(doc_ops[j])
        if doc_params is not None:
            pj = doc_params[j]
        ops, text, props = gen_doc(pj, int(dd))
        ins = (ops["tc"] & 0xF) == 0
        ops["payload"][ins] += t_base
        ann = (ops["tc"] & 0xF) == 2
        ops["payload"][ann] += p_base
        all_ops.append(ops)
        all_text.append(text)
        all_props.append(props)
        t_base += len(text)
        p_base += len(props)
        off.append(off[-1] + len(ops))
    return (np.concatenate(all_ops), np.concatenate(all_text) if all_text else np.zeros(0, np.uint16),
            np.concatenate(all_props) if all_props else np.zeros(0, PROP_DTYPE), np.array(off, np.int64))


def replay_doc(ops, text, props, tables: Tables, client_names) -> Doc:
    d = Doc()
    names = _cstr_array(client_names)
    d._names = names
    t = text if len(text) else np.zeros(1, np.uint16)
    pr = props if len(props) else np.zeros(1, PROP_DTYPE)
    d.L.mto_apply_packed(d.h, ops.ctypes.data, len(ops), t.ctypes.data, pr.ctypes.data, tables.h, names,
                         len(client_names))
    return d


def replay_batch(ops, off, text, props, tables: Tables, client_names, n_threads=None):
    L = lib()
    n_docs = len(off) - 1
    dig = np.zeros(n_docs, np.uint64)
    st = np.zeros(n_docs, np.int32)
    names = _cstr_array(client_names)
    t = text if len(text) else np.zeros(1, np.uint16)
    pr = props if len(props) else np.zeros(1, PROP_DTYPE)
    n_threads = n_threads or os.cpu_count() or 1
    secs = L.mto_replay_batch(ops.ctypes.data, off.ctypes.data, n_docs, t.ctypes.data, pr.ctypes.data, tables.h,
                              names, len(client_names), n_threads, dig.ctypes.data, st.ctypes.data)
    return secs, dig, st
