"""Python host layer over libmtreplay.so (include/mtreplay.h).

Mirrors the reference's per-document surface so tests read like the reference's own:

    reference (packages/dds/merge-tree/src, sequence/src)      here
    ------------------------------------------------------      ---------------------------------
    new Client(...); client.startOrUpdateCollaboration(id)      ReplayBatch(n_docs, observer=id)
    client.applyMsg(msg) for msg in log                         batch.ingest_messages(logs); batch.run()
    client.insertTextLocal / removeRangeLocal / annotateRange-  {"sequenceNumber": -1, ...} entries of a
      Local, then applyMsg(own sequenced msg) (ack)               writer's log: ingest_messages(logs, observer=[ids])
    sharedString.getText()                                      batch.doc(i).get_text()
    client.getPropertiesAtPosition(pos)                         batch.doc(i).get_properties_at_position(pos)
    new SnapshotV1(mt, logger).extractSync(); emit()            batch.doc(i).snapshot_v1()
    thrown Error from applyMsg                                  batch.doc(i).status (MT_* code)

Every op is applied by the HIP kernel; this module only marshals.  Loading fails loudly
when the compiled library is missing or no GPU is present (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes as C
import json
import os
from pathlib import Path

import numpy as np

from .oplog import OP_DTYPE, PROP_DTYPE, PackedBatch, Packer

LIB_PATH = Path(os.environ.get("FLUIDFRAMEWORK_AMD_LIB") or Path(__file__).resolve().parent / "libmtreplay.so")
ABI_VERSION = 8  # include/mtreplay.h MT_ABI_VERSION

MT_OK, MT_INVALID_POS, MT_SEQ_ORDER, MT_MSN_ORDER, MT_UNSUPPORTED, MT_BAD_INPUT, MT_CAPACITY, MT_INTERNAL = range(8)
MT_ERR_HIP, MT_ERR_ARG, MT_ERR_STATE, MT_ERR_NO_DEVICE = 100, 101, 102, 103

# every entry point declared in include/mtreplay.h
EXPORTS = [
    "mt_status_string", "mt_batch_create", "mt_batch_destroy", "mt_batch_set_tables", "mt_batch_set_clients",
    "mt_batch_ingest", "mt_batch_generate", "mt_batch_run", "mt_batch_launch", "mt_batch_sync",
    "mt_batch_get_stats", "mt_batch_algorithmic_bytes", "mt_doc_status", "mt_doc_text", "mt_doc_props_runs",
    "mt_doc_snapshot_v1", "mt_doc_snapshot_blob", "mt_doc_digest", "mt_doc_shape", "mt_doc_dump", "mt_batch_log_sizes",
    "mt_batch_download_log", "mt_batch_doc_counters", "mt_batch_device_digests", "mt_batch_snapshots",
    "mt_doc_snapshot_v1_device", "mt_batch_snapshot_index", "mt_batch_snapshot_copy", "mt_batch_launch_info",
    "mt_batch_snapshot_digests", "mt_batch_generate_docs", "mt_pack_json", "mt_packed_destroy", "mt_packed_error",
    "mt_packed_sizes", "mt_packed_arrays", "mt_packed_key", "mt_packed_value", "mt_packed_doc_clients",
    "mt_packed_client", "mt_batch_ingest_packed", "mt_batch_log_sizes_docs", "mt_batch_download_log_docs",
    "mt_build_id", "mt_abi_version", "mt_doc_find_tile", "mt_doc_regenerated_ops", "mt_pack_json_gpu", "mt_batch_ingest_json_gpu",
    "mt_doc_stack_context", "mt_doc_consensus_events",
]
SNAP_MAX_BLOBS = 32
SNAP_META = 1 + 3 * SNAP_MAX_BLOBS
DOC_COUNTERS = ("status", "min_seq", "cur_seq", "depth", "n_entries", "text_top", "pool_top", "ops_done",
                "max_unsettled", "max_slots", "max_blocks", "max_heap", "fail_op", "cap_kind", "launch", "reserved")


class MtError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: {status_string(code)} ({code})")
        self.code = code


class JsonGpuStats(C.Structure):
    """mt_json_gpu_stats (include/mtreplay.h)"""

    _fields_ = [("ms_scan", C.c_double), ("ms_count", C.c_double), ("ms_clients", C.c_double),
                ("ms_write", C.c_double), ("ms_props", C.c_double), ("ms_host", C.c_double),
                ("ms_total", C.c_double), ("n_msgs", C.c_int64), ("n_ops", C.c_int64), ("n_text", C.c_int64),
                ("n_props", C.c_int64), ("fail_bits", C.c_uint32), ("reserved", C.c_int32)]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved"}


class NotOnGpuPath(RuntimeError):
    """A JSON batch outside the GPU parser's fast path (mt_json_gpu.h): use the host parser."""

    def __init__(self, bad_doc: int, fail_bits: int):
        super().__init__(f"document {bad_doc} needs the host JSON parser (reasons 0x{fail_bits:x})")
        self.bad_doc = bad_doc
        self.fail_bits = fail_bits


class GenParams(C.Structure):
    """mt_gen_params (include/mt_gen.h)"""

    _fields_ = [("n_ops", C.c_int32), ("n_clients", C.c_int32), ("max_lag", C.c_int32),
                ("pct_insert", C.c_int32), ("pct_remove", C.c_int32), ("min_len", C.c_int32),
                ("max_insert", C.c_int32), ("pct_newline", C.c_int32), ("seed", C.c_uint64)]


class BatchOptions(C.Structure):
    _fields_ = [("chunk_size", C.c_int32), ("seg_cap", C.c_int32),
                ("arena_factor", C.c_int32), ("pool_per_op", C.c_int32),
                ("max_retries", C.c_int32)]


class LaunchInfo(C.Structure):
    _fields_ = [("seg_class", C.c_int32), ("n_docs", C.c_int32), ("resumed", C.c_int32), ("lds_bytes", C.c_int32),
                ("ms", C.c_float), ("start_ms", C.c_float), ("ops", C.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class BatchStats(C.Structure):
    _fields_ = [("n_docs", C.c_int64), ("n_ops", C.c_int64), ("ops_applied", C.c_int64),
                ("docs_failed", C.c_int64), ("max_oe", C.c_int32), ("max_slots", C.c_int32),
                ("max_blocks", C.c_int32), ("max_heap", C.c_int32), ("lds_bytes", C.c_int32),
                ("launches", C.c_int32), ("kernel_ms", C.c_float), ("total_ms", C.c_float),
                ("lds_class", C.c_int32), ("reserved", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# the generator's key / value / client tables (include/mt_gen.h MT_GEN_N_KEYS, MT_GEN_N_VALUES)
GEN_KEYS = ["bold", "italic", "color", "size"]
GEN_VALUES = ["null", "true", '"red"', '"green"', '"blue"'] + [str(v) for v in range(8, 25)]


def gen_client_names(n_clients: int) -> list:
    """short id 0 = the observer "readonly", 1.. = "A", "B", .. (mt_gen.h)"""
    return ["readonly"] + [chr(ord("A") + i) for i in range(n_clients)]


def gen_params(n_ops, n_clients=8, max_lag=32, pct_insert=60, pct_remove=40, min_len=4, max_insert=8,
               pct_newline=2, seed=0xDEADBEEF) -> GenParams:
    return GenParams(n_ops, n_clients, max_lag, pct_insert, pct_remove, min_len, max_insert, pct_newline, seed)


_lib = None


def lib():
    """Load libmtreplay.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise FileNotFoundError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(str(LIB_PATH))
    vp, i32, i64, cp = C.c_void_p, C.c_int32, C.c_int64, C.c_char_p
    P = C.POINTER
    L.mt_build_id.argtypes = []
    L.mt_build_id.restype = cp
    # the in-tree library must have been built from the sources next to it (buildinfo.py); a stale
    # binary is refused rather than tested (FLUIDFRAMEWORK_AMD_LIB overrides skip the check)
    from . import buildinfo
    if not os.environ.get("FLUIDFRAMEWORK_AMD_LIB") and buildinfo.sources_present():
        want, got = buildinfo.src_hash(), L.mt_build_id().decode()
        if got != want:
            raise RuntimeError(f"{LIB_PATH} was built from other sources (build id {got}, sources {want}): "
                               "rebuild with __graft_entry__.build()")
    L.mt_abi_version.argtypes = []
    L.mt_abi_version.restype = C.c_int32
    if L.mt_abi_version() != ABI_VERSION:  # struct layouts below are those of include/mtreplay.h v8
        raise RuntimeError(f"{LIB_PATH}: C ABI version {L.mt_abi_version()}, this binding speaks {ABI_VERSION}")
    L.mt_status_string.argtypes = [C.c_int]
    L.mt_status_string.restype = cp
    L.mt_batch_create.argtypes = [P(vp), i64, P(BatchOptions)]
    L.mt_batch_destroy.argtypes = [vp]
    L.mt_batch_destroy.restype = None
    L.mt_batch_set_tables.argtypes = [vp, P(cp), i32, P(cp), i32]
    L.mt_batch_set_clients.argtypes = [vp, i64, P(cp), i32]
    L.mt_batch_ingest.argtypes = [vp, vp, vp, vp, i64, vp, i64]
    L.mt_batch_generate.argtypes = [vp, P(GenParams), i64]
    L.mt_batch_generate_docs.argtypes = [vp, P(GenParams), vp, vp]
    L.mt_pack_json.argtypes = [P(vp), i64, vp, vp, cp, i32, P(i64)]
    L.mt_packed_destroy.argtypes = [vp]
    L.mt_packed_destroy.restype = None
    L.mt_packed_error.argtypes = [vp]
    L.mt_packed_error.restype = cp
    L.mt_packed_sizes.argtypes = [vp, P(i64), P(i64), P(i64), P(i32), P(i32)]
    L.mt_packed_arrays.argtypes = [vp, vp, vp, vp, vp]
    for fn in ("mt_packed_key", "mt_packed_value"):
        getattr(L, fn).argtypes = [vp, i32]
        getattr(L, fn).restype = cp
    L.mt_packed_doc_clients.argtypes = [vp, i64]
    L.mt_packed_doc_clients.restype = i32
    L.mt_packed_client.argtypes = [vp, i64, i32]
    L.mt_packed_client.restype = cp
    L.mt_batch_ingest_packed.argtypes = [vp, vp]
    L.mt_pack_json_gpu.argtypes = [P(vp), i64, vp, vp, cp, P(i64), P(JsonGpuStats)]
    L.mt_batch_ingest_json_gpu.argtypes = [vp, vp, vp, i64, vp, cp, P(i64), P(JsonGpuStats)]
    L.mt_batch_run.argtypes = [vp, vp]
    L.mt_batch_launch.argtypes = [vp, vp]
    L.mt_batch_sync.argtypes = [vp]
    L.mt_batch_get_stats.argtypes = [vp, P(BatchStats)]
    L.mt_batch_algorithmic_bytes.argtypes = [vp, P(C.c_double)]
    L.mt_doc_status.argtypes = [vp, i64]
    L.mt_doc_status.restype = i32
    for fn in ("mt_doc_text", "mt_doc_props_runs", "mt_doc_shape", "mt_doc_dump", "mt_doc_regenerated_ops",
               "mt_doc_consensus_events"):
        getattr(L, fn).argtypes = [vp, i64, C.c_char_p, i64, P(i64)]
    L.mt_doc_snapshot_v1.argtypes = [vp, i64, P(i32)]
    L.mt_doc_snapshot_blob.argtypes = [vp, i64, i32, C.c_char_p, i64, C.c_char_p, i64, P(i64)]
    L.mt_doc_digest.argtypes = [vp, i64, P(C.c_uint64)]
    L.mt_batch_log_sizes.argtypes = [vp, P(i64), P(i64), P(i64)]
    L.mt_batch_download_log.argtypes = [vp, vp, vp, vp, vp]
    L.mt_batch_log_sizes_docs.argtypes = [vp, i64, i64, P(i64), P(i64), P(i64)]
    L.mt_batch_download_log_docs.argtypes = [vp, i64, i64, vp, vp, vp, vp]
    L.mt_batch_doc_counters.argtypes = [vp, vp]
    L.mt_batch_device_digests.argtypes = [vp, vp, i32]
    L.mt_batch_launch_info.argtypes = [vp, i32, P(LaunchInfo)]
    L.mt_batch_snapshots.argtypes = [vp, P(i64), P(C.c_float)]
    L.mt_doc_snapshot_v1_device.argtypes = [vp, i64, P(i32)]
    L.mt_batch_snapshot_index.argtypes = [vp, vp, vp]
    L.mt_batch_snapshot_copy.argtypes = [vp, vp, i32]
    L.mt_batch_snapshot_digests.argtypes = [vp, vp, i32]
    L.mt_doc_find_tile.argtypes = [vp, i64, i64, cp, i32, P(i64), C.c_char_p, i64, P(i64)]
    L.mt_doc_stack_context.argtypes = [vp, i64, i64, P(cp), i32, C.c_char_p, i64, P(i64)]
    _lib = L
    return L


def status_string(code: int) -> str:
    return lib().mt_status_string(code).decode()


def _chk(rc: int, what: str):
    if rc != MT_OK:
        raise MtError(rc, what)


def _cstrs(strs):
    arr = (C.c_char_p * max(1, len(strs)))()
    for k, s in enumerate(strs):
        arr[k] = s.encode("utf-8", "surrogatepass")  # WTF-8: lone surrogates survive
    return arr


def json_concat(docs):
    """Documents (JSON text / bytes / message lists) back to back: (bytes, doc_off int64[D + 1])."""
    bufs = [d if isinstance(d, bytes) else (d if isinstance(d, str) else json.dumps(d)).encode("utf-8",
                                                                                          "surrogatepass")
            for d in docs]
    off = np.zeros(len(bufs) + 1, np.int64)
    if bufs:
        off[1:] = np.cumsum([len(x) for x in bufs])
    return b"".join(bufs), off


class PackedJson:
    """Native JSON ingest result (mt_pack_json): ISequencedDocumentMessage logs parsed and packed
    on host threads, with the packing rules of oplog.Packer."""

    def __init__(self, docs, observer: str = "readonly", n_threads: int = 0):
        bufs = [d if isinstance(d, bytes) else (d if isinstance(d, str) else json.dumps(d)).encode("utf-8",
                                                                                              "surrogatepass")
                for d in docs]
        n = len(bufs)
        ptrs = (C.c_char_p * max(1, n))(*bufs)
        lens = np.array([len(x) for x in bufs] or [0], np.int64)
        h, bad = C.c_void_p(), C.c_int64(-1)
        rc = lib().mt_pack_json(C.byref(h), n, ptrs, lens.ctypes.data, observer.encode("utf-8"), n_threads,
                                C.byref(bad))
        self.h = h
        self.n_docs = n
        if rc != MT_OK:
            err = lib().mt_packed_error(h).decode("utf-8", "replace") if h else ""
            self.close()
            raise MtError(rc, f"mt_pack_json: {err}")

    def close(self):
        if self.h:
            lib().mt_packed_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def arrays(self):
        """PackedBatch (oplog.py) view: ops, doc_op_off, text, props, keys, values, clients."""
        L = lib()
        no, nt, npr, nk, nv = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int32(), C.c_int32()
        _chk(L.mt_packed_sizes(self.h, C.byref(no), C.byref(nt), C.byref(npr), C.byref(nk), C.byref(nv)), "sizes")
        ops = np.zeros(no.value, OP_DTYPE)
        off = np.zeros(self.n_docs + 1, np.int64)
        text = np.zeros(max(1, nt.value), np.uint16)
        props = np.zeros(max(1, npr.value), PROP_DTYPE)
        _chk(L.mt_packed_arrays(self.h, ops.ctypes.data, off.ctypes.data, text.ctypes.data, props.ctypes.data),
             "arrays")
        dec = lambda b: b.decode("utf-8", "surrogatepass")  # noqa: E731  (WTF-8)
        keys = [dec(L.mt_packed_key(self.h, i)) for i in range(nk.value)]
        values = [dec(L.mt_packed_value(self.h, i)) for i in range(nv.value)]
        clients = [[dec(L.mt_packed_client(self.h, d, i)) for i in range(L.mt_packed_doc_clients(self.h, d))]
                   for d in range(self.n_docs)]
        return PackedBatch(ops=ops, doc_op_off=off, text=text[: nt.value], props=props[: npr.value], keys=keys,
                           values=values, clients=clients)


class PackedJsonGpu(PackedJson):
    """The same packed result from the GPU parser (mt_pack_json_gpu, mt_json_gpu.hip); raises
    NotOnGpuPath for a batch outside its fast path."""

    def __init__(self, docs, observer: str = "readonly"):
        buf, off = json_concat(docs)
        h, bad, st = C.c_void_p(), C.c_int64(-1), JsonGpuStats()
        rc = lib().mt_pack_json_gpu(C.byref(h), len(off) - 1, buf, off.ctypes.data, observer.encode("utf-8"),
                                    C.byref(bad), C.byref(st))
        self.h = h if rc == MT_OK else None
        self.n_docs = len(off) - 1
        self.stats = st.as_dict()
        if rc == MT_UNSUPPORTED:
            raise NotOnGpuPath(bad.value, st.fail_bits)
        if rc != MT_OK:
            raise MtError(rc, "mt_pack_json_gpu")


class DocView:
    """Read-out of one replayed document (a merge-tree Client after its last applyMsg)."""

    def __init__(self, batch: "ReplayBatch", index: int):
        self.batch, self.index = batch, index

    @property
    def status(self) -> int:
        return int(lib().mt_doc_status(self.batch.h, self.index))

    def _string(self, fn) -> str:
        n = C.c_int64(0)
        _chk(fn(self.batch.h, self.index, None, 0, C.byref(n)), fn.__name__)
        buf = C.create_string_buffer(n.value + 1)
        _chk(fn(self.batch.h, self.index, buf, n.value + 1, C.byref(n)), fn.__name__)
        return buf.raw[: n.value].decode("utf-8")

    def get_text(self) -> str:
        return self._string(lib().mt_doc_text)

    def props_runs(self) -> list:
        return json.loads(self._string(lib().mt_doc_props_runs))

    def get_properties_at_position(self, pos: int):
        for start, length, props in self.props_runs():
            if start <= pos < start + length:
                return None if props is None else json.loads(props)
        return None

    def find_tile(self, start_pos: int, label: str, preceding: bool = True):
        """Client.findTile(startPos, tileLabel, preceding) (client.ts:1073-1076): None when there is
        no tile, else {"pos": .., "props": marker properties}."""
        L = lib()
        pos, n = C.c_int64(-1), C.c_int64(0)
        args = (self.batch.h, self.index, start_pos, label.encode("utf-8"), 1 if preceding else 0, C.byref(pos))
        _chk(L.mt_doc_find_tile(*args, None, 0, C.byref(n)), "mt_doc_find_tile")
        if pos.value < 0:
            return None
        buf = C.create_string_buffer(n.value + 1)
        _chk(L.mt_doc_find_tile(*args, buf, n.value + 1, C.byref(n)), "mt_doc_find_tile")
        raw = buf.raw[: n.value].decode("utf-8")
        return {"pos": pos.value, "props": json.loads(raw) if raw else None}

    def get_stack_context(self, start_pos: int, range_labels) -> dict:
        """Client.getStackContext(startPos, rangeLabels) (client.ts:946-948; SharedSegmentSequence
        .getStackContext, sequence.ts:377): {label: [{"pos", "refType"[, "props"]}, ...]}, each stack
        bottom to top, keys in JS object order."""
        L = lib()
        labels = list(range_labels)
        arr = (C.c_char_p * max(1, len(labels)))(*[l.encode("utf-8") for l in labels])
        n = C.c_int64(0)
        args = (self.batch.h, self.index, start_pos, arr, len(labels))
        _chk(L.mt_doc_stack_context(*args, None, 0, C.byref(n)), "mt_doc_stack_context")
        buf = C.create_string_buffer(n.value + 1)
        _chk(L.mt_doc_stack_context(*args, buf, n.value + 1, C.byref(n)), "mt_doc_stack_context")
        return json.loads(buf.raw[: n.value].decode("utf-8"))

    def regenerated_ops(self) -> list:
        """Client.regeneratePendingOp results of the log's reconnect (regenerate) records, in order."""
        return json.loads(self._string(lib().mt_doc_regenerated_ops))

    def consensus_events(self) -> list:
        """The consensus callbacks of a writer replica (annotateMarkerNotifyConsensus), in call
        order: [{"markerId", "seq", "minSeq"}, ...]."""
        return json.loads(self._string(lib().mt_doc_consensus_events))

    def shape(self) -> str:
        return self._string(lib().mt_doc_shape)

    def dump(self) -> str:
        return self._string(lib().mt_doc_dump)

    def digest(self) -> int:
        out = C.c_uint64(0)
        _chk(lib().mt_doc_digest(self.batch.h, self.index, C.byref(out)), "mt_doc_digest")
        return int(out.value)

    def snapshot_v1(self, device: bool = False) -> dict:
        """{blob path: JSON} of SnapshotV1.  device=True: the blobs ReplayBatch.snapshots()
        serialized on the GPU; False: the host serializer over the same final table."""
        L = lib()
        n = C.c_int32(0)
        if device:
            _chk(L.mt_doc_snapshot_v1_device(self.batch.h, self.index, C.byref(n)), "mt_doc_snapshot_v1_device")
        else:
            _chk(L.mt_doc_snapshot_v1(self.batch.h, self.index, C.byref(n)), "mt_doc_snapshot_v1")
        out = {}
        for i in range(n.value):
            name = C.create_string_buffer(64)
            size = C.c_int64(0)
            _chk(L.mt_doc_snapshot_blob(self.batch.h, self.index, i, name, 64, None, 0, C.byref(size)), "blob")
            buf = C.create_string_buffer(size.value + 1)
            _chk(L.mt_doc_snapshot_blob(self.batch.h, self.index, i, name, 64, buf, size.value + 1, C.byref(size)),
                 "blob")
            out[name.value.decode()] = buf.raw[: size.value].decode("utf-8")
        return out


class ReplayBatch:
    """A batch of SharedString documents replayed on one MI355X (the current HIP device)."""

    def __init__(self, n_docs: int, **options):
        self.n_docs = int(n_docs)
        opts = BatchOptions(**options)
        h = C.c_void_p()
        _chk(lib().mt_batch_create(C.byref(h), self.n_docs, C.byref(opts)), "mt_batch_create")
        self.h = h
        self._keep = []

    def close(self):
        if getattr(self, "h", None):
            lib().mt_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- input
    def set_tables(self, keys, values):
        k, v = _cstrs(keys), _cstrs(values)
        self._keep += [k, v]
        _chk(lib().mt_batch_set_tables(self.h, k, len(keys), v, len(values)), "mt_batch_set_tables")

    def set_clients(self, names, doc: int = -1):
        a = _cstrs(names)
        _chk(lib().mt_batch_set_clients(self.h, doc, a, len(names)), "mt_batch_set_clients")

    def ingest(self, ops, doc_op_off, text, props):
        ops = np.ascontiguousarray(ops, OP_DTYPE)
        off = np.ascontiguousarray(doc_op_off, np.int64)
        text = np.ascontiguousarray(text if len(text) else np.zeros(1, np.uint16), np.uint16)
        props = np.ascontiguousarray(props if len(props) else np.zeros(1, PROP_DTYPE), PROP_DTYPE)
        if len(off) != self.n_docs + 1:
            raise ValueError("doc_op_off must have n_docs + 1 entries")
        if off[0] != 0 or (len(off) > 1 and (np.diff(off) < 0).any()) or int(off[-1]) > len(ops):
            raise ValueError("doc_op_off must start at 0, be non-decreasing and end within ops")
        _chk(lib().mt_batch_ingest(self.h, ops.ctypes.data, off.ctypes.data, text.ctypes.data, len(text),
                                   props.ctypes.data, len(props)), "mt_batch_ingest")

    def ingest_packed(self, pb: PackedBatch):
        self.set_tables(pb.keys or ["_"], pb.values)
        shared = pb.clients[0] if pb.clients and all(c == pb.clients[0] for c in pb.clients) else None
        if shared is not None:
            self.set_clients(shared)
        else:
            for i, names in enumerate(pb.clients):
                self.set_clients(names, i)
        self.ingest(pb.ops, pb.doc_op_off, pb.text, pb.props)

    def ingest_messages(self, docs, observer="readonly"):
        """docs: one ISequencedDocumentMessage list (dicts or JSON strings) per document.
        observer: the replicas' long id, or one per document (writer replicas: their unsequenced
        messages, sequenceNumber -1, are local ops; their sequenced ones ack them)."""
        reps = [observer] * len(docs) if isinstance(observer, str) else list(observer)
        p = Packer(observer=reps[0] if reps else "readonly")
        for msgs, rep in zip(docs, reps):
            p.add_document(msgs, rep)
        pb = p.finish()
        if len(pb.doc_op_off) != self.n_docs + 1:
            raise ValueError("expected one message list per document")
        self.ingest_packed(pb)
        return pb

    def ingest_json(self, docs, observer: str = "readonly", n_threads: int = 0, device: str = "auto"):
        """Parse + pack JSON message logs natively and ingest them.  docs: per document a JSON
        array text (str/bytes) or a list of message dicts.  device "gpu": the GPU parser
        (mt_batch_ingest_json_gpu; NotOnGpuPath outside its fast path), "host": mt_pack_json on
        host threads, "auto": the GPU parser, the host parser for batches outside its fast path.
        Returns {"path": "gpu" | "host", ...GPU parser stats}."""
        if device not in ("auto", "gpu", "host"):
            raise ValueError("device must be auto, gpu or host")
        info = {"path": "host"}
        if device != "host":
            buf, off = json_concat(docs)
            try:
                info.update(self.ingest_json_gpu(buf, off, observer))
                info["path"] = "gpu"
                return info
            except NotOnGpuPath as e:
                if device == "gpu":
                    raise
                info.update(bad_doc=e.bad_doc, fail_bits=e.fail_bits)
        pj = PackedJson(docs, observer, n_threads)
        try:
            _chk(lib().mt_batch_ingest_packed(self.h, pj.h), "mt_batch_ingest_packed")
        finally:
            pj.close()
        return info

    def ingest_json_gpu(self, buf: bytes, doc_off, observer: str = "readonly", d_json=None) -> dict:
        """GPU JSON ingest of documents back to back in `buf` (doc_off[D + 1]); d_json: the same
        bytes already on the device (a pointer, e.g. a torch uint8 tensor's data_ptr(), 64 bytes
        readable past the end) — the scan / parse stages then read HBM; `buf` is still required and
        must hold the same bytes (key, value and client-name strings are interned from the host
        copy).  Returns the stage timings."""
        off = np.ascontiguousarray(doc_off, np.int64)
        if len(off) != self.n_docs + 1:
            raise ValueError("doc_off must have n_docs + 1 entries")
        bad, st = C.c_int64(-1), JsonGpuStats()
        rc = lib().mt_batch_ingest_json_gpu(self.h, buf, off.ctypes.data, self.n_docs, d_json, observer.encode("utf-8"),
                                            C.byref(bad), C.byref(st))
        if rc == MT_UNSUPPORTED:
            raise NotOnGpuPath(bad.value, st.fail_bits)
        _chk(rc, "mt_batch_ingest_json_gpu")
        return st.as_dict()

    def generate(self, params: GenParams, doc_first: int = 0):
        _chk(lib().mt_batch_generate(self.h, C.byref(params), doc_first), "mt_batch_generate")

    def generate_docs(self, params: GenParams, doc_ids, doc_ops):
        """Generate documents with the given global indices and op counts (params.n_ops unused)."""
        ids = np.ascontiguousarray(doc_ids, np.int64)
        ops = np.ascontiguousarray(doc_ops, np.int32)
        if len(ids) != self.n_docs or len(ops) != self.n_docs:
            raise ValueError("doc_ids / doc_ops must have n_docs entries")
        _chk(lib().mt_batch_generate_docs(self.h, C.byref(params), ids.ctypes.data, ops.ctypes.data),
             "mt_batch_generate_docs")

    # -- run
    def run(self, stream=None):
        _chk(lib().mt_batch_run(self.h, stream), "mt_batch_run")

    def launch(self, stream=None):
        _chk(lib().mt_batch_launch(self.h, stream), "mt_batch_launch")

    def sync(self):
        _chk(lib().mt_batch_sync(self.h), "mt_batch_sync")

    def stats(self) -> dict:
        s = BatchStats()
        _chk(lib().mt_batch_get_stats(self.h, C.byref(s)), "mt_batch_get_stats")
        return s.as_dict()

    def algorithmic_bytes(self) -> float:
        b = C.c_double(0)
        _chk(lib().mt_batch_algorithmic_bytes(self.h, C.byref(b)), "mt_batch_algorithmic_bytes")
        return b.value

    def doc(self, i: int) -> DocView:
        if not 0 <= i < self.n_docs:
            raise IndexError(i)
        return DocView(self, i)

    def counters(self) -> np.ndarray:
        """Per-document run counters (mt_batch_doc_counters) as a structured array."""
        a = np.zeros((self.n_docs, len(DOC_COUNTERS)), np.int32)
        _chk(lib().mt_batch_doc_counters(self.h, a.ctypes.data), "doc counters")
        return np.rec.fromarrays(a.T, names=list(DOC_COUNTERS))

    def device_digests(self, out=None):
        """Per-document 8-byte device digests of the last run (mt_batch_device_digests).
        out: None -> numpy uint64 array; a torch int64 CUDA tensor of n_docs -> filled in place."""
        if out is None:
            a = np.zeros(self.n_docs, np.uint64)
            _chk(lib().mt_batch_device_digests(self.h, a.ctypes.data, 0), "mt_batch_device_digests")
            return a
        if out.numel() != self.n_docs or out.element_size() != 8 or not out.is_contiguous():
            raise ValueError("out must be a contiguous 8-byte tensor of n_docs elements")
        _chk(lib().mt_batch_device_digests(self.h, out.data_ptr(), 1 if out.is_cuda else 0), "mt_batch_device_digests")
        return out

    def launches(self) -> list:
        """Per-launch info of the last run (mt_batch_launch_info): class, docs, resumed, ms, ops."""
        out = []
        for i in range(self.stats()["launches"]):
            li = LaunchInfo()
            _chk(lib().mt_batch_launch_info(self.h, i, C.byref(li)), "mt_batch_launch_info")
            out.append(li.as_dict())
        return out

    def snapshots(self) -> dict:
        """SnapshotV1 of every document serialized on the GPU (mt_batch_snapshots).  Returns
        {"bytes": total, "device_ms": both passes}; read back with doc(i).snapshot_v1(device=True)
        or snapshot_buffer()."""
        total, ms = C.c_int64(0), C.c_float(0)
        _chk(lib().mt_batch_snapshots(self.h, C.byref(total), C.byref(ms)), "mt_batch_snapshots")
        return {"bytes": int(total.value), "device_ms": float(ms.value)}

    def snapshot_digests(self, out=None):
        """Per-document 64-bit digests of the GPU SnapshotV1 bytes (mt_batch_snapshot_digests);
        out: None -> numpy uint64, or a contiguous 8-byte torch tensor of n_docs (filled)."""
        if out is None:
            a = np.zeros(self.n_docs, np.uint64)
            _chk(lib().mt_batch_snapshot_digests(self.h, a.ctypes.data, 0), "mt_batch_snapshot_digests")
            return a
        if out.numel() != self.n_docs or out.element_size() != 8 or not out.is_contiguous():
            raise ValueError("out must be a contiguous 8-byte tensor of n_docs elements")
        _chk(lib().mt_batch_snapshot_digests(self.h, out.data_ptr(), 1 if out.is_cuda else 0),
             "mt_batch_snapshot_digests")
        return out

    def snapshot_index(self):
        """(doc_off[n_docs+1], meta[n_docs, SNAP_META]) of the last snapshots() call."""
        off = np.zeros(self.n_docs + 1, np.int64)
        meta = np.zeros((self.n_docs, SNAP_META), np.int32)
        _chk(lib().mt_batch_snapshot_index(self.h, off.ctypes.data, meta.ctypes.data), "mt_batch_snapshot_index")
        return off, meta

    def snapshot_copy(self, out):
        """Copy the last snapshots() buffer into `out`: a contiguous uint8 torch tensor (CUDA: device
        to device) or numpy array of at least doc_off[-1] bytes."""
        if hasattr(out, "data_ptr"):
            if out.element_size() != 1 or not out.is_contiguous():
                raise ValueError("out must be a contiguous uint8 tensor")
            _chk(lib().mt_batch_snapshot_copy(self.h, out.data_ptr(), 1 if out.is_cuda else 0),
                 "mt_batch_snapshot_copy")
        else:
            _chk(lib().mt_batch_snapshot_copy(self.h, out.ctypes.data, 0), "mt_batch_snapshot_copy")
        return out

    def snapshot_buffer(self):
        """(bytes, doc_off[n_docs+1], meta[n_docs, SNAP_META]) of the last snapshots() call."""
        off = np.zeros(self.n_docs + 1, np.int64)
        meta = np.zeros((self.n_docs, SNAP_META), np.int32)
        _chk(lib().mt_batch_snapshot_index(self.h, off.ctypes.data, meta.ctypes.data), "mt_batch_snapshot_index")
        buf = np.zeros(max(1, int(off[-1])), np.uint8)
        _chk(lib().mt_batch_snapshot_copy(self.h, buf.ctypes.data, 0), "mt_batch_snapshot_copy")
        return buf[: int(off[-1])].tobytes(), off, meta

    def statuses(self) -> np.ndarray:
        L = lib()
        return np.array([L.mt_doc_status(self.h, i) for i in range(self.n_docs)], np.int32)

    def download_log(self, d0: int = 0, d1: int | None = None):
        """(ops, doc_op_off, text, props) of documents [d0, d1) (default: all) as a standalone log:
        offsets from 0, their texts back to back, prop records with batch-global offsets."""
        L = lib()
        d1 = self.n_docs if d1 is None else d1
        n_ops, n_text, n_props = C.c_int64(), C.c_int64(), C.c_int64()
        _chk(L.mt_batch_log_sizes_docs(self.h, d0, d1, C.byref(n_ops), C.byref(n_text), C.byref(n_props)),
             "log sizes")
        ops = np.zeros(n_ops.value, OP_DTYPE)
        off = np.zeros(d1 - d0 + 1, np.int64)
        text = np.zeros(max(1, n_text.value), np.uint16)
        props = np.zeros(max(1, n_props.value), PROP_DTYPE)
        _chk(L.mt_batch_download_log_docs(self.h, d0, d1, ops.ctypes.data, off.ctypes.data, text.ctypes.data,
                                          props.ctypes.data), "mt_batch_download_log_docs")
        return ops, off, text[: n_text.value], props[: n_props.value]
