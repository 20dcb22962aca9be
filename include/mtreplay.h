/*
 * mtreplay.h — C ABI of libmtreplay.so, the MI355X batch replay engine for sequenced
 * merge-tree ops (the drop-in for the reference's Client.applyMsg observer path).
 *
 * Boundary (reference interface each entry point replaces):
 *   mt_batch_create/destroy     new Client(specToSegment, logger, {newMergeTreeSnapshotFormat:true})
 *                               + startOrUpdateCollaboration("readonly") per document
 *                               (merge-tree/src/client.ts:74-83, 1051-1071)
 *   mt_batch_set_clients        Client.getOrAddShortClientId / getLongClientId
 *                               (client.ts:636-652): long ids for short ids 0..n-1
 *   mt_batch_set_tables         property keys/values as they appear in IMergeTreeAnnotateMsg.props /
 *                               IJSONSegment.props (ops.ts:63-97); values are JSON.stringify texts
 *   mt_batch_ingest             the ISequencedDocumentMessage streams Client.applyMsg consumes
 *                               (client.ts:797-819; protocol.ts:132-172), packed (mt_oplog.h)
 *   mt_batch_run / mt_batch_sync
 *                               for each doc: for (msg of log) client.applyMsg(msg)
 *   mt_doc_status               the exception an applyMsg would throw (mergeTree.ts:2210-2216,
 *                               client.ts:461-464, 824-826) as a per-document code
 *   mt_doc_text                 SharedString.getText() (sequence/src/sharedString.ts:211-214 ->
 *                               MergeTreeTextHelper.getText, textSegment.ts:154-172)
 *   mt_doc_find_tile            Client.findTile(startPos, label, preceding) (client.ts:1073-1076)
 *   mt_doc_stack_context        Client.getStackContext(startPos, rangeLabels) (client.ts:946-948)
 *   mt_doc_props_runs           Client.getPropertiesAtPosition(pos) for every pos (client.ts:1009-1023),
 *                               run-length encoded
 *   mt_doc_snapshot_v1/_blob    new SnapshotV1(mergeTree, logger).extractSync(); emit()
 *                               (merge-tree/src/snapshotV1.ts:85-247): blob path + contents
 *   mt_batch_snapshots + mt_doc_snapshot_v1_device / mt_batch_snapshot_index / _copy
 *                               the same SnapshotV1 blobs for every document, serialized on the GPU
 *                               (snapshotV1.ts:85-247 for a whole batch of documents at once)
 *   mt_doc_digest               FNV-1a-64 over the final segment table (DESIGN.md "State digest")
 *   mt_batch_device_digests     8-byte per-document fingerprint of the final state computed on the
 *                               GPU (what rank 0 gathers over RCCL; no reference counterpart)
 *
 * Conventions: every call returns an int status (MT_OK = 0); output buffers are caller
 * owned and sized by calling with cap = 0 (the required length is returned in *len).
 * Strings are UTF-8.  No torch types cross this boundary; device memory is owned by the
 * batch.  A batch is bound to the HIP device current at mt_batch_create.
 */
#ifndef MTREPLAY_H
#define MTREPLAY_H

#include <stdint.h>

#include "mt_gen.h"
#include "mt_oplog.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MT_API __attribute__((visibility("default")))

/* Version of this header's binary interface: bumped on every change of a struct layout or an entry
   point's signature, so a binding built against another header fails at load (mt_abi_version())
   instead of passing fields at the wrong offsets.
   4: round 3 dropped oe_cap / blk_cap / heap_cap from mt_batch_options and added n_docs to
      mt_batch_ingest_json_gpu; round 4 added mt_abi_version.
   5: 15-bit short client ids (mt_oplog.h: high bits in mt_op.flags 11-13, insert prop counts
      <= 127, sentinels 0x7FFE / 0x7FFF); OutRec meta: clientId [0,15), removedClientId [15,30).
   6: writer consensus (mt_oplog.h MT_RELF_NOTIFY; a consensus ack's pos1 = relativePos1.id) and
      relative positions in local ops; mt_doc_consensus_events.
   7: mt_batch_snapshots keeps documents of more than MT_SNAP_MAX_BLOBS blobs on the GPU (their
      meta row's n_blobs exceeds MT_SNAP_MAX_BLOBS; the row holds the first MT_SNAP_MAX_BLOBS).
   8: inserts of any number of props (mt_oplog.h MT_OPF_NPROPS_EXT: a leading {MT_KEY_NPROPS,
      count} record past 126); mt_launch_info.start_ms (was reserved). */
#define MT_ABI_VERSION 8

enum mt_status_code {
    MT_OK = 0,
    MT_INVALID_POS = 1,  /* "MergeTree insert failed" */
    MT_SEQ_ORDER = 2,    /* sequence number went backwards */
    MT_MSN_ORDER = 3,    /* minimumSequenceNumber went backwards / above seq */
    MT_UNSUPPORTED = 4,  /* op outside the device model or limits (> 32765 clients) */
    MT_BAD_INPUT = 5,
    MT_CAPACITY = 6,     /* document exceeded the largest device capacity class */
    MT_INTERNAL = 7,
    MT_ERR_HIP = 100,
    MT_ERR_ARG = 101,
    MT_ERR_STATE = 102,
    MT_ERR_NO_DEVICE = 103
};

typedef struct mt_batch mt_batch;

typedef struct mt_batch_options {
    int32_t chunk_size;      /* SnapshotV1 chunk size; 0 -> 10000 (snapshotV1.ts:40)              */
    int32_t seg_cap;         /* segment slots of the first LDS capacity class (rounded up to a
                                class: 64 .. 4096); 0 -> derived from the ops per document        */
    int32_t arena_factor;    /* text arena = factor * payload + 4096 code units; 0 -> 4            */
    int32_t pool_per_op;     /* prop pool words per annotate / props insert; 0 -> 96               */
    int32_t max_retries;     /* capacity-class escalations for docs that overflow; 0 -> the whole ladder; < 0: none
                                (documents short of headroom still checkpoint: capacity planning)  */
} mt_batch_options;

typedef struct mt_batch_stats {
    int64_t n_docs;
    int64_t n_ops;          /* ops in the log                                                   */
    int64_t ops_applied;    /* ops applied before a document stopped                            */
    int64_t docs_failed;
    int32_t max_oe, max_slots, max_blocks, max_heap; /* high-water marks over all docs         */
    int32_t lds_bytes;      /* per-doc LDS of the first launch                                  */
    int32_t launches;       /* replay launches incl. capacity escalations                       */
    float kernel_ms;        /* device time of the replay launch(es) (hipEvents, batch stream)    */
    float total_ms;         /* mt_batch_run wall time incl. escalations                         */
    int32_t lds_class;      /* segment slots of the first launch's capacity class               */
    int32_t reserved;
} mt_batch_stats;

MT_API const char *mt_status_string(int code);

MT_API int mt_batch_create(mt_batch **out, int64_t n_docs, const mt_batch_options *opts);
MT_API void mt_batch_destroy(mt_batch *b);

MT_API int mt_batch_set_tables(mt_batch *b, const char *const *keys, int32_t n_keys,
                               const char *const *values_json, int32_t n_values);
/* doc < 0: the table for every document */
MT_API int mt_batch_set_clients(mt_batch *b, int64_t doc, const char *const *names, int32_t n);

/* host arrays; ops of doc d are ops[doc_op_off[d] .. doc_op_off[d+1]); insert payload offsets
   index `text`, annotate / insert-props offsets index `props` */
MT_API int mt_batch_ingest(mt_batch *b, const mt_op *ops, const int64_t *doc_op_off, const uint16_t *text,
                           int64_t n_text, const mt_prop *props, int64_t n_props);
/* JSON op logs: each document is one JSON array of
   ISequencedDocumentMessage (the file driver's messages.json, packages/drivers/file-driver/src/
   fileDeltaStorageService.ts:23-31), parsed and packed on n_threads host threads (<= 0: all
   cores) with the packing rules of fluidframework_amd/oplog.py / js/index.js.  On failure
   *bad_doc is the first failing document and mt_packed_error says why; *out is still set
   (destroy it).  mt_batch_ingest_packed = set_tables + set_clients + ingest of the result. */
typedef struct mt_packed mt_packed;
MT_API int mt_pack_json(mt_packed **out, int64_t n_docs, const char *const *doc_json, const int64_t *doc_len,
                        const char *observer, int32_t n_threads, int64_t *bad_doc);
MT_API void mt_packed_destroy(mt_packed *p);
MT_API const char *mt_packed_error(const mt_packed *p);
MT_API int mt_packed_sizes(const mt_packed *p, int64_t *n_ops, int64_t *n_text, int64_t *n_props, int32_t *n_keys,
                           int32_t *n_values);
MT_API int mt_packed_arrays(const mt_packed *p, mt_op *ops, int64_t *doc_op_off, uint16_t *text, mt_prop *props);
MT_API const char *mt_packed_key(const mt_packed *p, int32_t i);     /* WTF-8 */
MT_API const char *mt_packed_value(const mt_packed *p, int32_t i);   /* JSON text */
MT_API int32_t mt_packed_doc_clients(const mt_packed *p, int64_t doc);
MT_API const char *mt_packed_client(const mt_packed *p, int64_t doc, int32_t i);
MT_API int mt_batch_ingest_packed(mt_batch *b, const mt_packed *p);

/* JSON op logs parsed on the GPU (fluidframework_amd/csrc/mt_json_gpu.hip): the same records,
   text and tables as mt_pack_json for the observer fast path — sequenced messages whose contents
   are insert (text / {text, props} / markers) / remove / annotate (no combiningOp but rewrite) /
   relative positions / a one-level group of those, and a writer replica's (observer's) local
   messages (sequenceNumber -1) and acks — not regenerate events, notifyConsensus, a local insert
   with an end, or an ack with relative positions.  A batch with any other
   document returns MT_UNSUPPORTED with *bad_doc set and nothing changed: parse it with
   mt_pack_json (the bindings' ingest_json does).  json: the documents back to back, document d =
   json[doc_off[d] .. doc_off[d+1]), doc_off has n_docs + 1 entries and n_docs must equal the
   batch's (else MT_ERR_ARG).  d_json: the same bytes already on the device (NULL: copied here),
   4-byte aligned and readable 64 bytes past the end; the host copy `json` is still read (key,
   value and client-name strings are interned from it), so both must hold the same bytes.  Replaces the host parse of Client.applyMsg's input
   (clientReplayTool.ts:194-252 feeding client.ts:797-819). */
typedef struct mt_json_gpu_stats {
    double ms_scan, ms_count, ms_clients, ms_write, ms_props; /* device stages (hipEvents) */
    double ms_host;                                           /* host merge of the key / value tables */
    double ms_total;                                          /* wall time of the call */
    int64_t n_msgs, n_ops, n_text, n_props;
    uint32_t fail_bits;                                       /* why *bad_doc left the fast path */
    int32_t reserved;
} mt_json_gpu_stats;
MT_API int mt_pack_json_gpu(mt_packed **out, int64_t n_docs, const char *json, const int64_t *doc_off,
                            const char *observer, int64_t *bad_doc, mt_json_gpu_stats *stats);
MT_API int mt_batch_ingest_json_gpu(mt_batch *b, const char *json, const int64_t *doc_off, int64_t n_docs, const void *d_json,
                                    const char *observer, int64_t *bad_doc, mt_json_gpu_stats *stats);

/* synthesize logs on the device (include/mt_gen.h); doc_first = global index of doc 0 */
MT_API int mt_batch_generate(mt_batch *b, const mt_gen_params *p, int64_t doc_first);
/* the same with per-document global indices (stream seeds) and op counts (p->n_ops ignored):
   mixed-size batches, e.g. config 4's Zipf sizes after LPT assignment to this GPU */
MT_API int mt_batch_generate_docs(mt_batch *b, const mt_gen_params *p, const int64_t *doc_ids,
                                  const int32_t *doc_ops);

/* launch the replay on `hip_stream` (NULL = the batch's own stream) and wait for it */
MT_API int mt_batch_run(mt_batch *b, void *hip_stream);
/* launch without waiting; mt_batch_sync waits and collects per-doc results */
MT_API int mt_batch_launch(mt_batch *b, void *hip_stream);
MT_API int mt_batch_sync(mt_batch *b);
MT_API int mt_batch_get_stats(mt_batch *b, mt_batch_stats *out);
/* one replay launch of the last run: launch 0 holds every document, later ones the documents
   escalated to a larger capacity class (mt_batch_stats.launches of them) */
typedef struct mt_launch_info {
    int32_t seg_class;      /* segment slots of the launch's capacity class                  */
    int32_t n_docs;         /* documents (workgroups) in the launch                           */
    int32_t resumed;        /* of them resumed from a checkpoint (the rest start from op 0)   */
    int32_t lds_bytes;      /* dynamic LDS per document (0: HBM class)                        */
    float ms;               /* device time (hipEvents on the launch's stream)                 */
    float start_ms;         /* its start, from the run's start (concurrent launches overlap)  */
    int64_t ops;            /* ops applied by this launch                                     */
} mt_launch_info;
MT_API int mt_batch_launch_info(mt_batch *b, int32_t i, mt_launch_info *out);
/* algorithmic HBM bytes of one replay (DESIGN.md "Roofline"): ops, payloads, final table, text */
MT_API int mt_batch_algorithmic_bytes(mt_batch *b, double *bytes);

MT_API int32_t mt_doc_status(mt_batch *b, int64_t doc);
/* per-document run counters, MT_DOC_COUNTERS int32 per document (capacity planning / stats):
   status, min_seq, cur_seq, depth, n_entries, text_top, pool_top, ops_done, max_unsettled,
   max_slots, max_blocks, max_heap, fail_op, cap_kind, launch, reserved */
#define MT_DOC_COUNTERS 16
MT_API int mt_batch_doc_counters(mt_batch *b, int32_t *out);
MT_API int mt_doc_text(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len);
MT_API int mt_doc_props_runs(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len);
/* Client.findTile(startPos, tileLabel, preceding) (merge-tree/src/client.ts:1073-1076,
   mergeTree.ts:1763-1789) on the document's final state: *tile_pos = the tile marker's position
   (-1: no tile); props_buf gets JSON.stringify(marker.properties) (size query with cap 0).
   MT_UNSUPPORTED: the document annotates referenceTileLabels (the reference's block tile maps
   would be stale) or holds a label list other than an array of strings. */
MT_API int mt_doc_find_tile(mt_batch *b, int64_t doc, int64_t start_pos, const char *label_utf8, int32_t preceding,
                            int64_t *tile_pos, char *props_buf, int64_t props_cap, int64_t *props_len);
/* Client.getStackContext(startPos, rangeLabels) (merge-tree/src/client.ts:946-948 ->
   mergeTree.ts:1750-1760; SharedSegmentSequence.getStackContext, sequence/src/sequence.ts:377) on
   the document's final state: JSON {label: [{"pos": P, "refType": T[, "props": {...}]}, ...]} — the
   range stacks of NestBegin / NestEnd markers (referenceRangeLabels), bottom to top, keys in JS
   object order (size query with cap 0).  MT_UNSUPPORTED: the document annotates
   referenceRangeLabels (the reference's block maps would be stale) or holds a label list other
   than an array of strings. */
MT_API int mt_doc_stack_context(mt_batch *b, int64_t doc, int64_t start_pos, const char *const *labels_utf8,
                                int32_t n_labels, char *buf, int64_t cap, int64_t *len);
/* Client.regeneratePendingOp results (client.ts:855-893) of the document's MT_OP_REGENERATE
   records (a writer replica reconnecting), in order: a JSON array of the regenerated ops, one per
   reset message (a GROUP op when it regenerates to more or fewer than one op) */
MT_API int mt_doc_regenerated_ops(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len);
/* The consensus callbacks of a writer replica's replay, in call order: a JSON array of
   {"markerId": id, "seq": S, "minSeq": M} — Client.annotateMarkerNotifyConsensus (client.ts:113-134;
   a local message with "notifyConsensus": true) registered the marker id, the ack at seq S ran
   updateConsensusProperty (980-987) and minSeq M >= S called consensusInfo.callback(marker)
   (mergeTree.ts:1701-1716).  Listeners not yet called are not listed. */
MT_API int mt_doc_consensus_events(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len);
MT_API int mt_doc_snapshot_v1(mt_batch *b, int64_t doc, int32_t *n_blobs);
MT_API int mt_doc_snapshot_blob(mt_batch *b, int64_t doc, int32_t i, char *name, int64_t name_cap, char *buf,
                                int64_t cap, int64_t *len);
/* SnapshotV1 of every document on the GPU (mt_snapshot.hip: a sizing pass, a host prefix sum of
   the bytes, a writing pass) into one device buffer of *total_bytes; *device_ms = both passes.
   Blobs of a document lie back to back (header, body_0, ..) at doc_off[doc].  A meta row holds
   n_blobs and the entries of the first MT_SNAP_MAX_BLOBS blobs (n_blobs may be larger: the device
   keeps every blob; mt_doc_snapshot_v1_device returns them all); a document the device leaves to
   the host serializer gets size 0 there and n_blobs 0. */
#define MT_SNAP_MAX_BLOBS 32
#define MT_SNAP_META (1 + 3 * MT_SNAP_MAX_BLOBS) /* n_blobs, then (segmentCount, length, bytes) */
MT_API int mt_batch_snapshots(mt_batch *b, int64_t *total_bytes, float *device_ms);
/* after mt_batch_snapshots: the GPU blobs of `doc` become what mt_doc_snapshot_blob returns
   (a document the device left to the host: the host serializer, as mt_doc_snapshot_v1) */
MT_API int mt_doc_snapshot_v1_device(mt_batch *b, int64_t doc, int32_t *n_blobs);
/* doc_off[n_docs + 1] byte offsets; blob_meta[n_docs * MT_SNAP_META] (either may be NULL) */
MT_API int mt_batch_snapshot_index(mt_batch *b, int64_t *doc_off, int32_t *blob_meta);
MT_API int mt_batch_snapshot_copy(mt_batch *b, void *dst, int32_t dst_is_device);
/* per-document 64-bit digest of the GPU SnapshotV1 bytes (all blobs in order; 0 for a document
   left to the host serializer), into dst[n_docs] (device pointer when dst_is_device) — with
   mt_batch_device_digests, the per-document summary rank 0 gathers (config 5) */
MT_API int mt_batch_snapshot_digests(mt_batch *b, uint64_t *dst, int32_t dst_is_device);
MT_API int mt_doc_digest(mt_batch *b, int64_t doc, uint64_t *out);
/* per-document device digests of the last run into dst[n_docs] (a device pointer when
   dst_is_device, else host memory) */
MT_API int mt_batch_device_digests(mt_batch *b, uint64_t *dst, int32_t dst_is_device);
MT_API int mt_doc_shape(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len);
/* debugging aid: the final segment table, one line per entry */
MT_API int mt_doc_dump(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len);

/* the (ingested or generated) log in host memory, batch-global offsets (CPU baseline / parity) */
MT_API int mt_batch_log_sizes(mt_batch *b, int64_t *n_ops, int64_t *n_text, int64_t *n_props);
MT_API int mt_batch_download_log(mt_batch *b, mt_op *ops, int64_t *doc_op_off, uint16_t *text, mt_prop *props);
/* the same for documents [d0, d1) only (a bounded sample of a large batch): offsets from 0, text of
   those documents back to back, prop records [0, *n_props) of the batch */
MT_API int mt_batch_log_sizes_docs(mt_batch *b, int64_t d0, int64_t d1, int64_t *n_ops, int64_t *n_text,
                                   int64_t *n_props);
MT_API int mt_batch_download_log_docs(mt_batch *b, int64_t d0, int64_t d1, mt_op *ops, int64_t *doc_op_off,
                                      uint16_t *text, mt_prop *props);
/* hash of the sources this library was built from (__graft_entry__.py SRC, sha256 hex prefix) */
MT_API const char *mt_build_id(void);
/* MT_ABI_VERSION of the header the library was built with */
MT_API int32_t mt_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
