/*
 * mt_oplog.h — packed sequenced merge-tree op log (shared by the C-ABI library,
 * the HIP kernels, the host layers and the test oracle).
 *
 * One record = one ISequencedDocumentMessage carrying one IMergeTreeDeltaOp:
 *   message fields  : server/routerlicious/packages/protocol-definitions/src/protocol.ts:132-172
 *                     (clientId, sequenceNumber, referenceSequenceNumber,
 *                      minimumSequenceNumber, type "op", contents)
 *   op contents     : packages/dds/merge-tree/src/ops.ts:29-110
 *                     insert {type:0,pos1,seg}, remove {type:1,pos1,pos2},
 *                     annotate {type:2,pos1,pos2,props}, group {type:3,ops:[...]}
 *
 * A GROUP message is encoded as consecutive records sharing seq/ref_seq/msn;
 * every member except the last carries MT_OPF_GROUP_CONT (Client.applyRemoteOp
 * applies the members, then Client.applyMsg runs updateSeqNumbers once:
 * merge-tree/src/client.ts:782-790, 797-819).
 *
 * Strings never enter a record: text lives in a UTF-16 code-unit arena and
 * property keys/values are interned ids (value id 0 == JSON null == delete key,
 * merge-tree/src/properties.ts:95-116).
 */
#ifndef MT_OPLOG_H
#define MT_OPLOG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum mt_op_type {
    MT_OP_INSERT = 0,   /* MergeTreeDeltaType.INSERT   */
    MT_OP_REMOVE = 1,   /* MergeTreeDeltaType.REMOVE   */
    MT_OP_ANNOTATE = 2, /* MergeTreeDeltaType.ANNOTATE */
    /* SnapshotLoader (merge-tree/src/snapshotLoader.ts:36-205), a document's first records:
       LOAD_HEADER  one segment of the "header" chunk; the run of them is built bottom-up as
                    MergeTree.reloadFromSegments does (mergeTree.ts:1195-1251)
       COLLAB       startOrUpdateCollaboration(observer, minSeq = msn, currentSeq = seq)
       LOAD_BODY    one segment of a body chunk, appended at the end with insertSegments
                    (refSeq UniversalSequenceNumber); MT_OPF_GROUP_CONT chains the members of
                    one batch (consecutive NonCollabClient / UniversalSequenceNumber segments)
       A LOAD record is an insert record (payload / flags / pos2 as for MT_OP_INSERT) with
       client = the segment's clientId (MT_CLIENT_NONCOLLAB for NonCollabClient), seq = its
       seq (0 = UniversalSequenceNumber), ref_seq = its removedSeq (MT_SEQ_NONE if not
       removed) and msn = its removedClientId (MT_CLIENT_NONE if not removed). */
    MT_OP_LOAD_HEADER = 3,
    MT_OP_LOAD_BODY = 4,
    MT_OP_COLLAB = 5,
    /* RELPOS  the relative positions of the record that follows it (same client / seq / refSeq /
               msn, always MT_OPF_GROUP_CONT): an op with pos1 (pos2) undefined and relativePos1
               (relativePos2) given takes posFromRelativePos (client.ts:485-502, mergeTree.ts:
               1942-1966).  pos1 / pos2 = value id of relativePosN.id (0: none), payload /
               payload_len = offsetN (int32), flags = MT_RELF_*. */
    MT_OP_RELPOS = 6,
    /* REGENERATE  a writer replica's Client.regeneratePendingOp(resetOp, oldest pending group)
                   (client.ts:708-766, 855-893) on reconnect: seq -1, client 0, ref_seq = the reset
                   op's type (insert / remove / annotate), flags / payload / payload_len = its
                   flags and prop records (annotate); a GROUP reset op is one record per member,
                   MT_OPF_GROUP_CONT on all but the last.  The regenerated ops are an output
                   (mt_doc_regenerated_ops); their sequenced messages later ack the new groups. */
    MT_OP_REGENERATE = 7,
    MT_OP_NOOP = 15     /* non-"op" message: only client registration + updateSeqNumbers */
};
enum mt_relpos_flags {
    MT_RELF_POS1 = 0x10u,    /* pos1 of the next record is relativePos1            */
    MT_RELF_POS2 = 0x20u,    /* pos2 of the next record is relativePos2            */
    MT_RELF_BEFORE1 = 0x40u, /* relativePos1.before is truthy                      */
    MT_RELF_BEFORE2 = 0x80u,
    MT_RELF_OFF1 = 0x100u,   /* relativePos1.offset is defined (payload)           */
    MT_RELF_OFF2 = 0x200u,   /* relativePos2.offset is defined (payload_len)       */
    /* a local RELPOS of the replica's Client.annotateMarkerNotifyConsensus(marker, props, callback)
       (client.ts:113-134): the annotate that follows registers pendingConsensus[marker id] when it
       applies; payload = the raw value id of relativePos1.id (the op has no offsets) */
    MT_RELF_NOTIFY = 0x2u
};
/* The replica's own sequenced consensus annotate (an ack; its positions are not read) carries in
   pos1 the raw value id of relativePos1.id (0: none a Map lookup could match) for
   updateConsensusProperty (client.ts:980-987); the library puts its marker-id key in pos2. */
/* short client ids are 15-bit: 0 .. 32765 per document (0 = the observer; Client.getOrAddShortClientId,
   client.ts:636-660, numbers every long id a document's log names, and a real messages.json names a
   new one on every reconnect), 0x7FFE / 0x7FFF are sentinels.  A record's `client` bit-field holds
   the low 12 bits, flags bits 11-13 the high 3 (MT_OP_CLIENT / MT_OPF_CLIENT_HI). */
#define MT_CLIENT_NONCOLLAB 0x7FFEu /* NonCollabClient (constants.ts:15); long id "original" */
#define MT_CLIENT_NONE 0x7FFFu
#define MT_MAX_CLIENTS 0x7FFE      /* short ids 0 .. 32765 per document (0 = the observer)       */
#define MT_OPF_CLIENT_HI_MASK 0x3800u
#define MT_OPF_CLIENT_HI(c) ((uint16_t)((((uint32_t)(c) >> 12) & 7u) << 11))
#define MT_OP_CLIENT(o) ((uint32_t)(o).client | ((((uint32_t)(o).flags >> 11) & 7u) << 12))
#define MT_SEQ_NONE 0x7FFFFFFF
#define MT_OP_IS_INSERT_LIKE(t) ((t) == MT_OP_INSERT || (t) == MT_OP_LOAD_HEADER || (t) == MT_OP_LOAD_BODY)

/* Writer replicas (the local-client path): a record with seq == -1 (UnassignedSequenceNumber) is
   a local op of the replica (client 0), applied in its local view and kept pending; a sequenced
   record of client 0 acks the oldest pending group (client.ts:797-819, mergeTree.ts:1893-1929). */
#define MT_SEQ_LOCAL (-1)

/* mt_op.flags: bits 0-3 public flags, bits 4-10 the prop count of an insert (0..126; 127 =
   MT_OPF_NPROPS_EXT: the count is in the first prop record), bits 11-13 the short client id's high
   bits (every record type), bits 14-15 are internal to the library (set at ingest: the insert's
   text contains a '\n' / its last code unit is '\n') */
enum mt_op_flags {
    MT_OPF_GROUP_CONT = 1u, /* more members of the same GROUP message follow          */
    MT_OPF_MARKER = 2u,     /* insert of a Marker: payload = refType, payload_len = 1  */
    MT_OPF_HAS_PROPS = 4u,  /* insert seg carries a props object (may be empty {})     */
    MT_OPF_REWRITE = 8u     /* annotate with combiningOp {name:"rewrite"}              */
};
/* An annotate's combiningOp other than "rewrite" (properties.ts:26-60 combine, called by
   SegmentPropertiesManager.addProperties, segmentPropertiesManager.ts:96-101): flags bits 4-5 of
   an ANNOTATE record (insert records use bits 4-13 for their prop count).  The op's props keys
   select the keys to combine; their values are ignored — the reference passes the local
   `newValue` (still undefined) to combine at segmentPropertiesManager.ts:98, not newProps[key].
   Three records follow the op's payload_len prop records, all with key MT_KEY_COMBINE:
   defaultValue, minValue (value ids; MT_VALUE_UNDEFINED when absent) and a result slot that the
   packers leave MT_VALUE_UNDEFINED and the library fills at ingest. */
enum mt_combine_kind {
    MT_COMBINE_NONE = 0,      /* no combiningOp (or "rewrite": MT_OPF_REWRITE)               */
    MT_COMBINE_INCR = 1,      /* {name:"incr"}                                                */
    MT_COMBINE_CONSENSUS = 2, /* {name:"consensus"}                                           */
    MT_COMBINE_OTHER = 3      /* any other truthy combiningOp: combine keeps the current value */
};
#define MT_OPF_COMBINE(f) (((uint32_t)(f) >> 4) & 0x3u)
#define MT_OPF_MAKE_COMBINE(kind) ((uint16_t)(((kind) & 0x3u) << 4))
#define MT_COMBINE_RECORDS 3u
#define MT_KEY_COMBINE 0xFFFFFFFFu
#define MT_VALUE_UNDEFINED 0xFFFFFFFFu
#define MT_OPF_BITS(f) ((f) & 0xFu)
/* the raw 7-bit field; use mt_insert_props() to read an insert's prop records */
#define MT_OPF_NPROPS(f) (((uint32_t)(f) >> 4) & 0x7Fu)
/* An insert (or LOAD record) with more than MT_OPF_NPROPS_INLINE props sets the field to
   MT_OPF_NPROPS_EXT and its prop records start with {MT_KEY_NPROPS, count}: any number of props
   (the reference's TextSegment.make / Marker.make copy every key, textSegment.ts:23-28,
   properties.ts:95) */
#define MT_OPF_NPROPS_INLINE 126u
#define MT_OPF_NPROPS_EXT 127u
#define MT_KEY_NPROPS 0xFFFFFFFEu
#define MT_OPF_MAKE(bits, nprops) \
    ((uint16_t)((((nprops) > MT_OPF_NPROPS_INLINE ? MT_OPF_NPROPS_EXT : ((nprops) & 0x7Fu)) << 4) | ((bits) & 0xFu)))
/* prop records an insert of n props occupies (the count record of an extended one included) */
#define MT_INSERT_PROP_RECORDS(n) ((n) > MT_OPF_NPROPS_INLINE ? (n) + 1u : (n))
#define MT_OPF_INTERNAL_HAS_NL 0x4000u
#define MT_OPF_INTERNAL_ENDS_NL 0x8000u
#define MT_OPF_INTERNAL (MT_OPF_INTERNAL_HAS_NL | MT_OPF_INTERNAL_ENDS_NL)

/* The first 16-bit word holds the record type (bits 0-3) and the low 12 bits of the short client id
   (bits 4-15): little-endian u16 `type | (client & 0xFFF) << 4`; the id's high 3 bits are flags bits
   11-13.  C / C++ / HIP read them through the bit-fields below and MT_OP_CLIENT; byte packers
   (Python, JS) write the words. */
typedef struct mt_op {
    uint16_t type : 4;    /* enum mt_op_type                                             */
    uint16_t client : 12; /* short client id, low 12 bits (index in the doc's client table;
                             0 is the observer itself, as Client.startOrUpdateCollaboration
                             assigns it first: client.ts:1051-1062); MT_OP_CLIENT            */
    uint16_t flags;       /* enum mt_op_flags | nprops<<4                                  */
    int32_t seq;          /* sequenceNumber                                                */
    int32_t ref_seq;      /* referenceSequenceNumber                                       */
    int32_t msn;          /* minimumSequenceNumber                                         */
    int32_t pos1;         /* insert: pos; remove/annotate: start                           */
    int32_t pos2;         /* remove/annotate: end; insert with props: prop record offset   */
    uint32_t payload;     /* insert: text offset (code units); annotate: prop record offset;
                             marker insert: refType                                         */
    uint32_t payload_len; /* insert: text length; annotate: prop count                     */
} mt_op;

typedef struct mt_prop {
    uint32_t key;   /* interned key id                       */
    uint32_t value; /* interned value id; 0 = null (delete)  */
} mt_prop;

#define MT_VALUE_NULL 0u

/* An insert's prop records: *first = index of its first (key, value) record in `props`, returns
   their count (the 7-bit flags field, or for MT_OPF_NPROPS_EXT the count record at op->pos2) */
#if defined(__HIPCC__)
__host__ __device__
#endif
static inline uint32_t mt_insert_props(const mt_op *op, const mt_prop *props, uint32_t *first) {
    const uint32_t n = MT_OPF_NPROPS(op->flags);
    if (n != MT_OPF_NPROPS_EXT) {
        *first = (uint32_t)op->pos2;
        return n;
    }
    *first = (uint32_t)op->pos2 + 1u;
    return props[op->pos2].value;
}

#ifdef __cplusplus
static_assert(sizeof(mt_op) == 32, "mt_op is 32 bytes");
#else
_Static_assert(sizeof(mt_op) == 32, "mt_op is 32 bytes");
#endif

#ifdef __cplusplus
}
#endif
#endif /* MT_OPLOG_H */
