// mt_device.h — shared constants and record layouts of the MI355X merge-tree replay engine.
//
// Used by the HIP kernels (mt_engine.hip) and the host side of the C-ABI library
// (mt_host.cpp).  Everything here is plain data; no torch types, no STL.
#pragma once

#include <stdint.h>

#include "../../include/mt_oplog.h"

namespace mt {

// status codes (include/mtreplay.h MT_STATUS_*; the first six match the oracle's)
enum : int32_t {
    ST_OK = 0,
    ST_INVALID_POS = 1,  // "MergeTree insert failed" (merge-tree/src/mergeTree.ts:2210-2216)
    ST_SEQ_ORDER = 2,    // client.ts:461-462, 824
    ST_MSN_ORDER = 3,    // client.ts:463-464, mergeTree.ts:1719-1722
    ST_UNSUPPORTED = 4,  // outside the observer path / device limits (e.g. > 32765 clients)
    ST_BAD_INPUT = 5,
    ST_CAPACITY = 6,     // per-document LDS/HBM capacity exceeded: re-run with larger caps
    ST_INTERNAL = 7
};

constexpr int kWave = 64;
constexpr int kMaxNodes = 8;            // MaxNodesInBlock, mergeTree.ts:334
constexpr uint32_t kGranularity = 256;  // TextSegmentGranularity, mergeTree.ts:1059
constexpr int kZamboniMax = 2;          // zamboniSegmentsMaxCount, mergeTree.ts:1061
constexpr int kMaxClients = MT_MAX_CLIENTS;  // short client ids 0..32765 (0x7FFE NonCollabClient, 0x7FFF none)
constexpr int32_t kNoneSeq = 0x7FFFFFFF;  // removedSeq === undefined
constexpr uint32_t kOutBlockEnd = 0x80000000u;  // OutRec.blk of the entry that ends a leaf block
__host__ __device__ constexpr bool out_is_end(uint32_t blk) { return (blk & kOutBlockEnd) != 0; }
constexpr uint32_t kNoClient = MT_CLIENT_NONE;
constexpr uint32_t kOvlMaskClients = 31u; // overlap sets of clients < 31 are a bit mask (see kOvlList)
constexpr uint32_t kOvlList = 0x80000000u;  // cold.y with this bit: pool offset of an overlap-client list
constexpr uint32_t kPoolOvlTag = 0x40000000u;  // header word of an overlap-list pool record: n | tag

// value flags (mt_values.h kVal*): matchProperties of two interned values is class equality,
// else membership of the pair in the exception list (both kValIrregular); kValUnknown: undecided
// kVNum: `v += undefined` is NaN; kVNever: matches nothing (NaN, a consensus {value: undefined});
// kVSeqM1: an object with own seq === -1 (consensus would update it in place)
constexpr uint8_t kVFalsy = 1u, kVIrregular = 2u, kVUnknown = 4u, kVNum = 8u, kVNever = 16u, kVSeqM1 = 32u;
// prop-set hash bits (mt_engine.hip props_extend): bit 0 every value regular, bit 1 a value matches nothing
constexpr uint32_t kSetRegular = 1u, kSetNever = 2u;

// device matchProperties of two values (R(a, b), mt_values.cpp): 1 match, 0 no, -1 undecided
__device__ __forceinline__ int value_rel(uint32_t va, uint32_t vb, const uint32_t *vclass, const uint8_t *vflags,
                                         uint32_t n_values, const uint64_t *exc, uint32_t n_exc) {
    if (va >= n_values || vb >= n_values) return va == vb ? 1 : 0;
    const uint32_t fa = vflags[va], fb = vflags[vb];
    if ((fa | fb) & kVNever) return 0;  // NaN !== NaN
    if (va == vb || vclass[va] == vclass[vb]) return 1;
    if ((fa | fb) & kVUnknown) return -1;
    if (!(fa & fb & kVIrregular)) return 0;
    const uint64_t key = (uint64_t)va << 32 | vb;
    uint32_t lo = 0, hi = n_exc;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (exc[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo < n_exc && exc[lo] == key ? 1 : 0;
}

// needsScour tri-state (mergeTree.ts:63, 1279, 1438)
constexpr int8_t kScourUndef = -1, kScourFalse = 0, kScourTrue = 1;

// OutRec meta word (the device's final table, mt_host.cpp, mt_snapshot.hip, mt_digest.hip):
//   [0,15)  clientId (short id)        [15,30) removedClientId (kNoClient = none)
//   [30]    Marker                      [31]    removedClientOverlap is non-empty
// The engine's per-slot LDS meta is narrower (mt_engine.hip SlotMeta): flags plus the index of the
// slot's unsettled-overlay entry; client ids live in the cold record and in the overlay entry.
constexpr uint32_t kMetaCli = 0x7FFFu;
constexpr uint32_t kMetaRcliShift = 15;
constexpr uint32_t kMetaMarker = 1u << 30;
constexpr uint32_t kMetaHasOvl = 1u << 31;
__host__ __device__ constexpr uint32_t meta_cli(uint32_t m) { return m & kMetaCli; }
__host__ __device__ constexpr uint32_t meta_rcli(uint32_t m) { return (m >> kMetaRcliShift) & kMetaCli; }
// canonical slot meta of a checkpoint image: 7 flag bits at [24, 31), the overlay-entry index below
// (kCanonNoEntry: settled).  Flag order: linked, Marker, ends-'\n', has props, has '\n', removed,
// pending (a writer's unacked local segment group holds the slot)
constexpr uint32_t kCanonNoEntry = 0xFFFFFFu;
// a writer replica's pending-group membership: bit G & 31 of the 32-bit mask in the slot's cold
// record (cold[2 slot + 1].w) for group G
constexpr int kPendMaskBits = 32;
constexpr int32_t kUnassignedSeq = -1;  // UnassignedSequenceNumber (constants.ts:11): real seqs of pending ops
constexpr int32_t kSeq16Span = 0xFFF0;    // LDS classes: cur_seq - base must stay below (else cap_kind 8)
constexpr uint32_t kHeapInvalid = 0xFFFFFFFFu;  // heap entry whose segment was merged away / unlinked
constexpr uint16_t kNoBlock = 0xFFFFu;

// one output record per leaf or end-of-leaf-block entry (doc order), 8 x u32
struct OutRec {
    uint32_t len;    // cachedLength (0 for a block marker)
    int32_t seq;
    int32_t rseq;    // kNoneSeq when not removed
    uint32_t meta;   // client ids, Marker, has-overlap (kMetaCli, kMetaRcliShift, kMetaMarker, kMetaHasOvl)
    uint32_t ovl;    // removedClientOverlap: bit mask of clients < 31, or kOvlList | pool offset of
                     // a [n | kPoolOvlTag, 0, client x n] list
    uint32_t props;  // prop-set id in the doc's pool (0 = undefined)
    uint32_t toff;   // text offset in the doc's text region (Marker: refType; the end record of a leaf
                     // block: the interior blocks that end with it)
    uint32_t blk;    // leaf block id; | kOutBlockEnd for the entry that ends the block
};
static_assert(sizeof(OutRec) == 32, "OutRec");

// per-document scalar results
struct DocOut {
    int32_t status;
    int32_t min_seq;
    int32_t cur_seq;
    int32_t depth;
    int32_t n_out;      // OutRec count
    uint32_t text_top;  // text region high-water mark (code units)
    uint32_t pool_top;  // prop pool high-water mark (words)
    int32_t ops_done;   // ops applied before status != OK
    int32_t max_oe;     // output entries (leaves + leaf blocks); then high-water marks
    int32_t max_slots;
    int32_t max_blocks;
    int32_t max_heap;
    int32_t fail_op;    // index of the op that failed (-1)
    int32_t cap_kind;   // ST_CAPACITY cause: 1 LDS tables, 2 text arena, 3 prop pool, 4 out records,
                        // 5 (unused since round 4: a collab window wider than kSeq16Span ops
                        //   re-runs in a spill class, cap_kind 8),
                        // 6 LDS headroom: state checkpointed before op ops_done (resumable),
                        // 8 a segment longer than an LDS class's 16-bit lengths, or a collab
                        //   window of kSeq16Span ops or more (16-bit relative seqs): re-run from
                        //   scratch in a spill class (32-bit lengths and relative seqs)
    int32_t gen_text;   // generator: payload code units written
    int32_t gen_props;  // generator: prop records written
};
static_assert(sizeof(DocOut) == 64, "DocOut");

// per-document capacities of the LDS-resident state
struct Caps {
    int32_t seg;   // segment slots
    int32_t oe;    // output entries (segments + one end marker per leaf block)
    int32_t blk;   // blocks
    int32_t heap;  // zamboni heap entries
    int32_t ulist; // unsettled-overlay list entries
    int32_t iblk;  // LDS classes: interior block ids [blk - iblk, blk), the only ones with settled /
                   // overlay lengths (a leaf block's length is the sum over its leaves); 0: one pool
};

// Capacity classes are compile-time: each class is its own kernel instantiation
// (mt_kernels.hip), so every LDS array base is an immediate offset and no SGPRs hold
// table pointers or bounds.
// The LDS classes are sized to the residency they buy: LDS is allocated in 1,280-byte granules
// (128 per CU; measured with tools/probe/lds_residency.hip, profiles/r01_lds_residency.json) and
// the replay kernel's 128 VGPRs cap a CU at 16 workgroups, so each class is the largest slot
// count whose layout fits floor(128 / n) granules for n = 16, 14, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3
// and 2 documents per CU (tools/class_sizes.cpp); 128 keeps small documents' buffers small and
// 7,266 is the largest layout within the 160 KiB of one CU (minus the generator's static LDS).
// Beyond the LDS ladder (32-bit slot / block ids and lengths):
//  - the GIANT class (2,000,000 slots): segment and low-level block tables in HBM, everything a
//    per-op walk touches first in the CU's LDS — the interior blocks of levels >=
//    kGiantLdsLevel (the top of the tree), the overlay list, the zamboni heap and the scalars; one
//    document per CU (config 4's Zipf tail, ~10^6 segments);
//  - the HBM class (2,097,152 slots): every table in HBM, the fallback for a giant document whose
//    LDS-resident parts outgrow the CU.
// The replay kernel is latency bound, so a launch's rate grows with the documents per CU.
constexpr int kGiantSeg = 2000000;
constexpr int kHbmSeg = 2097152;
// the class list (X-macro: mt_host.cpp declares each class's kernels from it; __graft_entry__.py
// builds one object per entry)
#define MT_CLASS_LIST(X) \
    X(128) X(464) X(563) X(659) X(756) X(847) X(1036) X(1216) X(1400) X(1679) X(2046) X(2688) X(3499) X(3937) X(7961) \
    X(2000000) X(2097152)
#define MT_CLASS_SEG_(S) S,
constexpr int kClassSegs[] = {MT_CLASS_LIST(MT_CLASS_SEG_)};
static_assert(kClassSegs[15] == kGiantSeg && kClassSegs[16] == kHbmSeg, "spill classes last");
constexpr int kNumClasses = 17;
constexpr int kGiantClass = kNumClasses - 2;
constexpr int kHbmClass = kNumClasses - 1;
constexpr int kLastLdsClass = kGiantClass - 1;
constexpr int kReplayStartClass = 1;  // replay starts documents in at most the 16-per-CU class
// the kernels that append early-escalation notices (ReplayParams.notice): those of the classes a
// first replay launch runs in
__host__ __device__ constexpr bool notice_class(int seg) { return seg <= kClassSegs[kReplayStartClass]; }
constexpr bool is_giant_seg(int seg) { return seg == kGiantSeg; }
// giant class: block ids [0, kGiantLdsBlocks) are LDS-resident and given to blocks of level >=
// kGiantLdsLevel (0 = leaf blocks); lower levels (and high ones once the LDS ids run out) take
// HBM ids [kGiantLdsBlocks, cap.blk).  The overlay list and the heap have LDS capacities: a
// document short of them checkpoints into the HBM class.
constexpr int kGiantLdsBlocks = 2304;
constexpr int kGiantLdsLevel = 3;
constexpr int kGiantHeap = 1024;
constexpr int kGiantUlist = 1024;
constexpr int kGiantChainRec = 4;  // HBM-resident blocks recorded per overlay list entry
// The giant class's replay workgroup holds a second wave that prefetches (mt_engine.hip
// giant_prefetch): the replaying wave publishes in LDS words [0] the index of the op it applies,
// [1] root, [2] depth, [7] giant_run(w) / giant_done(w); word [6] is the prefetch wave's sink.
// The state words name the workgroup's document slot w: LDS keeps its contents between the
// workgroups a CU runs, so a state left by an earlier document never matches a later one's.
constexpr int kGiantPubWords = 8;
__host__ __device__ constexpr uint32_t giant_run(int64_t w) { return 0x80000000u ^ (uint32_t)(2 * w); }
__host__ __device__ constexpr uint32_t giant_done(int64_t w) { return 0x80000000u ^ (uint32_t)(2 * w + 1); }
constexpr int kGiantThreads = 128;
constexpr int kCapCheckpoint = 6;  // DocOut.cap_kind of a checkpointed (resumable) document
constexpr int kCapLongSeg = 8;     // beyond an LDS class's 16-bit lengths or relative seqs: a spill class

// Writer replicas (the local-client path, mergeTree.ts:1893-1929, client.ts:588-625): per document
// a pending-group region in HBM, persistent across launches (u32 words):
//   [0] pending groups n   [1] id G of the oldest (groups are numbered in creation order)
//   [2] first entry that may be live   [3] entries used
//   [kPendDesc ..) per group G, at G mod pend_groups(cap): {type | flags << 16, prop-record offset,
//                  prop count, localSeq}
//   [pend_entries(cap) ..) `cap` entries {G, slot} in append order (the group's `segments` array
//   order: members as the op reached them, split-off halves appended when the split happens)
//   word 4: collabWindow.localSeq (one per applied local op); a group's desc .w = its localSeq
// `cap` (ReplayParams.pend_cap) is a power of two the host sizes from the log (mt_host.cpp
// writer_regions: 4 entries per group of the most unacked local ops any replica holds, at least
// 4,096); cap / 4 groups may be pending at once (more: MT_UNSUPPORTED, only if the log's own count
// was exceeded).  A segment's groups are the bits G & 31 of a 32-bit mask in its cold record: exact
// while at most 32 groups are pending; beyond, a bit stands for every live group 32 apart and
// membership is decided by the groups' entry lists
constexpr int kPendDesc = 8;
__host__ __device__ constexpr uint32_t pend_groups(int32_t cap) { return (uint32_t)cap >> 2; }
__host__ __device__ constexpr uint32_t pend_entries(int32_t cap) { return (uint32_t)kPendDesc + 4u * pend_groups(cap); }
constexpr int kCapPending = 9;  // DocOut.cap_kind: the pending-entry region is full (terminal)
constexpr int kCapRegen = 10;   // DocOut.cap_kind: the regenerated-op output region is full (terminal)
// DocOut.cap_kind 3 (the prop pool) from an observer replay kernel of an LDS class: a property set or
// op past one pair per lane there, or a full pool.  The host re-runs the document from scratch in the
// class's mt_bigprops_kernel_<SEG> (mt_engine.hip props_extend_big), and its later escalations stay in
// the bigprops kernels; a full pool stops it there again (terminal).  (A kind of its own measured
// worse: the distinct constant alone moved class 756's SGPR spills from 182 to 260.)
constexpr int kCapPool = 3;
constexpr int64_t pend_words(int32_t cap) { return (int64_t)pend_entries(cap) + 2ll * cap; }
// regenerated ops of MT_OP_REGENERATE records, per document (u32 words): [0] words used (from 2),
// [1] records; per record {GROUP_CONT flag, ops} then per op {type, pos1, pos2, a, b, c, nprops, 0}
// + nprops (key, value) pairs.  insert: a = 1 | refType << 1 for a Marker (else 0), b = text offset
// in the document's payload, c = length, the pairs = its properties (nprops 0xFFFFFFFF: none);
// annotate: a = flags, b / c = the reset op's prop records; remove: nothing more
constexpr int kRegenOpWords = 8;

// writer consensus (Client.annotateMarkerNotifyConsensus / updateConsensusProperty, client.ts:113-134,
// 980-987), per document (u32 words), persistent across launches: [0] registered ids, [1] min-seq
// listeners queued, [2] listeners fired, [3] id capacity, [4] listener capacity, [5..8) 0; from word
// kConsHdr the pendingConsensus keys (raw value ids of marker ids), then per listener {raw id, seq,
// registered, minSeq when it fired, seq of the message that fired it}.  The host sizes both parts from the log (one id per notify
// record, one listener per consensus ack), so neither can overflow.
constexpr int kConsHdr = 8;
constexpr int kConsLis = 5;
constexpr uint32_t kCombineConsensusAck = 4u;  // props_extend: updateConsensusProperty's re-combine
constexpr uint32_t kCombineConsensusLocal = 5u;  // props_extend: a local consensus (seq -1)
constexpr int64_t cons_words(int64_t n_ids, int64_t n_lis) { return kConsHdr + n_ids + kConsLis * n_lis; }

// checkpoint image of one document (u32 words): header + the used prefix of every LDS table
constexpr int kCkHdr = 32;
constexpr int64_t ck_words(int seg) { return 9ll * seg + 1024; }
// the words a checkpoint image uses: per slot len, canonical meta, block; per overlay entry slot,
// seq, removedSeq (32-bit relative), clients; per block parent, 8 children, count | leaf | scour,
// settled length; the heap
constexpr int64_t ck_used_words(int64_t slots, int64_t nu, int64_t blocks, int64_t hn) {
    return kCkHdr + 3 * slots + 4 * nu + 11 * blocks + 2 * (hn + 1);
}
// cold records per slot in HBM: {props, ovl, toff, tcap} and {seq, rseq, clientId | removedClientId
// << 16, pending-group mask (writers)} (the real seqs and client ids)
constexpr int kColdPerSlot = 2;
constexpr Caps class_caps(int seg) {
    // the overlay list (unsettled segments, ~100-200 at a lag <= 32) is sized to the collab window;
    // the largest classes, where a document with a wide window ends up, can hold half their slots
    if (is_giant_seg(seg))
        return Caps{seg, seg + seg * 3 / 10 + 24, seg * 3 / 10 + 24 + kGiantLdsBlocks, kGiantHeap, kGiantUlist, 0};
    if (seg > 65000)  // the HBM class
        return Caps{seg, seg + seg * 3 / 10 + 24, seg * 3 / 10 + 24, seg / 16 + 80, seg / 2, 0};
    // leaf blocks ~0.23 per slot, interior ~0.05 (fan-out 4..7); the overlay list holds at least 208
    // entries, so a document whose collab window keeps ~180 segments unsettled (config 2's widest, with
    // the 24-entry headroom) stays in the 16-per-CU class instead of finishing alone in a later launch
    return Caps{seg, seg + seg * 3 / 10 + 24, seg * 3 / 10 + 24, seg / 16 + 80,
                seg >= 3500 ? seg / 2 : (seg / 16 + 160 > 208 ? seg / 16 + 160 : 208), seg / 16 + 16};
}

// LDS layout of one document (byte offsets; every array 16-byte aligned)
struct Layout {
    uint32_t len, meta, sblk, ulist, usr, ucm;
    uint32_t bparent, bchild, bcount, bleaf, bscour, bslen, bacc, bep, heap, scratch, hdr, grec, pub, bytes;
};
constexpr int kHdrWords = 24;  // per-document scalars kept in LDS (mt_engine.hip LWord)
constexpr uint32_t lds_align(uint32_t x) { return (x + 15u) & ~15u; }
// The HBM class (tables in global memory) holds giant documents: 32-bit slot / block ids and
// segment lengths.  The LDS classes use 16-bit ones (a longer segment moves the document to the
// HBM class, cap_kind 8).
constexpr bool is_hbm_seg(int seg) { return seg > 65000; }
constexpr uint32_t len_bytes(int seg) { return is_hbm_seg(seg) ? 4u : 2u; }
constexpr uint32_t idx_bytes(int seg) { return is_hbm_seg(seg) ? 4u : 2u; }
// per-slot meta: 16 bits (7 flags + a 9-bit overlay-entry index) while the overlay list holds at most
// 510 entries, else 32 bits (mt_engine.hip SlotMeta)
constexpr uint32_t meta_bytes(int seg) { return !is_hbm_seg(seg) && class_caps(seg).ulist <= 510 ? 2u : 4u; }
// The giant class: make_layout is its HBM image (slot tables and the blocks of HBM ids; the LDS-
// resident parts get no room there) and make_glayout its LDS part.
constexpr Layout make_layout(int seg) {
    const Caps c = class_caps(seg);
    if (is_giant_seg(seg)) {
        Layout L{};
        uint32_t o = 0;
        L.len = o;     o = lds_align(o + 4u * c.seg);
        L.meta = o;    o = lds_align(o + 4u * c.seg);
        L.sblk = o;    o = lds_align(o + 4u * c.seg);
        L.bparent = o; o = lds_align(o + 4u * c.blk);
        L.bchild = o;  o = lds_align(o + 32u * c.blk);
        L.bcount = o;  o = lds_align(o + 1u * c.blk);
        L.bleaf = o;   o = lds_align(o + 1u * c.blk);
        L.bscour = o;  o = lds_align(o + 1u * c.blk);
        L.bslen = o;   o = lds_align(o + 4u * c.blk);
        L.bacc = o;    o = lds_align(o + 4u * c.blk);
        L.bep = o;     o = lds_align(o + 4u * c.blk);
        L.ulist = L.usr = L.ucm = L.heap = L.scratch = L.hdr = L.grec = o;  // in LDS (make_glayout)
        L.bytes = o;
        return L;
    }
    Layout L{};
    uint32_t o = 0;
    L.len = o;     o = lds_align(o + len_bytes(seg) * c.seg);
    L.meta = o;    o = lds_align(o + meta_bytes(seg) * c.seg);
    L.sblk = o;    o = lds_align(o + idx_bytes(seg) * c.seg);   // a free slot's s_blk links the free list
    L.ulist = o;   o = lds_align(o + idx_bytes(seg) * c.ulist);
    L.usr = o;     o = lds_align(o + (is_hbm_seg(seg) ? 8u : 4u) * c.ulist);
    L.ucm = o;     o = lds_align(o + 4u * c.ulist);
    L.bparent = o; o = lds_align(o + idx_bytes(seg) * c.blk);  // a free block's b_parent links the free list
    L.bchild = o;  o = lds_align(o + 8u * idx_bytes(seg) * c.blk);
    L.bcount = o;  o = lds_align(o + 1u * c.blk);
    L.bleaf = o;   o = lds_align(o + 1u * c.blk);
    L.bscour = o;  o = lds_align(o + 1u * c.blk);
    L.bslen = o;   o = lds_align(o + 4u * (c.iblk ? c.iblk : c.blk));  // interior blocks only (c.iblk)
    L.bacc = o;    o = lds_align(o + 4u * (c.iblk ? c.iblk : c.blk));
    L.bep = o;     o = lds_align(o + (is_hbm_seg(seg) ? 4u * c.blk : 0u));
    L.heap = o;    o = lds_align(o + 8u * (c.heap + 2));
    L.scratch = o; o = lds_align(o + 4u * 128);
    L.hdr = o;     o = lds_align(o + 4u * kHdrWords);
    L.grec = o;
    L.bytes = o;
    return L;
}

constexpr Layout make_glayout() {
    Layout L{};
    uint32_t o = 0;
    const uint32_t K = (uint32_t)kGiantLdsBlocks;
    L.hdr = o;     o = lds_align(o + 4u * kHdrWords);
    L.scratch = o; o = lds_align(o + 4u * 128);
    L.heap = o;    o = lds_align(o + 8u * (kGiantHeap + 2));
    L.ulist = o;   o = lds_align(o + 4u * kGiantUlist);
    L.usr = o;     o = lds_align(o + 8u * kGiantUlist);
    L.ucm = o;     o = lds_align(o + 4u * kGiantUlist);
    L.bparent = o; o = lds_align(o + 4u * K);
    L.bchild = o;  o = lds_align(o + 32u * K);
    L.bcount = o;  o = lds_align(o + 1u * K);
    L.bleaf = o;   o = lds_align(o + 1u * K);
    L.bscour = o;  o = lds_align(o + 1u * K);
    L.bslen = o;   o = lds_align(o + 4u * K);
    L.bacc = o;    o = lds_align(o + 4u * K);
    L.bep = o;     o = lds_align(o + 4u * K);
    L.grec = o;    o = lds_align(o + 4u * kGiantChainRec * kGiantUlist);  // the overlay's chain records
    L.pub = o;     o = lds_align(o + 4u * kGiantPubWords);  // the state the prefetch wave reads
    L.len = L.meta = L.sblk = o;  // in HBM (make_layout)
    L.bytes = o;
    return L;
}
static_assert(make_glayout().bytes <= 160u * 1024u - 256u, "giant class LDS");

// waves per SIMD a class's replay kernel must allow (its VGPR budget is 512 / this): the documents
// its LDS layout lets a CU hold, over 4 SIMDs (the HBM class: its launches hold a few documents)
constexpr int class_waves_per_eu(int seg) {
    if (is_hbm_seg(seg)) return 1;
    const uint32_t granules = (make_layout(seg).bytes + 1279u) / 1280u;
    int docs = (int)(128u / granules);
    if (docs > 16) docs = 16;
    return (docs + 3) / 4;
}

// matchProperties / rewrite tables of the interned property values (device memory, one per batch)
struct ValueTables {
    const uint8_t *flags;  // per value id: kVFalsy (rewrite semantics), kVIrregular, kVUnknown, kVNum, kVNever, kVSeqM1
    const uint32_t *cls;   // per value id: structural matchProperties class (mt_values.cpp)
    const uint64_t *exc;   // sorted (u << 32 | v): values matching across classes
    uint32_t n_values, n_exc;
    uint32_t nan_id;       // the NaN value (combine "incr"); 0xFFFFFFFF when the log has none
};

// kernel parameters
struct ReplayParams {
    const void *ops;              // mt_op[]
    const int64_t *doc_op_off;    // [n_docs+1]
    uint16_t *text;               // text heap (code units)
    const uint64_t *doc_text_base;
    const uint32_t *doc_text_len; // payload length (arena starts here)
    const uint32_t *doc_text_cap;
    uint32_t *pool;               // prop-set pool (words)
    const uint64_t *doc_pool_base;
    const uint32_t *doc_pool_cap;
    const void *props_in;         // mt_prop[] (op prop records, batch-global offsets)
    const ValueTables *vt;        // property value tables (device memory)
    OutRec *out;                  // [n_docs * out_cap]
    DocOut *doc_out;
    int64_t n_docs;               // workgroups in this launch
    int64_t doc_first;            // generator: global doc index of blockIdx.x == 0
    const int32_t *doc_list;      // non-null: blockIdx.x replays doc doc_list[blockIdx.x]
                                  // (capacity escalation); out/doc_out stay indexed by blockIdx.x
    int32_t out_cap;
    // generator mode (non-null gen): ops/text/props are written, not read
    const void *gen;              // mt_gen_params*
    void *gen_ops;                // mt_op[], document d's ops at doc_op_off[d]
    void *gen_props;              // mt_prop[], document d's records at 2 * doc_op_off[d]
    const int64_t *gen_doc_ids;   // per document: global index seeding its stream (null: doc_first + d)
    const int32_t *gen_doc_ops;   // per document: ops to generate (null: gen->n_ops)
    uint64_t *prof;               // MT_PROF builds: kProfSlots cycle counters per workgroup
    uint4 *cold;                  // [n_docs * cap.seg * kColdPerSlot] cold segment records
    // capacity escalation by checkpoint: a document short of LDS headroom writes its state to
    // ck_out[w] and stops; a later launch in a larger class resumes it from ck_in[ck_src[w]]
    uint32_t *ck_out;             // [n_docs * ck_words(SEG)] or null (largest class: no checkpoint)
    const uint32_t *ck_in;        // previous launch's checkpoints (null: fresh start)
    const int32_t *ck_src;        // per workgroup: index into ck_in / cold_in, -1: fresh start
    const uint4 *cold_in;         // previous launch's cold records
    int64_t ck_in_words;          // stride of ck_in
    int32_t cold_in_seg;          // stride of cold_in
    uint8_t *hbm_state;           // HBM class: per-workgroup table images (make_layout(kHbmSeg).bytes each)
    // MergeTree.idToSegment (mergeTree.ts:1098) per document, persistent across launches:
    // {marker-id key, slot} entries in mapping order (kIdUnlinked: the marker was unlinked)
    uint2 *idmap;
    const uint64_t *doc_idmap_base;
    // writer replicas (mt_writer_kernel_<SEG>): per-document pending-group regions (pend_words)
    uint32_t *pend;
    const uint64_t *doc_pend_base;
    int32_t pend_cap;             // entries per document
    uint32_t *regen;              // regenerated ops (kRegenOpWords layout), per document
    const uint64_t *doc_regen_base;
    int32_t regen_cap;            // words per document
    uint32_t *cons;               // consensus regions (cons_words layout), per document; null: none
    const uint64_t *doc_cons_base;
    // batches whose annotates touch referenceTileLabels / referenceRangeLabels: per output record,
    // the prop set a marker's leaf block last rebuilt its tile / range maps from (blockUpdate,
    // mergeTree.ts:2748-2767; annotates do not run it, so those maps go stale), else null
    uint32_t *lab_out;            // [n_docs * out_cap]
    // early escalation (a launch whose documents are expected to finish in its class): a document
    // that stops short of capacity anyway appends {workgroup + 1, launch | cap_kind << 24, ops_done,
    // max_oe} to this host-visible ring (slot from notice_count, device memory) once everything it
    // wrote is past its XCD's L2, so the host starts its next class while the launch still runs
    uint32_t *notice;             // host memory (4 words per entry), or null
    uint32_t *notice_count;
    int32_t launch_id;
    // writer replicas escalated early (mt_host.cpp poll_notices): their waves raise their issue
    // priority, so a replica outgrowing its first class replays beside that launch's waves at close
    // to its rate alone instead of becoming the step's tail
    int32_t urgent;
};
constexpr uint32_t kIdUnlinked = 0xFFFFFFFFu;
constexpr uint32_t kIdKeyUnsupported = 0xFFFFFFFFu;  // RELPOS key the host cannot resolve safely
constexpr int kProfSlots = 16;

// mt_digest.hip: per-document device digest of one launch's results
struct DigestParams {
    const OutRec *out;         // this launch's records [n * out_cap]
    const DocOut *doc_out;     // this launch's per-document results
    const int32_t *doc_list;   // workgroup -> document (null: identity)
    int64_t n;                 // workgroups of the launch
    int32_t out_cap;
    const uint16_t *text;
    const uint64_t *doc_text_base;
    const uint32_t *pool;
    const uint64_t *doc_pool_base;
    const uint8_t *final_mask; // per workgroup: 1 when this launch holds the document's final result
    uint64_t *dst;             // [n_docs]
};


// mt_snapshot.hip: SnapshotV1 (extractSync + emit) of one launch's documents on the GPU
constexpr int kSnapMaxChunks = 32;  // blobs per document (320k code units at chunk_size 10000)
constexpr int kSnapMeta = 1 + 3 * kSnapMaxChunks;  // per doc: n_chunks, then (count, length, bytes) per chunk
struct SnapParams {
    const OutRec *out;
    const DocOut *doc_out;
    const int32_t *doc_list;
    int64_t n;
    int32_t out_cap;
    const uint16_t *text;
    const uint64_t *doc_text_base;
    const uint32_t *pool;
    const uint64_t *doc_pool_base;
    const uint8_t *strs;        // UTF-8 bytes of the string tables below
    const uint32_t *key_str;    // per key: (offset, length) of JSON.stringify(key)
    const uint32_t *key_rank;   // per key: its array index, 0xFFFFFFFF for an ordinary key
    const uint32_t *val_str;    // per value: (offset, length) of its JSON text
    const uint32_t *cli_str;    // client table entries: (offset, length) of JSON.stringify(long id)
    const int32_t *doc_cli;     // per document: (first entry, count) in cli_str; null: the shared table
    int32_t cli_first, cli_n;   // the shared client table (entries 0, 1 of cli_str: "undefined", "original")
    const uint8_t *final_mask;  // per workgroup: 1 when this launch holds the document's final table
    int32_t n_keys, n_values;   // key_str has n_keys + 1 entries (the last is "?")
    const uint8_t *value_flags; // matchProperties of values (as ReplayParams)
    const uint32_t *value_class;
    const uint64_t *exc;
    uint32_t n_exc;
    int32_t chunk_size;
    int32_t pass;               // 0: sizes into meta / bytes, 1: write into dst
    int32_t *meta;              // [n_docs * kSnapMeta]
    int64_t *bytes;             // [n_docs] total bytes of the document's blobs (-1: not on the GPU)
    uint8_t *dst;
    const int64_t *dst_off;     // [n_docs]
    // per workgroup w, out_cap entries each: the sizing kernel stores every record's escaped text
    // bytes (rec_bytes[w * out_cap + record]) and every queued segment's framing bytes before / after
    // its text (seg_frame[2 * (w * out_cap + first record)] / [+1]); the writing kernel reads them
    // instead of sizing again (null: both kernels size)
    uint32_t *rec_bytes;
    uint32_t *seg_frame;
    // chunks beyond the meta row's kSnapMaxChunks: per document d, (count, length, bytes) triples at
    // chunk_ext[chunk_ext_off[d] ..chunk_ext_off[d + 1]) (null: kSnapMaxChunks at most)
    int32_t *chunk_ext;
    const int64_t *chunk_ext_off;
};

}  // namespace mt
