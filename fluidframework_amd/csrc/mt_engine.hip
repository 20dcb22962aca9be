// mt_engine.hip — MI355X (gfx950) batch replay of sequenced merge-tree ops.
//
// One 64-lane wavefront (= one workgroup) owns one document for the whole op log.  The
// document's merge-tree lives in LDS as the reference's own B-tree (MaxNodesInBlock = 8,
// mergeTree.ts:334): leaf blocks list segment slots, interior blocks list blocks, every
// child list is one 16-byte row that a wave reads with one lane per child.
//
//   s_*[slot]   length, flags + overlay-entry index (SlotMeta), leaf block: 6 B of LDS per slot.
//               A settled segment (below) needs nothing else for nodeLength: every valid view sees
//               its length, or 0 when removed.
//   u_*[entry]  the unsettled segments (the collab window's "hot" set, ~100-250 per document):
//               slot, 16-bit sequence numbers relative to a per-document base that follows minSeq
//               (seq16 | rseq16 << 16), client ids and the has-overlap flag.
//               The cold fields (prop-set id, removedClientOverlap, text offset/capacity, the real
//               seq / removedSeq and client ids for output) live in a per-document HBM table
//               `cold[2 * slot + {0,1}]` (2 x 16 B).
//   b_*[block]  children[8], count, parent, needsScour, and the block's SETTLED length.
//   heap        the zamboni heap (collections.ts:213-265), in VGPRs.
//
// Position resolution (PartialSequenceLengths, partialLengths.ts, in the reference) is a
// settled/unsettled split.  A segment is *settled* once seq <= minSeq and it is either not
// removed or removed at or below minSeq: every valid op view (refSeq >= minSeq) then sees
// exactly `len` (not removed) or 0 (removed) of it, so the block sums b_slen are view
// independent and maintained incrementally.  The few unsettled segments (inserted or
// removed inside the collab window) form the overlay: per op, every lane takes one of
// them, evaluates nodeLength (mergeTree.ts:1659-1699) for the op's (refSeq, clientId) and
// adds it into b_acc along its ancestor chain (LDS atomics).  A block's view length is then
// b_slen + b_acc, and insertingWalk (mergeTree.ts:2345-2474) / nodeMap (2903-2965) descend
// the tree level by level, one lane per child, with an 8-lane prefix scan per level —
// O(depth) LDS round trips per op instead of the O(segments) scans of a flat table.
// refSeq < minSeq (outside valid logs) falls back to an overlay over every segment with
// b_slen ignored, so block lengths stay the exact leaf sums either way.
//
// Block splits, pack and zamboni follow mergeTree.ts:1289-1478, 2476-2489 exactly, so
// leaf-block membership — and hence SnapshotV1 bytes — match the reference.
//
// No MFMA: the path is integer scan / tree work bound by LDS latency.

#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/mt_gen.h"
#include "../../include/mt_oplog.h"
#include "mt_device.h"

namespace mt {

#define MT_FI __device__ __attribute__((always_inline)) inline

// 1: the LDS classes also descend with descend_giant's walk (every child's row loaded in the round
// that loads the children's lengths: one dependent LDS round trip per level instead of two).
// Measured slower there (config 3, 8,192 documents, same box: 118.2M vs 122.5M ops/s — eight
// times the LDS reads per level, and the row permute, outweigh the round trip saved in LDS), so
// only the giant class, whose lower levels are HBM round trips, uses it.
#ifndef MT_DESCENT_ONE_ROUND
#define MT_DESCENT_ONE_ROUND 0
#endif

// 1: a scour's text appends of <= 64 code units are queued (up to 4) and issued together, so their
// HBM loads overlap instead of each waiting for the previous copy (0 = one copy at a time); giant
// class only (Engine::kTextBatch)
#ifndef MT_TEXT_BATCH
#define MT_TEXT_BATCH 1
#endif

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int32_t rfl(int32_t x) { return (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)x); }
__device__ __forceinline__ uint32_t rdl(uint32_t x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ int32_t rdl(int32_t x, int l) { return (int32_t)__builtin_amdgcn_readlane((uint32_t)x, l); }

// wave64 inclusive prefix sum on DPP (GFX9 row_shr + row_bcast): no LDS round trips
__device__ __forceinline__ uint32_t scan_incl(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}
// inclusive prefix sum over lanes 0..7 (one child row); other lanes hold garbage
__device__ __forceinline__ uint32_t scan8(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    return v;
}
// sum over each aligned group of 8 lanes (every lane of the group gets it)
__device__ __forceinline__ uint32_t sum8(uint32_t v) {
    v += (uint32_t)__shfl_xor((int)v, 1, 64);
    v += (uint32_t)__shfl_xor((int)v, 2, 64);
    v += (uint32_t)__shfl_xor((int)v, 4, 64);
    return v;
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int first_lane(uint64_t b) { return __builtin_ctzll(b); }

// Lane-to-lane ordering inside the single wave that owns a document.  A wavefront's LDS and
// vector-memory instructions execute and complete in program order (AMDGPU memory model:
// wavefront scope needs no waits), so only the compiler must be kept from reordering
// accesses across the point: no s_waitcnt, no s_barrier.
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void lds_add(uint32_t *p, uint32_t v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ uint32_t hash_pair(uint32_t k, uint32_t v) {
    uint32_t h = k * 0x9E3779B1u ^ (v + 0x7F4A7C15u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h | 1u;
}

// Phase cycle counters (MT_PROF builds only): 0 kernel, 1 descents, 2 split, 3 insert,
// 4 range walk, 5 zamboni, 6 overlay, 7 scour, 8 text, 9 heap, 10 pack, 11 settle, 12 the scour's
// wait for its cold records, 13 resolve_cold, 14 heap_forget, 15 unused
#ifdef MT_PROF
struct PfScope {
    uint64_t &acc;
    uint64_t t0;
    __device__ explicit PfScope(uint64_t &a) : acc(a), t0(clock64()) {}
    __device__ ~PfScope() { acc += clock64() - t0; }
};
#define PF_SCOPE(k) PfScope _pf_scope(pf[k])
#else
#define PF_SCOPE(k) (void)0
#endif

// result of a descent: leaf block, child index, view positions
struct Walk {
    int32_t blk;    // leaf block (-1: the walk found nothing)
    int32_t k;      // insert mode: insert before child k (k == n: at the block end)
    int32_t n;      // child count of blk
    uint32_t base;  // view position of the block start
    uint32_t excl;  // insert mode: view position before child k
    int32_t ok;     // insert mode: the walk found an insertion point
    uint32_t slot;  // insert mode, giant class: the slot of child k (k < n), from the walk's leaf row
};

// A per-document scalar kept in LDS instead of a scalar register: the engine's rarely used state
// (text / pool semispaces, GC counters, high-water marks) would otherwise be live in SGPRs across
// the whole op loop and spill.  Every lane reads / writes the same word.
template <typename T>
struct LWord {
    T *p;
    MT_FI operator T() const { return (T)rfl((uint32_t)*p); }
    MT_FI LWord &operator=(T v) {
        *p = v;
        return *this;
    }
    // assignment between words copies the value, never the address
    MT_FI LWord &operator=(const LWord &o) { return *this = T(o); }
    MT_FI LWord &operator+=(T v) { return *this = (T)(T(*this) + v); }
    MT_FI LWord &operator++(int) { return *this = (T)(T(*this) + 1); }
};

// A block table.  In the giant class block ids [0, kGiantLdsBlocks) live in the CU's LDS (the
// interior blocks near the root) and the rest in HBM: an access branches on the id to an LDS
// (ds_*) or a global (global_*) instruction — the pointers carry their address spaces, so no flat
// access (which would make every LDS access wait for the wave's outstanding HBM traffic).  Every
// other class has one base.  kShift: log2 of the entries per block (b_child: 8).
#define MT_AS_LDS __attribute__((address_space(3)))
#define MT_AS_GLOBAL __attribute__((address_space(1)))
template <typename T, int kShift, bool kSplit>
struct BArr;
template <typename T, int kShift>
struct BArr<T, kShift, false> {
    T *p;
    MT_FI T &operator[](uint32_t i) const { return p[i]; }
    MT_FI void add(uint32_t i, T v) const { __hip_atomic_fetch_add(&p[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT); }
};
template <typename T, int kShift>
struct BArr<T, kShift, true> {
    MT_AS_LDS T *lds;   // entries of the LDS-resident ids
    MT_AS_GLOBAL T *p;  // the HBM table, indexed by the full id (ids below kGiantLdsBlocks unused)
    MT_FI static bool in_lds(uint32_t i) { return (i >> kShift) < (uint32_t)kGiantLdsBlocks; }
    struct Ref {
        const BArr &a;
        uint32_t i;
        MT_FI operator T() const {
            if (in_lds(i)) return a.lds[i];
            return a.p[i];
        }
        MT_FI Ref &operator=(T v) {
            if (in_lds(i)) a.lds[i] = v;
            else a.p[i] = v;
            return *this;
        }
        MT_FI Ref &operator=(const Ref &o) { return *this = (T)o; }
    };
    MT_FI Ref operator[](uint32_t i) const { return Ref{*this, i}; }
    MT_FI void add(uint32_t i, T v) const {
        if (in_lds(i)) __hip_atomic_fetch_add(&lds[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        else __hip_atomic_fetch_add(&p[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
};

// kW: a writer replica (the local-client path: local ops with UnassignedSequenceNumber, pending
// segment groups acked by the replica's own sequenced messages); compiled as mt_writer_kernel_<SEG>
// so the observer kernels carry none of it
// kBig: property sets past one pair per lane (props_extend_big) — compiled into the writer, load
// and mt_bigprops_kernel_<SEG> kernels and the spill classes; the observer replay kernels of the LDS
// classes stop such a document with cap_kind 3 (kCapPool) and the host re-runs it in the bigprops
// kernel, so their op loop carries none of it (its registers are the replay's bound)
template <int SEG, bool kW = false, bool kBigK = false>
struct Engine {
    static constexpr bool kBig = kW || kBigK || is_hbm_seg(SEG);
    static constexpr Caps cap = class_caps(SEG);
    static constexpr Layout lay = make_layout(SEG);
    using Len = std::conditional_t<len_bytes(SEG) == 2u, uint16_t, uint32_t>;
    // slot and block ids: 16-bit in the LDS classes, 32-bit in the HBM class (giant documents)
    using Idx = std::conditional_t<idx_bytes(SEG) == 2u, uint16_t, uint32_t>;
    static constexpr uint32_t kNoBlk = idx_bytes(SEG) == 2u ? 0xFFFFu : 0xFFFFFFFFu;
    static constexpr bool kHbm = is_hbm_seg(SEG);
    static constexpr bool kGiant = is_giant_seg(SEG);
    // batched text appends in the giant class only: measured on one box, config 3 at 8,192 documents
    // with batching in the classes of <= 2 waves per SIMD 119.9M vs 122.0M ops/s (a scour rarely
    // merges more than one leaf, so the queue only adds instructions; the 128-VGPR classes spill
    // with it), the giant class 20.81 vs 21.24 us per op (profiles/r03_ab_experiments.json)
    static constexpr bool kTextBatch = MT_TEXT_BATCH && kGiant;
    static constexpr Layout glay = make_glayout();
    template <typename T, int kShift = 0>
    using BA = BArr<T, kShift, kGiant>;
    static constexpr uint32_t kMaxLen = len_bytes(SEG) == 2u ? 0xFFFFu : 0xFFFFFFFFu;
    // Block pools.  LDS classes: leaf blocks take ids [0, kLB), interior blocks [kLB, cap.blk); only
    // interior blocks keep settled / overlay lengths (b_slen, b_acc indexed by si(id)) — a leaf
    // block's length is the sum over its <= 7 leaves, evaluated where a walk needs it.  The giant and
    // HBM classes keep full-size tables (leaf entries unused) and their own pools.
    static constexpr bool kSplitPools = cap.iblk > 0;
    static constexpr int32_t kLB = kSplitPools ? cap.blk - cap.iblk : 0;
    MT_FI static uint32_t si(uint32_t b) { return kSplitPools ? b - (uint32_t)kLB : b; }
    // SlotMeta: 7 flags above a kUB-bit index of the slot's overlay entry (kUNone: settled)
    using Meta = std::conditional_t<meta_bytes(SEG) == 2u, uint16_t, uint32_t>;
    static constexpr int kUB = 8 * (int)sizeof(Meta) - 7;
    static constexpr uint32_t kUNone = (1u << kUB) - 1u;
    static constexpr uint32_t kFLinked = 1u << kUB, kFMarker = 2u << kUB, kFEndsNL = 4u << kUB,
                              kFHasProps = 8u << kUB, kFHasNL = 16u << kUB, kFRemoved = 32u << kUB,
                              kFPending = 64u << kUB;
    static_assert(cap.ulist < (int32_t)kUNone, "overlay-entry index");
    // u_cm: clientId | removedClientId << kCmR | has-overlap (15-bit short ids)
    static constexpr int kCmR = 15;
    static constexpr uint32_t kCmOvl = 1u << 30;
    // an overlay entry's sequence numbers relative to sbase: seq | removedSeq << kRB, 16-bit each in
    // the LDS classes (a collab window of kSeq16Span ops or more moves the document to a spill
    // class), 32-bit in the giant and HBM classes (no window limit)
    using USr = std::conditional_t<kHbm, uint64_t, uint32_t>;
    static constexpr int kRB = kHbm ? 32 : 16;
    static constexpr uint32_t kRMask = kHbm ? 0xFFFFFFFFu : 0xFFFFu;
    static constexpr uint32_t kRNone = kRMask;             // removedSeq === undefined
    static constexpr uint32_t kRUnassigned = kRMask - 1u;  // a pending local insert / remove
    MT_FI static uint32_t us_q(USr x) { return (uint32_t)x & kRMask; }
    MT_FI static uint32_t us_r(USr x) { return (uint32_t)(x >> kRB); }
    MT_FI static USr us_make(uint32_t q, uint32_t r) { return (USr)q | ((USr)r << kRB); }
    // ---- LDS state
    Len *s_len;
    Meta *s_meta;  // flags | overlay-entry index; a free slot: kUNone
    Idx *s_blk;    // leaf block; of a free slot: the next free slot (kNoBlk ends the list)
    Idx *u_list;   // overlay entries: exactly the unsettled slots, unordered
    USr *u_sr;       // seq | rseq << kRB, relative to sbase (kRNone: not removed)
    uint32_t *u_cm;  // clientId | removedClientId << kCmR | kCmOvl
    BA<Idx> b_parent;  // b_parent of a free block links the free block list
    BA<Idx, 3> b_child;
    BA<uint8_t> b_count, b_leaf;
    BA<int8_t> b_scour;
    BA<uint32_t> b_slen, b_acc;
    BA<uint32_t> b_ep;   // HBM / giant class: the overlay epoch that last wrote b_acc[B] (no O(blocks) clear)
    uint32_t ov_epoch;
    // giant class: the HBM-resident blocks the last overlay added into (kGiantChainRec per overlay
    // list entry, kNoBlk-padded); their b_acc is zeroed before the next overlay, so HBM b_acc needs
    // no epoch tags (a zero invariant between overlays) and the adds are fire-and-forget atomics
    uint32_t *g_rec;
    int32_t g_nrec;
    uint32_t *scratch;  // 128 words
    // ---- uniform scalars
    int32_t slot_top, free_head, free_n, blk_top, n_bfree, bfree_head, root, depth, hn, nu;
    // giant class: the LDS-resident block ids [0, lds_top) and their free list (blk_top / bfree_head
    // are the HBM ids, from kGiantLdsBlocks)
    int32_t lds_top, n_lfree, lfree_head;
    int32_t min_seq, cur_seq, status, settled_min;
    int32_t sbase;  // the overlay entries' 16-bit sequence numbers are relative to sbase (<= minSeq)
    int32_t splits;                 // leaf/interior block splits so far (overlay staleness)
    int32_t ov_splits, ov_full;     // overlay computed at `ov_splits`; full (refSeq < minSeq) mode
    uint32_t arena_top, pool_top;
    // text: payload | semispace A | semispace B; prop pool: [0] reserved | A | B (LDS words)
    LWord<uint32_t> pay_end, arena_base, arena_end, semi_t, pool_base, pool_end, semi_p;
    LWord<int32_t> pool_gcs, text_gcs;
    // Splits of the current op (at most two): the cold records of both halves and the left
    // half's ends-with-'\n' are resolved after the op's LDS work, so the HBM latency of the
    // cold-record and text loads overlaps it.  A pending split's two cold records are held
    // lane-distributed (lane i < 8: word i) in one VGPR, so they cost no scalar registers.
    int32_t pend_n, pend_cold;
    LWord<uint32_t> ps0, pn0, pr0, pch0, ps1, pn1, pr1, pch1;
    uint32_t pv0, pv1;
    LWord<int32_t> max_heap, max_u;
    // marker ids (idToSegment) and the positions an MT_OP_RELPOS record resolved for the next op
    LWord<int32_t> idmap_n, rel_pend, rel_p1, rel_p2;
    uint2 *idmap;
    // writer replicas: the document's pending-group region (mt_device.h kPendDesc / pend_entries)
    // and its group count (kept in HBM word 0 as well, so checkpoints carry it)
    uint32_t *pend;
    int32_t pend_cap_e, n_pend;
    uint32_t *regen;  // regenerated ops (mt_device.h kRegenOpWords), regen_cap words
    int32_t regen_cap;
    // writer consensus: the document's region (mt_device.h kConsHdr; null: the batch has none), the
    // seq of its oldest unfired min-seq listener (INT32_MAX: none), and the marker id a local notify
    // RELPOS hands to the annotate after it
    uint32_t *cons;
    int32_t cons_next, ntf;
    uint32_t ntf_raw;
    int32_t htop;
    uint2 *h_ent;
    // ---- global
    uint4 *cold;  // cold segment records {props, ovl, toff, tcap}
    uint16_t *text;
    uint32_t text_cap;
    uint32_t *pool;
    uint32_t pool_cap;
    const mt_prop *props_in;
    const ValueTables *vt;  // value flags / classes / exceptions (scalar loads where used)
    int lane;
    // label tracking (ReplayParams.lab_out): a Marker's cold.w (its text capacity otherwise, unused
    // by markers) holds the prop set its leaf block's last blockUpdate read the tile / range labels
    // from; lab_refresh runs where the reference runs blockUpdate on a leaf block
    bool lab;
    LWord<int32_t> cap_kind;
#ifdef MT_PROF
    uint64_t pf[kProfSlots];
#endif

    // ------------------------------------------------------------------ layout
    // tb: the document's tables (LDS, or the HBM image of the HBM / giant class); lb: the giant
    // class's LDS part (make_glayout)
    MT_FI void carve(uint8_t *tb, uint8_t *lb) {
        s_len = (Len *)(tb + lay.len);
        s_meta = (Meta *)(tb + lay.meta);
        s_blk = (Idx *)(tb + lay.sblk);
        uint8_t *xb = kGiant ? lb : tb;  // the per-op state: in LDS for the giant class
        const Layout &xl = kGiant ? glay : lay;
        u_list = (Idx *)(xb + xl.ulist);
        u_sr = (USr *)(xb + xl.usr);
        u_cm = (uint32_t *)(xb + xl.ucm);
        b_parent.p = (decltype(b_parent.p))(tb + lay.bparent);
        b_child.p = (decltype(b_child.p))(tb + lay.bchild);
        b_count.p = (decltype(b_count.p))(tb + lay.bcount);
        b_leaf.p = (decltype(b_leaf.p))(tb + lay.bleaf);
        b_scour.p = (decltype(b_scour.p))(tb + lay.bscour);
        b_slen.p = (decltype(b_slen.p))(tb + lay.bslen);
        b_acc.p = (decltype(b_acc.p))(tb + lay.bacc);
        b_ep.p = (decltype(b_ep.p))(tb + lay.bep);
        if constexpr (kGiant) {
            b_parent.lds = (MT_AS_LDS Idx *)(lb + glay.bparent);
            b_child.lds = (MT_AS_LDS Idx *)(lb + glay.bchild);
            b_count.lds = (MT_AS_LDS uint8_t *)(lb + glay.bcount);
            b_leaf.lds = (MT_AS_LDS uint8_t *)(lb + glay.bleaf);
            b_scour.lds = (MT_AS_LDS int8_t *)(lb + glay.bscour);
            b_slen.lds = (MT_AS_LDS uint32_t *)(lb + glay.bslen);
            b_acc.lds = (MT_AS_LDS uint32_t *)(lb + glay.bacc);
            b_ep.lds = (MT_AS_LDS uint32_t *)(lb + glay.bep);
        }
        h_ent = (uint2 *)(xb + xl.heap);
        scratch = (uint32_t *)(xb + xl.scratch);
        if constexpr (kGiant) g_rec = (uint32_t *)(lb + glay.grec);  // make_glayout: the chain records
        uint32_t *hw = (uint32_t *)(xb + xl.hdr);
        pay_end.p = hw + 0;
        arena_base.p = hw + 1;
        arena_end.p = hw + 2;
        semi_t.p = hw + 3;
        pool_base.p = hw + 4;
        pool_end.p = hw + 5;
        semi_p.p = hw + 6;
        pool_gcs.p = (int32_t *)hw + 7;
        text_gcs.p = (int32_t *)hw + 8;
        max_heap.p = (int32_t *)hw + 9;
        max_u.p = (int32_t *)hw + 10;
        cap_kind.p = (int32_t *)hw + 11;
        ps0.p = hw + 12;
        pn0.p = hw + 13;
        pr0.p = hw + 14;
        pch0.p = hw + 15;
        ps1.p = hw + 16;
        pn1.p = hw + 17;
        pr1.p = hw + 18;
        pch1.p = hw + 19;
        idmap_n.p = (int32_t *)hw + 20;
        rel_pend.p = (int32_t *)hw + 21;
        rel_p1.p = (int32_t *)hw + 22;
        rel_p2.p = (int32_t *)hw + 23;
    }

    MT_FI void set_fail(int32_t st) {
        if (status == ST_OK) status = st;
    }
    MT_FI void cap_fail(int32_t kind) {
        if (status == ST_OK) {
            status = ST_CAPACITY;
            cap_kind = kind;
        }
    }

    // ------------------------------------------------------------------ init
    MT_FI void init() {
        slot_top = 0;
        free_head = -1;
        free_n = 0;
        blk_top = kGiant ? kGiantLdsBlocks : 0;
        n_bfree = 0;
        bfree_head = -1;
        lds_top = 0;
        n_lfree = 0;
        lfree_head = -1;
        sbase = 0;
        clear_epochs();
        hn = 0;
        nu = 0;
        min_seq = 0;
        cur_seq = 0;
        settled_min = 0;
        status = ST_OK;
        cap_kind = 0;
        pend_n = 0;
        pend_cold = 0;
        splits = 0;
        ov_splits = -1;
        ov_full = 0;
        max_heap = 0;
        max_u = 0;
        idmap_n = 0;
        rel_pend = 0;
        // initialNode (mergeTree.ts:1125): an empty root leaf block
        root = alloc_block(1, 0);
        depth = 1;
        // heap entry 0 is the sentinel LRUSegmentComparer.min = { maxSeq: -2 } (never compared);
        // its 8 bytes hold the SnapshotLoader's batch state (insert position, batch open), so
        // checkpoints carry it and the replay kernel keeps no registers for it
        htop = kNoneSeq;
        if (lane == 0) h_ent[0] = make_uint2(0u, 0u);
        wsync();
    }

    // ------------------------------------------------------------------ allocation
    MT_FI int32_t alloc_slot() {
        int32_t s;
        if (free_head >= 0) {
            s = free_head;
            const uint32_t nx = rfl((uint32_t)s_blk[s]);
            free_head = nx == kNoBlk ? -1 : (int32_t)nx;
            free_n--;
        } else {
            if (slot_top >= cap.seg) {
                cap_fail(1);
                return -1;
            }
            s = slot_top++;
        }
        return s;
    }
    // level: the block's height above the leaf blocks (0: a leaf block; a block's level never changes)
    MT_FI int32_t alloc_block(int leaf, int32_t level) {
        int32_t b;
        if (kSplitPools && level >= 1) {  // the interior pool
            if (n_lfree > 0) {
                b = lfree_head;
                lfree_head = (int32_t)rfl((uint32_t)b_parent[b]);
                if (lfree_head == (int32_t)kNoBlk) lfree_head = -1;
                n_lfree--;
            } else if (lds_top < cap.iblk) {
                b = kLB + lds_top++;
            } else {
                cap_fail(1);
                return kLB;
            }
        } else if (kGiant && level >= kGiantLdsLevel && (n_lfree > 0 || lds_top < kGiantLdsBlocks)) {
            if (n_lfree > 0) {
                b = lfree_head;
                lfree_head = (int32_t)rfl((uint32_t)b_parent[b]);
                if (lfree_head == (int32_t)kNoBlk) lfree_head = -1;
                n_lfree--;
            } else {
                b = lds_top++;
            }
        } else if (n_bfree > 0) {
            b = bfree_head;
            bfree_head = (int32_t)rfl((uint32_t)b_parent[b]);
            if (bfree_head == (int32_t)kNoBlk) bfree_head = -1;
            n_bfree--;
        } else {
            const int32_t top = kSplitPools ? kLB : cap.blk;
            if (blk_top >= top || (uint32_t)blk_top >= kNoBlk) {
                cap_fail(1);
                return 0;
            }
            b = blk_top++;
        }
        b_leaf[b] = (uint8_t)leaf;
        b_count[b] = 0;
        b_scour[b] = kScourUndef;
        b_parent[b] = (Idx)kNoBlk;
        if (!kSplitPools || !leaf) b_slen[si(b)] = 0;
        return b;
    }
    // the second pool: interior ids (LDS classes) / LDS-resident ids (giant class)
    MT_FI static bool in_second_pool(int32_t b) { return kSplitPools ? b >= kLB : (kGiant && b < kGiantLdsBlocks); }
    MT_FI void free_block(int32_t b) {
        if (in_second_pool(b)) {
            b_parent[b] = (Idx)(lfree_head < 0 ? (int32_t)kNoBlk : (int32_t)lfree_head);
            lfree_head = b;
            n_lfree++;
            return;
        }
        b_parent[b] = (Idx)(bfree_head < 0 ? (int32_t)kNoBlk : (int32_t)bfree_head);
        bfree_head = b;
        n_bfree++;
    }

    // ------------------------------------------------------------------ visibility
    // seq relative to sbase, clamped at 0 (a value below the base is <= every valid refSeq)
    MT_FI uint32_t rel(int32_t q) const {
        const int32_t d = q - sbase;
        return d <= 0 ? 0u : (uint32_t)d;
    }
    // removedClientOverlap membership (addOverlappingClient, mergeTree.ts:2544-2552): a bit mask
    // of clients < 31 in cold.y, else a client list in the pool
    __device__ __forceinline__ bool ovl_has(uint32_t slot, uint32_t c) const {
        const uint32_t o = cold[2 * slot].y;
        if (!(o & kOvlList)) return c < kOvlMaskClients && ((o >> c) & 1u);
        const uint32_t *r = pool + (o & ~kOvlList);
        const uint32_t n = r[0] & ~kPoolOvlTag;
        bool hit = false;
        for (uint32_t i = 0; i < n; i++) hit |= r[2 + i] == c;
        return hit;
    }
    // nodeLength of one leaf for (refSeq, clientId) + breakTie's leaf rule (mergeTree.ts:2248-2277).
    // Valid views (refSeq >= minSeq >= sbase): a settled leaf is seen whole (or not at all when
    // removed) by every one of them; an unsettled leaf's overlay entry holds its 16-bit relative seqs
    // and client ids.  A view below minSeq (outside valid logs) reads the real seqs and client ids from
    // the cold records.
    __device__ __forceinline__ void view_of(uint32_t slot, int32_t ref, uint32_t c, uint32_t &vlen, bool &tie) const {
        const uint32_t meta = s_meta[slot];
        const uint32_t len = s_len[slot];
        bool vis, rle, rem;
        bool pending = false;  // writer: an unacked local insert (seq === UnassignedSequenceNumber)
        if (ref >= min_seq) {
            const uint32_t ui = meta & kUNone;
            if (ui == kUNone) {
                const bool rm = (meta & kFRemoved) != 0u;
                vlen = rm ? 0u : len;
                tie = !rm;
                return;
            }
            const USr sr = u_sr[ui];
            const uint32_t cm = u_cm[ui];
            const uint32_t rr = (uint32_t)(ref - sbase);
            vis = ((cm & kMetaCli) == c) || (us_q(sr) <= rr);
            rle = us_r(sr) <= rr;
            if constexpr (kW) pending = us_q(sr) == kRUnassigned;
            rem = (((cm >> kCmR) & kMetaCli) == c) || rle;
            if (!rem && (cm & kCmOvl)) rem = ovl_has(slot, c);
        } else {
            const uint4 q = cold[2 * slot + 1];
            const uint32_t cli = q.z & kMetaCli, rcli = (q.z >> 16) & kMetaCli;
            if constexpr (kW) {
                pending = (int32_t)q.x == kUnassignedSeq;
                vis = (cli == c) || (!pending && (int32_t)q.x <= ref);
                rle = (int32_t)q.y != kUnassignedSeq && (int32_t)q.y <= ref;
            } else {
                vis = (cli == c) || ((int32_t)q.x <= ref);
                rle = (int32_t)q.y <= ref;
            }
            rem = (rcli == c) || rle;
            if (!rem && (meta & kFRemoved)) rem = ovl_has(slot, c);
        }
        vlen = (vis && !rem) ? len : 0u;
        // breakTie's leaf rule: a remote op does not insert before a pending local segment; the
        // local client breaks every tie it reaches (mergeTree.ts:2263-2271)
        tie = !rle && (!kW || c == 0u || !pending);
    }
    MT_FI static bool is_settled(uint32_t meta) { return (meta & kUNone) == kUNone; }
    // a leaf's contribution to the settled block sums
    __device__ __forceinline__ uint32_t settled_len(uint32_t slot) const {
        const uint32_t meta = s_meta[slot];
        return (is_settled(meta) && !(meta & kFRemoved)) ? s_len[slot] : 0u;
    }
    // canonical relative seq of a checkpoint image (32-bit; 0xFFFFFFFF none, 0xFFFFFFFE unassigned)
    MT_FI static uint32_t canon_rel(uint32_t r) { return r >= kRUnassigned ? r - kRMask + 0xFFFFFFFFu : r; }
    MT_FI static uint32_t uncanon_rel(uint32_t r) { return r >= 0xFFFFFFFEu ? r - 0xFFFFFFFFu + kRMask : r; }
    // canonical meta of a checkpoint image (mt_device.h kCanonNoEntry) and back
    MT_FI static uint32_t meta_canon(uint32_t m) {
        const uint32_t i = m & kUNone;
        return (i == kUNone ? kCanonNoEntry : i) | ((m >> kUB) << 24);
    }
    MT_FI static uint32_t meta_uncanon(uint32_t c) {
        const uint32_t i = c & kCanonNoEntry;
        return (i == kCanonNoEntry ? kUNone : i) | ((c >> 24) << kUB);
    }
    // the OutRec meta word of a slot (client ids from the cold record)
    MT_FI static uint32_t meta_out(uint32_t m, uint32_t clients, uint32_t ovl) {
        uint32_t r = (clients & kMetaCli) | (((clients >> 16) & kMetaCli) << kMetaRcliShift);
        if (m & kFMarker) r |= kMetaMarker;
        if (ovl) r |= kMetaHasOvl;
        return r;
    }
    // nodeLength of the unsettled segment of overlay entry j (slot) in a valid view (refSeq >= minSeq)
    __device__ __forceinline__ uint32_t view_entry(uint32_t j, uint32_t slot, int32_t ref, uint32_t c) const {
        const USr sr = u_sr[j];
        const uint32_t cm = u_cm[j];
        const uint32_t len = s_len[slot];
        const uint32_t rr = (uint32_t)(ref - sbase);
        const bool vis = ((cm & kMetaCli) == c) || (us_q(sr) <= rr);
        bool rem = (((cm >> kCmR) & kMetaCli) == c) || (us_r(sr) <= rr);
        if (!rem && (cm & kCmOvl)) rem = ovl_has(slot, c);
        return (vis && !rem) ? len : 0u;
    }

    // ------------------------------------------------------------------ ancestor chains
    // every active lane adds v into arr[si(B)] for the interior blocks B on the chain above leaf block
    // b (all leaves sit at depth - 1, so the walk is depth - 1 uniform steps)
    template <typename Arr>
    MT_FI void chain_add(Arr &arr, bool act, uint32_t b, uint32_t v) {
        if (act) b = b_parent[b];
        for (int32_t l = 1; l < depth; l++) {
            if (act && b != kNoBlk) {
                arr.add(si(b), v);
                b = b_parent[b];
            }
        }
    }
    // uniform: b_slen += v on the interior chain above leaf block b
    MT_FI void chain_add_uniform(int32_t b, uint32_t v) {
        wsync();
        b = b_parent[b];
        while (b != (int32_t)kNoBlk) {
            uint32_t x = b_slen[si(b)];
            int32_t p = b_parent[b];
            b_slen[si(b)] = x + v;
            b = p;
        }
        wsync();
    }

    // the overlay's b_acc: in the HBM class a block first touched in this epoch is reset before
    // the adds (every lane of a shared block writes the same reset)
    MT_FI void ov_chain_add(bool act, uint32_t b, uint32_t v) {
        if constexpr (kHbm) {
            uint32_t c = act ? (uint32_t)b_parent[b] : kNoBlk;
            for (int32_t l = 1; l < depth; l++) {
                if (act && c != kNoBlk) {
                    if (b_ep[c] != ov_epoch) {
                        b_acc[c] = 0u;
                        b_ep[c] = ov_epoch;
                    }
                    c = b_parent[c];
                }
            }
            wsync();
        }
        chain_add(b_acc, act, b, v);
    }
    MT_FI void clear_epochs() {
        ov_epoch = 0;
        if constexpr (kGiant) {  // once per launch: LDS epochs, and the zero invariant of HBM b_acc
            for (int32_t i = lane; i < kGiantLdsBlocks; i += kWave) b_ep.lds[i] = 0xFFFFFFFFu;
            g_nrec = 0;
            giant_clear_acc(true);
        } else if constexpr (kHbm) {  // once per launch: the tables are uninitialised device memory
            for (int32_t i = lane; i < cap.blk; i += kWave) b_ep[i] = 0xFFFFFFFFu;
            wsync();
        }
    }
    // an interior block's overlay length
    MT_FI uint32_t ov_acc(uint32_t b) const {
        if constexpr (kGiant) {
            if (b < (uint32_t)kGiantLdsBlocks) return b_ep.lds[b] == ov_epoch ? b_acc.lds[b] : 0u;
            return b_acc.p[b];  // zero unless the current overlay added into it
        }
        if constexpr (kHbm) return b_ep[b] == ov_epoch ? b_acc[b] : 0u;
        return b_acc[si(b)];
    }
    // an interior block's view length (settled sum + overlay)
    MT_FI uint32_t iview(uint32_t b) const { return ov_acc(b) + (ov_full ? 0u : b_slen[si(b)]); }
    // giant class: zero the HBM b_acc entries the last overlay wrote (and every one, once per
    // launch, when `all`: the tables are uninitialised device memory)
    MT_FI void giant_clear_acc(bool all) {
        if (all) {
            for (int32_t i = kGiantLdsBlocks + lane; i < cap.blk; i += kWave) b_acc.p[i] = 0u;
        } else {
            for (int32_t i = lane; i < g_nrec; i += kWave) {
                const uint32_t r = g_rec[i];
                if (r != kNoBlk) b_acc.p[r] = 0u;
            }
        }
        g_nrec = 0;
        wsync();
    }

    // giant class: the overlay of up to 4 x 64 list entries at once (their HBM loads — fields, leaf
    // block, parents — overlap); LDS-resident blocks accumulate in LDS (epoch-tagged), HBM ones with
    // fire-and-forget atomics on a zeroed b_acc, recorded for the next clear

    MT_FI void overlay_giant(int32_t ref, uint32_t c) {
        giant_clear_acc(false);
        ov_epoch++;
        ov_full = ref < min_seq;
        if (ov_full) {  // a view below minSeq (outside valid logs): every segment — the HBM class
            cap_fail(1);
            return;
        }
        for (int32_t g0 = 0; g0 < nu; g0 += 4 * kWave) {
            uint32_t slot[4], vlen[4], b[4], nh[4];
            bool act[4];
            int32_t wk[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int32_t j = g0 + k * kWave + lane;
                act[k] = j < nu;
                wk[k] = act[k] ? j : -1;
                slot[k] = act[k] ? (uint32_t)u_list[j] : 0u;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                vlen[k] = 0;
                b[k] = kNoBlk;
                nh[k] = 0;
                if (act[k]) {
                    vlen[k] = view_entry((uint32_t)wk[k], slot[k], ref, c);
                    b[k] = s_blk[slot[k]];
                }
                act[k] = act[k] && vlen[k] > 0u;
            }
#pragma unroll
            for (int k = 0; k < 4; k++)  // the chain starts above the leaf block (interior blocks only)
                if (act[k]) b[k] = b_parent[b[k]];
            for (int32_t l = 1; l < depth; l++) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (!act[k] || b[k] == kNoBlk) continue;
                    if (b[k] < (uint32_t)kGiantLdsBlocks) {
                        if (b_ep.lds[b[k]] != ov_epoch) {
                            b_acc.lds[b[k]] = 0u;
                            b_ep.lds[b[k]] = ov_epoch;
                        }
                    }
                }
                wsync();
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (!act[k] || b[k] == kNoBlk) continue;
                    if (b[k] < (uint32_t)kGiantLdsBlocks) {
                        __hip_atomic_fetch_add(&b_acc.lds[b[k]], vlen[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                    } else {
                        __hip_atomic_fetch_add(&b_acc.p[b[k]], vlen[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        if (nh[k] < (uint32_t)kGiantChainRec) g_rec[wk[k] * kGiantChainRec + nh[k]] = b[k];
                        nh[k]++;
                    }
                }
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (act[k] && b[k] != kNoBlk) b[k] = b_parent[b[k]];
            }
            bool over = false;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (wk[k] >= 0)
                    for (uint32_t q = act[k] ? nh[k] : 0u; q < (uint32_t)kGiantChainRec; q++) g_rec[wk[k] * kGiantChainRec + q] = kNoBlk;
                over |= act[k] && nh[k] > (uint32_t)kGiantChainRec;
            }
            if (ballot(over)) cap_fail(1);  // more HBM blocks on a chain than recorded: the HBM class
        }
        g_nrec = nu * kGiantChainRec;
        ov_splits = splits;
        wsync();
    }

    // blockUpdate of leaf block blk (mergeTree.ts:2748-2767): its markers' tile / range maps read the
    // current labels (label tracking only)
    MT_FI void lab_refresh(int32_t blk) {
        if (!lab) return;
        const int32_t n = b_count[blk];
        if (lane < n) {
            const uint32_t sl = b_child[blk * 8 + lane];
            if (s_meta[sl] & kFMarker) cold[2 * sl].w = cold[2 * sl].x;
        }
        wsync();
    }
    // a new segment's two cold records {props, no overlap, text offset, text capacity} and {seq,
    // removedSeq, client ids, no pending groups}: one dword per lane 0-7, a single 32-byte store
    MT_FI void cold_init(uint32_t slot, uint32_t props, uint32_t toff, uint32_t tcap, uint32_t seq, uint32_t rseq,
                         uint32_t clients) {
        uint32_t v = 0u;
        v = lane == 0 ? props : v;
        v = lane == 2 ? toff : v;
        v = lane == 3 ? tcap : v;
        v = lane == 4 ? seq : v;
        v = lane == 5 ? rseq : v;
        v = lane == 6 ? clients : v;
        if (lane < 8) reinterpret_cast<uint32_t *>(cold + 2 * slot)[lane] = v;
    }
    // a new overlay entry for `slot` (its meta word gets the entry's index)
    MT_FI void u_push(uint32_t slot, USr sr, uint32_t cm) {
        if (nu >= cap.ulist) {
            cap_fail(1);
            return;
        }
        u_list[nu] = (Idx)slot;
        u_sr[nu] = sr;
        u_cm[nu] = cm;
        s_meta[slot] = (Meta)((s_meta[slot] & ~kUNone) | (uint32_t)nu);
        nu++;
        if (nu > max_u) max_u = nu;
        wsync();
    }

    // Per-op overlay: b_acc[B] = sum of nodeLength(refSeq, c) over the unsettled segments under
    // B (or over all segments in full mode).
    MT_FI void overlay(int32_t ref, uint32_t c) {
        PF_SCOPE(6);
        if constexpr (kGiant) {
            overlay_giant(ref, c);
            return;
        }
        wsync();
        if constexpr (kHbm) {
            ov_epoch++;  // blocks of other epochs read as 0 (giant documents: ~10^5 blocks)
        } else {
            for (int32_t i = lane; i < (kSplitPools ? lds_top : blk_top); i += kWave) b_acc[i] = 0u;
        }
        wsync();
        ov_full = ref < min_seq;
        if (!ov_full) {
            for (int32_t base = 0; base < nu; base += kWave) {
                const int32_t j = base + lane;
                const bool in = j < nu;
                uint32_t vlen = 0, b = 0;
                if (in) {
                    const uint32_t slot = u_list[j];
                    vlen = view_entry((uint32_t)j, slot, ref, c);
                    b = s_blk[slot];
                }
                ov_chain_add(in && vlen > 0u, b, vlen);
            }
        } else {
            for (int32_t base = 0; base < slot_top; base += kWave) {
                const int32_t slot = base + lane;
                bool live = slot < slot_top && (s_meta[slot] & kFLinked);
                uint32_t vlen = 0, b = 0;
                bool tie;
                if (live) {
                    view_of((uint32_t)slot, ref, c, vlen, tie);
                    b = s_blk[slot];
                }
                ov_chain_add(live && vlen > 0u, b, vlen);
            }
        }
        ov_splits = splits;
        wsync();
    }
    MT_FI void ensure_overlay(int32_t ref, uint32_t c) {
        if (ov_splits != splits) overlay(ref, c);
    }

    // settle every overlay entry that minSeq has caught up with (before zamboni scours), and
    // rebase the 16-bit seqs of the rest on minSeq; the kept entries are compacted in order and
    // their slots' meta words follow
    MT_FI void settle_all() {
        PF_SCOPE(11);
        int32_t w = 0;
        const uint32_t m16 = (uint32_t)(min_seq - sbase);
        wsync();
        for (int32_t b0 = 0; b0 < nu; b0 += kWave) {
            const int32_t j = b0 + lane;
            const bool in = j < nu;
            uint32_t slot = 0, cm = 0, add = 0, b = 0;
            USr sr = 0;
            bool elig = false;
            if (in) {
                slot = u_list[j];
                sr = u_sr[j];
                cm = u_cm[j];
                const uint32_t q = us_q(sr), r = us_r(sr);
                elig = q <= m16 && (r == kRNone || r <= m16);
                // a diverged writer's group-free segment with seq -1, removed at or below minSeq
                // (op_ack): length 0 to every view, unlinked by the next scour of its block
                if constexpr (kW)
                    elig = elig || (q == kRUnassigned && r <= m16 && !(s_meta[slot] & kFPending));
                if (elig) {
                    if (r == kRNone) add = s_len[slot];
                    b = s_blk[slot];
                }
            }
            const bool keep = in && !elig;
            const uint64_t km = ballot(keep);
            const int32_t dst = w + __popcll(km & ((1ull << lane) - 1ull));
            wsync();
            if (keep) {
                const uint32_t q = us_q(sr), r = us_r(sr);
                uint32_t nq = q > m16 ? q - m16 : 0u;
                uint32_t nr = r == kRNone ? kRNone : (r > m16 ? r - m16 : 0u);
                if constexpr (kW) {  // pending local ops keep their sentinel
                    if (q == kRUnassigned) nq = kRUnassigned;
                    if (r == kRUnassigned) nr = kRUnassigned;
                }
                u_list[dst] = (Idx)slot;
                u_sr[dst] = us_make(nq, nr);
                u_cm[dst] = cm;
                if (dst != j) s_meta[slot] = (Meta)((s_meta[slot] & ~kUNone) | (uint32_t)dst);
            }
            if (elig) s_meta[slot] = (Meta)(s_meta[slot] | kUNone);
            w += __popcll(km);
            chain_add(b_slen, elig && add > 0u, b, add);
        }
        nu = w;
        sbase = min_seq;
        settled_min = min_seq;
        ov_splits = -1;  // b_slen moved under the overlay
        wsync();
    }
    // ------------------------------------------------------------------ descent
    // insertingWalk (mergeTree.ts:2345-2474) in insert mode: at every interior level the first
    // child whose cumulative view length reaches pos (breakTie is true for blocks); in the leaf
    // block the first leaf with pos < len or the leaf tie rule, else the block end.
    // strict mode (nodeMap's start < len, mergeTree.ts:2903-2965): first child whose cumulative
    // length exceeds pos; returns only the leaf block and its start position.
    // Levels whose children are interior blocks use their settled sums + overlay (giant class: every
    // child's row loaded in the round that loads the children's lengths — lane i: row entry i & 7 of
    // child i >> 3 — so an HBM level costs one dependent round trip; the chosen child's row moves to
    // lanes 0-7 by a permute).  The level-1 block's children are leaf blocks, which keep no length: all
    // their leaves are evaluated at once (lane = 8 x child + entry), the leaf blocks' lengths are
    // group sums, and the chosen leaf block's leaves move to lanes 0-7 for the leaf rule.
    MT_FI Walk descend(uint32_t pos, int32_t ref, uint32_t c, bool strict) {
        PF_SCOPE(1);
        Walk W;
        W.blk = -1;
        W.k = 0;
        W.n = 0;
        W.base = 0;
        W.excl = 0;
        W.ok = 0;
        W.slot = 0;
        int32_t N = root;
        uint32_t base = 0;
        const bool lanes8 = lane < kMaxNodes;
        int32_t n = b_count[N];
        uint32_t row = lanes8 ? (uint32_t)b_child[N * 8 + lane] : 0u;
        for (int32_t l = 0; l + 2 < depth; l++) {
            uint32_t nrow = 0;
            if constexpr (kGiant || MT_DESCENT_ONE_ROUND) {
                const uint32_t myc = (uint32_t)__shfl((int)row, lane >> 3, kWave);
                nrow = (lane >> 3) < n ? (uint32_t)b_child[myc * 8 + (lane & 7)] : 0u;
            }
            uint32_t v = 0, cnt = 0;
            if (lane < n) {
                v = iview(row);
                cnt = b_count[row];
            }
            const uint32_t incl = scan8(v) + base;
            const uint64_t hb = ballot(lanes8 && lane < n && (strict ? incl > pos : incl >= pos));
            if (!hb) return W;
            const int f = first_lane(hb);
            base = rdl(incl - v, f);
            N = (int32_t)rdl(row, f);
            n = (int32_t)rdl(cnt, f);
            if constexpr (kGiant || MT_DESCENT_ONE_ROUND) {
                row = (uint32_t)__shfl((int)nrow, 8 * f + (lane & 7), kWave);
                if (!lanes8) row = 0u;
            } else {
                row = lanes8 ? (uint32_t)b_child[N * 8 + lane] : 0u;
            }
        }
        uint32_t vlen = 0;
        bool tie = false;
        if (depth >= 2) {
            const int32_t ci = lane >> 3, j = lane & 7;
            const uint32_t cb = (uint32_t)__shfl((int)row, ci, kWave);
            const bool cin = ci < n;
            const uint32_t cn = cin ? (uint32_t)b_count[cb] : 0u;
            const uint32_t sl = cin ? (uint32_t)b_child[cb * 8 + j] : 0u;
            if (cin && (uint32_t)j < cn) view_of(sl, ref, c, vlen, tie);
            const uint32_t gsum = sum8(vlen);
            const uint32_t cl = (uint32_t)__shfl((int)gsum, 8 * lane, kWave);
            const uint32_t incl = scan8(cl) + base;
            const uint64_t hb = ballot(lanes8 && lane < n && (strict ? incl > pos : incl >= pos));
            if (!hb) return W;
            const int f = first_lane(hb);
            base = rdl(incl - cl, f);
            N = (int32_t)rdl(row, f);
            n = (int32_t)rdl(cn, 8 * f);
            W.blk = N;
            W.n = n;
            W.base = base;
            if (strict) return W;
            const int src = 8 * f + (lane & 7);
            vlen = (uint32_t)__shfl((int)vlen, src, kWave);
            tie = __shfl((int)tie, src, kWave) != 0;
            row = (uint32_t)__shfl((int)sl, src, kWave);
        } else {  // the root is the only (leaf) block
            W.blk = N;
            W.n = n;
            W.base = base;
            if (strict) return W;
            if (lane < n) view_of(row, ref, c, vlen, tie);
        }
        if (lane >= n) vlen = 0u;
        const uint32_t incl = scan8(vlen) + base;
        const uint32_t excl = incl - vlen;
        const uint64_t cb = ballot(lanes8 && lane < n && (incl > pos || (excl == pos && vlen == 0u && tie)));
        if (cb) {
            const int f = first_lane(cb);
            W.k = f;
            W.excl = rdl(excl, f);
            W.ok = 1;
            W.slot = rdl(row, f);
        } else {
            const uint32_t end = n > 0 ? rdl(incl, n - 1) : base;
            W.k = n;
            W.excl = end;
            W.ok = end == pos;
        }
        return W;
    }

    // the settled length of a block: an interior block's b_slen, a leaf block's sum over its leaves
    MT_FI uint32_t blk_settled(uint32_t b, bool leafb) {
        if (!leafb) return b_slen[si(b)];
        const int32_t n = b_count[b];
        const uint32_t x = lane < n ? settled_len(b_child[b * 8 + lane]) : 0u;
        return rdl(sum8(x), 0);
    }
    // per lane: the settled length of leaf block b (each lane its own block, <= 7 leaves)
    MT_FI uint32_t leaf_block_settled(uint32_t b) {
        const int32_t n = b_count[b];
        uint32_t x = 0;
        for (int32_t j = 0; j < n; j++) x += settled_len(b_child[b * 8 + j]);
        return x;
    }

    // ------------------------------------------------------------------ text helpers
    // lane-parallel copy of n code units inside the doc's text region
    MT_FI void text_copy(uint32_t dst, uint32_t src, uint32_t n) {
        for (uint32_t i = lane; i < n; i += kWave) text[dst + i] = text[src + i];
    }
    // the queued copies (lane i of dd / ds / dl: copy i, each <= 64 units): every load, then every
    // store.  Their regions are disjoint: each destination is its head's free capacity, each source
    // a merged leaf's own text (capacity regions of live segments never overlap).
    static constexpr int kTextQ = 4;
    MT_FI void text_flush(uint32_t dd, uint32_t ds, uint32_t dl, int32_t &nq) {
        uint32_t v[kTextQ];
#pragma unroll
        for (int i = 0; i < kTextQ; i++) {
            v[i] = 0u;
            if (i < nq && (uint32_t)lane < rdl(dl, i)) v[i] = text[rdl(ds, i) + (uint32_t)lane];
        }
#pragma unroll
        for (int i = 0; i < kTextQ; i++)
            if (i < nq && (uint32_t)lane < rdl(dl, i)) text[rdl(dd, i) + (uint32_t)lane] = (uint16_t)v[i];
        nq = 0;
    }
    // Bump allocation in the active text semispace; when it is full, live text moves to the
    // other semispace (text_gc) and the garbage left by reallocating merges is dropped.
    MT_FI uint32_t arena_alloc(uint32_t n) {
        const uint32_t n16 = (n + 1u) & ~1u;  // 4-byte granules
        if (arena_top + n16 > arena_end) {
            text_gc();
            if (arena_top + n16 > arena_end) {
                cap_fail(2);
                return 0;
            }
        }
        uint32_t o = arena_top;
        arena_top += n16;
        return o;
    }

    // copy every linked segment's arena text into the other semispace
    MT_FI void text_gc() {
        resolve_cold();  // pending split records must be in HBM before they are rewritten
        const uint32_t nb = arena_base == pay_end ? pay_end + semi_t : pay_end;
        uint32_t top = nb;
        wsync();
        for (int32_t base = 0; base < slot_top; base += kWave) {
            const int32_t slot = base + lane;
            bool mv = false;
            uint4 cr = make_uint4(0, 0, 0, 0);
            if (slot < slot_top) {
                const uint32_t m = s_meta[slot];
                if ((m & kFLinked) && !(m & kFMarker)) {
                    cr = cold[2 * slot];
                    mv = cr.z >= arena_base && cr.z < arena_end;
                }
            }
            uint64_t msk = ballot(mv);
            while (msk) {
                const int f = first_lane(msk);
                msk &= msk - 1;
                const uint32_t sl = (uint32_t)(base + f);
                const uint32_t len = s_len[sl];
                // packed tightly: short segments would otherwise waste most of a semispace
                const uint32_t cap16 = (len + 1u) & ~1u;
                if (top + cap16 > nb + semi_t) {
                    cap_fail(2);
                    return;
                }
                text_copy(top, rdl(cr.z, f), len);
                if (lane == f) {
                    cr.z = top;
                    cr.w = cap16;
                    cold[2 * sl] = cr;
                }
                top += cap16;
            }
            wsync();
        }
        arena_base = nb;
        arena_end = nb + semi_t;
        arena_top = top;
        text_gcs++;
        wsync();
    }

    // make room for `words` in the prop pool: semispace copy of the live records when full
    // (Cheney-style: a copied record's header becomes a forwarding pointer, so sets shared by
    // several segments are copied once).  Live records: the prop sets of linked segments
    // (cold.x) and their overlap-client lists (cold.y with kOvlList).
    MT_FI uint32_t pool_forward(uint32_t o, uint32_t nb, uint32_t &top) {
        const uint32_t hdr = pool[o];
        if (hdr == 0xFFFFFFFFu) return pool[o + 1];
        const uint32_t w = (hdr & kPoolOvlTag) ? 2u + (hdr & ~kPoolOvlTag) : 2u + 2u * hdr;
        if (top + w > nb + semi_p) {
            cap_fail(3);
            return 0;
        }
        for (uint32_t i = lane; i < w; i += kWave) pool[top + i] = pool[o + i];
        wsync();
        const uint32_t nid = top;
        top += w;
        if (lane == 0) {
            pool[o] = 0xFFFFFFFFu;
            pool[o + 1] = nid;
        }
        wsync();
        return nid;
    }
    MT_FI void pool_reserve(uint32_t words) {
        if (pool_top + words <= pool_end) return;
        resolve_cold();
        const uint32_t nb = pool_base == 1u ? 1u + semi_p : 1u;
        uint32_t top = nb;
        wsync();
        for (int32_t b0 = 0; b0 < slot_top; b0 += kWave) {
            const int32_t slot = b0 + lane;
            uint32_t old = 0, ovl = 0, lw = 0;
            if (slot < slot_top) {
                const uint32_t m = s_meta[slot];
                if (m & kFLinked) {
                    const uint4 cr = cold[2 * slot];
                    if (m & kFHasProps) old = cr.x;
                    if (cr.y & kOvlList) ovl = cr.y & ~kOvlList;
                    if (lab && (m & kFMarker)) lw = cr.w;  // the labels snapshot's prop set
                }
            }
            uint64_t msk = ballot(old != 0u);
            while (msk) {
                const int f = first_lane(msk);
                msk &= msk - 1;
                const uint32_t nid = pool_forward(rdl(old, f), nb, top);
                if (status) return;
                if (lane == 0) cold[2 * (uint32_t)(b0 + f)].x = nid;
                wsync();
            }
            msk = ballot(ovl != 0u);
            while (msk) {
                const int f = first_lane(msk);
                msk &= msk - 1;
                const uint32_t nid = pool_forward(rdl(ovl, f), nb, top);
                if (status) return;
                if (lane == 0) cold[2 * (uint32_t)(b0 + f)].y = nid | kOvlList;
                wsync();
            }
            msk = ballot(lw != 0u);
            while (msk) {
                const int f = first_lane(msk);
                msk &= msk - 1;
                const uint32_t nid = pool_forward(rdl(lw, f), nb, top);  // (already moved: forwarded)
                if (status) return;
                if (lane == 0) cold[2 * (uint32_t)(b0 + f)].w = nid;
                wsync();
            }
        }
        pool_base = nb;
        pool_end = nb + semi_p;
        pool_top = top;
        pool_gcs++;
        wsync();
        if (pool_top + words > pool_end) cap_fail(3);
    }

    // ------------------------------------------------------------------ block tree
    MT_FI int32_t child_index(int32_t p, int32_t c) {
        int32_t n = b_count[p];
        bool hit = lane < n && b_child[p * 8 + lane] == (Idx)c;
        uint64_t b = ballot(hit);
        return b ? first_lane(b) : -1;
    }

    // updateRoot (mergeTree.ts:1876-1887)
    MT_FI void update_root(int32_t split_node) {
        int32_t nr = alloc_block(0, depth);  // the old root is at level depth - 1
        if (status) return;
        const bool leafs = depth == 1;  // the old root and its split-off half are leaf blocks
        const uint32_t sl = blk_settled((uint32_t)root, leafs) + blk_settled((uint32_t)split_node, leafs);
        b_child[nr * 8 + 0] = (Idx)root;
        b_child[nr * 8 + 1] = (Idx)split_node;
        b_count[nr] = 2;
        b_slen[si(nr)] = sl;
        b_parent[root] = (Idx)nr;
        b_parent[split_node] = (Idx)nr;
        root = nr;
        depth++;
        wsync();
    }

    // insertingWalk's "insert the split-off node after its source" (mergeTree.ts:2446-2453),
    // cascading MergeTree.split (2476-2489) up the interior levels and updateRoot at the top.
    MT_FI void insert_child_after(int32_t p, int32_t after, int32_t nc) {
        for (int32_t level = 1;; level++) {  // p's level
            int32_t i = child_index(p, after);
            int32_t n = b_count[p];
            wsync();
            Idx v = 0;
            if (lane > i && lane < n) v = b_child[p * 8 + lane];
            wsync();
            if (lane > i && lane < n) b_child[p * 8 + lane + 1] = v;
            wsync();
            b_child[p * 8 + i + 1] = (Idx)nc;
            b_parent[nc] = (Idx)p;
            b_count[p] = (uint8_t)(n + 1);
            wsync();
            if (n + 1 < kMaxNodes) return;
            // split the interior block p: children 4..7 move to m
            int32_t m = alloc_block(0, level);
            if (status) return;
            splits++;
            wsync();
            uint32_t moved;
            if (level == 1) {  // p's children are leaf blocks: the moved settled length from their leaves
                const int32_t ci = 4 + (lane >> 3), j = lane & 7;
                uint32_t x = 0;
                if (lane < 32) {
                    const uint32_t cb = b_child[p * 8 + ci];
                    if ((uint32_t)j < (uint32_t)b_count[cb]) x = settled_len(b_child[cb * 8 + j]);
                }
                moved = rdl(scan_incl(x), 63);
            } else {
                const uint32_t x = lane >= 4 && lane < 8 ? (uint32_t)b_slen[si(b_child[p * 8 + lane])] : 0u;
                moved = rdl(sum8(x), 0);
            }
            wsync();
            if (lane >= 4 && lane < 8) {
                Idx c = b_child[p * 8 + lane];
                b_child[m * 8 + lane - 4] = c;
                b_parent[c] = (Idx)m;
            }
            wsync();
            b_count[m] = 4;
            b_count[p] = 4;
            b_slen[si(m)] = moved;
            b_slen[si(p)] = b_slen[si(p)] - moved;
            wsync();
            if (p == root) {
                update_root(m);
                return;
            }
            after = p;
            nc = m;
            p = b_parent[p];
        }
    }

    // MergeTree.split on a leaf block that now holds 8 children; returns the new right block.
    MT_FI int32_t split_leaf(int32_t blk) {
        int32_t nb = alloc_block(1, 0);
        if (status) return blk;
        splits++;
        wsync();
        if (lane >= 4 && lane < 8) {
            Idx c = b_child[blk * 8 + lane];
            b_child[nb * 8 + lane - 4] = c;
            s_blk[c] = (Idx)nb;
        }
        wsync();
        b_count[nb] = 4;
        b_count[blk] = 4;  // (leaf blocks keep no length; the parent's settled sum is unchanged)
        wsync();
        if (blk == root) update_root(nb);
        else insert_child_after(b_parent[blk], blk, nb);
        return nb;
    }

    // ------------------------------------------------------------------ split / insert leaves
    // insert slot before child k of leaf block blk; returns the block the new leaf ends up in
    MT_FI int32_t insert_leaf(int32_t blk, int32_t k, uint32_t slot) {
        const int32_t n = b_count[blk];
        wsync();
        Idx v = 0;
        const bool mv = lane >= k && lane < n;
        if (mv) v = b_child[blk * 8 + lane];
        wsync();
        if (mv) b_child[blk * 8 + lane + 1] = v;
        wsync();
        b_child[blk * 8 + k] = (Idx)slot;
        s_blk[slot] = (Idx)blk;
        b_count[blk] = (uint8_t)(n + 1);
        wsync();
        if (n + 1 >= kMaxNodes) {
            int32_t nb = split_leaf(blk);
            lab_refresh(blk);  // MergeTree.split updates both halves
            lab_refresh(nb);
            if (k >= kMaxNodes / 2) return nb;
            return blk;
        }
        lab_refresh(blk);  // insertingWalk's blockUpdateLength of the leaf block
        return blk;
    }

    // BaseSegment.splitAt + TextSegment.createSplitSegmentAt (mergeTree.ts:524-568,
    // textSegment.ts:103-111): the right part becomes a new leaf right after child k of blk.
    // The settled sums do not change (both halves inherit the segment's state).  The cold
    // record is read now and written back in resolve_cold(); a second split of the same op
    // forwards the first one's pending records instead of reading HBM.
    // Returns the leaf block the right half landed in (-1: no split).
    MT_FI int32_t split_at(int32_t blk, int32_t k, uint32_t r, uint32_t slot_hint) {
        PF_SCOPE(2);
        // the giant class takes the slot from the walk's leaf row (an HBM re-read otherwise)
        const uint32_t slot = kGiant ? slot_hint : rfl((uint32_t)b_child[blk * 8 + k]);
        const uint32_t meta = s_meta[slot];
        if (meta & kFMarker) return -1;  // Marker.createSplitSegmentAt returns undefined
        // the slot's two cold records, lane-distributed (lane i < 8: word i)
        uint32_t pv;
        if (pend_n > 0 && slot == ps0) {
            resolve_splits();  // (inverted range) the first split's left half is cut again
            pv = lane == 3 ? pr0 : pv0;
        } else if (pend_n > 0 && slot == pn0) {
            pv = pv0 + (lane == 2 ? pr0 : 0u) - (lane == 3 ? pr0 : 0u);
        } else {
            pv = lane < 8 ? reinterpret_cast<const uint32_t *>(cold + 2 * slot)[lane] : 0u;
        }
        const int32_t ns = alloc_slot();
        if (ns < 0) return -1;
        const uint32_t len = s_len[slot];
        if (pend_n == 0) {
            ps0 = slot;
            pn0 = (uint32_t)ns;
            pr0 = r;
            pv0 = pv;
        } else {
            ps1 = slot;
            pn1 = (uint32_t)ns;
            pr1 = r;
            pv1 = pv;
        }
        pend_n++;
        s_len[ns] = (Len)(len - r);
        s_meta[ns] = (Meta)(meta | kUNone);  // inherits ends-NL of the tail, linked, removed, pending
        s_len[slot] = (Len)r;
        wsync();
        if (!is_settled(meta)) {  // the right half gets a copy of the overlay entry
            const uint32_t ui = meta & kUNone;
            u_push((uint32_t)ns, u_sr[ui], u_cm[ui]);
        }
        if constexpr (kW) {
            // segmentGroups.copyTo (mergeTree.ts:560): the right half joins every group of the
            // segment, oldest first, at the end of each group's segments; its cold record (written
            // by resolve_cold) carries the same pending mask
            if (meta & kFPending) {
                const uint32_t m = rdl(pv, 7);
                const uint32_t head = pend_word(1);
                for (int32_t i = 0; i < n_pend && !status; i++)
                    if (in_group(head + (uint32_t)i, slot, m)) entry_append(head + (uint32_t)i, (uint32_t)ns);
                if (status) return -1;
            }
        }
        const int32_t nb = insert_leaf(blk, k + 1, (uint32_t)ns);
        if (rdl(pv, 1)) resolve_cold();  // view_of reads the halves' overlap masks from HBM
        return nb;
    }

    // write the pending splits' cold records and start the text loads for ends-with-'\n': the
    // left half keeps its records with tcap = r, the right half gets (toff + r, tcap - r) and a
    // copy of the seq record
    MT_FI void resolve_cold() {
        PF_SCOPE(13);
        for (int32_t i = pend_cold; i < pend_n; i++) {
            const uint32_t sl = i ? ps1 : ps0, ns = i ? pn1 : pn0, r = i ? pr1 : pr0;
            const uint32_t pv = i ? pv1 : pv0;
            if (lane == 3) reinterpret_cast<uint32_t *>(cold + 2 * sl)[3] = r;
            if (lane < 8)
                reinterpret_cast<uint32_t *>(cold + 2 * ns)[lane] = pv + (lane == 2 ? r : 0u) - (lane == 3 ? r : 0u);
            // a text without any '\n' cannot end in one: no HBM read
            const uint32_t ch = (s_meta[sl] & kFHasNL) ? (uint32_t)text[rdl(pv, 2) + r - 1] : 0u;
            if (i) pch1 = ch;
            else pch0 = ch;
        }
        pend_cold = pend_n;
    }

    MT_FI void resolve_splits() {
        if (pend_n == 0) return;
        resolve_cold();
        for (int32_t i = 0; i < pend_n; i++) {
            const uint32_t sl = i ? ps1 : ps0;
            const uint32_t ch = i ? pch1 : pch0;
            const uint32_t m = s_meta[sl];
            s_meta[sl] = (Meta)(ch == (uint32_t)'\n' ? (m | kFEndsNL) : (m & ~kFEndsNL));
        }
        pend_n = 0;
        pend_cold = 0;
        wsync();
    }

    // ensureIntervalBoundary (mergeTree.ts:2241-2245): split the leaf that strictly contains pos
    // in the op's view.  Returns the insert-mode walk for pos *after* the split.
    MT_FI Walk boundary(uint32_t pos, int32_t ref, uint32_t c) {
        ensure_overlay(ref, c);
        Walk W = descend(pos, ref, c, false);
        if (W.blk >= 0 && W.ok && W.k < W.n && W.excl < pos) {
            const int32_t s0 = splits;
            const int32_t nb = split_at(W.blk, W.k, pos - W.excl, W.slot);
            if (status) return W;
            if (splits == s0) {
                // no block split: the left half ends at pos, the right half (k + 1) starts there
                W.k += 1;
                W.n += 1;
            } else {
                // The leaf block (7 children + the right half) split 4 + 4 (split_leaf).  The
                // walk the reference repeats lands here without a new descent: every block left
                // of the left half's block ends before pos, and the first one reaching pos is
                //  - blk itself when both halves stayed in it (right half at k + 1 <= 3),
                //  - blk at its end when the left half is blk's last child (k + 1 == 4: blk ends
                //    exactly at pos, and no leaf after it in blk can tie),
                //  - the new block otherwise, right half at k + 1 - 4 (blk ends before pos).
                // W.base is left stale: boundary's callers read only blk / k / n / ok.
                const int32_t kr = W.k + 1;
                if (kr < kMaxNodes / 2) {
                    W.k = kr;
                } else if (kr == kMaxNodes / 2) {
                    W.k = kMaxNodes / 2;
                } else {
                    W.blk = nb;
                    W.k = kr - kMaxNodes / 2;
                }
                W.n = kMaxNodes / 2;
            }
            W.excl = pos;
        }
        return W;
    }

    // ------------------------------------------------------------------ writer: pending segment groups
    // MergeTree.pendingSegments / SegmentGroup (mergeTree.ts:1093, 1922-1929) in the document's HBM
    // region (mt_device.h kPendDesc / pend_entries); lane 0 writes, every lane reads back.
    MT_FI uint32_t pend_word(int i) const { return rfl(pend[i]); }
    static constexpr uint32_t kPmb = (uint32_t)kPendMaskBits - 1u;  // group G's mask bit: G & kPmb
    MT_FI uint32_t pend_mask(uint32_t slot) const { return rfl(cold[2 * slot + 1].w); }
    MT_FI void pend_set_mask(uint32_t slot, uint32_t m) {
        if (lane == 0) cold[2 * slot + 1].w = m;
        const uint32_t meta = s_meta[slot];
        s_meta[slot] = (Meta)(m ? (meta | kFPending) : (meta & ~kFPending));
        wsync();
    }
    MT_FI uint32_t *pdesc(uint32_t G) const { return pend + kPendDesc + 4 * (G & (pend_groups(pend_cap_e) - 1u)); }
    // is `slot` (pending mask m) a member of the live group G?  The mask bit decides while at most 32
    // groups are pending; beyond, groups 32 apart share a bit and G's entries decide
    MT_FI bool in_group(uint32_t G, uint32_t slot, uint32_t m) {
        if (!((m >> (G & kPmb)) & 1u)) return false;
        return n_pend <= kPendMaskBits || entry_has(G, slot);
    }
    MT_FI bool entry_has(uint32_t G, uint32_t slot) {
        const uint32_t start = pend_word(2), n = pend_word(3);
        const uint2 *E = (const uint2 *)(pend + pend_entries(pend_cap_e));
        for (uint32_t b0 = start; b0 < n; b0 += kWave) {
            const uint32_t j = b0 + (uint32_t)lane;
            bool hit = false;
            if (j < n) {
                const uint2 e = E[j];
                hit = e.x == G && e.y == slot;
            }
            if (ballot(hit)) return true;
        }
        return false;
    }
    // after `slot` leaves group G: may bit G & 63 go?  (not while another live group sharing it,
    // other than `skip`, holds the segment)
    MT_FI bool bit_free_after(uint32_t G, uint32_t slot, uint32_t head, uint32_t skip) {
        if (n_pend <= kPendMaskBits) return true;
        for (uint32_t o = (G - head) & kPmb; o < (uint32_t)n_pend; o += (uint32_t)kPendMaskBits) {
            const uint32_t H = head + o;
            if (H != G && H != skip && entry_has(H, slot)) return false;
        }
        return true;
    }
    // localSeq of the live group of type T holding `slot` (0xFFFFFFFF: none)
    MT_FI uint32_t group_lseq(uint32_t slot, uint32_t m, uint32_t T) {
        const uint32_t head = pend_word(1);
        for (int32_t i = 0; i < n_pend; i++) {
            const uint32_t G = head + (uint32_t)i;
            if (!((m >> (G & kPmb)) & 1u)) continue;
            const uint32_t *dp = pdesc(G);
            if ((rfl(dp[0]) & 0xFFu) != T) continue;
            if (in_group(G, slot, m)) return rfl(dp[3]);
        }
        return 0xFFFFFFFFu;
    }
    // live entries (of pending groups) move to the front, in order
    MT_FI void pend_compact() {
        const uint32_t head = pend_word(1), start = pend_word(2), n = pend_word(3);
        uint2 *E = (uint2 *)(pend + pend_entries(pend_cap_e));
        uint32_t w = 0;
        for (uint32_t b0 = start; b0 < n; b0 += kWave) {
            const uint32_t j = b0 + (uint32_t)lane;
            const uint2 e = j < n ? E[j] : make_uint2(0u, 0u);
            const bool live = j < n && e.x - head < (uint32_t)n_pend;
            const uint64_t m = ballot(live);
            if (live) E[w + __popcll(m & ((1ull << lane) - 1ull))] = e;
            w += __popcll(m);
        }
        if (lane == 0) {
            pend[2] = 0u;
            pend[3] = w;
        }
    }
    // SegmentGroupCollection.enqueue (segmentGroupCollection.ts:24-27): group G gets `slot` last
    MT_FI void entry_append(uint32_t G, uint32_t slot) {
        uint32_t n = pend_word(3);
        if (n >= (uint32_t)pend_cap_e) {
            pend_compact();
            n = pend_word(3);
            if (n >= (uint32_t)pend_cap_e) {
                cap_fail(kCapPending);
                return;
            }
        }
        if (lane == 0) {
            ((uint2 *)(pend + pend_entries(pend_cap_e)))[n] = make_uint2(G, slot);
            pend[3] = n + 1u;
        }
    }
    // addToPendingList (mergeTree.ts:1922-1929) for the current local op: its group is created with
    // its first segment (cur_g < 0 until then)
    int32_t cur_g;
    MT_FI void pend_add(uint32_t slot, const mt_op &op) {
        resolve_cold();  // the split halves' cold records (pending masks) are in HBM
        if (cur_g < 0) {
            if (n_pend >= (int32_t)pend_groups(pend_cap_e)) {
                set_fail(ST_UNSUPPORTED);
                return;
            }
            cur_g = (int32_t)(pend_word(1) + (uint32_t)n_pend);
            const uint32_t lseq = pend_word(4);  // collabWindow.localSeq of this op
            if (lane == 0) {
                *(uint4 *)pdesc((uint32_t)cur_g) =
                    make_uint4((uint32_t)op.type | ((uint32_t)op.flags << 16), op.payload, op.payload_len, lseq);
                pend[0] = (uint32_t)(n_pend + 1);
            }
            n_pend++;
        }
        entry_append((uint32_t)cur_g, slot);
        if (status) return;
        pend_set_mask(slot, pend_mask(slot) | (1u << ((uint32_t)cur_g & kPmb)));
    }
    // the keys of the pending local annotates holding `slot` (lane j < npk: key j) and whether one of
    // them is a rewrite: SegmentPropertiesManager.pendingKeyUpdateCount / pendingRewriteCount
    // (segmentPropertiesManager.ts:12-14, 49-51, 56-63)
    MT_FI void pending_keys(uint32_t slot, uint32_t &pk, uint32_t &npk, bool &prw) {
        const uint32_t m = pend_mask(slot);
        const uint32_t head = pend_word(1);
        npk = 0;
        pk = 0;
        prw = false;
        for (int32_t i = 0; i < n_pend; i++) {
            const uint32_t G = head + (uint32_t)i;
            if (!((m >> (G & kPmb)) & 1u)) continue;
            const uint32_t *dp = pdesc(G);
            const uint32_t tf = rfl(dp[0]), off = rfl(dp[1]), cnt = rfl(dp[2]);
            if ((tf & 0xFFu) != MT_OP_ANNOTATE) continue;
            if (!in_group(G, slot, m)) continue;
            if ((tf >> 16) & MT_OPF_REWRITE) prw = true;
            for (uint32_t k = 0; k < cnt; k++) {
                const uint32_t key = rfl(props_in[off + k].key);
                if (ballot((uint32_t)lane < npk && pk == key)) continue;
                if (npk >= 64u) {
                    set_fail(ST_UNSUPPORTED);
                    return;
                }
                if ((uint32_t)lane == npk) pk = key;
                npk++;
            }
        }
    }
    // is `key` among the cnt prop records at props_in[off...]?  (wave-uniform)
    MT_FI bool key_among(uint32_t off, uint32_t cnt, uint32_t key) const {
        for (uint32_t k0 = 0; k0 < cnt; k0 += kWave) {
            const uint32_t k = k0 + (uint32_t)lane;
            if (ballot(k < cnt && props_in[off + k].key == key)) return true;
        }
        return false;
    }
    // Client.ackPendingSegment -> MergeTree.ackPendingSegment (client.ts:588-625, mergeTree.ts:
    // 1893-1920) with BaseSegment.ack (487-522): the oldest group's segments, in group order, are
    // acked by the rules of the *incoming* op's type — whatever op made the group (a replica whose
    // local op was dropped as an invalid range acks the next op's group with this one) — each then
    // addToLRUSet; then zamboni.  insert: assert(seq === Unassigned), seq = the message's; remove:
    // assert(removedSeq), removedSeq = the message's unless a sequenced remove replaced the local one;
    // annotate: assert(propertyManager), ackPendingProperties(op) decrements the pending counts of the
    // op's keys.  A failing assert stops the document (MT_BAD_INPUT) at this record, as the reference
    // throws here.  The device derives a segment's pending keys from the annotate groups still
    // holding it (pending_keys); an annotate ack whose literal decrements differ from dropping the
    // group (another op's keys, a rewrite count off by one), or an ack that leaves a segment with an
    // unassigned seq / removedSeq and no group, is a state the device does not model: MT_UNSUPPORTED.
    MT_FI void op_ack(const mt_op &op) {
        if (n_pend > 0) {
            const uint32_t head = pend_word(1);
            const uint32_t b = head & kPmb;
            const uint32_t *dh = pdesc(head);
            const uint32_t tf = rfl(dh[0]), g_off = rfl(dh[1]), g_cnt = rfl(dh[2]);
            if (op.type != MT_OP_INSERT && op.type != MT_OP_REMOVE && op.type != MT_OP_ANNOTATE) {
                set_fail(ST_BAD_INPUT);  // BaseSegment.ack: unrecognized operation type
                return;
            }
            // annotate: does dropping the group change the pending keys exactly as the op's ack does?
            const bool g_ann = (tf & 0xFFu) == MT_OP_ANNOTATE;
            const bool g_rw = g_ann && (((tf >> 16) & MT_OPF_REWRITE) != 0u);
            const bool o_rw = (op.flags & MT_OPF_REWRITE) != 0u;
            const uint32_t o_off = (uint32_t)op.payload, o_cnt = (uint32_t)op.payload_len;
            bool same = false;
            if (op.type == MT_OP_ANNOTATE && g_ann && g_rw == o_rw) {
                same = true;
                for (uint32_t k = 0; same && k < o_cnt; k++) same = key_among(g_off, g_cnt, rfl(props_in[o_off + k].key));
                for (uint32_t k = 0; same && k < g_cnt; k++) same = key_among(o_off, o_cnt, rfl(props_in[g_off + k].key));
            }
            const uint32_t start = pend_word(2), n = pend_word(3);
            const uint2 *E = (const uint2 *)(pend + pend_entries(pend_cap_e));
            for (uint32_t b0 = start; b0 < n; b0 += kWave) {
                const uint32_t j = b0 + (uint32_t)lane;
                const uint2 e = j < n ? E[j] : make_uint2(head + 1u, 0u);
                uint64_t hm = ballot(j < n && e.x == head);
                while (hm) {
                    const uint32_t slot = rdl(e.y, first_lane(hm));
                    hm &= hm - 1;
                    const uint32_t meta = rfl((uint32_t)s_meta[slot]);
                    const uint32_t ui = meta & kUNone;
                    const USr sr = ui != kUNone ? u_sr[ui] : us_make(0u, kRNone);
                    uint32_t sq = rfl(us_q(sr)), srr = rfl(us_r(sr));
                    if (op.type == MT_OP_INSERT) {
                        if (ui == kUNone || sq != kRUnassigned) {
                            set_fail(ST_BAD_INPUT);
                            return;
                        }
                        sq = rel(op.seq);
                        u_sr[ui] = us_make(sq, srr);
                        if (lane == 0) cold[2 * slot + 1].x = (uint32_t)op.seq;
                    } else if (op.type == MT_OP_REMOVE) {
                        if (!(meta & kFRemoved)) {
                            set_fail(ST_BAD_INPUT);
                            return;
                        }
                        if (ui != kUNone && srr == kRUnassigned) {
                            srr = rel(op.seq);
                            u_sr[ui] = us_make(sq, srr);
                            if (lane == 0) cold[2 * slot + 1].y = (uint32_t)op.seq;
                        }
                    } else {
                        if (!(meta & kFHasProps)) {  // assert(!!this.propertyManager)
                            set_fail(ST_BAD_INPUT);
                            return;
                        }
                        if (!same) {
                            // literal: the op's keys that are pending lose one count (and a rewrite
                            // one rewrite); derived: the group's keys (and its rewrite) go
                            uint32_t pk, npk;
                            bool prw;
                            pending_keys(slot, pk, npk, prw);
                            if (status) return;
                            bool ok = o_rw == g_rw;
                            for (uint32_t k = 0; ok && k < o_cnt; k++) {
                                const uint32_t key = rfl(props_in[o_off + k].key);
                                const bool pend_k = ballot((uint32_t)lane < npk && pk == key) != 0;
                                ok = pend_k == (g_ann && key_among(g_off, g_cnt, key));
                            }
                            for (uint32_t k = 0; ok && g_ann && k < g_cnt; k++)
                                ok = key_among(o_off, o_cnt, rfl(props_in[g_off + k].key));
                            if (!ok) {
                                set_fail(ST_UNSUPPORTED);
                                return;
                            }
                        }
                    }
                    wsync();
                    if (bit_free_after(head, slot, head, head)) {
                        const uint32_t m = pend_mask(slot) & ~(1u << b);
                        pend_set_mask(slot, m);
                        // no group left, yet an unassigned seq (a diverged replica's ack): scourNode
                        // sees `seq <= minSeq` / `removedSeq <= minSeq` for -1 and the group-free test
                        // passes.  A removed one is then view-independent (length 0 to every view):
                        // it settles and is unlinked as the reference's scour does; other shapes are
                        // not modelled.
                        if (m == 0u && ui != kUNone && (sq == kRUnassigned || srr == kRUnassigned)) {
                            if (sq == kRUnassigned && srr != kRUnassigned && srr != kRNone) settled_min = min_seq - 1;
                            else {
                                set_fail(ST_UNSUPPORTED);
                                return;
                            }
                        }
                    }
                    add_to_lru(rfl((int32_t)s_blk[slot]), slot, op.seq);
                    lab_refresh(rfl((int32_t)s_blk[slot]));  // blockUpdatePathLengths(segment.parent)
                    if (status) return;
                }
            }
            // the next live entry (later groups' entries may sit behind this group's)
            uint32_t ns = n;
            for (uint32_t b0 = start; b0 < n; b0 += kWave) {
                const uint32_t j = b0 + (uint32_t)lane;
                const uint64_t lm = ballot(j < n && E[j].x - (head + 1u) < (uint32_t)(n_pend - 1));
                if (lm) {
                    ns = b0 + (uint32_t)first_lane(lm);
                    break;
                }
            }
            if (lane == 0) {
                pend[0] = (uint32_t)(n_pend - 1);
                pend[1] = head + 1u;
                pend[2] = ns;
            }
            n_pend--;
        }
        zamboni();
    }

    // insertingWalk's continuePredicate for a remote insert (blockInsert.continueFrom, mergeTree.ts:
    // 2154-2161, 2431-2436): a walk that finishes at the end of a leaf block continues into the next
    // one while the first segment after the block that the local view holds (rightExcursion ->
    // nodeMap: not removed) is a pending local insert; it goes on at that block's start (pos 0 there)
    MT_FI Walk continue_walk(Walk W, int32_t ref, uint32_t c) {
        for (;;) {
            const int32_t nb = next_leaf_block(W.blk);
            bool cont = false;
            for (int32_t b = nb; b >= 0; b = next_leaf_block(b)) {
                const int32_t n = b_count[b];
                bool live = false, pins = false;
                if (lane < n) {
                    const uint32_t m = s_meta[b_child[b * 8 + lane]];
                    live = !(m & kFRemoved);
                    if (live && !is_settled(m)) pins = us_q(u_sr[m & kUNone]) == kRUnassigned;
                }
                const uint64_t lm = ballot(live);
                if (lm) {
                    cont = (ballot(pins) >> first_lane(lm)) & 1ull;
                    break;
                }
            }
            if (!cont) return W;
            const int32_t n = b_count[nb];
            const uint32_t pos = W.excl;
            uint32_t vlen = 0;
            bool tie = false;
            if (lane < n) view_of((uint32_t)b_child[nb * 8 + lane], ref, c, vlen, tie);
            const uint32_t incl = scan8(vlen) + pos;
            const uint32_t excl = incl - vlen;
            const uint64_t cb = ballot(lane < n && lane < kMaxNodes && (incl > pos || (excl == pos && vlen == 0u && tie)));
            W.blk = nb;
            W.n = n;
            W.ok = 1;
            W.base = pos;
            if (cb) {
                W.k = first_lane(cb);
                return W;
            }
            W.k = n;  // every leaf of the block is invisible to the op: its end is still pos
        }
    }

    // addToLRUSet (mergeTree.ts:1273-1283); seq > currentSeq holds for sequenced remote ops
    MT_FI void add_to_lru(int32_t blk, uint32_t slot, int32_t seq) {
        if (b_scour[blk] != kScourTrue && seq > cur_seq) {
            b_scour[blk] = kScourTrue;
            heap_add(slot, seq);
        }
    }

    // ------------------------------------------------------------------ heap (collections.ts:213-265)
    // The LRU heap lives in LDS as 8-byte {key, seq} entries, 1-based; a sift-down level reads
    // both children with one 16-byte load.  Same array layout and sift order as Heap.add /
    // Heap.get, hence the same pop order on seq ties.  `htop` caches heap[1].seq.
    MT_FI void heap_add(uint32_t key, int32_t seq) {
        PF_SCOPE(9);
        if (hn + 1 > cap.heap) {
            cap_fail(1);
            return;
        }
        hn++;
        int32_t k = hn;
        // sift up: parents larger than the new entry move down into the hole
        while (k > 1) {
            const uint2 pe = h_ent[k >> 1];
            const int32_t ps = (int32_t)rfl(pe.y);
            if (!(ps - seq > 0)) break;
            h_ent[k] = pe;
            k >>= 1;
        }
        h_ent[k] = make_uint2(key, (uint32_t)seq);
        if (k == 1) htop = seq;
        if (hn > max_heap) max_heap = hn;
        wsync();
    }
    // The sift-down reads three levels below the hole per LDS round trip (lanes 0-1: its children,
    // 2-5: their children, 6-13: the next level), then compares level by level from registers: the
    // same comparisons as one level per load, a third of the dependent round trips.
    MT_FI void heap_get(uint32_t &key, int32_t &seq) {
        PF_SCOPE(9);
        const uint2 top = h_ent[1];
        const uint2 last = h_ent[hn];
        key = rfl(top.x);
        seq = (int32_t)rfl(top.y);
        const int32_t ls = (int32_t)rfl(last.y);
        hn--;
        int32_t k = 1;
        int32_t newtop = ls;
        bool done = false;
        while (!done && (k << 1) <= hn) {
            const int32_t k0 = k;
            // lane l < 14: level L = 1, 2, 3 below k0 (lanes 2^L - 2 .. 2^(L+1) - 3), entry 2^L k0 + (l - 2^L + 2)
            const int32_t L = lane < 2 ? 1 : lane < 6 ? 2 : 3;
            const int32_t idx = (k0 << L) + lane - ((1 << L) - 2);
            uint2 e = make_uint2(0u, 0u);
            if (lane < 14 && idx <= hn) e = h_ent[idx];
#pragma unroll
            for (int lv = 1; lv <= 3; lv++) {
                const int32_t j0 = k << 1;
                if (j0 > hn) {
                    done = true;
                    break;
                }
                const int l0 = ((1 << lv) - 2) + (j0 - (k0 << lv));
                int32_t j = j0;
                uint32_t jk = rdl(e.x, l0);
                int32_t sj = (int32_t)rdl(e.y, l0);
                if (j0 < hn) {
                    const int32_t sj1 = (int32_t)rdl(e.y, l0 + 1);
                    if (sj - sj1 > 0) {
                        j = j0 + 1;
                        sj = sj1;
                        jk = rdl(e.x, l0 + 1);
                    }
                }
                if (ls - sj <= 0) {
                    done = true;
                    break;
                }
                h_ent[k] = make_uint2(jk, (uint32_t)sj);
                if (k == 1) newtop = sj;
                k = j;
            }
        }
        if (hn >= 1) h_ent[k] = last;
        htop = hn >= 1 ? newtop : kNoneSeq;
        wsync();
    }

    // Heap entries hold segment identity (the reference's Heap of {node, maxSeq}): when scour frees
    // slots (merged away / unlinked: parent = undefined, mergeTree.ts:1317, 1341, 1438), the
    // entries naming them are invalidated, so a slot reused later is never scoured by an old
    // entry.  `slot` holds the lanes' slots, `freeM` the freed lanes.
    MT_FI void heap_forget(uint32_t slot, uint64_t freeM) {
        PF_SCOPE(14);
        for (int32_t j0 = 1; j0 <= hn; j0 += kWave) {
            const int32_t j = j0 + lane;
            const uint32_t key = j <= hn ? h_ent[j].x : kHeapInvalid;
            bool hit = false;
            for (uint64_t m = freeM; m; m &= m - 1) hit |= key == rdl(slot, first_lane(m));
            if (hit && key != kHeapInvalid) h_ent[j].x = kHeapInvalid;
        }
        wsync();
    }

    // ------------------------------------------------------------------ marker ids, relative positions
    // mapIdToSegment (mergeTree.ts:1185-1187): entries in mapping order; a lookup takes the only
    // entry of its key (a key mapped twice is left to the host: the reference re-maps ids on every
    // blockUpdate of a block, so which marker it names depends on which block was updated last)
    MT_FI void idmap_add(uint32_t key, uint32_t slot) {
        const int32_t n = idmap_n;
        if (lane == 0) idmap[n] = make_uint2(key, slot);
        idmap_n = n + 1;
        wsync();
    }
    // zamboni unlinked these markers (lanes in m): the reference's map keeps the detached segment,
    // whose getPosition is 0 (no parent)
    MT_FI void idmap_forget(uint32_t slot, uint64_t m) {
        const int32_t n = idmap_n;
        for (int32_t j0 = 0; j0 < n; j0 += kWave) {
            const int32_t j = j0 + lane;
            const uint32_t s = j < n ? idmap[j].y : kIdUnlinked;
            bool hit = false;
            for (uint64_t mm = m; mm; mm &= mm - 1) hit |= s == rdl(slot, first_lane(mm));
            if (hit) idmap[j].y = kIdUnlinked;
        }
        wsync();
    }
    // getPosition (mergeTree.ts:1586-1603): the view length of everything before `slot` on its
    // path to the root (block lengths from the settled sums + this op's overlay)
    MT_FI uint32_t get_position(uint32_t slot, int32_t ref, uint32_t c) {
        int32_t B = (int32_t)rfl((uint32_t)s_blk[slot]);
        uint32_t pos = 0, child = slot;
        for (int32_t level = 0; B != (int32_t)kNoBlk; level++) {
            const int32_t n = b_count[B];
            const uint32_t row = lane < n ? (uint32_t)b_child[B * 8 + lane] : kNoBlk;
            const uint64_t at = ballot(lane < n && row == child);
            const int32_t k = at ? first_lane(at) : n;
            uint32_t v = 0;
            if (level == 0) {  // the leaves before it
                if (lane < k) {
                    bool tie;
                    view_of(row, ref, c, v, tie);
                }
            } else if (level == 1) {  // the leaf blocks before it: their leaves (lane = 8 x block + entry)
                const int32_t ci = lane >> 3, j = lane & 7;
                const uint32_t cb = (uint32_t)__shfl((int)row, ci, kWave);
                if (ci < k && (uint32_t)j < (uint32_t)b_count[cb]) {
                    bool tie;
                    view_of(b_child[cb * 8 + j], ref, c, v, tie);
                }
            } else if (lane < k) {
                v = iview(row);
            }
            pos += rdl(scan_incl(v), 63);
            child = (uint32_t)B;
            B = (int32_t)rfl((uint32_t)b_parent[B]);
        }
        return pos;
    }
    // MT_OP_RELPOS: posFromRelativePos (mergeTree.ts:1942-1966) for the next record's pos1 / pos2
    // (client.ts:485-502).  An id with no marker gives -1 in the reference and a position below 0
    // is passed on; both, and keys the host flagged, end the document as MT_UNSUPPORTED.
    // `local`: a writer's local op (getValidOpRange's local check follows): a position of -1 (no such
    // marker) or below 0 reaches the check, which drops the op.
    MT_FI void op_relpos(const mt_op &op, bool local = false) {
        ov_splits = -1;
        ensure_overlay(op.ref_seq, MT_OP_CLIENT(op));
        int32_t pend = 0;
        for (int k = 0; k < 2; k++) {
            if (!(op.flags & (k ? MT_RELF_POS2 : MT_RELF_POS1))) continue;
            const uint32_t key = (uint32_t)(k ? op.pos2 : op.pos1);
            const int32_t n = idmap_n;
            uint32_t found = 0, slot = kIdUnlinked;
            for (int32_t j0 = 0; j0 < n; j0 += kWave) {
                const int32_t j = j0 + lane;
                const uint2 e = j < n ? idmap[j] : make_uint2(0u, 0u);
                const uint64_t hm = ballot(j < n && e.x == key);
                if (hm) slot = rdl(e.y, first_lane(hm));
                found += __popcll(hm);
            }
            if (key == kIdKeyUnsupported || found > 1u || (!local && (key == 0u || found != 1u))) {
                set_fail(ST_UNSUPPORTED);
                return;
            }
            int64_t pos = -1;
            if (key != 0u && found == 1u) {
                pos = slot == kIdUnlinked ? 0 : (int64_t)get_position(slot, op.ref_seq, MT_OP_CLIENT(op));
                const int32_t off = (int32_t)(k ? op.payload_len : op.payload);
                if (!(op.flags & (k ? MT_RELF_BEFORE2 : MT_RELF_BEFORE1))) {
                    pos += 1;  // marker.cachedLength
                    if (op.flags & (k ? MT_RELF_OFF2 : MT_RELF_OFF1)) pos += off;
                } else if (op.flags & (k ? MT_RELF_OFF2 : MT_RELF_OFF1)) {
                    pos -= off;
                }
            }
            if (local && pos < 0) pos = -1;
            if (pos > 0x7FFFFFFF || (!local && pos < 0)) {
                set_fail(ST_UNSUPPORTED);
                return;
            }
            if (k) rel_p2 = (int32_t)pos;
            else rel_p1 = (int32_t)pos;
            pend |= 1 << k;
        }
        rel_pend = pend;
    }

    // ------------------------------------------------------------------ properties
    // prop-set record in the doc pool: [n, hash, (key, value) x n] in insertion order.  The hash is
    // order-insensitive over (key, structural value class); its bit 0 is set when no value of the
    // set is irregular (mt_values.cpp), so equal classes decide matchProperties and unequal hashes
    // reject without reading the records.
    // matchProperties(a, b) (properties.ts:62-93) of two sets, a the earlier segment's
    MT_FI bool props_match(uint32_t a, uint32_t ha, uint32_t b, uint32_t hb) {
        if (a == 0 || b == 0) return a == b;
        if ((ha | hb) & kSetNever) return false;  // a value that matches nothing (NaN !== NaN)
        if (a == b) return true;
        if ((ha & hb & kSetRegular) && ha != hb) return false;
        const uint32_t na = pool[a], nb = pool[b];
        if (na != nb) return false;
        if constexpr (!kBig) {  // sets of at most 64 pairs: one of a's per lane
            bool ok = true, unk = false;
            if ((uint32_t)lane < na) {
                const uint32_t k = pool[a + 2 + 2 * lane], va = pool[a + 3 + 2 * lane];
                int rel = 0;
                for (uint32_t i = 0; i < nb; i++)
                    if (pool[b + 2 + 2 * i] == k)
                        rel = value_rel(va, pool[b + 3 + 2 * i], vt->cls, vt->flags, vt->n_values, vt->exc, vt->n_exc);
                ok = rel == 1;
                unk = rel < 0;
            }
            if (ballot(unk)) set_fail(ST_UNSUPPORTED);  // an undecided structural compare (kVUnknown)
            return ballot(!ok) == 0;
        }
        // one of a's pairs per lane, 64 at a time (sets of any size)
        for (uint32_t b0 = 0; b0 < na; b0 += kWave) {
            const uint32_t j = b0 + (uint32_t)lane;
            bool ok = true, unk = false;
            if (j < na) {
                const uint32_t k = pool[a + 2 + 2 * j], va = pool[a + 3 + 2 * j];
                int rel = 0;
                for (uint32_t i = 0; i < nb; i++)
                    if (pool[b + 2 + 2 * i] == k)
                        rel = value_rel(va, pool[b + 3 + 2 * i], vt->cls, vt->flags, vt->n_values, vt->exc, vt->n_exc);
                ok = rel == 1;
                unk = rel < 0;
            }
            if (ballot(unk)) {  // an undecided structural compare (kVUnknown)
                set_fail(ST_UNSUPPORTED);
                return false;
            }
            if (ballot(!ok)) return false;
        }
        return true;
    }

    // combiningOp (segmentPropertiesManager.ts:96-101, properties.ts:26-60) per key, lane-parallel
    // (an op's keys are distinct, so its keys do not see each other): the value to assign — a
    // present key keeps its value (assigning it is the identity) except that "incr" makes a number
    // / boolean / NaN NaN; an absent key gets the host's result (0: stays absent).  Lane i < nop
    // holds key ok_k; keys / vals (scratch) hold the set's n pairs.  Returns true when the device
    // cannot reproduce it (incr of a string / object, consensus updating a shared object in place,
    // an undefined result): the document is MT_UNSUPPORTED.
    // (big: the set's pairs are in the pool at big[2 j], big[2 j + 1] instead, any n)
    MT_FI bool combine_values(uint32_t ckind, const mt_prop *op, uint32_t nop, uint32_t n, uint32_t ok_k,
                              uint32_t &ok_v, bool inplace = false, const uint32_t *big = nullptr) {
        // the result slot: value = an absent key's result, key = the NaN value for "incr"
        // (mt_host.cpp rc_resolve_combine)
        const mt_prop res = op[nop + 2];
        const uint32_t nv = vt->n_values;
        uint32_t ev = MT_VALUE_NULL;
        if (kBig && big) {
            for (uint32_t j = 0; j < n; j++)
                if (big[2 * j] == ok_k) ev = big[2 * j + 1];
        } else {
            // lane j < n: the set's pair j; lane i < nop finds its key among them
            const uint32_t kj = (uint32_t)lane < n ? scratch[lane] : MT_KEY_COMBINE;
            const uint32_t vj = (uint32_t)lane < n ? scratch[64 + lane] : MT_VALUE_NULL;
            for (uint32_t j = 0; j < n; j++)
                if (rdl(kj, (int)j) == ok_k) ev = rdl(vj, (int)j);
        }
        bool bad = false;
        if ((uint32_t)lane < nop) {
            if (ev != MT_VALUE_NULL) {
                const uint32_t f = ev < nv ? vt->flags[ev] : 0u;
                // incr: `v += undefined` is NaN for a number / boolean; a string or object would
                // concatenate "undefined" (not modelled on the device).  consensus of an object
                // with seq === -1 would update a shared object in place.
                // (a local consensus sets such an object's seq to -1: no change, kCombineConsensusLocal)
                bad = ckind == MT_COMBINE_INCR ? (!(f & kVNum) || res.key >= nv)
                                               : ((ckind == MT_COMBINE_CONSENSUS || ckind == kCombineConsensusAck) &&
                                                  (f & kVSeqM1));
                ok_v = ckind == MT_COMBINE_INCR ? res.key : ev;
                // the { value: undefined, seq: -1 } this replica's local consensus made (the slot's
                // key: mt_host.cpp rc_resolve_combine) is a marker's own object (markers never
                // split): a sequenced consensus — updateConsensusProperty's re-combine at the ack,
                // or a remote op while the local one is pending (`inplace`) — sets its seq in
                // place, giving the value an absent key gets
                if (ev == res.key && (ckind == kCombineConsensusAck || (ckind == MT_COMBINE_CONSENSUS && inplace))) {
                    ok_v = res.value;
                    bad = res.value != MT_VALUE_NULL && res.value >= nv;
                }
            } else {
                ok_v = res.value;
                bad = res.value != MT_VALUE_NULL && res.value >= nv;
            }
        }
        return ballot(bad) != 0;
    }

    // props_extend for a set that may outgrow one pair per lane (TextSegment.make / annotate copy
    // any number of keys: properties.ts:95, textSegment.ts:23-28): the new set is built in place in
    // the pool, 64 pairs at a time — the old pairs copied, rewrite's deletions compacted, then the
    // op's pairs applied in order (delete: the pairs after it move down one) — with the semantics and
    // the content hash of the lane path, so both give equal sets equal hashes.  A combiningOp over
    // more than 64 keys is MT_UNSUPPORTED (its per-key results are held one per lane).
    MT_FI uint32_t props_extend_big(uint32_t old, const mt_prop *op, uint32_t nop, bool rewrite, uint32_t &hout,
                                    uint32_t ckind, uint32_t pk, uint32_t npk, bool inplace) {
        if constexpr (!kBig) return 0;
        if (ckind != MT_COMBINE_NONE && nop > 64u) {
            set_fail(ST_UNSUPPORTED);
            return 0;
        }
        const uint32_t n0 = old ? rfl(pool[old]) : 0u;
        if (pool_top + 2u + 2u * (n0 + nop) > pool_end) {
            cap_fail(3);
            return 0;
        }
        const uint32_t id = pool_top;
        uint32_t *kv = pool + id + 2;  // pair j: kv[2 j] key, kv[2 j + 1] value
        for (uint32_t i = (uint32_t)lane; i < 2u * n0; i += kWave) kv[i] = pool[old + 2 + i];
        wsync();
        uint32_t n = n0;
        uint32_t ok_v = 0;  // a combiningOp's value for op key `lane`
        if (ckind != MT_COMBINE_NONE) {
            uint32_t ok_k = 0;
            if ((uint32_t)lane < nop) {
                ok_k = op[lane].key;
                ok_v = op[lane].value;
            }
            if (combine_values(ckind, op, nop, n, ok_k, ok_v, inplace, kv)) {
                set_fail(ST_UNSUPPORTED);
                return 0;
            }
        }
        if (rewrite) {  // delete existing keys whose new value is absent or falsy (segmentPropertiesManager.ts:70-80)
            uint32_t w = 0;
            for (uint32_t b0 = 0; b0 < n; b0 += kWave) {
                const uint32_t j = b0 + (uint32_t)lane;
                uint32_t k = 0, v = 0;
                bool keep = false;
                if (j < n) {
                    k = kv[2 * j];
                    v = kv[2 * j + 1];
                    for (uint32_t i = 0; i < nop; i++) {
                        const mt_prop q = op[i];
                        if (q.key == k && q.value < vt->n_values && !(vt->flags[q.value] & 1u)) keep = true;
                    }
                    for (uint32_t i = 0; i < npk; i++) keep |= rdl(pk, (int)i) == k;
                }
                const uint64_t km = ballot(keep);
                wsync();  // the chunk is read before it is compacted (destinations <= sources)
                if (keep) {
                    const uint32_t dst = w + (uint32_t)__popcll(km & ((1ull << lane) - 1ull));
                    kv[2 * dst] = k;
                    kv[2 * dst + 1] = v;
                }
                w += (uint32_t)__popcll(km);
                wsync();
            }
            n = w;
        }
        for (uint32_t i = 0; i < nop; i++) {
            const uint32_t k = rfl(op[i].key);
            const uint32_t v = ckind != MT_COMBINE_NONE ? rdl(ok_v, (int)i) : rfl(op[i].value);
            if (npk && ballot((uint32_t)lane < npk && pk == k)) continue;  // a pending local key
            int32_t at = -1;
            for (uint32_t b0 = 0; b0 < n && at < 0; b0 += kWave) {
                const uint32_t j = b0 + (uint32_t)lane;
                const uint64_t hb = ballot(j < n && kv[2 * j] == k);
                if (hb) at = (int32_t)(b0 + (uint32_t)first_lane(hb));
            }
            if (v == MT_VALUE_NULL) {
                if (at >= 0) {
                    for (uint32_t b0 = (uint32_t)at + 1u; b0 < n; b0 += kWave) {
                        const uint32_t j = b0 + (uint32_t)lane;
                        uint32_t kk = 0, vv = 0;
                        if (j < n) {
                            kk = kv[2 * j];
                            vv = kv[2 * j + 1];
                        }
                        wsync();
                        if (j < n) {
                            kv[2 * j - 2] = kk;
                            kv[2 * j - 1] = vv;
                        }
                        wsync();
                    }
                    n--;
                }
            } else if (at >= 0) {
                if (lane == 0) kv[2 * (uint32_t)at + 1] = v;
                wsync();
            } else {
                if (lane == 0) {
                    kv[2 * n] = k;
                    kv[2 * n + 1] = v;
                }
                n++;
                wsync();
            }
        }
        uint32_t h = 0;
        bool irr = false, never = false;
        for (uint32_t b0 = 0; b0 < n; b0 += kWave) {
            const uint32_t j = b0 + (uint32_t)lane;
            if (j < n) {
                const uint32_t k = kv[2 * j], v = kv[2 * j + 1];
                const bool known = v < vt->n_values;
                const uint32_t f = known ? vt->flags[v] : 0u;
                h += hash_pair(k, known ? vt->cls[v] : 0xFFFFFFFFu - v);
                never |= (f & kVNever) != 0;
                irr |= !known || (f & (kVIrregular | kVUnknown | kVNever));
            }
        }
        for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, kWave);
        h = (rfl(h) & ~(kSetRegular | kSetNever)) | (ballot(irr) ? 0u : kSetRegular) | (ballot(never) ? kSetNever : 0u);
        if (lane == 0) {
            pool[id] = n;
            pool[id + 1] = h;
        }
        pool_top = id + 2u + 2u * n;
        hout = h;
        wsync();
        return id;
    }

    // SegmentPropertiesManager.addProperties for a sequenced remote op (or insert-time props):
    // start from `old` (0 = undefined -> new empty map), apply rewrite then the op's pairs in
    // order (null deletes: properties.ts:95-116).  Returns the new set id (hash in hout).
    // ckind != 0: a combiningOp (segmentPropertiesManager.ts:96-101, properties.ts:26-60) — only
    // the op's keys count; a key the set lacks gets `cres` (the host's combine of an undefined
    // current value, mt_host.cpp rc_resolve_combine; 0 = stays absent), a key it has keeps its
    // value, except that "incr" turns a number / boolean / NaN into NaN.
    // Writer: pk / npk (lane j < npk: key j) are the keys of pending local annotates on the segment,
    // which a remote op leaves alone (shouldModifyKey, segmentPropertiesManager.ts:56-63).
    // Sets and ops of at most 64 pairs together are built in LDS, one pair per lane; larger ones
    // in the pool itself (props_extend_big).  The caller reserved 2 + 2 (set size + nop) pool words.
    MT_FI uint32_t props_extend(uint32_t old, const mt_prop *op, uint32_t nop, bool rewrite, uint32_t &hout,
                                uint32_t ckind = 0u, uint32_t pk = 0u, uint32_t npk = 0u, bool inplace = false) {
        uint32_t *keys = scratch;
        uint32_t *vals = scratch + 64;
        uint32_t n = old ? pool[old] : 0u;
#ifdef MT_EXP_NOBIG
        if (n + nop > 64u) { cap_fail(3); return 0; }
#else
        if constexpr (kBig) {
            if (n + nop > 64u) return props_extend_big(old, op, nop, rewrite, hout, ckind, pk, npk, inplace);
        } else if (n > 64u || nop > 64u) {
            cap_fail(kCapPool);  // the bigprops kernel re-runs the document
            return 0;
        }
#endif
        wsync();
        if ((uint32_t)lane < n) {
            keys[lane] = pool[old + 2 + 2 * lane];
            vals[lane] = pool[old + 3 + 2 * lane];
        }
        uint32_t ok_k = 0, ok_v = 0;
        if ((uint32_t)lane < nop) {
            // the lane index through an empty asm: the address is formed here, not hoisted out of the
            // op loop into a register the 128-VGPR classes would spill
            uint32_t li = (uint32_t)lane;
            asm volatile("" : "+v"(li));
            const mt_prop pr = op[li];
            ok_k = pr.key;
            ok_v = pr.value;
        }
        wsync();
        if (ckind != MT_COMBINE_NONE && combine_values(ckind, op, nop, n, ok_k, ok_v, inplace)) {
            set_fail(ST_UNSUPPORTED);
            return 0;
        }
        if (rewrite) {
            // delete existing keys whose new value is absent or falsy (segmentPropertiesManager.ts:70-80)
            bool keep = false;
            if ((uint32_t)lane < n) {
                uint32_t k = keys[lane];
                for (uint32_t i = 0; i < nop; i++) {
                    uint32_t kk = rdl(ok_k, (int)i), vv = rdl(ok_v, (int)i);
                    if (kk == k && vv < vt->n_values && !(vt->flags[vv] & 1u)) keep = true;
                }
                for (uint32_t i = 0; i < npk; i++) keep |= rdl(pk, (int)i) == k;
            }
            uint64_t kb = ballot(keep && (uint32_t)lane < n);
            uint32_t nk = 0, kv = 0, vv2 = 0;
            if ((uint32_t)lane < n) {
                kv = keys[lane];
                vv2 = vals[lane];
            }
            wsync();
            if (keep) {
                uint32_t dst = __popcll(kb & ((1ull << lane) - 1ull));
                keys[dst] = kv;
                vals[dst] = vv2;
            }
            nk = __popcll(kb);
            n = nk;
            wsync();
        }
        for (uint32_t i = 0; i < nop; i++) {
            uint32_t k = rdl(ok_k, (int)i), v = rdl(ok_v, (int)i);
            if (npk && ballot((uint32_t)lane < npk && pk == k)) continue;  // a pending local key
            bool hit = (uint32_t)lane < n && keys[lane] == k;
            uint64_t b = ballot(hit);
            if (v == MT_VALUE_NULL) {
                if (b) {
                    int at = first_lane(b);
                    uint32_t kk = 0, vv = 0;
                    bool mv = (uint32_t)lane > (uint32_t)at && (uint32_t)lane < n;
                    if (mv) {
                        kk = keys[lane];
                        vv = vals[lane];
                    }
                    wsync();
                    if (mv) {
                        keys[lane - 1] = kk;
                        vals[lane - 1] = vv;
                    }
                    n--;
                    wsync();
                }
            } else if (b) {
                int at = first_lane(b);
                if (lane == 0) vals[at] = v;
                wsync();
            } else {
                if (n >= 64u) {
                    cap_fail(kCapPool);
                    return 0;
                }
                if (lane == 0) {
                    keys[n] = k;
                    vals[n] = v;
                }
                n++;
                wsync();
            }
        }
        uint32_t words = 2 + 2 * n;
        if (pool_top + words > pool_end) {
            cap_fail(3);
            return 0;
        }
        uint32_t id = pool_top;
        pool_top += words;
        uint32_t h = 0;
        bool irr = false, never = false;
        if ((uint32_t)lane < n) {
            uint32_t k = keys[lane], v = vals[lane];
            const bool known = v < vt->n_values;
            const uint32_t f = known ? vt->flags[v] : 0u;
            h = hash_pair(k, known ? vt->cls[v] : 0xFFFFFFFFu - v);
            never = (f & kVNever) != 0;
            irr = !known || (f & (kVIrregular | kVUnknown | kVNever));
            pool[id + 2 + 2 * lane] = k;
            pool[id + 3 + 2 * lane] = v;
        }
        // order-insensitive content hash (matchProperties ignores key order), bit 0 = regular,
        // bit 1 = a value that matches nothing (such a set does not even match itself)
        for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, kWave);
        h = (rfl(h) & ~(kSetRegular | kSetNever)) | (ballot(irr) ? 0u : kSetRegular) | (ballot(never) ? kSetNever : 0u);
        if (lane == 0) {
            pool[id] = n;
            pool[id + 1] = h;
        }
        hout = h;
        wsync();
        return id;
    }

    // ------------------------------------------------------------------ scour / pack / zamboni
    // scourNode (mergeTree.ts:1289-1365) over up to 64 leaves, one per lane (`slot`, valid for
    // lane < n), which may come from several blocks: `startM` marks each block's first leaf,
    // where the append chain restarts (each scourNode call starts afresh).  Kept slots are
    // written to hold[0..] in order; returns their count.  Only settled leaves are merged or
    // unlinked (settle_all ran at this minSeq), so the settled block sums are unchanged.
    // The TextSegment.canAppend chain (textSegment.ts:63-68, whose length test depends on
    // earlier appends) runs serially on scalars.
    MT_FI int32_t scour(uint32_t slot, int32_t n, uint64_t startM, uint32_t *hold) {
        PF_SCOPE(7);
        const bool in = lane < n;
        uint32_t meta = 0, len = 0;
        uint4 cr = make_uint4(0, 0, 0, 0);
        if (in) {
            meta = s_meta[slot];
            len = s_len[slot];
        }
        // settle_all ran at this minSeq: a settled leaf has seq <= minSeq, and removedSeq <= minSeq
        // when removed; every other leaf is unsettled
        const bool sett = in && is_settled(meta);
        const bool rem = (meta & kFRemoved) != 0u;
        // writer: a segment in a pending group is held as is and breaks the append chain
        // (scourNode: segmentGroups not empty, mergeTree.ts:1295, 1353-1356)
        const bool pend = kW && (meta & kFPending) != 0u;
        const bool cand = sett && !rem && !pend;
        const uint32_t mprev = __shfl_up(meta, 1, kWave);
        const uint64_t candM = ballot(cand);
        const uint64_t freeR = ballot(sett && rem && !pend);
        const uint64_t liveM = ballot(in);
        // lane k may append to the chain ending at lane k - 1 (TextSegment.canAppend without its
        // length rule, plus matchProperties): both candidates, same block, neither a Marker, the
        // tail not ending in '\n'
        const bool pair = lane > 0 && cand && ((candM >> (lane - 1)) & 1ull) && !((startM >> lane) & 1ull) &&
                          !(meta & kFMarker) && !(mprev & kFMarker) && !(mprev & kFEndsNL);
        // matchProperties: two leaves without prop sets match without reading HBM
        const bool noprops = !((meta | mprev) & kFHasProps);
        uint64_t pairM = ballot(pair && noprops);
        const uint64_t withM = ballot(pair && !noprops);
        const uint64_t longM = ballot(in && len > kGranularity);
        // the cold records (HBM) only of the leaves a candidate pair involves, both sides — every
        // read below (prop sets, the append heads and tails) is of such a leaf; each record is its
        // own 128-byte line (measured: 6 % of the replay's fetched bytes)
        {
            const uint64_t allP = pairM | withM;
            if ((((allP | (allP >> 1)) >> lane) & 1ull) != 0ull) cr = cold[2 * slot];
#ifdef MT_PROF
            if (allP) {  // the wait for those records (and any earlier vector-memory traffic)
                PF_SCOPE(12);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
#endif
        }
        bool serial = false;
        if (withM) {
            const uint32_t props = cr.x, ph = props ? pool[props + 1] : 0u;
            // an irregular set (a value matching across structural classes) makes matchProperties
            // intransitive: decide the chains serially against their heads, as scourNode does (only
            // leaves in a pair carry their set here: a chain without an irregular set merges the
            // same pairwise as serially)
            serial = ballot(cand && props != 0u && !(ph & 1u)) != 0;
            if (!serial) {
                const uint32_t pprev = __shfl_up(props, 1, kWave), hprev = __shfl_up(ph, 1, kWave);
                const bool peq = pprev == props;
                const bool pmaybe = !peq && props != 0u && pprev != 0u && hprev == ph;
                pairM |= withM & ballot(peq);
                uint64_t maybeM = withM & ballot(pmaybe);
                while (maybeM) {  // equal hashes, different sets: compare contents (rare)
                    const int k = first_lane(maybeM);
                    maybeM &= maybeM - 1;
                    if (props_match(rdl(props, k - 1), rdl(ph, k - 1), rdl(props, k), rdl(ph, k))) pairM |= 1ull << k;
                }
            }
        }
        uint64_t mergeM;
        if (serial) {
            // scourNode's loop (mergeTree.ts:1300-1345): prev = the chain head; canAppend's
            // structural part is lane-pairwise (pair), its length rule and matchProperties use the head
            const uint64_t structM = ballot(pair);
            mergeM = 0;
            int32_t h = 0;
            uint32_t acc = 0;
            for (int32_t k = 0; k < n; k++) {
                const uint32_t lk = rdl(len, k);
                if ((structM >> k) & 1ull) {
                    const uint32_t pa = rdl(cr.x, h), pb = rdl(cr.x, k);
                    if ((acc <= kGranularity || lk <= kGranularity) &&
                        props_match(pa, pa ? rfl(pool[pa + 1]) : 0u, pb, pb ? rfl(pool[pb + 1]) : 0u)) {
                        mergeM |= 1ull << k;
                        acc += lk;
                        continue;
                    }
                }
                h = k;
                acc = lk;
            }
        } else if (!(pairM & longM)) {
            // every appended leaf is <= 256 long, so the length rule never fails: all pairs merge
            mergeM = pairM;
        } else {
            // a long leaf appends only while its chain is still <= 256 long: walk the chains
            mergeM = 0;
            uint32_t acc = 0;
            for (int32_t k = 0; k < n; k++) {
                const uint32_t lk = rdl(len, k);
                if (((pairM >> k) & 1ull) && (acc <= kGranularity || lk <= kGranularity)) {
                    mergeM |= 1ull << k;
                    acc += lk;
                } else {
                    acc = lk;
                }
            }
        }
        if (status) return 0;
        // chain head of every appended lane: the last non-appended lane before it
        const uint32_t head = 63u - (uint32_t)__builtin_clzll((~mergeM & ((1ull << lane) - 1ull)) | 1ull);
        // TextSegment.append for every merge, head by head in document order
        if (mergeM) {
            PF_SCOPE(8);
            uint64_t m = mergeM;
            int32_t h = -1;
            uint32_t hslot = 0, pl = 0, ptoff = 0, pcap = 0, hmeta = 0, hprops = 0, hov = 0;
            bool gcd = false;  // a compaction (text_gc, only from arena_alloc below) moved the texts
            uint32_t dd = 0, ds = 0, dl = 0;  // queued text copies (MT_TEXT_BATCH), lane i = copy i
            int32_t nq = 0;
            while (m) {
                const int k = first_lane(m);
                m &= m - 1;
                const int32_t hk_ = (int32_t)rdl(head, k);
                if (hk_ != h) {
                    h = hk_;
                    hslot = rdl(slot, h);
                    pl = rdl(len, h);
                    hprops = rdl(cr.x, h);
                    hov = rdl(cr.y, h);
                    ptoff = rdl(cr.z, h);
                    pcap = rdl(cr.w, h);
                    hmeta = rdl(meta, h);
                }
                const uint32_t fslot = rdl(slot, k), sl = rdl(len, k);
                uint32_t stoff = rdl(cr.z, k), stcap = rdl(cr.w, k);
                if (gcd) {  // a compaction moved texts: offsets are in HBM again
                    const uint4 hc = cold[2 * hslot], fc = cold[2 * fslot];
                    ptoff = hc.z;
                    pcap = hc.w;
                    stoff = fc.z;
                    stcap = fc.w;
                }
                const uint32_t need = pl + sl;
                if (need > kMaxLen) {  // beyond 16-bit lengths: the document continues in the HBM class
                    if (nq) text_flush(dd, ds, dl, nq);
                    cap_fail(kCapLongSeg);
                    return 0;
                }
                bool append = false;
                if (pcap == pl && ptoff + pl == stoff) {
                    // texts already adjacent (split halves, consecutive payloads): take over the region
                    pcap = pl + stcap;
                } else if (pcap >= need) {
                    append = true;
                } else if (ptoff >= arena_base && ptoff < arena_end && ptoff + pcap == arena_top &&
                           ptoff + 2u * need <= arena_end) {
                    // last allocation of the arena: grow in place
                    pcap = 2u * need;
                    arena_top = ptoff + pcap;
                    append = true;
                } else {
                    // reallocate; a compaction inside arena_alloc moves every text, so the head
                    // is written back first and both offsets re-read afterwards (the queued copies
                    // land first: the head's text and the compaction read them)
                    if (nq) text_flush(dd, ds, dl, nq);
                    s_len[hslot] = (Len)pl;
                    if (lane == 0) cold[2 * hslot] = make_uint4(hprops, hov, ptoff, pcap);
                    wsync();
                    const uint32_t ncap = 2u * need;
                    const int32_t g0 = text_gcs;
                    const uint32_t dst = arena_alloc(ncap);
                    if (status) return 0;
                    if (text_gcs != g0) {
                        gcd = true;
                        ptoff = cold[2 * hslot].z;
                        stoff = cold[2 * fslot].z;
                    }
#ifndef MT_EXP_NOTEXT
                    text_copy(dst, ptoff, pl);
                    text_copy(dst + pl, stoff, sl);
#endif
                    ptoff = dst;
                    pcap = (ncap + 1u) & ~1u;
                }
#ifdef MT_EXP_NOTEXT  // experiment: the merges' text copies skipped (an upper bound of hiding them)
                append = false;
#endif
                if (append) {
                    if (kTextBatch && sl <= (uint32_t)kWave) {
                        if (nq == kTextQ) text_flush(dd, ds, dl, nq);
                        if (lane == nq) {
                            dd = ptoff + pl;
                            ds = stoff;
                            dl = sl;
                        }
                        nq++;
                    } else {
                        text_copy(ptoff + pl, stoff, sl);
                    }
                }
                pl = need;
                const uint32_t fm = rdl(meta, k);
                hmeta = (hmeta & ~kFEndsNL) | (fm & (kFEndsNL | kFHasNL));
                s_len[hslot] = (Len)pl;
                if (lane == 0) cold[2 * hslot] = make_uint4(hprops, hov, ptoff, pcap);
                s_meta[hslot] = (Meta)hmeta;
                wsync();
            }
            if (nq) text_flush(dd, ds, dl, nq);
        }
        // unlink removed-below-minSeq leaves and appended ones; keep the rest in order
        const uint64_t freeM = freeR | mergeM;
        const uint64_t holdM = liveM & ~freeM;
        const uint64_t below = (1ull << lane) - 1ull;
        wsync();
        // freed slots are pushed on the free list, linked through s_blk in lane order
        const uint64_t above = ~((2ull << lane) - 1ull);
        const uint64_t nxtM = freeM & above;
        const int32_t nxt = __shfl((int)slot, nxtM ? first_lane(nxtM) : 0, kWave);
        if ((freeM >> lane) & 1ull) {
            s_meta[slot] = (Meta)kUNone;  // unlinked
            s_blk[slot] = (Idx)(nxtM ? (uint32_t)nxt : (free_head < 0 ? kNoBlk : (uint32_t)free_head));
        }
        if (freeM) {
            free_head = (int32_t)rdl(slot, first_lane(freeM));
            heap_forget(slot, freeM);
            const uint64_t mkM = freeR & ballot((meta & kFMarker) != 0u);
            if (mkM) idmap_forget(slot, mkM);
        }
        free_n += __popcll(freeM);
        if ((holdM >> lane) & 1ull) hold[__popcll(holdM & below)] = slot;
        wsync();
        return __popcll(holdM);
    }

    // Regroup `nk` children (hold[0..nk)) of `parent`'s former child blocks into
    // floor(nk / 4) (1..7) new blocks of near-equal size, first blocks one larger
    // (pack, mergeTree.ts:1389-1411).  Leaf mode also moves the leaves' s_blk.
    MT_FI int32_t regroup(int32_t parent, int32_t pn, const uint32_t *hold, int32_t nk, int leaf, int32_t level) {
        int32_t cc = nk / (kMaxNodes / 2);
        if (cc > kMaxNodes - 1) cc = kMaxNodes - 1;
        if (cc < 1) cc = 1;
        const int32_t base = nk / cc, extra = nk % cc;
        wsync();
        // the cc new blocks (MergeTree.makeBlock) reuse the ids of the old child blocks; surplus old
        // blocks go to the free list, missing ones come off it
        uint32_t id = lane < pn ? (uint32_t)b_child[parent * 8 + lane] : 0u;
        wsync();
        for (int32_t q = cc; q < pn; q++) free_block((int32_t)rdl(id, q));
        for (int32_t q = pn; q < cc; q++) {
            const int32_t nb = alloc_block(leaf, level);
            if (status) return cc;
            if (lane == q) id = (uint32_t)nb;
        }
        wsync();
        if (lane < cc) {
            b_leaf[id] = (uint8_t)leaf;
            b_scour[id] = kScourUndef;
            b_parent[id] = (Idx)parent;
            if (!leaf) b_slen[si(id)] = 0u;
            b_count[id] = (uint8_t)(base + (lane < extra ? 1 : 0));
            b_child[parent * 8 + lane] = (Idx)id;
        }
        // leaf i goes to block q at position p
        uint32_t c = 0, sl = 0;
        const bool in = lane < nk;
        if (in) c = hold[lane];
        const int32_t big = extra * (base + 1);
        const int32_t q = lane < big ? lane / (base + 1) : extra + (lane - big) / (base > 0 ? base : 1);
        const int32_t p = lane < big ? lane % (base + 1) : (lane - big) % (base > 0 ? base : 1);
        const uint32_t nb = (uint32_t)__shfl((int)id, in ? q : 0, kWave);
        wsync();
        if (in) {
            b_child[nb * 8 + p] = (Idx)c;
            if (leaf) {
                s_blk[c] = (Idx)nb;  // (leaf blocks keep no length)
            } else {
                b_parent[c] = (Idx)nb;
                sl = level == 1 ? leaf_block_settled(c) : (uint32_t)b_slen[si(c)];
            }
        }
        wsync();
        if (!leaf && in && sl) b_slen.add(si(nb), sl);
        b_count[parent] = (uint8_t)cc;
        splits++;  // structure changed under the overlay
        wsync();
        return cc;
    }

    // the children of parent's child blocks, in order, gathered one per lane (8 lanes per
    // child block) and compacted into dst[0..total); returns total, block starts in *startM
    MT_FI int32_t gather_grandchildren(int32_t parent, int32_t pn, uint32_t *dst, uint64_t *startM) {
        const int32_t ci = lane >> 3, j = lane & 7;
        uint32_t cb = 0, cn = 0, g = 0;
        if (ci < pn) {
            cb = b_child[parent * 8 + ci];
            cn = b_count[cb];
            g = b_child[cb * 8 + j];
        }
        const bool valid = ci < pn && (uint32_t)j < cn;
        const uint64_t vm = ballot(valid);
        const int32_t total = __popcll(vm);
        wsync();
        if (valid) dst[__popcll(vm & ((1ull << lane) - 1ull))] = g | (j == 0 ? 0x80000000u : 0u);
        wsync();
        const uint32_t e = lane < total ? dst[lane] : 0u;
        *startM = ballot(lane < total && (e >> 31));
        wsync();
        if (lane < total) dst[lane] = e & 0x7FFFFFFFu;
        wsync();
        return total;
    }

    // pack for an interior block `blk` (its parent's children are interior blocks);
    // repeats upward while the parent underflows (mergeTree.ts:1414-1419)
    MT_FI void pack_interior(int32_t blk) {
        for (int32_t level = 1;; level++) {  // blk's level (its parent's children are regrouped)
            const int32_t parent = b_parent[blk];
            const int32_t pn = b_count[parent];
            uint64_t sm;
            const int32_t total = gather_grandchildren(parent, pn, scratch, &sm);
            const int32_t cc = regroup(parent, pn, scratch, total, 0, level);
            if (status) return;
            if (cc < kMaxNodes / 2 && parent != root) blk = parent;
            else return;
        }
    }

    // pack for a leaf block (mergeTree.ts:1368-1420): every sibling leaf block is scoured and
    // the surviving leaves are regrouped into floor(total / 4) (1..7) new leaf blocks
    MT_FI void pack_leaf(int32_t blk) {
        PF_SCOPE(10);
        const int32_t parent = b_parent[blk];
        const int32_t pn = b_count[parent];
        uint32_t *gat = scratch;
        uint32_t *hold = scratch + 64;
        uint64_t startM;
        const int32_t total = gather_grandchildren(parent, pn, gat, &startM);
        const uint32_t slot = lane < total ? gat[lane] : 0u;
        const int32_t nk = scour(slot, total, startM, hold);
        if (status) return;
        const int32_t cc = regroup(parent, pn, hold, nk, 1, 0);
        if (status) return;
        if (lab)  // every packed block: nodeUpdateLengthNewStructure (mergeTree.ts:1404)
            for (int32_t q = 0; q < cc; q++) lab_refresh(rfl((int32_t)b_child[parent * 8 + q]));
        if (cc < kMaxNodes / 2 && parent != root) pack_interior(parent);
    }

    // zamboniSegments (mergeTree.ts:1422-1478)
    MT_FI void zamboni() {
        PF_SCOPE(5);
        for (int it = 0; it < kZamboniMax; it++) {
            if (hn < 1 || htop > min_seq) break;
            if (settled_min != min_seq) settle_all();
            uint32_t key;
            int32_t mseq;
            heap_get(key, mseq);
            if (key == kHeapInvalid) continue;  // the segment was merged away / unlinked: parent undefined
            const uint32_t slot = key;
            const int32_t blk = s_blk[slot];
            // the block's scour state, child count and row loaded together (one round in the giant
            // class, whose leaf blocks are in HBM)
            const int8_t sc = b_scour[blk];
            const int32_t cnt = b_count[blk];
            const uint32_t row = lane < kMaxNodes ? (uint32_t)b_child[blk * 8 + lane] : 0u;
            if (sc == kScourFalse) continue;
            const uint32_t cs = lane < cnt ? row : 0u;
            uint32_t *hold = scratch;
            const int32_t nk = scour(cs, cnt, 1ull, hold);
            if (status) return;
            b_scour[blk] = kScourFalse;
            if (nk < cnt) {
                wsync();
                if (lane < nk) b_child[blk * 8 + lane] = (Idx)hold[lane];
                b_count[blk] = (uint8_t)nk;
                splits++;
                wsync();
                if (nk < kMaxNodes / 2 && blk != root) pack_leaf(blk);
                else lab_refresh(blk);  // blockUpdatePathLengths(block)
                if (status) return;
            }
        }
    }

    // setMinSeq (mergeTree.ts:1718-1736) via Client.updateSeqNumbers (client.ts:821-828)
    MT_FI void update_seq_numbers(int32_t msn, int32_t seq) {
        if (!(cur_seq <= seq)) {
            set_fail(ST_SEQ_ORDER);
            return;
        }
        cur_seq = seq;
        if (!(msn <= seq)) {
            set_fail(ST_MSN_ORDER);
            return;
        }
        if (!(min_seq <= msn)) {
            set_fail(ST_MSN_ORDER);
            return;
        }
        if (msn > min_seq) {
            min_seq = msn;
            zamboni();
            if constexpr (kW) {
                if (msn >= cons_next) consensus_fire();
            }
        }
    }

    // ------------------------------------------------------------------ ops
    // insertSegments + blockInsert for one remote segment (mergeTree.ts:1968-1998, 2141-2224):
    // ensureIntervalBoundary(pos) then the inserting walk, which after the split resolves to
    // the split's right half (unless the split restructured the tree: then it walks again).
    // `loaded`: a SnapshotLoader body segment (refSeq UniversalSequenceNumber) carrying its own
    // removal info (op.ref_seq / op.msn) and its settled state.
    template <bool loaded>
    MT_FI void insert_one(const mt_op &op, uint32_t c, uint32_t pos, int32_t ref) {
        ov_splits = -1;
        Walk W = boundary(pos, ref, c);
        if (status) return;
        const bool marker = (op.flags & MT_OPF_MARKER) != 0;
        const uint32_t len = marker ? 1u : op.payload_len;
        const bool local = kW && op.seq == kUnassignedSeq;  // a writer's own unacked insert
        if constexpr (kW) {
            if (!local && n_pend > 0 && len > 0 && W.blk >= 0 && W.ok && W.k == W.n) W = continue_walk(W, ref, c);
        }
        if (len > 0) {
            PF_SCOPE(3);
            if (W.blk < 0 || !W.ok) {
                set_fail(ST_INVALID_POS);
                return;
            }
            if (len > kMaxLen) {
                cap_fail(kCapLongSeg);
                return;
            }
            int32_t slot = alloc_slot();
            if (slot < 0) return;
            uint32_t props = 0, ph = 0;
            if (op.flags & MT_OPF_HAS_PROPS) {
                if constexpr (kBig) {
                    uint32_t p0 = 0;
                    const uint32_t np = mt_insert_props(&op, props_in, &p0);
                    pool_reserve(2u + 2u * np);
                    if (status) return;
                    props = props_extend(0, props_in + p0, np, false, ph);
                } else {
                    // (an extended count, MT_OPF_NPROPS_EXT = 127 > 64, stops in props_extend with
                    // kCapPool before any record is read: the bigprops kernel re-runs the document)
                    pool_reserve(2u + 2u * MT_OPF_NPROPS(op.flags));
                    if (status) return;
                    props = props_extend(0, props_in + op.pos2, MT_OPF_NPROPS(op.flags), false, ph);
                }
                if (status) return;
            }
            const int32_t rseq = loaded ? op.ref_seq : kNoneSeq;
            const uint32_t rcli = loaded && rseq != kNoneSeq ? ((uint32_t)op.msn & kMetaCli) : kNoClient;
            // a loaded segment below the collab window is settled: it joins the settled sums
            // after the leaf insert (while it moves through block splits it counts as unsettled)
            const bool settled = loaded && op.seq <= min_seq && (rseq == kNoneSeq || rseq <= min_seq);
            uint32_t meta = kFLinked | kUNone;
            if (marker) meta |= kFMarker;
            if (op.flags & MT_OPF_INTERNAL_ENDS_NL) meta |= kFEndsNL;
            if (op.flags & MT_OPF_INTERNAL_HAS_NL) meta |= kFHasNL;
            if (props) meta |= kFHasProps;
            if (rseq != kNoneSeq) meta |= kFRemoved;
            s_len[slot] = (Len)len;
            const USr sr = us_make(local ? kRUnassigned : rel(op.seq), rseq == kNoneSeq ? kRNone : rel(rseq));
            cold_init(slot, props, op.payload, marker ? props : len, (uint32_t)op.seq, (uint32_t)rseq, (c & kMetaCli) | (rcli << 16));
            s_meta[slot] = (Meta)meta;
            wsync();
            // (a settled loaded segment too, while it moves through block splits: it joins the
            // settled sums after the leaf insert)
            u_push((uint32_t)slot, sr, (c & kMetaCli) | (rcli << kCmR));
            if (status) return;
            int32_t blk = insert_leaf(W.blk, W.k, (uint32_t)slot);
            if (status) return;
            if (settled) {  // its entry is still the last one (leaf inserts push none)
                nu--;
                s_meta[slot] = (Meta)(s_meta[slot] | kUNone);
                wsync();
                if (rseq == kNoneSeq) chain_add_uniform(rfl((int32_t)s_blk[slot]), len);
            }
            // saveIfLocal (mergeTree.ts:2164-2179)
            if (local) pend_add((uint32_t)slot, op);
            else if (op.seq > min_seq) add_to_lru(blk, (uint32_t)slot, op.seq);
            // blockInsert maps a marker's id (mergeTree.ts:2200-2205); the host put the id's key
            // in payload_len (0: no id)
            if (marker && op.payload_len) idmap_add(op.payload_len, (uint32_t)slot);
        }
        resolve_splits();
        if (local) return;  // no zamboni after a local op (mergeTree.ts:1994-1997)
        if (!loaded || !(op.flags & MT_OPF_GROUP_CONT)) zamboni();
    }
    MT_FI void op_insert(const mt_op &op) { insert_one<false>(op, MT_OP_CLIENT(op), (uint32_t)op.pos1, op.ref_seq); }

    // ------------------------------------------------------------------ SnapshotLoader
    // (snapshotLoader.ts:36-205) — the header chunk's segments, MergeTree.reloadFromSegments
    // (mergeTree.ts:1195-1251): blocks of MaxNodesInBlock - 1 children built bottom up.  Appending
    // leaf by leaf to the rightmost path (a new block at a level once the last is full, a new
    // root once the top level has two blocks) gives exactly those blocks.  Lengths and the
    // overlay are set up by op_collab, once minSeq is known.
    MT_FI void op_load_header(const mt_op &op) {
        ov_splits = -1;
        const bool marker = (op.flags & MT_OPF_MARKER) != 0;
        const uint32_t len = marker ? 1u : op.payload_len;
        if (len > kMaxLen) {
            cap_fail(kCapLongSeg);
            return;
        }
        int32_t slot = alloc_slot();
        if (slot < 0) return;
        uint32_t props = 0, ph = 0;
        if (op.flags & MT_OPF_HAS_PROPS) {
            uint32_t p0 = 0;
            const uint32_t np = mt_insert_props(&op, props_in, &p0);
            if (!kBig && np > 64u) {  // (LOAD records: the load kernel is kBig)
                cap_fail(kCapPool);
                return;
            }
            pool_reserve(2u + 2u * np);
            if (status) return;
            props = props_extend(0, props_in + p0, np, false, ph);
            if (status) return;
        }
        const int32_t rseq = op.ref_seq;
        const uint32_t rcli = rseq != kNoneSeq ? ((uint32_t)op.msn & kMetaCli) : kNoClient;
        uint32_t meta = kFLinked | kUNone;  // the overlay entries are made by op_collab from the real seqs
        if (marker) meta |= kFMarker;
        if (op.flags & MT_OPF_INTERNAL_ENDS_NL) meta |= kFEndsNL;
        if (op.flags & MT_OPF_INTERNAL_HAS_NL) meta |= kFHasNL;
        if (props) meta |= kFHasProps;
        if (rseq != kNoneSeq) meta |= kFRemoved;
        s_len[slot] = (Len)len;
        cold_init(slot, props, op.payload, marker ? props : len, (uint32_t)op.seq, (uint32_t)rseq,
                  (MT_OP_CLIENT(op) & kMetaCli) | (rcli << 16));
        s_meta[slot] = (Meta)meta;
        wsync();
        // reloadFromSegments' blockUpdate maps the ids of markers with localNetLength > 0
        // (addNodeReferences, mergeTree.ts:270-285): not removed ones
        if (marker && op.payload_len && rseq == kNoneSeq) idmap_add(op.payload_len, (uint32_t)slot);
        // the rightmost leaf block
        int32_t b = root;
        for (int32_t l = 0; l + 1 < depth; l++) b = rfl((int32_t)b_child[b * 8 + b_count[b] - 1]);
        int32_t n = b_count[b];
        if (n < kMaxNodes - 1) {
            b_child[b * 8 + n] = (Idx)slot;
            b_count[b] = (uint8_t)(n + 1);
            s_blk[slot] = (Idx)b;
            wsync();
            return;
        }
        int32_t child = alloc_block(1, 0);
        if (status) return;
        b_child[child * 8] = (Idx)slot;
        b_count[child] = 1;
        s_blk[slot] = (Idx)child;
        wsync();
        int32_t left = b;
        for (int32_t level = 1;; level++) {  // the level of left's parent (and of np)
            const int32_t p = b_parent[left];
            if (p == (int32_t)kNoBlk) {  // left is the root: the top level now has two blocks
                const int32_t r = alloc_block(0, level);
                if (status) return;
                b_child[r * 8] = (Idx)left;
                b_child[r * 8 + 1] = (Idx)child;
                b_count[r] = 2;
                b_parent[left] = (Idx)r;
                b_parent[child] = (Idx)r;
                root = r;
                depth++;
                break;
            }
            const int32_t pn = b_count[p];
            if (pn < kMaxNodes - 1) {
                b_child[p * 8 + pn] = (Idx)child;
                b_count[p] = (uint8_t)(pn + 1);
                b_parent[child] = (Idx)p;
                break;
            }
            const int32_t np = alloc_block(0, level);
            if (status) return;
            b_child[np * 8] = (Idx)child;
            b_count[np] = 1;
            b_parent[child] = (Idx)np;
            child = np;
            left = p;
        }
        splits++;
        wsync();
    }

    // startOrUpdateCollaboration(observer, minSeq, currentSeq) after loadHeader
    // (snapshotLoader.ts:147-160; client.ts:1051-1071): the settled sums and the overlay list
    // of the loaded tree (MergeTree.startCollaboration recomputes the partial lengths)
    MT_FI void op_collab(const mt_op &op) {
        min_seq = op.msn;
        cur_seq = op.seq;
        settled_min = min_seq;
        sbase = min_seq;
        ov_splits = -1;
        if (!kHbm && cur_seq - sbase >= kSeq16Span) {  // 16-bit relative seqs: load in the HBM class
            cap_fail(kCapLongSeg);
            return;
        }
        wsync();
        for (int32_t i = lane; i < (kSplitPools ? lds_top : blk_top); i += kWave) b_slen[i] = 0u;
        wsync();
        for (int32_t base = 0; base < slot_top; base += kWave) {
            const int32_t slot = base + lane;
            uint32_t meta = 0;
            bool live = false, sett = false;
            uint32_t add = 0, b = 0, cm = 0;
            USr sr = 0;
            if (slot < slot_top) {
                meta = s_meta[slot];
                live = (meta & kFLinked) != 0;
                if (live) {
                    const uint4 q = cold[2 * slot + 1];  // the loaded segment's real seqs and clients
                    const int32_t sq = (int32_t)q.x, rs = (int32_t)q.y;
                    sett = sq <= min_seq && (rs == kNoneSeq || rs <= min_seq);
                    if (sett && rs == kNoneSeq) add = s_len[slot];
                    b = s_blk[slot];
                    sr = us_make(rel(sq), rs == kNoneSeq ? kRNone : rel(rs));
                    cm = (q.z & kMetaCli) | (((q.z >> 16) & kMetaCli) << kCmR);
                }
            }
            const bool un = live && !sett;
            const uint64_t um = ballot(un);
            if (nu + __popcll(um) > cap.ulist) {
                cap_fail(1);
                return;
            }
            if (un) {
                const uint32_t e = (uint32_t)nu + (uint32_t)__popcll(um & ((1ull << lane) - 1ull));
                s_meta[slot] = (Meta)((meta & ~kUNone) | e);
                u_list[e] = (Idx)slot;
                u_sr[e] = sr;
                u_cm[e] = cm;
            }
            nu += __popcll(um);
            if (nu > max_u) max_u = nu;
            chain_add(b_slen, add > 0u, b, add);
        }
        wsync();
    }

    // MergeTree.length of the local view (root.cachedLength: localNetLength, mergeTree.ts:1161)
    MT_FI uint32_t local_length() {
        uint32_t sum = 0;
        for (int32_t base = 0; base < slot_top; base += kWave) {
            const int32_t slot = base + lane;
            uint32_t v = 0;
            if (slot < slot_top) {
                const uint32_t m = s_meta[slot];
                if ((m & kFLinked) && !(m & kFRemoved)) v = s_len[slot];
            }
            sum += rdl(scan_incl(v), 63);
        }
        return sum;
    }

    // loadBody (snapshotLoader.ts:166-205): insertSegments(root.cachedLength, batch,
    // UniversalSequenceNumber, client, seq); members of a batch go in at advancing positions
    MT_FI void op_load_body(const mt_op &op) {
        const uint2 st = h_ent[0];  // {insert position, batch open}
        const uint32_t pos = rfl(st.y) ? rfl(st.x) : local_length();
        const uint32_t len = (op.flags & MT_OPF_MARKER) ? 1u : op.payload_len;
        insert_one<true>(op, MT_OP_CLIENT(op), pos, 0);
        wsync();
        if (lane == 0) h_ent[0] = make_uint2(pos + len, (op.flags & MT_OPF_GROUP_CONT) ? 1u : 0u);
        wsync();
    }

    // markRangeRemoved / annotateRange (mergeTree.ts:2565-2719): both boundaries, then the
    // nodeMap range walk leaf block by leaf block
    MT_FI void op_range(const mt_op &op) {
        const uint32_t c = MT_OP_CLIENT(op);
        const int32_t ref = op.ref_seq;
        const uint32_t start = (uint32_t)op.pos1, end = (uint32_t)op.pos2;
        ov_splits = -1;
        const int32_t s0 = splits;
        const Walk W = boundary(start, ref, c);
        if (status) return;
        const bool wok = W.blk >= 0 && splits == s0;  // no block split: W.base is the block's start
        boundary(end, ref, c);
        if (status) return;
        // nodeMap visits leaves with vlen > 0 and E < end and P > start: none when end <= start
        // (both boundaries were cut, so no leaf can straddle them).  When neither boundary split a
        // block, the walk starts at the first boundary's leaf block: every leaf before it ends
        // before start (insertingWalk takes the first block reaching start), so the range walk
        // from there visits exactly nodeMap's leaves, without a third descent.
        if (end > start) range_walk(op, start, end, wok && splits == s0 ? W.blk : -1, W.base);
        resolve_splits();
        if (kW && op.seq == kUnassignedSeq) return;  // a local op: no zamboni (mergeTree.ts:2600, 2713)
        zamboni();
    }

    // addOverlappingClient (mergeTree.ts:2544-2552) for the lanes of `m`: client c joins each
    // segment's removedClientOverlap.  Clients < 31 set a bit of the mask in cold.y; a larger
    // client turns the set into a pool list [n | kPoolOvlTag, 0, clients...] (rare: concurrent
    // removes by a client beyond the 31st).
    MT_FI void ovl_add(uint32_t slot, uint64_t m, uint32_t c) {
        for (; m; m &= m - 1) {
            const uint32_t sl = rdl(slot, first_lane(m));
            // a concurrently removed segment visible to the op: unsettled
            const uint32_t ui = rfl((uint32_t)s_meta[sl]) & kUNone;
            const uint32_t cm = rfl(u_cm[ui]);
            const uint32_t o = (cm & kCmOvl) ? rfl(cold[2 * sl].y) : 0u;
            if (!(o & kOvlList) && c < kOvlMaskClients) {
                if (lane == 0) cold[2 * sl].y = o | (1u << c);
            } else {
                // members of the old set, then c (no compaction here: a full pool stops the
                // document with MT_CAPACITY, cap_kind 3)
                const uint32_t n_old = (o & kOvlList) ? (pool[o & ~kOvlList] & ~kPoolOvlTag) : (uint32_t)__popc(o);
                if (pool_top + 3u + n_old > pool_end) {
                    cap_fail(3);
                    return;
                }
                const uint32_t ol = o & ~kOvlList;
                const uint32_t id = pool_top;
                pool_top += 3u + n_old;
                if (o & kOvlList) {
                    for (uint32_t i = lane; i < n_old; i += kWave) pool[id + 2 + i] = pool[ol + 2 + i];
                } else {
                    const bool bit = lane < (int)kOvlMaskClients && ((o >> lane) & 1u);
                    const uint64_t bm = ballot(bit);
                    if (bit) pool[id + 2 + __popcll(bm & ((1ull << lane) - 1ull))] = (uint32_t)lane;
                }
                if (lane == 0) {
                    pool[id] = (n_old + 1u) | kPoolOvlTag;
                    pool[id + 1] = 0u;
                    pool[id + 2 + n_old] = c;
                    cold[2 * sl].y = id | kOvlList;
                }
            }
            u_cm[ui] = cm | kCmOvl;
            wsync();
        }
    }

    // *closes: the interior blocks that end with b (the levels climbed to the next leaf block)
    MT_FI int32_t next_leaf_block(int32_t b, int32_t *closes = nullptr) {
        for (int32_t up = 0;; up++) {
            int32_t p = b_parent[b];
            if (p == (int32_t)kNoBlk) {
                if (closes) *closes = up;
                return -1;
            }
            // child_index with the row kept: the next sibling comes from the same load
            const int32_t n = b_count[p];
            const uint32_t row = lane < n ? (uint32_t)b_child[p * 8 + lane] : kNoBlk;
            const uint64_t hm = ballot(row == (uint32_t)b);
            const int32_t i = hm ? first_lane(hm) : -1;
            if (i + 1 < n) {
                if (closes) *closes = up;
                b = (int32_t)rdl(row, i + 1);
                // every leaf is at depth 0: `up` levels down the left edge
                for (int32_t d = 0; d < up; d++) b = b_child[b * 8];
                return b;
            }
            b = p;
        }
    }

    // blk0 >= 0: start at leaf block blk0 (view position base0) instead of a strict descent
    MT_FI void range_walk(const mt_op &op, uint32_t start, uint32_t end, int32_t blk0 = -1, uint32_t base0 = 0) {
        const uint32_t c = MT_OP_CLIENT(op);
        const int32_t ref = op.ref_seq;
        resolve_cold();  // the walk reads / updates cold records of split halves
        ensure_overlay(ref, c);
        Walk W;
        if (blk0 >= 0) {
            W.blk = blk0;
            W.base = base0;
        } else {
            W = descend(start, ref, c, true);
        }
        PF_SCOPE(4);
        const bool is_remove = op.type == MT_OP_REMOVE;
        const bool rewrite = (op.flags & MT_OPF_REWRITE) != 0;
        const bool local = kW && op.seq == kUnassignedSeq;  // a writer's own unacked op
        // per-op memo old prop-set -> new prop-set (annotate)
        uint32_t memo_n = 0;
        uint32_t memo_old = 0, memo_new = 0, memo_h = 0;  // lane i holds entry i
        int32_t blk = W.blk;
        uint32_t base = W.base;
        while (blk >= 0) {
            const int32_t n = b_count[blk];
            uint32_t slot = 0, vlen = 0;
            bool tie;
            if (lane < n) {
                slot = b_child[blk * 8 + lane];
                view_of(slot, ref, c, vlen, tie);
            }
            const uint32_t incl = scan8(vlen) + base;
            const uint32_t excl = incl - vlen;
            const bool hit = lane < n && lane < kMaxNodes && vlen > 0u && excl < end && incl > start;
            uint64_t hb = ballot(hit);
            const uint32_t bend = n > 0 ? rdl(incl, n - 1) : base;
            if (is_remove && hb) lab_refresh(blk);  // nodeMap's post action: afterMarkRemoved (mergeTree.ts:2660-2667)
            if (is_remove) {
                uint32_t meta = 0, ui = kUNone, cm = 0;
                USr sr = 0;
                if (hit) {
                    meta = s_meta[slot];
                    ui = meta & kUNone;
                    if (ui != kUNone) {
                        sr = u_sr[ui];
                        cm = u_cm[ui];
                    }
                }
                // a visible leaf already removed is a concurrent removal (hence unsettled):
                // addOverlappingClient below; a pending local removal is replaced instead
                const bool again = hit && (meta & kFRemoved) && !(kW && us_r(sr) == kRUnassigned);
                // first remover; or (writer) a sequenced remove replacing a pending local one
                // (mergeTree.ts:2624-2630: its client and seq, no overlap entry)
                const bool first = hit && !again;
                const uint32_t rq = local ? kRUnassigned : rel(op.seq);
                // a settled leaf removed now leaves the settled sums and joins the overlay
                const bool newu = first && ui == kUNone;
                const uint64_t um = ballot(newu);
                if (um && nu + __popcll(um) > cap.ulist) {
                    cap_fail(1);
                    return;
                }
                const uint32_t lost = um ? rdl(sum8(newu ? s_len[slot] : 0u), 0) : 0u;
                wsync();
                if (first) {
                    if (ui != kUNone) {
                        u_sr[ui] = us_make(us_q(sr), rq);
                        u_cm[ui] = (cm & ~(kMetaCli << kCmR)) | ((c & kMetaCli) << kCmR);
                    } else {
                        ui = (uint32_t)nu + (uint32_t)__popcll(um & ((1ull << lane) - 1ull));
                        u_list[ui] = (Idx)slot;
                        u_sr[ui] = us_make(0u, rq);  // seq <= minSeq: relative 0 (its clientId is never compared)
                        u_cm[ui] = kNoClient | ((c & kMetaCli) << kCmR);
                    }
                    s_meta[slot] = (Meta)(((meta | kFRemoved) & ~kUNone) | ui);
                    cold[2 * slot + 1].y = (uint32_t)op.seq;
                    reinterpret_cast<uint16_t *>(&cold[2 * slot + 1].z)[1] = (uint16_t)(c & kMetaCli);
                }
                if (um) {
                    nu += __popcll(um);
                    if (nu > max_u) max_u = nu;
                    chain_add_uniform(blk, 0u - lost);
                }
                const uint64_t againM = ballot(again);
                if (againM) {
                    ovl_add(slot, againM, c);
                    if (status) return;
                }
            }
            wsync();
            uint32_t oldp = 0;
            if (!is_remove && hit) oldp = cold[2 * slot].x;
            // in document order: properties (annotate) and addToLRUSet
            while (hb) {
                const int f = first_lane(hb);
                hb &= hb - 1;
                const uint32_t sl = rdl(slot, f);
                if (!is_remove) {
                    int32_t g0 = pool_gcs;
                    if constexpr (kBig) {  // room for the largest set this op can make from the segment's
                        const uint32_t o0 = rdl(oldp, f);
                        const uint32_t n0 = o0 ? rfl(pool[o0]) : 0u;
                        pool_reserve(2u + 2u * ((n0 > 64u ? n0 : 64u) + op.payload_len));
                    } else {
                        pool_reserve(2u + 2u * (64u + op.payload_len));
                    }
                    if (status) return;
                    uint32_t old;
                    if (pool_gcs != g0) {  // ids moved
                        memo_n = 0;
                        oldp = hit ? cold[2 * slot].x : 0u;
                    }
                    old = rdl(oldp, f);
                    uint64_t mb = ballot((uint32_t)lane < memo_n && memo_old == old);
                    uint32_t nid, nh;
                    bool pseg = false;
                    if constexpr (kW) pseg = !local && (s_meta[sl] & kFPending);
                    if (pseg) {
                        // a remote annotate of a segment with pending local annotates
                        // (segmentPropertiesManager.ts:48-92): nothing while a local rewrite is
                        // pending, else the pending keys are left alone unless the op combines
                        uint32_t pk, npk;
                        bool prw;
                        pending_keys(sl, pk, npk, prw);
                        if (status) return;
                        const uint32_t ck = MT_OPF_COMBINE(op.flags);
                        nid = prw ? old
                                  : props_extend(old, props_in + op.payload, op.payload_len, rewrite, nh, ck, pk,
                                                 ck ? 0u : npk, (rfl((uint32_t)s_meta[sl]) & kFMarker) != 0u);
                        if (status) return;
                    } else if (mb) {
                        int m = first_lane(mb);
                        nid = rdl(memo_new, m);
                        nh = rdl(memo_h, m);
                    } else {
                        const uint32_t ck = MT_OPF_COMBINE(op.flags);
                        nid = props_extend(old, props_in + op.payload, op.payload_len, rewrite, nh,
                                           local && ck == MT_COMBINE_CONSENSUS ? kCombineConsensusLocal : ck);
                        if (status) return;
                        if (memo_n < 64u) {
                            if ((uint32_t)lane == memo_n) {
                                memo_old = old;
                                memo_new = nid;
                                memo_h = nh;
                            }
                            memo_n++;
                        }
                    }
                    if (lane == 0) cold[2 * sl].x = nid;
                    if (nid) s_meta[sl] = (Meta)(s_meta[sl] | kFHasProps);
                }
                if (local) pend_add(sl, op);
                else add_to_lru(blk, sl, op.seq);
                if (status) return;
            }
            wsync();
            if (bend >= end) break;
            blk = next_leaf_block(blk);
            base = bend;
        }
    }

    // SnapshotLoader records (mt_load_kernel only): no sequence checks, no updateSeqNumbers
    MT_FI void apply_load(const mt_op &op) {
        pend_n = 0;
        const uint32_t oc = MT_OP_CLIENT(op);
        const bool noncollab = oc == MT_CLIENT_NONCOLLAB;
        if (op.type != MT_OP_COLLAB && (oc == 0 || (oc >= (uint32_t)kMaxClients && !noncollab))) {
            set_fail(ST_UNSUPPORTED);
            return;
        }
        if (op.type == MT_OP_LOAD_HEADER) op_load_header(op);
        else if (op.type == MT_OP_COLLAB) op_collab(op);
        else op_load_body(op);
        resolve_splits();
    }

    // a local op of a writer replica: Client.insertSegmentLocal / removeRangeLocal /
    // annotateRangeLocal (client.ts:201-291) -> applyXOp with the local args (currentSeq, own
    // client, UnassignedSequenceNumber; 553-563).  getValidOpRange's local check (504-543): an
    // invalid range is logged (InvalidOpRange) and the op is not applied.
    MT_FI void op_local(mt_op op) {
        if (MT_OP_CLIENT(op) != 0u) {
            set_fail(ST_BAD_INPUT);
            return;
        }
        if (op.type == MT_OP_REGENERATE) {
            op_regenerate(op);
            return;
        }
        if (op.type == MT_OP_RELPOS) {  // posFromRelativePos in the local view (client.ts:485-502)
            ntf = (op.flags & MT_RELF_NOTIFY) ? 1 : 0;
            ntf_raw = op.payload;
            op.ref_seq = cur_seq;
            op_relpos(op, true);
            return;
        }
        const bool notify = ntf != 0;
        ntf = 0;
        if (notify && !(op.type == MT_OP_ANNOTATE && MT_OPF_COMBINE(op.flags) == MT_COMBINE_CONSENSUS)) {
            set_fail(ST_BAD_INPUT);
            return;
        }
        if (op.type != MT_OP_INSERT && op.type != MT_OP_REMOVE && op.type != MT_OP_ANNOTATE) {
            if (op.type != MT_OP_NOOP) set_fail(ST_BAD_INPUT);
            return;
        }
        const int32_t len = (int32_t)view_length(cur_seq, 0u);  // getLength(): the local view
        const int32_t st = op.pos1;
        if (st < 0 || st > len || (st == len && op.type != MT_OP_INSERT)) return;
        if (op.type != MT_OP_INSERT && op.pos2 <= st) return;
        op.ref_seq = cur_seq;
        cur_g = -1;
        ov_splits = -1;
        if (lane == 0) pend[4] = pend_word(4) + 1u;  // ++collabWindow.localSeq (mergeTree.ts:1976, 2571, 2613)
        if (op.type == MT_OP_INSERT) insert_one<false>(op, 0u, (uint32_t)st, cur_seq);
        else op_range(op);
        // annotateMarkerNotifyConsensus: pendingConsensus.set(marker.getId(), ...) once the
        // annotate applied (client.ts:124-130)
        if (notify && !status) consensus_register(ntf_raw);
    }

    // pendingConsensus.set(id, ...): the registered ids, each once (a Map key)
    MT_FI void consensus_register(uint32_t raw) {
        if (!cons) {
            set_fail(ST_BAD_INPUT);
            return;
        }
        const uint32_t nreg = rfl(cons[0]), capr = rfl(cons[3]);
        bool have = false;
        for (uint32_t b0 = 0; b0 < nreg; b0 += kWave) {
            const uint32_t j = b0 + (uint32_t)lane;
            have |= ballot(j < nreg && cons[kConsHdr + j] == raw) != 0;
        }
        if (have) return;
        if (nreg >= capr) {
            set_fail(ST_BAD_INPUT);
            return;
        }
        if (lane == 0) {
            cons[kConsHdr + nreg] = raw;
            cons[0] = nreg + 1u;
        }
    }

    // Client.updateConsensusProperty (client.ts:980-987) after the ack of the replica's consensus
    // annotate: pendingConsensus.get(op.relativePos1.id) (op.pos1: its raw value id) — when
    // registered, the marker (idToSegment[id]: op.pos2) re-combines the op's keys with the sequenced
    // seq and no collab window (segmentPropertiesManager.ts:35-111); either way a min-seq listener at
    // seq is queued (mergeTree.ts:1701-1707), whose callback an unregistered id lacks.
    MT_FI void consensus_ack(const mt_op &op) {
        if (!cons) {
            set_fail(ST_BAD_INPUT);
            return;
        }
        const uint32_t raw = (uint32_t)op.pos1;
        const uint32_t nreg = rfl(cons[0]), nlis = rfl(cons[1]), capr = rfl(cons[3]), capl = rfl(cons[4]);
        bool reg = false;
        for (uint32_t b0 = 0; raw && b0 < nreg; b0 += kWave) {
            const uint32_t j = b0 + (uint32_t)lane;
            reg |= ballot(j < nreg && cons[kConsHdr + j] == raw) != 0;
        }
        if (reg) {
            const uint32_t key = (uint32_t)op.pos2;
            const int32_t n = idmap_n;
            uint32_t found = 0, slot = kIdUnlinked;
            for (int32_t j0 = 0; j0 < n; j0 += kWave) {
                const int32_t j = j0 + lane;
                const uint2 e = j < n ? idmap[j] : make_uint2(0u, 0u);
                const uint64_t hm = ballot(j < n && e.x == key);
                if (hm) slot = rdl(e.y, first_lane(hm));
                found += __popcll(hm);
            }
            if (key == 0u || key == kIdKeyUnsupported || found != 1u) {
                set_fail(ST_UNSUPPORTED);
                return;
            }
            if (slot != kIdUnlinked) {
                {
                    const uint32_t o0 = rfl(cold[2 * slot].x);
                    const uint32_t n0 = o0 ? rfl(pool[o0]) : 0u;
                    pool_reserve(2u + 2u * ((n0 > 64u ? n0 : 64u) + op.payload_len));
                }
                if (status) return;
                const uint32_t old = rfl(cold[2 * slot].x);
                uint32_t nh;
                const uint32_t nid = props_extend(old, props_in + op.payload, op.payload_len, false, nh,
                                                  kCombineConsensusAck);
                if (status) return;
                if (lane == 0) cold[2 * slot].x = nid;
                if (nid) s_meta[slot] = (Meta)(s_meta[slot] | kFHasProps);
                wsync();
            }
        }
        if (nlis >= capl) {
            set_fail(ST_BAD_INPUT);
            return;
        }
        uint32_t *L = cons + kConsHdr + capr + kConsLis * nlis;
        if (lane < kConsLis) L[lane] = lane == 0 ? raw : lane == 1 ? (uint32_t)op.seq : lane == 2 ? (uint32_t)reg : 0u;
        if (lane == 0) cons[1] = nlis + 1u;
        if (cons_next == INT32_MAX) cons_next = op.seq;
    }

    // notifyMinSeqListeners (mergeTree.ts:1709-1716) for the consensus listeners: those at seq <=
    // minSeq fire in seq order (the host orders equal seqs as the reference's heap does); a
    // listener without a registered id dereferences an undefined consensusInfo (a TypeError)
    MT_FI void consensus_fire() {
        const uint32_t nlis = rfl(cons[1]), capr = rfl(cons[3]);
        uint32_t head = rfl(cons[2]);
        uint32_t *L0 = cons + kConsHdr + capr;
        for (; head < nlis; head++) {
            const uint32_t s = rfl(L0[kConsLis * head + 1]);
            if ((int32_t)s > min_seq) break;
            if (!rfl(L0[kConsLis * head + 2])) {
                set_fail(ST_UNSUPPORTED);
                return;
            }
            if (lane == 0) {
                L0[kConsLis * head + 3] = (uint32_t)min_seq;
                L0[kConsLis * head + 4] = (uint32_t)cur_seq;
            }
        }
        if (lane == 0) cons[2] = head;
        cons_next = head < nlis ? (int32_t)rfl(L0[kConsLis * head + 1]) : INT32_MAX;
    }

    // Client.regeneratePendingOp(resetOp, oldest pending group) -> resetPendingDeltaToOps
    // (client.ts:708-766): the group's segments in document order, each at its
    // findReconnectionPostition (674-706: the length before it of the segments inserted and not
    // removed as of the group's localSeq), get one op and one new group each (queued last, same
    // localSeq); the ops are written to the document's regen region (mt_device.h kRegenOpWords).
    MT_FI void op_regenerate(const mt_op &op) {
        const uint32_t T = (uint32_t)op.ref_seq;
        if (n_pend == 0 || T > MT_OP_ANNOTATE) {
            set_fail(ST_BAD_INPUT);
            return;
        }
        resolve_cold();
        const uint32_t head = pend_word(1), gb = head & kPmb;
        const uint32_t L = rfl(pdesc(head)[3]);
        if ((rfl(pdesc(head)[0]) & 0xFFu) != T) {
            set_fail(ST_BAD_INPUT);
            return;
        }
        // the record header: GROUP_CONT of the reset op member, ops (filled in below)
        uint32_t used = rfl(regen[0]);
        if (used < 2u) used = 2u;
        const uint32_t hdr = used;
        if (used + 2u > (uint32_t)regen_cap) {
            cap_fail(kCapRegen);
            return;
        }
        used += 2u;
        uint32_t nops = 0;
        int32_t blk = root;
        while (!b_leaf[blk]) blk = b_child[blk * 8];
        uint32_t base = 0;
        for (; blk >= 0 && !status; blk = next_leaf_block(blk)) {
            const int32_t n = b_count[blk];
            uint32_t slot = 0, meta = 0, len = 0;
            USr sr = 0;
            uint32_t m = 0;
            bool member = false;
            uint32_t contrib = 0;
            if (lane < n) {
                slot = b_child[blk * 8 + lane];
                meta = s_meta[slot];
                len = s_len[slot];
                // the relative seqs (a settled leaf: 0, and 0 or kRNone for the removal)
                sr = !is_settled(meta) ? u_sr[meta & kUNone] : us_make(0u, (meta & kFRemoved) ? 0u : kRNone);
                // seg.localSeq / localRemovedSeq: the localSeq of its pending insert / remove group
                uint32_t ins_l = 0xFFFFFFFFu, rem_l = 0xFFFFFFFFu;
                if (meta & kFPending) {
                    m = cold[2 * slot + 1].w;
                    member = (m >> gb) & 1u;
                    for (uint32_t mm = m; mm; mm &= mm - 1) {
                        // the live group of bit bi (exact while <= 32 are pending; else recomputed below)
                        const uint32_t bi = (uint32_t)__builtin_ctz(mm);
                        const uint32_t *dp = pdesc(head + ((bi - head) & kPmb));
                        const uint32_t t = dp[0] & 0xFFu, ls = dp[3];
                        if (t == MT_OP_INSERT) ins_l = ls;
                        if (t == MT_OP_REMOVE) rem_l = ls;
                    }
                }
                const bool pins = us_q(sr) == kRUnassigned, prem = us_r(sr) == kRUnassigned;
                const bool inserted = !pins || ins_l <= L;
                const bool not_removed = !(meta & kFRemoved) || (prem && rem_l != 0xFFFFFFFFu && rem_l > L);
                contrib = inserted && not_removed ? len : 0u;
            }
            if (n_pend > kPendMaskBits) {
                // more than 32 groups pending: mask bits are shared by groups 32 apart, so the
                // segment's insert / remove groups and membership come from the entry lists
                uint64_t pm = ballot(lane < n && (meta & kFPending));
                while (pm) {
                    const int f = first_lane(pm);
                    pm &= pm - 1;
                    const uint32_t sl = rdl(slot, f);
                    const uint32_t mf = rdl(m, f);
                    const uint32_t il = group_lseq(sl, mf, MT_OP_INSERT), rl = group_lseq(sl, mf, MT_OP_REMOVE);
                    const bool mem = in_group(head, sl, mf);
                    if (lane == f) {
                        const bool pins = us_q(sr) == kRUnassigned, prem = us_r(sr) == kRUnassigned;
                        const bool inserted = !pins || il <= L;
                        const bool not_removed = !(meta & kFRemoved) || (prem && rl != 0xFFFFFFFFu && rl > L);
                        contrib = inserted && not_removed ? len : 0u;
                        member = mem;
                    }
                }
            }
            const uint32_t incl = scan8(contrib) + base;
            const uint32_t excl = incl - contrib;
            base = rdl(incl, kMaxNodes - 1);
            uint64_t mb = ballot(lane < n && member);
            while (mb && !status) {
                const int f = first_lane(mb);
                mb &= mb - 1;
                const uint32_t sl = rdl(slot, f), pos = rdl(excl, f), ln = rdl(len, f);
                const uint32_t sq_f = rdl(us_q(sr), f), sr_f = rdl(us_r(sr), f);
                const uint32_t mt_f = rdl(meta, f);
                const uint32_t mask = rdl(m, f);
                bool made = true;
                uint32_t w[kRegenOpWords] = {T, pos, pos + ln, 0u, 0u, 0u, 0u, 0u};
                uint32_t props = 0, np = 0;
                if (T == MT_OP_INSERT) {
                    if (sq_f != kRUnassigned) {  // assert(segment.seq === UnassignedSequenceNumber)
                        set_fail(ST_BAD_INPUT);
                        return;
                    }
                    const uint4 cr = cold[2 * sl];
                    w[3] = (mt_f & kFMarker) ? (1u | (rfl(cr.z) << 1)) : 0u;
                    w[4] = (mt_f & kFMarker) ? 0u : rfl(cr.z);
                    w[5] = ln;
                    props = (mt_f & kFHasProps) ? rfl(cr.x) : 0u;
                    np = props ? pool[props] : 0xFFFFFFFFu;
                    w[6] = np;
                } else if (T == MT_OP_REMOVE) {
                    made = sr_f == kRUnassigned;  // only while the local remove is pending
                } else {
                    w[3] = op.flags;
                    w[4] = op.payload;
                    w[5] = op.payload_len;
                }
                uint32_t nm = bit_free_after(head, sl, head, head) ? mask & ~(1u << gb) : mask;
                if (made) {
                    const uint32_t words = kRegenOpWords + (np != 0xFFFFFFFFu ? 2u * np : 0u);
                    if (used + words > (uint32_t)regen_cap) {
                        cap_fail(kCapRegen);
                        return;
                    }
                    if (lane < kRegenOpWords) {
                        uint32_t v = 0;
#pragma unroll
                        for (int i = 0; i < kRegenOpWords; i++)
                            if (lane == i) v = w[i];
                        regen[used + lane] = v;
                    }
                    for (uint32_t i = lane; props && i < 2u * np; i += kWave) regen[used + kRegenOpWords + i] = pool[props + 2 + i];
                    used += words;
                    nops++;
                    // the new group of this segment alone (same localSeq), queued last
                    if (n_pend >= (int32_t)pend_groups(pend_cap_e)) {
                        set_fail(ST_UNSUPPORTED);
                        return;
                    }
                    const uint32_t ng = head + (uint32_t)n_pend;
                    if (lane == 0) {
                        *(uint4 *)pdesc(ng) = make_uint4(T | ((uint32_t)op.flags << 16), op.payload, op.payload_len, L);
                        pend[0] = (uint32_t)(n_pend + 1);
                    }
                    n_pend++;
                    entry_append(ng, sl);
                    if (status) return;
                    nm |= 1u << (ng & kPmb);
                }
                pend_set_mask(sl, nm);
            }
        }
        if (status) return;
        if (lane == 0) {
            regen[hdr] = op.flags & MT_OPF_GROUP_CONT;
            regen[hdr + 1] = nops;
            regen[0] = used;
            regen[1] = regen[1] + 1u;
            pend[0] = (uint32_t)(n_pend - 1);  // the reset group leaves the queue
            pend[1] = head + 1u;
        }
        n_pend--;
    }

    MT_FI void apply(mt_op op) {
        pend_n = 0;
        if (rel_pend) {  // the positions the MT_OP_RELPOS record before this one resolved
            const int32_t rp = rel_pend;
            if (rp & 1) op.pos1 = rel_p1;
            if (rp & 2) op.pos2 = rel_p2;
            rel_pend = 0;
        }
        if constexpr (kW) {
            if (op.seq == kUnassignedSeq) {  // a local op of this replica (mt_oplog.h)
                op_local(op);
                resolve_splits();
                return;
            }
        }
        if (MT_OP_CLIENT(op) >= (uint32_t)kMaxClients || (!kW && MT_OP_CLIENT(op) == 0 && op.type != MT_OP_NOOP)) {
            set_fail(ST_UNSUPPORTED);
            return;
        }
        // the LDS classes' 16-bit relative seqs need seq - sbase < kSeq16Span: rebase on minSeq; a
        // collab window wider than that re-runs the document in a spill class (32-bit relative seqs)
        if constexpr (!kHbm) {
            if (op.seq - sbase >= kSeq16Span / 2 && min_seq > sbase) settle_all();
            if (op.seq - sbase >= kSeq16Span) {
                cap_fail(kCapLongSeg);
                return;
            }
        }
        if constexpr (kW) {
            if (MT_OP_CLIENT(op) == 0 && op.type != MT_OP_NOOP) {
                // the replica's own sequenced message acks its oldest pending group (client.ts:
                // 810-812; a GROUP acks one group per member); positions are not read
                if (op.type != MT_OP_RELPOS) op_ack(op);
                // updateConsensusProperty after the ack (client.ts:596-600)
                if (op.type == MT_OP_ANNOTATE && MT_OPF_COMBINE(op.flags) == MT_COMBINE_CONSENSUS && !status)
                    consensus_ack(op);
                resolve_splits();
                if (status) return;
                if (!(op.flags & MT_OPF_GROUP_CONT)) update_seq_numbers(op.msn, op.seq);
                return;
            }
        }
        switch (op.type) {
            case MT_OP_INSERT: op_insert(op); break;
            case MT_OP_REMOVE:
            case MT_OP_ANNOTATE: op_range(op); break;
            case MT_OP_RELPOS: op_relpos(op); break;
            case MT_OP_NOOP: break;
            default: set_fail(ST_BAD_INPUT); return;
        }
        resolve_splits();  // on early exits (capacity) keep the table consistent
        if (status) return;
        if (op.type != MT_OP_NOOP) {
            // completeAndLogOp (client.ts:461-464)
            if (!(cur_seq < op.seq)) {
                set_fail(ST_SEQ_ORDER);
                return;
            }
            if (!(min_seq <= op.msn)) {
                set_fail(ST_MSN_ORDER);
                return;
            }
        }
        if (!(op.flags & MT_OPF_GROUP_CONT)) update_seq_numbers(op.msn, op.seq);
    }

    // MergeTree.getLength(refSeq, clientId) (generator)
    MT_FI uint32_t view_length(int32_t ref, uint32_t c) {
        uint32_t sum = 0;
        if (ref >= min_seq) {
            sum = blk_settled((uint32_t)root, depth == 1);
            for (int32_t base = 0; base < nu; base += kWave) {
                const int32_t j = base + lane;
                uint32_t vlen = 0;
                if (j < nu) vlen = view_entry((uint32_t)j, u_list[j], ref, c);
                sum += rdl(scan_incl(vlen), 63);
            }
        } else {
            for (int32_t base = 0; base < slot_top; base += kWave) {
                const int32_t slot = base + lane;
                uint32_t vlen = 0;
                if (slot < slot_top && (s_meta[slot] & kFLinked)) {
                    bool tie;
                    view_of((uint32_t)slot, ref, c, vlen, tie);
                }
                sum += rdl(scan_incl(vlen), 63);
            }
        }
        return sum;
    }

    // ------------------------------------------------------------------ checkpoint / resume
    // LDS headroom for one more op (two splits + an insert, a split cascade per leaf insert,
    // a range op's heap / overlay pushes, a pack); below it the document is checkpointed and
    // resumed in a larger capacity class instead of failing mid-op.  (The overlay list keeps 16
    // entries, as the heap does: an op pushes one per segment it makes unsettled, and one that
    // pushes more fails with cap_kind 1 and re-runs from scratch in the next class.  24 sent a
    // writer replica of config 2 that peaks at 187 of class 464's 208 entries into a second launch
    // of its own, the step's tail)
    MT_FI bool low_headroom() const {
        const int32_t fs = cap.seg - slot_top + free_n;
        if constexpr (kSplitPools) {
            const int32_t fl = kLB - blk_top + n_bfree, fi = cap.iblk - lds_top + n_lfree;
            return fs < 6 || fl < 16 || fi < 2 * depth + 10 || cap.heap - hn < 16 || cap.ulist - nu < 16;
        }
        const int32_t fb = cap.blk - blk_top + n_bfree;
        return fs < 6 || fb < 2 * depth + 10 || cap.heap - hn < 16 || cap.ulist - nu < 16;
    }
    template <typename A>
    MT_FI void dump(uint32_t *&p, const A &src, int32_t n) {
        for (int32_t i = lane; i < n; i += kWave) p[i] = (uint32_t)src[i];
        p += n;
    }
    template <typename A>
    MT_FI void load(const uint32_t *&p, A dst, int32_t n) {
        for (int32_t i = lane; i < n; i += kWave) dst[i] = p[i];
        p += n;
    }
    // block ids in the image are index-width independent: kNoBlk (0xFFFF in the LDS classes,
    // 0xFFFFFFFF in the HBM class) is stored as 0xFFFFFFFF
    template <typename A>
    MT_FI void dump_blk(uint32_t *&p, const A &src, int32_t n) {
        for (int32_t i = lane; i < n; i += kWave) p[i] = src[i] == (Idx)kNoBlk ? 0xFFFFFFFFu : (uint32_t)src[i];
        p += n;
    }
    template <typename A>
    MT_FI void load_blk(const uint32_t *&p, A dst, int32_t n) {
        for (int32_t i = lane; i < n; i += kWave) dst[i] = p[i] == 0xFFFFFFFFu ? (Idx)kNoBlk : (Idx)p[i];
        p += n;
    }
    // Image block ids are dense and class independent: the first pool's ids [0, blk_top), then (split
    // pools) the interior ids kLB + i as blk_top + i.  Both free lists keep their links (image ids).
    MT_FI uint32_t img_id(uint32_t b) const {
        if (b == kNoBlk) return 0xFFFFFFFFu;
        if constexpr (kSplitPools) return b >= (uint32_t)kLB ? (uint32_t)blk_top + (b - (uint32_t)kLB) : b;
        return b;
    }
    MT_FI uint32_t cls_id(uint32_t x, uint32_t nl) const {  // image id -> this class's id
        if (x == 0xFFFFFFFFu) return kNoBlk;
        if constexpr (kSplitPools) return x < nl ? x : (uint32_t)kLB + (x - nl);
        return x;
    }
    MT_FI void checkpoint(uint32_t *ck, int32_t ops_done) {
        resolve_splits();
        wsync();
        if constexpr (kGiant) {
            // the image has one id space (the HBM class restores it): the LDS free list joins the
            // HBM one; LDS ids never handed out ([lds_top, kGiantLdsBlocks)) stay unreferenced
            if (n_lfree > 0) {
                int32_t t = lfree_head;
                for (int32_t i = 1; i < n_lfree; i++) t = (int32_t)rfl((uint32_t)b_parent[t]);
                b_parent[t] = (Idx)(bfree_head < 0 ? kNoBlk : (uint32_t)bfree_head);
                bfree_head = lfree_head;
                n_bfree += n_lfree;
                lfree_head = -1;
                n_lfree = 0;
                wsync();
            }
        }
        if (lane == 0) {
            ck[0] = 0x4D54434Bu;  // "MTCK"
            ck[1] = (uint32_t)ops_done;
            ck[2] = (uint32_t)slot_top;
            ck[3] = (uint32_t)free_head;
            ck[4] = (uint32_t)free_n;
            ck[5] = (uint32_t)(blk_top + (kSplitPools ? lds_top : 0));  // image blocks
            ck[6] = (uint32_t)n_bfree;
            ck[7] = img_id((uint32_t)root);
            ck[8] = (uint32_t)depth;
            ck[9] = (uint32_t)hn;
            ck[10] = (uint32_t)nu;
            ck[11] = (uint32_t)min_seq;
            ck[12] = (uint32_t)cur_seq;
            ck[13] = (uint32_t)settled_min;
            ck[14] = (uint32_t)htop;
            ck[15] = arena_top;
            ck[16] = pool_top;
            ck[17] = arena_base;
            ck[18] = pool_base;
            ck[19] = (uint32_t)pool_gcs;
            ck[20] = (uint32_t)text_gcs;
            ck[21] = (uint32_t)max_heap;
            ck[22] = (uint32_t)max_u;
            ck[23] = (uint32_t)sbase;
            ck[24] = bfree_head < 0 ? 0xFFFFFFFFu : img_id((uint32_t)bfree_head);
            ck[25] = (uint32_t)(int32_t)idmap_n;
            ck[26] = (uint32_t)(int32_t)rel_pend;
            ck[27] = (uint32_t)(int32_t)rel_p1;
            ck[28] = (uint32_t)(int32_t)rel_p2;
            ck[29] = (uint32_t)blk_top;  // the first pool's image ids
            ck[30] = kSplitPools ? (uint32_t)n_lfree : 0u;
            ck[31] = kSplitPools && lfree_head >= 0 ? img_id((uint32_t)lfree_head) : 0xFFFFFFFFu;
        }
        uint32_t *p = ck + kCkHdr;
        dump(p, s_len, slot_top);
        for (int32_t i = lane; i < slot_top; i += kWave) p[i] = meta_canon(s_meta[i]);
        p += slot_top;
        dump_blk(p, s_blk, slot_top);  // (free slots: the free-list links)
        dump(p, u_list, nu);
        for (int32_t i = lane; i < nu; i += kWave) {  // canonical 32-bit relative seqs
            const USr x = u_sr[i];
            p[2 * i] = canon_rel(us_q(x));
            p[2 * i + 1] = canon_rel(us_r(x));
        }
        p += 2 * nu;
        dump(p, u_cm, nu);
        // blocks in image order: parent, 8 child entries (interior rows as image ids; one word each, so
        // the image is index-width independent), count | leaf | scour, settled length (0: leaf blocks)
        const int32_t nimg = blk_top + (kSplitPools ? lds_top : 0);
        for (int32_t i = lane; i < nimg; i += kWave) {
            const uint32_t b = cls_id((uint32_t)i, (uint32_t)blk_top);
            p[i] = img_id(b_parent[b]);
            const uint32_t cnt = b_count[b], lf = b_leaf[b];
            for (int32_t j = 0; j < 8; j++) {
                const uint32_t x = b_child[b * 8 + j];
                p[nimg + 8 * i + j] = (lf || (uint32_t)j >= cnt) ? x : img_id(x);
            }
            p[9 * nimg + i] = cnt | (lf << 8) | ((uint32_t)(uint8_t)b_scour[b] << 16);
            p[10 * nimg + i] = (kSplitPools && lf) ? 0u : (uint32_t)b_slen[si(b)];
        }
        p += 11 * nimg;
        dump(p, (const uint32_t *)h_ent, 2 * (hn + 1));
    }
    // returns the number of ops the checkpoint had applied
    MT_FI int32_t restore(const uint32_t *ck, const uint4 *cold_src) {
        clear_epochs();
        const int32_t ops_done = (int32_t)rfl(ck[1]);
        slot_top = (int32_t)rfl(ck[2]);
        free_head = (int32_t)rfl(ck[3]);
        free_n = (int32_t)rfl(ck[4]);
        const int32_t nimg = (int32_t)rfl(ck[5]);
        const uint32_t nl = rfl(ck[29]);
        blk_top = kSplitPools ? (int32_t)nl : nimg;
        lds_top = kSplitPools ? nimg - (int32_t)nl : 0;
        n_bfree = (int32_t)rfl(ck[6]);
        root = (int32_t)cls_id(rfl(ck[7]), nl);
        depth = (int32_t)rfl(ck[8]);
        hn = (int32_t)rfl(ck[9]);
        nu = (int32_t)rfl(ck[10]);
        min_seq = (int32_t)rfl(ck[11]);
        cur_seq = (int32_t)rfl(ck[12]);
        settled_min = (int32_t)rfl(ck[13]);
        htop = (int32_t)rfl(ck[14]);
        arena_top = rfl(ck[15]);
        pool_top = rfl(ck[16]);
        arena_base = rfl(ck[17]);
        pool_base = rfl(ck[18]);
        pool_gcs = (int32_t)rfl(ck[19]);
        text_gcs = (int32_t)rfl(ck[20]);
        max_heap = (int32_t)rfl(ck[21]);
        max_u = (int32_t)rfl(ck[22]);
        sbase = (int32_t)rfl(ck[23]);
        bfree_head = rfl(ck[24]) == 0xFFFFFFFFu ? -1 : (int32_t)cls_id(rfl(ck[24]), nl);
        n_lfree = kSplitPools ? (int32_t)rfl(ck[30]) : 0;
        lfree_head = kSplitPools && rfl(ck[31]) != 0xFFFFFFFFu ? (int32_t)cls_id(rfl(ck[31]), nl) : -1;
        idmap_n = (int32_t)rfl(ck[25]);
        rel_pend = (int32_t)rfl(ck[26]);
        rel_p1 = (int32_t)rfl(ck[27]);
        rel_p2 = (int32_t)rfl(ck[28]);
        arena_end = arena_base + semi_t;
        pool_end = pool_base + semi_p;
        const uint32_t *p = ck + kCkHdr;
        load(p, s_len, slot_top);
        for (int32_t i = lane; i < slot_top; i += kWave) s_meta[i] = (Meta)meta_uncanon(p[i]);
        p += slot_top;
        load_blk(p, s_blk, slot_top);
        load(p, u_list, nu);
        for (int32_t i = lane; i < nu; i += kWave) u_sr[i] = us_make(uncanon_rel(p[2 * i]), uncanon_rel(p[2 * i + 1]));
        p += 2 * nu;
        load(p, u_cm, nu);
        if constexpr (kGiant) {
            restore_giant_blocks(p, nimg, rfl(ck[31]), (int32_t)rfl(ck[30]));
            p += 11 * (int64_t)nimg;
        } else {
            for (int32_t i = lane; i < nimg; i += kWave) {
                const uint32_t b = cls_id((uint32_t)i, nl);
                const uint32_t v = p[9 * nimg + i];
                const uint32_t cnt = v & 0xFFu, lf = (v >> 8) & 0xFFu;
                b_parent[b] = (Idx)cls_id(p[i], nl);
                b_count[b] = (uint8_t)cnt;
                b_leaf[b] = (uint8_t)lf;
                b_scour[b] = (int8_t)(uint8_t)(v >> 16);
                for (int32_t j = 0; j < 8; j++) {
                    const uint32_t x = p[nimg + 8 * i + j];
                    b_child[b * 8 + j] = (Idx)((lf || (uint32_t)j >= cnt) ? x : cls_id(x, nl));
                }
                if (!(kSplitPools && lf)) b_slen[si(b)] = p[10 * nimg + i];
            }
            p += 11 * (int64_t)nimg;
            if constexpr (!kSplitPools) {  // one pool: the image's second free list joins the first
                const int32_t n2 = (int32_t)rfl(ck[30]);
                if (n2 > 0) {
                    wsync();
                    const int32_t h2 = (int32_t)cls_id(rfl(ck[31]), nl);
                    if (n_bfree == 0) {
                        bfree_head = h2;
                    } else {
                        int32_t t = bfree_head;
                        for (int32_t k = 1; k < n_bfree; k++) t = (int32_t)rfl((uint32_t)b_parent[t]);
                        b_parent[t] = (Idx)h2;
                    }
                    n_bfree += n2;
                }
            }
        }
        load(p, (uint32_t *)h_ent, 2 * (hn + 1));
        for (int32_t i = lane; i < kColdPerSlot * slot_top; i += kWave) cold[i] = cold_src[i];
        wsync();
        return ops_done;
    }

    // giant class: the checkpoint's blocks (image ids [0, n)) are renumbered as they load — levels
    // >= kGiantLdsLevel to LDS ids (while they last), the others to HBM ids from kGiantLdsBlocks —
    // and the image's free blocks are dropped.  Per image block, the HBM b_ep / b_acc entries of
    // ids kGiantLdsBlocks + i serve as temporaries (level, new id); clear_epochs() resets b_ep.
    MT_FI void restore_giant_blocks(const uint32_t *img, int32_t n, uint32_t free2_head, int32_t n_free2) {
        const uint32_t *ip = img;           // b_parent (0xFFFFFFFF: none; free blocks: the free list)
        const uint32_t *ic = img + n;       // b_child rows
        const uint32_t *ik = img + 9 * n;   // count | leaf << 8 | scour << 16
        const uint32_t *is = img + 10 * n;  // b_slen (settled lengths)
        MT_AS_GLOBAL uint32_t *tlev = b_ep.p + kGiantLdsBlocks;
        MT_AS_GLOBAL uint32_t *tmap = b_acc.p + kGiantLdsBlocks;
        constexpr uint32_t kFree = 0xFFFFFFFFu;
        for (int32_t i = lane; i < n; i += kWave) tlev[i] = 0u;
        wsync();
        {  // the image's free lists (their links are b_parent)
            int32_t t = bfree_head;
            for (int32_t k = 0; k < n_bfree && t >= 0 && t < n; k++) {
                if (lane == 0) tlev[t] = kFree;
                t = (int32_t)rfl(ip[t]);
            }
            t = free2_head == 0xFFFFFFFFu ? -1 : (int32_t)free2_head;
            for (int32_t k = 0; k < n_free2 && t >= 0 && t < n; k++) {
                if (lane == 0) tlev[t] = kFree;
                t = (int32_t)rfl(ip[t]);
            }
        }
        wsync();
        // level = depth - 1 - (distance to the root); ids in image order, LDS ids first come first
        int32_t nl = 0, nh = 0;
        for (int32_t b0 = 0; b0 < n; b0 += kWave) {
            const int32_t i = b0 + lane;
            const bool live = i < n && tlev[i] != kFree;
            int32_t dist = 0;
            uint32_t c = live ? (uint32_t)i : kFree;
            for (int32_t l = 0; l + 1 < depth; l++) {
                const uint32_t q = c != kFree ? ip[c] : kFree;
                if (q != kFree) dist++;
                c = q;
            }
            const int32_t level = depth - 1 - dist;
            const bool cand = live && level >= kGiantLdsLevel;
            const uint64_t below = (1ull << lane) - 1ull;
            const int32_t rl = nl + __popcll(ballot(cand) & below);
            const bool inl = cand && rl < kGiantLdsBlocks;
            const uint64_t hm = ballot(live && !inl);
            const uint32_t nid = inl ? (uint32_t)rl : (uint32_t)(kGiantLdsBlocks + nh + __popcll(hm & below));
            if (live) tmap[i] = nid;
            nl += __popcll(ballot(inl));
            nh += __popcll(hm);
        }
        wsync();
        for (int32_t b0 = 0; b0 < n; b0 += kWave) {
            const int32_t i = b0 + lane;
            if (i < n && tlev[i] != kFree) {
                const uint32_t nb = tmap[i], par = ip[i], k = ik[i];
                b_parent[nb] = par == kFree ? (Idx)kNoBlk : (Idx)tmap[par];
                b_count[nb] = (uint8_t)k;
                b_leaf[nb] = (uint8_t)(k >> 8);
                b_scour[nb] = (int8_t)(uint8_t)(k >> 16);
                b_slen[nb] = is[i];
            }
        }
        // child rows: 8 lanes per block
        for (int32_t e0 = 0; e0 < 8 * n; e0 += kWave) {
            const int32_t e = e0 + lane, i = e >> 3, j = e & 7;
            if (e < 8 * n && tlev[i] != kFree) {
                const uint32_t k = ik[i], c = ic[e];
                const bool leaf = ((k >> 8) & 0xFFu) != 0u;
                b_child[tmap[i] * 8 + j] = (Idx)(!leaf && (uint32_t)j < (k & 0xFFu) ? tmap[c] : c);
            }
        }
        for (int32_t b0 = 0; b0 < slot_top; b0 += kWave) {
            const int32_t sl = b0 + lane;
            if (sl < slot_top && (s_meta[sl] & kFLinked)) s_blk[sl] = (Idx)tmap[(uint32_t)s_blk[sl]];
        }
        wsync();
        root = (int32_t)rfl(tmap[root]);
        lds_top = nl;
        blk_top = kGiantLdsBlocks + nh;
        bfree_head = -1;
        n_bfree = 0;
        lfree_head = -1;
        n_lfree = 0;
        clear_epochs();
    }

    // ------------------------------------------------------------------ output
    // the leaves in document order, each leaf block closed by an end-marker record
    MT_FI void write_out(OutRec *out, int32_t out_cap, DocOut *dout, int32_t ops_done, int32_t fail_op,
                         uint32_t *lab_out = nullptr) {
        resolve_splits();
        wsync();
        int32_t w = 0;
        int32_t blk = root;
        // a document that ran out of LDS capacity is re-run or resumed: no records
        if (status == ST_CAPACITY && (cap_kind == 1 || cap_kind == kCapCheckpoint || cap_kind == kCapLongSeg)) blk = -1;
        else
            while (!b_leaf[blk]) blk = b_child[blk * 8];
        while (blk >= 0) {
            const int32_t n = b_count[blk];
            const int32_t j = w + lane;
            // the end record of a leaf block carries the interior blocks that end with it, so the
            // host can rebuild the whole tree (getStackContext's block deltas)
            int32_t closes = 0;
            const int32_t nxt = next_leaf_block(blk, &closes);
            if (lane <= n && j < out_cap) {
                OutRec r;
                if (lane < n) {
                    const uint32_t slot = b_child[blk * 8 + lane];
                    const uint32_t cs = slot < (uint32_t)SEG ? slot : 0u;
                    const uint4 cr = cold[2 * cs], sq = cold[2 * cs + 1];
                    r.len = s_len[slot];
                    r.seq = (int32_t)sq.x;
                    r.rseq = (int32_t)sq.y;
                    r.meta = meta_out(s_meta[slot], sq.z, cr.y);
                    r.ovl = cr.y;
                    r.props = cr.x;
                    r.toff = cr.z;
                    r.blk = (uint32_t)blk;
                    if (lab_out) lab_out[j] = (s_meta[slot] & kFMarker) ? cr.w : 0u;
                } else {
                    r.len = 0;
                    r.seq = 0;
                    r.rseq = kNoneSeq;
                    r.meta = 0;
                    r.ovl = 0;
                    r.props = 0;
                    r.toff = (uint32_t)closes;
                    r.blk = (uint32_t)blk | kOutBlockEnd;
                }
                out[j] = r;
            }
            w += n + 1;
            blk = nxt;
        }
        if (lane == 0) {
            DocOut o;
            o.status = (w > out_cap && status == ST_OK) ? ST_CAPACITY : status;
            o.cap_kind = (w > out_cap && status == ST_OK) ? 4 : cap_kind;
            o.min_seq = min_seq;
            o.cur_seq = cur_seq;
            o.depth = depth;
            o.n_out = w <= out_cap ? w : out_cap;
            o.text_top = arena_top;
            o.pool_top = pool_top;
            o.ops_done = ops_done;
            o.max_oe = max_u;
            o.max_slots = slot_top;
            o.max_blocks = kGiant ? blk_top - kGiantLdsBlocks + lds_top : blk_top;
            o.max_heap = max_heap;
            o.fail_op = fail_op;
            o.gen_text = 0;
            o.gen_props = 0;
            *dout = o;
        }
    }
};

// ---------------------------------------------------------------------- kernels
__device__ __forceinline__ mt_op load_op_lane(const mt_op *ops, int64_t i, int64_t end) {
    mt_op o;
    if (i < end) {
        const uint4 *p = (const uint4 *)(ops + i);
        uint4 a = p[0], b = p[1];
        __builtin_memcpy(&o, &a, 16);
        __builtin_memcpy((char *)&o + 16, &b, 16);
    } else {
        __builtin_memset(&o, 0, sizeof o);
    }
    return o;
}

__device__ __forceinline__ mt_op bcast_op(const mt_op &o, int l) {
    uint32_t w[8];
    __builtin_memcpy(w, &o, 32);
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = rdl(w[i], l);
    mt_op r;
    __builtin_memcpy(&r, w, 32);
    return r;
}

template <int SEG, bool kW, bool kBigK>
MT_FI void engine_setup(Engine<SEG, kW, kBigK> &E, const ReplayParams &P, int64_t w, int64_t d, uint8_t *smem) {
    E.lane = threadIdx.x;
    if constexpr (is_giant_seg(SEG)) {
        extern __shared__ __attribute__((aligned(16))) uint8_t gsmem[];
        E.carve(smem, gsmem);
    } else {
        E.carve(smem, nullptr);
    }
    E.cold = P.cold + w * (int64_t)SEG * kColdPerSlot;
    E.text = P.text + P.doc_text_base[d];
    E.text_cap = P.doc_text_cap[d];
    E.pay_end = (P.doc_text_len[d] + 15u) & ~15u;
    E.semi_t = E.text_cap > E.pay_end ? ((E.text_cap - E.pay_end) / 2u) & ~15u : 0u;
    E.arena_base = E.pay_end;
    E.arena_end = E.pay_end + E.semi_t;
    E.arena_top = E.pay_end;
    E.pool = P.pool + P.doc_pool_base[d];
    E.pool_cap = P.doc_pool_cap[d];
    E.semi_p = E.pool_cap > 1u ? (E.pool_cap - 1u) / 2u : 0u;
    E.pool_base = 1;  // id 0 = undefined
    E.pool_end = 1 + E.semi_p;
    E.pool_top = 1;
    E.pool_gcs = 0;
    E.text_gcs = 0;
    E.props_in = (const mt_prop *)P.props_in;
    E.vt = P.vt;
    E.idmap = P.idmap ? P.idmap + P.doc_idmap_base[d] : nullptr;
    E.lab = P.lab_out != nullptr;
    if constexpr (kW) {
        E.pend = P.pend + P.doc_pend_base[d];
        E.pend_cap_e = P.pend_cap;
        E.regen = P.regen + P.doc_regen_base[d];
        E.regen_cap = P.regen_cap;
        E.n_pend = 0;
        E.cur_g = -1;
        E.cons = P.cons ? P.cons + P.doc_cons_base[d] : nullptr;
        E.cons_next = INT32_MAX;
        E.ntf = 0;
        E.ntf_raw = 0;
    }
    E.init();
}

// Base of the document's tables: the workgroup's LDS, or for the HBM class its image in
// global memory (same layout, same engine code; every table access becomes a global one).
template <int SEG>
MT_FI uint8_t *tables(const ReplayParams &P, int64_t w) {
    if constexpr (is_hbm_seg(SEG)) {  // the HBM and giant classes
        return P.hbm_state + w * (int64_t)make_layout(SEG).bytes;
    } else {
        extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
        return smem;
    }
}

// kLoad: apply only the document's leading SnapshotLoader records, then checkpoint at the
// first other record (cap_kind kCapCheckpoint); the replay launch resumes there.
// Workgroup index w writes its results at w; document d; src >= 0: resume from the checkpoint
// ck_in[src] (kSrcList: src = ck_src[w]).  Returns true if the document stopped at a checkpoint.
constexpr int32_t kSrcList = -2;
template <int SEG, bool kLoad, bool kW = false, bool kBigK = false>
MT_FI bool replay_one(const ReplayParams &P, int64_t w, int64_t d, int32_t src) {
    uint8_t *smem = tables<SEG>(P, w);
    Engine<SEG, kW, kBigK || kLoad> E;
#ifdef MT_PROF
    for (int k = 0; k < kProfSlots; k++) E.pf[k] = 0;
    const uint64_t t_kernel = clock64();
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();  // 100 MHz: the launch's drain profile
#endif
    engine_setup(E, P, w, d, smem);
    const mt_op *ops = (const mt_op *)P.ops;
    const int64_t b0 = P.doc_op_off[d], b1 = P.doc_op_off[d + 1];
    int32_t done = 0, fail_op = -1;
    if (P.ck_in) {
        if (src == kSrcList) src = P.ck_src[w];
        if (src >= 0) {
            const uint32_t *ck = P.ck_in + src * P.ck_in_words;
            const uint4 *cold_src = P.cold_in + (int64_t)src * P.cold_in_seg * kColdPerSlot;
            if constexpr (is_giant_seg(SEG)) {
                // an image whose overlay list or heap exceed the giant class's LDS capacities passes
                // through unchanged (image and cold records) to the HBM class
                const int32_t hn = (int32_t)rfl(ck[9]), nu = (int32_t)rfl(ck[10]);
                if (P.ck_out && (nu + 24 > E.cap.ulist || hn + 16 > E.cap.heap)) {
                    const int32_t st = (int32_t)rfl(ck[2]), bt = (int32_t)rfl(ck[5]);
                    const int64_t words = ck_used_words(st, nu, bt, hn);
                    uint32_t *out = P.ck_out + w * ck_words(SEG);
                    for (int64_t i = E.lane; i < words; i += kWave) out[i] = ck[i];
                    for (int64_t i = E.lane; i < (int64_t)kColdPerSlot * st; i += kWave) E.cold[i] = cold_src[i];
                    if (E.lane == 0) {
                        DocOut o{};
                        o.status = ST_CAPACITY;
                        o.cap_kind = kCapCheckpoint;
                        o.ops_done = (int32_t)ck[1];
                        o.fail_op = (int32_t)ck[1];
                        o.max_slots = st;
                        P.doc_out[w] = o;
                    }
                    return true;
                }
            }
            done = E.restore(ck, cold_src);
        }
    }
    // writer batches: the pending-group region persists across launches.  A fresh start (first run,
    // a re-run from scratch, or the SnapshotLoader's run before the replay) clears it; a resumed
    // writer document reads its group count back.
    const bool resumed = P.ck_in && src >= 0;
    if (P.pend && !resumed && E.lane == 0) {
        uint32_t *pr = P.pend + P.doc_pend_base[d];
        pr[0] = 0u;
        pr[1] = 0u;
        pr[2] = 0u;
        pr[3] = 0u;
        pr[4] = 0u;
        uint32_t *rg = P.regen + P.doc_regen_base[d];
        rg[0] = 2u;
        rg[1] = 0u;
        if (P.cons) {
            uint32_t *cs = P.cons + P.doc_cons_base[d];
            cs[0] = 0u;
            cs[1] = 0u;
            cs[2] = 0u;
        }
    }
    if constexpr (kW) {
        E.n_pend = resumed ? (int32_t)E.pend_word(0) : 0;
        if (resumed && E.cons) {  // the oldest unfired listener of a resumed document
            const uint32_t nl = rfl(E.cons[1]), hd = rfl(E.cons[2]);
            E.cons_next = hd < nl ? (int32_t)rfl(E.cons[kConsHdr + rfl(E.cons[3]) + kConsLis * hd + 1]) : INT32_MAX;
        }
    }
    // ops stream through registers 64 at a time (coalesced 2 KiB loads), broadcast by readlane
    mt_op cur = load_op_lane(ops, b0 + done + E.lane, b1);
    for (int64_t base = b0 + done; base < b1 && E.status == ST_OK; base += kWave) {
        mt_op nxt = load_op_lane(ops, base + kWave + E.lane, b1);
        int64_t n = b1 - base < kWave ? b1 - base : kWave;
        for (int i = 0; i < n; i++) {
            if constexpr (kLoad) {  // the loader stops at the first record that is not a LOAD one
                const uint32_t t = rdl((uint32_t)cur.type, i);
                if (P.ck_out && (E.low_headroom() || !(t == MT_OP_LOAD_HEADER || t == MT_OP_LOAD_BODY || t == MT_OP_COLLAB))) {
                    E.checkpoint(P.ck_out + w * ck_words(SEG), done);
                    E.status = ST_CAPACITY;
                    E.cap_kind = kCapCheckpoint;
                    fail_op = (int32_t)(base - b0 + i);
                    break;
                }
                E.apply_load(bcast_op(cur, i));
            } else {
                if (P.ck_out && E.low_headroom()) {
                    E.checkpoint(P.ck_out + w * ck_words(SEG), done);
                    E.status = ST_CAPACITY;
                    E.cap_kind = kCapCheckpoint;
                    fail_op = (int32_t)(base - b0 + i);
                    break;
                }
                mt_op op = bcast_op(cur, i);
                if constexpr (is_giant_seg(SEG) && !kW) {
                    // the prefetch wave's inputs (giant_prefetch): this op's index, the tree's root / depth
                    if (!kLoad && E.lane == 0) {
                        uint32_t *pub = (uint32_t *)((uint8_t *)E.scratch - make_glayout().scratch + make_glayout().pub);
                        __hip_atomic_store(pub + 1, (uint32_t)E.root, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(pub + 2, (uint32_t)E.depth, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(pub, (uint32_t)(base - b0 + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(pub + 7, giant_run(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                E.apply(op);
            }
            if (E.status != ST_OK) {
                fail_op = (int32_t)(base - b0 + i);
                break;
            }
            done++;
        }
        cur = nxt;
    }
    E.write_out(P.out + w * (int64_t)P.out_cap, P.out_cap, P.doc_out + w, done, fail_op,
                P.lab_out ? P.lab_out + w * (int64_t)P.out_cap : nullptr);
#ifdef MT_PROF
    E.pf[0] = clock64() - t_kernel;
    E.pf[kProfSlots - 1] = (rt_start << 32) | (__builtin_amdgcn_s_memrealtime() & 0xFFFFFFFFu);
    if (P.prof && E.lane < kProfSlots) {
        uint64_t v = E.pf[0];
        for (int k = 1; k < kProfSlots; k++)
            if (E.lane == k) v = E.pf[k];
        P.prof[w * kProfSlots + E.lane] = v;
    }
#endif
    return E.status == ST_CAPACITY && E.cap_kind == kCapCheckpoint;
}

// The giant class's prefetch wave (the replay workgroup's second wave; it only reads).  A giant
// document's lower tree levels, segment tables and cold records are in HBM, and every op walks
// them with dependent loads (~30 per op).  While the replaying wave applies op k, this wave walks
// the tree as it stands (racy reads: every id is bounds-checked and a wrong turn only wastes a
// prefetch) towards op k + 1's positions, and to the leaf block of the zamboni heap's top segment,
// loading what those walks read — block rows, lengths, the leaves' lengths / meta words and cold
// records — so the replaying wave's dependent loads find the lines in the CU's L1 / the XCD's L2.
// It stops when the replaying wave publishes giant_done(w), or after 10 s without a new op index
// (a state word left in LDS by an earlier workgroup names another w and is ignored).
template <int SEG>
MT_FI void giant_prefetch(const ReplayParams &P, int64_t w, int64_t d) {
    if constexpr (is_giant_seg(SEG)) {
        extern __shared__ __attribute__((aligned(16))) uint8_t gsmem[];
        Engine<SEG> E;
        E.lane = (int)threadIdx.x - kWave;
        E.carve(tables<SEG>(P, w), gsmem);
        E.cold = P.cold + w * (int64_t)SEG * kColdPerSlot;
        const int lane = E.lane;
        uint32_t *pub = (uint32_t *)(gsmem + make_glayout().pub);
        const mt_op *ops = (const mt_op *)P.ops + P.doc_op_off[d];
        const int64_t n_ops = P.doc_op_off[d + 1] - P.doc_op_off[d];
        constexpr uint32_t kBlk = (uint32_t)E.cap.blk, kSeg = (uint32_t)SEG;
        uint32_t sink = 0;
        int32_t last = -1;
        uint64_t t_prog = __builtin_amdgcn_s_memrealtime();
        // touch the leaves of leaf block b: lengths, meta words, cold records
        auto leaves = [&](uint32_t b, bool cold) {
            if (b >= kBlk) return;
            const uint32_t n = E.b_count[b];
            const uint32_t s = lane < 8 && (uint32_t)lane < n ? (uint32_t)E.b_child[b * 8 + lane] : kSeg;
            if (s < kSeg) {
                sink += (uint32_t)E.s_len[s] + (uint32_t)E.s_meta[s];
                if (cold) sink += E.cold[2 * s].x;
            }
        };
        // the inserting walk's path towards pos (settled lengths only), then the leaf block's leaves
        auto walk = [&](uint32_t root, int32_t depth, uint32_t pos) {
            uint32_t N = root, base = 0;
            for (int32_t l = 0; l + 2 < depth; l++) {
                if (N >= kBlk) return;
                const uint32_t n = E.b_count[N];
                const uint32_t c = lane < 8 && (uint32_t)lane < n ? (uint32_t)E.b_child[N * 8 + lane] : kBlk;
                const uint32_t v = c < kBlk ? (uint32_t)E.b_slen[c] : 0u;
                const uint32_t incl = scan8(v) + base;
                const uint64_t hb = ballot(lane < 8 && c < kBlk && incl >= pos);
                const int f = hb ? first_lane(hb) : (n > 0 && n <= 8 ? (int)n - 1 : 0);
                base = rdl(incl - v, f);
                N = rdl(c, f);
            }
            if (N >= kBlk) return;
            if (depth < 2) {
                leaves(N, true);
                return;
            }
            // the level-1 block: every leaf block's row and leaves (lane = 8 x leaf block + entry)
            const uint32_t n = E.b_count[N];
            const uint32_t ci = (uint32_t)lane >> 3, j = (uint32_t)lane & 7;
            const uint32_t cb = ci < n && ci < 8 ? (uint32_t)E.b_child[N * 8 + ci] : kBlk;
            const uint32_t cn = cb < kBlk ? (uint32_t)E.b_count[cb] : 0u;
            const uint32_t s = j < cn && j < 8 ? (uint32_t)E.b_child[cb * 8 + j] : kSeg;
            uint32_t len = 0;
            if (s < kSeg) {
                len = E.s_len[s];
                sink += (uint32_t)E.s_meta[s];
            }
            const uint32_t gs = sum8(len);
            const uint32_t cl = (uint32_t)__shfl((int)gs, 8 * lane, kWave);
            const uint32_t incl = scan8(cl) + base;
            const uint64_t hb = ballot(lane < 8 && (uint32_t)lane < n && incl >= pos);
            if (hb) leaves(rdl(cb, 8 * first_lane(hb)), true);
        };
        for (;;) {
            const uint32_t st = __hip_atomic_load(pub + 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (st == giant_done(w)) break;
            const int32_t k = (int32_t)__hip_atomic_load(pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            if (st != giant_run(w) || k == last) {
                if (now - t_prog > 1000000000ull) break;  // 10 s (100 MHz) without a new op
                __builtin_amdgcn_s_sleep(2);
                continue;
            }
            last = k;
            t_prog = now;
            const uint32_t root = rfl(__hip_atomic_load(pub + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            const int32_t depth = (int32_t)rfl(__hip_atomic_load(pub + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (root >= kBlk || depth < 1 || depth > 16) continue;
            if (k >= 0 && k + 1 < n_ops) {
                const mt_op op = ops[k + 1];
                if (op.type <= MT_OP_ANNOTATE && op.pos1 >= 0) {
                    walk(root, depth, (uint32_t)op.pos1);
                    if (op.type != MT_OP_INSERT && op.pos2 > op.pos1) walk(root, depth, (uint32_t)op.pos2);
                }
            }
            // the block zamboni pops next: the heap top's leaf block
            const uint32_t key = rfl(E.h_ent[1].x);
            if (key < kSeg) leaves((uint32_t)E.s_blk[key], true);
        }
        if (lane == 0) pub[6] = sink;  // (keeps the loads; the prefetch wave's own word)
    }
}

// Early escalation (ReplayParams.notice, mt_host.cpp mt_batch_sync): a document that ends with
// MT_CAPACITY tells the host at once.  The agent-scope release makes everything the wave wrote — the
// checkpoint image, cold records, text arena, prop pool, per-document regions — visible past this
// XCD's L2 before the ring entry (system scope, host memory) is; the next class's launch, which
// the host starts after reading the entry, acquires at its dispatch.
MT_FI void escalation_notice(const ReplayParams &P, int64_t w) {
    wsync();  // the DocOut row this wave just stored
    if (threadIdx.x != 0) return;
    const DocOut o = P.doc_out[w];
    if (o.status != ST_CAPACITY) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t slot = __hip_atomic_fetch_add(P.notice_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t *e = P.notice + 4ull * slot;
    __hip_atomic_store(e + 1, (uint32_t)P.launch_id | ((uint32_t)o.cap_kind << 24), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(e + 2, (uint32_t)o.ops_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(e + 3, (uint32_t)o.max_oe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(e, (uint32_t)w + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one workgroup per document (blockIdx.x); the giant class's observer replay adds the prefetch wave
template <int SEG, bool kLoad, bool kW = false, bool kBigK = false>
MT_FI void replay_body(const ReplayParams &P) {
    const int64_t w = (int64_t)blockIdx.x;
    if (w >= P.n_docs) return;
    const int64_t d = P.doc_list ? (int64_t)P.doc_list[w] : w;
    if constexpr (kW && !notice_class(SEG))  // (an early escalation runs in a later class)
        if (P.urgent) __builtin_amdgcn_s_setprio(3);
    if constexpr (is_giant_seg(SEG) && !kLoad && !kW && !kBigK) {
        extern __shared__ __attribute__((aligned(16))) uint8_t gsmem[];
        uint32_t *pub = (uint32_t *)(gsmem + make_glayout().pub);
        if (threadIdx.x >= (unsigned)kWave) {
            giant_prefetch<SEG>(P, w, d);
            return;
        }
        replay_one<SEG, kLoad, kW, kBigK>(P, w, d, kSrcList);
        if (threadIdx.x == 0) __hip_atomic_store(pub + 7, giant_done(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
        replay_one<SEG, kLoad, kW, kBigK>(P, w, d, kSrcList);
    }
    // (first launches only: the classes replay starts documents in; the larger classes keep their codegen)
    if constexpr (!kLoad && notice_class(SEG))
        if (P.notice) escalation_notice(P, w);
}

// Generator: draws each op from the issuer's view (include/mt_gen.h, DESIGN.md
// "Synthetic op logs"), writes the record + payload, then applies it as the observer.
template <int SEG>
MT_FI void generate_body(const ReplayParams &P) {
    const int64_t w = (int64_t)blockIdx.x;
    if (w >= P.n_docs) return;
    const int64_t d = P.doc_list ? (int64_t)P.doc_list[w] : w;  // re-generation of overflowed docs
    uint8_t *smem = tables<SEG>(P, w);
    const mt_gen_params g = *(const mt_gen_params *)P.gen;
    Engine<SEG> E;
#ifdef MT_PROF
    for (int k = 0; k < kProfSlots; k++) E.pf[k] = 0;
#endif
    engine_setup(E, P, w, d, smem);
    const int64_t op_base = P.doc_op_off[d];
    const int32_t n_ops = P.gen_doc_ops ? P.gen_doc_ops[d] : g.n_ops;
    mt_op *ops_out = (mt_op *)P.gen_ops + op_base;
    mt_prop *props_out = (mt_prop *)P.gen_props;
    const int64_t prop_base = 2 * op_base;
    E.props_in = props_out;
    uint64_t x = mt_rng_seed(g.seed, (uint64_t)(P.gen_doc_ids ? P.gen_doc_ids[d] : P.doc_first + d));
    __shared__ int32_t lref[64];  // last refSeq per client (160 B static + 16-aligned dynamic base)
    lref[E.lane] = 0;
    wsync();
    uint32_t pay_top = 0, np = 0;
    int32_t done = 0, fail_op = -1;
    for (int32_t k = 1; k <= n_ops; k++) {
        mt_op op;
        op.seq = k;
        int32_t c = 1 + (int32_t)mt_rng_below(&x, (uint32_t)g.n_clients);
        int32_t lag = (int32_t)mt_rng_below(&x, (uint32_t)g.max_lag + 1u);
        int32_t ref = k - 1 - lag;
        int32_t lr = lref[c];
        if (ref < lr) ref = lr;
        wsync();
        lref[c] = ref;
        wsync();
        int32_t msn = lref[1];
        for (int32_t i = 2; i <= g.n_clients; i++) {
            int32_t v = lref[i];
            if (v < msn) msn = v;
        }
        uint32_t len = rfl(E.view_length(ref, (uint32_t)c));
        uint32_t u = mt_rng_below(&x, 100);
        int type;
        if ((int32_t)len < g.min_len || (int32_t)u < g.pct_insert) type = MT_OP_INSERT;
        else if ((int32_t)u < g.pct_insert + g.pct_remove) type = MT_OP_REMOVE;
        else type = MT_OP_ANNOTATE;
        op.type = (uint16_t)type;
        op.client = (uint16_t)c;
        op.flags = 0;
        op.ref_seq = ref;
        op.msn = msn;
        op.pos1 = op.pos2 = 0;
        op.payload = op.payload_len = 0;
        if (type == MT_OP_INSERT) {
            op.pos1 = (int32_t)mt_rng_below(&x, len + 1u);
            uint32_t n = 1u + mt_rng_below(&x, (uint32_t)g.max_insert);
            if (pay_top + n > P.doc_text_len[d]) {
                E.cap_fail(2);
                fail_op = k - 1;
                break;
            }
            op.payload = pay_top;
            op.payload_len = n;
            uint16_t ch = 0;
            bool has_nl = false;
            for (uint32_t i = 0; i < n; i++) {
                uint32_t r = mt_rng_below(&x, 100);
                if ((int32_t)r < g.pct_newline) {
                    ch = (uint16_t)'\n';
                    has_nl = true;
                } else {
                    uint32_t a = mt_rng_below(&x, 27);  // "abcdefghijklmnopqrstuvwxyz "
                    ch = a < 26u ? (uint16_t)('a' + a) : (uint16_t)' ';
                }
                if (E.lane == 0) E.text[pay_top + i] = ch;
            }
            if (ch == (uint16_t)'\n') op.flags |= MT_OPF_INTERNAL_ENDS_NL;
            if (has_nl) op.flags |= MT_OPF_INTERNAL_HAS_NL;
            pay_top += n;
        } else {
            uint32_t rl = 1;
            while (rl < len && mt_rng_below(&x, 4) != 0) rl++;
            uint32_t start = mt_rng_below(&x, len - rl + 1u);
            op.pos1 = (int32_t)start;
            op.pos2 = (int32_t)(start + rl);
            if (type == MT_OP_ANNOTATE) {
                uint32_t nk = 1u + mt_rng_below(&x, 2);
                uint32_t k0 = mt_rng_below(&x, 4);
                uint32_t k1 = (k0 + 1u + mt_rng_below(&x, 3)) % 4u;
                op.payload = (uint32_t)(prop_base + np);
                op.payload_len = nk;
                for (uint32_t i = 0; i < nk; i++) {
                    uint32_t v;
                    if (mt_rng_below(&x, 10) == 0) v = 0;
                    else if ((i ? k1 : k0) <= 1) v = 1;
                    else if ((i ? k1 : k0) == 2) v = 2 + mt_rng_below(&x, 3);
                    else v = 5 + mt_rng_below(&x, 17);
                    if (E.lane == 0) {
                        props_out[prop_base + np].key = i ? k1 : k0;
                        props_out[prop_base + np].value = v;
                    }
                    np++;
                }
            }
        }
        if (E.lane == 0) ops_out[k - 1] = op;
        wsync();
        E.apply(op);
        if (E.status != ST_OK) {
            fail_op = k - 1;
            break;
        }
        done++;
    }
    E.write_out(P.out + w * (int64_t)P.out_cap, P.out_cap, P.doc_out + w, done, fail_op);
    if (E.lane == 0) {
        P.doc_out[w].gen_text = (int32_t)pay_top;
        P.doc_out[w].gen_props = (int32_t)np;
    }
}

}  // namespace mt
