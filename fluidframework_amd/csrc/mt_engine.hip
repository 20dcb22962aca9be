// mt_engine.hip — MI355X (gfx950) batch replay of sequenced merge-tree ops.
//
// One 64-lane wavefront (= one workgroup) owns one document for the whole op log; the
// document's merge-tree lives in LDS as a flat, wave-scannable structure:
//
//   oe[]        document order of the tree's leaves: each entry is (leaf block id << 16 | slot);
//               every leaf block ends with a marker entry (slot 0xFFFF), so empty leaf blocks
//               (pack can create them, mergeTree.ts:1383-1386) stay addressable.
//   s_*[slot]   segment fields (SoA): length, seq, removedSeq, client ids, overlap mask,
//               prop-set id, text offset/capacity.
//   b_*[block]  B-tree blocks (MaxNodesInBlock = 8): parent, child count, needsScour,
//               interior child lists.  Leaf membership is implicit in oe.
//   h_*         the zamboni heap (collections.ts:213-265), same algorithm, same tie order.
//
// Position resolution replaces PartialSequenceLengths (partialLengths.ts) by a per-op,
// lane-parallel visibility test of every leaf (nodeLength, mergeTree.ts:1659-1699) and a
// wave prefix scan; the B-tree walk of insertingWalk (mergeTree.ts:2345-2474) reduces to
// "first entry that satisfies the leaf tie rule, else the end of the first leaf block whose
// cumulative length reaches pos" (DESIGN.md "Flat insertingWalk").  Block splits, pack and
// zamboni follow mergeTree.ts:1289-1478, 2476-2489 exactly, so leaf-block membership — and
// hence SnapshotV1 bytes — match the reference.
//
// No MFMA: the path is integer scan / compaction work bound by LDS latency and HBM.

#include <hip/hip_runtime.h>

#include "../../include/mt_gen.h"
#include "../../include/mt_oplog.h"
#include "mt_device.h"

namespace mt {

#define MT_FI __device__ __attribute__((always_inline)) inline

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

__device__ __forceinline__ uint32_t hash_pair(uint32_t k, uint32_t v) {
    uint32_t h = k * 0x9E3779B1u ^ (v + 0x7F4A7C15u) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h | 1u;
}

// Phase cycle counters (MT_PROF builds only; tools/prof_phases.py): 0 kernel, 1 scans,
// 2 split, 3 insert, 4 range walk, 5 zamboni, 6 oe shifts, 7 scour
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

struct Loc {
    int32_t idx;    // oe index
    uint32_t excl;  // view position before entry idx
    int32_t found;
    int32_t marker;
};

template <int SEG>
struct Engine {
    static constexpr Caps cap = class_caps(SEG);
    static constexpr Layout lay = make_layout(SEG);
    // ---- LDS state
    uint32_t *oe;
    uint32_t *s_len, *s_meta, *s_ovl, *s_props, *s_toff, *s_tcap, *s_phash;
    int32_t *s_seq, *s_rseq;
    uint16_t *s_free;
    uint16_t *b_parent, *b_free, *b_child;
    uint8_t *b_count, *b_leaf;
    int8_t *b_scour;
    uint32_t *scratch;  // 256 words
    // ---- uniform scalars
    int32_t n_oe, slot_top, n_free, blk_top, n_bfree, root, depth, hn;
    int32_t min_seq, cur_seq, status;
    uint32_t arena_top, pool_top;
    uint32_t pay_end, arena_base, arena_end, semi_t;  // text: payload | semispace A | semispace B
    uint32_t pool_base, pool_end, semi_p;             // prop pool: [0] reserved | A | B
    int32_t pool_gcs, text_gcs;
    // ends-with-'\n' of a split's left half, resolved after the op's LDS work so the text load
    // latency overlaps it (at most two splits per op)
    int32_t pend_n;
    uint32_t pend_slot0, pend_slot1, pend_ch0, pend_ch1;
    int32_t max_oe, max_heap;
    uint32_t hk[kHeapRegs];
    int32_t hs[kHeapRegs];
    int32_t split_mark;  // oe index of the end marker the last leaf split inserted, -1: none
    // ---- global
    uint16_t *text;
    uint32_t text_cap;
    uint32_t *pool;
    uint32_t pool_cap;
    const mt_prop *props_in;
    const uint8_t *value_flags;
    uint32_t n_values;
    int lane;
#ifdef MT_PROF
    uint64_t pf[kProfSlots];
#endif

    // ------------------------------------------------------------------ layout
    MT_FI void carve(uint8_t *base) {
        oe = (uint32_t *)(base + lay.oe);
        s_len = (uint32_t *)(base + lay.len);
        s_seq = (int32_t *)(base + lay.seq);
        s_rseq = (int32_t *)(base + lay.rseq);
        s_meta = (uint32_t *)(base + lay.meta);
        s_ovl = (uint32_t *)(base + lay.ovl);
        s_props = (uint32_t *)(base + lay.props);
        s_toff = (uint32_t *)(base + lay.toff);
        s_tcap = (uint32_t *)(base + lay.tcap);
        s_phash = (uint32_t *)(base + lay.phash);
        s_free = (uint16_t *)(base + lay.sfree);
        b_parent = (uint16_t *)(base + lay.bparent);
        b_free = (uint16_t *)(base + lay.bfree);
        b_child = (uint16_t *)(base + lay.bchild);
        b_count = (uint8_t *)(base + lay.bcount);
        b_leaf = (uint8_t *)(base + lay.bleaf);
        b_scour = (int8_t *)(base + lay.bscour);
        scratch = (uint32_t *)(base + lay.scratch);
    }

    int32_t cap_kind;
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
        n_oe = 0;
        slot_top = 0;
        n_free = 0;
        blk_top = 0;
        n_bfree = 0;
        hn = 0;
        min_seq = 0;
        cur_seq = 0;
        status = ST_OK;
        cap_kind = 0;
        pend_n = 0;
        split_mark = -1;
        max_oe = 0;
        max_heap = 0;
        // initialNode (mergeTree.ts:1125): an empty root leaf block
        root = alloc_block(1);
        depth = 1;
        b_parent[root] = 0xFFFF;  // lane-uniform writes (every lane stores the same value)
        oe_insert(0, (uint32_t)root << 16 | kMarkerSlot);
        // heap entry 0 is the sentinel LRUSegmentComparer.min = { maxSeq: -2 } (never compared)
        for (int i = 0; i < kHeapRegs; i++) {
            hk[i] = 0;
            hs[i] = -2;
        }
        wsync();
    }

    // ------------------------------------------------------------------ allocation
    MT_FI int32_t alloc_slot() {
        int32_t s;
        if (n_free > 0) {
            s = rfl((int32_t)s_free[n_free - 1]);
            n_free--;
        } else {
            if (slot_top >= cap.seg) {
                cap_fail(1);
                return -1;
            }
            s = slot_top++;
            s_meta[s] = 0;  // generation 0
        }
        return s;
    }
    MT_FI void free_slot(int32_t s) {
        uint32_t m = s_meta[s];
        uint32_t gen = (m >> 16) + 1;
        s_meta[s] = (gen << 16);  // unlinked, next generation
        s_free[n_free] = (uint16_t)s;
        n_free++;
    }
    MT_FI int32_t alloc_block(int leaf) {
        int32_t b;
        if (n_bfree > 0) {
            b = rfl((int32_t)b_free[n_bfree - 1]);
            n_bfree--;
        } else {
            if (blk_top >= cap.blk || blk_top >= 0xFFFF) {
                cap_fail(1);
                return 0;
            }
            b = blk_top++;
        }
        b_leaf[b] = (uint8_t)leaf;
        b_count[b] = 0;
        b_scour[b] = kScourUndef;
        b_parent[b] = 0xFFFF;
        return b;
    }
    MT_FI void free_block(int32_t b) {
        b_free[n_bfree] = (uint16_t)b;
        n_bfree++;
    }

    // ------------------------------------------------------------------ oe shifting
    // insert entry e before index p (lane-parallel shift right by one)
    MT_FI void oe_insert(int32_t p, uint32_t e) {
        PF_SCOPE(6);
        if (n_oe + 1 > cap.oe) {
            cap_fail(1);
            return;
        }
        wsync();
        for (int32_t base = ((n_oe - 1 - p) / kWave) * kWave + p; base >= p; base -= kWave) {
            int32_t j = base + lane;
            uint32_t v = 0;
            bool ok = j < n_oe;
            if (ok) v = oe[j];
            wsync();
            if (ok) oe[j + 1] = v;
            wsync();
        }
        if (lane == 0) oe[p] = e;
        n_oe++;
        if (n_oe > max_oe) max_oe = n_oe;
        wsync();
    }
    // move oe[from, n_oe) to start at `to` (to < from: left shift; to > from: right shift)
    MT_FI void oe_move_tail(int32_t from, int32_t to) {
        PF_SCOPE(6);
        int32_t cnt = n_oe - from;
        int32_t new_n = to + cnt;
        if (new_n > cap.oe) {
            cap_fail(1);
            return;
        }
        wsync();
        if (to < from) {
            for (int32_t base = 0; base < cnt; base += kWave) {
                int32_t j = base + lane;
                uint32_t v = 0;
                if (j < cnt) v = oe[from + j];
                wsync();
                if (j < cnt) oe[to + j] = v;
                wsync();
            }
        } else if (to > from) {
            for (int32_t base = ((cnt - 1) / kWave) * kWave; base >= 0; base -= kWave) {
                int32_t j = base + lane;
                uint32_t v = 0;
                if (j < cnt) v = oe[from + j];
                wsync();
                if (j < cnt) oe[to + j] = v;
                wsync();
            }
        }
        n_oe = new_n;
        if (n_oe > max_oe) max_oe = n_oe;
        wsync();
    }

    // ------------------------------------------------------------------ visibility
    // nodeLength of one leaf for (refSeq, clientId) + breakTie's leaf rule (mergeTree.ts:2248-2277)
    __device__ __forceinline__ void view_of(uint32_t e, int32_t ref, uint32_t c, uint32_t &vlen, bool &tie,
                                            bool &mk) const {
        uint32_t slot = e & 0xFFFFu;
        if (slot == kMarkerSlot) {
            vlen = 0;
            tie = false;
            mk = true;
            return;
        }
        mk = false;
        uint32_t meta = s_meta[slot];
        int32_t seq = s_seq[slot];
        int32_t rseq = s_rseq[slot];
        uint32_t ovl = s_ovl[slot];
        uint32_t len = s_len[slot];
        uint32_t cli = meta & 63u, rcli = (meta >> 6) & 63u;
        bool vis = (cli == c) || (seq <= ref);
        bool rem = (rcli == c) || ((ovl >> c) & 1u) || (rseq <= ref);
        vlen = (vis && !rem) ? len : 0u;
        tie = !(rseq <= ref);
    }

    // insertingWalk target for pos under (ref, c): see header comment
    // Scanning may start at any index `from` whose view position `carry` is known and before
    // which no entry satisfies the walk's stop condition.
    MT_FI Loc locate(uint32_t pos, int32_t ref, uint32_t c, int32_t from = 0, uint32_t carry = 0) {
        PF_SCOPE(1);
        Loc L;
        L.found = 0;
        L.idx = -1;
        L.excl = 0;
        L.marker = 0;
        for (int32_t base = from; base < n_oe; base += kWave) {
            int32_t j = base + lane;
            bool valid = j < n_oe;
            uint32_t vlen = 0;
            bool tie = false, mk = false;
            if (valid) view_of(oe[j], ref, c, vlen, tie, mk);
            uint32_t incl = scan_incl(vlen) + carry;
            uint32_t excl = incl - vlen;
            bool cond = valid && !mk && (incl > pos || (excl == pos && vlen == 0 && tie));
            bool mhit = valid && mk && incl >= pos;
            uint64_t b = ballot(cond || mhit);
            if (b) {
                int f = first_lane(b);
                L.found = 1;
                L.idx = base + f;
                L.excl = rdl(excl, f);
                L.marker = (int32_t)((ballot(mhit) >> f) & 1ull);
                return L;
            }
            carry = rdl(incl, 63);
        }
        return L;
    }

    // the visible segment strictly containing pos (excl < pos < excl + vlen) at or after `from`:
    // the one ensureIntervalBoundary splits.  found = 0 when pos is already a boundary.
    MT_FI Loc containing(uint32_t pos, int32_t ref, uint32_t c, int32_t from, uint32_t carry) {
        PF_SCOPE(1);
        Loc L;
        L.found = 0;
        L.idx = -1;
        L.excl = 0;
        L.marker = 0;
        for (int32_t base = from; base < n_oe; base += kWave) {
            int32_t j = base + lane;
            bool valid = j < n_oe;
            uint32_t vlen = 0;
            bool tie = false, mk = false;
            if (valid) view_of(oe[j], ref, c, vlen, tie, mk);
            uint32_t incl = scan_incl(vlen) + carry;
            uint32_t excl = incl - vlen;
            uint64_t b = ballot(valid && incl > pos);
            if (b) {
                int f = first_lane(b);
                uint32_t e = rdl(excl, f);
                if (e < pos) {
                    L.found = 1;
                    L.idx = base + f;
                    L.excl = e;
                }
                return L;
            }
            carry = rdl(incl, 63);
        }
        return L;
    }

    // MergeTree.getLength(refSeq, clientId) (generator)
    MT_FI uint32_t view_length(int32_t ref, uint32_t c) {
        uint32_t carry = 0;
        for (int32_t base = 0; base < n_oe; base += kWave) {
            int32_t j = base + lane;
            uint32_t vlen = 0;
            bool tie, mk;
            if (j < n_oe) view_of(oe[j], ref, c, vlen, tie, mk);
            carry = rdl(scan_incl(vlen) + carry, 63);
        }
        return carry;
    }

    // first oe index with entry predicate; kind 0: slot == key, kind 1: block == key
    MT_FI int32_t find_entry(uint32_t key, int kind, int32_t from = 0) {
        for (int32_t base = from; base < n_oe; base += kWave) {
            int32_t j = base + lane;
            bool hit = false;
            if (j < n_oe) {
                uint32_t e = oe[j];
                hit = kind == 0 ? ((e & 0xFFFFu) == key) : ((e >> 16) == key);
            }
            uint64_t b = ballot(hit);
            if (b) return base + first_lane(b);
        }
        return -1;
    }
    // first index of block `blk`'s range, given an index inside it (ranges are <= 9 entries)
    MT_FI int32_t block_start_near(uint32_t blk, int32_t inside) {
        int32_t j = inside - 8 + lane;
        bool hit = lane < 17 && j >= 0 && j < n_oe && (oe[j] >> 16) == blk;
        uint64_t b = ballot(hit);
        return inside - 8 + first_lane(b);
    }

    // ------------------------------------------------------------------ text helpers
    MT_FI bool text_ends_nl(uint32_t toff, uint32_t len) const {
        return len > 0 && text[toff + len - 1] == (uint16_t)'\n';
    }
    // lane-parallel copy of n code units inside the doc's text region
    MT_FI void text_copy(uint32_t dst, uint32_t src, uint32_t n) {
        for (uint32_t i = lane; i < n; i += kWave) text[dst + i] = text[src + i];
    }
    // Bump allocation in the active text semispace; when it is full, live text moves to the
    // other semispace (text_gc) and the garbage left by reallocating merges is dropped.
    MT_FI uint32_t arena_alloc(uint32_t n) {
        uint32_t n16 = (n + 15u) & ~15u;
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

    // copy every linked segment's arena text into the other semispace (document order)
    MT_FI void text_gc() {
        uint32_t nb = arena_base == pay_end ? pay_end + semi_t : pay_end;
        uint32_t top = nb;
        wsync();
        for (int32_t base = 0; base < n_oe; base += kWave) {
            int32_t j = base + lane;
            uint32_t slot = j < n_oe ? (oe[j] & 0xFFFFu) : kMarkerSlot;
            bool mv = false;
            if (slot != kMarkerSlot) {
                uint32_t t = s_toff[slot];
                mv = !(s_meta[slot] & kMetaMarker) && t >= arena_base && t < arena_end;
            }
            uint64_t m = ballot(mv);
            while (m) {
                int f = first_lane(m);
                m &= m - 1;
                uint32_t sl = rdl(slot, f);
                uint32_t len = s_len[sl];
                uint32_t cap16 = (len + 15u) & ~15u;
                if (cap16 == 0) cap16 = 16;
                if (top + cap16 > nb + semi_t) {
                    cap_fail(2);
                    return;
                }
                text_copy(top, s_toff[sl], len);
                s_toff[sl] = top;
                s_tcap[sl] = cap16;
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

    // make room for `words` in the prop pool (semispace copy of the live sets when full)
    MT_FI void pool_reserve(uint32_t words) {
        if (pool_top + words <= pool_end) return;
        uint32_t nb = pool_base == 1u ? 1u + semi_p : 1u;
        uint32_t top = nb, last_old = 0, last_new = 0;
        wsync();
        for (int32_t base = 0; base < n_oe; base += kWave) {
            int32_t j = base + lane;
            uint32_t slot = j < n_oe ? (oe[j] & 0xFFFFu) : kMarkerSlot;
            bool mv = slot != kMarkerSlot && s_props[slot] != 0u;
            uint64_t m = ballot(mv);
            while (m) {
                int f = first_lane(m);
                m &= m - 1;
                uint32_t sl = rdl(slot, f);
                uint32_t old = s_props[sl];
                if (old != last_old) {
                    uint32_t w = 2u + 2u * pool[old];
                    if (top + w > nb + semi_p) {
                        cap_fail(3);
                        return;
                    }
                    for (uint32_t i = lane; i < w; i += kWave) pool[top + i] = pool[old + i];
                    last_old = old;
                    last_new = top;
                    top += w;
                }
                s_props[sl] = last_new;
            }
            wsync();
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
        bool hit = lane < n && b_child[p * 8 + lane] == (uint16_t)c;
        uint64_t b = ballot(hit);
        return b ? first_lane(b) : -1;
    }

    // updateRoot (mergeTree.ts:1876-1887)
    MT_FI void update_root(int32_t split_node) {
        int32_t nr = alloc_block(0);
        if (status) return;
        b_child[nr * 8 + 0] = (uint16_t)root;
        b_child[nr * 8 + 1] = (uint16_t)split_node;
        b_count[nr] = 2;
        b_parent[root] = (uint16_t)nr;
        b_parent[split_node] = (uint16_t)nr;
        root = nr;
        depth++;
    }

    // insertingWalk's "insert the split-off node after its source" (mergeTree.ts:2446-2453),
    // cascading MergeTree.split (2476-2489) up the interior levels and updateRoot at the top.
    MT_FI void insert_child_after(int32_t p, int32_t after, int32_t nc) {
        for (;;) {
            int32_t i = child_index(p, after);
            int32_t n = b_count[p];
            wsync();
            uint16_t v = 0;
            if (lane > i && lane < n) v = b_child[p * 8 + lane];
            wsync();
            if (lane > i && lane < n) b_child[p * 8 + lane + 1] = v;
            wsync();
            b_child[p * 8 + i + 1] = (uint16_t)nc;
            b_parent[nc] = (uint16_t)p;
            b_count[p] = (uint8_t)(n + 1);
            wsync();
            if (n + 1 < kMaxNodes) return;
            // split the interior block p: children 4..7 move to m
            int32_t m = alloc_block(0);
            if (status) return;
            wsync();
            if (lane < 4) {
                uint16_t c = b_child[p * 8 + 4 + lane];
                b_child[m * 8 + lane] = c;
                b_parent[c] = (uint16_t)m;
            }
            wsync();
            b_count[m] = 4;
            b_count[p] = 4;
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

    // MergeTree.split on a leaf block whose range starts at s and now holds 8 children.
    // Returns the new right block.
    MT_FI int32_t split_leaf(int32_t blk, int32_t s) {
        int32_t nb = alloc_block(1);
        if (status) return blk;
        wsync();
        // children 4..7 and the block's end marker move to the new block
        if (lane >= 4 && lane <= 8) {
            uint32_t e = oe[s + lane];
            oe[s + lane] = ((uint32_t)nb << 16) | (e & 0xFFFFu);
        }
        wsync();
        b_count[nb] = 4;
        b_count[blk] = 4;
        split_mark = s + 4;
        oe_insert(s + 4, ((uint32_t)blk << 16) | kMarkerSlot);
        if (status) return nb;
        if (blk == root) update_root(nb);
        else insert_child_after(b_parent[blk], blk, nb);
        return nb;
    }

    // ------------------------------------------------------------------ split / insert leaves
    // insert a leaf before oe index idx into the leaf block owning oe[idx]; returns the
    // block the new leaf ends up in (after a possible split)
    MT_FI int32_t insert_leaf(int32_t idx, uint32_t slot) {
        uint32_t blk = rfl(oe[idx] >> 16);
        oe_insert(idx, (blk << 16) | slot);
        if (status) return (int32_t)blk;
        int32_t cnt = b_count[blk] + 1;
        b_count[blk] = (uint8_t)cnt;
        wsync();
        if (cnt >= kMaxNodes) {
            int32_t s = block_start_near(blk, idx);
            int32_t nb = split_leaf((int32_t)blk, s);
            if (idx - s >= 4) return nb;
        }
        return (int32_t)blk;
    }

    // BaseSegment.splitAt + TextSegment.createSplitSegmentAt (mergeTree.ts:524-568,
    // textSegment.ts:103-111): the right part becomes a new leaf right after the left one
    // Returns the left half's oe index afterwards (a leaf split may insert an end marker before it).
    MT_FI int32_t split_at(int32_t idx, uint32_t r) {
        PF_SCOPE(2);
        split_mark = -1;
        uint32_t slot = rfl(oe[idx] & 0xFFFFu);
        uint32_t meta = s_meta[slot];
        if (meta & kMetaMarker) return idx;  // Marker.createSplitSegmentAt returns undefined
        int32_t ns = alloc_slot();
        if (ns < 0) return idx;
        uint32_t len = s_len[slot], toff = s_toff[slot], tcap = s_tcap[slot];
        uint32_t last = text[toff + r - 1];  // consumed in resolve_splits()
        if (pend_n == 0) {
            pend_slot0 = slot;
            pend_ch0 = last;
        } else {
            pend_slot1 = slot;
            pend_ch1 = last;
        }
        pend_n++;
        s_len[ns] = len - r;
        s_seq[ns] = s_seq[slot];
        s_rseq[ns] = s_rseq[slot];
        s_ovl[ns] = s_ovl[slot];
        s_props[ns] = s_props[slot];
        s_phash[ns] = s_phash[slot];
        s_toff[ns] = toff + r;
        s_tcap[ns] = tcap - r;
        uint32_t gen = s_meta[ns] & 0xFFFF0000u;
        s_meta[ns] = (meta & 0x0000FFFFu) | gen;  // inherits ends-NL of the original tail
        s_len[slot] = r;
        s_tcap[slot] = r;
        wsync();
        insert_leaf(idx + 1, (uint32_t)ns);
        return shifted(idx);
    }
    // index of a pre-split entry at or before the split point after the last split_at
    MT_FI int32_t shifted(int32_t i) const { return (split_mark >= 0 && split_mark <= i) ? i + 1 : i; }

    MT_FI void resolve_splits() {
        if (pend_n > 0) {
            uint32_t m = s_meta[pend_slot0];
            s_meta[pend_slot0] = pend_ch0 == (uint32_t)'\n' ? (m | kMetaEndsNL) : (m & ~kMetaEndsNL);
        }
        if (pend_n > 1) {
            uint32_t m = s_meta[pend_slot1];
            s_meta[pend_slot1] = pend_ch1 == (uint32_t)'\n' ? (m | kMetaEndsNL) : (m & ~kMetaEndsNL);
        }
        pend_n = 0;
        wsync();
    }


    // addToLRUSet (mergeTree.ts:1273-1283); seq > currentSeq holds for sequenced remote ops
    MT_FI void add_to_lru(int32_t blk, uint32_t slot, int32_t seq) {
        if (b_scour[blk] != kScourTrue && seq > cur_seq) {
            b_scour[blk] = kScourTrue;
            heap_add(slot | (s_meta[slot] & 0xFFFF0000u), seq);
        }
    }

    // ------------------------------------------------------------------ heap (collections.ts:213-265)
    // The LRU heap lives in VGPRs: entry k is lane k & 63 of register k >> 6, so sifting is
    // readlane / writelane arithmetic with no memory round trips.  Same array layout and sift
    // order as Heap.add / Heap.get, hence the same pop order on seq ties.
    MT_FI int32_t hseq(int32_t k) const {
        int32_t v = 0;
#pragma unroll
        for (int i = 0; i < kHeapRegs; i++)
            if ((k >> 6) == i) v = rdl(hs[i], k & 63);
        return v;
    }
    MT_FI uint32_t hkey(int32_t k) const {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < kHeapRegs; i++)
            if ((k >> 6) == i) v = rdl(hk[i], k & 63);
        return v;
    }
    MT_FI void hset(int32_t k, uint32_t key, int32_t seq) {
#pragma unroll
        for (int i = 0; i < kHeapRegs; i++)
            if ((k >> 6) == i && lane == (k & 63)) {
                hk[i] = key;
                hs[i] = seq;
            }
    }
    MT_FI void heap_add(uint32_t key, int32_t seq) {
        PF_SCOPE(9);
        if (hn + 1 > cap.heap || hn + 1 >= 64 * kHeapRegs) {
            cap_fail(hn + 1 >= 64 * kHeapRegs ? 5 : 1);
            return;
        }
        hn++;
        int32_t k = hn;
        // sift up: parents larger than the new entry move down into the hole
        while (k > 1) {
            int32_t ps = hseq(k >> 1);
            if (!(ps - seq > 0)) break;
            hset(k, hkey(k >> 1), ps);
            k >>= 1;
        }
        hset(k, key, seq);
        if (hn > max_heap) max_heap = hn;
    }
    MT_FI void heap_get(uint32_t &key, int32_t &seq) {
        PF_SCOPE(9);
        key = hkey(1);
        seq = hseq(1);
        uint32_t lk = hkey(hn);
        int32_t ls = hseq(hn);
        hn--;
        int32_t k = 1;
        while ((k << 1) <= hn) {
            int32_t j = k << 1;
            int32_t sj = hseq(j);
            if (j < hn) {
                int32_t sj1 = hseq(j + 1);
                if (sj - sj1 > 0) {
                    j++;
                    sj = sj1;
                }
            }
            if (ls - sj <= 0) break;
            hset(k, hkey(j), sj);
            k = j;
        }
        if (hn >= 1) hset(k, lk, ls);
    }

    // ------------------------------------------------------------------ properties
    // prop-set record in the doc pool: [n, hash, (key, value) x n] in insertion order
    MT_FI bool props_match(uint32_t a, uint32_t ha, uint32_t b, uint32_t hb) {
        if (a == b) return true;
        if (a == 0 || b == 0) return false;
        if (ha != hb) return false;
        uint32_t na = pool[a], nb = pool[b];
        if (na != nb) return false;
        bool ok = true;
        if ((uint32_t)lane < na) {
            uint32_t k = pool[a + 2 + 2 * lane], v = pool[a + 3 + 2 * lane];
            bool f = false;
            for (uint32_t i = 0; i < nb; i++)
                if (pool[b + 2 + 2 * i] == k && pool[b + 3 + 2 * i] == v) f = true;
            ok = f;
        }
        return ballot(!ok) == 0;
    }

    // SegmentPropertiesManager.addProperties for a sequenced remote op (or insert-time props):
    // start from `old` (0 = undefined -> new empty map), apply rewrite then the op's pairs in
    // order (null deletes: properties.ts:95-116).  Returns the new set id (hash in hout).
    MT_FI uint32_t props_extend(uint32_t old, const mt_prop *op, uint32_t nop, bool rewrite, uint32_t &hout) {
        uint32_t *keys = scratch;
        uint32_t *vals = scratch + 128;
        uint32_t n = old ? pool[old] : 0u;
        if (n > 64u || nop > 64u) {
            cap_fail(3);
            return 0;
        }
        wsync();
        if ((uint32_t)lane < n) {
            keys[lane] = pool[old + 2 + 2 * lane];
            vals[lane] = pool[old + 3 + 2 * lane];
        }
        uint32_t ok_k = 0, ok_v = 0;
        if ((uint32_t)lane < nop) {
            ok_k = op[lane].key;
            ok_v = op[lane].value;
        }
        wsync();
        if (rewrite) {
            // delete existing keys whose new value is absent or falsy (segmentPropertiesManager.ts:70-80)
            bool keep = false;
            if ((uint32_t)lane < n) {
                uint32_t k = keys[lane];
                for (uint32_t i = 0; i < nop; i++) {
                    uint32_t kk = rdl(ok_k, (int)i), vv = rdl(ok_v, (int)i);
                    if (kk == k && vv < n_values && !(value_flags[vv] & 1u)) keep = true;
                }
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
                    cap_fail(3);
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
        if ((uint32_t)lane < n) {
            uint32_t k = keys[lane], v = vals[lane];
            h = hash_pair(k, v);
            pool[id + 2 + 2 * lane] = k;
            pool[id + 3 + 2 * lane] = v;
        }
        // order-insensitive content hash (matchProperties ignores key order)
        for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o, kWave);
        h = rfl(h);
        if (lane == 0) {
            pool[id] = n;
            pool[id + 1] = h;
        }
        hout = h;
        wsync();
        return id;
    }

    // ------------------------------------------------------------------ scour / pack / zamboni
    // scourNode (mergeTree.ts:1289-1365) over the leaf entries oe[s, s+n), n <= 64, which may
    // span several blocks (their end markers reset the append chain, as each scourNode call
    // starts afresh).  Kept slots are appended to hold[nh..] in order; returns the new count.
    // The leaves are gathered one per lane; only the TextSegment.canAppend chain (textSegment.ts:
    // 63-68, whose length test depends on earlier appends) runs serially, on scalars.
    MT_FI int32_t scour_range(int32_t s, int32_t n, uint32_t *hold, int32_t nh) {
        PF_SCOPE(7);
        const bool in = lane < n;
        const uint32_t e = in ? oe[s + lane] : (uint32_t)kMarkerSlot;
        const uint32_t slot = e & 0xFFFFu;
        const bool mk = slot == kMarkerSlot;
        int32_t rseq = kNoneSeq, seq = 0;
        uint32_t meta = 0, len = 0, props = 0, ph = 0, toff = 0, tcap = 0;
        if (!mk) {
            rseq = s_rseq[slot];
            seq = s_seq[slot];
            meta = s_meta[slot];
            len = s_len[slot];
            props = s_props[slot];
            ph = s_phash[slot];
            toff = s_toff[slot];
            tcap = s_tcap[slot];
        }
        const bool rem = !mk && rseq != kNoneSeq;
        const bool cand = !mk && !rem && seq <= min_seq;
        const uint32_t pprev = __shfl_up(props, 1, kWave), hprev = __shfl_up(ph, 1, kWave);
        const bool peq = lane > 0 && pprev == props;
        const bool pmaybe = lane > 0 && !peq && props != 0u && pprev != 0u && hprev == ph;
        const uint64_t candM = ballot(cand), peqM = ballot(peq), maybeM = ballot(pmaybe);
        const uint64_t freeR = ballot(rem && rseq <= min_seq);
        const uint64_t liveM = ballot(in && !mk);
        uint64_t mergeM = 0;
        uint32_t head = 0;  // lane f (merged): lane of its chain head
        {
            int32_t prev = -1;
            uint32_t acc = 0;
            bool pnl = false, pmk = false;
            for (int32_t k = 0; k < n; k++) {
                if (!((candM >> k) & 1ull)) {
                    prev = -1;
                    continue;
                }
                const uint32_t lk = rdl(len, k), mk_ = rdl(meta, k);
                bool can = false;
                if (prev >= 0 && !pmk && !(mk_ & kMetaMarker) && !pnl && (acc <= kGranularity || lk <= kGranularity)) {
                    if ((peqM >> k) & 1ull) can = true;
                    else if ((maybeM >> k) & 1ull)
                        can = props_match(rdl(props, k - 1), rdl(ph, k - 1), rdl(props, k), rdl(ph, k));
                }
                if (can) {
                    mergeM |= 1ull << k;
                    if (lane == k) head = (uint32_t)prev;
                    acc += lk;
                } else {
                    prev = k;
                    acc = lk;
                    pmk = (mk_ & kMetaMarker) != 0;
                }
                pnl = (mk_ & kMetaEndsNL) != 0;
            }
        }
        // TextSegment.append for every merge, head by head in document order
        if (mergeM) {
            PF_SCOPE(8);
            uint64_t m = mergeM;
            int32_t h = -1;
            uint32_t hslot = 0, pl = 0, ptoff = 0, pcap = 0, hmeta = 0;
            int32_t gcs0 = text_gcs;
            while (m) {
                const int k = first_lane(m);
                m &= m - 1;
                const int32_t hk_ = (int32_t)rdl(head, k);
                if (hk_ != h) {
                    h = hk_;
                    hslot = rdl(slot, h);
                    pl = rdl(len, h);
                    ptoff = rdl(toff, h);
                    pcap = rdl(tcap, h);
                    hmeta = rdl(meta, h);
                }
                const uint32_t fslot = rdl(slot, k), sl = rdl(len, k);
                uint32_t stoff = rdl(toff, k), stcap = rdl(tcap, k);
                if (text_gcs != gcs0) {  // a compaction moved texts: offsets live in LDS again
                    ptoff = s_toff[hslot];
                    pcap = s_tcap[hslot];
                    stoff = s_toff[fslot];
                    stcap = s_tcap[fslot];
                }
                const uint32_t need = pl + sl;
                if (pcap == pl && ptoff + pl == stoff) {
                    // texts already adjacent (split halves, consecutive payloads): take over the region
                    pcap = pl + stcap;
                } else if (pcap >= need) {
                    text_copy(ptoff + pl, stoff, sl);
                } else if (ptoff >= arena_base && ptoff < arena_end && ptoff + pcap == arena_top &&
                           ptoff + ((2u * need + 15u) & ~15u) <= arena_end) {
                    // last allocation of the arena: grow in place
                    pcap = (2u * need + 15u) & ~15u;
                    arena_top = ptoff + pcap;
                    text_copy(ptoff + pl, stoff, sl);
                } else {
                    // reallocate; a compaction inside arena_alloc moves every text, so the head
                    // is written back first and both offsets re-read afterwards
                    s_len[hslot] = pl;
                    s_toff[hslot] = ptoff;
                    s_tcap[hslot] = pcap;
                    wsync();
                    const uint32_t ncap = 2u * need;
                    const uint32_t dst = arena_alloc(ncap);
                    if (status) return nh;
                    if (text_gcs != gcs0) {
                        ptoff = s_toff[hslot];
                        stoff = s_toff[fslot];
                    }
                    text_copy(dst, ptoff, pl);
                    text_copy(dst + pl, stoff, sl);
                    ptoff = dst;
                    pcap = (ncap + 15u) & ~15u;
                }
                pl = need;
                hmeta = (hmeta & ~kMetaEndsNL) | (rdl(meta, k) & kMetaEndsNL);
                s_len[hslot] = pl;
                s_toff[hslot] = ptoff;
                s_tcap[hslot] = pcap;
                s_meta[hslot] = hmeta;
                wsync();
            }
        }
        // unlink removed-below-minSeq leaves and appended ones; keep the rest in order
        const uint64_t freeM = freeR | mergeM;
        const uint64_t holdM = liveM & ~freeM;
        const uint64_t below = (1ull << lane) - 1ull;
        if ((freeM >> lane) & 1ull) {
            s_meta[slot] = ((meta >> 16) + 1u) << 16;  // unlinked, next generation
            s_free[n_free + __popcll(freeM & below)] = (uint16_t)slot;
        }
        if ((holdM >> lane) & 1ull) hold[nh + __popcll(holdM & below)] = slot;
        n_free += __popcll(freeM);
        wsync();
        return nh + __popcll(holdM);
    }

    // pack for an interior block `blk` (its parent's children are interior blocks);
    // repeats upward while the parent underflows (mergeTree.ts:1414-1419)
    MT_FI void pack_interior(int32_t blk) {
        for (;;) {
            int32_t parent = b_parent[blk];
            int32_t pn = b_count[parent];
            uint32_t *hold = scratch;  // grandchildren block ids
            int32_t total = 0;
            for (int32_t ci = 0; ci < pn; ci++) {
                int32_t cb = b_child[parent * 8 + ci];
                int32_t cn = b_count[cb];
                wsync();
                if (lane < cn) hold[total + lane] = b_child[cb * 8 + lane];
                total += cn;
                wsync();
            }
            int32_t child_count = total / (kMaxNodes / 2);
            if (child_count > kMaxNodes - 1) child_count = kMaxNodes - 1;
            if (child_count < 1) child_count = 1;
            int32_t base = total / child_count, extra = total % child_count;
            for (int32_t i = 0; i < pn; i++) free_block(b_child[parent * 8 + i]);
            int32_t read = 0;
            for (int32_t i = 0; i < child_count; i++) {
                int32_t nbi = alloc_block(0);
                if (status) return;
                int32_t cnt = base + (i < extra ? 1 : 0);
                wsync();
                if (lane < cnt) {
                    uint16_t g = (uint16_t)hold[read + lane];
                    b_child[nbi * 8 + lane] = g;
                    b_parent[g] = (uint16_t)nbi;
                }
                wsync();
                b_count[nbi] = (uint8_t)cnt;
                b_parent[nbi] = (uint16_t)parent;
                b_child[parent * 8 + i] = (uint16_t)nbi;
                read += cnt;
            }
            b_count[parent] = (uint8_t)child_count;
            wsync();
            if (child_count < kMaxNodes / 2 && parent != root) blk = parent;
            else return;
        }
    }

    // pack for a leaf block (mergeTree.ts:1368-1420)
    MT_FI void pack_leaf(int32_t blk, int32_t hint) {
        int32_t parent = b_parent[blk];
        int32_t pn = b_count[parent];
        int32_t first = b_child[parent * 8 + 0];
        int32_t s0 = find_entry((uint32_t)first, 1, 0);
        if (s0 < 0) {
            set_fail(ST_INTERNAL);
            return;
        }
        (void)hint;
        uint32_t *hold = scratch + 128;
        int32_t s = s0;
        for (int32_t ci = 0; ci < pn; ci++) s += b_count[b_child[parent * 8 + ci]] + 1;  // leaves + marker
        if (s - s0 > kWave) {
            set_fail(ST_INTERNAL);
            return;
        }
        int32_t total;
        {
            PF_SCOPE(10);
            total = scour_range(s0, s - s0, hold, 0);
        }
        if (status) return;
        int32_t old_end = s;  // one past the last marker
        int32_t child_count = total / (kMaxNodes / 2);
        if (child_count > kMaxNodes - 1) child_count = kMaxNodes - 1;
        if (child_count < 1) child_count = 1;
        int32_t base = total / child_count, extra = total % child_count;
        for (int32_t i = 0; i < pn; i++) free_block(b_child[parent * 8 + i]);
        int32_t new_len = total + child_count;
        oe_move_tail(old_end, s0 + new_len);
        if (status) return;
        // write the regrouped range, one new leaf block at a time
        int32_t read = 0, w = s0;
        for (int32_t i = 0; i < child_count; i++) {
            int32_t nbi = alloc_block(1);
            if (status) return;
            int32_t cnt = base + (i < extra ? 1 : 0);
            wsync();
            if (lane < cnt) oe[w + lane] = ((uint32_t)nbi << 16) | hold[read + lane];
            if (lane == cnt) oe[w + lane] = ((uint32_t)nbi << 16) | kMarkerSlot;
            wsync();
            b_count[nbi] = (uint8_t)cnt;
            b_parent[nbi] = (uint16_t)parent;
            b_child[parent * 8 + i] = (uint16_t)nbi;
            read += cnt;
            w += cnt + 1;
        }
        b_count[parent] = (uint8_t)child_count;
        wsync();
        if (child_count < kMaxNodes / 2 && parent != root) pack_interior(parent);
    }

    // zamboniSegments (mergeTree.ts:1422-1478)
    MT_FI void zamboni() {
        PF_SCOPE(5);
        for (int it = 0; it < kZamboniMax; it++) {
            if (hn < 1 || hseq(1) > min_seq) break;
            uint32_t key;
            int32_t mseq;
            heap_get(key, mseq);
            uint32_t slot = key & 0xFFFFu;
            uint32_t meta = s_meta[slot];
            if ((meta & 0xFFFF0000u) != (key & 0xFFFF0000u) || !(meta & kMetaLinked)) continue;  // parent undefined
            int32_t idx = find_entry(slot, 0, 0);
            if (idx < 0) {
                set_fail(ST_INTERNAL);
                return;
            }
            int32_t blk = rfl((int32_t)(oe[idx] >> 16));
            if (b_scour[blk] == kScourFalse) continue;
            int32_t s = block_start_near((uint32_t)blk, idx);
            int32_t cnt = b_count[blk];
            uint32_t *hold = scratch;
            int32_t nk = scour_range(s, cnt, hold, 0);
            if (status) return;
            b_scour[blk] = kScourFalse;
            if (nk < cnt) {
                wsync();
                if (lane < nk) oe[s + lane] = ((uint32_t)blk << 16) | hold[lane];
                if (lane == nk) oe[s + lane] = ((uint32_t)blk << 16) | kMarkerSlot;
                wsync();
                oe_move_tail(s + cnt + 1, s + nk + 1);
                b_count[blk] = (uint8_t)nk;
                wsync();
                if (nk < kMaxNodes / 2 && blk != root) pack_leaf(blk, s);
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
        }
    }

    // ------------------------------------------------------------------ ops
    // insertSegments + blockInsert for one remote segment (mergeTree.ts:1968-1998, 2141-2224)
    MT_FI void op_insert(const mt_op &op) {
        uint32_t c = op.client;
        uint32_t pos = (uint32_t)op.pos1;
        // ensureIntervalBoundary (mergeTree.ts:2241-2245) and the insertingWalk share one scan:
        // the walk's target is the segment the boundary split cuts, whose left half keeps every
        // entry before it, so the walk resumes at that half with the same view position.
        Loc L = locate(pos, op.ref_seq, c);
        if (L.found && !L.marker && L.excl < pos) {
            int32_t li = split_at(L.idx, pos - L.excl);
            if (status) return;
            L = locate(pos, op.ref_seq, c, li, L.excl);
        }
        bool marker = (op.flags & MT_OPF_MARKER) != 0;
        uint32_t len = marker ? 1u : op.payload_len;
        if (len > 0) {
            PF_SCOPE(3);
            if (!L.found) {
                set_fail(ST_INVALID_POS);
                return;
            }
            int32_t slot = alloc_slot();
            if (slot < 0) return;
            uint32_t props = 0, ph = 0;
            if (op.flags & MT_OPF_HAS_PROPS) {
                pool_reserve(2u + 2u * MT_OPF_NPROPS(op.flags));
                if (status) return;
                props = props_extend(0, props_in + op.pos2, MT_OPF_NPROPS(op.flags), false, ph);
                if (status) return;
            }
            uint32_t gen = s_meta[slot] & 0xFFFF0000u;
            uint32_t meta = gen | kMetaLinked | (c & 63u) | (kNoClient << 6);
            if (marker) meta |= kMetaMarker;
            if (op.flags & MT_OPF_INTERNAL_ENDS_NL) meta |= kMetaEndsNL;
            s_len[slot] = len;
            s_seq[slot] = op.seq;
            s_rseq[slot] = kNoneSeq;
            s_ovl[slot] = 0;
            s_props[slot] = props;
            s_phash[slot] = ph;
            s_toff[slot] = marker ? op.payload : op.payload;
            s_tcap[slot] = marker ? 0u : len;
            s_meta[slot] = meta;
            wsync();
            int32_t blk = insert_leaf(L.idx, (uint32_t)slot);
            if (status) return;
            // saveIfLocal (mergeTree.ts:2164-2179)
            if (op.seq > min_seq) add_to_lru(blk, (uint32_t)slot, op.seq);
        }
        resolve_splits();
        zamboni();
    }

    // markRangeRemoved / annotateRange range walk (nodeMap, mergeTree.ts:2903-2965)
    MT_FI void op_range(const mt_op &op) {
        uint32_t c = op.client;
        int32_t ref = op.ref_seq;
        uint32_t start = (uint32_t)op.pos1, end = (uint32_t)op.pos2;
        // ensureIntervalBoundary(start), ensureIntervalBoundary(end) (mergeTree.ts:2241-2245,
        // 2903-2904): every entry before the start walk's target ends at or before `start`, so
        // the end search and the range walk resume there with its view position.
        Loc A = locate(start, ref, c);
        if (!A.found) {
            resolve_splits();
            zamboni();
            return;
        }
        int32_t from = A.idx;
        uint32_t carry = A.excl;
        if (!A.marker && A.excl < start) {
            from = split_at(A.idx, start - A.excl);
            if (status) return;
        }
        if (end > start) {
            Loc B = containing(end, ref, c, from, carry);
            if (B.found) {
                split_at(B.idx, end - B.excl);
                if (status) return;
                from = shifted(from);
            }
        } else if (end < start) {
            // inverted range: nothing is marked, but the end boundary is still cut
            Loc B = containing(end, ref, c, 0, 0);
            if (B.found) {
                split_at(B.idx, end - B.excl);
                if (status) return;
            }
            from = 0;
            carry = 0;
        }
        const bool is_remove = op.type == MT_OP_REMOVE;
        const bool rewrite = (op.flags & MT_OPF_REWRITE) != 0;
        // per-op memo old prop-set -> new prop-set (annotate)
        uint32_t memo_n = 0;
        uint32_t memo_old = 0, memo_new = 0, memo_h = 0;  // lane i holds entry i
        {
        PF_SCOPE(4);
        for (int32_t base = from; base < n_oe; base += kWave) {
            int32_t j = base + lane;
            bool valid = j < n_oe;
            uint32_t e = valid ? oe[j] : 0u;
            uint32_t vlen = 0;
            bool tie, mk;
            if (valid) view_of(e, ref, c, vlen, tie, mk);
            uint32_t incl = scan_incl(vlen) + carry;
            uint32_t excl = incl - vlen;
            bool hit = valid && vlen > 0 && excl < end && incl > start;
            uint64_t hb = ballot(hit);
            bool past = valid && excl >= end;
            uint64_t pb = ballot(past);
            if (is_remove && hit) {
                uint32_t slot = e & 0xFFFFu;
                if (s_rseq[slot] != kNoneSeq) {
                    s_ovl[slot] |= 1u << c;  // addOverlappingClient (mergeTree.ts:2544-2552)
                } else {
                    s_rseq[slot] = op.seq;
                    s_meta[slot] = (s_meta[slot] & ~(63u << 6)) | ((c & 63u) << 6);
                }
            }
            wsync();
            // in document order: properties (annotate) and addToLRUSet
            while (hb) {
                int f = first_lane(hb);
                hb &= hb - 1;
                uint32_t e2 = rdl(e, f);
                uint32_t slot = e2 & 0xFFFFu;
                int32_t blk = (int32_t)(e2 >> 16);
                if (!is_remove) {
                    int32_t g0 = pool_gcs;
                    pool_reserve(2u + 2u * (64u + op.payload_len));
                    if (status) return;
                    if (pool_gcs != g0) memo_n = 0;  // ids moved
                    uint32_t old = s_props[slot];
                    uint64_t mb = ballot((uint32_t)lane < memo_n && memo_old == old);
                    uint32_t nid, nh;
                    if (mb) {
                        int m = first_lane(mb);
                        nid = rdl(memo_new, m);
                        nh = rdl(memo_h, m);
                    } else {
                        nid = props_extend(old, props_in + op.payload, op.payload_len, rewrite, nh);
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
                    s_props[slot] = nid;
                    s_phash[slot] = nh;
                }
                add_to_lru(blk, slot, op.seq);
                if (status) return;
            }
            wsync();
            if (pb) break;
            carry = rdl(incl, 63);
        }
        }
        resolve_splits();
        zamboni();
    }

    MT_FI void apply(const mt_op &op) {
        pend_n = 0;
        if (op.client >= kMaxClients || (op.client == 0 && op.type != MT_OP_NOOP)) {
            set_fail(ST_UNSUPPORTED);
            return;
        }
        switch (op.type) {
            case MT_OP_INSERT: op_insert(op); break;
            case MT_OP_REMOVE:
            case MT_OP_ANNOTATE: op_range(op); break;
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

    // ------------------------------------------------------------------ output
    MT_FI void write_out(OutRec *out, int32_t out_cap, DocOut *dout, int32_t ops_done, int32_t fail_op) {
        wsync();
        int32_t n = n_oe <= out_cap ? n_oe : out_cap;
        for (int32_t j = lane; j < n; j += kWave) {
            uint32_t e = oe[j];
            uint32_t slot = e & 0xFFFFu;
            OutRec r;
            if (slot == kMarkerSlot) {
                r.len = 0;
                r.seq = 0;
                r.rseq = kNoneSeq;
                r.meta = 0;
                r.ovl = 0;
                r.props = 0;
                r.toff = 0;
            } else {
                r.len = s_len[slot];
                r.seq = s_seq[slot];
                r.rseq = s_rseq[slot];
                r.meta = s_meta[slot];
                r.ovl = s_ovl[slot];
                r.props = s_props[slot];
                r.toff = s_toff[slot];
            }
            r.blk = e;
            out[j] = r;
        }
        if (lane == 0) {
            DocOut o;
            o.status = (n_oe > out_cap && status == ST_OK) ? ST_CAPACITY : status;
            o.cap_kind = (n_oe > out_cap && status == ST_OK) ? 4 : cap_kind;
            o.min_seq = min_seq;
            o.cur_seq = cur_seq;
            o.depth = depth;
            o.n_out = n;
            o.text_top = arena_top;
            o.pool_top = pool_top;
            o.ops_done = ops_done;
            o.max_oe = max_oe;
            o.max_slots = slot_top;
            o.max_blocks = blk_top;
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

template <int SEG>
MT_FI void engine_setup(Engine<SEG> &E, const ReplayParams &P, int64_t d, uint8_t *smem) {
    E.lane = threadIdx.x;
    E.carve(smem);
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
    E.value_flags = P.value_flags;
    E.n_values = P.n_values;
    E.init();
}

template <int SEG>
MT_FI void replay_body(const ReplayParams &P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int64_t w = (int64_t)blockIdx.x;
    if (w >= P.n_docs) return;
    const int64_t d = P.doc_list ? (int64_t)P.doc_list[w] : w;
    Engine<SEG> E;
#ifdef MT_PROF
    for (int k = 0; k < kProfSlots; k++) E.pf[k] = 0;
    const uint64_t t_kernel = clock64();
#endif
    engine_setup(E, P, d, smem);
    const mt_op *ops = (const mt_op *)P.ops;
    const int64_t b0 = P.doc_op_off[d], b1 = P.doc_op_off[d + 1];
    int32_t done = 0, fail_op = -1;
    // ops stream through registers 64 at a time (coalesced 2 KiB loads), broadcast by readlane
    mt_op cur = load_op_lane(ops, b0 + E.lane, b1);
    for (int64_t base = b0; base < b1 && E.status == ST_OK; base += kWave) {
        mt_op nxt = load_op_lane(ops, base + kWave + E.lane, b1);
        int64_t n = b1 - base < kWave ? b1 - base : kWave;
        for (int i = 0; i < n; i++) {
            mt_op op = bcast_op(cur, i);
            E.apply(op);
            if (E.status != ST_OK) {
                fail_op = (int32_t)(base - b0 + i);
                break;
            }
            done++;
        }
        cur = nxt;
    }
    E.write_out(P.out + w * (int64_t)P.out_cap, P.out_cap, P.doc_out + w, done, fail_op);
#ifdef MT_PROF
    E.pf[0] = clock64() - t_kernel;
    if (P.prof && E.lane < kProfSlots) {
        uint64_t v = E.pf[0];
        for (int k = 1; k < kProfSlots; k++)
            if (E.lane == k) v = E.pf[k];
        P.prof[w * kProfSlots + E.lane] = v;
    }
#endif
}

// Generator: draws each op from the issuer's view (include/mt_gen.h, DESIGN.md
// "Synthetic op logs"), writes the record + payload, then applies it as the observer.
template <int SEG>
MT_FI void generate_body(const ReplayParams &P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int64_t w = (int64_t)blockIdx.x;
    if (w >= P.n_docs) return;
    const int64_t d = P.doc_list ? (int64_t)P.doc_list[w] : w;  // re-generation of overflowed docs
    const mt_gen_params g = *(const mt_gen_params *)P.gen;
    Engine<SEG> E;
    engine_setup(E, P, d, smem);
    mt_op *ops_out = (mt_op *)P.gen_ops + d * (int64_t)g.n_ops;
    mt_prop *props_out = (mt_prop *)P.gen_props;
    const int64_t prop_base = d * (int64_t)(2 * g.n_ops);
    E.props_in = props_out;
    uint64_t x = mt_rng_seed(g.seed, (uint64_t)(P.doc_first + d));
    __shared__ int32_t lref[64];  // last refSeq per client (160 B static + 16-aligned dynamic base)
    lref[E.lane] = 0;
    wsync();
    uint32_t pay_top = 0, np = 0;
    int32_t done = 0, fail_op = -1;
    for (int32_t k = 1; k <= g.n_ops; k++) {
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
        op.type = (uint8_t)type;
        op.client = (uint8_t)c;
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
            for (uint32_t i = 0; i < n; i++) {
                uint32_t r = mt_rng_below(&x, 100);
                if ((int32_t)r < g.pct_newline) {
                    ch = (uint16_t)'\n';
                } else {
                    uint32_t a = mt_rng_below(&x, 27);  // "abcdefghijklmnopqrstuvwxyz "
                    ch = a < 26u ? (uint16_t)('a' + a) : (uint16_t)' ';
                }
                if (E.lane == 0) E.text[pay_top + i] = ch;
            }
            if (ch == (uint16_t)'\n') op.flags |= MT_OPF_INTERNAL_ENDS_NL;
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
