// mt_snapshot.hip — SnapshotV1 serialization of final segment tables on the GPU.
//
// Reference: SnapshotV1.extractSync + emit (packages/dds/merge-tree/src/snapshotV1.ts:85-247)
// with the chunk format of snapshotChunks.ts:122-131 and segment.toJSONObject()
// (textSegment.ts:48-54, mergeTree.ts:652-656).  Output is byte-identical to the host
// serializer mt_doc_snapshot_v1 (mt_host.cpp), which the parity tests compare it against.
//
// One wavefront per document walks the document's mt::OutRec records in order:
//   * records removed at or below minSeq are dropped (snapshotV1.ts:178-186);
//   * records at or below minSeq that are not removed coalesce into runs — text after text,
//     the run not ending in '\n', either side <= TextSegmentGranularity, equal properties
//     (snapshotV1.ts:191-210: canAppend + matchProperties);
//   * everything else is written standalone with seq / client / removedSeq / removedClient.
// Segments close a chunk once its length reaches chunk_size (snapshotV1.ts:132-160), so chunk
// boundaries are known on the fly.  Two launches per batch: pass 0 sizes every chunk (count,
// length, bytes) into P.meta; the host prefix-sums the per-document bytes; pass 1 writes the
// blobs back to back at P.dst + P.dst_off[doc] (header blob first, then body_0 ..).
//
// JSON strings are escaped lane-parallel, 64 UTF-16 code units per step: per-unit byte counts
// (JSON.stringify escapes, UTF-8 widths, surrogate pairs -> 4 bytes, lone surrogates -> \udxxx),
// a wave exclusive scan for offsets, then every lane stores its bytes.  A high surrogate at
// the end of a record is carried into the next record of the same run, so pairs split across
// coalesced records join exactly as in the reference's concatenated string.
#include <hip/hip_runtime.h>

#include "../../include/mt_oplog.h"
#include "mt_device.h"

namespace mt {
namespace {

constexpr uint32_t kNoRank = 0xFFFFFFFFu;

__device__ __constant__ uint64_t kPow10[20] = {1ull,
                                               10ull,
                                               100ull,
                                               1000ull,
                                               10000ull,
                                               100000ull,
                                               1000000ull,
                                               10000000ull,
                                               100000000ull,
                                               1000000000ull,
                                               10000000000ull,
                                               100000000000ull,
                                               1000000000000ull,
                                               10000000000000ull,
                                               100000000000000ull,
                                               1000000000000000ull,
                                               10000000000000000ull,
                                               100000000000000000ull,
                                               1000000000000000000ull,
                                               10000000000000000000ull};

__device__ __forceinline__ uint32_t lane() { return threadIdx.x; }
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }

// wave-wide scans on DPP lane moves (no LDS round trips): within each row of 16 lanes row_shr 1, 2,
// 4, 8 (a lane whose source is outside the row adds 0), then row 0's total into row 1 and row 2's
// into row 3 (row_bcast:15), then rows 0-1's total into rows 2-3 (row_bcast:31)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    uint32_t x = v;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total) {
    const uint32_t x = wave_incl_scan(v);
    *total = rl(x, 63);
    return x - v;
}
// the value of lane - 1 (lane 0: 0) and of lane + 1 (lane 63: 0): DPP wave_shr:1 / wave_shl:1
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);
}

__device__ __forceinline__ bool is_hi(uint32_t c) { return c >= 0xD800u && c <= 0xDBFFu; }
__device__ __forceinline__ bool is_lo(uint32_t c) { return c >= 0xDC00u && c <= 0xDFFFu; }

// Uniform writer: every lane tracks `pos`; kWrite=false only counts bytes.
template <bool kWrite>
struct Writer {
    uint8_t *dst;
    int64_t pos;

    __device__ __forceinline__ void byte(uint32_t c) {
        if (kWrite && lane() == 0) dst[pos] = (uint8_t)c;
        pos++;
    }
    // a string literal (read-only data in global memory, one byte per lane)
    template <int N>
    __device__ __forceinline__ void lit(const char (&s)[N]) {
        static_assert(N - 1 <= 64, "literal longer than a wave");
        const char *p = s;
        if (kWrite && lane() < (uint32_t)(N - 1)) dst[pos + lane()] = (uint8_t)p[lane()];
        pos += N - 1;
    }
    __device__ __forceinline__ void copy(const uint8_t *src, uint32_t n) {
        if (kWrite)
            for (uint32_t i = lane(); i < n; i += 64) dst[pos + i] = src[i];
        pos += n;
    }
    // std::to_string of a signed 64-bit value
    __device__ __forceinline__ void num(int64_t v) {
        if (v < 0) {
            byte('-');
            v = -v;
        }
        const uint64_t u = (uint64_t)v;
        int nd = 1;
        while (nd < 20 && u >= kPow10[nd]) nd++;
        if (kWrite && lane() < (uint32_t)nd) dst[pos + lane()] = (uint8_t)('0' + (u / kPow10[nd - 1 - lane()]) % 10);
        pos += nd;
    }
    // JSON string body of the virtual array v[0..m): v[0] = carry (when has_carry) followed by
    // t[0..n).  Unless `last`, a trailing high surrogate is held back in *carry_out.
    __device__ __forceinline__ void text(const uint16_t *t, uint32_t n, int32_t carry, bool last, int32_t *carry_out) {
        const uint32_t hc = carry >= 0 ? 1u : 0u, m = n + hc;
        uint32_t me = m;
        *carry_out = -1;
        if (!last && m > 0) {
            const uint32_t c = (m - 1 >= hc) ? t[m - 1 - hc] : (uint32_t)carry;
            if (is_hi(c)) {
                me = m - 1;
                *carry_out = (int32_t)c;
            }
        }
        for (uint32_t base = 0; base < me; base += 64) {
            const uint32_t k = base + lane();
            auto at = [&](uint32_t i) -> uint32_t { return i < hc ? (uint32_t)carry : (uint32_t)t[i - hc]; };
            uint32_t c = 0, p = 0, nx = 0, nb = 0;
            if (k < me) {
                c = at(k);
                p = k > 0 ? at(k - 1) : 0u;
                nx = k + 1 < m ? at(k + 1) : 0u;
                if (c == 0x22 || c == 0x5C || c == 0x08 || c == 0x0C || c == 0x0A || c == 0x0D || c == 0x09) nb = 2;
                else if (c < 0x20) nb = 6;
                else if (is_hi(c)) nb = is_lo(nx) ? 4 : 6;
                else if (is_lo(c)) nb = is_hi(p) ? 0 : 6;
                else nb = c < 0x80 ? 1 : c < 0x800 ? 2 : 3;
            }
            uint32_t tot;
            const uint32_t off = wave_excl_scan(nb, &tot);
            if (kWrite && nb) {
                uint8_t *o = dst + pos + off;
                const char *hex = "0123456789abcdef";
                if (nb == 2 && c < 0x80) {
                    o[0] = '\\';
                    o[1] = c == 0x22 ? '"' : c == 0x5C ? '\\' : c == 0x08 ? 'b' : c == 0x0C ? 'f' : c == 0x0A ? 'n'
                                                                                    : c == 0x0D ? 'r' : 't';
                } else if (nb == 6) {
                    o[0] = '\\';
                    o[1] = 'u';
                    o[2] = hex[(c >> 12) & 15];
                    o[3] = hex[(c >> 8) & 15];
                    o[4] = hex[(c >> 4) & 15];
                    o[5] = hex[c & 15];
                } else if (nb == 4) {
                    const uint32_t cp = 0x10000u + ((c - 0xD800u) << 10) + (nx - 0xDC00u);
                    o[0] = (uint8_t)(0xF0 | (cp >> 18));
                    o[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
                    o[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
                    o[3] = (uint8_t)(0x80 | (cp & 0x3F));
                } else if (nb == 1) {
                    o[0] = (uint8_t)c;
                } else if (nb == 2) {
                    o[0] = (uint8_t)(0xC0 | (c >> 6));
                    o[1] = (uint8_t)(0x80 | (c & 0x3F));
                } else {
                    o[0] = (uint8_t)(0xE0 | (c >> 12));
                    o[1] = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
                    o[2] = (uint8_t)(0x80 | (c & 0x3F));
                }
            }
            pos += tot;
        }
    }
};

struct Rec {  // one OutRec, wave-uniform
    uint32_t len, meta, props, toff, blk;
    int32_t seq, rseq;
    uint32_t lastc;  // last code unit of a text record with len > 0
};

// lane l of the tile holds record base + l
struct Tile {
    uint32_t len, meta, props, toff, blk, lastc;
    int32_t seq, rseq;
    __device__ __forceinline__ void load(const OutRec *rec, int32_t i, int32_t n, const uint16_t *text) {
        uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, kOutBlockEnd);
        if (i < n) {
            a = reinterpret_cast<const uint4 *>(rec + i)[0];
            b = reinterpret_cast<const uint4 *>(rec + i)[1];
        }
        len = a.x;
        seq = (int32_t)a.y;
        rseq = (int32_t)a.z;
        meta = a.w;
        props = b.y;
        toff = b.z;
        blk = b.w;
        uint32_t lc = 0;
        if (!out_is_end(blk) && !(meta & kMetaMarker) && len > 0) lc = text[toff + len - 1];
        lastc = lc;
    }
    __device__ __forceinline__ Rec get(uint32_t l) const {
        Rec r;
        r.len = rl(len, l);
        r.meta = rl(meta, l);
        r.props = rl(props, l);
        r.toff = rl(toff, l);
        r.blk = rl(blk, l);
        r.seq = (int32_t)rl((uint32_t)seq, l);
        r.rseq = (int32_t)rl((uint32_t)rseq, l);
        r.lastc = rl(lastc, l);
        return r;
    }
};

template <bool kWrite>
struct Doc {
    const SnapParams &P;
    const OutRec *rec;
    const uint16_t *text;
    const uint32_t *pool;
    int32_t n_out, min_seq, cur_seq;
    int32_t cli_first, cli_n;
    Writer<kWrite> W;
    int32_t *mrow;
    // chunking
    int32_t nch = 0;       // chunks closed
    bool open = false;
    int64_t ccount = 0, clen = 0, total_count = 0, total_len = 0;
    int64_t seg_bytes_at_open = 0;
    bool overflow = false;
    int64_t all_len = 0, all_count = 0;  // pass 1: the document's totals from pass 0
    // coalescing run (snapshotV1.ts:191-210)
    bool have_prev = false, run_text = false, run_ends_nl = false;
    int32_t run_first = 0, run_last = 0;
    int64_t run_len = 0;
    uint32_t run_props = 0, run_ref = 0;

    __device__ Doc(const SnapParams &p, const OutRec *r, const uint16_t *t, const uint32_t *pl, const DocOut &o,
                   int32_t cf, int32_t cn, uint8_t *dst, int32_t *mr)
        : P(p), rec(r), text(t), pool(pl), n_out(o.n_out), min_seq(o.min_seq), cur_seq(o.cur_seq), cli_first(cf),
          cli_n(cn), W{dst, 0}, mrow(mr) {}

    __device__ __forceinline__ static bool skipped(const Rec &r, int32_t min_seq) {
        if (out_is_end(r.blk)) return true;
        // unacked inserts and segments removed at or below the MSN (a pending local remove has
        // removedSeq -1) are elided (snapshotV1.ts:184-186)
        return r.seq == kUnassignedSeq || (r.rseq != kNoneSeq && r.rseq <= min_seq);
    }

    __device__ __forceinline__ void str(const uint32_t *tab, uint32_t i) { W.copy(P.strs + tab[2 * i], tab[2 * i + 1]); }
    __device__ __forceinline__ void client(uint32_t id) {
        if (id < (uint32_t)cli_n) str(P.cli_str, (uint32_t)cli_first + id);
        else str(P.cli_str, id == MT_CLIENT_NONCOLLAB ? 1u : 0u);  // "original" / "undefined"
    }
    __device__ __forceinline__ uint32_t key_rank(uint32_t k) const {
        return k < (uint32_t)P.n_keys ? P.key_rank[k] : kNoRank;
    }
    __device__ __forceinline__ void prop_entry(uint32_t id, uint32_t i, bool &first) {
        const uint32_t k = pool[id + 2 + 2 * i], v = pool[id + 3 + 2 * i];
        if (!first) W.byte(',');
        first = false;
        str(P.key_str, k < (uint32_t)P.n_keys ? k : (uint32_t)P.n_keys);
        W.byte(':');
        str(P.val_str, v < (uint32_t)P.n_values ? v : 0u);
    }
    // JSON.stringify(properties): array-index keys ascending, then insertion order
    __device__ __forceinline__ void props_json(uint32_t id) {
        const uint32_t n = pool[id];
        W.byte('{');
        bool first = true;
        bool any_index = false;
        for (uint32_t base = 0; base < n; base += 64) {
            const uint32_t i = base + lane();
            const bool ix = i < n && key_rank(pool[id + 2 + 2 * i]) != kNoRank;
            any_index |= __ballot(ix) != 0;
        }
        if (any_index) {
            int64_t last = -1;
            for (;;) {
                uint32_t best = kNoRank, best_i = 0;
                for (uint32_t base = 0; base < n; base += 64) {
                    const uint32_t i = base + lane();
                    uint32_t r = i < n ? key_rank(pool[id + 2 + 2 * i]) : kNoRank;
                    if ((int64_t)r <= last) r = kNoRank;
                    uint32_t m = r;
                    for (int off = 32; off > 0; off >>= 1) m = min(m, (uint32_t)__shfl_xor(m, off, 64));
                    if (m < best) {
                        best = m;
                        best_i = base + (uint32_t)__builtin_ctzll(__ballot(r == m));
                    }
                }
                if (best == kNoRank) break;
                prop_entry(id, best_i, first);
                last = best;
            }
        }
        for (uint32_t i = 0; i < n; i++)
            if (key_rank(pool[id + 2 + 2 * i]) == kNoRank) prop_entry(id, i, first);
        W.byte('}');
    }
    // matchProperties(a, c) over the pool's (key, value) lists (properties.ts:62-93): same key
    // set, values compared structurally (value_rel: class equality or a listed exception); an
    // undecided comparison leaves the document to the host serializer
    __device__ __forceinline__ bool props_match(uint32_t a, uint32_t c) {
        if (!a || !c) return a == c;
        const uint32_t ha = pool[a + 1], hc = pool[c + 1];
        if ((ha | hc) & kSetNever) return false;  // a value that matches nothing (NaN !== NaN)
        if (a == c) return true;
        const uint32_t na = pool[a], nc = pool[c];
        if (na != nc) return false;
        if ((ha & hc & kSetRegular) && ha != hc) return false;
        for (uint32_t base = 0; base < na; base += 64) {
            const uint32_t i = base + lane();
            int rel = 1;
            if (i < na) {
                const uint32_t ka = pool[a + 2 + 2 * i], va = pool[a + 3 + 2 * i];
                rel = 0;
                for (uint32_t j = 0; j < nc; j++)
                    if (pool[c + 2 + 2 * j] == ka)
                        rel = value_rel(va, pool[c + 3 + 2 * j], P.value_class, P.value_flags, (uint32_t)P.n_values,
                                        P.exc, P.n_exc);
            }
            if (__ballot(rel < 0)) {
                overflow = true;
                return false;
            }
            if (__ballot(rel != 1)) return false;
        }
        return true;
    }

    // ---- chunks
    template <class Wr>
    __device__ __forceinline__ void header(Wr &w, int64_t count, int64_t length) {
        w.lit("{\"version\":\"1\",\"segmentCount\":");
        w.num(count);
        w.lit(",\"length\":");
        w.num(length);
        w.lit(",\"segments\":[");
    }
    template <class Wr>
    __device__ __forceinline__ void trailer(Wr &w, int32_t c, int64_t start, int32_t n_chunks, int64_t tlen,
                            int64_t tcount) {
        w.lit("],\"startIndex\":");
        w.num(start);
        if (c == 0) {
            w.lit(",\"headerMetadata\":{\"minSequenceNumber\":");
            w.num(min_seq);
            w.lit(",\"sequenceNumber\":");
            w.num(cur_seq);
            w.lit(",\"orderedChunkMetadata\":[{\"id\":\"header\"}");
            for (int32_t bi = 1; bi < n_chunks; bi++) {
                w.lit(",{\"id\":\"body_");
                w.num(bi - 1);
                w.lit("\"}");
            }
            w.lit("],\"totalLength\":");
            w.num(tlen);
            w.lit(",\"totalSegmentCount\":");
            w.num(tcount);
            w.byte('}');
        }
        w.byte('}');
    }
    __device__ __forceinline__ void open_chunk() {
        open = true;
        ccount = clen = 0;
        if (kWrite) header(W, mrow[1 + 3 * nch], mrow[2 + 3 * nch]);
        seg_bytes_at_open = W.pos;
    }
    __device__ __forceinline__ void close_chunk() {
        if (nch >= kSnapMaxChunks) {
            overflow = true;
        } else if (kWrite) {
            trailer(W, nch, total_count, mrow[0], all_len, all_count);
        } else if (lane() == 0) {
            mrow[1 + 3 * nch] = (int32_t)ccount;
            mrow[2 + 3 * nch] = (int32_t)clen;
            mrow[3 + 3 * nch] = (int32_t)(W.pos - seg_bytes_at_open);  // segments + commas; framing added at the end
        }
        total_count += ccount;
        total_len += clen;
        nch++;
        open = false;
    }
    __device__ __forceinline__ void begin_seg() {
        if (!open) open_chunk();
        else W.byte(',');
    }
    __device__ __forceinline__ void end_seg(int64_t len) {
        ccount++;
        clen += len;
        if (clen >= P.chunk_size) close_chunk();
    }

    // ---- segments
    __device__ __forceinline__ void text_run() {
        W.byte('"');
        int32_t carry = -1;
        Tile T;
        for (int32_t base = run_first & ~63; base <= run_last; base += 64) {
            T.load(rec, base + (int32_t)lane(), n_out, text);
            const int32_t lo = max(base, run_first), hi = min(base + 63, run_last);
            for (int32_t i = lo; i <= hi; i++) {
                const Rec r = T.get((uint32_t)(i - base));
                if (skipped(r, min_seq)) continue;
                int32_t co;
                W.text(text + r.toff, r.len, carry, i == run_last, &co);
                carry = co;
            }
        }
        W.byte('"');
    }
    __device__ __forceinline__ void push_prev() {
        if (!have_prev) return;
        have_prev = false;
        begin_seg();
        if (run_text) {
            if (run_props) {
                W.lit("{\"text\":");
                text_run();
                W.lit(",\"props\":");
                props_json(run_props);
                W.byte('}');
            } else {
                text_run();
            }
        } else {
            W.lit("{\"marker\":{\"refType\":");
            W.num(run_ref);
            W.byte('}');
            if (run_props) {
                W.lit(",\"props\":");
                props_json(run_props);
            }
            W.byte('}');
        }
        end_seg(run_text ? run_len : 1);
    }
    __device__ __forceinline__ void set_prev(const Rec &r, int32_t i) {
        have_prev = true;
        run_text = !(r.meta & kMetaMarker);
        run_first = run_last = i;
        run_len = run_text ? r.len : 0;
        run_props = r.props;
        run_ref = r.toff;
        run_ends_nl = run_text && r.len > 0 && r.lastc == 0x0Au;
    }
    __device__ __forceinline__ void standalone(const Rec &r) {
        begin_seg();
        W.lit("{\"json\":");
        const bool txt = !(r.meta & kMetaMarker);
        if (txt) {
            if (r.props) W.lit("{\"text\":");
            int32_t co;
            W.byte('"');
            W.text(text + r.toff, r.len, -1, true, &co);
            W.byte('"');
            if (r.props) {
                W.lit(",\"props\":");
                props_json(r.props);
                W.byte('}');
            }
        } else {
            W.lit("{\"marker\":{\"refType\":");
            W.num(r.toff);
            W.byte('}');
            if (r.props) {
                W.lit(",\"props\":");
                props_json(r.props);
            }
            W.byte('}');
        }
        if (r.seq > min_seq) {
            W.lit(",\"seq\":");
            W.num(r.seq);
            W.lit(",\"client\":");
            client(meta_cli(r.meta));
        }
        if (r.rseq != kNoneSeq) {
            W.lit(",\"removedSeq\":");
            W.num(r.rseq);
            W.lit(",\"removedClient\":");
            client(meta_rcli(r.meta));
        }
        W.byte('}');
        end_seg(r.len);
    }

    __device__ __forceinline__ void walk() {
        Tile T;
        for (int32_t base = 0; base < n_out && !overflow; base += 64) {
            T.load(rec, base + (int32_t)lane(), n_out, text);
            const int32_t hi = min(64, n_out - base);
            for (int32_t j = 0; j < hi && !overflow; j++) {
                const Rec r = T.get((uint32_t)j);
                if (skipped(r, min_seq)) continue;
                const bool removed = r.rseq != kNoneSeq;
                if (r.seq <= min_seq && !removed) {
                    if (!have_prev) {
                        set_prev(r, base + j);
                        continue;
                    }
                    const bool txt = !(r.meta & kMetaMarker);
                    const bool can = run_text && txt && !run_ends_nl && (run_len <= kGranularity || r.len <= kGranularity);
                    if (can && props_match(run_props, r.props)) {
                        run_last = base + j;
                        run_len += r.len;
                        if (r.len > 0) run_ends_nl = r.lastc == 0x0Au;
                    } else {
                        push_prev();
                        set_prev(r, base + j);
                    }
                } else {
                    push_prev();
                    standalone(r);
                }
            }
        }
        if (!overflow) push_prev();
        if (!overflow && (open || nch == 0)) {
            if (!open) open_chunk();
            close_chunk();
        }
    }
};

template <bool kWrite>
__device__ __forceinline__ void snapshot_doc(const SnapParams &P, int64_t w) {
    const int64_t d = P.doc_list ? P.doc_list[w] : w;
    if (kWrite && P.bytes[d] < 0) return;
    const DocOut o = P.doc_out[w];
    int32_t cf = P.cli_first, cn = P.cli_n;
    if (P.doc_cli) {
        cf = P.doc_cli[2 * d];
        cn = P.doc_cli[2 * d + 1];
    }
    int32_t *mrow = P.meta + d * (int64_t)kSnapMeta;
    Doc<kWrite> D(P, P.out + w * (int64_t)P.out_cap, P.text + P.doc_text_base[d], P.pool + P.doc_pool_base[d], o, cf,
                  cn, kWrite ? P.dst + P.dst_off[d] : nullptr, mrow);
    if (kWrite)
        for (int32_t c = 0; c < mrow[0]; c++) {
            D.all_count += mrow[1 + 3 * c];
            D.all_len += mrow[2 + 3 * c];
        }
    D.walk();
    if (kWrite) return;
    // framing of each chunk, now that counts and totals are known
    int64_t total = 0;
    if (!D.overflow) {
        Writer<false> f{nullptr, 0};
        int64_t start = 0;
        for (int32_t c = 0; c < D.nch; c++) {
            const int64_t cnt = mrow[1 + 3 * c], len = mrow[2 + 3 * c];
            f.pos = mrow[3 + 3 * c];
            D.header(f, cnt, len);
            D.trailer(f, c, start, D.nch, D.total_len, D.total_count);
            if (lane() == 0) mrow[3 + 3 * c] = (int32_t)f.pos;
            total += f.pos;
            start += cnt;
        }
    }
    if (lane() == 0) {
        mrow[0] = D.overflow ? 0 : D.nch;
        P.bytes[d] = D.overflow ? -1 : total;
    }
}

// ---------------------------------------------------------------- lane-parallel serializer
// The same walk, re-organised so that HBM latency is paid per batch of 64, not per record:
//   stage 1, per tile of 64 records: every lane loads its record, classifies it (skipped /
//     settled / text / ends in '\n') and compares its properties with the previous kept
//     record's (matchProperties; consecutive comparisons decide a run because matchProperties is
//     an equivalence on decided pairs), then a register-only scalar loop applies the run rules
//     (canAppend + TextSegmentGranularity, snapshotV1.ts:191-210) and queues segments;
//   stage 2, per batch of 64 queued segments: lane j sizes segment j's JSON (a run's text escaped
//     as one string, its props, a marker, or a standalone record with seq / client fields),
//     a scalar loop places the segments in chunks (commas, headers, trailers: snapshotV1.ts:
//     132-160) and, in the writing pass, lane j writes segment j at its offset.
// Both passes rebuild the segments; pass 1 writes where pass 0 counted.
enum : uint32_t { kSegRun = 0, kSegMarker = 1, kSegAlone = 2 };
constexpr uint32_t kFSkip = 1, kFSettled = 2, kFText = 4, kFEndsNL = 8, kFMatch = 16, kFUndecided = 32,
                   kFFirstLo = 64, kFLastHi = 128;

// one lane's output: its own segment, bytes counted (kWrite false) or stored at o[n]
// one lane's output: bytes counted, and stored at o[n] when o is set (the writing pass)
struct LOut {
    uint8_t *o;
    uint32_t n;
    __device__ __forceinline__ void put(uint32_t c) {
        if (o) o[n] = (uint8_t)c;
        n++;
    }
    // a literal: its bytes are immediates (no loads), one store each
    template <int N>
    __device__ __forceinline__ void lit(const char (&s)[N]) {
        if (o) {
#pragma unroll
            for (int i = 0; i < N - 1; i++) o[n + i] = (uint8_t)s[i];
        }
        n += N - 1;
    }
    // a table string: eight loads in flight, then their stores (the source is read-only, but a
    // byte store may alias it as far as the compiler knows)
    __device__ __forceinline__ void bytes(const uint8_t *src, uint32_t len) {
        if (o)
            for (uint32_t i = 0; i < len; i += 8) {
                uint32_t t[8];
#pragma unroll
                for (int q = 0; q < 8; q++) t[q] = i + q < len ? src[i + q] : 0u;
#pragma unroll
                for (int q = 0; q < 8; q++)
                    if (i + q < len) o[n + i + q] = (uint8_t)t[q];
            }
        n += len;
    }
    // std::to_string of a 32-bit signed value
    __device__ __forceinline__ void num(int32_t v) {
        uint32_t u = (uint32_t)v;
        if (v < 0) {
            put('-');
            u = 0u - u;
        }
        const uint32_t nd = 1u + (u >= 10u) + (u >= 100u) + (u >= 1000u) + (u >= 10000u) + (u >= 100000u) +
                            (u >= 1000000u) + (u >= 10000000u) + (u >= 100000000u) + (u >= 1000000000u);
        if (o)
            for (uint32_t k = nd; k-- > 0;) {
                o[n + k] = (uint8_t)('0' + u % 10u);
                u /= 10u;
            }
        n += nd;
    }
};

// per-wave LDS of the batch text pass (one wave per workgroup): per record of a 64-record sub-tile
// its escaped bytes / output offset / prefix of bytes before it; per segment of the batch its text
// bytes (sizing) or its next free text byte (writing)
__shared__ uint32_t s_rt[64], s_ro[64], s_rx[64], s_seg[64];
// segments a tile closes (lane-parallel run formation), in order, before they join the queue:
// kind, first, last, props, ref, chunk length
__shared__ uint32_t s_q[6][72];

// JSON bytes of code unit c of one record's text, given its neighbours in the record (0: none)
__device__ __forceinline__ uint32_t unit_bytes(uint32_t c, uint32_t p, uint32_t nx) {
    if (c == 0x22 || c == 0x5C || c == 0x08 || c == 0x0C || c == 0x0A || c == 0x0D || c == 0x09) return 2;
    if (c < 0x20) return 6;
    if (is_hi(c)) return is_lo(nx) ? 4 : 6;
    if (is_lo(c)) return is_hi(p) ? 0 : 6;
    return c < 0x80 ? 1 : c < 0x800 ? 2 : 3;
}
__device__ __forceinline__ void unit_write(uint8_t *o, uint32_t nb, uint32_t c, uint32_t nx) {
    const char *hex = "0123456789abcdef";
    if (nb == 2 && c < 0x80) {
        o[0] = '\\';
        o[1] = c == 0x22 ? '"' : c == 0x5C ? '\\' : c == 0x08 ? 'b' : c == 0x0C ? 'f' : c == 0x0A ? 'n' : c == 0x0D ? 'r' : 't';
    } else if (nb == 6) {
        o[0] = '\\';
        o[1] = 'u';
        o[2] = (uint8_t)hex[(c >> 12) & 15];
        o[3] = (uint8_t)hex[(c >> 8) & 15];
        o[4] = (uint8_t)hex[(c >> 4) & 15];
        o[5] = (uint8_t)hex[c & 15];
    } else if (nb == 4) {
        const uint32_t cp = 0x10000u + ((c - 0xD800u) << 10) + (nx - 0xDC00u);
        o[0] = (uint8_t)(0xF0 | (cp >> 18));
        o[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
        o[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
        o[3] = (uint8_t)(0x80 | (cp & 0x3F));
    } else if (nb == 1) {
        o[0] = (uint8_t)c;
    } else if (nb == 2) {
        o[0] = (uint8_t)(0xC0 | (c >> 6));
        o[1] = (uint8_t)(0x80 | (c & 0x3F));
    } else if (nb == 3) {
        o[0] = (uint8_t)(0xE0 | (c >> 12));
        o[1] = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
        o[2] = (uint8_t)(0x80 | (c & 0x3F));
    }
}

// MT_SNAP_PROF builds: cycles per phase of the lane-parallel serializer, per document, in the
// tail of its meta row (pass 0 at [kSnapMeta-5, kSnapMeta), pass 1 at [kSnapMeta-10, kSnapMeta-5),
// in units of 64 cycles): tile loads / flags, the record loop, segment framing, text, placement
#ifdef MT_SNAP_PROF
#define SNAP_T0() const uint64_t t0_ = __builtin_readcyclecounter()
#define SNAP_ADD(k) pf[k] += __builtin_readcyclecounter() - t0_
#else
#define SNAP_T0()
#define SNAP_ADD(k)
#endif

template <bool kWrite>
struct LaneDoc {
    const SnapParams P;  // by value: a reference to the kernel argument would copy it to scratch
    const OutRec *rec;
    const uint16_t *text;
    const uint32_t *pool;
    int32_t n_out, min_seq, cur_seq;
    int32_t cli_first, cli_n;
    Writer<kWrite> W;  // the wave's cursor: commas, headers, trailers
    int32_t *mrow;
    uint32_t *rb, *sfr;  // this document's rows of P.rec_bytes / P.seg_frame (null: none)
    int32_t *ext = nullptr;            // chunk triples beyond the meta row (P.chunk_ext)
    int32_t max_ch = kSnapMaxChunks;   // chunks this document may hold on the GPU
    __device__ __forceinline__ int32_t *cm(int32_t c) const {
        return c < kSnapMaxChunks ? mrow + 1 + 3 * c : ext + 3 * (c - kSnapMaxChunks);
    }
    // chunking (as Doc)
    int32_t nch = 0;
    bool open = false;
    int64_t ccount = 0, clen = 0, total_count = 0, total_len = 0;
    int64_t seg_bytes_at_open = 0;
    bool overflow = false;
    int64_t all_len = 0, all_count = 0;
    // the open run
    bool have_prev = false, run_text = false, run_ends_nl = false, run_hi = false;
    int32_t run_first = 0, run_last = 0;
    uint32_t run_len = 0, run_props = 0, run_ref = 0;
    // queued segments, lane j = segment j: kind, first / last record, props, refType, chunk length
    uint32_t sk = 0, sp = 0, sr = 0, sn = 0;
    int32_t sf = 0, sl = 0;
    int32_t nseg = 0;
    // the last kept record of the previous tile: its props and whether it is settled text
    uint32_t carry_props = 0;
    bool carry_st = false;
#ifdef MT_SNAP_PROF
    uint64_t pf[5] = {0, 0, 0, 0, 0};
#endif

    __device__ LaneDoc(const SnapParams &p, const OutRec *r, const uint16_t *t, const uint32_t *pl, const DocOut &o,
                       int32_t cf, int32_t cn, uint8_t *dst, int32_t *mr)
        : P(p), rec(r), text(t), pool(pl), n_out(o.n_out), min_seq(o.min_seq), cur_seq(o.cur_seq), cli_first(cf),
          cli_n(cn), W{dst, 0}, mrow(mr), rb(nullptr), sfr(nullptr) {}

    __device__ __forceinline__ uint32_t key_rank(uint32_t k) const { return k < (uint32_t)P.n_keys ? P.key_rank[k] : kNoRank; }
    __device__ __forceinline__ bool skipped(uint32_t blk, int32_t seq, int32_t rseq) const {
        return out_is_end(blk) || seq == kUnassignedSeq || (rseq != kNoneSeq && rseq <= min_seq);
    }

    // ---- per-lane pieces of a segment
    template <class O>
    __device__ __forceinline__ void str(O &w, const uint32_t *tab, uint32_t i) {
        if (w.o) w.bytes(P.strs + tab[2 * i], tab[2 * i + 1]);
        else w.n += tab[2 * i + 1];
    }
    template <class O>
    __device__ __forceinline__ void entry(O &w, uint32_t id, uint32_t e, bool &first) {
        const uint32_t k = pool[id + 2 + 2 * e], v = pool[id + 3 + 2 * e];
        if (!first) w.put(',');
        first = false;
        str(w, P.key_str, k < (uint32_t)P.n_keys ? k : (uint32_t)P.n_keys);
        w.put(':');
        str(w, P.val_str, v < (uint32_t)P.n_values ? v : 0u);
    }
    // JSON.stringify(properties): array-index keys ascending, then insertion order
    template <class O>
    __device__ __forceinline__ void props_json(O &w, uint32_t id) {
        const uint32_t n = pool[id];
        w.put('{');
        bool first = true;
#ifdef MT_SNAP_PROF_NOPROPS  // timing experiment only: the props bytes are sized, not written
        if (true) {
            uint8_t *o_ = w.o;
            w.o = nullptr;
            for (uint32_t e = 0; e < n; e++) entry(w, id, e, first);
            w.put('}');
            w.o = o_;
            return;
        }
#endif
        if (!w.o) {  // the size does not depend on the order
            for (uint32_t e = 0; e < n; e++) entry(w, id, e, first);
            w.put('}');
            return;
        }
        bool any = false;
        for (uint32_t e = 0; e < n && !any; e++) any = key_rank(pool[id + 2 + 2 * e]) != kNoRank;
        if (any) {
            int64_t last = -1;
            for (;;) {
                uint32_t best = kNoRank, be = 0;
                for (uint32_t e = 0; e < n; e++) {
                    const uint32_t r = key_rank(pool[id + 2 + 2 * e]);
                    if (r != kNoRank && (int64_t)r > last && r < best) {
                        best = r;
                        be = e;
                    }
                }
                if (best == kNoRank) break;
                entry(w, id, be, first);
                last = best;
            }
        }
        for (uint32_t e = 0; e < n; e++)
            if (key_rank(pool[id + 2 + 2 * e]) == kNoRank) entry(w, id, e, first);
        w.put('}');
    }
    template <class O>
    __device__ __forceinline__ void marker(O &w, uint32_t ref, uint32_t props) {
        w.lit("{\"marker\":{\"refType\":");
        w.num((int32_t)ref);
        w.put('}');
        if (props) {
            w.lit(",\"props\":");
            props_json(w, props);
        }
        w.put('}');
    }
    template <class O>
    __device__ __forceinline__ void client(O &w, uint32_t id) {
        str(w, P.cli_str, id < (uint32_t)cli_n ? (uint32_t)cli_first + id : id == MT_CLIENT_NONCOLLAB ? 1u : 0u);
    }
    // a segment's JSON around its text: `pre` bytes, the text (tb bytes: text_pass), `post` bytes
    // (a marker: all `pre`, then a standalone one's seq / client fields in `post`).  o: the
    // segment's first byte in the writing pass, null when sizing.
    __device__ __forceinline__ void frame(uint32_t kind, int32_t first, uint32_t props, uint32_t ref, uint8_t *o,
                                          uint32_t tb, uint32_t &pre, uint32_t &post) {
        int32_t seq = 0, rseq = kNoneSeq;
        uint32_t meta = 0;
        const bool alone = kind == kSegAlone;
        if (alone) {
            const uint4 a = reinterpret_cast<const uint4 *>(rec + first)[0];
            const uint4 b = reinterpret_cast<const uint4 *>(rec + first)[1];
            seq = (int32_t)a.y;
            rseq = (int32_t)a.z;
            meta = a.w;
            props = b.y;
            ref = b.z;
        }
        const bool txt = kind == kSegRun || (alone && !(meta & kMetaMarker));
        LOut w{o, 0};
        if (alone) w.lit("{\"json\":");
        if (txt) {
            if (props) w.lit("{\"text\":");
            w.put('"');
            pre = w.n;
            w = LOut{o ? o + pre + tb : nullptr, 0};  // after the text
            w.put('"');
        } else {
            w.lit("{\"marker\":{\"refType\":");
            w.num((int32_t)ref);
            w.put('}');
        }
        if (props) {
            w.lit(",\"props\":");
            props_json(w, props);
        }
        if (!txt || props) w.put('}');
        if (!txt) {
            pre = w.n;
            w = LOut{o ? o + pre : nullptr, 0};
        }
        if (alone) {
            if (seq > min_seq) {
                w.lit(",\"seq\":");
                w.num(seq);
                w.lit(",\"client\":");
                client(w, meta_cli(meta));
            }
            if (rseq != kNoneSeq) {
                w.lit(",\"removedSeq\":");
                w.num(rseq);
                w.lit(",\"removedClient\":");
                client(w, meta_rcli(meta));
            }
            w.put('}');
        }
        post = w.n;
    }

    // The text of the batch's records R0..R1, one 64-record sub-tile at a time, 64 code units per
    // step across the wave (unit u of the sub-tile's concatenated texts: its record by a search of
    // the records' unit offsets).  Sizing adds every record's escaped bytes to its segment
    // (s_seg[j]); writing gives every record, in order, its segment's next text byte (s_seg[j]) and
    // stores each unit there plus the bytes before it in the record.  Surrogate pairs are joined
    // within a record; walk() sends a document whose run joins one across records to the host.
    __device__ __forceinline__ void text_pass(int32_t R0, int32_t R1, bool kW) {
        for (int32_t base = R0; base <= R1; base += 64) {
            const int32_t i = base + (int32_t)lane();
            uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, kOutBlockEnd);
            if (i <= R1) {
                a = reinterpret_cast<const uint4 *>(rec + i)[0];
                b = reinterpret_cast<const uint4 *>(rec + i)[1];
            }
            int j = 0;  // the batch segment holding record i: the last j with sf_j <= i
            for (int st = 32; st > 0; st >>= 1) {
                const int c = j + st;
                const int32_t f = __shfl(sf, c < 64 ? c : 63, 64);
                if (c < nseg && f <= i) j = c;
            }
            const uint32_t kj = (uint32_t)__shfl((int)sk, j, 64);
            const bool has = i <= R1 && !skipped(b.w, (int32_t)a.y, (int32_t)a.z) && !(a.w & kMetaMarker) &&
                             kj != kSegMarker;
            const uint32_t L = has ? a.x : 0u, toff = b.z;
            uint32_t tot;
            const uint32_t ex = wave_excl_scan(L, &tot);
            // the writing kernel takes the records' escaped bytes from the sizing kernel
            const bool stored = kWrite && rb != nullptr;
            if (!stored) {
                s_rt[lane()] = 0u;
                __syncthreads();
            }
#pragma nounroll
            for (int pass = 0; pass < (kW ? 2 : 1); pass++) {
                uint32_t G = 0;
                if (!(pass == 0 && stored)) {
                // two 64-unit windows per step (their text loads in flight together); the units'
                // neighbours come from the adjacent lanes / window (a record's units are
                // consecutive), only the step's last lane loads its right neighbour
                uint32_t cprev = 0;  // the previous step's last unit
#ifdef MT_SNAP_PROF_TEXT
                const uint64_t tw_ = __builtin_readcyclecounter();
#endif
                for (uint32_t s0 = 0; s0 < tot; s0 += 128) {
                    int r[2];
                    uint32_t k[2], rt[2], rn[2], c[2];
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        const uint32_t w0 = s0 + 64u * (uint32_t)q, u = w0 + lane();
                        // the record of unit u (the last r with ex_r <= u): a scalar pass over the few
                        // records overlapping the window, else a binary search
                        const uint64_t ovM = __ballot(L > 0u && ex < w0 + 64u && ex + L > w0);
                        int rq = 0;
                        uint32_t er = 0, tq = 0, lq = 0;
                        if (__popcll(ovM) <= 8) {
                            for (uint64_t m = ovM; m; m &= m - 1) {
                                const uint32_t x = (uint32_t)__builtin_ctzll(m), ex_x = rl(ex, x);
                                const uint32_t t_x = rl(toff, x), l_x = rl(L, x);
                                if (u >= ex_x) {
                                    rq = (int)x;
                                    er = ex_x;
                                    tq = t_x;
                                    lq = l_x;
                                }
                            }
                        } else {
                            for (int st = 32; st > 0; st >>= 1) {
                                const int cc = rq + st;
                                const uint32_t e = (uint32_t)__shfl((int)ex, cc < 64 ? cc : 63, 64);
                                if (cc < 64 && e <= u) rq = cc;
                            }
                            er = (uint32_t)__shfl((int)ex, rq, 64);
                            tq = (uint32_t)__shfl((int)toff, rq, 64);
                            lq = (uint32_t)__shfl((int)L, rq, 64);
                        }
                        r[q] = rq;
                        k[q] = u - er;
                        rt[q] = tq;
                        rn[q] = lq;
                        c[q] = u < tot ? (uint32_t)text[tq + u - er] : 0u;
                    }
                    const uint32_t u1 = s0 + 64u + lane();
                    uint32_t nxe = 0;
                    if (lane() == 63 && u1 < tot && k[1] + 1 < rn[1]) nxe = text[rt[1] + k[1] + 1];
                    const uint32_t c0_63 = rl(c[0], 63), c1_0 = rl(c[1], 0);
                    uint32_t p[2], nx[2], nb[2];
                    p[0] = from_prev_lane(c[0]);
                    p[1] = from_prev_lane(c[1]);
                    nx[0] = from_next_lane(c[0]);
                    nx[1] = from_next_lane(c[1]);
                    if (lane() == 0) {
                        p[0] = cprev;
                        p[1] = c0_63;
                    }
                    if (lane() == 63) {
                        nx[0] = c1_0;
                        nx[1] = nxe;
                    }
                    cprev = rl(c[1], 63);
#pragma unroll
                    for (int q = 0; q < 2; q++) {
                        const uint32_t u = s0 + 64u * (uint32_t)q + lane();
                        nb[q] = 0;
                        if (u < tot) {
                            if (k[q] == 0) p[q] = 0;
                            if (k[q] + 1 >= rn[q]) nx[q] = 0;
                            nb[q] = unit_bytes(c[q], p[q], nx[q]);
                        }
                    }
                    if (pass == 0) {
#pragma unroll
                        for (int q = 0; q < 2; q++)
                            if (s0 + 64u * (uint32_t)q + lane() < tot) atomicAdd(&s_rt[r[q]], nb[q]);
                    } else {
#pragma unroll
                        for (int q = 0; q < 2; q++) {
                            uint32_t st;
                            const uint32_t e = wave_excl_scan(nb[q], &st);
                            if (nb[q]) unit_write(W.dst + s_ro[r[q]] + (G + e - s_rx[r[q]]), nb[q], c[q], nx[q]);
                            G += st;
                        }
                    }
                }
#ifdef MT_SNAP_PROF_TEXT
                pf[4] += __builtin_readcyclecounter() - tw_;
#endif
                }
                __syncthreads();
                if (pass == 0) {
                    const uint32_t myrt = stored ? (i <= R1 ? rb[i] : 0u) : s_rt[lane()];
                    if (!kWrite && rb && i <= R1) rb[i] = myrt;
                    if (!kW) {
                        if (has) atomicAdd(&s_seg[j], myrt);
                    } else {
                        // record offsets: each record takes its segment's next text byte (the
                        // cursors lane-distributed: lane j holds segment j's); a segment's records
                        // are consecutive lanes, so a record's offset is the cursor plus the bytes of
                        // the segment's records before it in the sub-tile (an exclusive scan), and
                        // the segment's last record in the sub-tile advances the cursor
                        const bool inr = i <= R1;
                        const uint32_t v = inr ? myrt : 0u;
                        uint32_t xt;
                        const uint32_t X = wave_excl_scan(v, &xt);
                        const int jp = __shfl_up(j, 1, 64), jn = __shfl_down(j, 1, 64);
                        const bool inr_n = __shfl_down((int)inr, 1, 64) != 0;
                        const uint64_t sM = __ballot(inr && (lane() == 0 || jp != j));
                        const int fl = 63 - __builtin_clzll(sM & ((2ull << lane()) - 1ull) | 1ull);
                        const uint32_t Xf = (uint32_t)__shfl((int)X, fl, 64);
                        const uint32_t cj = (uint32_t)__shfl((int)s_seg[lane()], j, 64);
                        const uint32_t ro = cj + X - Xf;
                        __syncthreads();
                        if (inr && (lane() == 63 || jn != j || !inr_n)) s_seg[j] = ro + v;
                        s_ro[lane()] = ro;
                        s_rx[lane()] = X;
                    }
                    __syncthreads();
                }
            }
        }
    }

    // matchProperties(a, c) by one lane: 1, 0, or -1 (undecided: the document goes to the host)
    __device__ __forceinline__ int props_match_lane(uint32_t a, uint32_t c) const {
        if (!a || !c) return a == c;
        const uint32_t ha = pool[a + 1], hc = pool[c + 1];
        if ((ha | hc) & kSetNever) return 0;
        if (a == c) return 1;
        const uint32_t na = pool[a], nc = pool[c];
        if (na != nc) return 0;
        if ((ha & hc & kSetRegular) && ha != hc) return 0;
        if (na <= 8) {  // both sets' pairs loaded at once, compared in registers
            uint32_t ka[8], va[8], kc[8], vc[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const bool in = (uint32_t)q < na;
                ka[q] = in ? pool[a + 2 + 2 * q] : 0u;
                va[q] = in ? pool[a + 3 + 2 * q] : 0u;
                kc[q] = in ? pool[c + 2 + 2 * q] : 0u;
                vc[q] = in ? pool[c + 3 + 2 * q] : 0u;
            }
            int res = 1;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                if ((uint32_t)q >= na || res != 1) continue;
                uint32_t vb = 0xFFFFFFFFu;
                bool found = false;
#pragma unroll
                for (int r = 0; r < 8; r++)
                    if ((uint32_t)r < nc && kc[r] == ka[q]) {
                        vb = vc[r];
                        found = true;
                    }
                res = found ? value_rel(va[q], vb, P.value_class, P.value_flags, (uint32_t)P.n_values, P.exc, P.n_exc)
                            : 0;
            }
            return res;
        }
        for (uint32_t i = 0; i < na; i++) {
            const uint32_t ka = pool[a + 2 + 2 * i], va = pool[a + 3 + 2 * i];
            int rel = 0;
            for (uint32_t j = 0; j < nc; j++)
                if (pool[c + 2 + 2 * j] == ka)
                    rel = value_rel(va, pool[c + 3 + 2 * j], P.value_class, P.value_flags, (uint32_t)P.n_values, P.exc,
                                    P.n_exc);
            if (rel != 1) return rel;
        }
        return 1;
    }

    // ---- chunks (as Doc)
    template <class Wr>
    __device__ __forceinline__ void header(Wr &w, int64_t count, int64_t length) {
        w.lit("{\"version\":\"1\",\"segmentCount\":");
        w.num(count);
        w.lit(",\"length\":");
        w.num(length);
        w.lit(",\"segments\":[");
    }
    template <class Wr>
    __device__ __forceinline__ void trailer(Wr &w, int32_t c, int64_t start, int32_t n_chunks, int64_t tlen,
                                            int64_t tcount) {
        w.lit("],\"startIndex\":");
        w.num(start);
        if (c == 0) {
            w.lit(",\"headerMetadata\":{\"minSequenceNumber\":");
            w.num(min_seq);
            w.lit(",\"sequenceNumber\":");
            w.num(cur_seq);
            w.lit(",\"orderedChunkMetadata\":[{\"id\":\"header\"}");
            for (int32_t bi = 1; bi < n_chunks; bi++) {
                w.lit(",{\"id\":\"body_");
                w.num(bi - 1);
                w.lit("\"}");
            }
            w.lit("],\"totalLength\":");
            w.num(tlen);
            w.lit(",\"totalSegmentCount\":");
            w.num(tcount);
            w.byte('}');
        }
        w.byte('}');
    }
    __device__ __forceinline__ void open_chunk() {
        open = true;
        ccount = clen = 0;
        if (kWrite) header(W, cm(nch)[0], cm(nch)[1]);
        seg_bytes_at_open = W.pos;
    }
    __device__ __forceinline__ void close_chunk() {
        if (nch >= max_ch) {
            overflow = true;
        } else if (kWrite) {
            trailer(W, nch, total_count, mrow[0], all_len, all_count);
        } else if (lane() == 0) {
            int32_t *t = cm(nch);
            t[0] = (int32_t)ccount;
            t[1] = (int32_t)clen;
            t[2] = (int32_t)(W.pos - seg_bytes_at_open);
        }
        total_count += ccount;
        total_len += clen;
        nch++;
        open = false;
    }

    // ---- stage 2: place and write the queued segments
    __device__ __forceinline__ void flush() {
        if (nseg == 0 || overflow) return;
        const bool mine = (int32_t)lane() < nseg;
        const int32_t R0 = (int32_t)rl((uint32_t)sf, 0u), R1 = (int32_t)rl((uint32_t)sl, (uint32_t)(nseg - 1));
        uint32_t pre = 0, post = 0, tb = 0;
        int64_t my_off = 0;
        // sizing, then (writing pass) the framing and the text at the placed offsets
#pragma nounroll
        for (int wr = 0; wr < (kWrite ? 2 : 1) && !overflow; wr++) {
            {
                SNAP_T0();
                if (mine) {
                    if (kWrite && !wr && sfr) {  // the sizing kernel's framing sizes
                        pre = sfr[2 * sf];
                        post = sfr[2 * sf + 1];
                    } else {
                        frame(sk, sf, sp, sr, wr ? W.dst + my_off : nullptr, tb, pre, post);
                        if (!kWrite && sfr) {
                            sfr[2 * sf] = pre;
                            sfr[2 * sf + 1] = post;
                        }
                    }
                }
                __syncthreads();
                SNAP_ADD(2);
            }
            s_seg[lane()] = wr && mine ? (uint32_t)(my_off + pre) : 0u;
            __syncthreads();
            {
                SNAP_T0();
                text_pass(R0, R1, wr != 0);
                SNAP_ADD(3);
            }
            if (wr) break;
            tb = mine ? s_seg[lane()] : 0u;
            const uint32_t size = pre + tb + post;
#ifndef MT_SNAP_PROF_TEXT
            SNAP_T0();
#endif
            // a batch that closes no chunk (the open chunk stays below chunk_size): every segment
            // follows a comma, its offset an exclusive scan of the sizes
            uint32_t ltot;
            wave_excl_scan(mine ? sn : 0u, &ltot);
            if (open && clen + (int64_t)ltot < P.chunk_size) {
                uint32_t stot;
                const uint32_t ex = wave_excl_scan(mine ? size + 1u : 0u, &stot);
                my_off = W.pos + ex + 1;
                if (kWrite && mine) W.dst[my_off - 1] = (uint8_t)',';
                W.pos += stot;
                ccount += nseg;
                clen += ltot;
#ifndef MT_SNAP_PROF_TEXT
                SNAP_ADD(4);
#endif
                continue;
            }
            for (int32_t j = 0; j < nseg && !overflow; j++) {
                const uint32_t sz = rl(size, (uint32_t)j), ln = rl(sn, (uint32_t)j);
                if (!open) open_chunk();
                else W.byte(',');
                if ((int32_t)lane() == j) my_off = W.pos;
                W.pos += sz;
                ccount++;
                clen += ln;
                if (clen >= P.chunk_size) close_chunk();
            }
#ifndef MT_SNAP_PROF_TEXT
            SNAP_ADD(4);
#endif
        }
        nseg = 0;
    }
    __device__ __forceinline__ void queue(uint32_t kind, int32_t first, int32_t last, uint32_t props, uint32_t ref,
                                          uint32_t clen_) {
        if ((int32_t)lane() == nseg) {
            sk = kind;
            sf = first;
            sl = last;
            sp = props;
            sr = ref;
            sn = clen_;
        }
        ++nseg;
    }
    __device__ __forceinline__ void push_prev() {
        if (!have_prev) return;
        have_prev = false;
        queue(run_text ? kSegRun : kSegMarker, run_first, run_last, run_props, run_ref, run_text ? run_len : 1u);
    }

    // ---- stage 1, lane-parallel: a tile whose kept settled records are all 1..kGranularity long
    // (canAppend's length rule always holds and every appended record sets the run's ends-NL and
    // high-surrogate state) forms its runs from pairwise flags: a kept record continues the run of
    // the kept record before it (or the open run) when both are settled text, the earlier does not
    // end in '\n' and the properties match; every other kept record starts a segment.  The segments
    // the tile closes are staged in order (the open run first) and join the queue 64 at a time; the
    // tile's last run stays open.  Same segments, in the same order, as the record loop below.
    __device__ __forceinline__ void tile_runs(uint32_t f, uint64_t kept, uint64_t below, bool prev_st, uint32_t len,
                                              uint32_t props, uint32_t toff, int32_t base) {
        const uint32_t L = lane();
        const int pl = below ? 63 - __builtin_clzll(below) : 0;
        const uint32_t fp = (uint32_t)__shfl((int)f, pl, 64);
        const bool pnl = below ? (fp & kFEndsNL) != 0u : run_ends_nl;
        const bool phi = below ? (fp & kFLastHi) != 0u : run_hi;
        const bool cand = (f & (kFSkip | kFSettled | kFText)) == (kFSettled | kFText) && prev_st && !pnl;
        const bool join = cand && (f & kFMatch);
        // matchProperties undecided on the device, or a surrogate pair split across two records of
        // a run (the text pass joins pairs within a record): the host serializes the document
        if (__ballot((cand && (f & kFUndecided)) || (join && phi && (f & kFFirstLo)))) {
            overflow = true;
            return;
        }
        const uint64_t startM = kept & ~__ballot(join);
        const uint32_t klen = (f & kFSkip) ? 0u : len;
        uint32_t ltot;
        const uint32_t lex = wave_excl_scan(klen, &ltot), lin = lex + klen;
        // the kept records before the first start extend the open run (text, by construction)
        const int s0 = startM ? __builtin_ctzll(startM) : 64;
        const uint64_t pre = kept & (s0 < 64 ? (1ull << s0) - 1ull : ~0ull);
        if (pre) {
            const uint32_t lk = 63u - (uint32_t)__builtin_clzll(pre), fk = rl(f, lk);
            run_last = base + (int32_t)lk;
            run_len += rl(lin, lk);
            run_ends_nl = (fk & kFEndsNL) != 0u;
            run_hi = (fk & kFLastHi) != 0u;
        }
        if (!startM) return;
        // per start lane: its segment runs to the next start, its last record the last kept before it
        const uint64_t after = startM & ~((2ull << L) - 1ull);
        const int t = after ? __builtin_ctzll(after) : 64;
        const uint64_t upto = kept & (t < 64 ? (1ull << t) - 1ull : ~0ull);
        const int lk = upto ? 63 - __builtin_clzll(upto) : (int)L;
        const uint32_t rlen = (uint32_t)__shfl((int)lin, lk, 64) - lex;
        const uint32_t flk = (uint32_t)__shfl((int)f, lk, 64);
        const uint32_t sl_ = 63u - (uint32_t)__builtin_clzll(startM);
        const bool last_alone = !(rl(f, sl_) & kFSettled);
        const uint64_t qM = last_alone ? startM : startM & ~(1ull << sl_);
        const int32_t c0 = have_prev ? 1 : 0;
        const int32_t C = c0 + __popcll(qM);
        if (have_prev && L == 0) {
            s_q[0][0] = run_text ? kSegRun : kSegMarker;
            s_q[1][0] = (uint32_t)run_first;
            s_q[2][0] = (uint32_t)run_last;
            s_q[3][0] = run_props;
            s_q[4][0] = run_ref;
            s_q[5][0] = run_text ? run_len : 1u;
        }
        if ((qM >> L) & 1ull) {
            const uint32_t r = (uint32_t)c0 + (uint32_t)__popcll(qM & ((1ull << L) - 1ull));
            const bool alone = !(f & kFSettled), txt = (f & kFText) != 0u;
            s_q[0][r] = alone ? kSegAlone : txt ? kSegRun : kSegMarker;
            s_q[1][r] = (uint32_t)(base + (int32_t)L);
            s_q[2][r] = (uint32_t)(base + (alone ? (int32_t)L : lk));
            s_q[3][r] = props;
            s_q[4][r] = toff;
            s_q[5][r] = alone ? len : txt ? rlen : 1u;
        }
        // the tile's last start: an open run, or (alone) none
        if (last_alone) {
            have_prev = false;
        } else {
            const uint32_t fs = rl(f, sl_), fl = rl(flk, sl_);
            have_prev = true;
            run_text = (fs & kFText) != 0u;
            run_first = base + (int32_t)sl_;
            run_last = base + (int32_t)rl((uint32_t)lk, sl_);
            run_len = run_text ? rl(rlen, sl_) : 0u;
            run_props = rl(props, sl_);
            run_ref = rl(toff, sl_);
            run_ends_nl = (fl & kFEndsNL) != 0u;
            run_hi = (fl & kFLastHi) != 0u;
        }
        __syncthreads();
        for (int32_t taken = 0; taken < C;) {
            const int32_t k = min(C - taken, 64 - nseg);
            if ((int32_t)L >= nseg && (int32_t)L < nseg + k) {
                const int32_t q = taken + (int32_t)L - nseg;
                sk = s_q[0][q];
                sf = (int32_t)s_q[1][q];
                sl = (int32_t)s_q[2][q];
                sp = s_q[3][q];
                sr = s_q[4][q];
                sn = s_q[5][q];
            }
            nseg += k;
            taken += k;
            if (nseg == 64) flush();
            if (overflow) return;
        }
        __syncthreads();
    }

    // ---- stage 1
    __device__ __forceinline__ void walk() {
        for (int32_t base = 0; base < n_out && !overflow; base += 64) {
#ifdef MT_SNAP_PROF
            const uint64_t tt_ = __builtin_readcyclecounter();
#endif
            const int32_t i = base + (int32_t)lane();
            uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, kOutBlockEnd);
            if (i < n_out) {
                a = reinterpret_cast<const uint4 *>(rec + i)[0];
                b = reinterpret_cast<const uint4 *>(rec + i)[1];
            }
            const uint32_t len = a.x, meta = a.w, props = b.y, toff = b.z;
            const int32_t seq = (int32_t)a.y, rseq = (int32_t)a.z;
            const bool skip = skipped(b.w, seq, rseq);
            const bool txt = !(meta & kMetaMarker);
            const bool settled = !skip && seq <= min_seq && rseq == kNoneSeq;
            bool nl = false, flo = false, lhi = false;
            if (settled && txt && len > 0) {
                const uint32_t fc = text[toff], lc = text[toff + len - 1];
                nl = lc == 0x0Au;
                flo = is_lo(fc);
                lhi = is_hi(lc);
            }
            // the previous kept record (this tile, or the previous tile's last)
            const uint64_t kept = __ballot(!skip);
            const uint64_t below = kept & ((1ull << lane()) - 1ull);
            const int p = below ? 63 - __builtin_clzll(below) : 0;
            const uint32_t pprops = (uint32_t)__shfl((int)props, p, 64);
            const bool pst = (bool)__shfl((int)(settled && txt), p, 64);
            const uint32_t prev_props = below ? pprops : carry_props;
            const bool prev_st = below ? pst : carry_st;
            int m = 0;
            if (settled && txt && prev_st) m = props_match_lane(prev_props, props);
            const uint32_t f = (skip ? kFSkip : 0u) | (settled ? kFSettled : 0u) | (txt ? kFText : 0u) |
                               (nl ? kFEndsNL : 0u) | (m == 1 ? kFMatch : 0u) | (m < 0 ? kFUndecided : 0u) |
                               (flo ? kFFirstLo : 0u) | (lhi ? kFLastHi : 0u);
            if (kept) {
                const uint32_t lk = 63u - (uint32_t)__builtin_clzll(kept);
                carry_props = rl(props, lk);
                carry_st = (rl(f, lk) & (kFSettled | kFText)) == (kFSettled | kFText);
            }
            const int32_t hi = min(64, n_out - base);
            const bool last = base + 64 >= n_out;
#ifdef MT_SNAP_PROF
            pf[0] += __builtin_readcyclecounter() - tt_;
            const uint64_t tl_ = __builtin_readcyclecounter();
            const uint64_t fl_ = pf[2] + pf[3] + pf[4];
#endif
#ifndef MT_SNAP_RECORD_LOOP
            if (!__ballot(!skip && settled && (len > kGranularity || (txt && len == 0)))) {
                tile_runs(f, kept, below, prev_st, len, props, toff, base);
                if (last && !overflow) {  // the open run ends the document
                    push_prev();
                    flush();
                }
#ifdef MT_SNAP_PROF
                pf[1] += (__builtin_readcyclecounter() - tl_) - (pf[2] + pf[3] + pf[4] - fl_);
#endif
                if (overflow) return;
                continue;
            }
#endif
            // the records in order; the queue is flushed at one place (each record queues at most
            // two segments), and after the last record the open run is pushed and flushed there too
            bool pushed = false;
            for (int32_t j = 0;;) {
                for (; j < hi && nseg <= 62 && !overflow; j++) {
                    const uint32_t fj = rl(f, (uint32_t)j);
                    if (fj & kFSkip) continue;
                    const uint32_t lj = rl(len, (uint32_t)j), pj = rl(props, (uint32_t)j), tj = rl(toff, (uint32_t)j);
                    const int32_t idx = base + j;
                    if (fj & kFSettled) {
                        if (have_prev) {
                            const bool can = run_text && (fj & kFText) && !run_ends_nl &&
                                             (run_len <= kGranularity || lj <= kGranularity);
                            if (can && (fj & kFUndecided)) {
                                overflow = true;
                                break;
                            }
                            if (can && (fj & kFMatch)) {
                                run_last = idx;
                                run_len += lj;
                                if (lj > 0) {
                                    run_ends_nl = (fj & kFEndsNL) != 0;
                                    // a surrogate pair split across two records of the run: the text
                                    // pass joins pairs within a record only, so the host serializes it
                                    if (run_hi && (fj & kFFirstLo)) {
                                        overflow = true;
                                        break;
                                    }
                                    run_hi = (fj & kFLastHi) != 0;
                                }
                                continue;
                            }
                            push_prev();
                        }
                        have_prev = true;  // set_prev
                        run_text = (fj & kFText) != 0;
                        run_first = run_last = idx;
                        run_len = run_text ? lj : 0u;
                        run_props = pj;
                        run_ref = tj;
                        run_ends_nl = (fj & kFEndsNL) != 0;
                        run_hi = lj > 0 && (fj & kFLastHi) != 0;
                    } else {
                        push_prev();
                        queue(kSegAlone, idx, idx, pj, tj, lj);
                    }
                }
                if (overflow) return;
                const bool done = j >= hi;
                if (done && last && !pushed && nseg <= 63) {
                    push_prev();
                    pushed = true;
                }
                if (nseg > 62 || (done && last && pushed)) flush();
                if (overflow) return;
                if (done && (!last || pushed)) break;
            }
#ifdef MT_SNAP_PROF
            pf[1] += (__builtin_readcyclecounter() - tl_) - (pf[2] + pf[3] + pf[4] - fl_);
#endif
        }
        if (overflow) return;
        if (n_out <= 0) {
            push_prev();
            flush();
        }
        if (!overflow && (open || nch == 0)) {
            if (!open) open_chunk();
            close_chunk();
        }
    }
};

template <bool kWrite>
__device__ __forceinline__ void snapshot_doc_lanes(const SnapParams &P, int64_t w) {
    const int64_t d = P.doc_list ? P.doc_list[w] : w;
    if (kWrite && P.bytes[d] < 0) return;
    const DocOut o = P.doc_out[w];
    int32_t cf = P.cli_first, cn = P.cli_n;
    if (P.doc_cli) {
        cf = P.doc_cli[2 * d];
        cn = P.doc_cli[2 * d + 1];
    }
    int32_t *mrow = P.meta + d * (int64_t)kSnapMeta;
    LaneDoc<kWrite> D(P, P.out + w * (int64_t)P.out_cap, P.text + P.doc_text_base[d], P.pool + P.doc_pool_base[d], o,
                      cf, cn, kWrite ? P.dst + P.dst_off[d] : nullptr, mrow);
    if (P.rec_bytes) {
        D.rb = P.rec_bytes + w * (int64_t)P.out_cap;
        D.sfr = P.seg_frame + 2 * w * (int64_t)P.out_cap;
    }
    if (P.chunk_ext) {
        D.ext = P.chunk_ext + P.chunk_ext_off[d];
        D.max_ch = kSnapMaxChunks + (int32_t)((P.chunk_ext_off[d + 1] - P.chunk_ext_off[d]) / 3);
    }
    if (kWrite)
        for (int32_t c = 0; c < mrow[0]; c++) {
            D.all_count += D.cm(c)[0];
            D.all_len += D.cm(c)[1];
        }
    D.walk();
#ifdef MT_SNAP_PROF
    if (lane() == 0)
        for (int k = 0; k < 5; k++) mrow[kSnapMeta - (kWrite ? 10 : 5) + k] = (int32_t)(D.pf[k] >> 6);
#endif
    if (kWrite) return;
    int64_t total = 0;
    if (!D.overflow) {
        Writer<false> f{nullptr, 0};
        int64_t start = 0;
        for (int32_t c = 0; c < D.nch; c++) {
            int32_t *t = D.cm(c);
            const int64_t cnt = t[0], len = t[1];
            f.pos = t[2];
            D.header(f, cnt, len);
            D.trailer(f, c, start, D.nch, D.total_len, D.total_count);
            if (lane() == 0) t[2] = (int32_t)f.pos;
            total += f.pos;
            start += cnt;
        }
    }
    if (lane() == 0) {
        mrow[0] = D.overflow ? 0 : D.nch;
        P.bytes[d] = D.overflow ? -1 : total;
    }
}

}  // namespace

// the serial walker (one record at a time across the wave): kept for A/B (MT_SNAP_SERIAL=1)
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void mt_snapshot_serial_kernel(SnapParams P) {
    const int64_t w = blockIdx.x;
    if (w >= P.n || !P.final_mask[w]) return;
    if (P.pass) snapshot_doc<true>(P, w);
    else snapshot_doc<false>(P, w);
}

// pass 0 (sizes) and pass 1 (writes): separate kernels, each with its own register budget
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void mt_snapshot_size_kernel(SnapParams P) {
    const int64_t w = blockIdx.x;
    if (w >= P.n || !P.final_mask[w]) return;
    snapshot_doc_lanes<false>(P, w);
}
#ifndef MT_SNAP_WRITE_WPE
#define MT_SNAP_WRITE_WPE 4
#endif
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MT_SNAP_WRITE_WPE))) void mt_snapshot_kernel(SnapParams P) {
    const int64_t w = blockIdx.x;
    if (w >= P.n || !P.final_mask[w]) return;
    snapshot_doc_lanes<true>(P, w);
}

}  // namespace mt
