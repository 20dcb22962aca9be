// mt_json_gpu.hip — GPU JSON op-log ingest (the GPU half).
//
// Real op logs are JSON: one array of ISequencedDocumentMessage per document (the file driver's
// messages.json, fileDeltaStorageService.ts:23-31; each message goes to Client.applyMsg,
// client.ts:797-819).  mt_json.cpp parses them on host threads; this file does the same on the
// GPU for the observer fast path (mt_json_gpu.h) and produces the identical packed records
// (mt_oplog.h), text and interned key / value / client tables — or reports the first document
// that needs the host parser.  Stages (one wavefront per document unless noted):
//
//   scan     64 bytes per step: backslash runs -> unescaped quotes -> in-string mask (prefix
//            xor of the quote ballot), brackets outside strings -> depth; depth-1 '{' are the
//            message starts; the top level is validated (one '[' ... ']', exactly one ','
//            between messages, nothing else outside them)
//   count    one lane per message: a validating recursive-descent parse of the message
//            (Packer1::run's rules) -> records / code units / prop records; wave prefix sums
//            give each message its offsets in the document
//   clients  getOrAddShortClientId (client.ts:636-641): the observer is 0, every other long id
//            gets the next id at its first message; first appearance = the smallest message
//            index holding the name (hash table per document, CAS + atomicMin), ids = prefix
//            count of first appearances
//   write    the same parse again, writing records, UTF-16 text and the raw spans of prop keys
//            / values
//   props    the same first-appearance interning for keys and values per document; the host
//            merges the per-document tables batch-wide in document order (as mt_pack_json
//            does) and a remap pass writes the final ids
//
// Text layout: packed (payload = batch-global code-unit offset, mt_pack_json's format) or
// install (the replay's per-document arena, payload document-relative with the '\n' flags that
// mt_batch_ingest sets), so a parsed batch goes to the replay without a host round trip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <unordered_map>

#include "../../include/mtreplay.h"
#include "mt_json_gpu.h"

namespace mt {
namespace jg {

constexpr uint32_t kNullSpan = 0xFFFFFFFFu;
// on a prop value's span length: the source text is valid JSON but not in JSON.stringify form (a
// float, an object, a nested array, whitespace, other string escapes); the host interns
// JSON.stringify(JSON.parse(text)) for it (mt::json_canonical_value), so the tables stay the host
// parser's and only the few unique values per document are formatted on the CPU
constexpr uint32_t kSpanCanon = 0x80000000u;
constexpr uint32_t kIdKeyUnsupported = 0xFFFFFFFFu;  // mt_device.h: a RELPOS key the host cannot resolve
constexpr int kMaxProps = 16;      // keys per props object on the fast path

// reasons a document leaves the fast path (Result::fail_bits)
enum : uint32_t {
    kFSyntax = 1,   // not JSON the host parser accepts as is (it decides: maybe an error)
    kFShape = 2,    // a message / op shape outside the fast path (markers, escapes, floats ...)
    kFRange = 4,    // an integer outside int32
    kFWriter = 8,   // a writer replica's message outside the fast path (regenerate, notifyConsensus,
                    // an ack with relative positions, a local op of another client ...)
    kFClients = 16, // more than 32765 clients
    kFCap = 32      // more messages than the scan's per-document region holds
};

// message flags: an op message; a local (unsequenced) one; one with a RELPOS record
enum : uint32_t { kMsgOp = 1, kMsgLocal = 2, kMsgRel = 4 };

struct Params {
    const uint8_t *J;
    const int64_t *doc_off;
    int64_t D;
    // per message (region of document d starts at doc_off[d] / 64 + 2 d)
    uint32_t *m_start, *m_flags, *m_nrec, *m_ntext, *m_nprop, *m_recoff, *m_textoff, *m_propoff;
    uint32_t *m_cloff, *m_cllen, *m_cid, *m_npops, *m_nval, *m_valoff;
    const int32_t *chunk_doc;        // count / write passes: one wave per 64 messages of a document
    const uint32_t *chunk_first;
    // structural scan: one wave per kSegBytes of a document (segment g: doc seg_doc[g], bytes from
    // seg_start[g]); per-document segments seg_first[d] .. seg_first[d + 1]
    const int32_t *seg_doc;
    const uint32_t *seg_start;
    const int64_t *seg_first;
    int64_t G;
    uint32_t *sg_q, *sg_pre, *sg_post, *sg_flags, *sg_nmsg, *sg_fail, *sg_starts;
    int32_t *sg_d0, *sg_d1;
    // per document
    uint32_t *d_nmsg, *d_fail, *d_nrec, *d_ntext, *d_nprop, *d_npropops, *d_nnames, *d_nuk, *d_nuv, *d_nval;
    uint32_t *d_writer;  // per document: a writer replica's log (local ops or acks of its own)
    uint32_t *cl_ht;                 // per document cl_cap[d] slots from cl_base[d] (2 x its names + 1, a power of 2)
    const uint64_t *cl_base;
    const uint32_t *cl_cap;
    const uint64_t *names_base;      // per document: first word of its names in `names`
    uint32_t *nm_off, *nm_len;       // per message region: client id k's span at index k - 1
    uint32_t *names;                 // per document {off, len} of ids 1.. (compacted by jg_names_kernel)
    const uint8_t *obs;              // observer long id (UTF-8) + "null" at obs + 256
    uint32_t obs_len;
    // write
    const int64_t *op_base;          // per document: first record (batch-global)
    const uint64_t *text_dst;        // per document: first code unit of its text in `text`
    const uint32_t *text_pay;        // per document: payload of its first code unit
    const uint32_t *prop_base;       // per document: first prop record (batch-global)
    // value events: every interned value in the host packer's value() order — a relative
    // position's id, then the op's prop values; per document from val_base[d]
    const uint32_t *val_base;
    uint32_t *pe;                    // per prop record: its value event
    mt_op *ops;
    uint16_t *text;
    mt_prop *props;
    int install;
    uint32_t *pk_off, *pk_len, *pv_off, *pv_len;  // raw spans per prop record
    uint32_t *lk, *lv;                            // per-document ids per prop record
    uint32_t *uk_off, *uk_len, *uv_off, *uv_len;  // per-document unique spans (at prop_base)
    uint32_t *ht;                                  // prop hash tables (keys then values)
    const uint64_t *ht_base;                       // per document: its key table; values follow
    const uint32_t *ht_cap;                        // per document: slots per table (power of 2)
    const uint32_t *kmap, *vmap;                   // remap: per-document id -> batch id
};

__device__ __forceinline__ int lane_id() { return (int)threadIdx.x; }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t wave_incl(uint32_t v) {
    const int l = lane_id();
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (l >= o) v += t;
    }
    return v;
}
__device__ __forceinline__ uint64_t mregion(const int64_t *doc_off, int64_t d) {
    return (uint64_t)(doc_off[d] / 64 + 2 * d);
}

// ---------------------------------------------------------------- stage 1: structural scan
// A document is scanned in segments of kSegBytes, one wavefront each, so a batch of few long
// documents still fills the chip (simdjson's two-pass idea on 64-lane ballots):
//   A  per segment, with the in-string state at its start assumed 0: the parity of its unescaped
//      quotes and its net bracket depth for either start state (the in-string mask under the other
//      start state is the complement, so one pass gives both);
//   B  per segment, with the true start state (the XOR of the earlier segments' parities) and the
//      true start depth (their deltas for their start states): the message starts (depth-1 '{')
//      and the checks that need no global state; the commas before its first / after its last
//      message start go to C;
//   C  per document: the checks across segments (one '[', exactly one comma between messages, no
//      trailing comma, nothing after ']') and the message starts gathered in order.
// A quote's escape parity comes from the run of backslashes right before it; a segment reads
// the 64 bytes before its start for the run it begins in.
constexpr uint32_t kSegBytes = 65536;
constexpr uint32_t kSegStarts = kSegBytes / 64 + 2;  // message starts one segment can hold
enum : uint32_t { kSgMsg = 1, kSgEnd = 2, kSgOpenShift = 8 };

// bytes [start, end) of document d in 64-byte chunks, one byte per lane (outside [0, len):
// whitespace); f(pos0, c) per chunk with pos0 = document position of lane 0's byte.  Steps of 1 KB:
// four coalesced 256-byte dword loads in flight, chunk j rebuilt with one shuffle.
template <class F>
__device__ void for_chunks(const Params &P, int64_t d, uint32_t start, uint32_t end, F &&f) {
    const int lane = lane_id();
    const int64_t a = P.doc_off[d];
    const uint64_t abs0 = (uint64_t)a + start;
    const uint32_t shift = (uint32_t)(abs0 & 3);
    const uint32_t *w32 = (const uint32_t *)(P.J + (abs0 - shift));
    const uint32_t span = end - start + shift;
    const uint32_t nwords = (span + 3) >> 2;
    bool stop = false;
    for (uint32_t base = 0; base < span && !stop; base += 1024) {
        uint32_t w[4];
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t wi = (base >> 2) + 64u * (uint32_t)m + (uint32_t)lane;
            w[m] = wi < nwords ? w32[wi] : 0x20202020u;
        }
        for (int j = 0; j < 16 && !stop; j++) {
            const uint32_t pos0 = base + 64u * (uint32_t)j;
            if (pos0 >= span) break;
            const uint32_t word = __shfl(w[j >> 2], 16 * (j & 3) + (lane >> 2), 64);
            const uint32_t at = pos0 + (uint32_t)lane;
            const int c = (at >= shift && at < span) ? (int)((word >> (8 * (lane & 3))) & 0xFFu) : ' ';
            stop = f(start + pos0 - shift, c);  // (wraps below 0 only for lanes that are masked)
        }
    }
}

// the run of backslashes ending right before document position p (up to 63; 64 = "longer")
__device__ uint32_t bs_before(const Params &P, int64_t d, uint32_t p) {
    const int lane = lane_id();
    const int64_t q = (int64_t)p - 64 + lane;
    const int c = q >= 0 ? P.J[P.doc_off[d] + q] : ' ';
    const uint64_t bs = ballot(c == '\\');
    return bs == ~0ull ? 64u : (uint32_t)__builtin_clzll(~bs);
}

// unescaped quotes of a chunk, prefix-XORed: bit i = parity of those at or below i
__device__ __forceinline__ uint64_t quote_prefix(int c, uint32_t bs_run, uint64_t &bs_out) {
    const int lane = lane_id();
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    const uint64_t bs = ballot(c == '\\');
    const uint64_t nb = ~bs & below;
    const uint32_t run = nb ? (uint32_t)(lane - 1 - (63 - __builtin_clzll(nb))) : (uint32_t)lane + bs_run;
    uint64_t x = ballot(c == '"' && !(run & 1u));
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    x ^= x << 16;
    x ^= x << 32;
    bs_out = bs;
    return x;
}

extern "C" __global__ __launch_bounds__(64) void jg_seg_a_kernel(Params P) {
    const int64_t g = blockIdx.x;
    if (g >= P.G) return;
    const int64_t d = P.seg_doc[g];
    const uint32_t len = (uint32_t)(P.doc_off[d + 1] - P.doc_off[d]);
    const uint32_t start = P.seg_start[g], end = min(len, start + kSegBytes);
    uint32_t bs_run = bs_before(P, d, start), fail = bs_run >= 64 ? kFShape : 0u;
    bool in0 = false;
    int32_t d0 = 0, d1 = 0;
    uint32_t q = 0;
    for_chunks(P, d, start, end, [&](uint32_t, int c) {
        uint64_t bs;
        const uint64_t x = quote_prefix(c, bs_run, bs);
        const uint64_t S0 = in0 ? ~x : x;
        q ^= (uint32_t)__builtin_popcountll(x ^ (x << 1)) & 1u;  // unescaped quotes of the chunk
        in0 = (S0 >> 63) & 1ull;
        bs_run = bs == ~0ull ? bs_run + 64u : (uint32_t)__builtin_clzll(~bs);
        const uint64_t opn = ballot(c == '{' || c == '['), cls = ballot(c == '}' || c == ']');
        d0 += __builtin_popcountll(opn & ~S0) - __builtin_popcountll(cls & ~S0);
        d1 += __builtin_popcountll(opn & S0) - __builtin_popcountll(cls & S0);
        return false;
    });
    if (lane_id() == 0) {
        P.sg_q[g] = q;
        P.sg_d0[g] = d0;
        P.sg_d1[g] = d1;
        P.sg_fail[g] = fail;
    }
}

extern "C" __global__ __launch_bounds__(64) void jg_seg_b_kernel(Params P) {
    const int64_t g = blockIdx.x;
    if (g >= P.G) return;
    const int lane = lane_id();
    const int64_t d = P.seg_doc[g];
    const uint32_t len = (uint32_t)(P.doc_off[d + 1] - P.doc_off[d]);
    const uint32_t start = P.seg_start[g], end = min(len, start + kSegBytes);
    // the start state from the earlier segments of the document
    bool in_str = false;
    int32_t depth = 0;
    for (int64_t k = P.seg_first[d]; k < g; k++) {
        depth += in_str ? P.sg_d1[k] : P.sg_d0[k];
        in_str ^= P.sg_q[k] & 1u;
    }
    uint32_t fail = P.sg_fail[g];
    if (depth < 0) fail |= kFSyntax;
    uint32_t bs_run = bs_before(P, d, start);
    uint32_t commas = 0, pre = 0, post = 0, flags = 0, n = 0, opens = 0;
    uint32_t *starts = P.sg_starts + (uint64_t)g * kSegStarts;
    for_chunks(P, d, start, end, [&](uint32_t pos, int c) {
        uint64_t bs;
        const uint64_t x = quote_prefix(c, bs_run, bs);
        const uint64_t S = in_str ? ~x : x;  // 1: inside a string (opening quote included)
        in_str = (S >> 63) & 1ull;
        bs_run = bs == ~0ull ? bs_run + 64u : (uint32_t)__builtin_clzll(~bs);
        const bool ws = c == ' ' || c == '\t' || c == '\n' || c == '\r';
        const uint64_t nonws = ballot(!ws) & ~S;
        const uint64_t opn = ballot(c == '{' || c == '[') & ~S;
        const uint64_t cls = ballot(c == '}' || c == ']') & ~S;
        const uint64_t brace = ballot(c == '{' || c == '}');
        const uint64_t comma = ballot(c == ',') & ~S;
        uint64_t st = opn | cls;
        uint32_t lo = 0;
        // between structural characters one depth: at 0 only whitespace, at 1 whitespace + commas
        auto segment = [&](uint32_t hi) {
            if (hi > lo) {
                const uint64_t m = (hi >= 64 ? ~0ull : ((1ull << hi) - 1ull)) & ~((1ull << lo) - 1ull);
                if (depth == 0 && (nonws & m)) fail |= kFSyntax;
                if (depth == 1) {
                    if (nonws & ~comma & m) fail |= kFSyntax;
                    commas += (uint32_t)__builtin_popcountll(comma & m);
                }
            }
        };
        while (st && !fail) {
            const uint32_t t = (uint32_t)__builtin_ctzll(st);
            st &= st - 1;
            segment(t);
            lo = t + 1;
            const bool o = (opn >> t) & 1ull, br = (brace >> t) & 1ull;
            if (flags & kSgEnd) {
                fail |= kFSyntax;
                break;
            }
            if (o) {
                if (depth == 0) {
                    if (br) fail |= kFSyntax;  // the log is one array
                    opens++;
                } else if (depth == 1) {
                    if (!br) fail |= kFSyntax;  // a message must be an object
                    if (flags & kSgMsg) {
                        if (commas != 1u) fail |= kFSyntax;
                    } else {
                        pre = commas;
                    }
                    commas = 0;
                    if (n >= kSegStarts) fail |= kFCap;
                    else if (lane == 0) starts[n] = pos + t;
                    n++;
                    flags |= kSgMsg;
                }
                depth++;
            } else {
                if (depth <= 0) {
                    fail |= kFSyntax;
                    break;
                }
                depth--;
                if (depth == 0) {
                    if (br) fail |= kFSyntax;
                    if (flags & kSgMsg) {
                        if (commas) fail |= kFSyntax;  // no trailing comma
                    } else {
                        pre = commas;
                    }
                    commas = 0;
                    flags |= kSgEnd;
                }
            }
        }
        if (!fail) segment(64);
        return fail != 0;
    });
    if (flags & kSgMsg) post = commas;
    else if (!(flags & kSgEnd)) pre = commas;
    if (lane == 0) {
        P.sg_pre[g] = pre;
        P.sg_post[g] = post;
        P.sg_flags[g] = flags | (min(opens, 255u) << kSgOpenShift);
        P.sg_nmsg[g] = n;
        P.sg_fail[g] = fail;
    }
}

extern "C" __global__ __launch_bounds__(64) void jg_seg_c_kernel(Params P) {
    const int64_t d = blockIdx.x;
    if (d >= P.D) return;
    const int lane = lane_id();
    const uint64_t mb = mregion(P.doc_off, d);
    const uint32_t mcap = (uint32_t)(mregion(P.doc_off, d + 1) - mb);
    uint32_t fail = 0, cur = 0, nmsg = 0, opens = 0, q = 0;
    bool seen = false, ended = false;
    for (int64_t k = P.seg_first[d]; k < P.seg_first[d + 1]; k++) {
        const uint32_t f = P.sg_flags[k], n = P.sg_nmsg[k];
        fail |= P.sg_fail[k];
        q ^= P.sg_q[k] & 1u;
        opens += f >> kSgOpenShift;
        if (ended && ((f & (kSgMsg | kSgEnd)) || (f >> kSgOpenShift))) fail |= kFSyntax;
        if (f & kSgMsg) {
            if (cur + P.sg_pre[k] != (seen ? 1u : 0u)) fail |= kFSyntax;
            if (nmsg + n > mcap) fail |= kFCap;
            for (uint32_t i = (uint32_t)lane; !fail && i < n; i += 64)
                P.m_start[mb + nmsg + i] = P.sg_starts[(uint64_t)k * kSegStarts + i];
            nmsg += n;
            cur = P.sg_post[k];
            seen = true;
        } else {
            cur += P.sg_pre[k];
        }
        if (f & kSgEnd) {
            if (!(f & kSgMsg) && cur != 0) fail |= kFSyntax;  // "[..., ]" across segments
            ended = true;
        }
        if (fail) break;
    }
    if (opens != 1 || !ended || q) fail |= kFSyntax;
    if (lane == 0) {
        P.d_nmsg[d] = fail ? 0u : nmsg;
        P.d_fail[d] = fail;
    }
}

// ---------------------------------------------------------------- lane-serial JSON reading
// (host-callable too: tests/jg_parse_asan.cpp runs the lane parser on the CPU under
// AddressSanitizer over valid and mutated logs, checking every read and write stays in bounds)
struct Rd {
    // a lane's cursor over one document; bytes come through a 16-byte window (one aligned 128-bit
    // load per 16 bytes instead of a load per byte)
    const uint8_t *s;
    uint32_t p, n;
    uint32_t sh, wb = 0xFFFFFFFFu;
    uint4 w;
    __host__ __device__ Rd(const uint8_t *s_, uint32_t p_, uint32_t n_)
        : s(s_), p(p_), n(n_), sh((uint32_t)((uintptr_t)s_ & 15u)) {}
    __host__ __device__ uint32_t b(uint32_t k) {
        const uint32_t ak = k + sh, blk = ak & ~15u;
        if (blk != wb) {
            wb = blk;
            w = *(const uint4 *)(s - sh + blk);
        }
        const uint32_t o = ak & 15u;
        const uint32_t word = o < 8 ? (o < 4 ? w.x : w.y) : (o < 12 ? w.z : w.w);
        return (word >> ((o & 3u) * 8u)) & 0xFFu;
    }
    __host__ __device__ int at() { return p < n ? (int)b(p) : -1; }
    __host__ __device__ void ws() {
        while (p < n) {
            const uint32_t c = b(p);
            if (c == ' ' || c == '\t' || c == '\n' || c == '\r') p++;
            else break;
        }
    }
    __host__ __device__ bool lit(const char *wd, uint32_t k) {
        if (n - p < k) return false;
        for (uint32_t i = 0; i < k; i++)
            if (b(p + i) != (uint8_t)wd[i]) return false;
        p += k;
        return true;
    }
    // the key / string span [o, o + l) equals the C string wd
    __host__ __device__ bool is(uint32_t o, uint32_t l, const char *wd) {
        uint32_t i = 0;
        for (; wd[i]; i++)
            if (i >= l || b(o + i) != (uint8_t)wd[i]) return false;
        return i == l;
    }
    __host__ __device__ bool eq(uint32_t o1, uint32_t l1, uint32_t o2, uint32_t l2) {
        if (l1 != l2) return false;
        for (uint32_t i = 0; i < l1; i++)
            if (b(o1 + i) != b(o2 + i)) return false;
        return true;
    }
};

__host__ __device__ __forceinline__ bool is_digit(int c) { return c >= '0' && c <= '9'; }
__host__ __device__ __forceinline__ int hexv(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

// a string token: raw span of its contents; plain = no escapes, ASCII only
__host__ __device__ bool str_raw(Rd &r, uint32_t &off, uint32_t &len, bool &plain) {
    if (r.at() != '"') return false;
    r.p++;
    off = r.p;
    plain = true;
    for (;;) {
        if (r.p >= r.n) return false;
        const uint8_t c = r.b(r.p);
        if (c == '"') break;
        if (c < 0x20) return false;
        if (c == '\\') {
            plain = false;
            if (++r.p >= r.n) return false;
            const uint8_t e = r.b(r.p);
            if (e == 'u') {
                if (r.n - r.p < 5) return false;
                for (int i = 1; i <= 4; i++)
                    if (hexv(r.b(r.p + i)) < 0) return false;
                r.p += 4;
            } else if (!(e == '"' || e == '\\' || e == '/' || e == 'b' || e == 'f' || e == 'n' || e == 'r' ||
                         e == 't')) {
                return false;
            }
            r.p++;
            continue;
        }
        if (c >= 0x80) plain = false;
        r.p++;
    }
    len = r.p - off;
    r.p++;
    return true;
}

// the string token whose contents are [o, o + l) is already what JSON.stringify writes for the
// string it decodes to (so its source text can be interned as the value's JSON text): escapes only
// \" \\ \b \f \n \r \t and \u00xx (lowercase) for the other control characters; every other
// character raw, non-ASCII as well-formed shortest UTF-8 outside the surrogates
__host__ __device__ bool str_canonical(Rd &r, uint32_t o, uint32_t l) {
    for (uint32_t i = 0; i < l;) {
        const uint32_t c = r.b(o + i);
        if (c == '\\') {
            if (i + 1 >= l) return false;
            const uint32_t e = r.b(o + i + 1);
            if (e == '"' || e == '\\' || e == 'b' || e == 'f' || e == 'n' || e == 'r' || e == 't') {
                i += 2;
                continue;
            }
            if (e != 'u' || i + 6 > l) return false;
            uint32_t v = 0;
            for (uint32_t k = 2; k < 6; k++) {
                const uint32_t h = r.b(o + i + k);
                const int d = (h >= '0' && h <= '9') ? (int)(h - '0') : (h >= 'a' && h <= 'f') ? (int)(h - 'a' + 10) : -1;
                if (d < 0) return false;  // JSON.stringify writes lowercase hex
                v = v * 16 + (uint32_t)d;
            }
            if (v >= 0x20 || v == 8 || v == 9 || v == 10 || v == 12 || v == 13) return false;
            i += 6;
            continue;
        }
        if (c < 0x80) {
            i++;
            continue;
        }
        // well-formed UTF-8, shortest form, no surrogates
        const uint32_t k = (c & 0xE0) == 0xC0 ? 2u : (c & 0xF0) == 0xE0 ? 3u : (c & 0xF8) == 0xF0 ? 4u : 0u;
        if (!k || i + k > l) return false;
        uint32_t cp = c & (k == 2 ? 0x1Fu : k == 3 ? 0x0Fu : 0x07u);
        for (uint32_t q = 1; q < k; q++) {
            const uint32_t b = r.b(o + i + q);
            if ((b & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (b & 0x3Fu);
        }
        if ((k == 2 && cp < 0x80) || (k == 3 && cp < 0x800) || (k == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
            (cp >= 0xD800 && cp <= 0xDFFF))
            return false;
        i += k;
    }
    return true;
}

// a text string decoded to UTF-16 code units exactly as mt_json.cpp Dom::string (\u escapes
// kept as code units, UTF-8 -> UTF-16 with surrogate pairs); dst may be null (count only)
__host__ __device__ bool str_text(Rd &r, uint16_t *dst, uint32_t &units, bool &has_nl, bool &ends_nl) {
    if (r.at() != '"') return false;
    r.p++;
    units = 0;
    has_nl = ends_nl = false;
    uint32_t last = 0xFFFFFFFFu;
    auto put = [&](uint32_t u) {
        if (dst) dst[units] = (uint16_t)u;
        units++;
        last = u & 0xFFFFu;
        if (last == '\n') has_nl = true;
    };
    for (;;) {
        if (r.p >= r.n) return false;
        const uint8_t c = r.b(r.p);
        if (c == '"') break;
        if (c == '\\') {
            if (++r.p >= r.n) return false;
            const uint8_t e = r.b(r.p);
            switch (e) {
                case '"': put('"'); break;
                case '\\': put('\\'); break;
                case '/': put('/'); break;
                case 'b': put('\b'); break;
                case 'f': put('\f'); break;
                case 'n': put('\n'); break;
                case 'r': put('\r'); break;
                case 't': put('\t'); break;
                case 'u': {
                    if (r.n - r.p < 5) return false;
                    uint32_t v = 0;
                    for (int i = 1; i <= 4; i++) {
                        const int h = hexv(r.b(r.p + i));
                        if (h < 0) return false;
                        v = v * 16 + (uint32_t)h;
                    }
                    put(v);
                    r.p += 4;
                    break;
                }
                default: return false;
            }
            r.p++;
        } else if (c < 0x20) {
            return false;
        } else if (c < 0x80) {
            put(c);
            r.p++;
        } else {
            const int k = (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : (c & 0xF8) == 0xF0 ? 4 : 0;
            if (!k || r.n - r.p < (uint32_t)k) return false;
            uint32_t cp = c & (k == 2 ? 0x1Fu : k == 3 ? 0x0Fu : 0x07u);
            for (int i = 1; i < k; i++) {
                const uint8_t b = r.b(r.p + i);
                if ((b & 0xC0) != 0x80) return false;
                cp = (cp << 6) | (b & 0x3Fu);
            }
            r.p += (uint32_t)k;
            if (cp >= 0x10000) {
                cp -= 0x10000;
                put(0xD800u + (cp >> 10));
                put(0xDC00u + (cp & 0x3FFu));
            } else {
                put(cp);
            }
        }
    }
    r.p++;
    ends_nl = last == '\n';
    return true;
}

// a number token: 1 = canonical integer (no fraction / exponent, <= 18 digits) in v,
// 2 = another JSON number, 0 = not one the fast path reads like the host (strtod) would
__host__ __device__ int num_tok(Rd &r, int64_t &v, uint32_t &ndig) {
    uint32_t p = r.p;
    bool neg = false;
    if (p < r.n && r.b(p) == '-') {
        neg = true;
        p++;
    }
    if (p >= r.n || !is_digit(r.b(p))) return 0;
    bool canon = true;
    int64_t acc = 0;
    ndig = 0;
    if (r.b(p) == '0') {
        p++;
        ndig = 1;
        if (p < r.n && is_digit(r.b(p))) return 0;
    } else {
        while (p < r.n && is_digit(r.b(p))) {
            if (ndig < 18) acc = acc * 10 + (r.b(p) - '0');
            ndig++;
            p++;
        }
    }
    if (p < r.n && r.b(p) == '.') {
        canon = false;
        p++;
        if (p >= r.n || !is_digit(r.b(p))) return 0;
        while (p < r.n && is_digit(r.b(p))) p++;
    }
    if (p < r.n && (r.b(p) == 'e' || r.b(p) == 'E')) {
        canon = false;
        p++;
        if (p < r.n && (r.b(p) == '+' || r.b(p) == '-')) p++;
        if (p >= r.n || !is_digit(r.b(p))) return 0;
        while (p < r.n && is_digit(r.b(p))) p++;
    }
    if (p < r.n) {  // the host's number scan is greedy over [0-9.eE+-]
        const uint8_t c = r.b(p);
        if (is_digit(c) || c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-') return 0;
    }
    if (neg && ndig == 1 && acc == 0 && canon) canon = false;  // -0
    r.p = p;
    v = neg ? -acc : acc;
    if (ndig > 18) canon = false;
    return canon ? 1 : 2;
}

// any JSON value, validated (strings, numbers, literals, nesting up to 64 levels)
__host__ __device__ bool skip_value(Rd &r) {
    uint64_t stack = 0;  // bit k: container k is an object
    int sd = 0;
    bool want_key = false;
    for (;;) {
        r.ws();
        if (want_key) {
            uint32_t o, l;
            bool pl;
            if (!str_raw(r, o, l, pl)) return false;
            r.ws();
            if (r.at() != ':') return false;
            r.p++;
            r.ws();
            want_key = false;
        }
        const int c = r.at();
        bool done_value = true;
        if (c == '{' || c == '[') {
            r.p++;
            r.ws();
            if (r.at() == (c == '{' ? '}' : ']')) {
                r.p++;
            } else {
                if (sd >= 63) return false;
                stack = (stack << 1) | (c == '{' ? 1ull : 0ull);
                sd++;
                want_key = c == '{';
                done_value = false;
            }
        } else if (c == '"') {
            uint32_t o, l;
            bool pl;
            if (!str_raw(r, o, l, pl)) return false;
        } else if (c == 't') {
            if (!r.lit("true", 4)) return false;
        } else if (c == 'f') {
            if (!r.lit("false", 5)) return false;
        } else if (c == 'n') {
            if (!r.lit("null", 4)) return false;
        } else {
            int64_t v;
            uint32_t nd;
            if (!num_tok(r, v, nd)) return false;
        }
        if (!done_value) continue;
        // after a value: close containers / next element
        for (;;) {
            if (sd == 0) return true;
            r.ws();
            const bool obj = stack & 1ull;
            const int e = r.at();
            if (e == ',') {
                r.p++;
                want_key = obj;
                break;
            }
            if (e == (obj ? '}' : ']')) {
                r.p++;
                stack >>= 1;
                sd--;
                continue;
            }
            return false;
        }
    }
}

__host__ __device__ __forceinline__ bool span_eq(const uint8_t *a, uint32_t la, const uint8_t *b, uint32_t lb) {
    if (la != lb) return false;
    for (uint32_t i = 0; i < la; i++)
        if (a[i] != b[i]) return false;
    return true;
}
__device__ __forceinline__ uint32_t fnv32(const uint8_t *p, uint32_t n) {
    uint32_t h = 2166136261u;
    for (uint32_t i = 0; i < n; i++) h = (h ^ p[i]) * 16777619u;
    return h ^ (h >> 15);
}

// ---------------------------------------------------------------- per-message parse
struct MsgOut {
    uint32_t nrec = 0, ntext = 0, nprop = 0, npropops = 0, nval = 0;
    uint32_t cl_off = kNullSpan, cl_len = 4, flags = 0;
};

struct Ctx {  // write pass
    mt_op *ops = nullptr;       // this message's first record
    uint16_t *text = nullptr;   // this message's first code unit
    uint32_t pay = 0;           // payload of that code unit
    uint32_t gprop = 0;         // batch-global index of this message's first prop record
    uint32_t gval = 0;          // batch-global index of this message's first value event
    uint32_t *pk_off, *pk_len, *pv_off, *pv_len, *pe;  // keys per prop record, values per event
    uint16_t cid = 0;
    bool install = false;
};

struct OpInfo {
    int64_t type = -1;
    int32_t p1 = 0, p2 = 0;
    uint32_t seg_p = 0, props_p = 0, ops_p = 0, rel1_p = 0, rel2_p = 0;
    uint32_t seen = 0;
    bool rewrite = false;
};
enum { kOType = 1, kOPos1 = 2, kOPos2 = 4, kOSeg = 8, kOProps = 16, kOOps = 32, kORel1 = 64, kORel2 = 128 };

// an op object's members (pack_op / flatten / relpos / register rules, mt_json.cpp:596-649)
__host__ __device__ uint32_t parse_op(Rd &r, OpInfo &op) {
    if (r.at() != '{') return kFShape;
    r.p++;
    r.ws();
    if (r.at() == '}') {
        r.p++;
        return 0;
    }
    uint32_t extra = 0;
    for (;;) {
        r.ws();
        uint32_t ko, kl;
        bool plain;
        if (!str_raw(r, ko, kl, plain)) return kFSyntax;
        if (!plain) return kFShape;
        r.ws();
        if (r.at() != ':') return kFSyntax;
        r.p++;
        r.ws();
        uint32_t bit = 0;
        if (r.is(ko, kl, "type")) bit = kOType;
        else if (r.is(ko, kl, "pos1")) bit = kOPos1;
        else if (r.is(ko, kl, "pos2")) bit = kOPos2;
        else if (r.is(ko, kl, "seg")) bit = kOSeg;
        else if (r.is(ko, kl, "props")) bit = kOProps;
        else if (r.is(ko, kl, "ops")) bit = kOOps;
        else if (r.is(ko, kl, "relativePos1")) bit = kORel1;
        else if (r.is(ko, kl, "relativePos2")) bit = kORel2;
        if (bit) {
            if (op.seen & bit) return kFShape;  // a repeated key: the host keeps the last value
            op.seen |= bit;
        }
        if (bit == kOType || bit == kOPos1 || bit == kOPos2) {
            int64_t v;
            uint32_t nd;
            const int t = num_tok(r, v, nd);
            if (t != 1) return t ? kFShape : kFSyntax;
            if (v < -2147483648ll || v > 2147483647ll) return kFRange;
            if (bit == kOType) op.type = v;
            else if (bit == kOPos1) op.p1 = (int32_t)v;
            else op.p2 = (int32_t)v;
        } else {
            if (bit == kOSeg) op.seg_p = r.p;
            if (bit == kOProps) op.props_p = r.p;
            if (bit == kOOps) op.ops_p = r.p;
            if (bit == kORel1) op.rel1_p = r.p;
            if (bit == kORel2) op.rel2_p = r.p;
            if (!bit) {
                // combiningOp (a falsy one is ignored), register (null is absent): anything else
                // and relative positions leave the fast path
                const bool cop = r.is(ko, kl, "combiningOp"), reg = r.is(ko, kl, "register");
                if (cop || reg) {
                    if (extra & (cop ? 1u : 2u)) return kFShape;
                    extra |= cop ? 1u : 2u;
                    if (r.lit("null", 4) || (cop && r.lit("false", 5))) goto next;
                    if (cop && r.at() == '{') {
                        // {name: "rewrite"} (segmentPropertiesManager.ts:53-54): a flag; any other
                        // combiningOp carries defaultValue / minValue records: the host path
                        r.p++;
                        r.ws();
                        bool named = false;
                        if (r.at() != '}') {
                            for (;;) {
                                r.ws();
                                uint32_t no, nl;
                                bool pl;
                                if (!str_raw(r, no, nl, pl)) return kFSyntax;
                                if (!pl) return kFShape;
                                r.ws();
                                if (r.at() != ':') return kFSyntax;
                                r.p++;
                                r.ws();
                                if (r.is(no, nl, "name")) {
                                    uint32_t vo, vl;
                                    bool vp;
                                    if (named || r.at() != '"' || !str_raw(r, vo, vl, vp) || !vp ||
                                        !r.is(vo, vl, "rewrite"))
                                        return kFShape;
                                    named = true;
                                } else if (!skip_value(r)) {
                                    return kFSyntax;
                                }
                                r.ws();
                                if (r.at() == ',') {
                                    r.p++;
                                    continue;
                                }
                                if (r.at() == '}') break;
                                return kFSyntax;
                            }
                        }
                        r.p++;
                        if (!named) return kFShape;  // a truthy combiningOp without a name: "other"
                        op.rewrite = true;
                        goto next;
                    }
                    return kFShape;
                }
            }
            if (!skip_value(r)) return kFSyntax;
        }
    next:
        r.ws();
        const int c = r.at();
        if (c == ',') {
            r.p++;
            continue;
        }
        if (c == '}') {
            r.p++;
            return 0;
        }
        return kFSyntax;
    }
}

// a flat props object -> prop records (JS key order = insertion order: array-index keys leave
// the fast path; duplicates too)
template <bool W>
__host__ __device__ uint32_t props_obj(Rd &r, uint32_t &np, uint32_t gidx, uint32_t gev, const Ctx &cx) {
    if (r.at() != '{') return kFShape;
    r.p++;
    r.ws();
    np = 0;
    if (r.at() == '}') {
        r.p++;
        return 0;
    }
    uint32_t koff[kMaxProps], klen[kMaxProps];
    for (;;) {
        r.ws();
        uint32_t ko, kl;
        bool plain;
        if (!str_raw(r, ko, kl, plain)) return kFSyntax;
        if (!plain) return kFShape;
        bool digits = kl > 0;
        for (uint32_t i = 0; i < kl && digits; i++) digits = is_digit(r.b(ko + i));
        if (digits) return kFShape;
        for (uint32_t j = 0; j < np; j++)
            if (r.eq(koff[j], klen[j], ko, kl)) return kFShape;
        if (np >= (uint32_t)kMaxProps) return kFShape;
        koff[np] = ko;
        klen[np] = kl;
        r.ws();
        if (r.at() != ':') return kFSyntax;
        r.p++;
        r.ws();
        uint32_t vo = r.p, vl = 0;
        const int c = r.at();
        if (c == 'n') {
            if (!r.lit("null", 4)) return kFSyntax;
            vo = kNullSpan;
        } else if (c == 't') {
            if (!r.lit("true", 4)) return kFSyntax;
            vl = 4;
        } else if (c == 'f') {
            if (!r.lit("false", 5)) return kFSyntax;
            vl = 5;
        } else if (c == '"') {
            uint32_t so, sl;
            bool pl;
            if (!str_raw(r, so, sl, pl)) return kFSyntax;
            vl = sl + 2;  // a string already in JSON.stringify form: its source text
            if (!pl && !str_canonical(r, so, sl)) vl |= kSpanCanon;  // other escapes: the host re-quotes
        } else if (c == '-' || is_digit(c)) {
            int64_t v;
            uint32_t nd;
            const int t = num_tok(r, v, nd);
            if (!t) return kFSyntax;
            vl = r.p - vo;
            // a fraction / exponent, or more digits than Number::toString keeps exactly: the host
            // formats the double (shortest round trip)
            if (t != 1 || nd > 15) vl |= kSpanCanon;
        } else if (c == '[') {
            // a flat array already in JSON.stringify form (no whitespace, canonical elements:
            // what a log written by JSON.stringify holds, e.g. referenceTileLabels ["pg"]); any
            // other array is validated here and formatted by the host's js_stringify
            r.p++;
            bool canon = true;
            if (r.at() != ']') {
                for (;;) {
                    const int e = r.at();
                    if (e == '"') {
                        uint32_t so, sl;
                        bool pl;
                        if (!str_raw(r, so, sl, pl)) return kFSyntax;
                        if (!pl && !str_canonical(r, so, sl)) canon = false;
                    } else if (e == '-' || is_digit(e)) {
                        int64_t v;
                        uint32_t nd;
                        const int t = num_tok(r, v, nd);
                        if (!t) return kFSyntax;
                        if (t != 1 || nd > 15) canon = false;
                    } else if (!(r.lit("true", 4) || r.lit("false", 5) || r.lit("null", 4))) {
                        canon = false;  // nested containers / whitespace
                        break;
                    }
                    if (r.at() == ',') {
                        r.p++;
                        continue;
                    }
                    if (r.at() != ']') canon = false;
                    break;
                }
            }
            if (canon) {
                r.p++;
                vl = r.p - vo;
            } else {
                r.p = vo;
                if (!skip_value(r)) return kFSyntax;
                vl = (r.p - vo) | kSpanCanon;
            }
        } else if (c == '{') {
            // an object: validated here, formatted by the host's js_stringify (JS key order:
            // array-index keys first, duplicate keys, whitespace)
            if (!skip_value(r)) return kFSyntax;
            vl = (r.p - vo) | kSpanCanon;
        } else {
            return kFSyntax;
        }
        if (W) {
            cx.pk_off[gidx + np] = ko;
            cx.pk_len[gidx + np] = kl;
            cx.pe[gidx + np] = gev + np;
            cx.pv_off[gev + np] = vo;
            cx.pv_len[gev + np] = vl;
        }
        np++;
        r.ws();
        const int e = r.at();
        if (e == ',') {
            r.p++;
            continue;
        }
        if (e == '}') {
            r.p++;
            return 0;
        }
        return kFSyntax;
    }
}

// Packer1::relpos (mt_json.cpp:560-594): posN undefined and relativePosN truthy (N = 2 only for
// remove / annotate) -> an MT_OP_RELPOS record before the op (GROUP_CONT); a truthy id is a value
// event (its JSON text: a plain string, an integer or true), pos1 / pos2 = event + 1 until the remap
template <bool W>
__host__ __device__ uint32_t relpos_record(const uint8_t *s, uint32_t n, const OpInfo &op, const mt_op &base,
                                           MsgOut &mo, const Ctx &cx) {
    mt_op rr = base;
    rr.type = MT_OP_RELPOS;
    uint32_t rflags = MT_OPF_GROUP_CONT;
    for (int k = 0; k < 2; k++) {
        if ((op.seen & (k ? kOPos2 : kOPos1)) || !(op.seen & (k ? kORel2 : kORel1))) continue;
        if (k == 1 && op.type != 1 && op.type != 2) continue;
        Rd rq{s, k ? op.rel2_p : op.rel1_p, n};
        if (rq.lit("null", 4) || rq.lit("false", 5)) continue;  // falsy: no relative position
        if (rq.at() != '{') return kFShape;
        rflags |= k ? MT_RELF_POS2 : MT_RELF_POS1;
        rq.p++;
        rq.ws();
        uint32_t seen_k = 0;
        if (rq.at() != '}') {
            for (;;) {
                rq.ws();
                uint32_t ko, kl;
                bool plain;
                if (!str_raw(rq, ko, kl, plain)) return kFSyntax;
                if (!plain) return kFShape;
                rq.ws();
                if (rq.at() != ':') return kFSyntax;
                rq.p++;
                rq.ws();
                const uint32_t bit = rq.is(ko, kl, "id") ? 1u : rq.is(ko, kl, "before") ? 2u : rq.is(ko, kl, "offset") ? 4u : 0u;
                if (bit & seen_k) return kFShape;
                seen_k |= bit;
                const uint32_t vo = rq.p;
                const int c = rq.at();
                if (bit == 1u || bit == 2u) {
                    bool truthy = false;
                    if (c == '"') {
                        uint32_t so, sl;
                        bool pl;
                        if (!str_raw(rq, so, sl, pl)) return kFSyntax;
                        if (!pl && !str_canonical(rq, so, sl)) return kFShape;
                        truthy = sl > 0;
                    } else if (c == '-' || is_digit(c)) {
                        int64_t v;
                        uint32_t nd;
                        if (num_tok(rq, v, nd) != 1 || nd > 15) return kFShape;
                        truthy = v != 0;
                    } else if (rq.lit("true", 4)) {
                        truthy = true;
                    } else if (!(rq.lit("false", 5) || rq.lit("null", 4))) {
                        return kFShape;
                    }
                    if (truthy && bit == 2u) rflags |= k ? MT_RELF_BEFORE2 : MT_RELF_BEFORE1;
                    if (truthy && bit == 1u) {
                        const uint32_t ev = cx.gval + mo.nval;
                        if (W) {
                            cx.pv_off[ev] = vo;
                            cx.pv_len[ev] = rq.p - vo;
                        }
                        if (k) rr.pos2 = (int32_t)(ev + 1);
                        else rr.pos1 = (int32_t)(ev + 1);
                        mo.nval++;
                    }
                } else if (bit == 4u) {
                    // offset !== undefined: an integer, or null (adds 0)
                    int32_t o = 0;
                    if (!rq.lit("null", 4)) {
                        int64_t v;
                        uint32_t nd;
                        if (num_tok(rq, v, nd) != 1 || v < -2147483647ll || v > 2147483647ll) return kFShape;
                        o = (int32_t)v;
                    }
                    rflags |= k ? MT_RELF_OFF2 : MT_RELF_OFF1;
                    if (k) rr.payload_len = (uint32_t)o;
                    else rr.payload = (uint32_t)o;
                } else if (!skip_value(rq)) {
                    return kFSyntax;
                }
                rq.ws();
                if (rq.at() == ',') {
                    rq.p++;
                    continue;
                }
                if (rq.at() == '}') break;
                return kFSyntax;
            }
        }
    }
    if (rflags & (MT_RELF_POS1 | MT_RELF_POS2)) {
        rr.flags = (uint16_t)(rflags | (base.flags & MT_OPF_CLIENT_HI_MASK));
        if (W) cx.ops[mo.nrec] = rr;
        mo.nrec++;
        mo.flags |= kMsgRel;  // an ack reads no positions: the host parser drops it (clients stage)
        return 0;
    }
    return (op.seen & kOPos1) ? 0u : (uint32_t)kFShape;  // an op without a position
}

// one member op -> one record (Packer1::pack_op / pack_seg)
template <bool W>
__host__ __device__ uint32_t emit_op(const uint8_t *s, uint32_t n, const OpInfo &op, const mt_op &base, MsgOut &mo,
                            const Ctx &cx) {
    if (!(op.seen & kOType)) return kFShape;
    // a local insert with an end position fails in the host parser (getValidOpRange, client.ts:520-524)
    if (base.seq == -1 && op.type == 0 && (op.seen & (kOPos2 | kORel2))) return kFWriter;
    {
        const uint32_t f = relpos_record<W>(s, n, op, base, mo, cx);
        if (f) return f;
    }
    mt_op r = base;
    r.flags = (uint16_t)(MT_OPF_GROUP_CONT | (base.flags & MT_OPF_CLIENT_HI_MASK));  // GROUP_CONT: cleared on the message's last record
    r.pos1 = op.p1;
    r.pos2 = 0;
    r.payload = r.payload_len = 0;
    if (op.type == 0) {
        if (!(op.seen & kOSeg)) return kFShape;
        Rd rs{s, op.seg_p, n};
        uint32_t text_p = 0, props_p = 0, marker_p = 0;
        bool has_text = false, has_props = false, has_marker = false;
        if (rs.at() == '"') {
            text_p = op.seg_p;
            has_text = true;
        } else if (rs.at() == '{') {
            rs.p++;
            rs.ws();
            if (rs.at() == '}') return kFShape;
            for (;;) {
                rs.ws();
                uint32_t ko, kl;
                bool plain;
                if (!str_raw(rs, ko, kl, plain)) return kFSyntax;
                if (!plain) return kFShape;
                rs.ws();
                if (rs.at() != ':') return kFSyntax;
                rs.p++;
                rs.ws();
                if (rs.is(ko, kl, "text")) {
                    if (has_text || rs.at() != '"') return kFShape;
                    has_text = true;
                    text_p = rs.p;
                } else if (rs.is(ko, kl, "props")) {
                    if (has_props) return kFShape;
                    has_props = true;
                    props_p = rs.p;
                } else if (rs.is(ko, kl, "marker")) {
                    if (has_marker) return kFShape;
                    has_marker = true;
                    marker_p = rs.p;
                }
                if (!skip_value(rs)) return kFSyntax;
                rs.ws();
                const int c = rs.at();
                if (c == ',') {
                    rs.p++;
                    continue;
                }
                if (c == '}') break;
                return kFSyntax;
            }
            if (!has_text && !has_marker) return kFShape;
        } else {
            return kFShape;
        }
        uint32_t units = 0, ref_type = 0;
        bool has_nl = false, ends_nl = false;
        const bool marker = !has_text;  // pack_seg: "text" wins over "marker"
        if (marker) {
            // {marker: {refType}} (pack_seg, mt_json.cpp:522-528): payload = refType, length 1
            Rd rm{s, marker_p, n};
            if (rm.at() != '{') return kFShape;
            rm.p++;
            rm.ws();
            bool seen_rt = false;
            if (rm.at() != '}') {
                for (;;) {
                    rm.ws();
                    uint32_t ko, kl;
                    bool plain;
                    if (!str_raw(rm, ko, kl, plain)) return kFSyntax;
                    if (!plain) return kFShape;
                    rm.ws();
                    if (rm.at() != ':') return kFSyntax;
                    rm.p++;
                    rm.ws();
                    if (rm.is(ko, kl, "refType")) {
                        int64_t v;
                        uint32_t nd;
                        if (seen_rt || num_tok(rm, v, nd) != 1 || v < 0 || v > 0x7FFFFFFF) return kFShape;
                        seen_rt = true;
                        ref_type = (uint32_t)v;
                    } else if (!skip_value(rm)) {
                        return kFSyntax;
                    }
                    rm.ws();
                    const int c = rm.at();
                    if (c == ',') {
                        rm.p++;
                        continue;
                    }
                    if (c == '}') break;
                    return kFSyntax;
                }
            }
        } else {
            Rd rt{s, text_p, n};
            if (!str_text(rt, W ? cx.text + mo.ntext : nullptr, units, has_nl, ends_nl)) return kFSyntax;
        }
        uint32_t np = 0;
        bool hp = false;
        if (has_props) {
            Rd rp{s, props_p, n};
            const int c = rp.at();
            if (c == '{') {
                hp = true;
                const uint32_t f = props_obj<W>(rp, np, cx.gprop + mo.nprop, cx.gval + mo.nval, cx);
                if (f) return f;
            } else if (!(rp.lit("null", 4) || rp.lit("false", 5))) {
                return kFShape;  // arrays fail, other truthy values fail, 0 / "" are rare: host
            }
        }
        r.type = MT_OP_INSERT;
        if (hp) {
            r.flags |= (uint16_t)(MT_OPF_HAS_PROPS | (np << 4));
            r.pos2 = (int32_t)(cx.gprop + mo.nprop);
            mo.npropops++;
        }
        if (marker) {
            r.flags |= (uint16_t)MT_OPF_MARKER;
            r.payload = ref_type;
            r.payload_len = 1;  // the marker id (if any) replaces it at install (jg_markers_kernel)
        } else {
            r.payload = cx.pay + mo.ntext;
            r.payload_len = units;
        }
        if (cx.install && !marker) {
            if (has_nl) r.flags |= (uint16_t)MT_OPF_INTERNAL_HAS_NL;
            if (ends_nl) r.flags |= (uint16_t)MT_OPF_INTERNAL_ENDS_NL;
        }
        mo.ntext += units;
        mo.nprop += np;
        mo.nval += np;
    } else if (op.type == 1 || op.type == 2) {
        r.type = op.type == 1 ? MT_OP_REMOVE : MT_OP_ANNOTATE;
        r.pos2 = (op.seen & kOPos2) ? op.p2 : 0;
        if (op.type == 2) {
            if (!(op.seen & kOProps)) return kFShape;
            Rd rp{s, op.props_p, n};
            uint32_t np = 0;
            const uint32_t f = props_obj<W>(rp, np, cx.gprop + mo.nprop, cx.gval + mo.nval, cx);
            if (f) return f;
            r.payload = cx.gprop + mo.nprop;
            r.payload_len = np;
            if (op.rewrite) r.flags |= (uint16_t)MT_OPF_REWRITE;
            mo.nprop += np;
            mo.nval += np;
            mo.npropops++;
        }
    } else {
        return kFShape;
    }
    if (W) cx.ops[mo.nrec] = r;
    mo.nrec++;
    return 0;
}

// one message (Packer1::run's loop body): returns fail bits
template <bool W>
__host__ __device__ uint32_t parse_msg(const uint8_t *s, uint32_t n, uint32_t p0, MsgOut &mo, const Ctx &cx) {
    Rd r{s, p0 + 1, n};  // after '{'
    enum { kCl = 1, kSeq = 2, kRef = 4, kMsn = 8, kTy = 16, kCo = 32 };
    uint32_t seen = 0, contents_p = 0;
    int64_t seq = 0, ref = 0, msn = 0;
    bool is_op = false, notify = false;
    r.ws();
    if (r.at() == '}') return kFShape;
    for (;;) {
        r.ws();
        uint32_t ko, kl;
        bool plain;
        if (!str_raw(r, ko, kl, plain)) return kFSyntax;
        if (!plain) return kFShape;
        r.ws();
        if (r.at() != ':') return kFSyntax;
        r.p++;
        r.ws();
        uint32_t bit = 0;
        if (r.is(ko, kl, "clientId")) bit = kCl;
        else if (r.is(ko, kl, "sequenceNumber")) bit = kSeq;
        else if (r.is(ko, kl, "referenceSequenceNumber")) bit = kRef;
        else if (r.is(ko, kl, "minimumSequenceNumber")) bit = kMsn;
        else if (r.is(ko, kl, "type")) bit = kTy;
        else if (r.is(ko, kl, "contents")) bit = kCo;
        if (bit) {
            if (seen & bit) return kFShape;
            seen |= bit;
        }
        if (bit == kCl && r.at() == '"') {
            uint32_t o, l;
            bool pl;
            if (!str_raw(r, o, l, pl)) return kFSyntax;
            if (!pl) return kFShape;
            mo.cl_off = o;
            mo.cl_len = l;
        } else if (bit == kSeq || bit == kRef || bit == kMsn) {
            int64_t v;
            uint32_t nd;
            const int t = num_tok(r, v, nd);
            if (t != 1) return t ? kFShape : kFSyntax;
            if (v < -2147483648ll || v > 2147483647ll) return kFRange;
            (bit == kSeq ? seq : bit == kRef ? ref : msn) = v;
        } else if (bit == kTy && r.at() == '"') {
            uint32_t o, l;
            bool pl;
            if (!str_raw(r, o, l, pl)) return kFSyntax;
            if (!pl) return kFShape;
            is_op = l == 2 && r.b(o) == 'o' && r.b(o + 1) == 'p';
        } else {
            if (bit == kCo) contents_p = r.p;
            // {"notifyConsensus": truthy} on a local message (Client.annotateMarkerNotifyConsensus):
            // the host parser's; null / false are absent
            if (!bit && r.is(ko, kl, "notifyConsensus") && !(r.lit("null", 4) || r.lit("false", 5))) notify = true;
            // clientId / type of another JSON type: "null" / not an op (the host's rules)
            if (!skip_value(r)) return kFSyntax;
        }
        r.ws();
        const int c = r.at();
        if (c == ',') {
            r.p++;
            continue;
        }
        if (c == '}') {
            r.p++;
            break;
        }
        return kFSyntax;
    }
    r.ws();
    if (r.at() != ',' && r.at() != ']') return kFSyntax;
    // a writer replica's own unsequenced message (sequenceNumber -1) is a local op: no refSeq / msn
    // needed, msn 0 (mt_json.cpp Packer1::run); regenerate / non-op / notifyConsensus ones: host
    const bool local = (seen & kSeq) && seq == -1;
    if (local) {
        if (!is_op || notify) return kFWriter;
        if (!(seen & kRef)) ref = 0;
        msn = 0;
        mo.flags |= kMsgLocal;
    } else if ((seen & (kSeq | kRef | kMsn)) != (kSeq | kRef | kMsn)) {
        return kFShape;
    }
    if (is_op) mo.flags |= kMsgOp;
    mt_op base{};
    base.type = MT_OP_NOOP;
    base.client = (uint16_t)(cx.cid & 0xFFFu);  // the short id's high bits: flags 11-13 (mt_oplog.h)
    base.flags = MT_OPF_CLIENT_HI(cx.cid);
    base.seq = (int32_t)seq;
    base.ref_seq = (int32_t)ref;
    base.msn = (int32_t)msn;
    if (is_op && (seen & kCo)) {
        OpInfo top;
        Rd rc{s, contents_p, n};
        uint32_t f = parse_op(rc, top);
        if (f) return f;
        if ((top.seen & kOType) && top.type == 3) {  // GROUP: one level of member ops
            if (!(top.seen & kOOps)) return kFShape;
            Rd ro{s, top.ops_p, n};
            if (ro.at() != '[') return kFShape;
            ro.p++;
            ro.ws();
            if (ro.at() == ']') {
                ro.p++;
            } else {
                for (;;) {
                    ro.ws();
                    OpInfo m;
                    f = parse_op(ro, m);
                    if (f) return f;
                    if (!(m.seen & kOType) || m.type == 3) return kFShape;
                    f = emit_op<W>(s, n, m, base, mo, cx);
                    if (f) return f;
                    ro.ws();
                    const int c = ro.at();
                    if (c == ',') {
                        ro.p++;
                        continue;
                    }
                    if (c == ']') break;
                    return kFSyntax;
                }
            }
        } else {
            f = emit_op<W>(s, n, top, base, mo, cx);
            if (f) return f;
        }
    }
    if (mo.nrec == 0) {  // not an op / no member: updateSeqNumbers only
        if (W) cx.ops[0] = base;
        mo.nrec = 1;
    } else if (W) {
        cx.ops[mo.nrec - 1].flags &= (uint16_t)~MT_OPF_GROUP_CONT;
    }
    return 0;
}

// ---------------------------------------------------------------- stage 2 / 4: parse passes
// one wavefront per 64 messages of a document (chunk_doc / chunk_first), so a batch of long
// documents fills the chip; the count pass stores per-message counts, jg_offsets_kernel turns them
// into each message's offsets in its document, the write pass writes there
template <bool W>
__device__ void parse_chunk(const Params &P) {
    const int64_t c = blockIdx.x;
    const int64_t d = P.chunk_doc[c];
    if (P.d_fail[d]) return;
    const int lane = lane_id();
    const int64_t a = P.doc_off[d];
    const uint32_t len = (uint32_t)(P.doc_off[d + 1] - a);
    const uint8_t *s = P.J + a;
    const uint64_t mb = mregion(P.doc_off, d);
    const uint32_t nmsg = P.d_nmsg[d];
    const uint32_t i = P.chunk_first[c] + (uint32_t)lane;
    if (i >= nmsg) return;
    const uint64_t m = mb + i;
    MsgOut mo;
    Ctx cx;
    if (W) {
        cx.ops = P.ops + P.op_base[d] + P.m_recoff[m];
        cx.text = P.text + P.text_dst[d] + P.m_textoff[m];
        cx.pay = P.text_pay[d] + P.m_textoff[m];
        cx.gprop = P.prop_base[d] + P.m_propoff[m];
        cx.gval = P.val_base[d] + P.m_valoff[m];
        cx.pe = P.pe;
        cx.pk_off = P.pk_off;
        cx.pk_len = P.pk_len;
        cx.pv_off = P.pv_off;
        cx.pv_len = P.pv_len;
        cx.cid = (uint16_t)P.m_cid[m];
        cx.install = P.install != 0;
    }
    const uint32_t f = parse_msg<W>(s, len, P.m_start[m], mo, cx);
    if (f) atomicOr(P.d_fail + d, f);
    if (!W) {
        P.m_flags[m] = mo.flags;
        P.m_nrec[m] = mo.nrec;
        P.m_ntext[m] = mo.ntext;
        P.m_nprop[m] = mo.nprop;
        P.m_npops[m] = mo.npropops;
        P.m_nval[m] = mo.nval;
        P.m_cloff[m] = mo.cl_off;
        P.m_cllen[m] = mo.cl_len;
    }
}
extern "C" __global__ __launch_bounds__(64) void jg_count_kernel(Params P) { parse_chunk<false>(P); }
extern "C" __global__ __launch_bounds__(64) void jg_write_kernel(Params P) { parse_chunk<true>(P); }

// per document: message offsets (exclusive prefix sums of the counts) and the totals
extern "C" __global__ __launch_bounds__(64) void jg_offsets_kernel(Params P) {
    const int64_t d = blockIdx.x;
    if (d >= P.D || P.d_fail[d]) return;
    const int lane = lane_id();
    const uint64_t mb = mregion(P.doc_off, d);
    const uint32_t nmsg = P.d_nmsg[d];
    uint32_t sr = 0, st = 0, sp = 0, so = 0, sv = 0;
    for (uint32_t i0 = 0; i0 < nmsg; i0 += 64) {
        const uint32_t i = i0 + (uint32_t)lane;
        const bool valid = i < nmsg;
        const uint64_t m = mb + i;
        const uint32_t nr = valid ? P.m_nrec[m] : 0u, nt = valid ? P.m_ntext[m] : 0u;
        const uint32_t np = valid ? P.m_nprop[m] : 0u, no = valid ? P.m_npops[m] : 0u;
        const uint32_t nv = valid ? P.m_nval[m] : 0u;
        const uint32_t ir = wave_incl(nr), it = wave_incl(nt), ip = wave_incl(np), io = wave_incl(no);
        const uint32_t iv = wave_incl(nv);
        if (valid) {
            P.m_recoff[m] = sr + ir - nr;
            P.m_textoff[m] = st + it - nt;
            P.m_propoff[m] = sp + ip - np;
            P.m_valoff[m] = sv + iv - nv;
        }
        sr += __shfl(ir, 63, 64);
        st += __shfl(it, 63, 64);
        sp += __shfl(ip, 63, 64);
        so += __shfl(io, 63, 64);
        sv += __shfl(iv, 63, 64);
    }
    if (lane == 0) {
        P.d_nrec[d] = sr;
        P.d_ntext[d] = st;
        P.d_nprop[d] = sp;
        P.d_npropops[d] = so;
        P.d_nval[d] = sv;
    }
}

// ---------------------------------------------------------------- first-appearance interning
// Entries are indices (+1) into the document's spans; a slot keeps the smallest index holding
// its string (CAS to claim, atomicMin on a match), so after every earlier index was inserted the
// slot's value is the string's first appearance.  cap: power of two, > distinct strings.
struct Spans {
    const uint8_t *s;          // document bytes
    const uint32_t *off, *len; // spans (kNullSpan: the text "null")
    uint64_t base;             // index of entry 0
    const uint8_t *null4;
    __device__ const uint8_t *ptr(uint32_t i) const { return off[base + i] == kNullSpan ? null4 : s + off[base + i]; }
    __device__ uint32_t n(uint32_t i) const { return off[base + i] == kNullSpan ? 4u : len[base + i] & ~kSpanCanon; }
};

// insert entry i; returns false when the table is full
__device__ bool ht_insert(uint32_t *tab, uint32_t cap, const Spans &S, uint32_t i) {
    const uint8_t *p = S.ptr(i);
    const uint32_t l = S.n(i);
    uint32_t slot = fnv32(p, l) & (cap - 1);
    for (uint32_t probe = 0; probe < cap; probe++) {
        const uint32_t v = atomicCAS(tab + slot, 0u, i + 1);
        if (v == 0) return true;
        const uint32_t j = v - 1;
        if (span_eq(S.ptr(j), S.n(j), p, l)) {
            atomicMin(tab + slot, i + 1);
            return true;
        }
        slot = (slot + 1) & (cap - 1);
    }
    return false;
}
// first appearance of entry i's string
__device__ uint32_t ht_first(const uint32_t *tab, uint32_t cap, const Spans &S, uint32_t i) {
    const uint8_t *p = S.ptr(i);
    const uint32_t l = S.n(i);
    uint32_t slot = fnv32(p, l) & (cap - 1);
    for (uint32_t probe = 0; probe < cap; probe++) {
        const uint32_t v = __hip_atomic_load(tab + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (v == 0) break;
        const uint32_t j = v - 1;
        if (span_eq(S.ptr(j), S.n(j), p, l)) return j;
        slot = (slot + 1) & (cap - 1);
    }
    return i;
}

// ids of n entries in first-appearance order: id(i) = first0 + number of first appearances
// before i's string's; skip(i): entries that take no id (the observer, null values).  ids[] is
// indexed like the spans; uniq_off / uniq_len receive each id's span.  Returns the id count, or
// 0xFFFFFFFF when the table overflowed.
template <class Skip>
__device__ uint32_t intern(uint32_t *tab, uint32_t cap, const Spans &S, uint32_t n, uint32_t first0, uint32_t *ids,
                           uint32_t *uniq_off, uint32_t *uniq_len, Skip skip) {
    const int lane = lane_id();
    uint32_t count = 0;
    bool full = false;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + (uint32_t)lane;
        const bool act = i < n && !skip(i);
        if (act && !ht_insert(tab, cap, S, i)) full = true;
        if (ballot(full)) return 0xFFFFFFFFu;
        __syncthreads();
        const uint32_t rep = act ? ht_first(tab, cap, S, i) : i;
        const bool fresh = act && rep == i;
        const uint64_t fm = ballot(fresh);
        const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
        if (fresh) {
            const uint32_t id = first0 + count + (uint32_t)__builtin_popcountll(fm & below);
            ids[S.base + i] = id;
            uniq_off[S.base + id - first0] = S.off[S.base + i];
            uniq_len[S.base + id - first0] = S.len[S.base + i];
        }
        __syncthreads();
        if (act && !fresh) ids[S.base + i] = ids[S.base + rep];
        count += (uint32_t)__builtin_popcountll(fm);
        __syncthreads();
    }
    return count;
}

// stage 3: short client ids
extern "C" __global__ __launch_bounds__(64) void jg_clients_kernel(Params P) {
    const int64_t d = blockIdx.x;
    if (d >= P.D || P.d_fail[d]) return;
    const int lane = lane_id();
    const uint64_t mb = mregion(P.doc_off, d);
    const uint32_t nmsg = P.d_nmsg[d];
    Spans S{P.J + P.doc_off[d], P.m_cloff, P.m_cllen, mb, P.obs + 256};
    uint32_t fail = 0;
    // the observer's own messages: short id 0.  A local op or an op of its own (an ack) makes the
    // document a writer replica's log; an ack with relative positions (whose RELPOS record the host
    // parser drops) and a local op of another client (an error there) leave the fast path
    uint32_t wr = 0;
    for (uint32_t i0 = 0; i0 < nmsg; i0 += 64) {
        const uint32_t i = i0 + (uint32_t)lane;
        if (i >= nmsg) continue;
        const uint32_t fl = P.m_flags[mb + i];
        if (span_eq(S.ptr(i), S.n(i), P.obs, P.obs_len)) {
            P.m_cid[mb + i] = 0;
            if (fl & (kMsgOp | kMsgLocal)) wr = 1;
            if ((fl & kMsgRel) && !(fl & kMsgLocal)) fail |= kFWriter;
        } else {
            P.m_cid[mb + i] = 0xFFFFFFFFu;
            if (fl & kMsgLocal) fail |= kFWriter;
        }
    }
    for (int o = 32; o > 0; o >>= 1) wr |= __shfl_xor(wr, o, 64);
    __syncthreads();
    uint32_t *tab = P.cl_ht + P.cl_base[d];
    const uint32_t *cid = P.m_cid;
    auto is_obs = [&](uint32_t i) { return cid[mb + i] == 0u; };
    const uint32_t cnt = intern(tab, P.cl_cap[d], S, nmsg, 1u, P.m_cid, P.nm_off, P.nm_len, is_obs);
    for (int o = 32; o > 0; o >>= 1) fail |= __shfl_xor(fail, o, 64);
    if (cnt == 0xFFFFFFFFu || cnt + 1 > (uint32_t)MT_MAX_CLIENTS) fail |= kFClients;
    if (lane == 0) {
        P.d_writer[d] = wr;
        P.d_nnames[d] = cnt == 0xFFFFFFFFu ? 0u : cnt + 1;
        if (fail) P.d_fail[d] = fail;
    }
}

// the documents' client-name spans (ids 1.., nm_off / nm_len of the message region) back to back
// for the host: names_base from the host's prefix sum of the name counts
extern "C" __global__ __launch_bounds__(64) void jg_names_kernel(Params P) {
    const int64_t d = blockIdx.x;
    if (d >= P.D) return;
    const uint32_t nn = P.d_nnames[d];
    const uint64_t mb = mregion(P.doc_off, d), nb = P.names_base[d];
    for (uint32_t k = (uint32_t)lane_id(); k + 1 < nn; k += 64) {
        P.names[nb + 2 * k] = P.nm_off[mb + k];
        P.names[nb + 2 * k + 1] = P.nm_len[mb + k];
    }
}

// stage 5: prop keys and values
extern "C" __global__ __launch_bounds__(64) void jg_props_kernel(Params P) {
    const int64_t d = blockIdx.x;
    if (d >= P.D) return;
    const uint32_t n = P.d_nprop[d], ne = P.d_nval[d];
    const uint64_t pb = P.prop_base[d], vb = P.val_base[d];
    const uint32_t cap = P.ht_cap[d];
    uint32_t *tk = P.ht + P.ht_base[d], *tv = tk + cap;
    const uint8_t *s = P.J + P.doc_off[d];
    Spans K{s, P.pk_off, P.pk_len, pb, P.obs + 256};
    Spans V{s, P.pv_off, P.pv_len, vb, P.obs + 256};
    const uint32_t nk = intern(tk, cap, K, n, 0u, P.lk, P.uk_off, P.uk_len, [](uint32_t) { return false; });
    const uint32_t *pvo = P.pv_off;
    auto is_null = [&](uint32_t i) { return pvo[vb + i] == kNullSpan; };
    for (uint32_t i = (uint32_t)lane_id(); i < ne; i += 64)
        if (is_null(i)) P.lv[vb + i] = 0;
    __syncthreads();
    const uint32_t nv = intern(tv, cap, V, ne, 1u, P.lv, P.uv_off, P.uv_len, is_null);
    if (lane_id() == 0) {
        P.d_nuk[d] = nk;
        P.d_nuv[d] = nv;
    }
}

// stage 6: batch-wide ids
extern "C" __global__ __launch_bounds__(64) void jg_remap_kernel(Params P) {
    const int64_t d = blockIdx.x;
    if (d >= P.D) return;
    const uint32_t n = P.d_nprop[d];
    const uint64_t pb = P.prop_base[d], vb = P.val_base[d];
    for (uint32_t i = (uint32_t)lane_id(); i < n; i += 64) {
        const uint32_t k = P.lk[pb + i], v = P.lv[P.pe[pb + i]];
        P.props[pb + i] = mt_prop{P.kmap[pb + k], v ? P.vmap[vb + v - 1] : 0u};
    }
    // relative positions: value event + 1 -> the batch value id of the id (0: none)
    const int64_t o0 = P.op_base[d], o1 = o0 + P.d_nrec[d];
    for (int64_t i = o0 + lane_id(); i < o1; i += 64) {
        if (P.ops[i].type != MT_OP_RELPOS) continue;
        const uint32_t e1 = (uint32_t)P.ops[i].pos1, e2 = (uint32_t)P.ops[i].pos2;
        const uint32_t v1 = e1 ? P.lv[e1 - 1] : 0u, v2 = e2 ? P.lv[e2 - 1] : 0u;
        P.ops[i].pos1 = (int32_t)(v1 ? P.vmap[vb + v1 - 1] : 0u);
        P.ops[i].pos2 = (int32_t)(v2 ? P.vmap[vb + v2 - 1] : 0u);
    }
}

// install: marker ids (resolve_marker_ids in mt_host.cpp: a marker insert whose props give a truthy
// markerId gets that id's key in payload_len, 0 otherwise; vkey maps value ids to keys) and the
// documents whose annotates touch referenceTileLabels (bit 0: their findTile queries are
// unsupported) or referenceRangeLabels (bit 1: getStackContext)
extern "C" __global__ __launch_bounds__(64) void jg_markers_kernel(const mt_op *ops, const int64_t *op_off,
                                                                 mt_op *ops_w, const mt_prop *props, int64_t D,
                                                                 uint32_t mk_key, uint32_t tile_key,
                                                                 uint32_t range_key,
                                                                 const uint32_t *vkey, uint32_t n_values,
                                                                 uint32_t *n_ids, uint32_t *tile_annot) {
    const int64_t d = blockIdx.x;
    if (d >= D) return;
    uint32_t cnt = 0, tile = 0, annot_mk = 0;
    for (int64_t i = op_off[d] + lane_id(); i < op_off[d + 1]; i += 64) {
        mt_op o = ops[i];
        if (o.type == MT_OP_INSERT && (o.flags & MT_OPF_MARKER)) {
            uint32_t id = 0;
            if (o.flags & MT_OPF_HAS_PROPS)
                for (uint32_t q = 0; q < MT_OPF_NPROPS(o.flags); q++) {
                    const mt_prop pr = props[o.pos2 + q];
                    if (pr.key == mk_key) id = pr.value < n_values ? vkey[pr.value] : 0u;
                }
            ops_w[i].payload_len = id;
            cnt += id != 0;
        } else if (o.type == MT_OP_ANNOTATE) {
            for (uint32_t q = 0; q < o.payload_len; q++) {
                if (props[o.payload + q].key == tile_key) tile |= 1u;
                if (props[o.payload + q].key == range_key) tile |= 2u;
                if (props[o.payload + q].key == mk_key) annot_mk = 1;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        cnt += __shfl_xor(cnt, off, 64);
        tile |= __shfl_xor(tile, off, 64);
        annot_mk |= __shfl_xor(annot_mk, off, 64);
    }
    // relative positions: an id's value -> its key; a document whose annotates touch markerId gets
    // kIdKeyUnsupported (resolve_marker_ids: the reference re-maps a re-annotated id only at a
    // later blockUpdate)
    for (int64_t i = op_off[d] + lane_id(); i < op_off[d + 1]; i += 64) {
        if (ops[i].type != MT_OP_RELPOS) continue;
        const uint32_t v1 = (uint32_t)ops[i].pos1, v2 = (uint32_t)ops[i].pos2;
        ops_w[i].pos1 = (int32_t)(annot_mk ? kIdKeyUnsupported : (v1 < n_values ? vkey[v1] : 0u));
        ops_w[i].pos2 = (int32_t)(annot_mk ? kIdKeyUnsupported : (v2 < n_values ? vkey[v2] : 0u));
    }
    if (lane_id() == 0) {
        n_ids[d] = cnt;
        tile_annot[d] = tile;
    }
}

}  // namespace jg
}  // namespace mt

// ---------------------------------------------------------------- host driver
namespace mt {
namespace jg {
namespace {

#define JGCHK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "mtreplay: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                                     \
            return MT_ERR_HIP;                                                                     \
        }                                                                                          \
    } while (0)

struct DevBufs {
    std::vector<void *> ptrs;
    ~DevBufs() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <class T>
    hipError_t get(T **p, size_t n) {
        *p = nullptr;
        hipError_t e = hipMalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) ptrs.push_back((void *)*p);
        return e;
    }
};

template <class T>
hipError_t dl(std::vector<T> &h, const T *d, size_t n, hipStream_t s) {
    h.resize(n);
    if (!n) return hipSuccess;
    hipError_t e = hipMemcpyAsync(h.data(), d, n * sizeof(T), hipMemcpyDeviceToHost, s);
    return e == hipSuccess ? hipStreamSynchronize(s) : e;
}

uint32_t pow2_at_least(uint64_t x) {
    uint32_t c = 16;
    while (c < x) c <<= 1;
    return c;
}

}  // namespace

int parse(const char *h_json, const int64_t *doc_off, int64_t D, const uint8_t *d_json_in, const char *observer,
          void *stream, const TextLayout *install, mt_op **d_ops_out, uint16_t **d_text_out, uint64_t *text_words,
          mt_prop **d_props_out, Result &res) {
    *d_ops_out = nullptr;
    *d_text_out = nullptr;
    *d_props_out = nullptr;
    res = Result{};
    if (D < 0 || !doc_off || doc_off[0] != 0) return MT_ERR_ARG;
    for (int64_t d = 0; d < D; d++)
        if (doc_off[d + 1] < doc_off[d] || doc_off[d + 1] - doc_off[d] > 0xFFFFFFF0ll) return MT_ERR_ARG;
    const std::string obs = observer ? observer : "readonly";
    if (obs.size() > 255) return MT_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t total = (uint64_t)doc_off[D];
    DevBufs B;
    Params P{};
    P.D = D;
    hipEvent_t ev[6];
    for (auto &e : ev) JGCHK(hipEventCreate(&e));
    struct EvFree {
        hipEvent_t *e;
        ~EvFree() {
            for (int i = 0; i < 6; i++) (void)hipEventDestroy(e[i]);
        }
    } evf{ev};
    const uint8_t *J = d_json_in;
    if (!J) {
        uint8_t *dj = nullptr;
        JGCHK(B.get(&dj, total + 64));
        JGCHK(hipMemcpyAsync(dj, h_json, total, hipMemcpyHostToDevice, s));
        JGCHK(hipMemsetAsync(dj + total, 0, 64, s));
        J = dj;
    }
    P.J = J;
    int64_t *d_off = nullptr;
    JGCHK(B.get(&d_off, (size_t)D + 1));
    JGCHK(hipMemcpyAsync(d_off, doc_off, 8 * ((size_t)D + 1), hipMemcpyHostToDevice, s));
    P.doc_off = d_off;
    const size_t M = (size_t)(total / 64 + 2 * (uint64_t)D + 2);
    uint32_t **marr[] = {&P.m_start, &P.m_flags, &P.m_nrec, &P.m_ntext, &P.m_nprop, &P.m_recoff,
                         &P.m_textoff, &P.m_propoff, &P.m_cloff, &P.m_cllen, &P.m_cid, &P.nm_off, &P.nm_len,
                         &P.m_npops, &P.m_nval, &P.m_valoff};
    for (uint32_t **a : marr) JGCHK(B.get(a, M));
    uint32_t **darr[] = {&P.d_nmsg, &P.d_fail, &P.d_nrec, &P.d_ntext, &P.d_nprop, &P.d_npropops,
                         &P.d_nnames, &P.d_nuk, &P.d_nuv, &P.d_nval, &P.d_writer};
    for (uint32_t **a : darr) JGCHK(B.get(a, (size_t)D));
    JGCHK(hipMemsetAsync(P.d_nrec, 0, 4 * (size_t)std::max<int64_t>(D, 1), s));
    JGCHK(hipMemsetAsync(P.d_writer, 0, 4 * (size_t)std::max<int64_t>(D, 1), s));
    JGCHK(hipMemsetAsync(P.d_ntext, 0, 4 * (size_t)std::max<int64_t>(D, 1), s));
    JGCHK(hipMemsetAsync(P.d_nprop, 0, 4 * (size_t)std::max<int64_t>(D, 1), s));
    JGCHK(hipMemsetAsync(P.d_npropops, 0, 4 * (size_t)std::max<int64_t>(D, 1), s));
    {
        uint8_t *o = nullptr;
        JGCHK(B.get(&o, 512));
        std::vector<uint8_t> ob(512, 0);
        memcpy(ob.data(), obs.data(), obs.size());
        memcpy(ob.data() + 256, "null", 4);
        JGCHK(hipMemcpyAsync(o, ob.data(), 512, hipMemcpyHostToDevice, s));
        P.obs = o;
        P.obs_len = (uint32_t)obs.size();
    }
    const unsigned grid = (unsigned)std::max<int64_t>(D, 1);
    // scan segments
    std::vector<int32_t> seg_doc;
    std::vector<uint32_t> seg_start;
    std::vector<int64_t> seg_first((size_t)D + 1, 0);
    for (int64_t d = 0; d < D; d++) {
        seg_first[(size_t)d] = (int64_t)seg_doc.size();
        const uint64_t len = (uint64_t)(doc_off[d + 1] - doc_off[d]);
        for (uint64_t st = 0; st < len; st += kSegBytes) {
            seg_doc.push_back((int32_t)d);
            seg_start.push_back((uint32_t)st);
        }
    }
    seg_first[(size_t)D] = (int64_t)seg_doc.size();
    const size_t G = seg_doc.size();
    P.G = (int64_t)G;
    int32_t *d_sdoc = nullptr;
    uint32_t *d_sstart = nullptr;
    int64_t *d_sfirst = nullptr;
    JGCHK(B.get(&d_sdoc, G));
    JGCHK(B.get(&d_sstart, G));
    JGCHK(B.get(&d_sfirst, (size_t)D + 1));
    if (G) {
        JGCHK(hipMemcpyAsync(d_sdoc, seg_doc.data(), 4 * G, hipMemcpyHostToDevice, s));
        JGCHK(hipMemcpyAsync(d_sstart, seg_start.data(), 4 * G, hipMemcpyHostToDevice, s));
    }
    JGCHK(hipMemcpyAsync(d_sfirst, seg_first.data(), 8 * ((size_t)D + 1), hipMemcpyHostToDevice, s));
    P.seg_doc = d_sdoc;
    P.seg_start = d_sstart;
    P.seg_first = d_sfirst;
    uint32_t **sarr[] = {&P.sg_q, &P.sg_pre, &P.sg_post, &P.sg_flags, &P.sg_nmsg, &P.sg_fail};
    for (uint32_t **a : sarr) JGCHK(B.get(a, G));
    JGCHK(B.get(&P.sg_d0, G));
    JGCHK(B.get(&P.sg_d1, G));
    JGCHK(B.get(&P.sg_starts, G * kSegStarts));
    void *args[] = {&P};
    JGCHK(hipEventRecord(ev[0], s));
    if (G) JGCHK(hipLaunchKernel((const void *)jg_seg_a_kernel, dim3((unsigned)G), dim3(64), args, 0, s));
    if (G) JGCHK(hipLaunchKernel((const void *)jg_seg_b_kernel, dim3((unsigned)G), dim3(64), args, 0, s));
    if (D) JGCHK(hipLaunchKernel((const void *)jg_seg_c_kernel, dim3(grid), dim3(64), args, 0, s));
    std::vector<uint32_t> nmsg;
    JGCHK(dl(nmsg, P.d_nmsg, (size_t)D, s));
    std::vector<int32_t> chunk_doc;
    std::vector<uint32_t> chunk_first;
    for (int64_t d = 0; d < D; d++)
        for (uint32_t i = 0; i < nmsg[(size_t)d]; i += 64) {
            chunk_doc.push_back((int32_t)d);
            chunk_first.push_back(i);
        }
    int32_t *d_cdoc = nullptr;
    uint32_t *d_cfirst = nullptr;
    JGCHK(B.get(&d_cdoc, chunk_doc.size()));
    JGCHK(B.get(&d_cfirst, chunk_doc.size()));
    if (!chunk_doc.empty()) {
        JGCHK(hipMemcpyAsync(d_cdoc, chunk_doc.data(), 4 * chunk_doc.size(), hipMemcpyHostToDevice, s));
        JGCHK(hipMemcpyAsync(d_cfirst, chunk_first.data(), 4 * chunk_first.size(), hipMemcpyHostToDevice, s));
    }
    P.chunk_doc = d_cdoc;
    P.chunk_first = d_cfirst;
    const unsigned cgrid = (unsigned)chunk_doc.size();
    void *argc[] = {&P};
    JGCHK(hipEventRecord(ev[1], s));
    if (cgrid) JGCHK(hipLaunchKernel((const void *)jg_count_kernel, dim3(cgrid), dim3(64), argc, 0, s));
    if (D) JGCHK(hipLaunchKernel((const void *)jg_offsets_kernel, dim3(grid), dim3(64), argc, 0, s));
    // client hash tables: a power of two > 2 x the names a document can hold (its messages, at most
    // MT_MAX_CLIENTS: a table too small for more names reports the document, kFClients)
    {
        std::vector<uint64_t> cl_base((size_t)D);
        std::vector<uint32_t> cl_cap((size_t)D);
        uint64_t csum = 0;
        for (int64_t d = 0; d < D; d++) {
            cl_cap[(size_t)d] = pow2_at_least(2ull * std::min<uint64_t>(nmsg[(size_t)d], MT_MAX_CLIENTS) + 1);
            cl_base[(size_t)d] = csum;
            csum += cl_cap[(size_t)d];
        }
        uint64_t *d_clb = nullptr;
        uint32_t *d_clc = nullptr;
        JGCHK(B.get(&P.cl_ht, (size_t)std::max<uint64_t>(csum, 1)));
        JGCHK(hipMemsetAsync(P.cl_ht, 0, 4 * std::max<uint64_t>(csum, 1), s));
        JGCHK(B.get(&d_clb, (size_t)D));
        JGCHK(B.get(&d_clc, (size_t)D));
        if (D) {
            JGCHK(hipMemcpyAsync(d_clb, cl_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice, s));
            JGCHK(hipMemcpyAsync(d_clc, cl_cap.data(), 4 * (size_t)D, hipMemcpyHostToDevice, s));
        }
        P.cl_base = d_clb;
        P.cl_cap = d_clc;
    }
    JGCHK(hipEventRecord(ev[2], s));
    if (D) JGCHK(hipLaunchKernel((const void *)jg_clients_kernel, dim3(grid), dim3(64), argc, 0, s));
    JGCHK(hipEventRecord(ev[3], s));
    std::vector<uint32_t> fail, nrec, ntext, nprop, npops, nval;
    JGCHK(dl(fail, P.d_fail, (size_t)D, s));
    for (int64_t d = 0; d < D; d++)
        if (fail[(size_t)d]) {
            res.status = MT_UNSUPPORTED;
            res.bad_doc = d;
            res.fail_bits = fail[(size_t)d];
            return MT_UNSUPPORTED;
        }
    JGCHK(dl(nrec, P.d_nrec, (size_t)D, s));
    JGCHK(dl(ntext, P.d_ntext, (size_t)D, s));
    JGCHK(dl(nprop, P.d_nprop, (size_t)D, s));
    JGCHK(dl(npops, P.d_npropops, (size_t)D, s));
    JGCHK(dl(nval, P.d_nval, (size_t)D, s));
    // batch layout: records and prop records back to back in document order
    res.doc_op_off.assign((size_t)D + 1, 0);
    std::vector<int64_t> op_base((size_t)D);
    std::vector<uint32_t> prop_base((size_t)D), val_base((size_t)D), text_pay((size_t)D);
    std::vector<uint64_t> text_dst((size_t)D);
    uint64_t tp = 0, pp = 0, vp = 0;
    for (int64_t d = 0; d < D; d++) {
        op_base[(size_t)d] = res.doc_op_off[(size_t)d];
        res.doc_op_off[(size_t)d + 1] = res.doc_op_off[(size_t)d] + nrec[(size_t)d];
        prop_base[(size_t)d] = (uint32_t)pp;
        val_base[(size_t)d] = (uint32_t)vp;
        vp += nval[(size_t)d];
        text_pay[(size_t)d] = (uint32_t)tp;
        text_dst[(size_t)d] = tp;
        tp += ntext[(size_t)d];
        pp += nprop[(size_t)d];
        res.n_msgs += nmsg[(size_t)d];
    }
    if (tp > 0xFFFFFFF0ull || pp > 0x7FFFFFF0ull || vp > 0x7FFFFFF0ull) return MT_ERR_ARG;
    res.n_ops = res.doc_op_off[(size_t)D];
    res.n_text = (int64_t)tp;
    res.n_props = (int64_t)pp;
    res.doc_text = ntext;
    res.doc_nprop_ops = npops;
    res.doc_nprops = nprop;
    uint64_t words = tp;
    if (install) {
        int rc = (*install)(res, text_dst, words);
        if (rc) return rc;
        std::fill(text_pay.begin(), text_pay.end(), 0u);
    }
    mt_op *d_ops = nullptr;
    uint16_t *d_text = nullptr;
    mt_prop *d_props = nullptr;
    if (hipMalloc((void **)&d_ops, std::max<size_t>((size_t)res.n_ops, 1) * sizeof(mt_op)) != hipSuccess)
        return MT_ERR_HIP;
    if (hipMalloc((void **)&d_text, std::max<uint64_t>(words, 1) * 2) != hipSuccess ||
        hipMalloc((void **)&d_props, std::max<uint64_t>(pp, 1) * sizeof(mt_prop)) != hipSuccess) {
        (void)hipFree(d_ops);
        (void)hipFree(d_text);
        return MT_ERR_HIP;
    }
    *d_ops_out = d_ops;
    *d_text_out = d_text;
    *d_props_out = d_props;
    *text_words = words;
    JGCHK(hipMemsetAsync(d_text, 0, std::max<uint64_t>(words, 1) * 2, s));
    P.ops = d_ops;
    P.text = d_text;
    P.props = d_props;
    P.install = install != nullptr;
    int64_t *d_opb = nullptr;
    uint64_t *d_tdst = nullptr;
    uint32_t *d_tpay = nullptr, *d_pb = nullptr, *d_vb = nullptr;
    JGCHK(B.get(&d_opb, (size_t)D));
    JGCHK(B.get(&d_tdst, (size_t)D));
    JGCHK(B.get(&d_tpay, (size_t)D));
    JGCHK(B.get(&d_pb, (size_t)D));
    JGCHK(B.get(&d_vb, (size_t)D));
    JGCHK(hipMemcpyAsync(d_opb, op_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice, s));
    JGCHK(hipMemcpyAsync(d_tdst, text_dst.data(), 8 * (size_t)D, hipMemcpyHostToDevice, s));
    JGCHK(hipMemcpyAsync(d_tpay, text_pay.data(), 4 * (size_t)D, hipMemcpyHostToDevice, s));
    JGCHK(hipMemcpyAsync(d_pb, prop_base.data(), 4 * (size_t)D, hipMemcpyHostToDevice, s));
    JGCHK(hipMemcpyAsync(d_vb, val_base.data(), 4 * (size_t)D, hipMemcpyHostToDevice, s));
    P.op_base = d_opb;
    P.text_dst = d_tdst;
    P.text_pay = d_tpay;
    P.prop_base = d_pb;
    P.val_base = d_vb;
    uint32_t **parr[] = {&P.pk_off, &P.pk_len, &P.lk, &P.uk_off, &P.uk_len, &P.pe};
    for (uint32_t **a : parr) JGCHK(B.get(a, (size_t)pp));
    uint32_t **varr[] = {&P.pv_off, &P.pv_len, &P.lv, &P.uv_off, &P.uv_len};
    for (uint32_t **a : varr) JGCHK(B.get(a, (size_t)vp));
    // prop hash tables: per document two tables of a power of two > 2 x its records
    std::vector<uint64_t> ht_base((size_t)D);
    std::vector<uint32_t> ht_cap((size_t)D);
    uint64_t hsum = 0;
    for (int64_t d = 0; d < D; d++) {
        ht_cap[(size_t)d] = pow2_at_least(2ull * std::max(nprop[(size_t)d], nval[(size_t)d]) + 1);
        ht_base[(size_t)d] = hsum;
        hsum += 2ull * ht_cap[(size_t)d];
    }
    uint64_t *d_htb = nullptr;
    uint32_t *d_htc = nullptr;
    JGCHK(B.get(&P.ht, (size_t)hsum));
    JGCHK(hipMemsetAsync(P.ht, 0, 4 * std::max<uint64_t>(hsum, 1), s));
    JGCHK(B.get(&d_htb, (size_t)D));
    JGCHK(B.get(&d_htc, (size_t)D));
    JGCHK(hipMemcpyAsync(d_htb, ht_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice, s));
    JGCHK(hipMemcpyAsync(d_htc, ht_cap.data(), 4 * (size_t)D, hipMemcpyHostToDevice, s));
    P.ht_base = d_htb;
    P.ht_cap = d_htc;
    void *args2[] = {&P};
    if (cgrid) JGCHK(hipLaunchKernel((const void *)jg_write_kernel, dim3(cgrid), dim3(64), args2, 0, s));
    JGCHK(hipEventRecord(ev[4], s));
    if (D) JGCHK(hipLaunchKernel((const void *)jg_props_kernel, dim3(grid), dim3(64), args2, 0, s));
    // host: batch-wide tables in first-appearance order (document order, then record order)
    std::vector<uint32_t> nuk, nuv, uko, ukl, uvo, uvl, nnames;
    JGCHK(dl(nuk, P.d_nuk, (size_t)D, s));
    JGCHK(dl(nuv, P.d_nuv, (size_t)D, s));
    JGCHK(dl(uko, P.uk_off, (size_t)pp, s));
    JGCHK(dl(ukl, P.uk_len, (size_t)pp, s));
    JGCHK(dl(uvo, P.uv_off, (size_t)vp, s));
    JGCHK(dl(uvl, P.uv_len, (size_t)vp, s));
    JGCHK(dl(nnames, P.d_nnames, (size_t)D, s));
    {
        std::vector<uint32_t> wr;
        JGCHK(dl(wr, P.d_writer, (size_t)D, s));
        res.writer = std::any_of(wr.begin(), wr.end(), [](uint32_t x) { return x != 0; });
    }
    std::vector<uint64_t> names_base((size_t)D);
    uint64_t nsum = 0;
    for (int64_t d = 0; d < D; d++) {
        names_base[(size_t)d] = nsum;
        nsum += 2ull * (nnames[(size_t)d] > 0 ? nnames[(size_t)d] - 1 : 0);
    }
    std::vector<uint32_t> names;
    {
        uint64_t *d_nb = nullptr;
        JGCHK(B.get(&P.names, (size_t)std::max<uint64_t>(nsum, 1)));
        JGCHK(B.get(&d_nb, (size_t)D));
        if (D) JGCHK(hipMemcpyAsync(d_nb, names_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice, s));
        P.names_base = d_nb;
        void *argn[] = {&P};
        if (D) JGCHK(hipLaunchKernel((const void *)jg_names_kernel, dim3(grid), dim3(64), argn, 0, s));
        JGCHK(dl(names, P.names, (size_t)nsum, s));  // names' spans by id - 1, document after document
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<uint32_t> kmap((size_t)std::max<uint64_t>(pp, 1)), vmap((size_t)std::max<uint64_t>(vp, 1));
    std::unordered_map<std::string, uint32_t> kid, vid{{"null", 0u}};
    res.values.assign(1, "null");
    res.clients.resize((size_t)D);
    for (int64_t d = 0; d < D; d++) {
        const char *js = h_json + doc_off[d];
        const uint32_t pb = prop_base[(size_t)d];
        for (uint32_t i = 0; i < nuk[(size_t)d]; i++) {
            std::string k(js + uko[pb + i], ukl[pb + i]);
            auto it = kid.find(k);
            if (it == kid.end()) {
                it = kid.emplace(k, (uint32_t)res.keys.size()).first;
                res.keys.push_back(k);
            }
            kmap[pb + i] = it->second;
        }
        const uint32_t vb = val_base[(size_t)d];
        for (uint32_t i = 0; i < nuv[(size_t)d]; i++) {
            std::string v(js + uvo[vb + i], uvl[vb + i] & ~kSpanCanon);
            if (uvl[vb + i] & kSpanCanon) {  // not in JSON.stringify form: JSON.stringify(JSON.parse(v))
                std::string cv;
                if (!json_canonical_value(v.data(), v.size(), cv)) {
                    res.status = MT_UNSUPPORTED;
                    res.bad_doc = d;
                    res.fail_bits = kFSyntax;
                    return MT_UNSUPPORTED;
                }
                v.swap(cv);
            }
            auto it = vid.find(v);
            if (it == vid.end()) {
                it = vid.emplace(v, (uint32_t)res.values.size()).first;
                res.values.push_back(v);
            }
            vmap[vb + i] = it->second;
        }
        auto &nm = res.clients[(size_t)d];
        nm.assign(1, obs);
        const uint32_t *nd = names.data() + names_base[(size_t)d];
        for (uint32_t i = 1; i < nnames[(size_t)d]; i++) {
            const uint32_t o = nd[2 * (i - 1)];
            nm.push_back(o == kNullSpan ? std::string("null") : std::string(js + o, nd[2 * (i - 1) + 1]));
        }
    }
    res.ms_host = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    uint32_t *d_km = nullptr, *d_vm = nullptr;
    JGCHK(B.get(&d_km, kmap.size()));
    JGCHK(B.get(&d_vm, vmap.size()));
    JGCHK(hipMemcpyAsync(d_km, kmap.data(), 4 * kmap.size(), hipMemcpyHostToDevice, s));
    JGCHK(hipMemcpyAsync(d_vm, vmap.data(), 4 * vmap.size(), hipMemcpyHostToDevice, s));
    P.kmap = d_km;
    P.vmap = d_vm;
    void *args3[] = {&P};
    if (D) JGCHK(hipLaunchKernel((const void *)jg_remap_kernel, dim3(grid), dim3(64), args3, 0, s));
    JGCHK(hipEventRecord(ev[5], s));
    JGCHK(hipStreamSynchronize(s));
    JGCHK(hipEventElapsedTime(&res.ms_scan, ev[0], ev[1]));
    JGCHK(hipEventElapsedTime(&res.ms_count, ev[1], ev[2]));
    JGCHK(hipEventElapsedTime(&res.ms_clients, ev[2], ev[3]));
    JGCHK(hipEventElapsedTime(&res.ms_write, ev[3], ev[4]));
    JGCHK(hipEventElapsedTime(&res.ms_props, ev[4], ev[5]));
    res.status = MT_OK;
    return MT_OK;
}

// Writer logs parsed here: the most unacked local ops any replica holds (its local records less
// the acks, its own sequenced records, before them, at the peak), for the pending-group region
// (mt_host.cpp writer_regions).  One lane per document, serial over its records.
extern "C" __global__ __launch_bounds__(64) void jg_pending_peak_kernel(const mt_op *ops, const int64_t *off, int64_t D,
                                                                        unsigned long long *peak) {
    const int64_t d = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (d >= D) return;
    int64_t pend = 0, mx = 0;
    for (int64_t i = off[d]; i < off[d + 1]; i++) {
        const mt_op o = ops[i];
        if (o.seq == MT_SEQ_LOCAL) mx = max(mx, ++pend);
        else if (o.seq > 0 && MT_OP_CLIENT(o) == 0 && pend > 0) pend--;
    }
    if (mx) atomicMax(peak, (unsigned long long)mx);
}

int pending_peak(const mt_op *d_ops, const int64_t *d_off, int64_t D, void *stream, int64_t *out) {
    *out = 0;
    if (D <= 0) return MT_OK;
    hipStream_t s = (hipStream_t)stream;
    unsigned long long *d_peak = nullptr, h = 0;
    JGCHK(hipMalloc(&d_peak, 8));
    int rc = MT_OK;
    const unsigned grid = (unsigned)((D + 63) / 64);
    void *args[] = {&d_ops, &d_off, &D, &d_peak};
    if (hipMemsetAsync(d_peak, 0, 8, s) != hipSuccess ||
        hipLaunchKernel((const void *)jg_pending_peak_kernel, dim3(grid), dim3(64), args, 0, s) != hipSuccess ||
        hipMemcpyAsync(&h, d_peak, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        rc = MT_ERR_HIP;
    (void)hipFree(d_peak);
    *out = (int64_t)h;
    return rc;
}

}  // namespace jg
}  // namespace mt
