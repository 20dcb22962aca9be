// mt_digest.hip — per-document digest of the final device state, computed on the GPU.
//
// One wavefront per document hashes the document's final segment table (mt::OutRec records
// in document order, leaf-block end markers included), each record together with its text
// code units and its prop-set contents, and the collab-window scalars.  It is the 8-byte
// per-document fingerprint that bench.py gathers to rank 0 over RCCL: it needs
// no host serialization, depends only on the op log (slot and block ids do not enter), and so
// is identical for a document whichever rank / launch / capacity class replayed it.
#include <hip/hip_runtime.h>

#include "../../include/mt_oplog.h"
#include "mt_device.h"

namespace mt {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finalizer
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}
__device__ __forceinline__ uint64_t fnv(uint64_t h, uint32_t w) {
    h ^= w;
    return h * 0x100000001B3ull;
}


// the client ids and the Marker bit as one word: clientId | removedClientId << 8 | Marker << 16 in
// the 8-bit encoding of the first engines (254 NonCollabClient, 255 none) for ids below 254, so the
// digests of such documents are unchanged; the ids from 254 to 4095 add their high bits above bit 16
__device__ __forceinline__ uint32_t id_enc(uint32_t id) {
    if (id == MT_CLIENT_NONCOLLAB) return 254u;
    if (id == kNoClient) return 255u;
    return id < 254u ? id : ((id & 0xFFu) | 0x100u | ((id >> 8) << 9));
}
__device__ __forceinline__ uint32_t id_word(uint32_t cli, uint32_t rcli, bool marker) {
    const uint32_t a = id_enc(cli), b = id_enc(rcli);
    return (a & 0xFFu) | ((b & 0xFFu) << 8) | (marker ? 1u << 16 : 0u) | ((a >> 8) << 17) | ((b >> 8) << 22);
}

extern "C" __global__ __launch_bounds__(64) void mt_digest_kernel(DigestParams P) {
    const int64_t w = blockIdx.x;
    if (w >= P.n) return;
    // a document checkpointed or re-run in a later launch gets its digest from that launch; the
    // launch holding its final result always writes one (also for a terminal MT_CAPACITY: no
    // records, the status enters the hash)
    if (!P.final_mask[w]) return;
    const DocOut o = P.doc_out[w];
    const int64_t d = P.doc_list ? P.doc_list[w] : w;
    const OutRec *rec = P.out + w * (int64_t)P.out_cap;
    const uint16_t *text = P.text + P.doc_text_base[d];
    const uint32_t *pool = P.pool + P.doc_pool_base[d];
    uint64_t acc = 0;
    for (int32_t i = threadIdx.x; i < o.n_out; i += 64) {
        const OutRec r = rec[i];
        uint64_t h = 0xCBF29CE484222325ull;
        if (out_is_end(r.blk)) {
            h = fnv(h, 0xB10CB10Cu);
        } else {
            h = fnv(h, r.len);
            h = fnv(h, (uint32_t)r.seq);
            h = fnv(h, (uint32_t)r.rseq);
            const uint32_t ci = meta_cli(r.meta), ri = meta_rcli(r.meta);
            h = fnv(h, id_word(ci, ri, (r.meta & kMetaMarker) != 0u));  // client ids, Marker
            // 15-bit ids beyond the first engines' 12-bit range add a word (digests of documents with
            // fewer clients are unchanged)
            if ((ci >= 4096u && ci != MT_CLIENT_NONCOLLAB && ci != kNoClient) ||
                (ri >= 4096u && ri != MT_CLIENT_NONCOLLAB && ri != kNoClient))
                h = fnv(h, ci | ri << 16);
            // removedClientOverlap as a set (mask of clients < 31, or a pool list)
            uint64_t ov = 0;
            if (r.ovl & kOvlList) {
                const uint32_t *l = pool + (r.ovl & ~kOvlList);
                const uint32_t n = l[0] & ~kPoolOvlTag;
                for (uint32_t k = 0; k < n; k++) ov += mix64(l[2 + k] + 1ull);
            } else {
                for (uint32_t m = r.ovl; m; m &= m - 1) ov += mix64((uint32_t)__builtin_ctz(m) + 1ull);
            }
            h = fnv(h, (uint32_t)ov);
            if (r.meta & kMetaMarker) {
                h = fnv(h, r.toff);  // refType
            } else {
                for (uint32_t k = 0; k < r.len; k++) h = fnv(h, text[r.toff + k]);
            }
            if (r.props) {
                const uint32_t np = pool[r.props];
                h = fnv(h, np);
                uint64_t ps = 0;  // key order does not matter to matchProperties
                for (uint32_t k = 0; k < np; k++)
                    ps += mix64(((uint64_t)pool[r.props + 2 + 2 * k] << 32) | pool[r.props + 3 + 2 * k]);
                h = fnv(h, (uint32_t)ps);
                h = fnv(h, (uint32_t)(ps >> 32));
            } else {
                h = fnv(h, 0xFFFFFFFFu);
            }
        }
        acc += mix64(h + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1));
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (threadIdx.x == 0) {
        uint64_t h = mix64(acc ^ 0x6D74646967657374ull);
        h = mix64(h + ((uint64_t)(uint32_t)o.depth << 32 | (uint32_t)o.n_out));
        h = mix64(h + ((uint64_t)(uint32_t)o.min_seq << 32 | (uint32_t)o.cur_seq));
        h = mix64(h + (uint64_t)(uint32_t)o.status);
        P.dst[d] = h;
    }
}

}  // namespace mt

namespace mt {

// 64-bit digest of each document's byte range [off, off + len) of a buffer (the GPU SnapshotV1
// blobs): mix64(len-seeded state ^ sum over 8-byte little-endian words k of
// mix64(word_k + (k + 1) * golden)), the last word zero-padded.  Order-dependent through k,
// lane-parallel.  Documents with len < 0 (not serialized on the GPU) get 0.  The buffer must
// be readable 8 bytes past its last range (the host pads the allocation).
extern "C" __global__ __launch_bounds__(64) void mt_bytes_digest_kernel(const uint8_t *buf, const int64_t *off,
                                                                      const int64_t *len, int64_t n, uint64_t *dst) {
    const int64_t d = blockIdx.x;
    if (d >= n) return;
    const int64_t L = len[d];
    if (L < 0) {
        if (threadIdx.x == 0) dst[d] = 0;
        return;
    }
    const int64_t o = off[d];
    const uint64_t *w64 = reinterpret_cast<const uint64_t *>(buf);
    uint64_t acc = 0;
    const int64_t nw = (L + 7) / 8;
    for (int64_t k = threadIdx.x; k < nw; k += 64) {
        const int64_t b = o + 8 * k;
        const int64_t q = b >> 3;
        const uint32_t sh = (uint32_t)(b & 7) * 8;
        uint64_t w = w64[q];
        if (sh) w = (w >> sh) | (w64[q + 1] << (64 - sh));
        const int64_t rem = L - 8 * k;
        if (rem < 8) w &= (1ull << (8 * rem)) - 1;
        acc += mix64(w + 0x9E3779B97F4A7C15ull * (uint64_t)(k + 1));
    }
    for (int s = 32; s > 0; s >>= 1) acc += __shfl_xor(acc, s, 64);
    if (threadIdx.x == 0) dst[d] = mix64(mix64((uint64_t)L ^ 0x736E617073686F74ull) ^ acc);
}

}  // namespace mt
