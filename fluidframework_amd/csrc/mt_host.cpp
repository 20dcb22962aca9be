// mt_host.cpp — host side of libmtreplay.so: the C ABI declared in include/mtreplay.h.
//
// Owns a batch of documents on one HIP device: stages packed op logs into per-document
// HBM regions, launches the replay kernels (mt_kernels.hip, one object per capacity class), escalates
// documents that overflow their LDS capacity class, and serializes per-document results
// (text, properties, SnapshotV1 blobs, digest) from the device's final segment tables.
//
// Nothing here replays ops: every op is applied by mt_replay_kernel on the GPU.  Without a
// usable HIP device mt_batch_create fails with MT_ERR_NO_DEVICE (there is no CPU path).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <atomic>
#include <vector>

#include "../../include/mtreplay.h"
#include "mt_device.h"
#include "mt_json_gpu.h"
#include "mt_values.h"

// kernels of each capacity class (mt_kernels.hip compiled with -DMT_SEG=<seg>)
#define MT_DECLARE_CLASS(S)                                                   \
    extern "C" __global__ void mt_replay_kernel_##S(mt::ReplayParams P);      \
    extern "C" __global__ void mt_writer_kernel_##S(mt::ReplayParams P);      \
    extern "C" __global__ void mt_bigprops_kernel_##S(mt::ReplayParams P);    \
    extern "C" __global__ void mt_load_kernel_##S(mt::ReplayParams P);        \
    extern "C" __global__ void mt_generate_kernel_##S(mt::ReplayParams P);
MT_CLASS_LIST(MT_DECLARE_CLASS)
extern "C" __global__ void mt_digest_kernel(mt::DigestParams P);
extern "C" __global__ void jg_markers_kernel(const mt_op *ops, const int64_t *op_off, mt_op *ops_w, const mt_prop *props,
                                             int64_t D, uint32_t mk_key, uint32_t tile_key, uint32_t range_key,
                                             const uint32_t *vkey,
                                             uint32_t n_values, uint32_t *n_ids, uint32_t *tile_annot);
extern "C" __global__ void mt_snapshot_kernel(mt::SnapParams P);
extern "C" __global__ void mt_snapshot_size_kernel(mt::SnapParams P);
extern "C" __global__ void mt_snapshot_serial_kernel(mt::SnapParams P);
extern "C" __global__ void mt_bytes_digest_kernel(const uint8_t *buf, const int64_t *off, const int64_t *len, int64_t n,
                                                  uint64_t *dst);

using mt::Caps;
using mt::DocOut;
using mt::OutRec;

namespace {

#define HIPCHK(x)                                                                                 \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "mtreplay: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                                    \
            return MT_ERR_HIP;                                                                    \
        }                                                                                         \
    } while (0)

template <class T>
static hipError_t dalloc(T **p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    return hipMalloc((void **)p, n * sizeof(T));
}

struct KernelClass {
    int seg;
    const void *replay;
    const void *generate;
    const void *load;
    const void *writer;    // replay + the local-client path (writer replicas)
    const void *bigprops;  // the observer replay with property sets of any size (mt_device.h kCapPool)
};
#define MT_KERNEL_CLASS_(S) {S, (const void *)mt_replay_kernel_##S, (const void *)mt_generate_kernel_##S, \
                             (const void *)mt_load_kernel_##S, (const void *)mt_writer_kernel_##S,    \
                             (const void *)mt_bigprops_kernel_##S},
static const KernelClass kKernels[mt::kNumClasses] = {MT_CLASS_LIST(MT_KERNEL_CLASS_)};
#undef MT_KERNEL_CLASS_
constexpr size_t kGenStaticLds = 256;  // generate_body's lref[64]

struct Launch {
    std::vector<int32_t> docs;  // empty: identity over all docs
    int cls = 0;                // index into kKernels
    Caps caps;
    int32_t out_cap = 0;
    OutRec *d_out = nullptr;
    uint32_t *d_lab = nullptr;   // label tracking: per record, a marker's labels snapshot (ReplayParams.lab_out)
    DocOut *d_docout = nullptr;
    int32_t *d_list = nullptr;
    uint64_t *d_prof = nullptr;  // MT_PROF builds
    uint4 *d_cold = nullptr;     // per-document cold segment records (class stride)
    uint32_t *d_ck = nullptr;    // checkpoints of documents short of LDS headroom
    int32_t *d_cksrc = nullptr;  // resume: per workgroup index into the previous launch (-1 fresh)
    uint8_t *d_state = nullptr;  // HBM class: per-workgroup table images
    std::vector<int32_t> cksrc;
    int src = -1;               // launch whose checkpoints / cold records cksrc indexes
    size_t lds = 0;
    float ms = 0;               // device time (hipEvents)
    int64_t ops = 0;            // ops applied by this launch (resumed documents: after their checkpoint)
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int level = 0;              // escalation depth (0: a first launch)
    int stream = 0;             // 0: the run stream, 1..3: aux stream k - 1, 4..5: early stream k - 4
    bool load = false;          // SnapshotLoader launch (mt_load_kernel): LOAD records, then a checkpoint
    bool big = false;           // observer documents with large property sets: mt_bigprops_kernel_<SEG>
    bool notice = false;        // appends early-escalation entries (mt_batch.h_notice)
    bool gathered = false;      // its results are gathered: later entries of it are not taken
    bool urgent = false;        // an early escalation (ReplayParams.urgent)
    int64_t early_ops = 0;      // ops of its documents that escalated early (poll_notices)
};

// workgroups (documents) of a launch
static int64_t launch_n(int64_t n_docs, const Launch &L) {
    return L.docs.empty() ? n_docs : (int64_t)L.docs.size();
}

struct DocRes {  // per-document result location
    int32_t launch = -1;
    int32_t idx = -1;
};

// ---------------------------------------------------------------- JSON helpers (JS semantics)
static void put_cp(std::string &o, uint32_t cp) {
    if (cp < 0x80) {
        o.push_back((char)cp);
    } else if (cp < 0x800) {
        o.push_back((char)(0xC0 | (cp >> 6)));
        o.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
        o.push_back((char)(0xE0 | (cp >> 12)));
        o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
        o.push_back((char)(0xF0 | (cp >> 18)));
        o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
        o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        o.push_back((char)(0x80 | (cp & 0x3F)));
    }
}

// UTF-16 -> UTF-8 (raw text; lone surrogates become U+FFFD)
static void utf16_to_utf8(std::string &o, const uint16_t *s, size_t n) {
    for (size_t i = 0; i < n; i++) {
        uint32_t c = s[i];
        if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
            put_cp(o, 0x10000 + ((c - 0xD800) << 10) + (uint32_t)(s[i + 1] - 0xDC00));
            i++;
        } else if (c >= 0xD800 && c <= 0xDFFF) {
            put_cp(o, 0xFFFD);
        } else {
            put_cp(o, c);
        }
    }
}

// JSON.stringify(string) of UTF-16 code units (well-formed: lone surrogates escaped)
static void json_quote16(std::string &o, const uint16_t *s, size_t n) {
    static const char *hex = "0123456789abcdef";
    o.push_back('"');
    for (size_t i = 0; i < n; i++) {
        uint32_t c = s[i];
        switch (c) {
            case 0x22: o += "\\\""; continue;
            case 0x5C: o += "\\\\"; continue;
            case 0x08: o += "\\b"; continue;
            case 0x0C: o += "\\f"; continue;
            case 0x0A: o += "\\n"; continue;
            case 0x0D: o += "\\r"; continue;
            case 0x09: o += "\\t"; continue;
            default: break;
        }
        if (c < 0x20) {
            o += "\\u00";
            o.push_back(hex[c >> 4]);
            o.push_back(hex[c & 15]);
        } else if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
            put_cp(o, 0x10000 + ((c - 0xD800) << 10) + (uint32_t)(s[i + 1] - 0xDC00));
            i++;
        } else if (c >= 0xD800 && c <= 0xDFFF) {
            o += "\\u";
            o.push_back(hex[c >> 12]);
            o.push_back(hex[(c >> 8) & 15]);
            o.push_back(hex[(c >> 4) & 15]);
            o.push_back(hex[c & 15]);
        } else {
            put_cp(o, c);
        }
    }
    o.push_back('"');
}

static std::vector<uint16_t> utf8_to_utf16(const std::string &s) {
    std::vector<uint16_t> out;
    size_t i = 0, L = s.size();
    const unsigned char *q = (const unsigned char *)s.data();
    while (i < L) {
        uint32_t c = q[i];
        int len = 1;
        if (c < 0x80) len = 1;
        else if ((c & 0xE0) == 0xC0) { len = 2; c &= 0x1F; }
        else if ((c & 0xF0) == 0xE0) { len = 3; c &= 0x0F; }
        else if ((c & 0xF8) == 0xF0) { len = 4; c &= 0x07; }
        else { out.push_back(0xFFFD); i++; continue; }
        if (i + (size_t)len > L) { out.push_back(0xFFFD); break; }
        bool bad = false;
        for (int m = 1; m < len; m++) {
            if ((q[i + m] & 0xC0) != 0x80) { bad = true; break; }
            c = (c << 6) | (q[i + m] & 0x3F);
        }
        if (bad) { out.push_back(0xFFFD); i++; continue; }
        i += (size_t)len;
        if (c >= 0x10000) {
            c -= 0x10000;
            out.push_back((uint16_t)(0xD800 + (c >> 10)));
            out.push_back((uint16_t)(0xDC00 + (c & 0x3FF)));
        } else {
            out.push_back((uint16_t)c);
        }
    }
    return out;
}

static void json_quote8(std::string &o, const std::string &s) {
    std::vector<uint16_t> u = utf8_to_utf16(s);
    json_quote16(o, u.data(), u.size());
}

// canonical array index (ordinary-object key enumeration puts these first, ascending)
static bool array_index(const std::string &k, uint32_t *idx) {
    if (k.empty() || k.size() > 10) return false;
    if (k[0] == '0') {
        if (k.size() != 1) return false;
        *idx = 0;
        return true;
    }
    uint64_t v = 0;
    for (char ch : k) {
        if (ch < '0' || ch > '9') return false;
        v = v * 10 + (uint64_t)(ch - '0');
    }
    if (v > 4294967294ull) return false;
    *idx = (uint32_t)v;
    return true;
}

static bool json_falsy(const std::string &v) {
    size_t a = v.find_first_not_of(" \t\r\n"), b = v.find_last_not_of(" \t\r\n");
    if (a == std::string::npos) return true;
    std::string t = v.substr(a, b - a + 1);
    if (t == "null" || t == "false" || t == "\"\"") return true;
    if (!t.empty() && (t[0] == '-' || (t[0] >= '0' && t[0] <= '9'))) {
        char *end = nullptr;
        double d = strtod(t.c_str(), &end);
        if (end && *end == 0 && d == 0.0) return true;
    }
    return false;
}

struct Fnv {
    uint64_t h = 0xcbf29ce484222325ull;
    void bytes(const void *p, size_t n) {
        const unsigned char *q = (const unsigned char *)p;
        for (size_t i = 0; i < n; i++) {
            h ^= q[i];
            h *= 0x100000001b3ull;
        }
    }
    void u32(uint32_t x) {
        unsigned char b[4] = {(unsigned char)x, (unsigned char)(x >> 8), (unsigned char)(x >> 16),
                              (unsigned char)(x >> 24)};
        bytes(b, 4);
    }
    void u64(uint64_t x) {
        u32((uint32_t)x);
        u32((uint32_t)(x >> 32));
    }
};
static uint64_t fnv_name(const std::string &s) {
    Fnv f;
    f.bytes(s.data(), s.size());
    return f.h;
}

}  // namespace

// ---------------------------------------------------------------- batch
struct mt_batch {
    int device = 0;
    hipStream_t stream = nullptr;
    // launch buffers of finished runs, by size, for the next run's launches (lbuf_alloc): a step
    // replays the same launch shapes, and a hipMalloc of the GBs a class launch holds costs tens of
    // ms of host time between a launch and its escalation
    std::multimap<size_t, void *> buf_cache;
    std::map<void *, size_t> buf_bytes;  // every cached-allocator buffer's size
    int64_t n_docs = 0;
    mt_batch_options opt{};
    // tables
    std::vector<std::string> keys, values;
    std::vector<uint8_t> key_is_index;
    std::vector<uint32_t> key_index;
    std::vector<uint8_t> value_flags;
    std::vector<uint32_t> value_class;  // structural matchProperties classes (mt_values.cpp)
    std::vector<uint64_t> value_exc;    // sorted cross-class matches (u << 32 | v)
    // values [0, n_user_values) are the caller's table (mt_batch_set_tables); the ingest appends
    // the results of combiningOps (combine_absent: NaN, consensus values, ...) after them
    size_t n_user_values = 1;
    uint32_t nan_id = 0xFFFFFFFFu;  // the derived NaN value (kValNever | kValNum), if any
    std::vector<std::string> clients;  // shared table
    std::unordered_map<int64_t, std::vector<std::string>> doc_clients;
    // log (device) + host mirror of the layout
    bool have_log = false, generated = false;
    // writer replicas (the log has local ops / own acks): mt_writer_kernel_<SEG> and per-document
    // pending-group regions (mt_device.h pend_words)
    bool writer = false;
    int32_t pend_cap = 0;
    int32_t regen_cap = 0;               // words per document of regenerated-op output
    uint32_t *d_regen = nullptr;
    uint64_t *d_regen_base = nullptr;
    uint32_t *d_cons = nullptr;          // writer consensus regions (mt_device.h kConsHdr); null: none
    uint64_t *d_cons_base = nullptr;
    std::vector<uint64_t> h_cons_base;
    std::vector<mt_prop> h_props_all;    // the ingested prop records (regenerated annotates' props)
    std::vector<uint64_t> h_regen_base;
    uint32_t *d_pend = nullptr;
    uint64_t *d_pend_base = nullptr;
    int64_t total_ops = 0, total_props = 0;
    int32_t max_ops_per_doc = 0;
    std::vector<int64_t> h_off;
    std::vector<int32_t> h_nload, h_nload_segs;  // leading SnapshotLoader records / segments per doc
    std::vector<uint8_t> h_tile_annot;  // per doc: an annotate touches referenceTileLabels (1) / referenceRangeLabels (2)
    bool lab_track = false;             // some document's annotates touch them: the replay tracks labels snapshots
    std::vector<uint64_t> h_text_base, h_pool_base;
    std::vector<uint32_t> h_text_len, h_text_cap, h_pool_cap;
    // MT_OP_RELPOS records hold marker-id keys on the device (resolve_marker_ids); key_value[k] is a
    // value id whose String() is key k, so mt_batch_download_log returns value ids again (a log
    // that re-ingests to the same keys)
    std::vector<uint32_t> key_value;
    uint64_t text_words = 0, pool_words = 0;
    mt_op *d_ops = nullptr;
    int64_t *d_off = nullptr;
    uint16_t *d_text = nullptr;
    uint64_t *d_text_base = nullptr, *d_pool_base = nullptr;
    uint2 *d_idmap = nullptr;          // per-document marker-id maps (mt_device.h ReplayParams.idmap)
    uint64_t *d_idmap_base = nullptr;
    uint32_t *d_text_len = nullptr, *d_text_cap = nullptr, *d_pool_cap = nullptr;
    uint32_t *d_pool = nullptr;
    mt_prop *d_props = nullptr;
    uint8_t *d_vflags = nullptr;
    uint32_t *d_vclass = nullptr;
    uint64_t *d_vexc = nullptr;
    mt::ValueTables *d_vt = nullptr;  // {d_vflags, d_vclass, d_vexc, counts} for the kernels
    double payload_units = 0, prop_records = 0;
    // launches / results
    std::vector<Launch> launches;
    std::vector<DocRes> where;
    std::vector<DocOut> docout;  // gathered per doc
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipStream_t aux[3] = {nullptr, nullptr, nullptr};  // concurrent first launches of mixed-size batches
    hipStream_t early_s[2] = {nullptr, nullptr};        // early escalations (Launch.stream 4, 5)
    hipStream_t cstream = nullptr;  // result gathers (never queued behind a running launch)
    hipEvent_t ev_user = nullptr;
    uint64_t *d_digest = nullptr;  // mt_batch_device_digests
    float kernel_ms = 0, total_ms = 0;
    bool ran = false;
    int first0 = 0, n_first = 0;  // replay launches [first0, n_first) of mt_batch_launch; before them
                                  // the SnapshotLoader launches, after them the escalations
    hipStream_t run_stream = nullptr;
    std::chrono::steady_clock::time_point t_launch;
    // early escalation (poll_notices): a ring of 4-word entries in coherent host memory the first
    // launches append to (ReplayParams.notice), its device-side counter, the host's read cursor,
    // the documents taken from their source launch, and early groups waiting for an idle stream
    uint32_t *h_notice = nullptr;
    uint32_t *d_notice = nullptr;       // device alias of h_notice
    uint32_t *d_notice_count = nullptr;
    int64_t notice_cap = 0, notice_read = 0, notice_alloc = 0;
    std::vector<uint8_t> taken;
    std::map<int, std::map<int, Launch>> early_groups;  // by source launch, then target (cls x2 + big)
    // single-document result cache
    int64_t cached_doc = -1;
    uint64_t load_gen = 0;         // bumped whenever load_doc loads a document's results
    std::shared_ptr<void> qtree;   // the loaded document's rebuilt tree + query maps (DocTree)
    std::vector<OutRec> c_recs;
    std::vector<uint32_t> c_lab;  // label tracking: per record, the prop set of the labels snapshot
    std::vector<uint16_t> c_text;
    std::vector<uint32_t> c_pool;
    DocOut c_out{};
    std::vector<std::string> c_blob_names, c_blobs;
    int64_t c_blob_doc = -1;
    // GPU SnapshotV1 of every document (mt_batch_snapshots)
    bool snap_ready = false;
    int32_t *d_snap_meta = nullptr;
    int64_t *d_snap_bytes = nullptr, *d_snap_off = nullptr;
    uint8_t *d_snap = nullptr;
    size_t snap_cap = 0;
    uint32_t *d_snap_scratch = nullptr;  // SnapParams.rec_bytes / seg_frame of every launch
    size_t snap_scratch_cap = 0;         // (u32 words)
    int32_t *d_chunk_ext = nullptr;      // chunk triples beyond the meta row (SnapParams.chunk_ext)
    int64_t *d_chunk_ext_off = nullptr;
    size_t chunk_ext_cap = 0, chunk_ext_off_n = 0;
    std::vector<int64_t> h_chunk_ext_off;
    std::vector<int64_t> h_snap_bytes, h_snap_off;
};

static void free_snap(mt_batch *b) {
    (void)hipFree(b->d_snap_meta);
    (void)hipFree(b->d_snap_bytes);
    (void)hipFree(b->d_snap_off);
    (void)hipFree(b->d_snap);
    (void)hipFree(b->d_snap_scratch);
    b->d_snap_scratch = nullptr;
    b->snap_scratch_cap = 0;
    (void)hipFree(b->d_chunk_ext);
    (void)hipFree(b->d_chunk_ext_off);
    b->d_chunk_ext = nullptr;
    b->d_chunk_ext_off = nullptr;
    b->chunk_ext_cap = b->chunk_ext_off_n = 0;
    b->h_chunk_ext_off.clear();
    b->d_snap_meta = nullptr;
    b->d_snap_bytes = b->d_snap_off = nullptr;
    b->d_snap = nullptr;
    b->snap_cap = 0;
    b->snap_ready = false;
}

// launch buffers: a cached one of the size (within 1/8 above it), else hipMalloc (on failure the
// cache is released and the allocation retried).  Every launch writes what it reads first, so a
// reused buffer's old contents are never seen.
static void lbuf_release(mt_batch *b) {
    for (auto &kv : b->buf_cache) {
        (void)hipFree(kv.second);
        b->buf_bytes.erase(kv.second);
    }
    b->buf_cache.clear();
}
template <class T>
static hipError_t lbuf_alloc(mt_batch *b, T **p, size_t n) {
    const size_t bytes = (n ? n : 1) * sizeof(T);
    auto it = b->buf_cache.lower_bound(bytes);
    if (it != b->buf_cache.end() && it->first - bytes <= bytes / 8) {
        *p = (T *)it->second;
        b->buf_cache.erase(it);
        return hipSuccess;
    }
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, bytes);
    if (e != hipSuccess && !b->buf_cache.empty()) {
        (void)hipGetLastError();
        lbuf_release(b);
        e = hipMalloc(&q, bytes);
    }
    if (e == hipSuccess) b->buf_bytes[q] = bytes;
    *p = (T *)q;
    return e;
}
static void lbuf_free(mt_batch *b, void *p) {
    if (!p) return;
    auto it = b->buf_bytes.find(p);
    if (it == b->buf_bytes.end()) {
        (void)hipFree(p);
        return;
    }
    b->buf_cache.emplace(it->second, p);
}

static void free_launches(mt_batch *b) {
    // what the cache still holds was not taken by the run that is ending: released, so the cache
    // never holds more than one run's launch buffers
    lbuf_release(b);
    // a run that ended early (an error in mt_batch_sync, or a launch without a sync) may still have
    // kernels in flight on the aux streams: their buffers are cached only once those have finished
    for (auto &L : b->launches)
        if (L.e1) (void)hipEventSynchronize(L.e1);
    for (auto &L : b->launches) {
        lbuf_free(b, L.d_out);
        lbuf_free(b, L.d_lab);
        lbuf_free(b, L.d_docout);
        lbuf_free(b, L.d_list);
        lbuf_free(b, L.d_prof);
        lbuf_free(b, L.d_cold);
        lbuf_free(b, L.d_ck);
        lbuf_free(b, L.d_cksrc);
        lbuf_free(b, L.d_state);
        if (L.e0) (void)hipEventDestroy(L.e0);
        if (L.e1) (void)hipEventDestroy(L.e1);
    }
    b->launches.clear();
}

static void free_log(mt_batch *b) {
    lbuf_release(b);  // a new log: other launch shapes
    (void)hipFree(b->d_ops);
    (void)hipFree(b->d_off);
    (void)hipFree(b->d_text);
    (void)hipFree(b->d_text_base);
    (void)hipFree(b->d_text_len);
    (void)hipFree(b->d_text_cap);
    (void)hipFree(b->d_pool);
    (void)hipFree(b->d_pool_base);
    (void)hipFree(b->d_pool_cap);
    (void)hipFree(b->d_props);
    (void)hipFree(b->d_idmap);
    (void)hipFree(b->d_idmap_base);
    b->d_idmap = nullptr;
    b->d_idmap_base = nullptr;
    (void)hipFree(b->d_pend);
    (void)hipFree(b->d_pend_base);
    b->d_pend = nullptr;
    b->d_pend_base = nullptr;
    (void)hipFree(b->d_regen);
    (void)hipFree(b->d_regen_base);
    b->d_regen = nullptr;
    b->d_regen_base = nullptr;
    (void)hipFree(b->d_cons);
    (void)hipFree(b->d_cons_base);
    b->d_cons = nullptr;
    b->d_cons_base = nullptr;
    b->h_cons_base.clear();
    b->writer = false;
    b->d_ops = nullptr;
    b->d_off = nullptr;
    b->d_text = nullptr;
    b->d_text_base = b->d_pool_base = nullptr;
    b->d_text_len = b->d_text_cap = b->d_pool_cap = nullptr;
    b->d_pool = nullptr;
    b->d_props = nullptr;
    b->have_log = false;
}

// internal (mt_json.cpp's mt_batch_ingest_packed): an ingest that fails after it installed new
// tables leaves no log behind, so no later run can decode the previous log against the new tables
void mt_internal_drop_log(mt_batch *b) {
    free_launches(b);
    free_log(b);
    b->ran = false;
    b->cached_doc = -1;
    b->c_blob_doc = -1;
}

#ifndef MT_BUILD_ID
#define MT_BUILD_ID "MTBUILDID:unstamped000000"
#endif
static const char kBuildId[] = MT_BUILD_ID;  // "MTBUILDID:" + 16 hex digits (buildinfo.py)

extern "C" {

MT_API const char *mt_build_id(void) { return kBuildId + 10; }
MT_API int32_t mt_abi_version(void) { return MT_ABI_VERSION; }

MT_API const char *mt_status_string(int code) {
    switch (code) {
        case MT_OK: return "ok";
        case MT_INVALID_POS: return "MergeTree insert failed (invalid position)";
        case MT_SEQ_ORDER: return "sequence number order violated";
        case MT_MSN_ORDER: return "minimum sequence number order violated";
        case MT_UNSUPPORTED: return "unsupported op for the observer replay path";
        case MT_BAD_INPUT: return "bad input";
        case MT_CAPACITY: return "document exceeds device capacity";
        case MT_INTERNAL: return "internal error";
        case MT_ERR_HIP: return "HIP runtime error";
        case MT_ERR_ARG: return "invalid argument";
        case MT_ERR_STATE: return "invalid batch state";
        case MT_ERR_NO_DEVICE: return "no HIP device";
        default: return "unknown";
    }
}

MT_API int mt_batch_create(mt_batch **out, int64_t n_docs, const mt_batch_options *opts) {
    if (!out || n_docs <= 0 || n_docs > (int64_t)0x7FFFFFFF) return MT_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MT_ERR_NO_DEVICE;
    mt_batch *b = new mt_batch();
    HIPCHK(hipGetDevice(&b->device));
    b->n_docs = n_docs;
    if (opts) b->opt = *opts;
    if (b->opt.chunk_size <= 0) b->opt.chunk_size = 10000;
    if (b->opt.arena_factor <= 0) b->opt.arena_factor = 4;
    if (b->opt.pool_per_op <= 0) b->opt.pool_per_op = 96;
    // the whole class ladder (363 -> 483 -> 600 -> 840 -> ... -> HBM class) by default; < 0: checkpoint,
    // but stop after the first launch
    if (b->opt.max_retries == 0) b->opt.max_retries = 2 * mt::kNumClasses;
    if (hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&b->ev0) != hipSuccess || hipEventCreate(&b->ev1) != hipSuccess) {
        delete b;
        return MT_ERR_HIP;
    }
    b->clients = {"readonly"};
    b->values = {"null"};
    b->value_flags = {1};
    *out = b;
    return MT_OK;
}

MT_API void mt_batch_destroy(mt_batch *b) {
    if (!b) return;
    free_launches(b);
    lbuf_release(b);
    free_snap(b);
    (void)hipFree(b->d_digest);
    free_log(b);
    if (b->h_notice) (void)hipHostFree(b->h_notice);
    (void)hipFree(b->d_notice_count);
    (void)hipFree(b->d_vflags);
    (void)hipFree(b->d_vclass);
    (void)hipFree(b->d_vexc);
    (void)hipFree(b->d_vt);
    if (b->ev0) (void)hipEventDestroy(b->ev0);
    if (b->ev1) (void)hipEventDestroy(b->ev1);
    for (hipStream_t a : b->aux)
        if (a) (void)hipStreamDestroy(a);
    for (hipStream_t a : b->early_s)
        if (a) (void)hipStreamDestroy(a);
    if (b->cstream) (void)hipStreamDestroy(b->cstream);
    if (b->ev_user) (void)hipEventDestroy(b->ev_user);
    if (b->stream) (void)hipStreamDestroy(b->stream);
    delete b;
}

static int ensure_tables(mt_batch *b);

// device copies of the value tables (matchProperties classes, flags, exceptions) for the kernels
struct DeviceValueTables {
    uint8_t *flags = nullptr;
    uint32_t *cls = nullptr;
    uint64_t *exc = nullptr;
    mt::ValueTables *vt = nullptr;
    void release() {
        (void)hipFree(flags);
        (void)hipFree(cls);
        (void)hipFree(exc);
        (void)hipFree(vt);
        *this = DeviceValueTables{};
    }
};
// uploads into `t` (all or nothing: on failure `t` is released and empty)
static int upload_value_tables(const std::vector<uint8_t> &flags, const std::vector<uint32_t> &cls,
                               const std::vector<uint64_t> &exc, uint32_t nan_id, DeviceValueTables &t) {
    hipError_t e = dalloc(&t.flags, flags.size());
    if (e == hipSuccess) e = hipMemcpy(t.flags, flags.data(), flags.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = dalloc(&t.cls, cls.size());
    if (e == hipSuccess) e = hipMemcpy(t.cls, cls.data(), 4 * cls.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = dalloc(&t.exc, exc.size());
    if (e == hipSuccess && !exc.empty()) e = hipMemcpy(t.exc, exc.data(), 8 * exc.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        mt::ValueTables vt{t.flags, t.cls, t.exc, (uint32_t)flags.size(), (uint32_t)exc.size(), nan_id};
        e = dalloc(&t.vt, 1);
        if (e == hipSuccess) e = hipMemcpy(t.vt, &vt, sizeof vt, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        fprintf(stderr, "mtreplay: value table upload failed: %s\n", hipGetErrorString(e));
        t.release();
        return MT_ERR_HIP;
    }
    return MT_OK;
}

// Built and uploaded into locals first: the batch's tables change only when every step succeeded,
// so a failed call leaves the previous keys, values and device tables installed together.
MT_API int mt_batch_set_tables(mt_batch *b, const char *const *keys, int32_t n_keys, const char *const *values_json,
                               int32_t n_values) {
    if (!b || n_keys < 0 || n_values < 1 || (n_keys > 0 && !keys) || !values_json) return MT_ERR_ARG;
    std::vector<std::string> nk(keys, keys + n_keys);
    std::vector<uint8_t> is_index((size_t)n_keys, 0);
    std::vector<uint32_t> index((size_t)n_keys, 0);
    for (int i = 0; i < n_keys; i++) {
        if (!keys[i]) return MT_ERR_ARG;
        uint32_t idx = 0;
        if (array_index(nk[(size_t)i], &idx)) {
            is_index[(size_t)i] = 1;
            index[(size_t)i] = idx;
        }
    }
    std::vector<std::string> values((size_t)n_values);
    std::vector<uint8_t> flags((size_t)n_values);
    for (int i = 0; i < n_values; i++) {
        values[(size_t)i] = (i == 0 || !values_json[i]) ? std::string("null") : std::string(values_json[i]);
        flags[(size_t)i] = json_falsy(values[(size_t)i]) ? mt::kValFalsy : 0;
    }
    // matchProperties classes of the values (nested objects compare structurally)
    std::vector<uint32_t> cls;
    std::vector<uint64_t> exc;
    mt::value_relations(values, cls, flags, exc);
    DeviceValueTables t;
    const int rc = upload_value_tables(flags, cls, exc, 0xFFFFFFFFu, t);
    if (rc) return rc;
    b->keys = std::move(nk);
    b->key_is_index = std::move(is_index);
    b->key_index = std::move(index);
    b->values = std::move(values);
    b->value_flags = std::move(flags);
    b->value_class = std::move(cls);
    b->value_exc = std::move(exc);
    b->n_user_values = (size_t)n_values;
    b->nan_id = 0xFFFFFFFFu;
    (void)hipFree(b->d_vflags);
    (void)hipFree(b->d_vclass);
    (void)hipFree(b->d_vexc);
    (void)hipFree(b->d_vt);
    b->d_vflags = t.flags;
    b->d_vclass = t.cls;
    b->d_vexc = t.exc;
    b->d_vt = t.vt;
    return MT_OK;
}

// the checks mt_batch_set_clients makes, so callers can validate every list before changing anything
static bool clients_ok(const mt_batch *b, int64_t doc, size_t n) {
    return n >= 1 && n <= (size_t)MT_MAX_CLIENTS && doc < b->n_docs;
}

MT_API int mt_batch_set_clients(mt_batch *b, int64_t doc, const char *const *names, int32_t n) {
    if (!b || !names || n < 0 || !clients_ok(b, doc, (size_t)n)) return MT_ERR_ARG;
    std::vector<std::string> v(names, names + n);
    if (doc < 0) {
        b->clients = v;
        b->doc_clients.clear();
    } else {
        b->doc_clients[doc] = v;
    }
    return MT_OK;
}

static const std::vector<std::string> &clients_of(mt_batch *b, int64_t doc) {
    auto it = b->doc_clients.find(doc);
    return it == b->doc_clients.end() ? b->clients : it->second;
}

static int ensure_tables(mt_batch *b) {
    if (b->value_class.size() != b->values.size())
        mt::value_relations(b->values, b->value_class, b->value_flags, b->value_exc);
    if (b->d_vt) return MT_OK;
    (void)hipFree(b->d_vflags);
    (void)hipFree(b->d_vclass);
    (void)hipFree(b->d_vexc);
    b->d_vflags = nullptr;
    b->d_vclass = nullptr;
    b->d_vexc = nullptr;
    DeviceValueTables t;
    const int rc = upload_value_tables(b->value_flags, b->value_class, b->value_exc, b->nan_id, t);
    if (rc) return rc;
    b->d_vflags = t.flags;
    b->d_vclass = t.cls;
    b->d_vexc = t.exc;
    b->d_vt = t.vt;
    return MT_OK;
}

// matchProperties of two interned values, host side (same rule as value_rel on the device)
static int host_value_rel(const mt_batch *b, uint32_t va, uint32_t vb) {
    const size_t n = b->value_class.size();
    if (va >= n || vb >= n) return va == vb ? 1 : 0;
    if ((b->value_flags[va] | b->value_flags[vb]) & mt::kValNever) return 0;  // NaN !== NaN
    if (va == vb) return 1;
    if (b->value_class[va] == b->value_class[vb]) return 1;
    const uint8_t fa = b->value_flags[va], fb = b->value_flags[vb];
    if ((fa | fb) & mt::kValUnknown) return -1;
    if (!(fa & fb & mt::kValIrregular)) return 0;
    return std::binary_search(b->value_exc.begin(), b->value_exc.end(), (uint64_t)va << 32 | vb) ? 1 : 0;
}

static uint32_t align16u(uint64_t x) { return (uint32_t)((x + 15) & ~15ull); }

// the replica's own sequenced consensus annotate (mt_oplog.h: updateConsensusProperty's inputs)
static bool is_consensus_ack(const mt_op &o) {
    return o.type == MT_OP_ANNOTATE && MT_OPF_COMBINE(o.flags) == MT_COMBINE_CONSENSUS && MT_OP_CLIENT(o) == 0 &&
           o.seq != mt::kUnassignedSeq;
}

// Marker ids and relative positions (idToSegment, posFromRelativePos: mergeTree.ts:1185,
// 1942-1966).  Ids are object keys, so both sides are compared as String(value): every marker
// insert / load record whose props give a truthy markerId gets that key's id (>= 1) in
// payload_len (0: no id; a marker's payload_len is otherwise unused), every MT_OP_RELPOS record
// its ids' keys in pos1 / pos2 (0: no id).  A document whose annotates touch markerId gets
// kIdKeyUnsupported instead: the reference re-maps a re-annotated id only at a later blockUpdate.
// idmap_base[d]: the first entry of document d's map (one per marker with an id).
static void resolve_marker_ids(mt_batch *b, std::vector<mt_op> &h_ops, const std::vector<int64_t> &off,
                               const mt_prop *props, int64_t n_props, std::vector<uint64_t> &idmap_base) {
    uint32_t mk = 0xFFFFFFFFu;
    for (size_t k = 0; k < b->keys.size(); k++)
        if (b->keys[k] == "markerId") mk = (uint32_t)k;
    std::unordered_map<std::u16string, uint32_t> keys;
    std::unordered_map<uint32_t, uint32_t> of_value;
    auto key_of = [&](uint32_t v) -> uint32_t {  // 0: no id (null / falsy / not a value)
        if (v == 0 || v >= b->values.size() || (b->value_flags[v] & mt::kValFalsy)) return 0;
        auto it = of_value.find(v);
        if (it != of_value.end()) return it->second;
        std::u16string s;
        uint32_t k = 0;
        if (mt::js_string_of(b->values[v], s)) {
            auto kt = keys.find(s);
            if (kt == keys.end()) {
                kt = keys.emplace(s, (uint32_t)keys.size() + 1).first;
                b->key_value.push_back(v);  // key kt->second == key_value.size() - 1
            }
            k = kt->second;
        }
        of_value.emplace(v, k);
        return k;
    };
    const size_t D = off.size() - 1;
    uint64_t total = 0;
    b->key_value.assign(1, 0u);  // key 0: no id
    for (size_t d = 0; d < D; d++) {
        idmap_base[d] = total;
        bool annot_mk = false;
        for (int64_t i = off[d]; i < off[d + 1]; i++) {
            mt_op &o = h_ops[(size_t)i];
            if (MT_OP_IS_INSERT_LIKE(o.type) && (MT_OPF_BITS(o.flags) & MT_OPF_MARKER)) {
                uint32_t id = 0;
                if (MT_OPF_BITS(o.flags) & MT_OPF_HAS_PROPS) {
                    uint32_t p0 = 0;
                    const uint32_t np = mt_insert_props(&o, props, &p0);
                    for (uint32_t q = 0; q < np; q++)
                        if ((int64_t)p0 + q < n_props && props[p0 + q].key == mk) id = key_of(props[p0 + q].value);
                }
                o.payload_len = id;
                if (id) total++;
            } else if (o.type == MT_OP_ANNOTATE) {
                for (uint32_t q = 0; q < o.payload_len; q++)
                    if (props[o.payload + q].key == mk) annot_mk = true;
            }
        }
        for (int64_t i = off[d]; i < off[d + 1]; i++) {
            mt_op &o = h_ops[(size_t)i];
            if (is_consensus_ack(o)) {  // pos1: relativePos1.id's raw value id; pos2: its marker-id key
                o.pos2 = (int32_t)(annot_mk ? mt::kIdKeyUnsupported : key_of((uint32_t)o.pos1));
                continue;
            }
            if (o.type != MT_OP_RELPOS) continue;
            o.pos1 = (int32_t)(annot_mk ? mt::kIdKeyUnsupported : key_of((uint32_t)o.pos1));
            o.pos2 = (int32_t)(annot_mk ? mt::kIdKeyUnsupported : key_of((uint32_t)o.pos2));
        }
    }
    idmap_base[D] = total;
}

// The result slot of every combining annotate (mt_oplog.h): the value Properties.combine gives a
// key that the segment does not have (segmentPropertiesManager.ts:93-98 with previousValue and
// newValue undefined: mt::combine_absent).  Results that are not values of the caller's table
// are appended to it (NaN and consensus objects match nothing: kValNever).  Keys the segment
// does have are combined on the device (incr of a number / boolean / NaN is NaN — the slot's key
// holds the NaN value's id for "incr" ops; consensus and other kinds keep the value).  h_props
// stays empty when the log has no combining op.
static void rc_resolve_combine(mt_batch *b, const mt_op *ops, int64_t N, const mt_prop *props, int64_t n_props,
                               std::vector<mt_prop> &h_props) {
    const size_t nu = b->n_user_values;
    const bool had_derived = b->values.size() != nu;
    bool any = false;
    for (int64_t i = 0; i < N && !any; i++) any = ops[i].type == MT_OP_ANNOTATE && MT_OPF_COMBINE(ops[i].flags);
    if (!any && !had_derived) return;
    b->values.resize(nu);
    b->value_flags.resize(nu);
    for (uint8_t &f : b->value_flags) f &= mt::kValFalsy;  // value_relations derives the rest again
    b->nan_id = 0xFFFFFFFFu;
    if (any) {
        h_props.assign(props, props + n_props);
        std::unordered_map<std::string, uint32_t> ids;  // text -> id of the ordinary values
        for (size_t v = 1; v < nu; v++) ids.emplace(b->values[v], (uint32_t)v);
        auto text_of = [&](uint32_t v) -> const std::string * {
            return v == MT_VALUE_UNDEFINED || v >= nu ? nullptr : &b->values[v];
        };
        auto append = [&](const std::string &t, uint8_t flags) {
            b->values.push_back(t);
            b->value_flags.push_back(flags);
            return (uint32_t)(b->values.size() - 1);
        };
        // NaN (JSON text "null"): `v += undefined` of a number / boolean, also on the device
        auto nan = [&]() {
            if (b->nan_id == 0xFFFFFFFFu) b->nan_id = append("null", mt::kValFalsy | mt::kValNum | mt::kValNever);
            return b->nan_id;
        };
        std::unordered_map<std::string, uint32_t> cons_ids;
        for (int64_t i = 0; i < N; i++) {
            const mt_op &o = ops[i];
            const uint32_t kind = o.type == MT_OP_ANNOTATE ? MT_OPF_COMBINE(o.flags) : 0u;
            if (!kind) continue;
            mt_prop *x = h_props.data() + o.payload + o.payload_len;
            if (kind == MT_COMBINE_INCR) x[2].key = nan();  // a present number / boolean becomes NaN
            if (x[0].value != MT_VALUE_UNDEFINED && x[0].value >= nu) {
                x[2].value = mt::kValueCombineFail;
                continue;
            }
            std::string out;
            const std::string nul = "null";
            const std::string *def = x[0].value == 0 ? &nul : text_of(x[0].value);
            const std::string *mn = x[1].value == 0 ? &nul : text_of(x[1].value);
            uint32_t u = mt::kValueCombineFail;
            switch (mt::combine_absent((int)kind, def, mn, o.seq, out)) {
                case mt::kCombineValue: {
                    if (out == "null") {
                        u = 0;
                        break;
                    }
                    auto it = ids.find(out);
                    if (it == ids.end()) it = ids.emplace(out, append(out, json_falsy(out) ? mt::kValFalsy : 0)).first;
                    u = it->second;
                    break;
                }
                case mt::kCombineMin: u = x[1].value; break;
                case mt::kCombineNaN: u = nan(); break;
                case mt::kCombineConsensus: {
                    // a local op's { value: undefined, seq: -1 } is updated in place by a later
                    // consensus (kValSeqM1)
                    auto it = cons_ids.find(out);
                    if (it == cons_ids.end())
                        it = cons_ids.emplace(out, append(out, mt::kValNever | (o.seq == mt::kUnassignedSeq ? mt::kValSeqM1 : 0))).first;
                    u = it->second;
                    break;
                }
                case mt::kCombineDelete: u = 0; break;
                default: break;
            }
            x[2].value = u;
            // a sequenced consensus (the ack of the replica's own one: updateConsensusProperty, or a
            // remote one): the slot's key names the { seq: -1 } object a local consensus made,
            // which it updates in place on a marker
            if (kind == MT_COMBINE_CONSENSUS && o.seq != mt::kUnassignedSeq) {
                std::string lo;
                if (mt::combine_absent((int)kind, def, mn, mt::kUnassignedSeq, lo) == mt::kCombineConsensus) {
                    auto it = cons_ids.find(lo);
                    if (it == cons_ids.end()) it = cons_ids.emplace(lo, append(lo, mt::kValNever | mt::kValSeqM1)).first;
                    x[2].key = it->second;
                }
            }
        }
    }
    // the value tables are rebuilt (classes, flags) and uploaded again
    b->value_class.clear();
    (void)hipFree(b->d_vflags);
    (void)hipFree(b->d_vclass);
    (void)hipFree(b->d_vexc);
    (void)hipFree(b->d_vt);
    b->d_vflags = nullptr;
    b->d_vclass = nullptr;
    b->d_vexc = nullptr;
    b->d_vt = nullptr;
}

// The device regions of a writer batch (a log with local ops or acks): pending-group regions
// (a power of two of entries per document, mt_device.h pend_groups: at least 4,096 or MT_PEND_CAP,
// and 4 per group of `max_pending`, the most unacked local ops any replica of the log holds —
// the live entries, compacted when full), regenerated-op output (MT_REGEN_CAP words per document
// with MT_OP_REGENERATE records, default 16384, 2 for the others) and the consensus regions.
static int writer_regions(mt_batch *b, int64_t D, const std::vector<uint8_t> &has_regen,
                          std::vector<uint64_t> &cons_base, const std::vector<uint32_t> &cons_img,
                          int64_t max_pending = 0) {
    const char *e = getenv("MT_PEND_CAP");
    int64_t want = std::max<int64_t>(e && atoi(e) > 0 ? atoi(e) : 4096, 4 * (max_pending + 64));
    int64_t cap = 4096;
    while (cap < want && cap < (int64_t)1 << 28) cap <<= 1;
    b->pend_cap = (int32_t)cap;
    const uint64_t words = (uint64_t)mt::pend_words(b->pend_cap);
    std::vector<uint64_t> pbase_((size_t)D + 1);
    for (int64_t d = 0; d <= D; d++) pbase_[(size_t)d] = (uint64_t)d * words;
    HIPCHK(dalloc(&b->d_pend, (size_t)(words * (uint64_t)D)));
    if (D > 0) HIPCHK(hipMemset(b->d_pend, 0, 4 * words * (uint64_t)D));
    HIPCHK(dalloc(&b->d_pend_base, (size_t)D + 1));
    HIPCHK(hipMemcpy(b->d_pend_base, pbase_.data(), 8 * ((size_t)D + 1), hipMemcpyHostToDevice));
    const char *er = getenv("MT_REGEN_CAP");
    const uint64_t rcap = er && atoi(er) > 0 ? (uint64_t)atoi(er) : 16384;
    std::vector<uint64_t> rbase((size_t)D + 1, 0);
    uint64_t rtot = 0;
    for (int64_t d = 0; d < D; d++) {
        rbase[(size_t)d] = rtot;
        rtot += has_regen[(size_t)d] ? rcap : 2;
    }
    rbase[(size_t)D] = rtot;
    b->regen_cap = (int32_t)rcap;
    HIPCHK(dalloc(&b->d_regen, (size_t)std::max<uint64_t>(rtot, 2)));
    HIPCHK(hipMemset(b->d_regen, 0, 4 * std::max<uint64_t>(rtot, 2)));
    HIPCHK(dalloc(&b->d_regen_base, (size_t)D + 1));
    HIPCHK(hipMemcpy(b->d_regen_base, rbase.data(), 8 * ((size_t)D + 1), hipMemcpyHostToDevice));
    // per-document caps differ (2 words without REGENERATE records): the device checks
    // regen_cap only after a REGENERATE record, which only the large regions see
    b->h_regen_base = std::move(rbase);
    if (!cons_img.empty()) {
        HIPCHK(dalloc(&b->d_cons, cons_img.size()));
        HIPCHK(hipMemcpy(b->d_cons, cons_img.data(), 4 * cons_img.size(), hipMemcpyHostToDevice));
        HIPCHK(dalloc(&b->d_cons_base, (size_t)D + 1));
        HIPCHK(hipMemcpy(b->d_cons_base, cons_base.data(), 8 * ((size_t)D + 1), hipMemcpyHostToDevice));
        b->h_cons_base = std::move(cons_base);
    }
    b->writer = true;
    return MT_OK;
}

MT_API int mt_batch_ingest(mt_batch *b, const mt_op *ops, const int64_t *doc_op_off, const uint16_t *text,
                           int64_t n_text, const mt_prop *props, int64_t n_props) {
    if (!b || !ops || !doc_op_off || doc_op_off[0] != 0 || n_text < 0 || n_props < 0) return MT_ERR_ARG;
    if (n_text > 0 && !text) return MT_ERR_ARG;
    if (n_props > 0 && !props) return MT_ERR_ARG;
    const int64_t D = b->n_docs;
    // every check runs on locals before the batch is touched: a failed (re-)ingest leaves the
    // previous log, its device buffers and its results intact
    for (int64_t d = 0; d < D; d++)
        if (doc_op_off[d + 1] < doc_op_off[d]) return MT_ERR_ARG;
    const int64_t N = doc_op_off[D];
    if (N < 0 || N > ((int64_t)1 << 40)) return MT_ERR_ARG;
    std::vector<int64_t> h_off(doc_op_off, doc_op_off + D + 1);
    std::vector<uint64_t> text_base((size_t)D, 0), pool_base((size_t)D, 0);
    std::vector<uint32_t> text_len((size_t)D, 0), text_cap((size_t)D, 0), pool_cap((size_t)D, 0);
    std::vector<int32_t> nload((size_t)D, 0), nload_segs((size_t)D, 0);
    uint64_t tbase = 0, pbase = 0;
    int32_t max_ops = 0;
    double payload_units = 0, prop_records = 0;
    for (int64_t d = 0; d < D; d++) {
        const int64_t a = h_off[d], e = h_off[d + 1];
        if (e - a > 0x7FFFFFFF) return MT_ERR_ARG;
        max_ops = std::max<int32_t>(max_ops, (int32_t)(e - a));
        for (int64_t i = a; i < e; i++) {  // leading SnapshotLoader records
            const uint8_t t = ops[i].type;
            if (t != MT_OP_LOAD_HEADER && t != MT_OP_LOAD_BODY && t != MT_OP_COLLAB) break;
            nload[d]++;
            if (t != MT_OP_COLLAB) nload_segs[d]++;
        }
        for (int64_t i = a + nload[d]; i < e; i++)  // LOAD records only lead a log
            if (ops[i].type == MT_OP_LOAD_HEADER || ops[i].type == MT_OP_LOAD_BODY || ops[i].type == MT_OP_COLLAB)
                return MT_ERR_ARG;
        uint64_t pay = 0, nprop_ops = 0, precs = 0;
        for (int64_t i = a; i < e; i++) {
            const mt_op &o = ops[i];
            if (MT_OP_IS_INSERT_LIKE(o.type) && !(MT_OPF_BITS(o.flags) & MT_OPF_MARKER)) {
                if ((int64_t)o.payload + (int64_t)o.payload_len > n_text) return MT_ERR_ARG;
                pay += o.payload_len;
            }
            if (o.type == MT_OP_ANNOTATE) {
                const int64_t extra = MT_OPF_COMBINE(o.flags) ? MT_COMBINE_RECORDS : 0;
                if ((int64_t)o.payload + (int64_t)o.payload_len + extra > n_props) return MT_ERR_ARG;
                for (int64_t x = 0; x < extra; x++)
                    if (props[o.payload + o.payload_len + x].key != MT_KEY_COMBINE) return MT_ERR_ARG;
                nprop_ops++;
                prop_records += o.payload_len;
                precs += o.payload_len;
            }
            if (o.type == MT_OP_REGENERATE && o.ref_seq == MT_OP_ANNOTATE &&
                (int64_t)o.payload + (int64_t)o.payload_len > n_props)
                return MT_ERR_ARG;
            if (MT_OP_IS_INSERT_LIKE(o.type) && (MT_OPF_BITS(o.flags) & MT_OPF_HAS_PROPS)) {
                if (o.pos2 < 0 || o.pos2 >= n_props + (MT_OPF_NPROPS(o.flags) == MT_OPF_NPROPS_EXT ? 0 : 1))
                    return MT_ERR_ARG;
                uint32_t p0 = 0;
                const uint32_t np = mt_insert_props(&o, props, &p0);
                if ((int64_t)p0 + (int64_t)np > n_props) return MT_ERR_ARG;
                if (MT_OPF_NPROPS(o.flags) == MT_OPF_NPROPS_EXT &&
                    (props[o.pos2].key != MT_KEY_NPROPS || np <= MT_OPF_NPROPS_INLINE))
                    return MT_ERR_ARG;
                nprop_ops++;
                prop_records += np;
                precs += np;
            }
        }
        payload_units += (double)pay;
        uint64_t cap = (uint64_t)align16u(pay) + (uint64_t)b->opt.arena_factor * pay + 4096;
        if (cap > 0xFFFFFFF0ull) return MT_ERR_ARG;
        text_base[d] = tbase;
        text_len[d] = (uint32_t)pay;
        text_cap[d] = (uint32_t)cap;
        tbase += align16u(cap);
        // prop sets of any size: besides the per-op allowance, room for the sets an op's records
        // can make (a few live copies of the largest ones between collections)
        uint64_t kd = 0;  // distinct keys of the document's prop records (sets of up to kd keys)
        if (precs > 64) {
            std::unordered_set<uint32_t> ks;
            for (int64_t i = a; i < e; i++) {
                const mt_op &o = ops[i];
                uint32_t p0 = 0, np = 0;
                if (o.type == MT_OP_ANNOTATE) {
                    p0 = o.payload;
                    np = o.payload_len;
                } else if (MT_OP_IS_INSERT_LIKE(o.type) && (MT_OPF_BITS(o.flags) & MT_OPF_HAS_PROPS)) {
                    np = mt_insert_props(&o, props, &p0);
                }
                for (uint32_t q = 0; q < np; q++) ks.insert(props[p0 + q].key);
            }
            kd = ks.size();
        }
        uint64_t pc = 1024 + (uint64_t)b->opt.pool_per_op * nprop_ops + (kd > 32 ? 8 * kd * kd + 8 * precs : 0);
        pool_base[d] = pbase;
        pool_cap[d] = (uint32_t)std::min<uint64_t>(pc, 0xFFFFFFF0ull);
        pbase += align16u(pc);
    }
    // findTile reads the block tile maps that blockUpdate rebuilds (mergeTree.ts:2748-2767); an
    // annotate of referenceTileLabels changes a marker's labels without one, so such documents'
    // tile queries are MT_UNSUPPORTED
    // (bit 0; bit 1: the same for referenceRangeLabels and getStackContext's rangeStacks)
    std::vector<uint8_t> tile_annot((size_t)D, 0);
    {
        uint32_t tk = 0xFFFFFFFFu, rk = 0xFFFFFFFFu;
        for (size_t k = 0; k < b->keys.size(); k++) {
            if (b->keys[k] == "referenceTileLabels") tk = (uint32_t)k;
            if (b->keys[k] == "referenceRangeLabels") rk = (uint32_t)k;
        }
        if (tk != 0xFFFFFFFFu || rk != 0xFFFFFFFFu)
            for (int64_t d = 0; d < D; d++)
                for (int64_t i = h_off[d]; i < h_off[d + 1] && tile_annot[(size_t)d] != 3; i++)
                    if (ops[i].type == MT_OP_ANNOTATE)
                        for (uint32_t q = 0; q < ops[i].payload_len; q++) {
                            if (props[ops[i].payload + q].key == tk) tile_annot[(size_t)d] |= 1;
                            if (props[ops[i].payload + q].key == rk) tile_annot[(size_t)d] |= 2;
                        }
    }
    // a writer replica's log: local ops (seq == UnassignedSequenceNumber) or sequenced messages of
    // the replica itself (short id 0) that ack them
    bool writer = false;
    for (int64_t d = 0; d < D && !writer; d++)
        for (int64_t i = h_off[d] + nload[d]; i < h_off[d + 1]; i++)
            if (ops[i].seq == mt::kUnassignedSeq || (MT_OP_CLIENT(ops[i]) == 0 && ops[i].type != MT_OP_NOOP)) {
                writer = true;
                break;
            }
    // writer consensus regions (mt_device.h kConsHdr): one id per notify RELPOS, one listener per ack
    // of a consensus annotate
    std::vector<uint64_t> cons_base((size_t)D + 1, 0);
    std::vector<uint32_t> cons_img;
    if (writer) {
        uint64_t ct = 0;
        for (int64_t d = 0; d < D; d++) {
            cons_base[(size_t)d] = ct;
            uint64_t ni = 0, nl = 0;
            for (int64_t i = h_off[d]; i < h_off[d + 1]; i++) {
                const mt_op &o = ops[i];
                if (o.type == MT_OP_RELPOS && o.seq == mt::kUnassignedSeq && (o.flags & MT_RELF_NOTIFY)) {
                    if (o.payload == 0 || o.payload >= b->n_user_values) return MT_ERR_ARG;
                    ni++;
                }
                if (is_consensus_ack(o)) {
                    if ((uint32_t)o.pos1 >= b->n_user_values) return MT_ERR_ARG;
                    nl++;
                }
            }
            if (ni + nl == 0) continue;
            if (ni > 0x7FFFFFFF || nl > 0x7FFFFFFF) return MT_ERR_ARG;
            cons_img.resize((size_t)(ct + (uint64_t)mt::cons_words((int64_t)ni, (int64_t)nl)), 0u);
            cons_img[(size_t)ct + 3] = (uint32_t)ni;
            cons_img[(size_t)ct + 4] = (uint32_t)nl;
            ct += (uint64_t)mt::cons_words((int64_t)ni, (int64_t)nl);
        }
        cons_base[(size_t)D] = ct;
    }
    // combiningOps: the value each one gives a key the segment does not have yet
    std::vector<mt_prop> h_props;
    rc_resolve_combine(b, ops, N, props, n_props, h_props);
    int rc = ensure_tables(b);
    if (rc) return rc;
    std::vector<mt_op> h_ops(ops, ops + N);
    std::vector<uint64_t> idmap_base((size_t)D + 1, 0);
    resolve_marker_ids(b, h_ops, h_off, props, n_props, idmap_base);
    std::vector<uint16_t> h_text(tbase ? tbase : 1, 0);
    for (int64_t d = 0; d < D; d++) {
        uint32_t w = 0;
        for (int64_t i = h_off[d]; i < h_off[d + 1]; i++) {
            mt_op &o = h_ops[i];
            if (MT_OP_IS_INSERT_LIKE(o.type) && !(MT_OPF_BITS(o.flags) & MT_OPF_MARKER)) {
                if (o.payload_len) memcpy(&h_text[text_base[d] + w], text + o.payload, 2ull * o.payload_len);
                o.flags &= (uint16_t)~MT_OPF_INTERNAL;
                if (o.payload_len && text[o.payload + o.payload_len - 1] == (uint16_t)'\n')
                    o.flags |= (uint16_t)MT_OPF_INTERNAL_ENDS_NL;
                for (uint32_t i = 0; i < o.payload_len; i++)
                    if (text[o.payload + i] == (uint16_t)'\n') {
                        o.flags |= (uint16_t)MT_OPF_INTERNAL_HAS_NL;
                        break;
                    }
                o.payload = w;
                w += o.payload_len;
            }
        }
    }
    // the validated log replaces the previous one
    free_launches(b);
    free_log(b);
    b->ran = false;
    b->cached_doc = -1;
    b->c_blob_doc = -1;
    b->h_off = std::move(h_off);
    b->h_props_all.assign(props, props + n_props);
    b->h_text_base = std::move(text_base);
    b->h_text_len = std::move(text_len);
    b->h_text_cap = std::move(text_cap);
    b->h_pool_base = std::move(pool_base);
    b->h_pool_cap = std::move(pool_cap);
    b->h_nload = std::move(nload);
    b->h_nload_segs = std::move(nload_segs);
    b->h_tile_annot = std::move(tile_annot);
    b->lab_track = std::any_of(b->h_tile_annot.begin(), b->h_tile_annot.end(), [](uint8_t t) { return t != 0; });
    b->payload_units = payload_units;
    b->prop_records = prop_records;
    b->text_words = tbase;
    b->pool_words = pbase;
    b->total_ops = N;
    b->total_props = n_props;
    b->max_ops_per_doc = max_ops;
    HIPCHK(dalloc(&b->d_ops, (size_t)N));
    HIPCHK(dalloc(&b->d_off, (size_t)D + 1));
    HIPCHK(dalloc(&b->d_text, (size_t)h_text.size()));
    HIPCHK(dalloc(&b->d_text_base, (size_t)D));
    HIPCHK(dalloc(&b->d_text_len, (size_t)D));
    HIPCHK(dalloc(&b->d_text_cap, (size_t)D));
    HIPCHK(dalloc(&b->d_pool, (size_t)pbase));
    HIPCHK(dalloc(&b->d_pool_base, (size_t)D));
    HIPCHK(dalloc(&b->d_pool_cap, (size_t)D));
    HIPCHK(dalloc(&b->d_props, (size_t)std::max<int64_t>(n_props, 1)));
    HIPCHK(dalloc(&b->d_idmap, (size_t)std::max<uint64_t>(idmap_base[(size_t)D], 1)));
    HIPCHK(dalloc(&b->d_idmap_base, (size_t)D + 1));
    HIPCHK(hipMemcpy(b->d_idmap_base, idmap_base.data(), 8 * ((size_t)D + 1), hipMemcpyHostToDevice));
    if (writer) {
        std::vector<uint8_t> has_regen((size_t)D, 0);
        // the most groups a replica can hold pending: local records less the acks (its own
        // sequenced records) before them, at the peak (an upper bound; a regenerate replaces groups)
        int64_t max_pending = 0;
        for (int64_t d = 0; d < D; d++) {
            int64_t pend = 0;
            for (int64_t i = b->h_off[(size_t)d]; i < b->h_off[(size_t)d + 1]; i++) {
                has_regen[(size_t)d] |= ops[i].type == MT_OP_REGENERATE;
                if (ops[i].seq == MT_SEQ_LOCAL) max_pending = std::max(max_pending, ++pend);
                else if (ops[i].seq > 0 && MT_OP_CLIENT(ops[i]) == 0 && pend > 0) pend--;
            }
        }
        const int rc2 = writer_regions(b, D, has_regen, cons_base, cons_img, max_pending);
        if (rc2) return rc2;
    }
    HIPCHK(hipMemcpy(b->d_ops, h_ops.data(), sizeof(mt_op) * (size_t)N, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_off, b->h_off.data(), sizeof(int64_t) * (size_t)(D + 1), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text, h_text.data(), 2 * h_text.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text_base, b->h_text_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text_len, b->h_text_len.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text_cap, b->h_text_cap.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_pool_base, b->h_pool_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_pool_cap, b->h_pool_cap.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    if (n_props > 0)
        HIPCHK(hipMemcpy(b->d_props, h_props.empty() ? props : h_props.data(), sizeof(mt_prop) * (size_t)n_props,
                         hipMemcpyHostToDevice));
    b->have_log = true;
    b->generated = false;
    return MT_OK;
}

static void json_gpu_stats(const mt::jg::Result &r, double ms_total, mt_json_gpu_stats *st) {
    if (!st) return;
    *st = mt_json_gpu_stats{};
    st->ms_scan = r.ms_scan;
    st->ms_count = r.ms_count;
    st->ms_clients = r.ms_clients;
    st->ms_write = r.ms_write;
    st->ms_props = r.ms_props;
    st->ms_host = r.ms_host;
    st->ms_total = ms_total;
    st->n_msgs = r.n_msgs;
    st->n_ops = r.n_ops;
    st->n_text = r.n_text;
    st->n_props = r.n_props;
    st->fail_bits = r.fail_bits;
}

MT_API int mt_pack_json_gpu(mt_packed **out, int64_t n_docs, const char *json, const int64_t *doc_off,
                            const char *observer, int64_t *bad_doc, mt_json_gpu_stats *stats) {
    if (!out || n_docs < 0 || !doc_off || (n_docs && !json)) return MT_ERR_ARG;
    *out = nullptr;
    if (bad_doc) *bad_doc = -1;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MT_ERR_NO_DEVICE;
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t s = nullptr;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    mt::jg::Result r;
    mt_op *d_ops = nullptr;
    uint16_t *d_text = nullptr;
    mt_prop *d_props = nullptr;
    uint64_t words = 0;
    int rc = mt::jg::parse(json, doc_off, n_docs, nullptr, observer, s, nullptr, &d_ops, &d_text, &words, &d_props, r);
    std::vector<mt_op> ops;
    std::vector<uint16_t> text;
    std::vector<mt_prop> props;
    if (rc == MT_OK) {
        ops.resize((size_t)r.n_ops);
        text.resize((size_t)r.n_text);
        props.resize((size_t)r.n_props);
        if (hipMemcpy(ops.data(), d_ops, sizeof(mt_op) * ops.size(), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(text.data(), d_text, 2 * text.size(), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(props.data(), d_props, sizeof(mt_prop) * props.size(), hipMemcpyDeviceToHost) != hipSuccess)
            rc = MT_ERR_HIP;
    }
    (void)hipFree(d_ops);
    (void)hipFree(d_text);
    (void)hipFree(d_props);
    (void)hipStreamDestroy(s);
    if (bad_doc) *bad_doc = r.bad_doc;
    json_gpu_stats(r, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                   stats);
    if (rc != MT_OK) return rc;
    *out = mt_packed_from(std::move(ops), std::move(r.doc_op_off), std::move(text), std::move(props),
                          std::move(r.keys), std::move(r.values), std::move(r.clients));
    return MT_OK;
}

// GPU parse straight into the replay's layout: per-document text arenas (payloads document-
// relative, the '\n' flags set), the same host metadata as mt_batch_ingest for a log of the
// GPU fast path (no LOAD / REGENERATE records, no combiningOps but rewrite, no consensus ids; a
// writer replica's local ops and acks get mt_batch_ingest's writer regions)
MT_API int mt_batch_ingest_json_gpu(mt_batch *b, const char *json, const int64_t *doc_off, int64_t n_docs,
                                    const void *d_json, const char *observer, int64_t *bad_doc,
                                    mt_json_gpu_stats *stats) {
    // n_docs: the caller's document count; doc_off[0..n_docs] is read, so a count that differs
    // from the batch's would read past the caller's arrays
    if (!b || !doc_off || n_docs != b->n_docs || (b->n_docs && !json) || ((uintptr_t)d_json & 3u)) return MT_ERR_ARG;
    if (bad_doc) *bad_doc = -1;
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t D = b->n_docs;
    std::vector<uint32_t> text_len((size_t)D), text_cap((size_t)D);
    mt::jg::TextLayout layout = [&](const mt::jg::Result &r, std::vector<uint64_t> &base, uint64_t &words) -> int {
        uint64_t tb = 0;
        for (int64_t d = 0; d < D; d++) {
            const uint64_t pay = r.doc_text[(size_t)d];
            const uint64_t cap = (uint64_t)align16u(pay) + (uint64_t)b->opt.arena_factor * pay + 4096;
            if (cap > 0xFFFFFFF0ull) return MT_ERR_ARG;
            base[(size_t)d] = tb;
            text_len[(size_t)d] = (uint32_t)pay;
            text_cap[(size_t)d] = (uint32_t)cap;
            tb += align16u(cap);
        }
        words = tb;
        return MT_OK;
    };
    mt::jg::Result r;
    mt_op *d_ops = nullptr;
    uint16_t *d_text = nullptr;
    mt_prop *d_props = nullptr;
    uint64_t words = 0;
    int rc = mt::jg::parse(json, doc_off, D, (const uint8_t *)d_json, observer, b->stream, &layout, &d_ops, &d_text,
                           &words, &d_props, r);
    auto drop = [&]() {
        (void)hipFree(d_ops);
        (void)hipFree(d_text);
        (void)hipFree(d_props);
    };
    if (bad_doc) *bad_doc = r.bad_doc;
    if (rc != MT_OK) {
        drop();
        json_gpu_stats(r, 0, stats);
        return rc;
    }
    std::vector<mt_prop> h_props((size_t)r.n_props);
    if (!h_props.empty() &&
        hipMemcpy(h_props.data(), d_props, sizeof(mt_prop) * h_props.size(), hipMemcpyDeviceToHost) != hipSuccess) {
        drop();
        return MT_ERR_HIP;
    }
    // marker ids and tile-label annotates (resolve_marker_ids / tile_annot of mt_batch_ingest) on
    // the device: a marker's markerId value -> its key (String(value); any consistent numbering
    // serves, the ids only key idToSegment for relative positions), per-document id counts
    uint32_t mk = 0xFFFFFFFFu, tk = 0xFFFFFFFFu, rk = 0xFFFFFFFFu;
    for (size_t k = 0; k < r.keys.size(); k++) {
        if (r.keys[k] == "markerId") mk = (uint32_t)k;
        if (r.keys[k] == "referenceTileLabels") tk = (uint32_t)k;
        if (r.keys[k] == "referenceRangeLabels") rk = (uint32_t)k;
    }
    std::vector<uint32_t> vkey(r.values.size(), 0u), n_ids((size_t)D, 0u), tile((size_t)D, 0u);
    std::vector<uint32_t> key_value(1, 0u);
    {
        std::unordered_map<std::u16string, uint32_t> km;
        for (size_t v = 1; v < r.values.size(); v++) {
            if (json_falsy(r.values[v])) continue;
            std::u16string str;
            if (!mt::js_string_of(r.values[v], str)) continue;
            auto it = km.find(str);
            if (it == km.end()) {
                it = km.emplace(str, (uint32_t)km.size() + 1).first;
                key_value.push_back((uint32_t)v);  // key it->second == key_value.size() - 1
            }
            vkey[v] = it->second;
        }
    }
    if (D > 0) {
        uint32_t *d_vkey = nullptr, *d_nids = nullptr, *d_tile = nullptr;
        int64_t *d_oo = nullptr;
        auto mfree = [&]() {
            (void)hipFree(d_vkey);
            (void)hipFree(d_nids);
            (void)hipFree(d_tile);
            (void)hipFree(d_oo);
        };
        if (dalloc(&d_vkey, vkey.size()) != hipSuccess || dalloc(&d_nids, (size_t)D) != hipSuccess ||
            dalloc(&d_tile, (size_t)D) != hipSuccess || dalloc(&d_oo, (size_t)D + 1) != hipSuccess ||
            hipMemcpy(d_vkey, vkey.data(), 4 * vkey.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(d_oo, r.doc_op_off.data(), 8 * ((size_t)D + 1), hipMemcpyHostToDevice) != hipSuccess) {
            mfree();
            drop();
            return MT_ERR_HIP;
        }
        const mt_op *ops_c = d_ops;
        const int64_t *oo_c = d_oo;
        const mt_prop *pr_c = d_props;
        const uint32_t *vk_c = d_vkey;
        uint32_t nv = (uint32_t)vkey.size();
        int64_t Dd = D;
        void *args[] = {&ops_c, &oo_c, &d_ops, &pr_c, &Dd, &mk, &tk, &rk, &vk_c, &nv, &d_nids, &d_tile};
        hipError_t e = hipLaunchKernel((const void *)jg_markers_kernel, dim3((unsigned)D), dim3(64), args, 0, b->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(b->stream);
        if (e == hipSuccess) e = hipMemcpy(n_ids.data(), d_nids, 4 * (size_t)D, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(tile.data(), d_tile, 4 * (size_t)D, hipMemcpyDeviceToHost);
        mfree();
        if (e != hipSuccess) {
            drop();
            return MT_ERR_HIP;
        }
    }
    // tables (as mt_batch_ingest_packed): the batch changes only after every device step succeeded
    std::vector<const char *> kp, vp;
    for (const auto &k : r.keys) kp.push_back(k.c_str());
    for (const auto &v : r.values) vp.push_back(v.c_str());
    static const char *none = "_";
    bool shared = true;
    for (int64_t d = 1; d < D && shared; d++) shared = r.clients[(size_t)d] == r.clients[0];
    // every client list is checked before the tables change (set_clients cannot fail after them)
    for (int64_t d = 0; d < (shared ? std::min<int64_t>(D, 1) : D); d++)
        if (!clients_ok(b, shared ? -1 : d, r.clients[(size_t)d].size())) {
            drop();
            return MT_ERR_ARG;
        }
    rc = mt_batch_set_tables(b, kp.empty() ? &none : kp.data(), kp.empty() ? 1 : (int32_t)kp.size(), vp.data(),
                             (int32_t)vp.size());
    auto set = [&](int64_t doc, const std::vector<std::string> &names) {
        std::vector<const char *> np;
        for (const auto &n : names) np.push_back(n.c_str());
        return mt_batch_set_clients(b, doc, np.data(), (int32_t)np.size());
    };
    if (!rc && D && shared) rc = set(-1, r.clients[0]);
    for (int64_t d = 0; !rc && !shared && d < D; d++) rc = set(d, r.clients[(size_t)d]);
    if (rc) {
        drop();
        return rc;
    }
    std::vector<uint64_t> idmap_base((size_t)D + 1, 0);
    for (int64_t d = 0; d < D; d++) idmap_base[(size_t)d + 1] = idmap_base[(size_t)d] + n_ids[(size_t)d];
    // the parsed log replaces the previous one (mt_batch_ingest's fields for this log shape)
    free_launches(b);
    free_log(b);
    b->key_value = std::move(key_value);
    b->ran = false;
    b->cached_doc = -1;
    b->c_blob_doc = -1;
    std::vector<uint64_t> text_base((size_t)D), pool_base((size_t)D);
    std::vector<uint32_t> pool_cap((size_t)D);
    uint64_t tb = 0, pb = 0;
    int32_t max_ops = 0;
    for (int64_t d = 0; d < D; d++) {
        text_base[(size_t)d] = tb;
        tb += align16u(text_cap[(size_t)d]);
        const uint64_t pc = 1024 + (uint64_t)b->opt.pool_per_op * r.doc_nprop_ops[(size_t)d];
        pool_base[(size_t)d] = pb;
        pool_cap[(size_t)d] = (uint32_t)std::min<uint64_t>(pc, 0xFFFFFFF0ull);
        pb += align16u(pc);
        max_ops = std::max<int32_t>(max_ops, (int32_t)(r.doc_op_off[(size_t)d + 1] - r.doc_op_off[(size_t)d]));
    }
    const int64_t N = r.n_ops;
    b->h_off = r.doc_op_off;
    b->h_props_all = std::move(h_props);
    b->h_text_base = text_base;
    b->h_text_len = text_len;
    b->h_text_cap = text_cap;
    b->h_pool_base = pool_base;
    b->h_pool_cap = pool_cap;
    b->h_nload.assign((size_t)D, 0);
    b->h_nload_segs.assign((size_t)D, 0);
    b->h_tile_annot.assign((size_t)D, 0);
    for (int64_t d = 0; d < D; d++) b->h_tile_annot[(size_t)d] = (uint8_t)(tile[(size_t)d] & 3u);
    b->lab_track = std::any_of(b->h_tile_annot.begin(), b->h_tile_annot.end(), [](uint8_t t) { return t != 0; });
    b->payload_units = (double)r.n_text;
    b->prop_records = (double)r.n_props;
    b->text_words = tb;
    b->pool_words = pb;
    b->total_ops = N;
    b->total_props = r.n_props;
    b->max_ops_per_doc = max_ops;
    b->d_ops = d_ops;
    b->d_text = d_text;
    b->d_props = d_props;
    HIPCHK(dalloc(&b->d_off, (size_t)D + 1));
    HIPCHK(dalloc(&b->d_text_base, (size_t)D));
    HIPCHK(dalloc(&b->d_text_len, (size_t)D));
    HIPCHK(dalloc(&b->d_text_cap, (size_t)D));
    HIPCHK(dalloc(&b->d_pool, (size_t)pb));
    HIPCHK(dalloc(&b->d_pool_base, (size_t)D));
    HIPCHK(dalloc(&b->d_pool_cap, (size_t)D));
    HIPCHK(dalloc(&b->d_idmap, (size_t)std::max<uint64_t>(idmap_base[(size_t)D], 1)));
    HIPCHK(dalloc(&b->d_idmap_base, (size_t)D + 1));
    HIPCHK(hipMemcpy(b->d_idmap_base, idmap_base.data(), 8 * ((size_t)D + 1), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_off, b->h_off.data(), sizeof(int64_t) * (size_t)(D + 1), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text_base, b->h_text_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text_len, b->h_text_len.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text_cap, b->h_text_cap.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_pool_base, b->h_pool_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_pool_cap, b->h_pool_cap.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    if (r.writer) {
        std::vector<uint64_t> cons_base((size_t)D + 1, 0);
        int64_t max_pending = 0;
        rc = mt::jg::pending_peak(b->d_ops, b->d_off, D, b->stream, &max_pending);
        if (rc) return rc;
        rc = writer_regions(b, D, std::vector<uint8_t>((size_t)D, 0), cons_base, {}, max_pending);
        if (rc) return rc;
    }
    b->have_log = true;
    b->generated = false;
    json_gpu_stats(r, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(),
                   stats);
    return MT_OK;
}

// capacity class index: derived from ops per document unless seg_cap is given; `level`
// escalates by whole classes.  Replay starts a document in at most the 16-documents-per-CU class
// (kReplayStartClass): the replay kernel is latency bound, so a launch's rate grows with the documents
// resident per CU (config 3, 65,536 docs: 203k ops/ms at 8 per CU, 113k at 5, 65k at 3), and a
// document escalates by checkpoint (an image round trip to HBM, ~1 ms per class for 65,536 docs)
// only when it needs the room.  The generator re-runs a document from scratch on overflow, so it
// starts in the class of the expected final size (`replay` false).
static int class_for(const mt_batch *b, int32_t ops_per_doc, int level, bool replay = true) {
    int32_t want = b->opt.seg_cap > 0 ? b->opt.seg_cap : ops_per_doc / 12 + 64;
    if (replay && b->opt.seg_cap <= 0) want = std::min<int32_t>(want, mt::kClassSegs[mt::kReplayStartClass]);
    int c = 0;
    while (c + 1 < mt::kNumClasses && mt::kClassSegs[c] < want) c++;
    c += level;
    return c < mt::kNumClasses ? c : mt::kNumClasses;  // kNumClasses: nothing larger
}
// dynamic LDS of a class's launch (the HBM class keeps its tables in global memory)
// (the giant class: its LDS part; its tables, like the HBM class's, are a per-document image in HBM)
static size_t class_lds(int c) {
    if (c == mt::kHbmClass) return 0;
    if (c == mt::kGiantClass) return mt::make_glayout().bytes;
    return mt::make_layout(mt::kClassSegs[c]).bytes;
}
static bool class_in_hbm(int c) { return c == mt::kHbmClass || c == mt::kGiantClass; }
static size_t class_state_bytes(int c) { return class_in_hbm(c) ? mt::make_layout(mt::kClassSegs[c]).bytes : 0; }
static int max_lds_bytes();
// the class an escalated document continues in: at least 1.1x the slots (every class of the
// ladder is a residency tier; skipping one costs more than the extra checkpoint)
static int resume_class(int c) {
    int n = c + 1;
    while (n < mt::kNumClasses && 10 * mt::kClassSegs[n] < 11 * mt::kClassSegs[c]) n++;
    if (n >= mt::kNumClasses) n = mt::kNumClasses - 1;
    while (n > c + 1 && class_lds(n) > (size_t)max_lds_bytes()) n--;
    return n;
}
// documents per giant / HBM-class launch: each holds its ~2M-slot tables, cold records, output
// records and (giant class) its checkpoint buffer in device memory (~220-290 MB), so a launch is
// bounded to ~24 GB
static size_t hbm_doc_bytes() {
    size_t m = 0;
    for (int cls : {mt::kGiantClass, mt::kHbmClass}) {
        const int seg = mt::kClassSegs[cls];
        const mt::Caps c = mt::class_caps(seg);
        size_t x = (size_t)mt::make_layout(seg).bytes + (size_t)c.seg * mt::kColdPerSlot * 16 + (size_t)c.oe * sizeof(OutRec);
        if (cls == mt::kGiantClass) x += 4 * (size_t)mt::ck_words(seg);
        m = std::max(m, x);
    }
    return m;
}
static const size_t kMaxHbmDocs = std::max<size_t>(1, ((size_t)24 << 30) / hbm_doc_bytes());
static size_t launch_chunk(int cls, size_t n) { return class_in_hbm(cls) ? kMaxHbmDocs : n; }
// where a document with a segment longer than the LDS classes' 16-bit lengths continues (from scratch)
static int long_seg_class(int cls) { return cls < mt::kGiantClass ? mt::kGiantClass : cls == mt::kGiantClass ? mt::kHbmClass : mt::kNumClasses; }
static bool class_usable(int c) { return c < mt::kNumClasses && class_lds(c) <= (size_t)max_lds_bytes(); }

static int max_lds_bytes() {
    static int v = -1;
    if (v < 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        hipDeviceProp_t p;
        v = 65536;
        if (hipGetDeviceProperties(&p, dev) == hipSuccess) {
            size_t m = std::max(p.sharedMemPerBlock, p.sharedMemPerBlockOptin);
            if (p.maxSharedMemoryPerMultiProcessor > m) m = p.maxSharedMemoryPerMultiProcessor;
            v = (int)m;
        }
        if (v > 160 * 1024) v = 160 * 1024;
        v -= (int)kGenStaticLds;  // static LDS of the generator kernel
    }
    return v;
}

static mt::ReplayParams base_params(mt_batch *b) {
    mt::ReplayParams P{};
    P.ops = b->d_ops;
    P.doc_op_off = b->d_off;
    P.text = b->d_text;
    P.doc_text_base = b->d_text_base;
    P.doc_text_len = b->d_text_len;
    P.doc_text_cap = b->d_text_cap;
    P.pool = b->d_pool;
    P.doc_pool_base = b->d_pool_base;
    P.doc_pool_cap = b->d_pool_cap;
    P.props_in = b->d_props;
    P.vt = b->d_vt;
    P.idmap = b->d_idmap;
    P.doc_idmap_base = b->d_idmap_base;
    P.pend = b->d_pend;
    P.doc_pend_base = b->d_pend_base;
    P.pend_cap = b->pend_cap;
    P.regen = b->d_regen;
    P.doc_regen_base = b->d_regen_base;
    P.regen_cap = b->regen_cap;
    P.cons = b->d_cons;
    P.doc_cons_base = b->d_cons_base;
    return P;
}

static int launch_replay(mt_batch *b, hipStream_t s, Launch &L) {
    int64_t n = L.docs.empty() ? b->n_docs : (int64_t)L.docs.size();
    L.caps = mt::class_caps(mt::kClassSegs[L.cls]);
    L.out_cap = L.caps.oe;
    L.lds = class_lds(L.cls);
    HIPCHK(lbuf_alloc(b, &L.d_out, (size_t)n * (size_t)L.out_cap));
    if (b->lab_track) HIPCHK(lbuf_alloc(b, &L.d_lab, (size_t)n * (size_t)L.out_cap));
    HIPCHK(lbuf_alloc(b, &L.d_docout, (size_t)n));
    HIPCHK(lbuf_alloc(b, &L.d_cold, (size_t)n * (size_t)L.caps.seg * mt::kColdPerSlot));
    // (the HBM class's table images: fresh allocations, as before)
    if (class_state_bytes(L.cls)) {
        hipError_t e = dalloc(&L.d_state, (size_t)n * class_state_bytes(L.cls));
        if (e != hipSuccess && !b->buf_cache.empty()) {  // cached buffers first
            (void)hipGetLastError();
            lbuf_release(b);
            e = dalloc(&L.d_state, (size_t)n * class_state_bytes(L.cls));
        }
        HIPCHK(e);
    }
    if (!L.docs.empty()) {
        HIPCHK(lbuf_alloc(b, &L.d_list, L.docs.size()));
        HIPCHK(hipMemcpyAsync(L.d_list, L.docs.data(), 4 * L.docs.size(), hipMemcpyHostToDevice, s));
    }
    // documents short of headroom checkpoint here unless this is the largest usable class
    const bool can_grow = (class_usable(L.cls + 1) && b->opt.max_retries != 0) || L.load;
    if (can_grow) HIPCHK(lbuf_alloc(b, &L.d_ck, (size_t)n * (size_t)mt::ck_words(L.caps.seg)));
    const Launch *prev = L.src >= 0 ? &b->launches[(size_t)L.src] : nullptr;
    if (!L.cksrc.empty()) {
        HIPCHK(lbuf_alloc(b, &L.d_cksrc, L.cksrc.size()));
        HIPCHK(hipMemcpyAsync(L.d_cksrc, L.cksrc.data(), 4 * L.cksrc.size(), hipMemcpyHostToDevice, s));
    }
    mt::ReplayParams P = base_params(b);
    P.out = L.d_out;
    P.lab_out = L.d_lab;
    P.doc_out = L.d_docout;
    P.n_docs = n;
    P.doc_list = L.d_list;
    P.out_cap = L.out_cap;
    P.cold = L.d_cold;
    P.hbm_state = L.d_state;
    P.ck_out = L.d_ck;
    static const bool urgent_ok = !getenv("MT_EARLY_SETPRIO") || atoi(getenv("MT_EARLY_SETPRIO")) > 0;
    P.urgent = L.urgent && urgent_ok ? 1 : 0;
    if (L.notice) {
        P.notice = b->d_notice;
        P.notice_count = b->d_notice_count;
        P.launch_id = (int32_t)(&L - b->launches.data());
    }
    if (!L.cksrc.empty() && prev) {
        P.ck_in = prev->d_ck;
        P.ck_src = L.d_cksrc;
        P.cold_in = prev->d_cold;
        P.ck_in_words = mt::ck_words(prev->caps.seg);
        P.cold_in_seg = prev->caps.seg;
    }
#ifdef MT_PROF
    HIPCHK(lbuf_alloc(b, &L.d_prof, (size_t)n * mt::kProfSlots));
    P.prof = L.d_prof;
#endif
    const void *fn = L.load     ? kKernels[L.cls].load
                     : b->writer ? kKernels[L.cls].writer
                     : L.big && !mt::is_hbm_seg(mt::kClassSegs[L.cls]) ? kKernels[L.cls].bigprops
                                 : kKernels[L.cls].replay;
    if (getenv("MT_DEBUG_LAUNCHES"))
        fprintf(stderr, "mtreplay: launch class %d docs %lld resumed %d level %d lds %zu load %d\n", mt::kClassSegs[L.cls],
                (long long)n, (int)L.cksrc.size(), L.level, L.lds, (int)L.load);
    if (L.lds > 64 * 1024) HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds));
    void *args[] = {&P};
    // the giant class's observer replay runs a prefetch wave beside the replaying one
    // (MT_GIANT_PREFETCH=0: the replaying wave alone, for A/B profiles of the prefetch)
    static const bool giant_pf = !getenv("MT_GIANT_PREFETCH") || atoi(getenv("MT_GIANT_PREFETCH")) > 0;
    const unsigned threads =
        (giant_pf && fn == kKernels[L.cls].replay && L.cls == mt::kGiantClass) ? (unsigned)mt::kGiantThreads : 64u;
    HIPCHK(hipLaunchKernel(fn, dim3((unsigned)n), dim3(threads), args, L.lds, s));
    return MT_OK;
}

// initial capacity class of every document from its own op count; documents of one class
// form one launch (the HBM class in chunks of kMaxHbmDocs), largest documents first within a
// launch (blocks dispatch roughly in index order: the longest serial replays start first).
// Launches of different classes run concurrently on the run stream and up to 3 aux streams.
static int gather_launch(mt_batch *b, int li);

MT_API int mt_batch_launch(mt_batch *b, void *hip_stream) {
    if (!b || !b->have_log) return MT_ERR_STATE;
    // launches go to the batch's own non-blocking streams, ordered after the caller's stream
    hipStream_t s = b->stream;
    if (hip_stream && (hipStream_t)hip_stream != s) {
        if (!b->ev_user) HIPCHK(hipEventCreateWithFlags(&b->ev_user, hipEventDisableTiming));
        HIPCHK(hipEventRecord(b->ev_user, (hipStream_t)hip_stream));
        HIPCHK(hipStreamWaitEvent(s, b->ev_user, 0));
    }
    free_launches(b);
    b->snap_ready = false;  // buffers are kept for the next mt_batch_snapshots
    b->ran = false;
    b->cached_doc = -1;
    b->c_blob_doc = -1;
    b->t_launch = std::chrono::steady_clock::now();
    HIPCHK(hipEventRecord(b->ev0, s));
    // initial class: from the op count, and for a document that starts from a snapshot from its
    // loaded segments too (documents start in LDS: the largest LDS class at most, a document
    // reaches the HBM class only through a checkpoint, after its first ops ran at LDS speed)
    auto first_class = [&](int64_t d) {
        int32_t ops = (int32_t)(b->h_off[d + 1] - b->h_off[d]);
        int c = class_for(b, ops, 0);
        if (b->opt.seg_cap <= 0 && b->h_nload[d] > 0)
            while (c + 1 < mt::kNumClasses && mt::kClassSegs[c] < b->h_nload_segs[d] + b->h_nload_segs[d] / 4 + 64) c++;
        c = std::min(c, mt::kLastLdsClass);
        while (c > 0 && !class_usable(c)) c--;
        return c;
    };
    if (b->docout.size() != (size_t)b->n_docs) {
        b->docout.assign((size_t)b->n_docs, DocOut{});
        b->where.assign((size_t)b->n_docs, DocRes{});
    }
    // SnapshotLoader phase (snapshotLoader.ts:36-205): the leading LOAD records of every document
    // that has them run in mt_load_kernel, which checkpoints at the first catch-up op; a document
    // whose loaded tree outgrows its class is loaded again (or resumed) in the next one.
    std::vector<int32_t> resume_li((size_t)b->n_docs, -1), resume_idx((size_t)b->n_docs, -1);
    std::vector<uint8_t> loaded_final((size_t)b->n_docs, 0);
    {
        std::map<int, std::pair<std::vector<int32_t>, std::vector<int32_t>>> work;  // cls -> (docs, cksrc)
        std::map<int, int> work_src;
        for (int64_t d = 0; d < b->n_docs; d++)
            if (b->h_nload[d] > 0) work[first_class(d)].first.push_back((int32_t)d), work[first_class(d)].second.push_back(-1);
        while (!work.empty()) {
            const int cls = work.begin()->first;
            auto item = std::move(work.begin()->second);
            const int src = work_src.count(cls) ? work_src[cls] : -1;
            work.erase(work.begin());
            work_src.erase(cls);
            const size_t chunk = launch_chunk(cls, item.first.size());
            for (size_t at = 0; at < item.first.size(); at += chunk) {
                Launch L;
                L.cls = cls;
                L.load = true;
                const size_t e = std::min(item.first.size(), at + chunk);
                L.docs.assign(item.first.begin() + (long)at, item.first.begin() + (long)e);
                L.cksrc.assign(item.second.begin() + (long)at, item.second.begin() + (long)e);
                L.src = src;
                if (std::all_of(L.cksrc.begin(), L.cksrc.end(), [](int32_t x) { return x < 0; })) {
                    L.cksrc.clear();
                    L.src = -1;
                }
                b->launches.push_back(std::move(L));
                const int li = (int)b->launches.size() - 1;
                Launch &N = b->launches.back();
                HIPCHK(hipEventCreate(&N.e0));
                HIPCHK(hipEventCreate(&N.e1));
                HIPCHK(hipEventRecord(N.e0, s));
                int rc = launch_replay(b, s, N);
                if (rc) return rc;
                HIPCHK(hipEventRecord(N.e1, s));
                HIPCHK(hipEventSynchronize(N.e1));
                HIPCHK(hipEventElapsedTime(&N.ms, N.e0, N.e1));
                rc = gather_launch(b, li);
                if (rc) return rc;
                const Launch &S = b->launches[(size_t)li];
                for (size_t i = 0; i < S.docs.size(); i++) {
                    const int32_t d = S.docs[i];
                    const DocOut &o = b->docout[(size_t)d];
                    const bool long_seg = o.status == MT_CAPACITY && o.cap_kind == mt::kCapLongSeg;
                    // (the SnapshotLoader runs in the LDS classes and the HBM class, not the giant one)
                    int nxt = long_seg ? mt::kHbmClass : std::min(resume_class(cls), mt::kNumClasses - 1);
                    if (nxt == mt::kGiantClass) nxt = mt::kHbmClass;
                    if (o.status == MT_CAPACITY && o.cap_kind == mt::kCapCheckpoint && o.ops_done >= b->h_nload[d]) {
                        resume_li[(size_t)d] = li;  // loaded: the replay resumes from this checkpoint
                        resume_idx[(size_t)d] = (int32_t)i;
                    } else if (o.status == MT_CAPACITY && (o.cap_kind == mt::kCapCheckpoint || o.cap_kind == 1 || long_seg) &&
                               class_usable(nxt) && nxt > cls) {
                        // short of room while loading: resume (checkpoint) or load again (overflow)
                        auto &w = work[nxt];
                        if (w.first.empty() || !work_src.count(nxt) || work_src[nxt] == li) {
                            w.first.push_back(d);
                            w.second.push_back(o.cap_kind == mt::kCapCheckpoint ? (int32_t)i : -1);
                            if (o.cap_kind == mt::kCapCheckpoint) work_src[nxt] = li;
                        } else {
                            w.first.push_back(d);
                            w.second.push_back(-1);  // a different source launch: load from scratch
                        }
                    } else {
                        loaded_final[(size_t)d] = 1;  // loaded with no catch-up ops, or failed
                    }
                }
            }
        }
    }
    b->first0 = (int)b->launches.size();
    // replay launches: one per (initial class, source load launch), largest documents first
    std::map<std::pair<int, int>, std::vector<int32_t>, std::greater<std::pair<int, int>>> groups;
    int64_t n_replay = 0;
    for (int64_t d = 0; d < b->n_docs; d++) {
        if (loaded_final[(size_t)d]) continue;
        const int src = resume_li[(size_t)d];
        const int c = src >= 0 ? b->launches[(size_t)src].cls : first_class(d);
        groups[{c, src}].push_back((int32_t)d);
        n_replay++;
    }
    for (auto &g : groups) {
        const int cls = g.first.first, src = g.first.second;
        std::vector<int32_t> &docs = g.second;
        if (groups.size() == 1 && !class_in_hbm(cls) && src < 0 && n_replay == b->n_docs) {
            // every document, in index order; split into `first_split` launches of contiguous
            // documents, each escalating on its own as it completes, so one part's next class
            // fills the CUs that another part's tail leaves idle
            // (2 parts: config 3 +2.1 %; 4 parts: -5 %, every stream busy so escalations queue behind
            // unrelated tails).  Only batches that climb the ladder: at least 32,768
            // documents (a few rounds of the chip's residency) of >= 4,096 ops on average (config
            // 5's 2k-op documents finish in 1-2 classes and ran 2.5 % slower split).  MT_FIRST_SPLIT
            // overrides the part count.
            static const int64_t first_split = getenv("MT_FIRST_SPLIT") ? atoi(getenv("MT_FIRST_SPLIT")) : 2;
            const int64_t parts = std::max<int64_t>(1, std::min<int64_t>(first_split, 4));
            if (parts == 1 || b->n_docs < 32768 || (!getenv("MT_FIRST_SPLIT") && b->total_ops < 4096 * b->n_docs)) {
                Launch L;
                L.cls = cls;
                b->launches.push_back(L);
                break;
            }
            for (int64_t q = 0; q < parts; q++) {
                Launch L;
                L.cls = cls;
                for (int64_t d = b->n_docs * q / parts; d < b->n_docs * (q + 1) / parts; d++) L.docs.push_back((int32_t)d);
                b->launches.push_back(std::move(L));
            }
            break;
        }
        std::stable_sort(docs.begin(), docs.end(), [&](int32_t x, int32_t y) {
            return b->h_off[x + 1] - b->h_off[x] > b->h_off[y + 1] - b->h_off[y];
        });
        const size_t chunk = launch_chunk(cls, docs.size());
        for (size_t at = 0; at < docs.size(); at += chunk) {
            Launch L;
            L.cls = cls;
            L.docs.assign(docs.begin() + at, docs.begin() + std::min(docs.size(), at + chunk));
            if (src >= 0) {
                L.src = src;
                for (int32_t d : L.docs) L.cksrc.push_back(resume_idx[(size_t)d]);
            }
            b->launches.push_back(std::move(L));
        }
    }
    // early escalation (poll_notices) for first launches that most of their documents are expected
    // to fit (>= 90 % by the op-count estimate): the few that outgrow the class start their next
    // launch while it runs.  Not for batches that climb the ladder (config 3), whose mass escalation
    // the two first launches schedule.  MT_EARLY_ESCALATION=0: off; 2: every first launch.
    b->taken.assign((size_t)b->n_docs, 0);
    b->early_groups.clear();
    b->notice_cap = b->notice_read = 0;
    {
        static const int early = getenv("MT_EARLY_ESCALATION") ? atoi(getenv("MT_EARLY_ESCALATION")) : 1;
        for (size_t i = (size_t)b->first0; i < b->launches.size() && early > 0 && b->opt.max_retries != 0; i++) {
            Launch &L = b->launches[i];
            if (class_in_hbm(L.cls) || !class_usable(L.cls + 1) || !mt::notice_class(mt::kClassSegs[L.cls])) continue;
            const int64_t n = launch_n(b->n_docs, L);
            int64_t fit = 0;
            for (int64_t k = 0; k < n; k++) {
                const int64_t d = L.docs.empty() ? k : L.docs[(size_t)k];
                fit += (b->h_off[(size_t)d + 1] - b->h_off[(size_t)d]) / 12 + 64 <= mt::kClassSegs[L.cls];
            }
            L.notice = early >= 2 || 10 * fit >= 9 * n;
            if (L.notice) b->notice_cap += n;
        }
        if (b->notice_cap > b->notice_alloc) {
            if (b->h_notice) (void)hipHostFree(b->h_notice);
            b->h_notice = nullptr;
            HIPCHK(hipHostMalloc((void **)&b->h_notice, 16 * (size_t)b->notice_cap, hipHostMallocCoherent | hipHostMallocMapped));
            HIPCHK(hipHostGetDevicePointer((void **)&b->d_notice, b->h_notice, 0));
            b->notice_alloc = b->notice_cap;
        }
        if (b->notice_cap && !b->d_notice_count) HIPCHK(hipMalloc((void **)&b->d_notice_count, 4));
        if (b->notice_cap) {
            // (the previous run's kernels have all finished: free_launches waited for them)
            memset(b->h_notice, 0, 16 * (size_t)b->notice_cap);
            HIPCHK(hipMemsetAsync(b->d_notice_count, 0, 4, s));
            HIPCHK(hipStreamSynchronize(s));
        }
    }
    for (size_t i = (size_t)b->first0; i < b->launches.size(); i++) {
        Launch &L = b->launches[i];
        hipStream_t ls = s;
        if (i > (size_t)b->first0) {
            L.stream = 1 + (int)((i - (size_t)b->first0 - 1) % 3);
            hipStream_t &a = b->aux[L.stream - 1];
            if (!a) HIPCHK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
            HIPCHK(hipStreamWaitEvent(a, b->ev0, 0));
            ls = a;
        }
        HIPCHK(hipEventCreate(&L.e0));
        HIPCHK(hipEventCreate(&L.e1));
        HIPCHK(hipEventRecord(L.e0, ls));
        int rc = launch_replay(b, ls, L);
        if (rc) return rc;
        HIPCHK(hipEventRecord(L.e1, ls));
        if (ls != s) HIPCHK(hipStreamWaitEvent(s, L.e1, 0));
    }
    b->n_first = (int)b->launches.size();
    HIPCHK(hipEventRecord(b->ev1, s));
    b->run_stream = s;
    return MT_OK;
}

static int gather_launch(mt_batch *b, int li) {
    Launch &L = b->launches[li];
    int64_t n = launch_n(b->n_docs, L);
    if (n == 0) return MT_OK;
#ifdef MT_PROF
    {
        std::vector<uint64_t> pf((size_t)n * mt::kProfSlots);
        HIPCHK(hipMemcpy(pf.data(), L.d_prof, 8 * pf.size(), hipMemcpyDeviceToHost));
        double sum[mt::kProfSlots] = {0}, mx = 0;
        for (int64_t i = 0; i < n; i++)
            for (int k = 0; k < mt::kProfSlots; k++) {
                sum[k] += (double)pf[(size_t)i * mt::kProfSlots + k];
                if (k == 0 && (double)pf[(size_t)i * mt::kProfSlots] > mx) mx = (double)pf[(size_t)i * mt::kProfSlots];
            }
        fprintf(stderr, "MT_PROF launch %d docs %lld lds %zu: mean cycles/doc", li, (long long)n, L.lds);
        static const char *nm[mt::kProfSlots - 1] = {"kernel", "descend", "split", "insert", "range", "zamboni", "overlay", "scour",
                                                     "text", "heap", "pack", "settle", "scold", "resolve", "hforget"};
        for (int k = 0; k < mt::kProfSlots - 1; k++) fprintf(stderr, " %s=%.0f", nm[k], sum[k] / (double)n);
        fprintf(stderr, " max_kernel=%.0f\n", mx);
        // drain profile from each document's start / end on the 100 MHz realtime counter (the
        // last slot: start << 32 | end, low 32 bits each): the launch's span, how many documents
        // were resident at the peak and on average, and the tail after the last document started
        std::vector<std::pair<int64_t, int>> ev;
        ev.reserve(2 * (size_t)n);
        const uint32_t ref = (uint32_t)(pf[mt::kProfSlots - 1] >> 32);
        int64_t t_end = 0, last_start = 0, busy = 0, dmax = 0;
        for (int64_t i = 0; i < n; i++) {
            const uint64_t v = pf[(size_t)i * mt::kProfSlots + mt::kProfSlots - 1];
            const int64_t a = (int32_t)((uint32_t)(v >> 32) - ref), e = (int32_t)((uint32_t)v - ref);
            ev.push_back({a, 1});
            ev.push_back({e, -1});
            busy += e - a;
            dmax = std::max(dmax, e - a);
            last_start = std::max(last_start, a);
            t_end = std::max(t_end, e);
        }
        std::sort(ev.begin(), ev.end());
        const int64_t t0 = ev.front().first;
        int cur = 0, peak = 0;
        for (auto &x : ev) peak = std::max(peak, cur += x.second);
        const double span = (double)(t_end - t0);
        fprintf(stderr, "MT_PROF drain %d docs %lld: span_ms=%.3f mean_doc_ms=%.3f max_doc_ms=%.3f peak_resident=%d "
                        "mean_resident=%.1f packing=%.4f last_start_ms=%.3f tail_ms=%.3f\n",
                li, (long long)n, span * 1e-5, (double)busy / (double)n * 1e-5, (double)dmax * 1e-5, peak,
                (double)busy / span, (double)busy / (span * peak), (double)(last_start - t0) * 1e-5,
                (double)(t_end - last_start) * 1e-5);
    }
#endif
    std::vector<DocOut> tmp((size_t)n);
    if (!b->cstream) HIPCHK(hipStreamCreateWithFlags(&b->cstream, hipStreamNonBlocking));
    HIPCHK(hipMemcpyAsync(tmp.data(), L.d_docout, sizeof(DocOut) * (size_t)n, hipMemcpyDeviceToHost, b->cstream));
    HIPCHK(hipStreamSynchronize(b->cstream));
    if (b->docout.size() != (size_t)b->n_docs) {
        b->docout.assign((size_t)b->n_docs, DocOut{});
        b->where.assign((size_t)b->n_docs, DocRes{});
    }
    L.ops = L.early_ops;
    for (int64_t i = 0; i < n; i++) {
        int64_t d = L.docs.empty() ? i : L.docs[i];
        if (L.notice && b->taken[(size_t)d]) continue;  // escalated early: its results are another launch's
        const bool resumed = !L.cksrc.empty() && L.cksrc[(size_t)i] >= 0;
        L.ops += tmp[i].ops_done - (resumed ? b->docout[d].ops_done : 0);
        b->docout[d] = tmp[i];
        b->where[d].launch = li;
        b->where[d].idx = (int32_t)i;
    }
    L.gathered = true;
    return MT_OK;
}

// Capacity escalation, scheduled as launches complete: a checkpointed document resumes, a
// document that overflowed mid-op re-runs from scratch, both in the next class with >= 1.2x the
// slots (docs per CU matter more than the number of resumes: each resume costs one LDS image
// round trip to HBM).  When a launch finishes, its escalated documents are grouped by target
// class and launched at once on the next of the run / aux streams, so a large document's chain
// of classes never waits for unrelated launches (mixed-size batches, config 4).
// The launch goes on the stream with the fewest pending launches (ties: `prefer`, the stream of
// the launch that just finished, which is idle): a stream still running an unrelated launch would
// queue it behind that launch's tail.  (Keeping escalations off the run stream, which joins every
// first launch, measured +0.4 % but made rocprofv3's kernel trace serialize the two chains' aux
// queues, so its kernel durations no longer matched the bench's)
static int launch_on(mt_batch *b, Launch &&L, int prefer, std::vector<int> &pending) {
    if (std::all_of(L.cksrc.begin(), L.cksrc.end(), [](int32_t x) { return x < 0; })) L.cksrc.clear();
    int busy[6] = {0, 0, 0, 0, 0, 0};
    for (int p : pending) busy[b->launches[(size_t)p].stream]++;
    int k = prefer;
    if (k < 4)  // (4, 5: the early-escalation streams, chosen by poll_notices)
        for (int j = 0; j < 4; j++)
            if (busy[j] < busy[k]) k = j;
    L.stream = k;
    b->launches.push_back(std::move(L));
    const int li = (int)b->launches.size() - 1;
    Launch &N = b->launches.back();
    hipStream_t s = b->run_stream;
    if (k >= 4) {
        // early escalations: two streams of their own, so a normal escalation never queues behind one
        // (a stream of the highest priority measured the same: the dispatcher still fills the CUs the
        // running launch frees with its own smaller workgroups first)
        hipStream_t &a = b->early_s[k - 4];
        if (!a) HIPCHK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        s = a;
    } else if (k > 0) {
        hipStream_t &a = b->aux[k - 1];
        if (!a) HIPCHK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        s = a;
    }
    HIPCHK(hipEventCreate(&N.e0));
    HIPCHK(hipEventCreate(&N.e1));
    HIPCHK(hipEventRecord(N.e0, s));
    int rc = launch_replay(b, s, N);
    if (rc) return rc;
    HIPCHK(hipEventRecord(N.e1, s));
    pending.push_back(li);
    return MT_OK;
}

// escalating documents that a launch at class 1400 (~8 wave slots per CU) still runs concurrently
static constexpr int64_t kTailDocs = 1024;

// The next launch of an escalating document of launch S (workgroup i, results o): its class, kernel
// and checkpoint source (i: resume; -1: from scratch).  False: nothing to escalate to (the document
// keeps its status).  n_ck: how many of S's documents checkpointed (a tail below kTailDocs).
static bool escalation_target(const mt_batch *b, const Launch &S, const DocOut &o, int64_t n_ck, int32_t i, int *cls_out,
                              bool *big_out, int32_t *src_out) {
    int32_t src;
    if (o.cap_kind == mt::kCapCheckpoint && S.d_ck) src = i;
    else if (o.cap_kind == 1 || o.cap_kind == 4 || o.cap_kind == mt::kCapLongSeg || (o.cap_kind == mt::kCapPool && !S.big))
        src = -1;
    else return false;
    // a large property set: the same class again, from scratch, in the bigprops kernel
    // (the observer kernels of the LDS classes stop on large sets with kCapPool; the writer,
    // load and spill-class kernels hold them, so there it is a full pool: terminal)
    const bool to_big = o.cap_kind == mt::kCapPool;
    if (to_big && (S.big || b->writer || S.load || mt::is_hbm_seg(mt::kClassSegs[S.cls]))) return false;
    int cls = to_big ? S.cls : resume_class(S.cls);
    // a tail document checkpointed for overlay-list room (a wide collab window; the list grows
    // only by seg/16 per class) steps to the first class with ~64 entries to spare instead of one
    // class at a time, each step a serial launch of its own.  Only in a tail (a launch too small
    // to fill the chip at the bigger class): with many documents escalating, the smaller class's
    // residency wins.
    static const bool ulist_jump = !getenv("MT_ULIST_JUMP") || atoi(getenv("MT_ULIST_JUMP")) > 0;
    if (ulist_jump && n_ck <= kTailDocs && o.cap_kind == mt::kCapCheckpoint && S.cls < mt::kLastLdsClass &&
        o.max_oe + 16 > (int32_t)mt::class_caps(mt::kClassSegs[S.cls]).ulist)
        while (cls < mt::kLastLdsClass && (int32_t)mt::class_caps(mt::kClassSegs[cls]).ulist < o.max_oe + 64) cls++;
    while (cls > S.cls + 1 && !class_usable(cls)) cls--;
    // a segment beyond 16-bit lengths: re-run from scratch in the giant class (32-bit lengths)
    if (o.cap_kind == mt::kCapLongSeg) cls = long_seg_class(S.cls);
    if (!class_usable(cls)) return false;  // largest class reached: the document keeps MT_CAPACITY
    *cls_out = cls;
    *big_out = S.big || to_big;
    *src_out = src;
    return true;
}

// Submit escalation groups (keyed by target class x2 + bigprops): longest remaining replay first
// (LPT: workgroups dispatch roughly in index order, so the documents with the most ops left start
// first and the launch's tail is short; MT_LPT=0: the source launch's order), the HBM class in
// bounded chunks.
static int submit_groups(mt_batch *b, std::map<int, Launch> &groups, int prefer, std::vector<int> &pending) {
    static const bool host_timing = getenv("MT_HOST_TIMING") != nullptr;
    static const bool lpt = !getenv("MT_LPT") || atoi(getenv("MT_LPT")) > 0;
    for (auto &kv : groups) {
        Launch &G = kv.second;
        if (!lpt) continue;
        std::vector<std::pair<int64_t, size_t>> key(G.docs.size());
        for (size_t k = 0; k < G.docs.size(); k++) {
            const int32_t d = G.docs[k];
            const int64_t n_ops = b->h_off[(size_t)d + 1] - b->h_off[(size_t)d];
            key[k] = {G.cksrc[k] >= 0 ? n_ops - b->docout[(size_t)d].ops_done : n_ops, k};
        }
        std::stable_sort(key.begin(), key.end(), [](const std::pair<int64_t, size_t> &x, const std::pair<int64_t, size_t> &y) {
            return x.first > y.first;
        });
        std::vector<int32_t> docs(G.docs.size()), cks(G.cksrc.size());
        for (size_t k = 0; k < key.size(); k++) {
            docs[k] = G.docs[key[k].second];
            cks[k] = G.cksrc[key[k].second];
        }
        G.docs.swap(docs);
        G.cksrc.swap(cks);
    }
    for (auto &kv : groups) {
        Launch &G = kv.second;
        // the HBM class holds ~220 MB per document: bounded launches
        const size_t chunk = launch_chunk(G.cls, G.docs.size());
        for (size_t at = 0; at < G.docs.size(); at += chunk) {
            Launch L;
            L.cls = G.cls;
            L.big = G.big;
            L.src = G.src;
            L.level = G.level;
            const size_t e = std::min(G.docs.size(), at + chunk);
            L.urgent = G.urgent;
            L.docs.assign(G.docs.begin() + (long)at, G.docs.begin() + (long)e);
            L.cksrc.assign(G.cksrc.begin() + (long)at, G.cksrc.begin() + (long)e);
            const auto tl0 = std::chrono::steady_clock::now();
            const int rc = launch_on(b, std::move(L), prefer, pending);
            if (rc) return rc;
            if (host_timing)
                fprintf(stderr, "MT_HOST   launch %d (class %d, %zu docs, stream %d) submitted at %.1f ms host (%.2f ms)\n",
                        (int)b->launches.size() - 1, mt::kClassSegs[G.cls], e - at, b->launches.back().stream,
                        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - b->t_launch).count(),
                        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl0).count());
        }
    }
    groups.clear();
    return MT_OK;
}

// Early escalation (ReplayParams.notice): read the ring entries the running launches appended — a
// document that stopped with MT_CAPACITY, everything it wrote already visible beyond its XCD — and
// start their next launches on an idle aux stream while their source launches still run, so a
// handful of documents outgrowing a class that fits the rest (writer config 2, config 5) no longer
// replay alone after it.  Entries whose source launch has no idle stream yet wait in early_groups;
// the source launch's completion submits what is left (flush_src).
static int poll_notices(mt_batch *b, std::vector<int> &pending, int flush_src) {
    while (b->notice_read < b->notice_cap) {
        volatile uint32_t *e = b->h_notice + 4 * b->notice_read;
        const uint32_t w1 = e[0];
        if (!w1) break;
        std::atomic_thread_fence(std::memory_order_acquire);
        const uint32_t lw = e[1];
        const int li = (int)(lw & 0xFFFFFFu);
        DocOut o{};
        o.status = MT_CAPACITY;
        o.cap_kind = (int32_t)(lw >> 24);
        o.ops_done = (int32_t)e[2];
        o.max_oe = (int32_t)e[3];
        b->notice_read++;
        if (li < 0 || li >= (int)b->launches.size()) return MT_INTERNAL;
        Launch &S = b->launches[(size_t)li];
        // an entry read after its launch's gather (the ring is read in slot order, and a slot a
        // running launch reserved but has not written yet holds back the ones after it): the
        // completion path escalated that document already
        if (S.gathered) continue;
        const int32_t i = (int32_t)w1 - 1;
        if (i < 0 || i >= (int32_t)launch_n(b->n_docs, S)) return MT_INTERNAL;
        const int64_t d = S.docs.empty() ? i : S.docs[(size_t)i];
        int cls = 0;
        bool big = false;
        int32_t src = -1;
        if (S.level >= b->opt.max_retries || !escalation_target(b, S, o, 1, i, &cls, &big, &src)) continue;
        b->docout[(size_t)d] = o;  // (the fields the escalation reads; the final launch's gather fills the rest)
        b->where[(size_t)d] = DocRes{li, i};
        b->taken[(size_t)d] = 1;
        S.early_ops += o.ops_done;  // (a first launch: no resumed documents)
        Launch &G = b->early_groups[li][2 * cls + (big ? 1 : 0)];
        G.cls = cls;
        G.big = big;
        G.src = li;
        G.level = S.level + 1;
        G.urgent = true;
        G.docs.push_back((int32_t)d);
        G.cksrc.push_back(src);
    }
    for (auto it = b->early_groups.begin(); it != b->early_groups.end();) {
        int idle = -1;
        if (it->first != flush_src) {
            int busy[6] = {0, 0, 0, 0, 0, 0};
            for (int p : pending) busy[b->launches[(size_t)p].stream]++;
            for (int k = 4; k < 6 && idle < 0; k++)
                if (!busy[k]) idle = k;
            if (idle < 0) {
                ++it;
                continue;
            }
        } else {
            idle = b->launches[(size_t)it->first].stream;
        }
        const int rc = submit_groups(b, it->second, idle, pending);
        if (rc) return rc;
        it = b->early_groups.erase(it);
    }
    return MT_OK;
}

// Capacity escalation, scheduled as launches complete: a checkpointed document resumes, a
// document that overflowed mid-op re-runs from scratch, both in the next class with >= 1.2x the
// slots (docs per CU matter more than the number of resumes: each resume costs one LDS image
// round trip to HBM).  When a launch finishes, its escalated documents are grouped by target
// class and launched at once on the next of the run / aux streams, so a large document's chain
// of classes never waits for unrelated launches (mixed-size batches, config 4).
// The launch goes on the stream with the fewest pending launches (ties: `prefer`, the stream of
// the launch that just finished, which is idle): a stream still running an unrelated launch would
// queue it behind that launch's tail.  (Keeping escalations off the run stream, which joins every
// first launch, measured +0.4 % but made rocprofv3's kernel trace serialize the two chains' aux
// queues, so its kernel durations no longer matched the bench's)
MT_API int mt_batch_sync(mt_batch *b) {
    if (!b || b->launches.empty()) return MT_ERR_STATE;
    std::vector<int> pending;
    for (int li = b->first0; li < b->n_first; li++) pending.push_back(li);
    int rc = MT_OK;
    while (!pending.empty()) {
        size_t k = 0;
        for (;; std::this_thread::sleep_for(std::chrono::microseconds(20))) {
            for (k = 0; k < pending.size(); k++) {
                hipError_t q = hipEventQuery(b->launches[(size_t)pending[k]].e1);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) HIPCHK(q);
            }
            if (k < pending.size()) break;
            if (b->notice_cap) {
                rc = poll_notices(b, pending, -1);
                if (rc) return rc;
            }
        }
        const int li = pending[k];
        pending.erase(pending.begin() + (long)k);
        {
            Launch &L = b->launches[(size_t)li];
            HIPCHK(hipEventElapsedTime(&L.ms, L.e0, L.e1));
        }
        if (b->notice_cap && b->launches[(size_t)li].notice) {  // its last entries, and what waits of it
            rc = poll_notices(b, pending, li);
            if (rc) return rc;
        }
        static const bool host_timing = getenv("MT_HOST_TIMING") != nullptr;
        const auto th0 = std::chrono::steady_clock::now();
        rc = gather_launch(b, li);
        if (rc) return rc;
        if (host_timing) {
            float at = 0;
            (void)hipEventElapsedTime(&at, b->ev0, b->launches[(size_t)li].e1);
            fprintf(stderr, "MT_HOST launch %d (class %d) ended at %.1f ms; seen at %.1f ms host; gather %.2f ms\n", li,
                    mt::kClassSegs[b->launches[(size_t)li].cls], at,
                    std::chrono::duration<double, std::milli>(th0 - b->t_launch).count(),
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count());
        }
        const Launch &S = b->launches[(size_t)li];
        if (S.level >= b->opt.max_retries) continue;
        // launch_on appends to b->launches, so S dangles after the first one: what the escalations
        // need of it is copied here
        const int prefer = S.stream;
        const Launch Sc = [&] {
            Launch c;
            c.cls = S.cls;
            c.big = S.big;
            c.load = S.load;
            c.d_ck = S.d_ck;
            c.level = S.level;
            return c;
        }();
        const int64_t n = launch_n(b->n_docs, S);
        std::vector<int32_t> sdocs = S.docs;
        // documents poll_notices took from this launch (a launch's escalated documents are not)
        const bool notice = S.notice;
        std::map<int, Launch> groups;  // by target class, x2 + 1 for the bigprops kernel
        auto doc_of = [&](int64_t i) { return sdocs.empty() ? i : (int64_t)sdocs[(size_t)i]; };
        int64_t n_ck = 0;
        for (int64_t i = 0; i < n; i++) {
            const int64_t d = doc_of(i);
            n_ck += b->docout[d].status == MT_CAPACITY && b->where[d].launch == li && !(notice && b->taken[(size_t)d]);
        }
        for (int64_t i = 0; i < n; i++) {
            const int64_t d = doc_of(i);
            const DocOut &o = b->docout[d];
            if (o.status != MT_CAPACITY || b->where[d].launch != li || (notice && b->taken[(size_t)d])) continue;
            int cls = 0;
            bool big = false;
            int32_t src = -1;
            if (!escalation_target(b, Sc, o, n_ck, (int32_t)i, &cls, &big, &src)) continue;
            Launch &L = groups[2 * cls + (big ? 1 : 0)];
            L.cls = cls;
            L.big = big;
            L.src = li;
            L.level = Sc.level + 1;
            L.docs.push_back((int32_t)d);
            L.cksrc.push_back(src);
        }
        rc = submit_groups(b, groups, prefer, pending);
        if (rc) return rc;
    }
    if (!b->early_groups.empty()) return MT_INTERNAL;  // (flushed when their source launch completed)
    // device wall time: from the first launch to the last completion
    float ms = 0, mx = 0;
    for (const Launch &L : b->launches) {
        HIPCHK(hipEventElapsedTime(&ms, b->ev0, L.e1));
        mx = std::max(mx, ms);
    }
    b->kernel_ms = mx;
    b->total_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - b->t_launch).count();
    b->ran = true;
    // every launch of the run is submitted: cached buffers it did not take are released, so the
    // cache never holds memory beside a run's own
    lbuf_release(b);
    return MT_OK;
}

MT_API int mt_batch_run(mt_batch *b, void *hip_stream) {
    int rc = mt_batch_launch(b, hip_stream);
    if (rc) return rc;
    return mt_batch_sync(b);
}

MT_API int mt_batch_device_digests(mt_batch *b, uint64_t *dst, int32_t dst_is_device) {
    if (!b || !dst) return MT_ERR_ARG;
    if (!b->ran) return MT_ERR_STATE;
    if (!b->d_digest) HIPCHK(dalloc(&b->d_digest, (size_t)b->n_docs));
    hipStream_t s = b->run_stream ? b->run_stream : b->stream;
    // every document is hashed by exactly the launch that holds its final result (where[]), so
    // each entry of dst is written by this call, whatever the document's status
    size_t max_n = 0;
    for (const Launch &L : b->launches) max_n = std::max(max_n, (size_t)launch_n(b->n_docs, L));
    std::vector<uint8_t> mask(max_n * b->launches.size(), 0);
    for (int64_t d = 0; d < b->n_docs; d++) {
        const DocRes &w = b->where[(size_t)d];
        if (w.launch < 0 || w.idx < 0) return MT_INTERNAL;
        mask[(size_t)w.launch * max_n + (size_t)w.idx] = 1;
    }
    uint8_t *d_mask = nullptr;
    HIPCHK(dalloc(&d_mask, mask.size()));
    HIPCHK(hipMemcpyAsync(d_mask, mask.data(), mask.size(), hipMemcpyHostToDevice, s));
    for (size_t li = 0; li < b->launches.size(); li++) {
        const Launch &L = b->launches[li];
        mt::DigestParams P{};
        P.out = L.d_out;
        P.doc_out = L.d_docout;
        P.doc_list = L.d_list;
        P.n = launch_n(b->n_docs, L);
        if (P.n == 0) continue;
        P.out_cap = L.out_cap;
        P.text = b->d_text;
        P.doc_text_base = b->d_text_base;
        P.pool = b->d_pool;
        P.doc_pool_base = b->d_pool_base;
        P.final_mask = d_mask + li * max_n;
        P.dst = b->d_digest;
        void *args[] = {&P};
        HIPCHK(hipLaunchKernel((const void *)mt_digest_kernel, dim3((unsigned)P.n), dim3(64), args, 0, s));
    }
    HIPCHK(hipMemcpyAsync(dst, b->d_digest, 8 * (size_t)b->n_docs,
                          dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    (void)hipFree(d_mask);
    return MT_OK;
}

MT_API int mt_batch_get_stats(mt_batch *b, mt_batch_stats *o) {
    if (!b || !o) return MT_ERR_ARG;
    memset(o, 0, sizeof *o);
    o->n_docs = b->n_docs;
    o->n_ops = b->total_ops;
    o->launches = (int32_t)b->launches.size();
    o->kernel_ms = b->kernel_ms;
    o->total_ms = b->total_ms;
    if (!b->launches.empty()) {
        o->lds_bytes = (int32_t)b->launches[0].lds;
        o->lds_class = mt::kClassSegs[b->launches[0].cls];
    }
    if (!b->ran) return MT_OK;
    for (int64_t d = 0; d < b->n_docs; d++) {
        const DocOut &x = b->docout[d];
        o->ops_applied += x.ops_done;
        if (x.status != MT_OK) o->docs_failed++;
        o->max_oe = std::max(o->max_oe, x.max_oe);
        o->max_slots = std::max(o->max_slots, x.max_slots);
        o->max_blocks = std::max(o->max_blocks, x.max_blocks);
        o->max_heap = std::max(o->max_heap, x.max_heap);
    }
    return MT_OK;
}

// DESIGN.md "Roofline": per document 32 B per op record + 2 B per inserted code unit + 8 B per
// prop record (read) + 32 B per final table entry + 2 B per final text code unit (written).
MT_API int mt_batch_launch_info(mt_batch *b, int32_t i, mt_launch_info *o) {
    if (!b || !o) return MT_ERR_ARG;
    if (!b->ran) return MT_ERR_STATE;
    if (i < 0 || i >= (int32_t)b->launches.size()) return MT_ERR_ARG;
    const Launch &L = b->launches[(size_t)i];
    memset(o, 0, sizeof *o);
    o->seg_class = mt::kClassSegs[L.cls];
    o->n_docs = (int32_t)launch_n(b->n_docs, L);
    o->resumed = (int32_t)std::count_if(L.cksrc.begin(), L.cksrc.end(), [](int32_t x) { return x >= 0; });
    o->lds_bytes = (int32_t)L.lds;
    o->ms = L.ms;
    if (L.e0 && b->ev0) (void)hipEventElapsedTime(&o->start_ms, b->ev0, L.e0);
    o->ops = L.ops;
    return MT_OK;
}

MT_API int mt_batch_algorithmic_bytes(mt_batch *b, double *bytes) {
    if (!b || !bytes || !b->ran) return MT_ERR_STATE;
    double t = 32.0 * (double)b->total_ops + 2.0 * b->payload_units + 8.0 * b->prop_records;
    for (int64_t d = 0; d < b->n_docs; d++) t += 32.0 * (double)b->docout[d].n_out;
    // final text: visible code units == sum of live lengths; bounded by the payload, use the
    // device-reported table (exact) when cached per doc would cost a download — estimate with
    // the table's live segment lengths is done by callers that need it exactly.
    *bytes = t;
    return MT_OK;
}

MT_API int32_t mt_doc_status(mt_batch *b, int64_t doc) {
    if (!b || !b->ran || doc < 0 || doc >= b->n_docs) return -MT_ERR_ARG;
    return b->docout[doc].status;
}

MT_API int mt_batch_doc_counters(mt_batch *b, int32_t *out) {
    if (!b || !out) return MT_ERR_ARG;
    if (!b->ran) return MT_ERR_STATE;
    static_assert(sizeof(DocOut) == 4 * MT_DOC_COUNTERS, "DocOut layout");
    static_assert(MT_SNAP_META == mt::kSnapMeta, "snapshot meta row");
    for (int64_t d = 0; d < b->n_docs; d++) {
        int32_t *o = out + d * MT_DOC_COUNTERS;
        memcpy(o, &b->docout[(size_t)d], sizeof(DocOut));
        o[14] = b->where[(size_t)d].launch;
        o[15] = 0;
    }
    return MT_OK;
}

// ---------------------------------------------------------------- per-document results
static int load_doc(mt_batch *b, int64_t d) {
    if (!b->ran) return MT_ERR_STATE;
    if (d < 0 || d >= b->n_docs) return MT_ERR_ARG;
    if (b->cached_doc == d) return MT_OK;
    const DocRes &w = b->where[d];
    const Launch &L = b->launches[w.launch];
    b->c_out = b->docout[d];
    b->c_recs.resize((size_t)b->c_out.n_out);
    if (b->c_out.n_out)
        HIPCHK(hipMemcpy(b->c_recs.data(), L.d_out + (size_t)w.idx * L.out_cap, sizeof(OutRec) * b->c_recs.size(),
                         hipMemcpyDeviceToHost));
    b->c_lab.assign(L.d_lab ? b->c_recs.size() : 0, 0u);
    if (L.d_lab && b->c_out.n_out)
        HIPCHK(hipMemcpy(b->c_lab.data(), L.d_lab + (size_t)w.idx * L.out_cap, 4 * b->c_lab.size(), hipMemcpyDeviceToHost));
    uint32_t tt = std::min<uint32_t>(b->c_out.text_top, b->h_text_cap[d]);
    b->c_text.resize(tt);
    if (tt) HIPCHK(hipMemcpy(b->c_text.data(), b->d_text + b->h_text_base[d], 2ull * tt, hipMemcpyDeviceToHost));
    uint32_t pt = std::min<uint32_t>(b->c_out.pool_top, b->h_pool_cap[d]);
    b->c_pool.resize(pt);
    if (pt) HIPCHK(hipMemcpy(b->c_pool.data(), b->d_pool + b->h_pool_base[d], 4ull * pt, hipMemcpyDeviceToHost));
    b->cached_doc = d;
    b->load_gen++;
    return MT_OK;
}

static bool rec_is_marker(const OutRec &r) { return mt::out_is_end(r.blk); }
static bool rec_removed(const OutRec &r) { return r.rseq != mt::kNoneSeq; }
static bool rec_is_text(const OutRec &r) { return !(r.meta & mt::kMetaMarker); }

static const std::string &client_name(mt_batch *b, int64_t d, uint32_t id, std::string &tmp) {
    const auto &t = clients_of(b, d);
    if (id < t.size()) return t[id];
    // NonCollabClient segments of a loaded snapshot: Client.getLongClientId(-2) is "original"
    tmp = id == MT_CLIENT_NONCOLLAB ? "original" : "undefined";
    return tmp;
}

// JSON.stringify(properties): ordinary-object key order (array indices ascending, then
// insertion order), values as given in the value table
static void props_json(mt_batch *b, uint32_t id, std::string &o) {
    const uint32_t *p = b->c_pool.data() + id;
    uint32_t n = p[0];
    std::vector<std::pair<uint64_t, uint32_t>> order;
    order.reserve(n);
    for (uint32_t i = 0; i < n; i++) {
        uint32_t k = p[2 + 2 * i];
        uint64_t rank = (k < b->key_is_index.size() && b->key_is_index[k]) ? (uint64_t)b->key_index[k]
                                                                            : (1ull << 32) + i;
        order.push_back({rank, i});
    }
    std::sort(order.begin(), order.end());
    o.push_back('{');
    for (size_t j = 0; j < order.size(); j++) {
        uint32_t i = order[j].second;
        uint32_t k = p[2 + 2 * i], v = p[3 + 2 * i];
        if (j) o.push_back(',');
        json_quote8(o, k < b->keys.size() ? b->keys[k] : std::string("?"));
        o.push_back(':');
        o += v < b->values.size() ? b->values[v] : std::string("null");
    }
    o.push_back('}');
}

// matchProperties(a, c) of two prop sets of the cached document (a the earlier segment's);
// *undecided is set when a structural comparison could not be decided (kValUnknown)
static bool props_match_host(mt_batch *b, uint32_t a, uint32_t c, bool *undecided) {
    if (!a || !c) return a == c;
    const uint32_t *pa = b->c_pool.data() + a, *pc = b->c_pool.data() + c;
    if (pa[0] != pc[0]) return false;
    for (uint32_t i = 0; i < pa[0]; i++) {
        int rel = 0;
        for (uint32_t j = 0; j < pc[0]; j++)
            if (pa[2 + 2 * i] == pc[2 + 2 * j]) rel = host_value_rel(b, pa[3 + 2 * i], pc[3 + 2 * j]);
        if (rel < 0) *undecided = true;
        if (rel != 1) return false;
    }
    return true;
}

// removedClientOverlap of a record of the cached document: a mask of clients < 31, or a pool list
static std::vector<uint32_t> ovl_clients(const mt_batch *b, uint32_t ovl) {
    std::vector<uint32_t> out;
    if (!(ovl & mt::kOvlList)) {
        for (uint32_t c = 0; c < mt::kOvlMaskClients; c++)
            if (ovl & (1u << c)) out.push_back(c);
        return out;
    }
    const uint32_t o = ovl & ~mt::kOvlList;
    if (o >= b->c_pool.size()) return out;
    const uint32_t n = b->c_pool[o] & ~mt::kPoolOvlTag;
    for (uint32_t i = 0; i < n && o + 2 + i < b->c_pool.size(); i++) out.push_back(b->c_pool[o + 2 + i]);
    return out;
}

static int out_str(const std::string &s, char *buf, int64_t cap, int64_t *len) {
    if (len) *len = (int64_t)s.size();
    if (buf && cap > 0) {
        int64_t m = std::min<int64_t>((int64_t)s.size(), cap - 1);
        memcpy(buf, s.data(), (size_t)m);
        buf[m] = 0;
    }
    return MT_OK;
}

MT_API int mt_doc_text(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len) {
    if (!b) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    std::string o;
    for (const OutRec &r : b->c_recs)
        if (!rec_is_marker(r) && !rec_removed(r) && rec_is_text(r))
            utf16_to_utf8(o, b->c_text.data() + r.toff, r.len);
    return out_str(o, buf, cap, len);
}

MT_API int mt_doc_props_runs(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len) {
    if (!b) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    std::string o = "[";
    std::string run_props;
    int64_t pos = 0, run_start = 0, run_len = 0;
    bool first = true;
    auto flush = [&]() {
        if (run_len <= 0) return;
        if (!first) o.push_back(',');
        first = false;
        o += "[" + std::to_string(run_start) + "," + std::to_string(run_len) + "," + run_props + "]";
    };
    for (const OutRec &r : b->c_recs) {
        if (rec_is_marker(r) || rec_removed(r)) continue;
        std::string pj;
        if (!r.props) {
            pj = "null";
        } else {
            std::string j;
            props_json(b, r.props, j);
            std::vector<uint16_t> u = utf8_to_utf16(j);
            json_quote16(pj, u.data(), u.size());
        }
        if (run_len > 0 && pj == run_props) {
            run_len += r.len;
        } else {
            flush();
            run_props = pj;
            run_start = pos;
            run_len = r.len;
        }
        pos += r.len;
    }
    flush();
    o.push_back(']');
    return out_str(o, buf, cap, len);
}

// The labels of a Tile marker (refHasTileLabels / refHasTileLabel, mergeTree.ts:580-597): its
// referenceTileLabels value parsed as an array of strings.  0: not a tile (no Tile refType or no
// truthy labels), 1: labels in `out`, -1: a value the device does not model (a string — for-of
// would visit its code points — or non-string elements, which the block maps key by String(x)
// while the leaf test compares with ===).
// (ref_labels_of: the same for the key `tk` of the ref types `type_mask` — Tile: referenceTileLabels;
// NestBegin | NestEnd: referenceRangeLabels, refHasRangeLabels mergeTree.ts:584-586)
// (props: the prop set to read, by default the record's current one)
static int ref_labels_of(mt_batch *b, const OutRec &r, uint32_t tk, uint32_t type_mask, std::vector<std::u16string> &out,
                         uint32_t props = 0xFFFFFFFFu) {
    out.clear();
    if (props == 0xFFFFFFFFu) props = r.props;
    if (!(r.meta & mt::kMetaMarker) || !(r.toff & type_mask) || !props || tk == 0xFFFFFFFFu) return 0;
    if ((size_t)props + 2 > b->c_pool.size()) return -1;
    const uint32_t *p = b->c_pool.data() + props;
    uint32_t v = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < p[0]; i++)
        if (p[2 + 2 * i] == tk) v = p[3 + 2 * i];
    if (v == 0xFFFFFFFFu || v >= b->values.size() || (b->value_flags[v] & mt::kValFalsy)) return 0;
    const std::string &j = b->values[v];
    size_t i = 0;
    auto ws = [&]() { while (i < j.size() && (j[i] == ' ' || j[i] == '\t' || j[i] == '\n' || j[i] == '\r')) i++; };
    ws();
    if (i >= j.size() || j[i] != '[') return -1;
    i++;
    ws();
    if (i < j.size() && j[i] == ']') return 1;
    for (;;) {
        ws();
        if (i >= j.size() || j[i] != '"') return -1;
        size_t e = i + 1;
        while (e < j.size() && j[e] != '"') e += j[e] == '\\' ? 2 : 1;
        if (e >= j.size()) return -1;
        std::u16string s;
        if (!mt::js_string_of(j.substr(i, e + 1 - i), s)) return -1;
        out.push_back(s);
        i = e + 1;
        ws();
        if (i < j.size() && j[i] == ',') {
            i++;
            continue;
        }
        return (i < j.size() && j[i] == ']') ? 1 : -1;
    }
}
static int tile_labels_of(mt_batch *b, const OutRec &r, uint32_t tk, std::vector<std::u16string> &out) {
    return ref_labels_of(b, r, tk, 1u, out);
}

// The document's block tree, rebuilt from its final table: the leaves in document order, each leaf
// block closed by an end record naming the interior blocks that end with it (mt_engine.hip
// write_out).  Level-0 nodes list leaves (indices into `leaves`), level l > 0 nodes list nodes.
namespace {
struct TNode {
    int level;
    std::vector<int64_t> kids;
    int64_t len = 0;  // the local view's length (cachedLength)
};
}  // namespace
static int64_t rebuild_tree(mt_batch *b, std::vector<TNode> &nodes, std::vector<const OutRec *> &leaves,
                            std::vector<int64_t> &leaf_rec) {
    const int D = std::max(1, b->c_out.depth);
    std::vector<int64_t> open((size_t)D + 1, -1);
    int64_t root = -1;
    std::function<int64_t(int)> get_open = [&](int l) -> int64_t {
        if (open[(size_t)l] >= 0) return open[(size_t)l];
        nodes.push_back(TNode{l, {}, 0});
        const int64_t n = (int64_t)nodes.size() - 1;
        open[(size_t)l] = n;
        if (l + 1 <= D - 1) {
            const int64_t p = get_open(l + 1);
            nodes[(size_t)p].kids.push_back(n);
        } else {
            root = n;
        }
        return n;
    };
    TNode cur{0, {}, 0};
    for (size_t j = 0; j < b->c_recs.size(); j++) {
        const OutRec &r = b->c_recs[j];
        if (!rec_is_marker(r)) {
            cur.kids.push_back((int64_t)leaves.size());
            leaves.push_back(&r);
            leaf_rec.push_back((int64_t)j);
            continue;
        }
        nodes.push_back(std::move(cur));
        cur = TNode{0, {}, 0};
        const int64_t n = (int64_t)nodes.size() - 1;
        if (D == 1) root = n;
        else nodes[(size_t)get_open(1)].kids.push_back(n);
        for (uint32_t l = 1; l <= r.toff && l < (uint32_t)D; l++) open[l] = -1;
    }
    // lengths, children before parents
    std::function<void(int64_t)> sum = [&](int64_t n) {
        TNode &t = nodes[(size_t)n];
        t.len = 0;
        for (int64_t k : t.kids) {
            if (t.level == 0) {
                t.len += rec_removed(*leaves[(size_t)k]) ? 0 : (int64_t)leaves[(size_t)k]->len;
            } else {
                sum(k);
                t.len += nodes[(size_t)k].len;
            }
        }
    };
    if (root >= 0) sum(root);
    return root;
}
// the prop set a leaf block's last blockUpdate read a marker's labels from: the device's labels
// snapshot when the batch tracks them (annotates of referenceTileLabels / referenceRangeLabels leave
// the block maps stale until the next blockUpdate), else the current one
static uint32_t snap_props(mt_batch *b, const OutRec &r, int64_t rec) {
    return b->c_lab.empty() ? r.props : b->c_lab[(size_t)rec];
}

namespace {
struct RangeStacks {  // label -> stack of leaf indices, in key creation order
    std::vector<std::pair<std::u16string, std::vector<int64_t>>> s;
    std::vector<int64_t> &get(const std::u16string &k) {
        for (auto &e : s)
            if (e.first == k) return e.second;
        s.push_back({k, {}});
        return s.back().second;
    }
};
using Labels = std::vector<std::u16string>;
// The loaded document's tree and the maps its queries read, built once per load_doc: findTile /
// getStackContext at every position (beastTest's checkStacksAllPositions) cost a descent each,
// not a rebuild.  Tile maps are built per label on first use (a block's maps are only read for
// the asked-for label); range stacks carry every label.
struct DocTree {
    uint64_t gen = 0;  // mt_batch.load_gen it was built for
    std::vector<TNode> nodes;
    std::vector<const OutRec *> leaves;
    std::vector<int64_t> leaf_rec, lpos;  // lpos[i]: local position of leaf i (lpos[n]: the length)
    int64_t root = -1;
    bool tile_ready = false, tile_bad = false;
    std::vector<Labels> tile_cur, tile_snap;  // current labels / as of the leaf block's last blockUpdate
    std::unordered_map<std::u16string, std::pair<std::vector<int64_t>, std::vector<int64_t>>> tile_maps;
    bool range_ready = false, range_bad = false;
    std::vector<Labels> range_cur;
    std::vector<RangeStacks> rs;
};
}  // namespace

static DocTree &doc_tree(mt_batch *b) {
    if (!b->qtree) b->qtree = std::make_shared<DocTree>();
    DocTree &T = *(DocTree *)b->qtree.get();
    if (T.gen != b->load_gen) {
        T = DocTree();
        T.gen = b->load_gen;
        T.root = rebuild_tree(b, T.nodes, T.leaves, T.leaf_rec);
        T.lpos.assign(T.leaves.size() + 1, 0);
        for (size_t i = 0; i < T.leaves.size(); i++)
            T.lpos[i + 1] = T.lpos[i] + (rec_removed(*T.leaves[i]) ? 0 : (int64_t)T.leaves[i]->len);
    }
    return T;
}

// Client.findTile(startPos, tileLabel, preceding) (client.ts:1073-1076 -> MergeTree.findTile,
// mergeTree.ts:1763-1789) on the document's final table, in the replica's local view
// (refSeq UniversalSequenceNumber): search (preceding, posPrecedesTile) or backwardSearch
// (mergeTree.ts:1797-1870) with recordTileStart / tileShift (1000-1040) over the rebuilt tree, whose
// blocks carry rightmostTiles / leftmostTiles as their last blockUpdate built them (2748-2767 ->
// addNodeReferences 263-317: a leaf block reads its markers' labels at that time — an annotate of
// referenceTileLabels does not run blockUpdate, so the maps keep the labels of the last one — and an
// interior block extends its children's maps).  Leaves compare their current labels.
MT_API int mt_doc_find_tile(mt_batch *b, int64_t doc, int64_t start_pos, const char *label_utf8, int32_t preceding,
                            int64_t *tile_pos, char *props_buf, int64_t props_cap, int64_t *props_len) {
    if (!b || !label_utf8 || !tile_pos) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    *tile_pos = -1;
    if (props_len) *props_len = 0;
    if (b->c_out.status != MT_OK) return b->c_out.status;
    const std::vector<uint16_t> lu = utf8_to_utf16(std::string(label_utf8));
    const std::u16string label(lu.begin(), lu.end());
    uint32_t tk = 0xFFFFFFFFu;
    for (size_t k = 0; k < b->keys.size(); k++)
        if (b->keys[k] == "referenceTileLabels") tk = (uint32_t)k;
    DocTree &T = doc_tree(b);
    if (T.root < 0) return MT_INTERNAL;
    const std::vector<TNode> &nodes = T.nodes;
    const std::vector<const OutRec *> &leaves = T.leaves;
    auto local_len = [](const OutRec &r) -> int64_t { return rec_removed(r) ? 0 : (int64_t)r.len; };
    if (!T.tile_ready) {
        // every tile marker's labels are parsed once, so an unmodelled value anywhere is reported
        T.tile_cur.resize(leaves.size());
        T.tile_snap.resize(leaves.size());
        for (size_t k = 0; k < leaves.size(); k++) {
            const OutRec &r = *leaves[k];
            if (tile_labels_of(b, r, tk, T.tile_cur[k]) < 0) T.tile_bad = true;
            if (local_len(r) > 0 && (r.meta & mt::kMetaMarker) && (r.toff & 1u) &&
                ref_labels_of(b, r, tk, 1u, T.tile_snap[k], snap_props(b, r, T.leaf_rec[k])) < 0)
                T.tile_bad = true;
        }
        T.tile_ready = true;
    }
    if (T.tile_bad) return MT_UNSUPPORTED;
    // refHasTileLabel on the current labels (the leaf tests of recordTileStart / tileShift)
    auto labelled = [&](int64_t k) {
        for (const auto &l : T.tile_cur[(size_t)k])
            if (l == label) return true;
        return false;
    };
    auto mit = T.tile_maps.find(label);
    if (mit == T.tile_maps.end()) {
        // every block's maps for `label`: rightmost / leftmost leaf, -1 none
        std::vector<int64_t> right(nodes.size(), -1), left(nodes.size(), -1);
        std::function<void(int64_t)> update = [&](int64_t n) {
            const TNode &t = nodes[(size_t)n];
            for (int64_t k : t.kids) {
                if (t.level == 0) {
                    for (const auto &l : T.tile_snap[(size_t)k])
                        if (l == label) {
                            right[(size_t)n] = k;  // addTile
                            if (left[(size_t)n] < 0) left[(size_t)n] = k;  // addTileIfNotPresent
                        }
                } else {
                    update(k);
                    if (right[(size_t)k] >= 0) right[(size_t)n] = right[(size_t)k];  // Properties.extend
                    if (left[(size_t)n] < 0) left[(size_t)n] = left[(size_t)k];     // extendIfUndefined
                }
            }
        };
        update(T.root);
        mit = T.tile_maps.emplace(label, std::make_pair(std::move(right), std::move(left))).first;
    }
    const std::vector<int64_t> &right = mit->second.first, &left = mit->second.second;
    const int64_t root = T.root;
    int64_t tile = -1;
    if (preceding) {  // search -> searchBlock (1797-1829)
        int64_t pos = start_pos;
        for (int64_t n = root; n >= 0;) {
            const TNode &t = nodes[(size_t)n];
            int64_t next = -1;
            bool hit = false;
            for (int64_t k : t.kids) {
                const int64_t len = t.level == 0 ? local_len(*leaves[(size_t)k]) : nodes[(size_t)k].len;
                if (pos < len) {
                    hit = true;
                    if (t.level == 0) {
                        if (labelled(k)) tile = k;  // recordTileStart
                    } else {
                        next = k;
                    }
                    break;
                }
                if (t.level == 0) {  // tileShift of a leaf
                    if (len > 0 && labelled(k)) tile = k;
                } else if (right[(size_t)k] >= 0) {  // tileShift of a block
                    tile = right[(size_t)k];
                }
                pos -= len;
            }
            n = hit ? next : -1;
        }
    } else if (start_pos <= nodes[(size_t)root].len) {  // backwardSearch (1831-1870)
        int64_t pos = start_pos, seg_end = nodes[(size_t)root].len;
        for (int64_t n = root; n >= 0;) {
            const TNode &t = nodes[(size_t)n];
            int64_t next = -1;
            bool hit = false;
            for (size_t i = t.kids.size(); i-- > 0;) {
                const int64_t k = t.kids[i];
                const int64_t len = t.level == 0 ? local_len(*leaves[(size_t)k]) : nodes[(size_t)k].len;
                const int64_t segpos = seg_end - len;
                if (pos >= segpos) {
                    hit = true;
                    if (t.level == 0) {
                        if (labelled(k)) tile = k;
                    } else {
                        next = k;
                    }
                    break;
                }
                if (t.level == 0) {
                    if (len > 0 && labelled(k)) tile = k;
                } else if (left[(size_t)k] >= 0) {
                    tile = left[(size_t)k];
                }
                seg_end = segpos;
            }
            n = hit ? next : -1;
        }
    }
    if (tile < 0) return MT_OK;
    *tile_pos = T.lpos[(size_t)tile];
    std::string pj;
    if (leaves[(size_t)tile]->props) props_json(b, leaves[(size_t)tile]->props, pj);
    return out_str(pj, props_buf, props_cap, props_len);
}

// Client.getStackContext(startPos, rangeLabels) (client.ts:946-948 -> MergeTree.getStackContext,
// mergeTree.ts:1750-1760; SharedSegmentSequence.getStackContext, sequence/src/sequence.ts:377) on the
// document's final state in the replica's local view, over the rebuilt tree.  Every block's
// rangeStacks is the one its last blockUpdate built (addNodeReferences / applyStackDelta,
// mergeTree.ts:229-317): a leaf block from its markers' labels at that time (the labels snapshot when
// an annotate changed them since: stale maps, as in the reference), an interior block from its
// children's deltas.  The search is searchBlock with rangeShift / recordRangeLeaf
// (mergeTree.ts:953-994, 1797-1829): a preceding block applies its whole delta (every label),
// preceding leaves of the containing leaf block and the containing leaf only the asked-for labels
// of their current labels.
// Output (repo-defined shape): {label: [{"pos":P,"refType":T[,"props":{..}]}, ..]} in JS key order,
// stacks bottom to top.

MT_API int mt_doc_stack_context(mt_batch *b, int64_t doc, int64_t start_pos, const char *const *labels_utf8,
                                int32_t n_labels, char *buf, int64_t cap, int64_t *len) {
    if (!b || n_labels < 0 || (n_labels > 0 && !labels_utf8)) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    if (len) *len = 0;
    if (b->c_out.status != MT_OK) return b->c_out.status;
    std::vector<std::u16string> want;
    for (int32_t i = 0; i < n_labels; i++) {
        if (!labels_utf8[i]) return MT_ERR_ARG;
        const std::vector<uint16_t> lu = utf8_to_utf16(std::string(labels_utf8[i]));
        want.emplace_back(lu.begin(), lu.end());
    }
    uint32_t rk = 0xFFFFFFFFu;
    for (size_t k = 0; k < b->keys.size(); k++)
        if (b->keys[k] == "referenceRangeLabels") rk = (uint32_t)k;
    DocTree &T = doc_tree(b);
    if (T.root < 0) return MT_INTERNAL;
    const std::vector<TNode> &nodes = T.nodes;
    const std::vector<const OutRec *> &leaves = T.leaves;
    auto local_len = [](const OutRec &r) -> int64_t { return rec_removed(r) ? 0 : (int64_t)r.len; };
    // applyRangeReference (mergeTree.ts:246-261): NestBegin pushes; an end pops a NestBegin on top
    auto apply_ref = [&](std::vector<int64_t> &st, int64_t leaf) {
        if (leaves[(size_t)leaf]->toff & 2u) {
            st.push_back(leaf);
        } else if (!st.empty() && (leaves[(size_t)st.back()]->toff & 2u)) {
            st.pop_back();
        } else {
            st.push_back(leaf);
        }
    };
    auto apply_delta = [&](RangeStacks &cur, const RangeStacks &delta) {  // applyStackDelta (229-244)
        for (const auto &e : delta.s) {
            if (e.second.empty()) continue;
            std::vector<int64_t> &c = cur.get(e.first);
            for (int64_t x : e.second) apply_ref(c, x);
        }
    };
    if (!T.range_ready) {
        // every label list is parsed once (the reference's blockUpdate iterates them all); blockUpdate's
        // rangeStacks, children before parents: a leaf block reads its markers' labels as of its last
        // blockUpdate (the labels snapshot)
        Labels labels;
        T.range_cur.resize(leaves.size());
        for (size_t k = 0; k < leaves.size(); k++)  // refHasRangeLabels + getRangeLabels (current)
            if (ref_labels_of(b, *leaves[k], rk, 6u, T.range_cur[k]) < 0) T.range_bad = true;
        T.rs.assign(nodes.size(), RangeStacks());
        std::function<void(int64_t)> update = [&](int64_t n) {
            const TNode &t = nodes[(size_t)n];
            for (int64_t k : t.kids) {
                if (t.level == 0) {
                    const OutRec &r = *leaves[(size_t)k];
                    if (local_len(r) <= 0 || !(r.meta & mt::kMetaMarker) || !(r.toff & 6u)) continue;
                    const int tl = ref_labels_of(b, r, rk, 6u, labels, snap_props(b, r, T.leaf_rec[(size_t)k]));
                    if (tl < 0) T.range_bad = true;
                    if (tl > 0)
                        for (const auto &l : labels) apply_ref(T.rs[(size_t)n].get(l), k);  // updateRangeInfo
                } else {
                    update(k);
                    apply_delta(T.rs[(size_t)n], T.rs[(size_t)k]);
                }
            }
        };
        update(T.root);
        T.range_ready = true;
    }
    if (T.range_bad) return MT_UNSUPPORTED;
    const std::vector<RangeStacks> &rs = T.rs;
    const int64_t root = T.root;
    RangeStacks out;
    auto leaf_marker = [&](int64_t k) {  // applyLeafRangeMarker (953-964): the asked-for labels in order
        for (const auto &w : want)
            for (const auto &l : T.range_cur[(size_t)k])
                if (l == w) {
                    apply_ref(out.get(w), k);
                    break;
                }
    };
    int64_t pos = start_pos;
    for (int64_t n = root;;) {
        const TNode &t = nodes[(size_t)n];
        int64_t next = -1;
        for (int64_t k : t.kids) {
            const int64_t len = t.level == 0 ? local_len(*leaves[(size_t)k]) : nodes[(size_t)k].len;
            if (pos < len) {
                if (t.level == 0) {
                    const OutRec &r = *leaves[(size_t)k];
                    if ((r.meta & mt::kMetaMarker) && (r.toff & 6u)) leaf_marker(k);  // recordRangeLeaf
                } else {
                    next = k;
                }
                break;
            }
            if (t.level == 0) {  // rangeShift of a leaf
                const OutRec &r = *leaves[(size_t)k];
                if (len > 0 && (r.meta & mt::kMetaMarker) && (r.toff & 6u)) leaf_marker(k);
            } else {  // rangeShift of a block
                apply_delta(out, rs[(size_t)k]);
            }
            pos -= len;
        }
        if (next < 0) break;
        n = next;
    }
    // JSON: integer-like keys ascending first, then creation order
    std::vector<size_t> order;
    std::vector<std::pair<uint32_t, size_t>> idx;
    for (size_t i = 0; i < out.s.size(); i++) {
        uint32_t v = 0;
        std::string k8;
        for (char16_t c : out.s[i].first) k8.push_back(c < 0x80 ? (char)c : '\x01');
        if (array_index(k8, &v)) idx.push_back({v, i});
    }
    std::sort(idx.begin(), idx.end());
    for (auto &e : idx) order.push_back(e.second);
    for (size_t i = 0; i < out.s.size(); i++) {
        uint32_t v = 0;
        std::string k8;
        for (char16_t c : out.s[i].first) k8.push_back(c < 0x80 ? (char)c : '\x01');
        if (!array_index(k8, &v)) order.push_back(i);
    }
    const std::vector<int64_t> &lpos = T.lpos;
    std::string o = "{";
    for (size_t q = 0; q < order.size(); q++) {
        const auto &e = out.s[order[q]];
        if (q) o.push_back(',');
        json_quote16(o, (const uint16_t *)e.first.data(), e.first.size());
        o += ":[";
        for (size_t j = 0; j < e.second.size(); j++) {
            const OutRec &r = *leaves[(size_t)e.second[j]];
            if (j) o.push_back(',');
            o += "{\"pos\":" + std::to_string(lpos[(size_t)e.second[j]]) + ",\"refType\":" + std::to_string(r.toff);
            if (r.props) {
                std::string pj;
                props_json(b, r.props, pj);
                o += ",\"props\":" + pj;
            }
            o.push_back('}');
        }
        o.push_back(']');
    }
    o.push_back('}');
    return out_str(o, buf, cap, len);
}

// JSON.stringify of a property object given as (key, value) records in insertion order (JS key
// order: integer-like keys first, as props_json does for pool sets)
static void pairs_json(mt_batch *b, const uint32_t *kv, uint32_t n, std::string &o) {
    std::vector<std::pair<uint64_t, uint32_t>> order;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t k = kv[2 * i];
        const uint64_t rank = (k < b->key_is_index.size() && b->key_is_index[k]) ? (uint64_t)b->key_index[k]
                                                                              : (1ull << 32) + i;
        order.push_back({rank, i});
    }
    std::sort(order.begin(), order.end());
    o.push_back('{');
    for (size_t j = 0; j < order.size(); j++) {
        const uint32_t k = kv[2 * order[j].second], v = kv[2 * order[j].second + 1];
        if (j) o.push_back(',');
        json_quote8(o, k < b->keys.size() ? b->keys[k] : std::string("?"));
        o.push_back(':');
        o += v < b->values.size() ? b->values[v] : std::string("null");
    }
    o.push_back('}');
}

// Client.regeneratePendingOp results of the document's MT_OP_REGENERATE records, in order: a JSON
// array with one element per regenerated message (records chained by MT_OPF_GROUP_CONT form one):
// the op, or createGroupOp(...ops) when it is not exactly one (client.ts:885), keys in
// opBuilder.ts order
MT_API int mt_doc_regenerated_ops(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len) {
    if (!b) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    std::string o = "[";
    if (b->writer && !b->h_regen_base.empty()) {
        const uint64_t a = b->h_regen_base[(size_t)doc], e = b->h_regen_base[(size_t)doc + 1];
        std::vector<uint32_t> w((size_t)(e - a));
        if (!w.empty())
            HIPCHK(hipMemcpy(w.data(), b->d_regen + a, 4 * w.size(), hipMemcpyDeviceToHost));
        const uint32_t used = w.size() >= 2 ? std::min<uint32_t>(w[0], (uint32_t)w.size()) : 0;
        std::vector<std::string> msg_ops;
        bool first_msg = true;
        for (uint32_t p = 2; p + 2 <= used;) {
            const uint32_t cont = w[p], nops = w[p + 1];
            p += 2;
            for (uint32_t k = 0; k < nops && p + mt::kRegenOpWords <= used; k++) {
                const uint32_t *r = &w[p];
                std::string j;
                if (r[0] == MT_OP_INSERT) {
                    j = "{\"pos1\":" + std::to_string(r[1]) + ",\"seg\":";
                    const bool has_props = r[6] != 0xFFFFFFFFu;
                    const uint32_t np = has_props ? r[6] : 0;
                    std::string pj;
                    if (has_props) pairs_json(b, r + mt::kRegenOpWords, np, pj);
                    if (r[3] & 1u) {
                        j += "{\"marker\":{\"refType\":" + std::to_string(r[3] >> 1) + "}";
                        if (has_props) j += ",\"props\":" + pj;
                        j += "}";
                    } else {
                        std::string t;
                        if ((size_t)r[4] + r[5] <= b->c_text.size())
                            json_quote16(t, b->c_text.data() + r[4], r[5]);
                        j += has_props ? "{\"text\":" + t + ",\"props\":" + pj + "}" : t;
                    }
                    j += ",\"type\":0}";
                    p += mt::kRegenOpWords + 2 * np;
                } else if (r[0] == MT_OP_REMOVE) {
                    j = "{\"pos1\":" + std::to_string(r[1]) + ",\"pos2\":" + std::to_string(r[2]) + ",\"type\":1}";
                    p += mt::kRegenOpWords;
                } else {
                    j = "{";
                    if (r[3] & MT_OPF_REWRITE) j += "\"combiningOp\":{\"name\":\"rewrite\"},";
                    j += "\"pos1\":" + std::to_string(r[1]) + ",\"pos2\":" + std::to_string(r[2]) + ",\"props\":";
                    std::vector<uint32_t> kv;
                    for (uint32_t q = 0; q < r[5] && (size_t)r[4] + q < b->h_props_all.size(); q++) {
                        kv.push_back(b->h_props_all[r[4] + q].key);
                        kv.push_back(b->h_props_all[r[4] + q].value);
                    }
                    std::string pj;
                    pairs_json(b, kv.data(), (uint32_t)(kv.size() / 2), pj);
                    j += pj + ",\"type\":2}";
                    p += mt::kRegenOpWords;
                }
                msg_ops.push_back(j);
            }
            if (!cont) {
                if (!first_msg) o.push_back(',');
                first_msg = false;
                if (msg_ops.size() == 1) {
                    o += msg_ops[0];
                } else {
                    o += "{\"ops\":[";
                    for (size_t i = 0; i < msg_ops.size(); i++) o += (i ? "," : "") + msg_ops[i];
                    o += "],\"type\":3}";
                }
                msg_ops.clear();
            }
        }
    }
    o.push_back(']');
    return out_str(o, buf, cap, len);
}

// The consensus callbacks a writer replica's replay made, in call order: each
// annotateMarkerNotifyConsensus whose ack registered a min-seq listener (client.ts:980-987) calls
// consensusInfo.callback(marker) when minSeq reaches the ack's seq (notifyMinSeqListeners,
// mergeTree.ts:1709-1716).  The device queues the listeners in seq order; equal seqs (one GROUP
// message) pop in the order of the reference's binary heap (collections.ts:213-265), which is
// replayed here from the registration and firing times.
MT_API int mt_doc_consensus_events(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len) {
    if (!b) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    std::string o = "[";
    if (b->d_cons && !b->h_cons_base.empty()) {
        const uint64_t a = b->h_cons_base[(size_t)doc], e = b->h_cons_base[(size_t)doc + 1];
        std::vector<uint32_t> w((size_t)(e - a));
        if (!w.empty()) HIPCHK(hipMemcpy(w.data(), b->d_cons + a, 4 * w.size(), hipMemcpyDeviceToHost));
        if (w.size() >= (size_t)mt::kConsHdr) {
            const uint32_t nl = std::min(w[1], w[4]), fired = std::min(w[2], nl);
            const uint32_t *L = w.data() + mt::kConsHdr + w[3];
            struct Lis {
                uint32_t i;
                int64_t s;
            };
            // timeline: registration at the ack's message, firing after that message's ack(s)
            std::vector<std::pair<int64_t, int64_t>> ev;  // (time, index): time = 2 seq (+1: firing)
            for (uint32_t i = 0; i < nl; i++) ev.push_back({2 * (int64_t)L[mt::kConsLis * i + 1], i});
            for (uint32_t i = 0; i < fired; i++) ev.push_back({2 * (int64_t)L[mt::kConsLis * i + 4] + 1, -1 - (int64_t)i});
            std::stable_sort(ev.begin(), ev.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
            std::vector<Lis> H(1, Lis{0, INT64_MIN});  // L[0]: comp.min
            auto cmp = [&](size_t x, size_t y) { return H[x].s - H[y].s; };
            std::vector<uint32_t> order;
            int64_t last_fire = -1;
            for (const auto &t : ev) {
                if (t.second >= 0) {  // Heap.add: push + fixup
                    H.push_back(Lis{(uint32_t)t.second, (int64_t)L[mt::kConsLis * t.second + 1]});
                    for (size_t k = H.size() - 1; k > 1 && cmp(k >> 1, k) > 0; k >>= 1) std::swap(H[k >> 1], H[k]);
                    continue;
                }
                if (t.first == last_fire) continue;  // one notifyMinSeqListeners per message
                last_fire = t.first;
                const int64_t msn = (int64_t)L[mt::kConsLis * (uint32_t)(-1 - t.second) + 3];
                while (H.size() > 1 && H[1].s <= msn) {  // Heap.get: last to the root + fixdown
                    order.push_back(H[1].i);
                    H[1] = H.back();
                    H.pop_back();
                    const size_t n = H.size() - 1;
                    for (size_t k = 1; (k << 1) <= n;) {
                        size_t j = k << 1;
                        if (j < n && cmp(j, j + 1) > 0) j++;
                        if (cmp(k, j) <= 0) break;
                        std::swap(H[k], H[j]);
                        k = j;
                    }
                }
            }
            for (size_t q = 0; q < order.size(); q++) {
                const uint32_t *r = L + mt::kConsLis * order[q];
                if (q) o.push_back(',');
                o += "{\"markerId\":";
                o += r[0] < b->values.size() ? b->values[r[0]] : std::string("null");
                o += ",\"seq\":" + std::to_string(r[1]) + ",\"minSeq\":" + std::to_string(r[3]) + "}";
            }
        }
    }
    o.push_back(']');
    return out_str(o, buf, cap, len);
}

// segment.toJSONObject() (textSegment.ts:48-54, mergeTree.ts:652-656)
static void seg_json(mt_batch *b, bool text, const uint16_t *t, size_t n, uint32_t ref_type, uint32_t props,
                     std::string &o) {
    if (text) {
        if (props) {
            o += "{\"text\":";
            json_quote16(o, t, n);
            o += ",\"props\":";
            props_json(b, props, o);
            o.push_back('}');
        } else {
            json_quote16(o, t, n);
        }
    } else {
        o += "{\"marker\":{\"refType\":" + std::to_string(ref_type) + "}";
        if (props) {
            o += ",\"props\":";
            props_json(b, props, o);
        }
        o.push_back('}');
    }
}

// SnapshotV1.extractSync + emit (snapshotV1.ts:85-247, snapshotChunks.ts:122-131)
MT_API int mt_doc_snapshot_v1(mt_batch *b, int64_t doc, int32_t *n_blobs) {
    if (!b) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    const int32_t min_seq = b->c_out.min_seq, cur_seq = b->c_out.cur_seq;
    std::vector<std::string> segs;
    std::vector<int64_t> lens;
    // coalescing candidate (a clone in the reference: snapshotV1.ts:191-210)
    bool have_prev = false, prev_text = true;
    std::vector<uint16_t> ptext;
    uint32_t pref = 0, pprops = 0;
    auto push_prev = [&]() {
        if (!have_prev) return;
        std::string j;
        seg_json(b, prev_text, ptext.data(), ptext.size(), pref, pprops, j);
        segs.push_back(j);
        lens.push_back(prev_text ? (int64_t)ptext.size() : 1);
        have_prev = false;
    };
    auto set_prev = [&](const OutRec &r) {
        have_prev = true;
        prev_text = rec_is_text(r);
        pref = r.toff;
        pprops = r.props;
        ptext.clear();
        if (prev_text) ptext.assign(b->c_text.begin() + r.toff, b->c_text.begin() + r.toff + r.len);
    };
    std::string tmp;
    bool undecided = false;
    for (const OutRec &r : b->c_recs) {
        if (rec_is_marker(r)) continue;
        bool removed = rec_removed(r);
        // unacked inserts and segments removed at or below the MSN (incl. a pending local remove,
        // removedSeq -1) are elided (snapshotV1.ts:184-186)
        if (r.seq == mt::kUnassignedSeq || (removed && r.rseq <= min_seq)) continue;
        if (r.seq <= min_seq && !removed) {
            if (!have_prev) {
                set_prev(r);
            } else {
                bool can = prev_text && rec_is_text(r) && !(!ptext.empty() && ptext.back() == (uint16_t)'\n') &&
                           (ptext.size() <= mt::kGranularity || r.len <= mt::kGranularity);
                if (can && props_match_host(b, pprops, r.props, &undecided)) {
                    ptext.insert(ptext.end(), b->c_text.begin() + r.toff, b->c_text.begin() + r.toff + r.len);
                } else {
                    push_prev();
                    set_prev(r);
                }
            }
        } else {
            push_prev();
            std::string j = "{\"json\":";
            seg_json(b, rec_is_text(r), b->c_text.data() + (rec_is_text(r) ? r.toff : 0), rec_is_text(r) ? r.len : 0,
                     r.toff, r.props, j);
            if (r.seq > min_seq) {
                j += ",\"seq\":" + std::to_string(r.seq) + ",\"client\":";
                json_quote8(j, client_name(b, doc, mt::meta_cli(r.meta), tmp));
            }
            if (removed) {
                j += ",\"removedSeq\":" + std::to_string(r.rseq) + ",\"removedClient\":";
                json_quote8(j, client_name(b, doc, mt::meta_rcli(r.meta), tmp));
            }
            j.push_back('}');
            segs.push_back(j);
            lens.push_back(r.len);
        }
    }
    push_prev();
    if (undecided) return MT_UNSUPPORTED;  // a structural matchProperties the tables could not decide
    // emit: chunks of >= chunk_size code units (each chunk includes the segment that crosses)
    struct Chunk {
        int64_t start, count, length;
    };
    std::vector<Chunk> chunks;
    int64_t total_count = 0, total_length = 0;
    do {
        int64_t length = 0, count = 0;
        while (length < b->opt.chunk_size && total_count + count < (int64_t)segs.size()) {
            length += lens[total_count + count];
            count++;
        }
        chunks.push_back({total_count, count, length});
        total_count += count;
        total_length += length;
    } while (total_count < (int64_t)segs.size());
    b->c_blob_names.clear();
    b->c_blobs.clear();
    for (size_t ci = 0; ci < chunks.size(); ci++) {
        std::string j = "{\"version\":\"1\",\"segmentCount\":" + std::to_string(chunks[ci].count) +
                        ",\"length\":" + std::to_string(chunks[ci].length) + ",\"segments\":[";
        for (int64_t k = 0; k < chunks[ci].count; k++) {
            if (k) j.push_back(',');
            j += segs[chunks[ci].start + k];
        }
        j += "],\"startIndex\":" + std::to_string(chunks[ci].start);
        if (ci == 0) {
            j += ",\"headerMetadata\":{\"minSequenceNumber\":" + std::to_string(min_seq) +
                 ",\"sequenceNumber\":" + std::to_string(cur_seq) + ",\"orderedChunkMetadata\":[{\"id\":\"header\"}";
            for (size_t bi = 1; bi < chunks.size(); bi++) j += ",{\"id\":\"body_" + std::to_string(bi - 1) + "\"}";
            j += "],\"totalLength\":" + std::to_string(total_length) +
                 ",\"totalSegmentCount\":" + std::to_string(total_count) + "}";
        }
        j.push_back('}');
        b->c_blob_names.push_back(ci == 0 ? std::string("header") : "body_" + std::to_string(ci - 1));
        b->c_blobs.push_back(j);
    }
    b->c_blob_doc = doc;
    if (n_blobs) *n_blobs = (int32_t)b->c_blobs.size();
    return MT_OK;
}

MT_API int mt_doc_snapshot_blob(mt_batch *b, int64_t doc, int32_t i, char *name, int64_t name_cap, char *buf,
                                int64_t cap, int64_t *len) {
    if (!b) return MT_ERR_ARG;
    if (b->c_blob_doc != doc) {
        int rc = mt_doc_snapshot_v1(b, doc, nullptr);
        if (rc) return rc;
    }
    if (i < 0 || i >= (int32_t)b->c_blobs.size()) return MT_ERR_ARG;
    if (name && name_cap > 0) snprintf(name, (size_t)name_cap, "%s", b->c_blob_names[i].c_str());
    return out_str(b->c_blobs[i], buf, cap, len);
}

// ---------------------------------------------------------------- SnapshotV1 on the GPU
// mt_snapshot.hip: pass 0 sizes every document's chunks, the host prefix-sums the bytes, pass 1
// writes all blobs into one device buffer.  Same bytes as mt_doc_snapshot_v1 above.
MT_API int mt_batch_snapshots(mt_batch *b, int64_t *total_bytes, float *device_ms) {
    if (!b) return MT_ERR_ARG;
    if (!b->ran) return MT_ERR_STATE;
    b->snap_ready = false;
    hipStream_t s = b->run_stream ? b->run_stream : b->stream;
    // string tables: JSON.stringify(key), value JSON texts, JSON.stringify(long client id)
    std::string strs;
    std::vector<uint32_t> key_str, key_rank, val_str, cli_str;
    auto add = [&](std::vector<uint32_t> &tab, const std::string &js) {
        tab.push_back((uint32_t)strs.size());
        tab.push_back((uint32_t)js.size());
        strs += js;
    };
    auto add_quoted = [&](std::vector<uint32_t> &tab, const std::string &raw) {
        std::string q;
        json_quote8(q, raw);
        add(tab, q);
    };
    for (size_t k = 0; k < b->keys.size(); k++) {
        add_quoted(key_str, b->keys[k]);
        key_rank.push_back(b->key_is_index[k] ? b->key_index[k] : 0xFFFFFFFFu);
    }
    add_quoted(key_str, "?");
    key_rank.push_back(0xFFFFFFFFu);
    for (const std::string &v : b->values) add(val_str, v);
    add_quoted(cli_str, "undefined");
    add_quoted(cli_str, "original");  // MT_CLIENT_NONCOLLAB
    const int32_t cli_first = 2, cli_n = (int32_t)b->clients.size();
    for (const std::string &c : b->clients) add_quoted(cli_str, c);
    std::vector<int32_t> doc_cli;
    if (!b->doc_clients.empty()) {
        doc_cli.resize(2 * (size_t)b->n_docs);
        for (int64_t d = 0; d < b->n_docs; d++) {
            auto it = b->doc_clients.find(d);
            if (it == b->doc_clients.end()) {
                doc_cli[2 * d] = cli_first;
                doc_cli[2 * d + 1] = cli_n;
            } else {
                doc_cli[2 * d] = (int32_t)(cli_str.size() / 2);
                doc_cli[2 * d + 1] = (int32_t)it->second.size();
                for (const std::string &c : it->second) add_quoted(cli_str, c);
            }
        }
    }
    if (strs.empty()) strs.push_back(0);
    uint8_t *d_strs = nullptr;
    uint32_t *d_key_str = nullptr, *d_key_rank = nullptr, *d_val_str = nullptr, *d_cli_str = nullptr;
    int32_t *d_doc_cli = nullptr;
    std::vector<uint8_t *> d_final(b->launches.size(), nullptr);
    hipEvent_t e0 = nullptr, e1 = nullptr, e_fork = nullptr, e_join[3] = {nullptr, nullptr, nullptr};
    int rc = MT_OK;
    auto fail = [&](int code) {
        rc = code;
        return code;
    };
    auto up = [&](auto **dp, const auto &v) -> bool {
        if (dalloc(dp, v.size()) != hipSuccess) return false;
        return hipMemcpyAsync(*dp, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice, s) == hipSuccess;
    };
    do {
        if (!up(&d_strs, strs) || !up(&d_key_str, key_str) || !up(&d_key_rank, key_rank) || !up(&d_val_str, val_str) ||
            !up(&d_cli_str, cli_str) || (!doc_cli.empty() && !up(&d_doc_cli, doc_cli))) {
            fail(MT_ERR_HIP);
            break;
        }
        if ((!b->d_snap_meta && dalloc(&b->d_snap_meta, (size_t)b->n_docs * mt::kSnapMeta) != hipSuccess) ||
            (!b->d_snap_bytes && dalloc(&b->d_snap_bytes, (size_t)b->n_docs) != hipSuccess) ||
            (!b->d_snap_off && dalloc(&b->d_snap_off, (size_t)b->n_docs + 1) != hipSuccess) ||
            hipMemsetAsync(b->d_snap_bytes, 0xFF, 8 * (size_t)b->n_docs, s) != hipSuccess) {
            fail(MT_ERR_HIP);
            break;
        }
        for (size_t li = 0; li < b->launches.size() && !rc; li++) {
            const Launch &L = b->launches[li];
            const int64_t n = launch_n(b->n_docs, L);
            std::vector<uint8_t> fm((size_t)n);
            for (int64_t i = 0; i < n; i++) fm[i] = b->where[L.docs.empty() ? i : L.docs[i]].launch == (int32_t)li;
            if (!up(&d_final[li], fm)) fail(MT_ERR_HIP);
        }
        if (rc) break;
        // per launch: rec_bytes and seg_frame rows (out_cap entries per document; 3 words per entry)
        std::vector<size_t> scr_off(b->launches.size() + 1, 0);
        for (size_t li = 0; li < b->launches.size(); li++)
            scr_off[li + 1] = scr_off[li] + 3 * (size_t)launch_n(b->n_docs, b->launches[li]) *
                                                (size_t)std::max<int32_t>(0, b->launches[li].out_cap);
        if (scr_off.back() > b->snap_scratch_cap) {
            (void)hipFree(b->d_snap_scratch);
            b->d_snap_scratch = nullptr;
            b->snap_scratch_cap = 0;
            if (dalloc(&b->d_snap_scratch, scr_off.back()) != hipSuccess) {
                fail(MT_ERR_HIP);
                break;
            }
            b->snap_scratch_cap = scr_off.back();
        }
        // chunks beyond the meta row: a document's chunks hold at most its table's code units and
        // markers (text_top + n_out) at chunk_size each, plus the last; a document that still runs
        // out (it cannot) goes to the host serializer
        b->h_chunk_ext_off.assign((size_t)b->n_docs + 1, 0);
        const int64_t cs = std::max<int64_t>(1, b->opt.chunk_size);
        for (int64_t d = 0; d < b->n_docs; d++) {
            const mt::DocOut &o = b->docout[d];
            const int64_t bound = ((int64_t)std::max<int64_t>(0, (int64_t)o.text_top) + std::max<int64_t>(0, (int64_t)o.n_out)) / cs + 2;
            b->h_chunk_ext_off[d + 1] = b->h_chunk_ext_off[d] + 3 * std::max<int64_t>(0, bound - mt::kSnapMaxChunks);
        }
        const size_t ext_words = (size_t)b->h_chunk_ext_off.back();
        if (ext_words > b->chunk_ext_cap) {
            (void)hipFree(b->d_chunk_ext);
            b->d_chunk_ext = nullptr;
            b->chunk_ext_cap = 0;
            if (dalloc(&b->d_chunk_ext, ext_words) != hipSuccess) {
                fail(MT_ERR_HIP);
                break;
            }
            b->chunk_ext_cap = ext_words;
        }
        if ((size_t)b->n_docs + 1 > b->chunk_ext_off_n) {
            (void)hipFree(b->d_chunk_ext_off);
            b->d_chunk_ext_off = nullptr;
            b->chunk_ext_off_n = 0;
            if (dalloc(&b->d_chunk_ext_off, (size_t)b->n_docs + 1) != hipSuccess) {
                fail(MT_ERR_HIP);
                break;
            }
            b->chunk_ext_off_n = (size_t)b->n_docs + 1;
        }
        if (hipMemcpyAsync(b->d_chunk_ext_off, b->h_chunk_ext_off.data(), 8 * b->h_chunk_ext_off.size(),
                           hipMemcpyHostToDevice, s) != hipSuccess) {
            fail(MT_ERR_HIP);
            break;
        }
        if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess ||
            hipEventCreateWithFlags(&e_fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e_join[0], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e_join[1], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e_join[2], hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(e0, s) != hipSuccess) {
            fail(MT_ERR_HIP);
            break;
        }
        for (int pass = 0; pass < 2 && !rc; pass++) {
            if (pass == 1) {
                // per-document offsets of the blobs
                b->h_snap_bytes.resize((size_t)b->n_docs);
                if (hipMemcpyAsync(b->h_snap_bytes.data(), b->d_snap_bytes, 8 * (size_t)b->n_docs,
                                   hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipStreamSynchronize(s) != hipSuccess) {
                    fail(MT_ERR_HIP);
                    break;
                }
                b->h_snap_off.assign((size_t)b->n_docs + 1, 0);
                for (int64_t d = 0; d < b->n_docs; d++)
                    b->h_snap_off[d + 1] = b->h_snap_off[d] + std::max<int64_t>(0, b->h_snap_bytes[d]);
                const size_t need = (size_t)std::max<int64_t>(1, b->h_snap_off.back());
                if (need > b->snap_cap) {
                    (void)hipFree(b->d_snap);
                    b->d_snap = nullptr;
                    b->snap_cap = 0;
                    // +64: mt_bytes_digest_kernel reads up to 8 bytes past the last range
                    if (dalloc(&b->d_snap, need + need / 8 + 64) != hipSuccess) {
                        fail(MT_ERR_HIP);
                        break;
                    }
                    b->snap_cap = need + need / 8;
                }
                if (hipMemcpyAsync(b->d_snap_off, b->h_snap_off.data(), 8 * b->h_snap_off.size(),
                                   hipMemcpyHostToDevice, s) != hipSuccess) {
                    fail(MT_ERR_HIP);
                    break;
                }
            }
            // every launch's documents on a stream of their own (the escalated launches hold a few
            // large documents each, whose serial walks otherwise follow the main launch)
            if (hipEventRecord(e_fork, s) != hipSuccess) {
                fail(MT_ERR_HIP);
                break;
            }
            int n_aux = 0;
            // the escalated launches first: their large documents' walks are the longest
            for (size_t lo = 1; lo <= b->launches.size(); lo++) {
                const size_t li = lo % b->launches.size();
                const Launch &L = b->launches[li];
                hipStream_t ls = s;
                if (li > 0 && launch_n(b->n_docs, L) > 0) {
                    hipStream_t &a = b->aux[n_aux++ % 3];
                    if ((!a && hipStreamCreateWithFlags(&a, hipStreamNonBlocking) != hipSuccess) ||
                        hipStreamWaitEvent(a, e_fork, 0) != hipSuccess) {
                        fail(MT_ERR_HIP);
                        break;
                    }
                    ls = a;
                }
                mt::SnapParams P{};
                P.out = L.d_out;
                P.doc_out = L.d_docout;
                P.doc_list = L.d_list;
                P.n = launch_n(b->n_docs, L);
                if (P.n == 0) continue;
                P.out_cap = L.out_cap;
                P.text = b->d_text;
                P.doc_text_base = b->d_text_base;
                P.pool = b->d_pool;
                P.doc_pool_base = b->d_pool_base;
                P.strs = d_strs;
                P.key_str = d_key_str;
                P.key_rank = d_key_rank;
                P.val_str = d_val_str;
                P.cli_str = d_cli_str;
                P.doc_cli = d_doc_cli;
                P.cli_first = cli_first;
                P.cli_n = cli_n;
                P.final_mask = d_final[li];
                P.n_keys = (int32_t)b->keys.size();
                P.n_values = (int32_t)b->values.size();
                P.value_flags = b->d_vflags;
                P.value_class = b->d_vclass;
                P.exc = b->d_vexc;
                P.n_exc = (uint32_t)b->value_exc.size();
                P.chunk_size = b->opt.chunk_size;
                P.pass = pass;
                P.meta = b->d_snap_meta;
                P.bytes = b->d_snap_bytes;
                P.dst = b->d_snap;
                P.dst_off = b->d_snap_off;
                // MT_SNAP_RESIZE=1: the writing kernel sizes again (A/B)
                static const bool resize = getenv("MT_SNAP_RESIZE") && atoi(getenv("MT_SNAP_RESIZE")) > 0;
                if (ext_words) {
                    P.chunk_ext = b->d_chunk_ext;
                    P.chunk_ext_off = b->d_chunk_ext_off;
                }
                if (!resize && b->d_snap_scratch) {
                    P.rec_bytes = b->d_snap_scratch + scr_off[li];
                    P.seg_frame = P.rec_bytes + (size_t)P.n * (size_t)P.out_cap;
                }
                void *args[] = {&P};
                // the lane-parallel serializer (a sizing and a writing kernel); MT_SNAP_SERIAL=1: the
                // record-at-a-time walker, both passes in one kernel
                static const bool serial = getenv("MT_SNAP_SERIAL") && atoi(getenv("MT_SNAP_SERIAL")) > 0;
                const void *kfn = serial ? (const void *)mt_snapshot_serial_kernel
                                 : pass ? (const void *)mt_snapshot_kernel : (const void *)mt_snapshot_size_kernel;
                if (hipLaunchKernel(kfn, dim3((unsigned)P.n), dim3(64), args, 0, ls) != hipSuccess) {
                    fail(MT_ERR_HIP);
                    break;
                }
            }
            // join: the caller's stream waits for the aux streams
            for (int k = 0; k < std::min(n_aux, 3) && !rc; k++)
                if (hipEventRecord(e_join[k], b->aux[k]) != hipSuccess || hipStreamWaitEvent(s, e_join[k], 0) != hipSuccess)
                    fail(MT_ERR_HIP);
        }
        if (rc) break;
        float ms = 0;
        if (hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
            hipEventElapsedTime(&ms, e0, e1) != hipSuccess) {
            fail(MT_ERR_HIP);
            break;
        }
        if (device_ms) *device_ms = ms;
        if (total_bytes) *total_bytes = b->h_snap_off.back();
        b->snap_ready = true;
    } while (0);
    (void)hipStreamSynchronize(s);
    (void)hipFree(d_strs);
    (void)hipFree(d_key_str);
    (void)hipFree(d_key_rank);
    (void)hipFree(d_val_str);
    (void)hipFree(d_cli_str);
    (void)hipFree(d_doc_cli);
    for (uint8_t *p : d_final) (void)hipFree(p);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (e_fork) (void)hipEventDestroy(e_fork);
    for (hipEvent_t e : e_join)
        if (e) (void)hipEventDestroy(e);
    return rc;
}

MT_API int mt_doc_snapshot_v1_device(mt_batch *b, int64_t doc, int32_t *n_blobs) {
    if (!b) return MT_ERR_ARG;
    if (!b->snap_ready) return MT_ERR_STATE;
    if (doc < 0 || doc >= b->n_docs) return MT_ERR_ARG;
    // documents beyond MT_SNAP_MAX_BLOBS blobs are serialized by the host path above
    if (b->h_snap_bytes[doc] < 0) return mt_doc_snapshot_v1(b, doc, n_blobs);
    std::vector<int32_t> meta(mt::kSnapMeta);
    HIPCHK(hipMemcpy(meta.data(), b->d_snap_meta + doc * (int64_t)mt::kSnapMeta, 4 * meta.size(), hipMemcpyDeviceToHost));
    if (meta[0] > mt::kSnapMaxChunks) {  // the chunks beyond the row
        const int64_t e0 = b->h_chunk_ext_off[doc], n_ext = 3 * (int64_t)(meta[0] - mt::kSnapMaxChunks);
        if (n_ext > b->h_chunk_ext_off[doc + 1] - e0) return MT_INTERNAL;
        meta.resize((size_t)(mt::kSnapMeta + n_ext));
        HIPCHK(hipMemcpy(meta.data() + mt::kSnapMeta, b->d_chunk_ext + e0, 4 * (size_t)n_ext, hipMemcpyDeviceToHost));
    }
    std::string all((size_t)b->h_snap_bytes[doc], '\0');
    if (!all.empty())
        HIPCHK(hipMemcpy(&all[0], b->d_snap + b->h_snap_off[doc], all.size(), hipMemcpyDeviceToHost));
    b->c_blob_names.clear();
    b->c_blobs.clear();
    size_t at = 0;
    for (int32_t c = 0; c < meta[0]; c++) {
        const size_t n = (size_t)meta[3 + 3 * c];
        if (at + n > all.size()) return MT_INTERNAL;
        b->c_blob_names.push_back(c == 0 ? std::string("header") : "body_" + std::to_string(c - 1));
        b->c_blobs.push_back(all.substr(at, n));
        at += n;
    }
    if (at != all.size()) return MT_INTERNAL;
    b->c_blob_doc = doc;
    if (n_blobs) *n_blobs = meta[0];
    return MT_OK;
}

MT_API int mt_batch_snapshot_index(mt_batch *b, int64_t *doc_off, int32_t *blob_meta) {
    if (!b) return MT_ERR_ARG;
    if (!b->snap_ready) return MT_ERR_STATE;
    if (doc_off) memcpy(doc_off, b->h_snap_off.data(), 8 * b->h_snap_off.size());
    if (blob_meta)
        HIPCHK(hipMemcpy(blob_meta, b->d_snap_meta, 4 * (size_t)b->n_docs * mt::kSnapMeta, hipMemcpyDeviceToHost));
    return MT_OK;
}

MT_API int mt_batch_snapshot_digests(mt_batch *b, uint64_t *dst, int32_t dst_is_device) {
    if (!b || !dst) return MT_ERR_ARG;
    if (!b->snap_ready) return MT_ERR_STATE;
    hipStream_t s = b->run_stream ? b->run_stream : b->stream;
    if (!b->d_digest) HIPCHK(dalloc(&b->d_digest, (size_t)b->n_docs));
    // d_snap_off holds the per-document starts, d_snap_bytes the sizes (-1: host serializer)
    HIPCHK(hipMemcpyAsync(b->d_snap_off, b->h_snap_off.data(), 8 * b->h_snap_off.size(), hipMemcpyHostToDevice, s));
    void *args[] = {&b->d_snap, &b->d_snap_off, &b->d_snap_bytes, &b->n_docs, &b->d_digest};
    HIPCHK(hipLaunchKernel((const void *)mt_bytes_digest_kernel, dim3((unsigned)b->n_docs), dim3(64), args, 0, s));
    HIPCHK(hipMemcpyAsync(dst, b->d_digest, 8 * (size_t)b->n_docs,
                          dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return MT_OK;
}

MT_API int mt_batch_snapshot_copy(mt_batch *b, void *dst, int32_t dst_is_device) {
    if (!b || !dst) return MT_ERR_ARG;
    if (!b->snap_ready) return MT_ERR_STATE;
    if (b->h_snap_off.back())
        HIPCHK(hipMemcpy(dst, b->d_snap, (size_t)b->h_snap_off.back(),
                         dst_is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost));
    return MT_OK;
}

MT_API int mt_doc_shape(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len) {
    if (!b) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    std::string o = "D" + std::to_string(b->c_out.depth) + ":";
    int cnt = 0;
    bool first = true;
    for (const OutRec &r : b->c_recs) {
        if (rec_is_marker(r)) {
            if (!first) o.push_back(',');
            first = false;
            o += std::to_string(cnt);
            cnt = 0;
        } else {
            cnt++;
        }
    }
    return out_str(o, buf, cap, len);
}

// DESIGN.md "State digest" (same definition as the test oracle's mto_state_digest)
MT_API int mt_doc_digest(mt_batch *b, int64_t doc, uint64_t *out) {
    if (!b || !out) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    Fnv f;
    std::string tmp;
    f.u32((uint32_t)b->c_out.depth);
    size_t i = 0, n = b->c_recs.size();
    while (i < n) {
        size_t j = i;
        while (j < n && !rec_is_marker(b->c_recs[j])) j++;
        f.u32(0xB10CB10Cu);
        f.u32((uint32_t)(j - i));
        for (size_t k = i; k < j; k++) {
            const OutRec &r = b->c_recs[k];
            bool text = rec_is_text(r), removed = rec_removed(r);
            uint64_t ovl = 0;
            for (uint32_t c : ovl_clients(b, r.ovl)) ovl += fnv_name(client_name(b, doc, c, tmp));
            f.u32(text ? 0u : 1u);
            f.u32(r.len);
            f.u32((uint32_t)r.seq);
            f.u64(fnv_name(client_name(b, doc, mt::meta_cli(r.meta), tmp)));
            f.u32(removed ? (uint32_t)r.rseq : 0xFFFFFFFFu);
            f.u64(removed ? fnv_name(client_name(b, doc, mt::meta_rcli(r.meta), tmp)) : 0ull);
            f.u64(ovl);
            if (!r.props) {
                f.u32(0xFFFFFFFFu);
            } else {
                std::string pj;
                props_json(b, r.props, pj);
                f.u32((uint32_t)pj.size());
                f.bytes(pj.data(), pj.size());
            }
            if (text) {
                for (uint32_t q = 0; q < r.len; q++) {
                    uint16_t c = b->c_text[r.toff + q];
                    unsigned char b2[2] = {(unsigned char)c, (unsigned char)(c >> 8)};
                    f.bytes(b2, 2);
                }
            } else {
                f.u32(r.toff);
            }
        }
        i = j + 1;
    }
    f.u32((uint32_t)b->c_out.min_seq);
    f.u32((uint32_t)b->c_out.cur_seq);
    f.u32((uint32_t)b->c_out.status);
    *out = f.h;
    return MT_OK;
}

// debugging aid: one line per oe entry (segment fields or end-of-block marker)
MT_API int mt_doc_dump(mt_batch *b, int64_t doc, char *buf, int64_t cap, int64_t *len) {
    if (!b) return MT_ERR_ARG;
    int rc = load_doc(b, doc);
    if (rc) return rc;
    std::string o = "status=" + std::to_string(b->c_out.status) + " min=" + std::to_string(b->c_out.min_seq) +
                    " cur=" + std::to_string(b->c_out.cur_seq) + " depth=" + std::to_string(b->c_out.depth) +
                    " ops_done=" + std::to_string(b->c_out.ops_done) + " fail_op=" + std::to_string(b->c_out.fail_op) +
                    " cap_kind=" + std::to_string(b->c_out.cap_kind) + "\n";
    std::string tmp;
    for (const OutRec &r : b->c_recs) {
        if (rec_is_marker(r)) {
            o += "  M blk=" + std::to_string(r.blk & ~mt::kOutBlockEnd) + "\n";
            continue;
        }
        o += "  S blk=" + std::to_string(r.blk) + " len=" + std::to_string(r.len) + " seq=" + std::to_string(r.seq) +
             " cli=" + client_name(b, doc, mt::meta_cli(r.meta), tmp) +
             " rseq=" + std::to_string(rec_removed(r) ? r.rseq : -1) + " rcli=" +
             (rec_removed(r) ? client_name(b, doc, mt::meta_rcli(r.meta), tmp) : std::string("-")) +
             " ovl=" + std::to_string(r.ovl) + " '";
        if (rec_is_text(r)) utf16_to_utf8(o, b->c_text.data() + r.toff, r.len);
        o += "'";
        if (r.props) {
            o += " ";
            props_json(b, r.props, o);
        }
        o += "\n";
    }
    return out_str(o, buf, cap, len);
}

// ---------------------------------------------------------------- logs
// prop records referenced by the ops of documents [d0, d1): [0, end)
static int64_t props_end(mt_batch *b, int64_t d0, int64_t d1, const mt_op *ops) {
    if (d0 == 0 && d1 == b->n_docs) return b->total_props;
    int64_t end = 0;
    const int64_t base = b->h_off[d0];
    for (int64_t i = b->h_off[d0]; i < b->h_off[d1]; i++) {
        const mt_op &o = ops[i - base];
        if (o.type == MT_OP_ANNOTATE) end = std::max<int64_t>(end, (int64_t)o.payload + o.payload_len);
        if (MT_OP_IS_INSERT_LIKE(o.type) && (MT_OPF_BITS(o.flags) & MT_OPF_HAS_PROPS)) {
            // an extended insert's count is in its first record (device memory): take everything
            if (MT_OPF_NPROPS(o.flags) == MT_OPF_NPROPS_EXT) return b->total_props;
            end = std::max<int64_t>(end, (int64_t)o.pos2 + MT_OPF_NPROPS(o.flags));
        }
    }
    return std::min(end, b->total_props);
}

static int download_ops(mt_batch *b, int64_t d0, int64_t d1, std::vector<mt_op> &ops) {
    ops.resize((size_t)(b->h_off[d1] - b->h_off[d0]));
    if (!ops.empty())
        HIPCHK(hipMemcpy(ops.data(), b->d_ops + b->h_off[d0], sizeof(mt_op) * ops.size(), hipMemcpyDeviceToHost));
    return MT_OK;
}

MT_API int mt_batch_log_sizes_docs(mt_batch *b, int64_t d0, int64_t d1, int64_t *n_ops, int64_t *n_text,
                                   int64_t *n_props) {
    if (!b || !b->have_log) return MT_ERR_STATE;
    if (d0 < 0 || d1 < d0 || d1 > b->n_docs) return MT_ERR_ARG;
    if (n_ops) *n_ops = b->h_off[d1] - b->h_off[d0];
    if (n_text) {
        int64_t t = 0;
        for (int64_t d = d0; d < d1; d++) t += b->h_text_len[d];
        *n_text = t;
    }
    if (n_props) {
        std::vector<mt_op> ops;
        if (!(d0 == 0 && d1 == b->n_docs)) {
            int rc = download_ops(b, d0, d1, ops);
            if (rc) return rc;
        }
        *n_props = props_end(b, d0, d1, ops.data());
    }
    return MT_OK;
}

// documents [d0, d1) as a standalone log: offsets from 0, the text of doc d follows doc d-1's,
// prop offsets unchanged (records [0, n_props) of the batch, n_props from the sizes call)
MT_API int mt_batch_download_log_docs(mt_batch *b, int64_t d0, int64_t d1, mt_op *ops, int64_t *doc_op_off,
                                      uint16_t *text, mt_prop *props) {
    if (!b || !b->have_log) return MT_ERR_STATE;
    if (d0 < 0 || d1 < d0 || d1 > b->n_docs) return MT_ERR_ARG;
    std::vector<mt_op> h;
    int rc = download_ops(b, d0, d1, h);
    if (rc) return rc;
    const int64_t base = b->h_off[d0];
    if (ops) {
        int64_t tb = 0;
        for (int64_t d = d0; d < d1; d++) {
            for (int64_t i = b->h_off[d]; i < b->h_off[d + 1]; i++) {
                mt_op &o = h[(size_t)(i - base)];
                o.flags &= (uint16_t)~MT_OPF_INTERNAL;
                if (o.type == MT_OP_RELPOS) {  // keys back to value ids (kIdKeyUnsupported: re-derived at ingest)
                    auto val = [&](int32_t k) {
                        return (uint32_t)k < b->key_value.size() ? (int32_t)b->key_value[(uint32_t)k] : 0;
                    };
                    o.pos1 = val(o.pos1);
                    o.pos2 = val(o.pos2);
                }
                if (MT_OP_IS_INSERT_LIKE(o.type) && !(MT_OPF_BITS(o.flags) & MT_OPF_MARKER)) o.payload += (uint32_t)tb;
            }
            tb += b->h_text_len[d];
        }
        if (!h.empty()) memcpy(ops, h.data(), sizeof(mt_op) * h.size());
    }
    if (doc_op_off)
        for (int64_t d = d0; d <= d1; d++) doc_op_off[d - d0] = b->h_off[d] - base;
    if (text) {
        int64_t tb = 0;
        for (int64_t d = d0; d < d1; d++) {
            if (b->h_text_len[d])
                HIPCHK(hipMemcpy(text + tb, b->d_text + b->h_text_base[d], 2ull * b->h_text_len[d], hipMemcpyDeviceToHost));
            tb += b->h_text_len[d];
        }
    }
    const int64_t np = props_end(b, d0, d1, h.data());
    if (props && np > 0) HIPCHK(hipMemcpy(props, b->d_props, sizeof(mt_prop) * (size_t)np, hipMemcpyDeviceToHost));
    return MT_OK;
}

MT_API int mt_batch_log_sizes(mt_batch *b, int64_t *n_ops, int64_t *n_text, int64_t *n_props) {
    if (!b || !b->have_log) return MT_ERR_STATE;
    return mt_batch_log_sizes_docs(b, 0, b->n_docs, n_ops, n_text, n_props);
}

MT_API int mt_batch_download_log(mt_batch *b, mt_op *ops, int64_t *doc_op_off, uint16_t *text, mt_prop *props) {
    if (!b || !b->have_log) return MT_ERR_STATE;
    return mt_batch_download_log_docs(b, 0, b->n_docs, ops, doc_op_off, text, props);
}

// ---------------------------------------------------------------- generator
static const char *GEN_KEYS[MT_GEN_N_KEYS] = {"bold", "italic", "color", "size"};
static const char *GEN_CLIENTS[] = {"readonly", "A", "B", "C", "D", "E", "F", "G", "H", "I", "J", "K", "L", "M",
                                    "N", "O", "P", "Q", "R", "S", "T", "U", "V", "W", "X", "Y", "Z"};

// generation of D documents: document d has global index doc_ids[d] (its stream's seed) and
// doc_ops[d] ops; logs are laid out back to back (doc_op_off = prefix sums of doc_ops)
static int generate_docs(mt_batch *b, const mt_gen_params *p, const std::vector<int64_t> &doc_ids,
                         const std::vector<int32_t> &doc_ops) {
    if (!b || !p || p->n_clients < 1 || p->n_clients > 26 || p->max_insert < 1) return MT_ERR_ARG;
    // fixed generator tables (include/mt_gen.h)
    std::vector<std::string> vals = {"null", "true", "\"red\"", "\"green\"", "\"blue\""};
    for (int s = 8; s <= 24; s++) vals.push_back(std::to_string(s));
    std::vector<const char *> vp, kp(GEN_KEYS, GEN_KEYS + MT_GEN_N_KEYS);
    for (auto &v : vals) vp.push_back(v.c_str());
    int rc = mt_batch_set_tables(b, kp.data(), MT_GEN_N_KEYS, vp.data(), (int32_t)vp.size());
    if (rc) return rc;
    rc = mt_batch_set_clients(b, -1, GEN_CLIENTS, p->n_clients + 1);
    if (rc) return rc;
    const int64_t D = b->n_docs;
    if ((int64_t)doc_ids.size() != D || (int64_t)doc_ops.size() != D) return MT_ERR_ARG;
    free_launches(b);
    free_log(b);
    b->h_off.resize(D + 1);
    b->h_off[0] = 0;
    b->h_nload.assign(D, 0);
    b->h_nload_segs.assign(D, 0);
    b->h_tile_annot.assign(D, 0);
    b->lab_track = false;
    int32_t max_ops = 0;
    for (int64_t d = 0; d < D; d++) {
        if (doc_ops[d] < 1) return MT_ERR_ARG;
        b->h_off[d + 1] = b->h_off[d] + doc_ops[d];
        max_ops = std::max(max_ops, doc_ops[d]);
    }
    const int64_t N = b->h_off[D];
    b->h_text_base.assign(D, 0);
    b->h_text_len.assign(D, 0);
    b->h_text_cap.assign(D, 0);
    b->h_pool_base.assign(D, 0);
    b->h_pool_cap.assign(D, 0);
    uint64_t tbase = 0, pbase = 0;
    const int32_t pct_ann = std::max(0, 100 - p->pct_insert - p->pct_remove);
    for (int64_t d = 0; d < D; d++) {
        const uint64_t pay_cap = (uint64_t)doc_ops[d] * (uint64_t)p->max_insert;
        const uint64_t cap = align16u(pay_cap) + (uint64_t)b->opt.arena_factor * pay_cap / 2 + 4096;
        const int64_t ann = (int64_t)doc_ops[d] * pct_ann / 100;
        const uint64_t pc = 1024 + (uint64_t)b->opt.pool_per_op * (uint64_t)(ann + ann / 2 + 16);
        if (cap > 0xFFFFFFF0ull || pc > 0xFFFFFFF0ull) return MT_ERR_ARG;
        b->h_text_base[d] = tbase;
        b->h_text_len[d] = (uint32_t)pay_cap;  // payload capacity: the arena starts after it
        b->h_text_cap[d] = (uint32_t)cap;
        b->h_pool_base[d] = pbase;
        b->h_pool_cap[d] = (uint32_t)pc;
        tbase += align16u(cap);
        pbase += align16u(pc);
    }
    b->text_words = tbase;
    b->pool_words = pbase;
    b->total_ops = N;
    b->total_props = 2 * N;
    b->max_ops_per_doc = max_ops;
    int rc2 = ensure_tables(b);
    if (rc2) return rc2;
    HIPCHK(dalloc(&b->d_ops, (size_t)N));
    HIPCHK(dalloc(&b->d_off, (size_t)D + 1));
    HIPCHK(dalloc(&b->d_text, (size_t)b->text_words));
    HIPCHK(dalloc(&b->d_text_base, (size_t)D));
    HIPCHK(dalloc(&b->d_text_len, (size_t)D));
    HIPCHK(dalloc(&b->d_text_cap, (size_t)D));
    HIPCHK(dalloc(&b->d_pool, (size_t)b->pool_words));
    HIPCHK(dalloc(&b->d_pool_base, (size_t)D));
    HIPCHK(dalloc(&b->d_pool_cap, (size_t)D));
    HIPCHK(dalloc(&b->d_props, (size_t)(2 * N)));
    HIPCHK(hipMemcpy(b->d_off, b->h_off.data(), 8 * (size_t)(D + 1), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text_base, b->h_text_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text_len, b->h_text_len.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_text_cap, b->h_text_cap.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_pool_base, b->h_pool_base.data(), 8 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(b->d_pool_cap, b->h_pool_cap.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    int64_t *d_ids = nullptr;
    int32_t *d_nops = nullptr;
    HIPCHK(dalloc(&d_ids, (size_t)D));
    HIPCHK(dalloc(&d_nops, (size_t)D));
    HIPCHK(hipMemcpy(d_ids, doc_ids.data(), 8 * (size_t)D, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_nops, doc_ops.data(), 4 * (size_t)D, hipMemcpyHostToDevice));
    mt_gen_params *d_gen = nullptr;
    HIPCHK(dalloc(&d_gen, 1));
    HIPCHK(hipMemcpy(d_gen, p, sizeof(mt_gen_params), hipMemcpyHostToDevice));
    // generation runs in each document's initial replay class; documents that overflow it are
    // generated again (deterministically, from their own seed) in the next larger class
    std::vector<DocOut> outs((size_t)D);
    std::map<int, std::vector<int32_t>> work;  // class -> documents
    for (int64_t d = 0; d < D; d++) {
        int c = std::min(class_for(b, doc_ops[d], 0, false), mt::kNumClasses - 1);
        while (c > 0 && !class_usable(c)) c--;
        work[c].push_back((int32_t)d);
    }
    while (!work.empty()) {
        const int cls = work.begin()->first;
        std::vector<int32_t> todo = std::move(work.begin()->second);
        work.erase(work.begin());
        const bool all = (int64_t)todo.size() == D;
        for (size_t at = 0; at < todo.size();) {
            // the HBM class holds ~220 MB per document: bounded launches
            const size_t n = std::min(todo.size() - at, launch_chunk(cls, todo.size() - at));
            Launch L;
            L.cls = cls;
            L.caps = mt::class_caps(mt::kClassSegs[cls]);
            L.out_cap = L.caps.oe;
            L.lds = class_lds(cls);
            HIPCHK(dalloc(&L.d_out, n * (size_t)L.out_cap));
            HIPCHK(dalloc(&L.d_docout, n));
            HIPCHK(dalloc(&L.d_cold, n * (size_t)L.caps.seg * mt::kColdPerSlot));
            if (class_state_bytes(cls)) HIPCHK(dalloc(&L.d_state, n * class_state_bytes(cls)));
            if (!all) {
                HIPCHK(dalloc(&L.d_list, n));
                HIPCHK(hipMemcpy(L.d_list, todo.data() + at, 4 * n, hipMemcpyHostToDevice));
            }
            mt::ReplayParams P = base_params(b);
            P.out = L.d_out;
            P.doc_out = L.d_docout;
            P.n_docs = (int64_t)n;
            P.doc_first = 0;
            P.doc_list = L.d_list;
            P.out_cap = L.out_cap;
            P.gen = d_gen;
            P.gen_ops = b->d_ops;
            P.gen_props = b->d_props;
            P.gen_doc_ids = d_ids;
            P.gen_doc_ops = d_nops;
            P.cold = L.d_cold;
            P.hbm_state = L.d_state;
            const void *fn = kKernels[cls].generate;
            if (L.lds > 64 * 1024)
                HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds));
            void *args[] = {&P};
            HIPCHK(hipLaunchKernel(fn, dim3((unsigned)n), dim3(64), args, L.lds, b->stream));
            HIPCHK(hipStreamSynchronize(b->stream));
            std::vector<DocOut> part(n);
            HIPCHK(hipMemcpy(part.data(), L.d_docout, sizeof(DocOut) * n, hipMemcpyDeviceToHost));
            (void)hipFree(L.d_out);
            (void)hipFree(L.d_docout);
            (void)hipFree(L.d_list);
            (void)hipFree(L.d_cold);
            (void)hipFree(L.d_state);
            for (size_t i = 0; i < n; i++) {
                const int32_t d = todo[at + i];
                outs[(size_t)d] = part[i];
                if (part[i].status == MT_CAPACITY && part[i].cap_kind == 1 && class_usable(cls + 1))
                    work[cls + 1].push_back(d);
                else if (part[i].status == MT_CAPACITY && part[i].cap_kind == mt::kCapLongSeg && long_seg_class(cls) < mt::kNumClasses)
                    work[long_seg_class(cls)].push_back(d);
            }
            at += n;
        }
    }
    (void)hipFree(d_gen);
    (void)hipFree(d_ids);
    (void)hipFree(d_nops);
    b->payload_units = 0;
    b->prop_records = 0;
    int bad = 0;
    for (int64_t d = 0; d < D; d++) {
        if (outs[d].status != MT_OK) bad++;
        b->payload_units += outs[d].gen_text;
        b->prop_records += outs[d].gen_props;
    }
    b->have_log = true;
    b->generated = true;
    b->ran = false;
    if (bad) {
        fprintf(stderr, "mtreplay: generator: %d documents failed (first status %d)\n", bad, outs[0].status);
        return MT_INTERNAL;
    }
    return MT_OK;
}

MT_API int mt_batch_generate(mt_batch *b, const mt_gen_params *p, int64_t doc_first) {
    if (!b || !p || p->n_ops < 1) return MT_ERR_ARG;
    std::vector<int64_t> ids((size_t)b->n_docs);
    for (int64_t d = 0; d < b->n_docs; d++) ids[(size_t)d] = doc_first + d;
    return generate_docs(b, p, ids, std::vector<int32_t>((size_t)b->n_docs, p->n_ops));
}

MT_API int mt_batch_generate_docs(mt_batch *b, const mt_gen_params *p, const int64_t *doc_ids,
                                  const int32_t *doc_ops) {
    if (!b || !p || !doc_ids || !doc_ops) return MT_ERR_ARG;
    return generate_docs(b, p, std::vector<int64_t>(doc_ids, doc_ids + b->n_docs),
                         std::vector<int32_t>(doc_ops, doc_ops + b->n_docs));
}

}  // extern "C"
