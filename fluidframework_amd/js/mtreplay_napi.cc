// mtreplay_napi.cc — thin N-API addon over the C ABI of libmtreplay.so (include/mtreplay.h).
//
// This is the binding a FluidFramework maintainer would add to drive the GPU replay from the
// reference's own runtime (Node): every function marshals JS values to plain pointers and
// sizes and calls one mt_* entry point; no replay logic lives here.  `runAsync` runs
// mt_batch_run on a libuv worker (napi_create_async_work), so the event loop stays responsive
// while the GPU replays (SURVEY.md §8b "Threading").
#include <node_api.h>

#include <string>
#include <vector>

#include "../../include/mtreplay.h"

namespace {

#define NAPI_OK(call)                                                   \
    do {                                                                \
        if ((call) != napi_ok) {                                        \
            napi_throw_error(env, nullptr, "N-API call failed: " #call); \
            return nullptr;                                             \
        }                                                               \
    } while (0)

napi_value throw_mt(napi_env env, int rc, const char *what) {
    std::string msg = std::string(what) + ": " + mt_status_string(rc);
    napi_value err, code, m;
    napi_create_string_utf8(env, msg.c_str(), msg.size(), &m);
    napi_create_error(env, nullptr, m, &err);
    napi_create_int32(env, rc, &code);
    napi_set_named_property(env, err, "code", code);
    napi_throw(env, err);
    return nullptr;
}
#define MT_OK_OR_THROW(call, what)                 \
    do {                                           \
        int rc_ = (call);                          \
        if (rc_ != MT_OK) return throw_mt(env, rc_, what); \
    } while (0)

std::vector<napi_value> args(napi_env env, napi_callback_info info, size_t n) {
    std::vector<napi_value> a(n);
    size_t argc = n;
    napi_get_cb_info(env, info, &argc, a.data(), nullptr, nullptr);
    return a;
}

mt_batch *batch_of(napi_env env, napi_value v) {
    void *p = nullptr;
    napi_get_value_external(env, v, &p);
    return static_cast<mt_batch *>(p);
}

int64_t i64(napi_env env, napi_value v) {
    int64_t x = 0;
    napi_get_value_int64(env, v, &x);
    return x;
}

std::string str(napi_env env, napi_value v) {
    size_t n = 0;
    napi_get_value_string_utf8(env, v, nullptr, 0, &n);
    std::string s(n, '\0');
    napi_get_value_string_utf8(env, v, &s[0], n + 1, &n);
    return s;
}

std::vector<std::string> strs(napi_env env, napi_value arr) {
    uint32_t n = 0;
    napi_get_array_length(env, arr, &n);
    std::vector<std::string> out(n);
    for (uint32_t i = 0; i < n; i++) {
        napi_value e;
        napi_get_element(env, arr, i, &e);
        out[i] = str(env, e);
    }
    return out;
}

void *typed(napi_env env, napi_value v, size_t *len) {
    napi_typedarray_type t;
    void *data = nullptr;
    napi_value ab;
    size_t off = 0;
    *len = 0;
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    if (is_ta) {
        napi_get_typedarray_info(env, v, &t, len, &data, &ab, &off);
        return data;
    }
    bool is_buf = false;
    napi_is_buffer(env, v, &is_buf);
    if (is_buf) {
        napi_get_buffer_info(env, v, &data, len);
        return data;
    }
    return nullptr;
}

void finalize_batch(napi_env, void *data, void *) { mt_batch_destroy(static_cast<mt_batch *>(data)); }

// ingestJson(h, [jsonText per document], observer, nThreads, device) -> "gpu" | "host":
// device "gpu" / "auto": the GPU parser (mt_batch_ingest_json_gpu); "auto" falls back to the host
// parser (mt_pack_json on host threads + mt_batch_ingest_packed) for a batch outside its fast path
napi_value ingest_json(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 5);
    mt_batch *b = batch_of(env, a[0]);
    std::vector<std::string> docs = strs(env, a[1]);
    std::string observer = str(env, a[2]);
    int32_t threads = (int32_t)i64(env, a[3]);
    napi_valuetype t;
    napi_typeof(env, a[4], &t);
    const std::string device = t == napi_string ? str(env, a[4]) : std::string("auto");
    if (observer.empty()) observer = "readonly";
    napi_value path;
    if (device != "host") {
        std::string all;
        std::vector<int64_t> off(1, 0);
        for (const auto &d : docs) {
            all += d;
            off.push_back((int64_t)all.size());
        }
        int64_t bad = -1;
        mt_json_gpu_stats st{};
        const int rc = mt_batch_ingest_json_gpu(b, all.data(), off.data(), (int64_t)docs.size(), nullptr,
                                                observer.c_str(), &bad, &st);
        if (rc == MT_OK) {
            napi_create_string_utf8(env, "gpu", NAPI_AUTO_LENGTH, &path);
            return path;
        }
        if (rc != MT_UNSUPPORTED || device == "gpu")
            return throw_mt(env, rc, ("mt_batch_ingest_json_gpu: document " + std::to_string(bad)).c_str());
    }
    std::vector<const char *> ptrs;
    std::vector<int64_t> lens;
    for (const auto &d : docs) {
        ptrs.push_back(d.c_str());
        lens.push_back((int64_t)d.size());
    }
    mt_packed *p = nullptr;
    int64_t bad = -1;
    int rc = mt_pack_json(&p, (int64_t)docs.size(), ptrs.data(), lens.data(), observer.c_str(), threads, &bad);
    if (rc != MT_OK) {
        std::string why = p ? mt_packed_error(p) : "";
        mt_packed_destroy(p);
        return throw_mt(env, rc, ("mt_pack_json: " + why).c_str());
    }
    rc = mt_batch_ingest_packed(b, p);
    mt_packed_destroy(p);
    MT_OK_OR_THROW(rc, "mt_batch_ingest_packed");
    napi_create_string_utf8(env, "host", NAPI_AUTO_LENGTH, &path);
    return path;
}

// createBatch(nDocs, {segCap, maxRetries}) -> external handle (mt_batch_create)
napi_value create_batch(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 2);
    mt_batch_options o{};
    napi_valuetype t;
    napi_typeof(env, a[1], &t);
    if (t == napi_object) {
        napi_value v;
        bool has = false;
        if (napi_has_named_property(env, a[1], "segCap", &has) == napi_ok && has) {
            napi_get_named_property(env, a[1], "segCap", &v);
            o.seg_cap = (int32_t)i64(env, v);
        }
        if (napi_has_named_property(env, a[1], "maxRetries", &has) == napi_ok && has) {
            napi_get_named_property(env, a[1], "maxRetries", &v);
            o.max_retries = (int32_t)i64(env, v);
        }
    }
    mt_batch *b = nullptr;
    MT_OK_OR_THROW(mt_batch_create(&b, i64(env, a[0]), &o), "mt_batch_create");
    napi_value h;
    NAPI_OK(napi_create_external(env, b, finalize_batch, nullptr, &h));
    return h;
}

// setTables(h, keys[], values[]) (mt_batch_set_tables)
napi_value set_tables(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 3);
    auto keys = strs(env, a[1]), values = strs(env, a[2]);
    std::vector<const char *> kp, vp;
    for (auto &k : keys) kp.push_back(k.c_str());
    for (auto &v : values) vp.push_back(v.c_str());
    MT_OK_OR_THROW(mt_batch_set_tables(batch_of(env, a[0]), kp.data(), (int32_t)kp.size(), vp.data(), (int32_t)vp.size()),
                   "mt_batch_set_tables");
    return nullptr;
}

// setClients(h, doc, names[]) (mt_batch_set_clients; doc -1: every document)
napi_value set_clients(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 3);
    auto names = strs(env, a[2]);
    std::vector<const char *> np;
    for (auto &n : names) np.push_back(n.c_str());
    MT_OK_OR_THROW(mt_batch_set_clients(batch_of(env, a[0]), i64(env, a[1]), np.data(), (int32_t)np.size()),
                   "mt_batch_set_clients");
    return nullptr;
}

// ingest(h, ops: Buffer of 32-byte mt_op, docOpOff: BigInt64Array, text: Uint16Array,
//        props: Uint32Array of (key, value) pairs) (mt_batch_ingest)
napi_value ingest(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 5);
    size_t n_ops_b = 0, n_off = 0, n_text = 0, n_props = 0;
    const mt_op *ops = (const mt_op *)typed(env, a[1], &n_ops_b);
    const int64_t *off = (const int64_t *)typed(env, a[2], &n_off);
    const uint16_t *text = (const uint16_t *)typed(env, a[3], &n_text);
    const mt_prop *props = (const mt_prop *)typed(env, a[4], &n_props);
    if (!ops || !off) {
        napi_throw_type_error(env, nullptr, "ingest(h, opsBuffer, BigInt64Array, Uint16Array, Uint32Array)");
        return nullptr;
    }
    // the C ABI takes the op count from docOpOff: check it against the buffers first
    mt_batch_stats st{};
    if (mt_batch_get_stats(batch_of(env, a[0]), &st) != MT_OK || n_off != (size_t)st.n_docs + 1 || off[0] != 0) {
        napi_throw_range_error(env, nullptr, "ingest: docOpOff must hold nDocs + 1 offsets starting at 0");
        return nullptr;
    }
    for (size_t i = 1; i < n_off; i++)
        if (off[i] < off[i - 1]) {
            napi_throw_range_error(env, nullptr, "ingest: docOpOff must be non-decreasing");
            return nullptr;
        }
    if ((uint64_t)off[n_off - 1] > n_ops_b / sizeof(mt_op)) {
        napi_throw_range_error(env, nullptr, "ingest: docOpOff ends beyond the ops buffer");
        return nullptr;
    }
    static const uint16_t z16 = 0;
    static const mt_prop zp{0, 0};
    MT_OK_OR_THROW(mt_batch_ingest(batch_of(env, a[0]), ops, off, text ? text : &z16, (int64_t)n_text,
                                   props ? props : &zp, (int64_t)(n_props / 2)),
                   "mt_batch_ingest");
    return nullptr;
}

// generate(h, {nOps, nClients, maxLag, pctInsert, pctRemove, minLen, maxInsert, pctNewline, seed}, docFirst)
napi_value generate(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 3);
    mt_gen_params p{};
    auto get = [&](const char *k, int32_t dflt) {
        napi_value v;
        bool has = false;
        if (napi_has_named_property(env, a[1], k, &has) != napi_ok || !has) return dflt;
        napi_get_named_property(env, a[1], k, &v);
        return (int32_t)i64(env, v);
    };
    p.n_ops = get("nOps", 1000);
    p.n_clients = get("nClients", 8);
    p.max_lag = get("maxLag", 32);
    p.pct_insert = get("pctInsert", 60);
    p.pct_remove = get("pctRemove", 40);
    p.min_len = get("minLen", 4);
    p.max_insert = get("maxInsert", 8);
    p.pct_newline = get("pctNewline", 2);
    p.seed = (uint64_t)(uint32_t)get("seed", (int32_t)0xDEADBEEF);
    MT_OK_OR_THROW(mt_batch_generate(batch_of(env, a[0]), &p, i64(env, a[2])), "mt_batch_generate");
    return nullptr;
}

napi_value run(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 1);
    MT_OK_OR_THROW(mt_batch_run(batch_of(env, a[0]), nullptr), "mt_batch_run");
    return nullptr;
}

struct RunWork {
    mt_batch *b;
    int rc;
    napi_deferred deferred;
    napi_async_work work;
};

// runAsync(h) -> Promise: mt_batch_run on a libuv worker thread
napi_value run_async(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 1);
    auto *w = new RunWork{batch_of(env, a[0]), 0, nullptr, nullptr};
    napi_value promise, name;
    NAPI_OK(napi_create_promise(env, &w->deferred, &promise));
    napi_create_string_utf8(env, "mt_batch_run", NAPI_AUTO_LENGTH, &name);
    NAPI_OK(napi_create_async_work(
        env, nullptr, name, [](napi_env, void *d) { auto *w = (RunWork *)d; w->rc = mt_batch_run(w->b, nullptr); },
        [](napi_env env, napi_status, void *d) {
            auto *w = (RunWork *)d;
            if (w->rc == MT_OK) {
                napi_value u;
                napi_get_undefined(env, &u);
                napi_resolve_deferred(env, w->deferred, u);
            } else {
                napi_value m, err, code;
                std::string msg = std::string("mt_batch_run: ") + mt_status_string(w->rc);
                napi_create_string_utf8(env, msg.c_str(), msg.size(), &m);
                napi_create_error(env, nullptr, m, &err);
                napi_create_int32(env, w->rc, &code);
                napi_set_named_property(env, err, "code", code);
                napi_reject_deferred(env, w->deferred, err);
            }
            napi_delete_async_work(env, w->work);
            delete w;
        },
        w, &w->work));
    NAPI_OK(napi_queue_async_work(env, w->work));
    return promise;
}

napi_value doc_status(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 2);
    napi_value r;
    napi_create_int32(env, mt_doc_status(batch_of(env, a[0]), i64(env, a[1])), &r);
    return r;
}

// size-query then fill: the C-ABI convention for caller-owned output buffers
napi_value string_out(napi_env env, napi_callback_info info,
                      int (*fn)(mt_batch *, int64_t, char *, int64_t, int64_t *), const char *what) {
    auto a = args(env, info, 2);
    mt_batch *b = batch_of(env, a[0]);
    int64_t doc = i64(env, a[1]), n = 0;
    MT_OK_OR_THROW(fn(b, doc, nullptr, 0, &n), what);
    std::string s((size_t)n + 1, '\0');
    MT_OK_OR_THROW(fn(b, doc, &s[0], n + 1, &n), what);
    napi_value r;
    NAPI_OK(napi_create_string_utf8(env, s.data(), (size_t)n, &r));
    return r;
}
napi_value doc_text(napi_env env, napi_callback_info info) { return string_out(env, info, mt_doc_text, "mt_doc_text"); }
napi_value doc_regenerated_ops(napi_env env, napi_callback_info info) {
    return string_out(env, info, mt_doc_regenerated_ops, "mt_doc_regenerated_ops");
}
napi_value doc_consensus_events(napi_env env, napi_callback_info info) {
    return string_out(env, info, mt_doc_consensus_events, "mt_doc_consensus_events");
}
napi_value doc_props_runs(napi_env env, napi_callback_info info) {
    return string_out(env, info, mt_doc_props_runs, "mt_doc_props_runs");
}

// docSnapshotV1(h, doc) -> { [blobName]: utf-8 JSON string } (SnapshotV1.extractSync + emit)
napi_value doc_snapshot(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 2);
    mt_batch *b = batch_of(env, a[0]);
    int64_t doc = i64(env, a[1]);
    int32_t nb = 0;
    MT_OK_OR_THROW(mt_doc_snapshot_v1(b, doc, &nb), "mt_doc_snapshot_v1");
    napi_value obj;
    NAPI_OK(napi_create_object(env, &obj));
    for (int32_t i = 0; i < nb; i++) {
        char name[64];
        int64_t n = 0;
        MT_OK_OR_THROW(mt_doc_snapshot_blob(b, doc, i, name, sizeof name, nullptr, 0, &n), "mt_doc_snapshot_blob");
        std::string s((size_t)n + 1, '\0');
        MT_OK_OR_THROW(mt_doc_snapshot_blob(b, doc, i, name, sizeof name, &s[0], n + 1, &n), "mt_doc_snapshot_blob");
        napi_value v;
        NAPI_OK(napi_create_string_utf8(env, s.data(), (size_t)n, &v));
        NAPI_OK(napi_set_named_property(env, obj, name, v));
    }
    return obj;
}

// docFindTile(h, doc, startPos, label, preceding) -> { pos, props } | undefined
// (Client.findTile, client.ts:1073-1076, via mt_doc_find_tile)
napi_value doc_find_tile(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 5);
    mt_batch *b = batch_of(env, a[0]);
    const int64_t doc = i64(env, a[1]), start = i64(env, a[2]);
    const std::string label = str(env, a[3]);
    bool prec = true;
    NAPI_OK(napi_get_value_bool(env, a[4], &prec));
    int64_t pos = -1, n = 0;
    MT_OK_OR_THROW(mt_doc_find_tile(b, doc, start, label.c_str(), prec ? 1 : 0, &pos, nullptr, 0, &n), "mt_doc_find_tile");
    napi_value r;
    if (pos < 0) {
        NAPI_OK(napi_get_undefined(env, &r));
        return r;
    }
    std::string props((size_t)n + 1, '\0');
    MT_OK_OR_THROW(mt_doc_find_tile(b, doc, start, label.c_str(), prec ? 1 : 0, &pos, &props[0], n + 1, &n),
                   "mt_doc_find_tile");
    napi_value vp, vs;
    NAPI_OK(napi_create_object(env, &r));
    NAPI_OK(napi_create_int64(env, pos, &vp));
    NAPI_OK(napi_create_string_utf8(env, props.data(), (size_t)n, &vs));
    NAPI_OK(napi_set_named_property(env, r, "pos", vp));
    NAPI_OK(napi_set_named_property(env, r, "props", vs));
    return r;
}

// docStackContext(h, doc, startPos, [rangeLabels]) -> JSON text of the stacks
// (Client.getStackContext, client.ts:946-948, via mt_doc_stack_context)
napi_value doc_stack_context(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 4);
    mt_batch *b = batch_of(env, a[0]);
    const int64_t doc = i64(env, a[1]), start = i64(env, a[2]);
    const std::vector<std::string> labels = strs(env, a[3]);
    std::vector<const char *> lp;
    for (const auto &l : labels) lp.push_back(l.c_str());
    int64_t n = 0;
    MT_OK_OR_THROW(mt_doc_stack_context(b, doc, start, lp.data(), (int32_t)lp.size(), nullptr, 0, &n),
                   "mt_doc_stack_context");
    std::string out((size_t)n + 1, '\0');
    MT_OK_OR_THROW(mt_doc_stack_context(b, doc, start, lp.data(), (int32_t)lp.size(), &out[0], n + 1, &n),
                   "mt_doc_stack_context");
    napi_value r;
    NAPI_OK(napi_create_string_utf8(env, out.data(), (size_t)n, &r));
    return r;
}

napi_value doc_digest(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 2);
    uint64_t d = 0;
    MT_OK_OR_THROW(mt_doc_digest(batch_of(env, a[0]), i64(env, a[1]), &d), "mt_doc_digest");
    napi_value r;
    NAPI_OK(napi_create_bigint_uint64(env, d, &r));
    return r;
}

// deviceDigests(h, out: BigUint64Array[nDocs]) (mt_batch_device_digests into host memory)
napi_value device_digests(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 2);
    size_t n = 0;
    uint64_t *dst = (uint64_t *)typed(env, a[1], &n);
    if (!dst) {
        napi_throw_type_error(env, nullptr, "deviceDigests(h, BigUint64Array)");
        return nullptr;
    }
    MT_OK_OR_THROW(mt_batch_device_digests(batch_of(env, a[0]), dst, 0), "mt_batch_device_digests");
    return nullptr;
}

napi_value stats(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 1);
    mt_batch_stats s{};
    MT_OK_OR_THROW(mt_batch_get_stats(batch_of(env, a[0]), &s), "mt_batch_get_stats");
    napi_value o, v;
    NAPI_OK(napi_create_object(env, &o));
    auto put = [&](const char *k, double x) {
        napi_create_double(env, x, &v);
        napi_set_named_property(env, o, k, v);
    };
    put("nDocs", (double)s.n_docs);
    put("nOps", (double)s.n_ops);
    put("opsApplied", (double)s.ops_applied);
    put("docsFailed", (double)s.docs_failed);
    put("launches", s.launches);
    put("kernelMs", s.kernel_ms);
    put("totalMs", s.total_ms);
    put("ldsBytes", s.lds_bytes);
    return o;
}

napi_value status_string(napi_env env, napi_callback_info info) {
    auto a = args(env, info, 1);
    const char *s = mt_status_string((int)i64(env, a[0]));
    napi_value r;
    NAPI_OK(napi_create_string_utf8(env, s, NAPI_AUTO_LENGTH, &r));
    return r;
}

constexpr napi_property_attributes kMethod =
    static_cast<napi_property_attributes>(napi_writable | napi_enumerable | napi_configurable);

napi_value init(napi_env env, napi_value exports) {
    // the library must speak this header's binary interface (struct layouts, signatures)
    if (mt_abi_version() != MT_ABI_VERSION) {
        napi_throw_error(env, nullptr, "libmtreplay.so: C ABI version differs from include/mtreplay.h");
        return nullptr;
    }
    const napi_property_descriptor d[] = {
        {"createBatch", nullptr, create_batch, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"setTables", nullptr, set_tables, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"setClients", nullptr, set_clients, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"ingest", nullptr, ingest, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"ingestJson", nullptr, ingest_json, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"generate", nullptr, generate, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"run", nullptr, run, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"runAsync", nullptr, run_async, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"docStatus", nullptr, doc_status, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"docText", nullptr, doc_text, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"docPropsRuns", nullptr, doc_props_runs, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"docSnapshotV1", nullptr, doc_snapshot, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"docDigest", nullptr, doc_digest, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"docFindTile", nullptr, doc_find_tile, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"docStackContext", nullptr, doc_stack_context, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"docRegeneratedOps", nullptr, doc_regenerated_ops, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"docConsensusEvents", nullptr, doc_consensus_events, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"deviceDigests", nullptr, device_digests, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"stats", nullptr, stats, nullptr, nullptr, nullptr, kMethod, nullptr},
        {"statusString", nullptr, status_string, nullptr, nullptr, nullptr, kMethod, nullptr},
    };
    napi_define_properties(env, exports, sizeof d / sizeof d[0], d);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
