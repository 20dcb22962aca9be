// mt_json_gpu.h — GPU JSON op-log ingest (mt_json_gpu.hip), host-side interface.
//
// The device parses per-document ISequencedDocumentMessage JSON arrays (the file driver's
// messages.json: fileDeltaStorageService.ts:23-31) into the packed records of mt_oplog.h with
// exactly the rules of mt_json.cpp's host parser (itself equal to the Python / JS packers), for
// the observer fast path: sequenced messages whose contents are insert (text, {text, props} or a
// marker), remove, annotate (no combiningOp or rewrite), relative positions, or a one-level GROUP
// of those, property values that are null / true / false / canonical integers / plain ASCII
// strings / flat arrays of those in JSON.stringify form.  Anything else (writer replicas,
// snapshots, escapes in keys or values, floats, objects as values, duplicate keys, > 4093
// clients, malformed JSON) is reported as "host parser needed"
// (MT_UNSUPPORTED + the first such document): the caller runs mt_pack_json for that batch.
#ifndef MT_JSON_GPU_H
#define MT_JSON_GPU_H

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "../../include/mt_oplog.h"

struct mt_packed;

namespace mt {
// JSON.stringify(JSON.parse(text)) of one JSON value with the host parser's JS semantics
// (mt_json.cpp: Number::toString, JS key order, duplicate keys, lone surrogates); false when
// [p, p + n) is not exactly one JSON value (surrounding whitespace allowed)
bool json_canonical_value(const char *p, size_t n, std::string &out);

namespace jg {

struct Result {
    int status = 0;         // MT_OK, MT_UNSUPPORTED (host parser needed), MT_ERR_*
    int64_t bad_doc = -1;   // first document outside the GPU fast path
    uint32_t fail_bits = 0; // reasons (kF* in mt_json_gpu.hip) of bad_doc
    bool writer = false;    // a writer replica's log (local ops / acks) in some document
    int64_t n_ops = 0, n_text = 0, n_props = 0, n_msgs = 0;
    std::vector<int64_t> doc_op_off;       // D + 1, batch-global record offsets
    std::vector<uint32_t> doc_text;        // code units per document
    std::vector<uint32_t> doc_nprop_ops;   // annotates + inserts carrying props (pool sizing)
    std::vector<uint32_t> doc_nprops;      // prop records per document
    std::vector<std::string> keys, values; // batch tables (values: JSON text, 0 = "null")
    std::vector<std::vector<std::string>> clients;  // per document, observer first
    float ms_scan = 0, ms_count = 0, ms_clients = 0, ms_write = 0, ms_props = 0;
    double ms_host = 0;                    // host merge of the interning tables
};

// text_base(res, base, total): the text destination of each document (install: the replay's
// arena layout, payloads document-relative with the '\n' flags; packed: nullptr -> the packed
// format, payloads batch-global).
using TextLayout = std::function<int(const Result &, std::vector<uint64_t> &, uint64_t &)>;

// Parse D documents: h_json (host copy, needed for the interning tables) with doc_off[D + 1];
// d_json: the same bytes on the device (nullptr: uploaded here), 4-byte aligned, readable 64 bytes
// past the end.
// On MT_OK *d_ops / *d_text / *d_props are device allocations owned by the caller.
int parse(const char *h_json, const int64_t *doc_off, int64_t D, const uint8_t *d_json, const char *observer,
          void *stream, const TextLayout *install, mt_op **d_ops, uint16_t **d_text, uint64_t *text_words,
          mt_prop **d_props, Result &res);

// the most unacked local ops any writer replica of a parsed log holds (mt_host.cpp writer_regions)
int pending_peak(const mt_op *d_ops, const int64_t *d_off, int64_t D, void *stream, int64_t *out);

}  // namespace jg
}  // namespace mt

// mt_json.cpp: an mt_packed from arrays (the GPU parser's packed output)
mt_packed *mt_packed_from(std::vector<mt_op> &&ops, std::vector<int64_t> &&off, std::vector<uint16_t> &&text,
                          std::vector<mt_prop> &&props, std::vector<std::string> &&keys,
                          std::vector<std::string> &&values, std::vector<std::vector<std::string>> &&clients);

#endif  // MT_JSON_GPU_H
