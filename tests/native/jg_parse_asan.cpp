// jg_parse_asan.cpp — TEST INFRASTRUCTURE: the GPU JSON parser's lane parser (mt_json_gpu.hip,
// parse_msg and everything below it, host-callable) run on the CPU under AddressSanitizer.
//
// usage: jg_parse_asan <file with one JSON document per line> <mutations per document> <seed>
// Every document (and every mutated copy: random bytes replaced / inserted / deleted, truncation)
// is laid out like on the device (inside a larger buffer at a random alignment, 64 bytes of zero
// padding after it); message starts come from a host restatement of the structural scan; every
// message is parsed twice like the count and write passes, the write pass into buffers of exactly
// the counted sizes, so any read or write out of bounds aborts.  Prints "ok <messages> <parsed>".
#include "../../fluidframework_amd/csrc/mt_json_gpu.hip"

#include <cstdio>
#include <fstream>
#include <random>
#include <string>
#include <vector>

using namespace mt::jg;

// parse()'s host merge formats off-form prop values with mt_json.cpp's JSON.stringify; the harness
// runs only the lane parser (parse() is never called), so it links without mt_json.cpp
bool mt::json_canonical_value(const char *, size_t, std::string &) { return false; }

static std::vector<uint32_t> message_starts(const std::string &d) {
    std::vector<uint32_t> st;
    int depth = 0;
    bool in_str = false, esc = false;
    for (uint32_t i = 0; i < d.size(); i++) {
        const char c = d[i];
        if (in_str) {
            if (esc) esc = false;
            else if (c == '\\') esc = true;
            else if (c == '"') in_str = false;
            continue;
        }
        if (c == '"') in_str = true;
        else if (c == '{' || c == '[') {
            if (depth == 1 && c == '{') st.push_back(i);
            depth++;
        } else if (c == '}' || c == ']') {
            if (--depth < 0) return {};
        }
    }
    return st;
}

static uint64_t parsed = 0, messages = 0;

static void run_doc(const std::string &d, std::mt19937_64 &rng) {
    const uint32_t lead = 64 + (uint32_t)(rng() % 16);
    std::vector<uint8_t> buf(lead + d.size() + 64, 0);  // the device buffer: documents + 64 B of padding
    memcpy(buf.data() + lead, d.data(), d.size());
    const uint8_t *s = buf.data() + lead;
    const uint32_t n = (uint32_t)d.size();
    for (uint32_t p0 : message_starts(d)) {
        messages++;
        MsgOut mo;
        Ctx cx;
        if (parse_msg<false>(s, n, p0, mo, cx)) continue;
        // write pass into exactly-sized heap buffers
        mt_op *ops = new mt_op[mo.nrec];
        uint16_t *text = new uint16_t[mo.ntext ? mo.ntext : 1];
        uint32_t *pk_off = new uint32_t[mo.nprop + 1], *pk_len = new uint32_t[mo.nprop + 1];
        uint32_t *pv_off = new uint32_t[mo.nval + 1], *pv_len = new uint32_t[mo.nval + 1];
        uint32_t *pe = new uint32_t[mo.nprop + 1];
        Ctx w;
        w.ops = ops;
        w.text = text;
        w.pay = 0;
        w.gprop = 0;
        w.pk_off = pk_off;
        w.pk_len = pk_len;
        w.pv_off = pv_off;
        w.pv_len = pv_len;
        w.pe = pe;
        w.gval = 0;
        w.cid = 1;
        w.install = (rng() & 1) != 0;
        MsgOut mw;
        const uint32_t f = parse_msg<true>(s, n, p0, mw, w);
        if (f || mw.nrec != mo.nrec || mw.ntext != mo.ntext || mw.nprop != mo.nprop || mw.nval != mo.nval) {
            fprintf(stderr, "count / write passes differ at %u\n", p0);
            abort();
        }
        for (uint32_t q = 0; q < mo.nprop; q++)  // spans inside the document, events in range
            if (pk_off[q] + pk_len[q] > n || pe[q] >= mo.nval) {
                fprintf(stderr, "prop record out of range at %u\n", p0);
                abort();
            }
        for (uint32_t q = 0; q < mo.nval; q++)
            if (pv_off[q] != kNullSpan && pv_off[q] + (pv_len[q] & ~kSpanCanon) > n) {
                fprintf(stderr, "value span outside the document at %u\n", p0);
                abort();
            }
        for (uint32_t q = 0; q < mo.nrec; q++)
            if (ops[q].type == MT_OP_RELPOS && ((uint32_t)ops[q].pos1 > mo.nval || (uint32_t)ops[q].pos2 > mo.nval)) {
                fprintf(stderr, "relative position event out of range at %u\n", p0);
                abort();
            }
        parsed++;
        delete[] ops;
        delete[] text;
        delete[] pk_off;
        delete[] pk_len;
        delete[] pv_off;
        delete[] pv_len;
        delete[] pe;
    }
}

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    std::ifstream in(argv[1]);
    const int muts = atoi(argv[2]);
    std::mt19937_64 rng(strtoull(argv[3], nullptr, 0));
    const char alpha[] = "{}[]\",:\\ 0123456789-.eEtruefalsn\"u\\";
    std::string line;
    while (std::getline(in, line)) {
        run_doc(line, rng);
        for (int k = 0; k < muts; k++) {
            std::string m = line;
            const int edits = 1 + (int)(rng() % 4);
            for (int e = 0; e < edits && !m.empty(); e++) {
                const size_t at = rng() % m.size();
                switch (rng() % 4) {
                    case 0: m[at] = alpha[rng() % (sizeof alpha - 1)]; break;
                    case 1: m.insert(at, 1, alpha[rng() % (sizeof alpha - 1)]); break;
                    case 2: m.erase(at, 1 + rng() % 8); break;
                    default: m.resize(at); break;
                }
            }
            run_doc(m, rng);
        }
    }
    printf("ok %llu %llu\n", (unsigned long long)messages, (unsigned long long)parsed);
    return 0;
}
