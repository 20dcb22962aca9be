// mt_values.cpp — matchProperties for interned property values (host side, no GPU).
//
// The device compares property sets by (key id, value id) records.  The reference's
// matchProperties (merge-tree/src/properties.ts:62-93) is structural: nested objects compare
// recursively and ignore key order, an array equals an index-keyed object, `for (key in v)` over
// a string enumerates its indices, and a falsy primitive "matches" a nested null.  It is also
// asymmetric and not transitive.  Per pair of top-level values (a from the earlier segment, b
// from the later one) the relation the device needs is
//     R(a, b) = typeof b === "object" ? matchProperties(a, b) : a === b
// (the per-key step of matchProperties over two property sets, which are Object.create(null)
// maps: same key set, then R for every key).
//
// Every value gets a structural class id (canonical form: objects as key-sorted maps, arrays as
// index maps, numbers by value, strings by UTF-16 content): equal classes always satisfy R.  The
// pairs of the batch's value table that satisfy R with *different* classes are listed
// explicitly ("exceptions"; both values get kValIrregular), so the device decides R exactly:
// class equality, else a lookup in the sorted exception list.  When the table is too large for
// the pairwise pass, object values get kValUnknown and a class-different comparison involving
// one makes the document MT_UNSUPPORTED instead of guessing.
//
// The semantics follow the test oracle's restatement (oracle/jsv.c jv_match_properties: own
// keys, array / string indices and "length"; prototype members are not modelled).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "mt_values.h"

namespace {

using u16s = std::u16string;

struct JV {
    enum Kind { NUL, TRUE, FALSE, NUM, STR, ARR, OBJ } kind = NUL;
    double num = 0;
    u16s str;
    std::vector<u16s> keys;  // OBJ: own keys (first-insertion order; duplicates: last value wins)
    std::vector<JV> vals;    // ARR elements / OBJ values
};

struct Parser {
    const char *p, *e;
    bool ok = true;
    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
    }
    static int hexv(char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    void put_cp(u16s &o, uint32_t cp) {
        if (cp >= 0x10000) {
            cp -= 0x10000;
            o.push_back((char16_t)(0xD800 + (cp >> 10)));
            o.push_back((char16_t)(0xDC00 + (cp & 0x3FF)));
        } else {
            o.push_back((char16_t)cp);
        }
    }
    bool string(u16s &o) {
        if (p >= e || *p != '"') return false;
        p++;
        while (p < e && *p != '"') {
            unsigned char c = (unsigned char)*p;
            if (c == '\\') {
                if (++p >= e) return false;
                char x = *p++;
                switch (x) {
                    case '"': o.push_back(u'"'); break;
                    case '\\': o.push_back(u'\\'); break;
                    case '/': o.push_back(u'/'); break;
                    case 'b': o.push_back(u'\b'); break;
                    case 'f': o.push_back(u'\f'); break;
                    case 'n': o.push_back(u'\n'); break;
                    case 'r': o.push_back(u'\r'); break;
                    case 't': o.push_back(u'\t'); break;
                    case 'u': {
                        if (e - p < 4) return false;
                        uint32_t v = 0;
                        for (int i = 0; i < 4; i++) {
                            int h = hexv(p[i]);
                            if (h < 0) return false;
                            v = v * 16 + (uint32_t)h;
                        }
                        p += 4;
                        o.push_back((char16_t)v);  // surrogates stay code units (JS strings)
                        break;
                    }
                    default: return false;
                }
                continue;
            }
            // UTF-8 (WTF-8: encoded lone surrogates pass through as code units)
            uint32_t cp = c;
            int len = 1;
            if (c < 0x80) len = 1;
            else if ((c & 0xE0) == 0xC0) len = 2, cp &= 0x1F;
            else if ((c & 0xF0) == 0xE0) len = 3, cp &= 0x0F;
            else if ((c & 0xF8) == 0xF0) len = 4, cp &= 0x07;
            else return false;
            if (e - p < len) return false;
            for (int i = 1; i < len; i++) cp = (cp << 6) | ((unsigned char)p[i] & 0x3F);
            p += len;
            put_cp(o, cp);
        }
        if (p >= e) return false;
        p++;
        return true;
    }
    bool value(JV &v, int depth) {
        if (depth > 64) return false;
        ws();
        if (p >= e) return false;
        if (*p == '{') {
            p++;
            v.kind = JV::OBJ;
            ws();
            if (p < e && *p == '}') {
                p++;
                return true;
            }
            for (;;) {
                ws();
                u16s k;
                if (!string(k)) return false;
                ws();
                if (p >= e || *p != ':') return false;
                p++;
                JV x;
                if (!value(x, depth + 1)) return false;
                auto it = std::find(v.keys.begin(), v.keys.end(), k);
                if (it != v.keys.end()) v.vals[(size_t)(it - v.keys.begin())] = std::move(x);
                else v.keys.push_back(std::move(k)), v.vals.push_back(std::move(x));
                ws();
                if (p < e && *p == ',') {
                    p++;
                    continue;
                }
                if (p < e && *p == '}') {
                    p++;
                    return true;
                }
                return false;
            }
        }
        if (*p == '[') {
            p++;
            v.kind = JV::ARR;
            ws();
            if (p < e && *p == ']') {
                p++;
                return true;
            }
            for (;;) {
                JV x;
                if (!value(x, depth + 1)) return false;
                v.vals.push_back(std::move(x));
                ws();
                if (p < e && *p == ',') {
                    p++;
                    continue;
                }
                if (p < e && *p == ']') {
                    p++;
                    return true;
                }
                return false;
            }
        }
        if (*p == '"') {
            v.kind = JV::STR;
            return string(v.str);
        }
        if (e - p >= 4 && !memcmp(p, "null", 4)) return v.kind = JV::NUL, p += 4, true;
        if (e - p >= 4 && !memcmp(p, "true", 4)) return v.kind = JV::TRUE, p += 4, true;
        if (e - p >= 5 && !memcmp(p, "false", 5)) return v.kind = JV::FALSE, p += 5, true;
        std::string t;
        while (p < e && (strchr("+-.eE", *p) || (*p >= '0' && *p <= '9'))) t.push_back(*p++);
        if (t.empty()) return false;
        char *end = nullptr;
        v.kind = JV::NUM;
        v.num = strtod(t.c_str(), &end);
        if (v.num == 0) v.num = 0;  // -0 === 0
        return end && *end == 0;
    }
};

bool truthy(const JV *v) {
    if (!v) return false;
    switch (v->kind) {
        case JV::NUL: case JV::FALSE: return false;
        case JV::NUM: return !(v->num == 0 || std::isnan(v->num));
        case JV::STR: return !v->str.empty();
        default: return true;
    }
}
bool typeof_object(const JV *v) { return v && (v->kind == JV::OBJ || v->kind == JV::ARR || v->kind == JV::NUL); }

bool array_index(const u16s &k, uint32_t *idx) {
    if (k.empty() || k.size() > 10) return false;
    if (k[0] == u'0') {
        if (k.size() != 1) return false;
        *idx = 0;
        return true;
    }
    uint64_t x = 0;
    for (char16_t c : k) {
        if (c < u'0' || c > u'9') return false;
        x = x * 10 + (uint64_t)(c - u'0');
    }
    if (x > 4294967294ull) return false;
    *idx = (uint32_t)x;
    return true;
}
u16s index_key(size_t i) {
    std::string s = std::to_string(i);
    return u16s(s.begin(), s.end());
}

// js_get of the oracle: own keys; array / string index and "length"; nothing on primitives
struct Got {
    const JV *v = nullptr;
    JV tmp;
    bool has = false;
};
void js_get(const JV *v, const u16s &k, Got &g) {
    g.v = nullptr;
    g.has = false;
    if (!v) return;
    static const u16s LENGTH = u"length";
    uint32_t idx;
    if (v->kind == JV::OBJ) {
        for (size_t i = 0; i < v->keys.size(); i++)
            if (v->keys[i] == k) {
                g.v = &v->vals[i];
                g.has = true;
                return;
            }
    } else if (v->kind == JV::ARR || v->kind == JV::STR) {
        const size_t n = v->kind == JV::ARR ? v->vals.size() : v->str.size();
        if (array_index(k, &idx)) {
            if (idx < n) {
                if (v->kind == JV::ARR) {
                    g.v = &v->vals[idx];
                } else {
                    g.tmp.kind = JV::STR;
                    g.tmp.str = u16s(1, v->str[idx]);
                    g.v = &g.tmp;
                }
                g.has = true;
            }
        } else if (k == LENGTH) {
            g.tmp.kind = JV::NUM;
            g.tmp.num = (double)n;
            g.v = &g.tmp;
            g.has = true;
        }
    }
}
std::vector<u16s> for_in_keys(const JV *v) {
    std::vector<u16s> out;
    if (!v) return out;
    if (v->kind == JV::OBJ) return v->keys;
    if (v->kind == JV::ARR || v->kind == JV::STR) {
        const size_t n = v->kind == JV::ARR ? v->vals.size() : v->str.size();
        for (size_t i = 0; i < n; i++) out.push_back(index_key(i));
    }
    return out;
}
bool strict_eq(const JV *a, const JV *b) {
    if (!a || !b) return a == b;
    if (a->kind != b->kind) return false;
    switch (a->kind) {
        case JV::NUL: case JV::TRUE: case JV::FALSE: return true;
        case JV::NUM: return a->num == b->num;
        case JV::STR: return a->str == b->str;
        default: return a == b;  // object identity: distinct table values are distinct objects
    }
}

// properties.ts:62-93
bool match_properties(const JV *a, const JV *b) {
    if (truthy(a)) {
        if (!truthy(b)) return false;
        for (const u16s &k : for_in_keys(a)) {
            Got gb, ga;
            js_get(b, k, gb);
            js_get(a, k, ga);
            if (!gb.has) return false;
            if (typeof_object(gb.v)) {
                if (!match_properties(ga.v, gb.v)) return false;
            } else if (!strict_eq(gb.v, ga.v)) {
                return false;
            }
        }
        for (const u16s &k : for_in_keys(b)) {
            Got ga;
            js_get(a, k, ga);
            if (!ga.has) return false;
        }
        return true;
    }
    return !truthy(b);
}

// canonical structural form, interned
struct Canon {
    std::map<std::string, uint32_t> ids;
    uint32_t id_of(const std::string &s) {
        auto it = ids.find(s);
        if (it != ids.end()) return it->second;
        const uint32_t id = (uint32_t)ids.size() + 1;
        ids.emplace(s, id);
        return id;
    }
    static void put_u16s(std::string &o, const u16s &s) {
        uint32_t n = (uint32_t)s.size();
        o.append((const char *)&n, 4);
        o.append((const char *)s.data(), 2 * s.size());
    }
    uint32_t of(const JV &v) {
        std::string o;
        switch (v.kind) {
            case JV::NUL: o = "N"; break;
            case JV::TRUE: o = "T"; break;
            case JV::FALSE: o = "F"; break;
            case JV::NUM: o = "n"; o.append((const char *)&v.num, 8); break;
            case JV::STR: o = "s"; put_u16s(o, v.str); break;
            case JV::ARR:
            case JV::OBJ: {
                std::vector<std::pair<u16s, uint32_t>> kv;
                for (size_t i = 0; i < v.vals.size(); i++)
                    kv.emplace_back(v.kind == JV::ARR ? index_key(i) : v.keys[i], of(v.vals[i]));
                std::sort(kv.begin(), kv.end());
                o = "o";
                for (auto &x : kv) {
                    put_u16s(o, x.first);
                    o.append((const char *)&x.second, 4);
                }
                break;
            }
        }
        return id_of(o);
    }
};

}  // namespace

namespace mt {

int value_relations(const std::vector<std::string> &values, std::vector<uint32_t> &cls, std::vector<uint8_t> &flags,
                    std::vector<uint64_t> &exc, int64_t max_pairs) {
    const size_t V = values.size();
    std::vector<JV> jv(V);
    std::vector<uint8_t> parsed(V, 0);
    cls.assign(V, 0);
    if (flags.size() != V) flags.resize(V, 0);
    exc.clear();
    Canon canon;
    for (size_t i = 0; i < V; i++) {
        if (flags[i] & kValNever) {  // derived values that match nothing: a class of their own
            cls[i] = canon.id_of("!" + std::to_string(i));
            continue;
        }
        Parser P{values[i].data(), values[i].data() + values[i].size()};
        JV v;
        if (P.value(v, 0)) {
            P.ws();
            if (P.p == P.e) {
                parsed[i] = 1;
                jv[i] = std::move(v);
            }
        }
        // an unparsable text only ever equals itself (its own class)
        cls[i] = parsed[i] ? canon.of(jv[i]) : canon.id_of("?" + values[i]);
        if (!parsed[i]) continue;
        const JV &x = jv[i];
        if (x.kind == JV::NUM || x.kind == JV::TRUE || x.kind == JV::FALSE) flags[i] |= kValNum;
        if (x.kind == JV::OBJ)
            for (size_t k = 0; k < x.keys.size(); k++)
                if (x.keys[k] == u"seq" && x.vals[k].kind == JV::NUM && x.vals[k].num == -1) flags[i] |= kValSeqM1;
    }
    // exceptions: R(u, v) with v an object / array (a top-level null means "delete": never stored)
    std::vector<size_t> objs;
    for (size_t i = 1; i < V; i++)
        if (parsed[i] && (jv[i].kind == JV::OBJ || jv[i].kind == JV::ARR)) objs.push_back(i);
    if (objs.empty()) return 0;
    if ((int64_t)objs.size() * (int64_t)V > max_pairs) {
        for (size_t v : objs) flags[v] |= kValUnknown;
        return 1;
    }
    for (size_t v : objs) {
        for (size_t u = 1; u < V; u++) {
            if (u == v || !parsed[u] || cls[u] == cls[v]) continue;
            if (match_properties(&jv[u], &jv[v])) {
                exc.push_back((uint64_t)u << 32 | (uint64_t)v);
                flags[u] |= kValIrregular;
                flags[v] |= kValIrregular;
            }
        }
    }
    std::sort(exc.begin(), exc.end());
    return 0;
}

namespace {
// JSON.stringify of a parsed value (key order: array indices ascending, then insertion order)
void stringify(const JV &v, std::string &o) {
    switch (v.kind) {
        case JV::NUL: o += "null"; return;
        case JV::TRUE: o += "true"; return;
        case JV::FALSE: o += "false"; return;
        case JV::NUM: json_number(o, v.num); return;
        case JV::STR: json_quote(o, v.str.data(), v.str.size()); return;
        case JV::ARR:
            o.push_back('[');
            for (size_t i = 0; i < v.vals.size(); i++) {
                if (i) o.push_back(',');
                stringify(v.vals[i], o);
            }
            o.push_back(']');
            return;
        case JV::OBJ: {
            std::vector<std::pair<uint32_t, size_t>> idx;
            std::vector<size_t> rest;
            for (size_t i = 0; i < v.keys.size(); i++) {
                uint32_t a;
                if (array_index(v.keys[i], &a)) idx.emplace_back(a, i);
                else rest.push_back(i);
            }
            std::sort(idx.begin(), idx.end());
            std::vector<size_t> order;
            for (auto &x : idx) order.push_back(x.second);
            order.insert(order.end(), rest.begin(), rest.end());
            o.push_back('{');
            for (size_t j = 0; j < order.size(); j++) {
                if (j) o.push_back(',');
                json_quote(o, v.keys[order[j]].data(), v.keys[order[j]].size());
                o.push_back(':');
                stringify(v.vals[order[j]], o);
            }
            o.push_back('}');
            return;
        }
    }
}
// String(v): "[object Object]" for a plain object, Array.prototype.join(",") for an array
void to_string(const JV &v, u16s &o) {
    switch (v.kind) {
        case JV::NUL: o += u"null"; return;
        case JV::TRUE: o += u"true"; return;
        case JV::FALSE: o += u"false"; return;
        case JV::NUM: {
            std::string t;
            json_number(t, v.num);
            o.append(t.begin(), t.end());
            return;
        }
        case JV::STR: o += v.str; return;
        case JV::OBJ: o += u"[object Object]"; return;
        case JV::ARR:
            for (size_t i = 0; i < v.vals.size(); i++) {
                if (i) o.push_back(u',');
                if (v.vals[i].kind != JV::NUL) to_string(v.vals[i], o);
            }
            return;
    }
}
bool parse(const std::string &t, JV &v) {
    Parser P{t.data(), t.data() + t.size()};
    if (!P.value(v, 0)) return false;
    P.ws();
    return P.p == P.e;
}
}  // namespace

bool js_string_of(const std::string &json, std::u16string &out) {
    JV v;
    if (!parse(json, v)) return false;
    out.clear();
    to_string(v, out);
    return true;
}

// combine kinds: include/mt_oplog.h mt_combine_kind (1 incr, 2 consensus, 3 other)
CombineResult combine_absent(int kind, const std::string *def, const std::string *min, int32_t seq, std::string &out) {
    JV d;
    if (def && !parse(*def, d)) return kCombineUnsupported;
    if (kind == 1) {  // incr: currentValue = defaultValue; currentValue += undefined
        if (!def || d.kind == JV::NUL || d.kind == JV::TRUE || d.kind == JV::FALSE || d.kind == JV::NUM)
            return kCombineNaN;  // NaN < minValue is false: no clamp
        u16s r;
        to_string(d, r);
        r += u"undefined";
        // `r < minValue`: r's ToNumber is NaN, so only a string comparison (minValue a string, or an
        // object / array compared through its String()) can hold: UTF-16 code-unit order
        JV m;
        if (min && parse(*min, m) && truthy(&m) && (m.kind == JV::STR || m.kind == JV::OBJ || m.kind == JV::ARR)) {
            u16s ms;
            to_string(m, ms);
            if (r < ms) return kCombineMin;
        }
        out.clear();
        json_quote(out, r.data(), r.size());
        return kCombineValue;
    }
    if (kind == 2) {  // consensus
        if (!def) {
            out = "{\"seq\":";
            json_number(out, (double)seq);
            out += "}";
            return kCombineConsensus;
        }
        if (d.kind == JV::NUL) return kCombineUnsupported;  // TypeError: reading seq of null
        if (d.kind == JV::OBJ)
            for (size_t k = 0; k < d.keys.size(); k++)
                if (d.keys[k] == u"seq" && d.vals[k].kind == JV::NUM && d.vals[k].num == -1) {
                    d.vals[k].num = (double)seq;  // cv.seq = seq on the op's defaultValue object
                    out.clear();
                    stringify(d, out);
                    return kCombineValue;
                }
        out = *def;
        return kCombineValue;
    }
    // any other combiningOp: combine returns currentValue (= defaultValue)
    if (!def) return kCombineUnsupported;  // properties[key] = undefined
    if (d.kind == JV::NUL) return kCombineDelete;
    out = *def;
    return kCombineValue;
}

}  // namespace mt
