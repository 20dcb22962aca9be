/*
 * jsv.c — JSON values with JavaScript semantics (TEST INFRASTRUCTURE ONLY).
 * See jsv.h for what this restates and why.
 */
#include "jsv.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ sb */
void sb_init(sb *b) { b->p = NULL; b->n = b->cap = 0; }
void sb_free(sb *b) { free(b->p); b->p = NULL; b->n = b->cap = 0; }
static void sb_grow(sb *b, size_t need) {
    if (b->n + need + 1 <= b->cap) return;
    size_t c = b->cap ? b->cap : 64;
    while (c < b->n + need + 1) c *= 2;
    b->p = (char *)realloc(b->p, c);
    b->cap = c;
}
void sb_putc(sb *b, char c) { sb_grow(b, 1); b->p[b->n++] = c; b->p[b->n] = 0; }
void sb_putn(sb *b, const char *s, size_t n) {
    sb_grow(b, n);
    memcpy(b->p + b->n, s, n);
    b->n += n;
    b->p[b->n] = 0;
}
void sb_puts(sb *b, const char *s) { sb_putn(b, s, strlen(s)); }

static void sb_put_cp(sb *b, uint32_t cp) {
    char t[4];
    if (cp < 0x80) { sb_putc(b, (char)cp); return; }
    if (cp < 0x800) {
        t[0] = (char)(0xC0 | (cp >> 6)); t[1] = (char)(0x80 | (cp & 0x3F));
        sb_putn(b, t, 2); return;
    }
    if (cp < 0x10000) {
        t[0] = (char)(0xE0 | (cp >> 12)); t[1] = (char)(0x80 | ((cp >> 6) & 0x3F));
        t[2] = (char)(0x80 | (cp & 0x3F));
        sb_putn(b, t, 3); return;
    }
    t[0] = (char)(0xF0 | (cp >> 18)); t[1] = (char)(0x80 | ((cp >> 12) & 0x3F));
    t[2] = (char)(0x80 | ((cp >> 6) & 0x3F)); t[3] = (char)(0x80 | (cp & 0x3F));
    sb_putn(b, t, 4);
}

void sb_put_u16_utf8(sb *b, const u16 *s, int n) {
    for (int i = 0; i < n; i++) {
        uint32_t c = s[i];
        if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
            uint32_t cp = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00);
            sb_put_cp(b, cp);
            i++;
        } else if (c >= 0xD800 && c <= 0xDFFF) {
            sb_put_cp(b, 0xFFFD);
        } else {
            sb_put_cp(b, c);
        }
    }
}

/* ------------------------------------------------------------------ values */
jv *jv_new(int kind) {
    jv *v = (jv *)calloc(1, sizeof(jv));
    v->kind = kind;
    v->rc = 1;
    return v;
}
jv *jv_new_num(double d) { jv *v = jv_new(JV_NUM); v->num = d; return v; }
jv *jv_new_str(const u16 *s, int n) {
    jv *v = jv_new(JV_STR);
    v->s = (u16 *)malloc(sizeof(u16) * (size_t)(n > 0 ? n : 1));
    if (n) memcpy(v->s, s, sizeof(u16) * (size_t)n);
    v->slen = n;
    return v;
}
jv *jv_new_str_ascii(const char *s) {
    int n = (int)strlen(s);
    jv *v = jv_new(JV_STR);
    v->s = (u16 *)malloc(sizeof(u16) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) v->s[i] = (u16)(unsigned char)s[i];
    v->slen = n;
    return v;
}
/* refcounts are atomic: property values from mto_tables are shared by the worker threads
   of mto_replay_batch */
jv *jv_ref(jv *v) {
    if (v) __atomic_add_fetch(&v->rc, 1, __ATOMIC_RELAXED);
    return v;
}
void jv_unref(jv *v) {
    if (!v) return;
    if (__atomic_sub_fetch(&v->rc, 1, __ATOMIC_ACQ_REL) > 0) return;
    free(v->s);
    for (int i = 0; i < v->n; i++) {
        jv_unref(v->vals[i]);
        if (v->keys) free(v->keys[i]);
    }
    free(v->vals);
    free(v->keys);
    free(v->klens);
    free(v);
}

int u16_eq(const u16 *a, int an, const u16 *b, int bn) {
    return an == bn && (an == 0 || memcmp(a, b, sizeof(u16) * (size_t)an) == 0);
}

static void jv_reserve(jv *o, int need) {
    if (o->n + need <= o->cap) return;
    int c = o->cap ? o->cap * 2 : 4;
    while (c < o->n + need) c *= 2;
    o->vals = (jv **)realloc(o->vals, sizeof(jv *) * (size_t)c);
    if (o->kind == JV_OBJ) {
        o->keys = (u16 **)realloc(o->keys, sizeof(u16 *) * (size_t)c);
        o->klens = (int *)realloc(o->klens, sizeof(int) * (size_t)c);
    }
    o->cap = c;
}

static int obj_find(const jv *o, const u16 *k, int kl) {
    for (int i = 0; i < o->n; i++)
        if (u16_eq(o->keys[i], o->klens[i], k, kl)) return i;
    return -1;
}
jv *jv_obj_get(const jv *o, const u16 *k, int kl) {
    int i = obj_find(o, k, kl);
    return i < 0 ? NULL : o->vals[i];
}
static int ascii_to_u16(const char *s, u16 *out, int cap) {
    int n = 0;
    while (s[n] && n < cap) { out[n] = (u16)(unsigned char)s[n]; n++; }
    return n;
}
jv *jv_obj_get_ascii(const jv *o, const char *k) {
    u16 t[256];
    int n = ascii_to_u16(k, t, 256);
    return jv_obj_get(o, t, n);
}
void jv_obj_set(jv *o, const u16 *k, int kl, jv *v) {
    int i = obj_find(o, k, kl);
    if (i >= 0) {
        jv_unref(o->vals[i]);
        o->vals[i] = v;
        return;
    }
    jv_reserve(o, 1);
    o->keys[o->n] = (u16 *)malloc(sizeof(u16) * (size_t)(kl > 0 ? kl : 1));
    if (kl) memcpy(o->keys[o->n], k, sizeof(u16) * (size_t)kl);
    o->klens[o->n] = kl;
    o->vals[o->n] = v;
    o->n++;
}
void jv_obj_set_ascii(jv *o, const char *k, jv *v) {
    u16 t[256];
    int n = ascii_to_u16(k, t, 256);
    jv_obj_set(o, t, n, v);
}
int jv_obj_del(jv *o, const u16 *k, int kl) {
    int i = obj_find(o, k, kl);
    if (i < 0) return 0;
    jv_unref(o->vals[i]);
    free(o->keys[i]);
    for (int j = i + 1; j < o->n; j++) {
        o->vals[j - 1] = o->vals[j];
        o->keys[j - 1] = o->keys[j];
        o->klens[j - 1] = o->klens[j];
    }
    o->n--;
    return 1;
}
jv *jv_obj_clone(const jv *o) {
    jv *c = jv_new(JV_OBJ);
    for (int i = 0; i < o->n; i++) jv_obj_set(c, o->keys[i], o->klens[i], jv_ref(o->vals[i]));
    return c;
}

int js_is_array_index(const u16 *k, int kl, uint32_t *idx) {
    if (kl == 0 || kl > 10) return 0;
    if (k[0] == '0') {
        if (kl != 1) return 0;
        if (idx) *idx = 0;
        return 1;
    }
    uint64_t v = 0;
    for (int i = 0; i < kl; i++) {
        if (k[i] < '0' || k[i] > '9') return 0;
        v = v * 10 + (uint64_t)(k[i] - '0');
    }
    if (v > 4294967294ull) return 0;
    if (idx) *idx = (uint32_t)v;
    return 1;
}

typedef struct { uint32_t idx; int pos; } ikey;
static int ikey_cmp(const void *a, const void *b) {
    const ikey *x = (const ikey *)a, *y = (const ikey *)b;
    return x->idx < y->idx ? -1 : x->idx > y->idx ? 1 : 0;
}
int jv_obj_enum(const jv *o, int *order) {
    int m = 0;
    ikey *ik = (ikey *)malloc(sizeof(ikey) * (size_t)(o->n + 1));
    for (int i = 0; i < o->n; i++) {
        uint32_t idx;
        if (js_is_array_index(o->keys[i], o->klens[i], &idx)) { ik[m].idx = idx; ik[m].pos = i; m++; }
    }
    qsort(ik, (size_t)m, sizeof(ikey), ikey_cmp);
    int n = 0;
    for (int i = 0; i < m; i++) order[n++] = ik[i].pos;
    for (int i = 0; i < o->n; i++)
        if (!js_is_array_index(o->keys[i], o->klens[i], NULL)) order[n++] = i;
    free(ik);
    return n;
}

/* ------------------------------------------------------------------ stringify */
static const char HEX[] = "0123456789abcdef";

void js_quote(sb *b, const u16 *s, int n) {
    sb_putc(b, '"');
    for (int i = 0; i < n; i++) {
        uint32_t c = s[i];
        switch (c) {
            case 0x22: sb_puts(b, "\\\""); continue;
            case 0x5C: sb_puts(b, "\\\\"); continue;
            case 0x08: sb_puts(b, "\\b"); continue;
            case 0x0C: sb_puts(b, "\\f"); continue;
            case 0x0A: sb_puts(b, "\\n"); continue;
            case 0x0D: sb_puts(b, "\\r"); continue;
            case 0x09: sb_puts(b, "\\t"); continue;
            default: break;
        }
        if (c < 0x20) {
            char t[7] = {'\\', 'u', '0', '0', HEX[c >> 4], HEX[c & 15], 0};
            sb_puts(b, t);
            continue;
        }
        if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] <= 0xDFFF) {
            sb_put_cp(b, 0x10000 + ((c - 0xD800) << 10) + (uint32_t)(s[i + 1] - 0xDC00));
            i++;
            continue;
        }
        if (c >= 0xD800 && c <= 0xDFFF) { /* well-formed JSON.stringify: lone surrogate escaped */
            char t[7] = {'\\', 'u', HEX[c >> 12], HEX[(c >> 8) & 15], HEX[(c >> 4) & 15], HEX[c & 15], 0};
            sb_puts(b, t);
            continue;
        }
        sb_put_cp(b, c);
    }
    sb_putc(b, '"');
}

/* ECMAScript Number::toString(10) (ES2019 7.1.12.1) */
void js_number(sb *b, double d) {
    char buf[64];
    if (isnan(d)) { sb_puts(b, "NaN"); return; }
    if (d == 0) { sb_putc(b, '0'); return; }
    if (d < 0) { sb_putc(b, '-'); d = -d; }
    if (isinf(d)) { sb_puts(b, "Infinity"); return; }
    /* shortest round-tripping digit string */
    char digits[32];
    int k = 0, e10 = 0;
    for (int p = 1; p <= 17; p++) {
        snprintf(buf, sizeof buf, "%.*e", p - 1, d);
        if (strtod(buf, NULL) == d || p == 17) {
            /* buf = d[.ddd]e[+-]xx */
            char *ep = strchr(buf, 'e');
            e10 = atoi(ep + 1);
            k = 0;
            for (char *q = buf; q < ep; q++)
                if (*q >= '0' && *q <= '9') digits[k++] = *q;
            while (k > 1 && digits[k - 1] == '0') k--;
            digits[k] = 0;
            break;
        }
    }
    int n = e10 + 1; /* value = 0.digits * 10^n */
    if (k <= n && n <= 21) {
        sb_putn(b, digits, (size_t)k);
        for (int i = 0; i < n - k; i++) sb_putc(b, '0');
    } else if (0 < n && n <= 21) {
        sb_putn(b, digits, (size_t)n);
        sb_putc(b, '.');
        sb_putn(b, digits + n, (size_t)(k - n));
    } else if (-6 < n && n <= 0) {
        sb_puts(b, "0.");
        for (int i = 0; i < -n; i++) sb_putc(b, '0');
        sb_putn(b, digits, (size_t)k);
    } else {
        int e = n - 1;
        sb_putc(b, digits[0]);
        if (k > 1) {
            sb_putc(b, '.');
            sb_putn(b, digits + 1, (size_t)(k - 1));
        }
        snprintf(buf, sizeof buf, "e%c%d", e < 0 ? '-' : '+', e < 0 ? -e : e);
        sb_puts(b, buf);
    }
}

void jv_stringify(const jv *v, sb *b) {
    if (!v) return;
    switch (v->kind) {
        case JV_UNDEF: return;
        case JV_NULL: sb_puts(b, "null"); return;
        case JV_FALSE: sb_puts(b, "false"); return;
        case JV_TRUE: sb_puts(b, "true"); return;
        case JV_NUM:
            if (isnan(v->num) || isinf(v->num)) sb_puts(b, "null");
            else js_number(b, v->num);
            return;
        case JV_STR: js_quote(b, v->s, v->slen); return;
        case JV_ARR:
            sb_putc(b, '[');
            for (int i = 0; i < v->n; i++) {
                if (i) sb_putc(b, ',');
                if (v->vals[i] == NULL || v->vals[i]->kind == JV_UNDEF) sb_puts(b, "null");
                else jv_stringify(v->vals[i], b);
            }
            sb_putc(b, ']');
            return;
        case JV_OBJ: {
            int *ord = (int *)malloc(sizeof(int) * (size_t)(v->n + 1));
            int n = jv_obj_enum(v, ord), first = 1;
            sb_putc(b, '{');
            for (int i = 0; i < n; i++) {
                const jv *x = v->vals[ord[i]];
                if (!x || x->kind == JV_UNDEF) continue;
                if (!first) sb_putc(b, ',');
                first = 0;
                js_quote(b, v->keys[ord[i]], v->klens[ord[i]]);
                sb_putc(b, ':');
                jv_stringify(x, b);
            }
            sb_putc(b, '}');
            free(ord);
            return;
        }
    }
}

/* ------------------------------------------------------------------ parse */
typedef struct { const char *p, *e; int err; } ps;

static void ws(ps *s) {
    while (s->p < s->e && (*s->p == ' ' || *s->p == '\t' || *s->p == '\n' || *s->p == '\r')) s->p++;
}

static uint32_t utf8_next(ps *s) {
    const unsigned char *q = (const unsigned char *)s->p;
    uint32_t c = q[0];
    int len = 1;
    if (c < 0x80) { s->p++; return c; }
    if ((c & 0xE0) == 0xC0) { len = 2; c &= 0x1F; }
    else if ((c & 0xF0) == 0xE0) { len = 3; c &= 0x0F; }
    else if ((c & 0xF8) == 0xF0) { len = 4; c &= 0x07; }
    else { s->p++; return 0xFFFD; }
    if (s->p + len > s->e) { s->p = s->e; return 0xFFFD; }
    for (int i = 1; i < len; i++) {
        if ((q[i] & 0xC0) != 0x80) { s->p += i; return 0xFFFD; }
        c = (c << 6) | (q[i] & 0x3F);
    }
    s->p += len;
    return c;
}

typedef struct { u16 *p; int n, cap; } u16buf;
static void u16_push(u16buf *b, u16 c) {
    if (b->n == b->cap) {
        b->cap = b->cap ? b->cap * 2 : 16;
        b->p = (u16 *)realloc(b->p, sizeof(u16) * (size_t)b->cap);
    }
    b->p[b->n++] = c;
}

static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

static int parse_string(ps *s, u16buf *out) {
    if (s->p >= s->e || *s->p != '"') return 0;
    s->p++;
    while (s->p < s->e) {
        char c = *s->p;
        if (c == '"') { s->p++; return 1; }
        if (c == '\\') {
            s->p++;
            if (s->p >= s->e) return 0;
            char t = *s->p++;
            switch (t) {
                case '"': u16_push(out, '"'); break;
                case '\\': u16_push(out, '\\'); break;
                case '/': u16_push(out, '/'); break;
                case 'b': u16_push(out, 8); break;
                case 'f': u16_push(out, 12); break;
                case 'n': u16_push(out, 10); break;
                case 'r': u16_push(out, 13); break;
                case 't': u16_push(out, 9); break;
                case 'u': {
                    if (s->p + 4 > s->e) return 0;
                    int v = 0;
                    for (int i = 0; i < 4; i++) {
                        int h = hexv(s->p[i]);
                        if (h < 0) return 0;
                        v = v * 16 + h;
                    }
                    s->p += 4;
                    u16_push(out, (u16)v);
                    break;
                }
                default: return 0;
            }
            continue;
        }
        if ((unsigned char)c < 0x20) return 0;
        uint32_t cp = utf8_next(s);
        if (cp >= 0x10000) {
            cp -= 0x10000;
            u16_push(out, (u16)(0xD800 + (cp >> 10)));
            u16_push(out, (u16)(0xDC00 + (cp & 0x3FF)));
        } else {
            u16_push(out, (u16)cp);
        }
    }
    return 0;
}

static jv *parse_value(ps *s, int depth);

static jv *parse_value(ps *s, int depth) {
    if (depth > 512) { s->err = 1; return NULL; }
    ws(s);
    if (s->p >= s->e) { s->err = 1; return NULL; }
    char c = *s->p;
    if (c == '{') {
        s->p++;
        jv *o = jv_new(JV_OBJ);
        ws(s);
        if (s->p < s->e && *s->p == '}') { s->p++; return o; }
        for (;;) {
            ws(s);
            u16buf k = {0, 0, 0};
            if (!parse_string(s, &k)) { free(k.p); s->err = 1; jv_unref(o); return NULL; }
            ws(s);
            if (s->p >= s->e || *s->p != ':') { free(k.p); s->err = 1; jv_unref(o); return NULL; }
            s->p++;
            jv *v = parse_value(s, depth + 1);
            if (!v) { free(k.p); jv_unref(o); return NULL; }
            jv_obj_set(o, k.p, k.n, v);
            free(k.p);
            ws(s);
            if (s->p < s->e && *s->p == ',') { s->p++; continue; }
            if (s->p < s->e && *s->p == '}') { s->p++; return o; }
            s->err = 1;
            jv_unref(o);
            return NULL;
        }
    }
    if (c == '[') {
        s->p++;
        jv *a = jv_new(JV_ARR);
        ws(s);
        if (s->p < s->e && *s->p == ']') { s->p++; return a; }
        for (;;) {
            jv *v = parse_value(s, depth + 1);
            if (!v) { jv_unref(a); return NULL; }
            jv_reserve(a, 1);
            a->vals[a->n++] = v;
            ws(s);
            if (s->p < s->e && *s->p == ',') { s->p++; continue; }
            if (s->p < s->e && *s->p == ']') { s->p++; return a; }
            s->err = 1;
            jv_unref(a);
            return NULL;
        }
    }
    if (c == '"') {
        u16buf b = {0, 0, 0};
        if (!parse_string(s, &b)) { free(b.p); s->err = 1; return NULL; }
        jv *v = jv_new_str(b.p, b.n);
        free(b.p);
        return v;
    }
    if (c == 't' && s->e - s->p >= 4 && !strncmp(s->p, "true", 4)) { s->p += 4; return jv_new(JV_TRUE); }
    if (c == 'f' && s->e - s->p >= 5 && !strncmp(s->p, "false", 5)) { s->p += 5; return jv_new(JV_FALSE); }
    if (c == 'n' && s->e - s->p >= 4 && !strncmp(s->p, "null", 4)) { s->p += 4; return jv_new(JV_NULL); }
    if (c == '-' || (c >= '0' && c <= '9')) {
        char buf[400];
        size_t n = 0;
        while (s->p < s->e && n < sizeof(buf) - 1 &&
               (strchr("+-0123456789.eE", *s->p) != NULL)) buf[n++] = *s->p++;
        buf[n] = 0;
        char *end;
        double d = strtod(buf, &end);
        if (end != buf + n) { s->err = 1; return NULL; }
        return jv_new_num(d);
    }
    s->err = 1;
    return NULL;
}

jv *jv_parse(const char *text, size_t len) {
    ps s = {text, text + len, 0};
    jv *v = parse_value(&s, 0);
    if (!v) return NULL;
    ws(&s);
    if (s.p != s.e) { jv_unref(v); return NULL; }
    return v;
}

/* ------------------------------------------------------------------ matchProperties */
/* property read `v[key]` for the value kinds JSON can produce (own properties only) */
static const jv *js_get(const jv *v, const u16 *k, int kl, jv **tmp) {
    static const u16 LENGTH[6] = {'l', 'e', 'n', 'g', 't', 'h'};
    uint32_t idx;
    *tmp = NULL;
    if (!v) return NULL;
    switch (v->kind) {
        case JV_OBJ: return jv_obj_get(v, k, kl);
        case JV_ARR:
            if (js_is_array_index(k, kl, &idx)) return idx < (uint32_t)v->n ? v->vals[idx] : NULL;
            if (u16_eq(k, kl, LENGTH, 6)) return (*tmp = jv_new_num(v->n));
            return NULL;
        case JV_STR:
            if (js_is_array_index(k, kl, &idx)) return idx < (uint32_t)v->slen ? (*tmp = jv_new_str(v->s + idx, 1)) : NULL;
            if (u16_eq(k, kl, LENGTH, 6)) return (*tmp = jv_new_num(v->slen));
            return NULL;
        default: return NULL;
    }
}

static int js_truthy(const jv *v) {
    if (!v) return 0;
    switch (v->kind) {
        case JV_UNDEF: case JV_NULL: case JV_FALSE: return 0;
        case JV_NUM: return !(v->num == 0 || isnan(v->num));
        case JV_STR: return v->slen > 0;
        default: return 1;
    }
}

int jv_truthy(const jv *v) { return js_truthy(v); }

/* a fresh copy of a parsed value (what JSON.parse of the same text returns): objects and arrays
   are new objects, primitives are immutable and shared */
jv *jv_deep_clone(const jv *v) {
    if (!v) return NULL;
    if (v->kind == JV_ARR) {
        jv *a = jv_new(JV_ARR);
        jv_reserve(a, v->n);
        for (int i = 0; i < v->n; i++) a->vals[i] = jv_deep_clone(v->vals[i]);
        a->n = v->n;
        return a;
    }
    if (v->kind == JV_OBJ) {
        jv *o = jv_new(JV_OBJ);
        for (int i = 0; i < v->n; i++) jv_obj_set(o, v->keys[i], v->klens[i], jv_deep_clone(v->vals[i]));
        return o;
    }
    return jv_ref((jv *)v);
}

static int js_typeof_object(const jv *v) {
    return v && (v->kind == JV_OBJ || v->kind == JV_ARR || v->kind == JV_NULL);
}

static int js_strict_eq(const jv *a, const jv *b) {
    if (!a || !b) return a == b || ((!a || a->kind == JV_UNDEF) && (!b || b->kind == JV_UNDEF));
    if (a->kind != b->kind) return 0;
    switch (a->kind) {
        case JV_UNDEF: case JV_NULL: case JV_TRUE: case JV_FALSE: return 1;
        case JV_NUM: return a->num == b->num;
        case JV_STR: return u16_eq(a->s, a->slen, b->s, b->slen);
        default: return a == b; /* object identity */
    }
}

/* enumerate `for (key in v)` keys into a temporary list */
typedef struct { u16 **k; int *kl; int n; u16 *store; } keylist;
static void for_in_keys(const jv *v, keylist *kl) {
    kl->n = 0; kl->k = NULL; kl->kl = NULL; kl->store = NULL;
    if (!v) return;
    if (v->kind == JV_OBJ) {
        int *ord = (int *)malloc(sizeof(int) * (size_t)(v->n + 1));
        int n = jv_obj_enum(v, ord);
        kl->k = (u16 **)malloc(sizeof(u16 *) * (size_t)(n + 1));
        kl->kl = (int *)malloc(sizeof(int) * (size_t)(n + 1));
        for (int i = 0; i < n; i++) { kl->k[i] = v->keys[ord[i]]; kl->kl[i] = v->klens[ord[i]]; }
        kl->n = n;
        free(ord);
    } else if (v->kind == JV_ARR || v->kind == JV_STR) {
        int n = v->kind == JV_ARR ? v->n : v->slen;
        kl->k = (u16 **)malloc(sizeof(u16 *) * (size_t)(n + 1));
        kl->kl = (int *)malloc(sizeof(int) * (size_t)(n + 1));
        kl->store = (u16 *)malloc(sizeof(u16) * 11 * (size_t)(n + 1));
        for (int i = 0; i < n; i++) {
            char t[12];
            int m = snprintf(t, sizeof t, "%d", i);
            u16 *dst = kl->store + 11 * i;
            for (int j = 0; j < m; j++) dst[j] = (u16)t[j];
            kl->k[i] = dst;
            kl->kl[i] = m;
        }
        kl->n = n;
    }
}
static void keylist_free(keylist *kl) { free(kl->k); free(kl->kl); free(kl->store); }

int jv_match_properties(const jv *a, const jv *b) {
    if (js_truthy(a)) {
        if (!js_truthy(b)) return 0;
        keylist ka;
        for_in_keys(a, &ka);
        int ok = 1;
        for (int i = 0; ok && i < ka.n; i++) {
            jv *t1, *t2;
            const jv *bv = js_get(b, ka.k[i], ka.kl[i], &t1);
            const jv *av = js_get(a, ka.k[i], ka.kl[i], &t2);
            if (!bv || bv->kind == JV_UNDEF) ok = 0;
            else if (js_typeof_object(bv)) { if (!jv_match_properties(av, bv)) ok = 0; }
            else if (!js_strict_eq(bv, av)) ok = 0;
            jv_unref(t1);
            jv_unref(t2);
        }
        keylist_free(&ka);
        if (!ok) return 0;
        keylist kb;
        for_in_keys(b, &kb);
        for (int i = 0; ok && i < kb.n; i++) {
            jv *t;
            const jv *av = js_get(a, kb.k[i], kb.kl[i], &t);
            if (!av || av->kind == JV_UNDEF) ok = 0;
            jv_unref(t);
        }
        keylist_free(&kb);
        return ok;
    }
    return js_truthy(b) ? 0 : 1;
}
