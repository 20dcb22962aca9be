/*
 * jsv.h — JSON values with JavaScript semantics, for the test oracle.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/README.md): nothing in the product
 * links this.  It restates the pieces of V8 behaviour the merge-tree path
 * depends on:
 *   - JSON.parse / JSON.stringify byte output (snapshotChunks.ts:122-131 emits
 *     JSON.stringify(chunk)), incl. well-formed escaping of lone surrogates and
 *     Number::toString formatting;
 *   - ordinary-object key enumeration order (integer indices ascending, then
 *     string keys in insertion order), which fixes the order of `props` keys;
 *   - Properties.matchProperties (merge-tree/src/properties.ts:62-93).
 * Strings are UTF-16 code units, as in JS.
 */
#ifndef MT_JSV_H
#define MT_JSV_H

#include <stddef.h>
#include <stdint.h>

typedef uint16_t u16;

enum { JV_UNDEF = 0, JV_NULL, JV_FALSE, JV_TRUE, JV_NUM, JV_STR, JV_ARR, JV_OBJ };

typedef struct jv {
    int kind;
    int rc;
    double num;
    u16 *s; /* JV_STR */
    int slen;
    int n, cap;     /* JV_ARR / JV_OBJ */
    struct jv **vals;
    u16 **keys;     /* JV_OBJ, insertion order */
    int *klens;
} jv;

/* growable UTF-8 byte buffer */
typedef struct sb {
    char *p;
    size_t n, cap;
} sb;

void sb_init(sb *b);
void sb_free(sb *b);
void sb_putc(sb *b, char c);
void sb_puts(sb *b, const char *s);
void sb_putn(sb *b, const char *s, size_t n);
void sb_put_u16_utf8(sb *b, const u16 *s, int n); /* raw text (lone surrogates -> U+FFFD) */

jv *jv_new(int kind);
jv *jv_new_num(double d);
jv *jv_new_str(const u16 *s, int n);
jv *jv_new_str_ascii(const char *s);
jv *jv_ref(jv *v);
void jv_unref(jv *v);

/* parse UTF-8 JSON text; returns NULL on error */
jv *jv_parse(const char *text, size_t len);
/* JSON.stringify(v) appended to b (undefined -> nothing) */
void jv_stringify(const jv *v, sb *b);
void js_quote(sb *b, const u16 *s, int n);  /* JSON string literal */
void js_number(sb *b, double d);            /* Number::toString(10) */

/* objects */
jv *jv_obj_get(const jv *o, const u16 *k, int kl);
jv *jv_obj_get_ascii(const jv *o, const char *k);
void jv_obj_set(jv *o, const u16 *k, int kl, jv *v); /* steals a reference to v */
void jv_obj_set_ascii(jv *o, const char *k, jv *v);
int jv_obj_del(jv *o, const u16 *k, int kl);
/* fills order[0..n) with indices of o's keys in JS enumeration order; returns n */
int jv_obj_enum(const jv *o, int *order);
/* shallow copy of an object (values shared) */
jv *jv_obj_clone(const jv *o);
/* 1 if key is a canonical array index (0 .. 2^32-2) */
int js_is_array_index(const u16 *k, int kl, uint32_t *idx);

/* JS ToBoolean; NULL stands for undefined */
int jv_truthy(const jv *v);
/* JSON.parse(JSON text of v) for parsed values: new objects / arrays, primitives shared */
jv *jv_deep_clone(const jv *v);

/* Properties.matchProperties(a, b); NULL stands for undefined */
int jv_match_properties(const jv *a, const jv *b);

int u16_eq(const u16 *a, int an, const u16 *b, int bn);

#endif
