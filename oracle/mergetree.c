/*
 * mergetree.c — CPU restatement of merge-tree observer replay (TEST INFRASTRUCTURE ONLY).
 *
 * Follows packages/dds/merge-tree/src (reference v0.29.0) structure-for-structure:
 * an explicit B-tree of MergeBlocks (MaxNodesInBlock = 8, mergeTree.ts:334) whose
 * leaves are TextSegment / Marker objects.  The one deliberate substitution:
 * PartialSequenceLengths (partialLengths.ts) is replaced by the exact leaf sum of
 * nodeLength() under the same (refSeq, clientId) view — the quantity the partial
 * lengths cache (partialLengths.ts:433-487; see DESIGN.md "Block lengths").
 *
 * Scope: the passive-observer path (every op remote, client.ts:797-819) plus the
 * non-collaborating local edit path that the reference's golden SnapshotV1 files
 * were generated with (sequence/src/test/generateSharedStrings.ts:24-97).
 */
#include <limits.h>
#include <math.h>
#include <pthread.h>
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "jsv.h"
#include "mt_oracle.h"

/* constants.ts:11-15 */
#define UNIVERSAL_SEQ 0
#define UNASSIGNED_SEQ (-1)
#define TREE_MAINT_SEQ (-2)
#define LOCAL_CLIENT (-1)
#define NONCOLLAB_CLIENT (-2)
/* mergeTree.ts:334, 1059, 1061 */
#define MAX_NODES 8
#define TEXT_GRANULARITY 256
#define ZAMBONI_MAX 2

#define SCOUR_UNDEF (-1)
#define SCOUR_FALSE 0
#define SCOUR_TRUE 1

enum { SEG_TEXT = 0, SEG_MARKER = 1 };

typedef struct Block Block;
struct Seg;

/* HierMergeBlock.rangeStacks (mergeTree.ts:49, 2755): String(label) -> Stack<ReferencePosition>, in
   key creation order (each stack bottom to top) */
typedef struct RStack {
    unsigned short *key;
    int klen;
    struct Seg **items;
    int n, cap;
} RStack;
struct RangeMap {
    RStack *s;
    int n, cap;
};

typedef struct Node {
    int is_leaf;
    Block *parent;
    int index;
    int cached_length;
} Node;

struct Block { /* MergeBlock / HierMergeBlock, mergeTree.ts:336-420 */
    Node n;
    int child_count;
    Node *children[MAX_NODES];
    int needs_scour; /* undefined / true / false (mergeTree.ts:63, 1279, 1438) */
    /* upper bounds of the seq / removedSeq of every leaf below (UnassignedSequenceNumber counts as
       +inf): a view with refSeq at or above both sees exactly cachedLength (block_partial_length) */
    int max_seq, max_rseq;
    Block *all_next;
    struct mto_doc *doc; /* for blockUpdate's marker-id bookkeeping (addNodeReferences) */
    /* HierMergeBlock.rightmostTiles / leftmostTiles (mergeTree.ts:386-399): String(label) -> the
       marker, rebuilt by every blockUpdate from the children (addNodeReferences, 263-318) */
    struct TileMap {
        u16 **keys;
        int *klens;
        struct Seg **segs;
        int n, cap;
    } rt, lt;
    struct RangeMap rs; /* rangeStacks, rebuilt by the same blockUpdate */
};

typedef struct Group Group;

typedef struct Seg { /* BaseSegment, mergeTree.ts:429-573 */
    Node n;
    int kind;
    u16 *text; /* TextSegment.text; length == n.cached_length */
    int tcap;
    int ref_type; /* Marker.refType */
    int seq;
    int client_id;
    int removed; /* removedSeq !== undefined */
    int removed_seq;
    int removed_client;
    int *ovl; /* removedClientOverlap, push order */
    int novl, covl;
    jv *props; /* properties (NULL = undefined) */
    struct Seg *all_next;
    const jv *id_jv; /* marker id value last mapped (id_idx: its idToSegment entry) */
    int id_idx;
    /* local-client state (mergeTree.ts:441-448): localSeq / localRemovedSeq (0 = undefined), the
       segment's SegmentGroupCollection (a FIFO of the pending groups holding it,
       segmentGroupCollection.ts:9-40) and SegmentPropertiesManager's pending counts
       (segmentPropertiesManager.ts:12-14; pend_keys is created with props, NULL = undefined) */
    int local_seq, local_removed_seq;
    Group **sg;
    int sg_head, sg_n, sg_cap;
    jv *pend_keys;
    int pend_rewrite;
} Seg;

struct Group { /* SegmentGroup (mergeTree.ts:198-201): { segments, localSeq } */
    Seg **segs;
    int n, cap;
    int local_seq;
    Group *all_next;
};

typedef struct { /* LRUSegment, mergeTree.ts:918-926 */
    Seg *seg;
    int max_seq;
} HeapEnt;

struct mto_tables {
    char **keys;
    u16 **keys16;
    int *keylen16;
    int n_keys;
    jv **values;
    int n_values;
};

/* a consensus ack's min-seq listener (MergeTree.addMinSeqListener, mergeTree.ts:1701-1707): the
   closure holds the consensusInfo pendingConsensus gave at the ack (marker NULL: undefined) */
typedef struct {
    int min_required;
    char *key; /* the marker id's JSON text */
    Seg *marker;
} ConsLis;

struct mto_doc {
    Block *root;
    struct {
        int client_id, collaborating, min_seq, current_seq;
    } cw; /* CollaborationWindow, mergeTree.ts:822-839 */
    HeapEnt *heap; /* Heap.L, collections.ts:213-265; heap[0] is the min sentinel */
    int hn, hcap;
    char **long_ids; /* shortClientIdMap (client.ts:70) */
    int n_ids, cap_ids;
    char *long_client_id;
    Seg *all_segs;
    Block *all_blocks;
    int status;
    char err[256];
    jmp_buf jb;
    int jb_armed;
    /* SnapshotV1 output */
    char **blob_names;
    sb *blobs;
    int n_blobs;
    /* packed-op client index -> short id cache */
    int pk_map[MT_MAX_CLIENTS + 2];
    /* MergeTree.idToSegment (mergeTree.ts:1098): String(markerId) -> marker */
    u16 **id_keys;
    int *id_klens;
    Seg **id_segs;
    int n_ids_map, cap_ids_map;
    int *id_hash; /* open addressing over id_keys (index + 1, 0 empty), id_hcap slots */
    int id_hcap;
    /* packed MT_OP_RELPOS: resolved positions for the next record (bit 0 pos1, bit 1 pos2) */
    int rel_pending, rel_pos1, rel_pos2;
    /* a Tile marker whose referenceTileLabels is not an array / string (for-of would throw in
       blockUpdate): tile queries report MTO_UNSUPPORTED */
    int tile_bad;
    /* the same for a NestBegin / NestEnd marker's referenceRangeLabels: getStackContext reports
       MTO_UNSUPPORTED */
    int range_bad;
    /* local-client path: collabWindow.localSeq (mergeTree.ts:831) and MergeTree.pendingSegments,
       the FIFO of SegmentGroups awaiting their ack (mergeTree.ts:1093, 1261) */
    int local_seq;
    Group **pend;
    int pend_head, pend_n, pend_cap;
    Group *all_groups;
    /* regeneratePendingOp outputs (JSON ops): the current reset message's ops, and every finished
       message's op (or group op), comma separated */
    sb regen_cur, regen_all;
    int regen_cur_n, regen_all_n;
    /* Client.pendingConsensus (client.ts:66): marker id (its JSON text) -> the marker it was
       registered with; MergeTree.minSeqListeners (mergeTree.ts:1101), a Heap with cons_lis[0] the
       min sentinel and n_lis members; the callbacks made ([{markerId, seq, minSeq}], comma joined);
       a packed notify RELPOS's id and marker for the local annotate after it */
    char **cons_keys;
    Seg **cons_marks;
    int n_cons, cap_cons;
    ConsLis *cons_lis;
    int n_lis, cap_lis;
    sb cons_events;
    int cons_events_n;
    char *ntf_key;
    Seg *ntf_marker;
};

/* ------------------------------------------------------------------ errors */
static void fail(mto_doc *d, int code, const char *fmt, ...) {
    if (d->status == MTO_OK) {
        d->status = code;
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(d->err, sizeof d->err, fmt, ap);
        va_end(ap);
    }
    if (d->jb_armed) longjmp(d->jb, 1);
}

/* ------------------------------------------------------------------ alloc */
static Block *make_block(mto_doc *d, int child_count) { /* MergeTree.makeBlock, mergeTree.ts:1114 */
    Block *b = (Block *)calloc(1, sizeof(Block));
    b->n.is_leaf = 0;
    b->child_count = child_count;
    b->needs_scour = SCOUR_UNDEF;
    b->max_seq = b->max_rseq = INT_MAX; /* unknown until block_update */
    b->doc = d;
    b->all_next = d->all_blocks;
    d->all_blocks = b;
    return b;
}

static Seg *new_seg(mto_doc *d, int kind) {
    Seg *s = (Seg *)calloc(1, sizeof(Seg));
    s->n.is_leaf = 1;
    s->kind = kind;
    s->seq = UNIVERSAL_SEQ;     /* BaseSegment.seq default, mergeTree.ts:434 */
    s->client_id = LOCAL_CLIENT; /* BaseSegment.clientId default, mergeTree.ts:433 */
    s->all_next = d->all_segs;
    d->all_segs = s;
    return s;
}

static Seg *new_text_seg(mto_doc *d, const u16 *t, int n) { /* TextSegment ctor, textSegment.ts:44-47 */
    Seg *s = new_seg(d, SEG_TEXT);
    s->tcap = n > 8 ? n : 8;
    s->text = (u16 *)malloc(sizeof(u16) * (size_t)s->tcap);
    if (n) memcpy(s->text, t, sizeof(u16) * (size_t)n);
    s->n.cached_length = n;
    return s;
}

static Seg *new_marker(mto_doc *d, int ref_type) { /* Marker ctor, mergeTree.ts:647-650 */
    Seg *s = new_seg(d, SEG_MARKER);
    s->ref_type = ref_type;
    s->n.cached_length = 1;
    return s;
}

static void seg_text_append(Seg *s, const u16 *t, int n) {
    int len = s->n.cached_length;
    if (len + n > s->tcap) {
        int c = s->tcap ? s->tcap : 8;
        while (c < len + n) c *= 2;
        s->text = (u16 *)realloc(s->text, sizeof(u16) * (size_t)c);
        s->tcap = c;
    }
    memcpy(s->text + len, t, sizeof(u16) * (size_t)n);
    s->n.cached_length = len + n;
}

static void assign_child(Block *b, Node *child, int index) { /* MergeBlock.assignChild, mergeTree.ts:375 */
    child->parent = b;
    child->index = index;
    b->children[index] = child;
}

/* ------------------------------------------------------------------ lengths */
static int local_net_length(const Seg *s) { /* mergeTree.ts:1161-1172 (single branch) */
    return s->removed ? 0 : s->n.cached_length;
}

static int node_total_length(const Node *n) { /* mergeTree.ts:422-427 */
    return n->is_leaf ? local_net_length((const Seg *)n) : n->cached_length;
}

static int seq_bound(int seq) { return seq == UNASSIGNED_SEQ ? INT_MAX : seq; }
static void map_marker_id(mto_doc *d, Seg *s);
static void block_update_tiles(Block *b);
static void block_update(Block *b) { /* mergeTree.ts:2748-2768 (cachedLength part) */
    int len = 0, ms = INT_MIN, mr = INT_MIN;
    for (int i = 0; i < b->child_count; i++) {
        Node *c = b->children[i];
        len += node_total_length(c);
        /* addNodeReferences (mergeTree.ts:270-285): a marker with localNetLength > 0 re-maps its id */
        if (c->is_leaf && local_net_length((const Seg *)c) > 0 && b->doc) map_marker_id(b->doc, (Seg *)c);
        if (c->is_leaf) {
            const Seg *sg = (const Seg *)c;
            if (seq_bound(sg->seq) > ms) ms = seq_bound(sg->seq);
            if (sg->removed && seq_bound(sg->removed_seq) > mr) mr = seq_bound(sg->removed_seq);
        } else {
            const Block *cb = (const Block *)c;
            if (cb->max_seq > ms) ms = cb->max_seq;
            if (cb->max_rseq > mr) mr = cb->max_rseq;
        }
    }
    b->n.cached_length = len;
    b->max_seq = ms;
    b->max_rseq = mr;
    block_update_tiles(b);
}
/* raise the bounds on the path above a leaf whose seq / removedSeq was just set */
static void bump_bounds(Seg *s) {
    const int q = seq_bound(s->seq), r = s->removed ? seq_bound(s->removed_seq) : INT_MIN;
    for (Block *b = s->n.parent; b; b = b->n.parent) {
        if (q > b->max_seq) b->max_seq = q;
        if (r > b->max_rseq) b->max_rseq = r;
    }
}

static int seg_has_overlap(const Seg *s, int client) {
    for (int i = 0; i < s->novl; i++)
        if (s->ovl[i] == client) return 1;
    return 0;
}

static int node_length(mto_doc *d, Node *node, int ref_seq, int client_id);

/* PartialSequenceLengths.getPartialLength substitute: exact leaf sum of nodeLength.  A subtree
   whose every seq and removedSeq is at or below refSeq is seen exactly as the local view sees it
   (visible, or removed), so its cachedLength is that sum (MTO_SLOW_LENGTHS=1 always recurses:
   tests/test_oracle_golden.py checks both agree). */
static int slow_lengths = -1;
static int block_partial_length(mto_doc *d, Block *b, int ref_seq, int client_id) {
    if (slow_lengths < 0) slow_lengths = getenv("MTO_SLOW_LENGTHS") != NULL;
    if (!slow_lengths && b->max_seq <= ref_seq && b->max_rseq <= ref_seq) return b->n.cached_length;
    int len = 0;
    for (int i = 0; i < b->child_count; i++) len += node_length(d, b->children[i], ref_seq, client_id);
    return len;
}

static int node_length(mto_doc *d, Node *node, int ref_seq, int client_id) { /* mergeTree.ts:1659-1699 */
    if (!d->cw.collaborating || d->cw.client_id == client_id) {
        if (!node->is_leaf) return node->cached_length;
        return local_net_length((Seg *)node);
    }
    if (!node->is_leaf) return block_partial_length(d, (Block *)node, ref_seq, client_id);
    Seg *s = (Seg *)node;
    if (s->client_id == client_id || (s->seq != UNASSIGNED_SEQ && s->seq <= ref_seq)) {
        if (s->removed) {
            if (s->removed_client == client_id || seg_has_overlap(s, client_id) ||
                (s->removed_seq != UNASSIGNED_SEQ && s->removed_seq <= ref_seq))
                return 0;
            return s->n.cached_length;
        }
        return s->n.cached_length;
    }
    return 0;
}

static int block_length(mto_doc *d, Block *b, int ref_seq, int client_id) { /* mergeTree.ts:1636-1642 */
    if (d->cw.collaborating && client_id != d->cw.client_id) return block_partial_length(d, b, ref_seq, client_id);
    return b->n.cached_length;
}

/* blockUpdateLength / nodeUpdateLengthNewStructure / blockUpdatePathLengths
   (mergeTree.ts:2721, 2770, 2781): with partial lengths substituted, only the
   local-view cachedLength needs maintenance. */
static void block_update_length(Block *b) { block_update(b); }
static void node_update_length_new_structure(Block *b) { block_update(b); }
static void block_update_path_lengths(Block *b) {
    while (b) {
        node_update_length_new_structure(b);
        b = b->n.parent;
    }
}

/* ------------------------------------------------------------------ heap (collections.ts:213-265) */
static int heap_count(mto_doc *d) { return d->hn - 1; }
static void heap_push_raw(mto_doc *d, HeapEnt e) {
    if (d->hn == d->hcap) {
        d->hcap = d->hcap ? d->hcap * 2 : 64;
        d->heap = (HeapEnt *)realloc(d->heap, sizeof(HeapEnt) * (size_t)d->hcap);
    }
    d->heap[d->hn++] = e;
}
static void heap_init(mto_doc *d) {
    d->hn = 0;
    HeapEnt min = {NULL, -2}; /* LRUSegmentComparer.min = { maxSeq: -2 } */
    heap_push_raw(d, min);
}
static int heap_cmp(const HeapEnt *a, const HeapEnt *b) { return a->max_seq - b->max_seq; }
static void heap_fixup(mto_doc *d, int k) {
    while (k > 1 && heap_cmp(&d->heap[k >> 1], &d->heap[k]) > 0) {
        HeapEnt t = d->heap[k >> 1];
        d->heap[k >> 1] = d->heap[k];
        d->heap[k] = t;
        k >>= 1;
    }
}
static void heap_fixdown(mto_doc *d, int k) {
    while ((k << 1) <= heap_count(d)) {
        int j = k << 1;
        if (j < heap_count(d) && heap_cmp(&d->heap[j], &d->heap[j + 1]) > 0) j++;
        if (heap_cmp(&d->heap[k], &d->heap[j]) <= 0) break;
        HeapEnt t = d->heap[k];
        d->heap[k] = d->heap[j];
        d->heap[j] = t;
        k = j;
    }
}
static void heap_add(mto_doc *d, Seg *s, int max_seq) {
    HeapEnt e = {s, max_seq};
    heap_push_raw(d, e);
    heap_fixup(d, heap_count(d));
}
static HeapEnt *heap_peek(mto_doc *d) { return heap_count(d) >= 1 ? &d->heap[1] : NULL; }
static HeapEnt heap_get(mto_doc *d) {
    HeapEnt x = d->heap[1];
    d->heap[1] = d->heap[heap_count(d)];
    d->hn--;
    heap_fixdown(d, 1);
    return x;
}

/* ------------------------------------------------------------------ properties */
/* A combiningOp other than "rewrite" (include/mt_oplog.h mt_combine_kind) */
typedef struct {
    int kind;      /* MT_COMBINE_INCR / _CONSENSUS / _OTHER */
    jv *def, *min; /* combiningOp.defaultValue / .minValue (the op's own objects); NULL = undefined */
} CombineOp;

/* growable UTF-16 buffer */
typedef struct {
    u16 *p;
    int n, cap;
} u16buf;
static void ub_put(u16buf *b, const u16 *s, int n) {
    if (b->n + n > b->cap) {
        b->cap = (b->n + n) * 2 + 16;
        b->p = (u16 *)realloc(b->p, sizeof(u16) * (size_t)b->cap);
    }
    if (n) memcpy(b->p + b->n, s, sizeof(u16) * (size_t)n);
    b->n += n;
}
static void ub_ascii(u16buf *b, const char *s) {
    while (*s) {
        u16 c = (u16)(unsigned char)*s++;
        ub_put(b, &c, 1);
    }
}
/* String(v) of a JSON-parsed value: Number::toString, "[object Object]" for a plain object,
   Array.prototype.join(",") for an array (null / undefined elements -> "") */
static void js_to_string(const jv *v, u16buf *b) {
    if (!v || v->kind == JV_UNDEF) { ub_ascii(b, "undefined"); return; }
    switch (v->kind) {
        case JV_NULL: ub_ascii(b, "null"); return;
        case JV_TRUE: ub_ascii(b, "true"); return;
        case JV_FALSE: ub_ascii(b, "false"); return;
        case JV_NUM: {
            sb t;
            sb_init(&t);
            js_number(&t, v->num);
            sb_putc(&t, 0);
            ub_ascii(b, t.p);
            sb_free(&t);
            return;
        }
        case JV_STR: ub_put(b, v->s, v->slen); return;
        case JV_OBJ: ub_ascii(b, "[object Object]"); return;
        default:
            for (int i = 0; i < v->n; i++) {
                if (i) ub_ascii(b, ",");
                const jv *e = v->vals[i];
                if (e && e->kind != JV_UNDEF && e->kind != JV_NULL) js_to_string(e, b);
            }
    }
}
/* `v += undefined` (properties.ts:34): ToPrimitive(v) is a string for strings, objects and
   arrays (string concatenation), else both sides go through ToNumber and undefined is NaN */
static jv *js_plus_undefined(const jv *v) {
    if (!v || v->kind == JV_UNDEF || v->kind == JV_NULL || v->kind == JV_TRUE || v->kind == JV_FALSE ||
        v->kind == JV_NUM)
        return jv_new_num(NAN);
    u16buf b = {NULL, 0, 0};
    js_to_string(v, &b);
    ub_ascii(&b, "undefined");
    jv *r = jv_new_str(b.p, b.n);
    free(b.p);
    return r;
}
/* `a < b` with a = js_plus_undefined's result (properties.ts:36): a is NaN or a string ending in
   "undefined", whose ToNumber is NaN, so only a string-to-string comparison (b a string, or an
   object / array whose ToPrimitive is its String()) can hold: UTF-16 code-unit order */
static int js_less_combined(const jv *a, const jv *b) {
    if (a->kind != JV_STR || !b || (b->kind != JV_STR && b->kind != JV_OBJ && b->kind != JV_ARR)) return 0;
    u16buf t = {NULL, 0, 0};
    js_to_string(b, &t);
    int n = a->slen < t.n ? a->slen : t.n, lt = a->slen < t.n;
    for (int i = 0; i < n; i++)
        if (a->s[i] != t.p[i]) {
            lt = a->s[i] < t.p[i];
            break;
        }
    free(t.p);
    return lt;
}
/* Properties.combine(combiningInfo, currentValue, newValue, seq) (properties.ts:26-60) with
   newValue undefined: segmentPropertiesManager.ts:98 passes its local `newValue`, not
   newProps[key].  Returns a new reference, NULL for undefined.  A consensus value object with
   seq === -1 is updated in place, so every segment sharing that object sees the new seq. */
static jv *js_combine(mto_doc *d, const CombineOp *co, jv *cur, int seq) {
    jv *cv = (cur && cur->kind != JV_UNDEF) ? cur : co->def;
    if (cv && cv->kind == JV_UNDEF) cv = NULL;
    switch (co->kind) {
        case MT_COMBINE_INCR: {
            jv *r = js_plus_undefined(cv);
            if (co->min && jv_truthy(co->min) && js_less_combined(r, co->min)) {
                jv_unref(r);
                r = jv_ref(co->min);
            }
            return r;
        }
        case MT_COMBINE_CONSENSUS:
            if (!cv) {
                jv *o = jv_new(JV_OBJ); /* { value: newValue, seq } */
                jv_obj_set_ascii(o, "value", jv_new(JV_UNDEF));
                jv_obj_set_ascii(o, "seq", jv_new_num(seq));
                return o;
            }
            if (cv->kind == JV_NULL) fail(d, MTO_UNSUPPORTED, "combine: TypeError reading seq of null");
            if (cv->kind == JV_OBJ) {
                const jv *sq = jv_obj_get_ascii(cv, "seq");
                if (sq && sq->kind == JV_NUM && sq->num == -1) jv_obj_set_ascii(cv, "seq", jv_new_num(seq));
            }
            return jv_ref(cv);
        default: return cv ? jv_ref(cv) : NULL;
    }
}

static int jv_truthy_value(const jv *v) {
    return v && !(v->kind == JV_NULL || v->kind == JV_FALSE || v->kind == JV_UNDEF ||
                  (v->kind == JV_NUM && (v->num == 0 || v->num != v->num)) || (v->kind == JV_STR && v->slen == 0));
}
/* pendingKeyUpdateCount[key] (undefined: 0) */
static int pend_count(const Seg *s, const u16 *k, int kl) {
    const jv *c = s->pend_keys ? jv_obj_get(s->pend_keys, k, kl) : NULL;
    return c ? (int)c->num : 0;
}
/* SegmentPropertiesManager.addProperties (segmentPropertiesManager.ts:35-111).  `rewrite`:
   combiningOp {name:"rewrite"}; `co`: any other combiningOp (NULL: none); `collab`:
   collabWindow.collaborating (false for the props a segment is made with).  A local op
   (seq === UnassignedSequenceNumber) counts its keys as pending; a remote op leaves pending keys
   alone unless it combines, and changes nothing while a local rewrite is pending. */
static void seg_add_properties(mto_doc *d, Seg *s, const jv *new_props, int rewrite, const CombineOp *co,
                               int seq, int collab) {
    if (!s->props) {
        s->props = jv_new(JV_OBJ);
        s->pend_keys = jv_new(JV_OBJ);
        s->pend_rewrite = 0;
    }
    if (s->pend_rewrite > 0 && seq != UNASSIGNED_SEQ && collab) return;
    if (!new_props || new_props->kind != JV_OBJ) fail(d, MTO_BAD_INPUT, "props is not an object");
    const int has_co = co && co->kind;
#define SHOULD_MODIFY(k, kl) (seq == UNASSIGNED_SEQ || !jv_obj_get(s->pend_keys, (k), (kl)) || has_co)
    if (rewrite) {
        if (collab && seq == UNASSIGNED_SEQ) s->pend_rewrite++;
        int *ord = (int *)malloc(sizeof(int) * (size_t)(s->props->n + 1));
        int n = jv_obj_enum(s->props, ord);
        /* collect keys first: deleting while enumerating */
        u16 **ks = (u16 **)malloc(sizeof(u16 *) * (size_t)(n + 1));
        int *kl = (int *)malloc(sizeof(int) * (size_t)(n + 1));
        int m = 0;
        for (int i = 0; i < n; i++) {
            const u16 *k = s->props->keys[ord[i]];
            const int klen = s->props->klens[ord[i]];
            if (!jv_truthy_value(jv_obj_get(new_props, k, klen)) && SHOULD_MODIFY(k, klen)) {
                ks[m] = (u16 *)malloc(sizeof(u16) * (size_t)(klen + 1));
                memcpy(ks[m], k, sizeof(u16) * (size_t)klen);
                kl[m++] = klen;
            }
        }
        for (int i = 0; i < m; i++) {
            jv_obj_del(s->props, ks[i], kl[i]);
            free(ks[i]);
        }
        free(ks);
        free(kl);
        free(ord);
    }
    int *ord = (int *)malloc(sizeof(int) * (size_t)(new_props->n + 1));
    int n = jv_obj_enum(new_props, ord);
    for (int i = 0; i < n; i++) {
        const u16 *k = new_props->keys[ord[i]];
        int kl = new_props->klens[ord[i]];
        jv *v = new_props->vals[ord[i]];
        if (collab) {
            if (seq == UNASSIGNED_SEQ) {
                jv_obj_set(s->pend_keys, k, kl, jv_new_num(pend_count(s, k, kl) + 1));
            } else if (!SHOULD_MODIFY(k, kl)) {
                continue;
            }
        }
        if (has_co) { /* newValue = combine(op, previousValue, newValue, seq) */
            jv *nv = js_combine(d, co, jv_obj_get(s->props, k, kl), seq);
            if (nv && nv->kind == JV_NULL) {
                jv_unref(nv);
                jv_obj_del(s->props, k, kl);
            } else {
                jv_obj_set(s->props, k, kl, nv ? nv : jv_new(JV_UNDEF)); /* properties[key] = undefined */
            }
        } else if (v->kind == JV_NULL) jv_obj_del(s->props, k, kl);
        else jv_obj_set(s->props, k, kl, jv_ref(v));
    }
#undef SHOULD_MODIFY
    free(ord);
}

/* SegmentPropertiesManager.ackPendingProperties (segmentPropertiesManager.ts:19-33) */
static void seg_ack_pending_properties(mto_doc *d, Seg *s, const jv *op_props, int rewrite) {
    if (!s->props) fail(d, MTO_BAD_INPUT, "ack: segment without a property manager");
    if (rewrite) s->pend_rewrite--;
    if (!op_props || op_props->kind != JV_OBJ) return;
    int *ord = (int *)malloc(sizeof(int) * (size_t)(op_props->n + 1));
    int n = jv_obj_enum(op_props, ord);
    for (int i = 0; i < n; i++) {
        const u16 *k = op_props->keys[ord[i]];
        const int kl = op_props->klens[ord[i]];
        if (jv_obj_get(s->pend_keys, k, kl)) {
            const int c = pend_count(s, k, kl);
            if (!(c > 0)) {
                free(ord);
                fail(d, MTO_BAD_INPUT, "ack: pendingKeyUpdateCount");
            }
            if (c - 1 == 0) jv_obj_del(s->pend_keys, k, kl);
            else jv_obj_set(s->pend_keys, k, kl, jv_new_num(c - 1));
        }
    }
    free(ord);
}

/* TextSegment.make(text, props) / Marker.make: `if (props) addProperties(props)` */
static void seg_init_props(mto_doc *d, Seg *s, const jv *props) {
    if (!props || props->kind == JV_NULL) return;
    if (props->kind == JV_FALSE || (props->kind == JV_NUM && props->num == 0) ||
        (props->kind == JV_STR && props->slen == 0))
        return;
    seg_add_properties(d, s, props, 0, NULL, 0, 0);
}

/* ------------------------------------------------------------------ pending segment groups */
/* SegmentGroupCollection.enqueue (segmentGroupCollection.ts:24-27): the segment's queue gets the
   group, the group's segments array gets the segment (at its end) */
static void seg_group_enqueue(Seg *s, Group *g) {
    if (s->sg_head + s->sg_n == s->sg_cap) {
        if (s->sg_head > 0) {
            memmove(s->sg, s->sg + s->sg_head, sizeof(Group *) * (size_t)s->sg_n);
            s->sg_head = 0;
        } else {
            s->sg_cap = s->sg_cap ? s->sg_cap * 2 : 4;
            s->sg = (Group **)realloc(s->sg, sizeof(Group *) * (size_t)s->sg_cap);
        }
    }
    s->sg[s->sg_head + s->sg_n++] = g;
    if (g->n == g->cap) {
        g->cap = g->cap ? g->cap * 2 : 4;
        g->segs = (Seg **)realloc(g->segs, sizeof(Seg *) * (size_t)g->cap);
    }
    g->segs[g->n++] = s;
}
static Group *seg_group_dequeue(Seg *s) { /* segmentGroupCollection.ts:29-31 */
    if (s->sg_n == 0) return NULL;
    s->sg_n--;
    return s->sg[s->sg_head++];
}
/* MergeTree.addToPendingList (mergeTree.ts:1922-1929): the op's group is created (and queued on
   pendingSegments) with its first segment */
static Group *add_to_pending_list(mto_doc *d, Seg *s, Group *g, int local_seq) {
    if (!g) {
        g = (Group *)calloc(1, sizeof(Group));
        g->local_seq = local_seq;
        g->all_next = d->all_groups;
        d->all_groups = g;
        if (d->pend_head + d->pend_n == d->pend_cap) {
            if (d->pend_head > 0) {
                memmove(d->pend, d->pend + d->pend_head, sizeof(Group *) * (size_t)d->pend_n);
                d->pend_head = 0;
            } else {
                d->pend_cap = d->pend_cap ? d->pend_cap * 2 : 16;
                d->pend = (Group **)realloc(d->pend, sizeof(Group *) * (size_t)d->pend_cap);
            }
        }
        d->pend[d->pend_head + d->pend_n++] = g;
    }
    seg_group_enqueue(s, g);
    return g;
}

/* ------------------------------------------------------------------ split / append */
/* BaseSegment.splitAt (mergeTree.ts:524-568) + TextSegment.createSplitSegmentAt
   (textSegment.ts:103-111); Marker.createSplitSegmentAt returns undefined. */
static Seg *seg_split_at(mto_doc *d, Seg *s, int pos) {
    if (!(pos > 0)) return NULL;
    if (s->kind != SEG_TEXT) return NULL;
    int len = s->n.cached_length;
    Seg *leaf = new_text_seg(d, s->text + pos, len - pos);
    s->n.cached_length = pos;
    if (s->props) { /* SegmentPropertiesManager.copyTo (segmentPropertiesManager.ts:113-125) */
        leaf->props = jv_obj_clone(s->props);
        leaf->pend_keys = jv_obj_clone(s->pend_keys);
        leaf->pend_rewrite = s->pend_rewrite;
    }
    leaf->n.parent = s->n.parent;
    leaf->removed_client = s->removed_client;
    leaf->removed_seq = s->removed_seq;
    leaf->removed = s->removed;
    leaf->local_removed_seq = s->local_removed_seq;
    leaf->seq = s->seq;
    leaf->local_seq = s->local_seq;
    leaf->client_id = s->client_id;
    if (s->novl) {
        leaf->ovl = (int *)malloc(sizeof(int) * (size_t)s->novl);
        memcpy(leaf->ovl, s->ovl, sizeof(int) * (size_t)s->novl);
        leaf->novl = leaf->covl = s->novl;
    }
    for (int i = 0; i < s->sg_n; i++) seg_group_enqueue(leaf, s->sg[s->sg_head + i]); /* segmentGroups.copyTo */
    return leaf;
}

/* TextSegment.canAppend (textSegment.ts:63-68); Marker.canAppend is false */
static int seg_can_append(const Seg *prev, const Seg *seg) {
    if (prev->kind != SEG_TEXT) return 0;
    int len = prev->n.cached_length;
    if (len > 0 && prev->text[len - 1] == '\n') return 0;
    if (seg->kind != SEG_TEXT) return 0;
    return prev->n.cached_length <= TEXT_GRANULARITY || seg->n.cached_length <= TEXT_GRANULARITY;
}

/* ------------------------------------------------------------------ tree structure */
static Block *split_block(mto_doc *d, Block *node) { /* MergeTree.split, mergeTree.ts:2476-2489 */
    int half = MAX_NODES / 2;
    Block *nn = make_block(d, half);
    node->child_count = half;
    for (int i = 0; i < half; i++) {
        assign_child(nn, node->children[half + i], i);
        node->children[half + i] = NULL;
    }
    node_update_length_new_structure(node);
    node_update_length_new_structure(nn);
    return nn;
}

static void update_root(mto_doc *d, Block *split_node) { /* mergeTree.ts:1876-1887 */
    if (split_node) {
        Block *nr = make_block(d, 2);
        nr->n.index = 0;
        assign_child(nr, &d->root->n, 0);
        assign_child(nr, &split_node->n, 1);
        d->root = nr;
        node_update_length_new_structure(d->root);
    }
}

/* ------------------------------------------------------------------ nodeMap (mergeTree.ts:2903-2965) */
typedef struct MapActions {
    int (*leaf)(mto_doc *d, Seg *s, int pos, int ref_seq, int client_id, int start, int end, void *ctx);
    int (*post)(mto_doc *d, Block *b, void *ctx);
    void *ctx;
} MapActions;

static int node_map(mto_doc *d, Block *node, MapActions *a, int pos, int ref_seq, int client_id, int start,
                    int end, int has_end) {
    if (!has_end) end = block_length(d, node, ref_seq, client_id);
    int go = 1;
    for (int ci = 0; ci < node->child_count; ci++) {
        Node *child = node->children[ci];
        int len = node_length(d, child, ref_seq, client_id);
        if (go && end > 0 && len > 0 && start < len) {
            if (!child->is_leaf) go = node_map(d, (Block *)child, a, pos, ref_seq, client_id, start, end, 1);
            else go = a->leaf(d, (Seg *)child, pos, ref_seq, client_id, start, end, a->ctx);
        }
        if (!go) break;
        pos += len;
        start -= len;
        end -= len;
    }
    if (go && a->post) go = a->post(d, node, a->ctx);
    return go;
}

/* rightExcursion (mergeTree.ts:2313-2343) used by blockInsert.continueFrom (2154-2161) */
static int check_seg_is_local(mto_doc *d, Seg *s, int pos, int r, int c, int st, int en, void *ctx) {
    (void)d; (void)pos; (void)r; (void)c; (void)st; (void)en;
    if (s->seq == UNASSIGNED_SEQ) *(int *)ctx = 1;
    return 0;
}
static int continue_from(mto_doc *d, Block *node) {
    int seg_is_local = 0;
    MapActions a = {check_seg_is_local, NULL, &seg_is_local};
    Node *start = &node->n;
    Block *parent = start->parent;
    while (parent) {
        int matched = 0;
        for (int ci = 0; ci < parent->child_count; ci++) {
            Node *c = parent->children[ci];
            if (matched) {
                int go;
                if (!c->is_leaf) go = node_map(d, (Block *)c, &a, 0, UNIVERSAL_SEQ, d->cw.client_id, 0, 0, 0);
                else go = check_seg_is_local(d, (Seg *)c, 0, UNIVERSAL_SEQ, d->cw.client_id, 0, 0, &seg_is_local);
                if (!go) return seg_is_local;
            } else {
                matched = (start == c);
            }
        }
        start = &parent->n;
        parent = parent->n.parent;
    }
    return seg_is_local;
}

/* ------------------------------------------------------------------ insertingWalk (mergeTree.ts:2345-2474) */
enum { LEAF_SPLIT = 0, LEAF_INSERT = 1 };
typedef struct {
    int kind;
    Seg *candidate;
    int has_continue;
} ICtx;

static Block UNFINISHED_NODE; /* MergeTree.theUnfinishedNode */

/* breakTie, mergeTree.ts:2248-2277 */
static int break_tie(mto_doc *d, int pos, Node *node, int ref_seq, int client_id) {
    if (node->is_leaf) {
        if (pos == 0) {
            Seg *s = (Seg *)node;
            if (s->removed && s->removed_seq != 0 && s->removed_seq <= ref_seq && s->removed_seq != UNASSIGNED_SEQ)
                return 0;
            if (client_id == d->cw.client_id) return 1;
            if (s->seq != UNASSIGNED_SEQ) return 1;
        }
        return 0;
    }
    return 1;
}

static Block *inserting_walk(mto_doc *d, Block *block, int pos, int ref_seq, int client_id, int seq, ICtx *ctx) {
    int ci;
    Node *new_node = NULL;
    Block *from_split = NULL;
    (void)from_split;
    for (ci = 0; ci < block->child_count; ci++) {
        Node *child = block->children[ci];
        int len = node_length(d, child, ref_seq, client_id);
        if (pos < len || (pos == len && break_tie(d, pos, child, ref_seq, client_id))) {
            if (!child->is_leaf) {
                Block *split_node = inserting_walk(d, (Block *)child, pos, ref_seq, client_id, seq, ctx);
                if (split_node == NULL) {
                    block_update_length(block);
                    return NULL;
                } else if (split_node == &UNFINISHED_NODE) {
                    pos -= len;
                    continue;
                } else {
                    new_node = &split_node->n;
                    from_split = split_node;
                    ci++;
                }
            } else {
                Seg *seg = (Seg *)child;
                /* context.leaf: splitLeafSegment (2225) or blockInsert.onLeaf (2180) */
                Node *next = NULL;
                if (ctx->kind == LEAF_SPLIT) {
                    Seg *n2 = seg_split_at(d, seg, pos);
                    next = n2 ? &n2->n : NULL;
                } else {
                    assign_child(block, &ctx->candidate->n, ci); /* replaceCurrent */
                    next = &seg->n;
                }
                if (next) {
                    new_node = next;
                    ci++;
                } else {
                    return NULL;
                }
            }
            break;
        } else {
            pos -= len;
        }
    }
    if (!new_node) {
        if (pos == 0) {
            if (seq != UNASSIGNED_SEQ && ctx->has_continue && continue_from(d, block)) return &UNFINISHED_NODE;
            if (ctx->kind == LEAF_INSERT) new_node = &ctx->candidate->n;
        }
    }
    if (new_node) {
        for (int i = block->child_count; i > ci; i--) {
            block->children[i] = block->children[i - 1];
            block->children[i]->index = i;
        }
        assign_child(block, new_node, ci);
        block->child_count++;
        if (block->child_count < MAX_NODES) {
            block_update_length(block);
            return NULL;
        }
        return split_block(d, block);
    }
    return NULL;
}

/* ensureIntervalBoundary, mergeTree.ts:2241-2245 */
static void ensure_interval_boundary(mto_doc *d, int pos, int ref_seq, int client_id) {
    ICtx ctx = {LEAF_SPLIT, NULL, 0};
    Block *sn = inserting_walk(d, d->root, pos, ref_seq, client_id, TREE_MAINT_SEQ, &ctx);
    update_root(d, sn);
}

/* addToLRUSet, mergeTree.ts:1273-1283 */
static void add_to_lru_set(mto_doc *d, Seg *s, int seq) {
    if (s->n.parent->needs_scour != SCOUR_TRUE && seq > d->cw.current_seq) {
        s->n.parent->needs_scour = SCOUR_TRUE;
        heap_add(d, s, seq);
    }
}

/* ------------------------------------------------------------------ zamboni */
typedef struct {
    Node **p;
    int n, cap;
} NodeVec;
static void nv_push(NodeVec *v, Node *x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 16;
        v->p = (Node **)realloc(v->p, sizeof(Node *) * (size_t)v->cap);
    }
    v->p[v->n++] = x;
}

/* scourNode, mergeTree.ts:1289-1365 (trackingCollection is empty on this path): a segment in a
   pending group is held as is */
static void scour_node(mto_doc *d, Block *node, NodeVec *hold) {
    Seg *prev = NULL;
    for (int k = 0; k < node->child_count; k++) {
        Node *child = node->children[k];
        if (child->is_leaf) {
            Seg *s = (Seg *)child;
            if (s->sg_n > 0) {
                nv_push(hold, child);
                prev = NULL;
            } else if (s->removed) {
                if (s->removed_seq > d->cw.min_seq) {
                    nv_push(hold, child);
                } else {
                    s->n.parent = NULL; /* unlink */
                }
                prev = NULL;
            } else {
                if (s->seq <= d->cw.min_seq) {
                    int can_append = prev && seg_can_append(prev, s) && jv_match_properties(prev->props, s->props) &&
                                     local_net_length(s) > 0;
                    if (can_append) {
                        seg_text_append(prev, s->text, s->n.cached_length); /* TextSegment.append */
                        s->n.parent = NULL;
                    } else {
                        nv_push(hold, child);
                        prev = local_net_length(s) > 0 ? s : NULL;
                    }
                } else {
                    nv_push(hold, child);
                    prev = NULL;
                }
            }
        } else {
            nv_push(hold, child);
            prev = NULL;
        }
    }
}

static int underflow(const Block *b) { return b->child_count < MAX_NODES / 2; } /* mergeTree.ts:1285 */

/* pack, mergeTree.ts:1368-1420 */
static void pack(mto_doc *d, Block *block) {
    Block *parent = block->n.parent;
    NodeVec hold = {0, 0, 0};
    for (int ci = 0; ci < parent->child_count; ci++) {
        Block *cb = (Block *)parent->children[ci];
        scour_node(d, cb, &hold);
        cb->n.parent = NULL;
    }
    int total = hold.n;
    int half = MAX_NODES / 2;
    int child_count = total / half;
    if (child_count > MAX_NODES - 1) child_count = MAX_NODES - 1;
    if (child_count < 1) child_count = 1;
    int base = total / child_count;
    int extra = total % child_count;
    Block *packed[MAX_NODES];
    int read = 0;
    for (int ni = 0; ni < child_count; ni++) {
        int cnt = base;
        if (extra > 0) {
            cnt++;
            extra--;
        }
        Block *pb = make_block(d, cnt);
        for (int j = 0; j < cnt; j++) assign_child(pb, hold.p[read++], j);
        pb->n.parent = parent;
        packed[ni] = pb;
        node_update_length_new_structure(pb);
    }
    free(hold.p);
    for (int j = 0; j < MAX_NODES; j++) parent->children[j] = NULL;
    for (int j = 0; j < child_count; j++) assign_child(parent, &packed[j]->n, j);
    parent->child_count = child_count;
    if (underflow(parent) && parent->n.parent) {
        pack(d, parent);
    } else {
        block_update_path_lengths(parent);
    }
}

/* zamboniSegments, mergeTree.ts:1422-1478 */
static void zamboni_segments(mto_doc *d) {
    if (!d->cw.collaborating) return;
    for (int i = 0; i < ZAMBONI_MAX; i++) {
        HeapEnt *top = heap_peek(d);
        if (!top || top->max_seq > d->cw.min_seq) break;
        HeapEnt e = heap_get(d);
        if (e.seg->n.parent && e.seg->n.parent->needs_scour != SCOUR_FALSE) {
            Block *block = e.seg->n.parent;
            NodeVec copy = {0, 0, 0};
            scour_node(d, block, &copy);
            block->needs_scour = SCOUR_FALSE;
            int nc = copy.n;
            if (nc < block->child_count) {
                block->child_count = nc;
                for (int j = 0; j < MAX_NODES; j++) block->children[j] = NULL;
                for (int j = 0; j < nc; j++) assign_child(block, copy.p[j], j);
                if (underflow(block) && block->n.parent) {
                    pack(d, block);
                } else {
                    block_update_path_lengths(block);
                }
            }
            free(copy.p);
        }
    }
}

/* ------------------------------------------------------------------ consensus (writer) */
static char *jv_json_text(const jv *v) {
    sb o;
    sb_init(&o);
    jv_stringify(v, &o);
    sb_putc(&o, 0);
    return o.p;
}
static int cons_find(mto_doc *d, const char *key) {
    for (int i = 0; i < d->n_cons; i++)
        if (!strcmp(d->cons_keys[i], key)) return i;
    return -1;
}
/* pendingConsensus.set(marker.getId(), {callback, marker}) (client.ts:124-130) */
static void cons_register(mto_doc *d, const char *key, Seg *m) {
    int i = cons_find(d, key);
    if (i < 0) {
        if (d->n_cons == d->cap_cons) {
            d->cap_cons = d->cap_cons ? 2 * d->cap_cons : 8;
            d->cons_keys = (char **)realloc(d->cons_keys, sizeof(char *) * (size_t)d->cap_cons);
            d->cons_marks = (Seg **)realloc(d->cons_marks, sizeof(Seg *) * (size_t)d->cap_cons);
        }
        i = d->n_cons++;
        d->cons_keys[i] = strdup(key);
    }
    d->cons_marks[i] = m;
}
/* Heap.add (collections.ts:236-248) with minListenerComparer (mergeTree.ts:1042-1045) */
static void cons_lis_add(mto_doc *d, int min_required, char *key, Seg *m) {
    if (d->n_lis + 2 > d->cap_lis) {
        d->cap_lis = d->cap_lis ? 2 * d->cap_lis : 8;
        d->cons_lis = (ConsLis *)realloc(d->cons_lis, sizeof(ConsLis) * (size_t)d->cap_lis);
    }
    int k = ++d->n_lis;
    d->cons_lis[k] = (ConsLis){min_required, key, m};
    ConsLis *L = d->cons_lis;
    while (k > 1 && L[k >> 1].min_required - L[k].min_required > 0) {
        ConsLis t = L[k >> 1];
        L[k >> 1] = L[k];
        L[k] = t;
        k >>= 1;
    }
}
/* Heap.get (collections.ts:228-234, 250-264) */
static ConsLis cons_lis_get(mto_doc *d) {
    ConsLis *L = d->cons_lis;
    const ConsLis x = L[1];
    L[1] = L[d->n_lis];
    d->n_lis--;
    const int n = d->n_lis;
    for (int k = 1; (k << 1) <= n;) {
        int j = k << 1;
        if (j < n && L[j].min_required - L[j + 1].min_required > 0) j++;
        if (L[k].min_required - L[j].min_required <= 0) break;
        ConsLis t = L[k];
        L[k] = L[j];
        L[j] = t;
        k = j;
    }
    return x;
}
/* notifyMinSeqListeners (mergeTree.ts:1709-1716): each listener at seq <= minSeq calls
   consensusInfo.callback(consensusInfo.marker) (client.ts:986) — recorded as an event; an
   unregistered id's consensusInfo is undefined (a TypeError) */
static void cons_notify(mto_doc *d) {
    while (d->n_lis > 0 && d->cons_lis[1].min_required <= d->cw.min_seq) {
        ConsLis x = cons_lis_get(d);
        if (!x.marker) {
            free(x.key);
            fail(d, MTO_UNSUPPORTED, "a consensus listener without pendingConsensus info (a TypeError)");
        }
        char num[96];
        if (d->cons_events_n++) sb_putc(&d->cons_events, ',');
        sb_puts(&d->cons_events, "{\"markerId\":");
        sb_puts(&d->cons_events, x.key);
        snprintf(num, sizeof num, ",\"seq\":%d,\"minSeq\":%d}", x.min_required, d->cw.min_seq);
        sb_puts(&d->cons_events, num);
        free(x.key);
    }
}
static void seg_add_properties(mto_doc *d, Seg *s, const jv *new_props, int rewrite, const CombineOp *co,
                               int seq, int collab);
/* Client.updateConsensusProperty(op, msg) (client.ts:980-987) after the ack: `rel1` is
   op.relativePos1 (NULL: undefined — reading .id throws) */
static void update_consensus_property(mto_doc *d, const jv *rel1, const jv *props, const CombineOp *co, int seq) {
    if (!rel1 || rel1->kind == JV_UNDEF || rel1->kind == JV_NULL)
        fail(d, MTO_UNSUPPORTED, "updateConsensusProperty: relativePos1 is undefined (a TypeError)");
    const jv *id = rel1->kind == JV_OBJ ? jv_obj_get_ascii(rel1, "id") : NULL;
    char *key = NULL;
    Seg *m = NULL;
    if (id && id->kind != JV_UNDEF && id->kind != JV_OBJ && id->kind != JV_ARR) {
        key = jv_json_text(id);
        const int r = cons_find(d, key);
        if (r >= 0) m = d->cons_marks[r];
    }
    /* consensusInfo.marker.addProperties(op.props, op.combiningOp, msg.sequenceNumber): no collab window */
    if (m) seg_add_properties(d, m, props, 0, co, seq, 0);
    cons_lis_add(d, seq, key ? key : strdup("null"), m);
}

/* setMinSeq, mergeTree.ts:1718-1736 */
static void set_min_seq(mto_doc *d, int min_seq) {
    if (!(min_seq <= d->cw.current_seq)) fail(d, MTO_MSN_ORDER, "minSeq %d > currentSeq %d", min_seq, d->cw.current_seq);
    if (!(d->cw.min_seq <= min_seq)) fail(d, MTO_MSN_ORDER, "minSeq moved backwards %d -> %d", d->cw.min_seq, min_seq);
    if (min_seq > d->cw.min_seq) {
        d->cw.min_seq = min_seq;
        zamboni_segments(d);
        if (d->n_lis) cons_notify(d);
    }
}

/* ------------------------------------------------------------------ edits */
/* insertSegments (mergeTree.ts:1968-1998) + blockInsert (2141-2224): ensureIntervalBoundary at
   pos, then each segment with cachedLength > 0 inserted at insertPos (advancing by its length),
   then one zamboni */
static void insert_segments(mto_doc *d, int pos, Seg **segs, int n, int ref_seq, int client_id, int seq) {
    ensure_interval_boundary(d, pos, ref_seq, client_id);
    const int local_seq = seq == UNASSIGNED_SEQ ? ++d->local_seq : 0; /* mergeTree.ts:1976 */
    Group *group = NULL;
    int insert_pos = pos;
    for (int i = 0; i < n; i++) {
        Seg *seg = segs[i];
        if (!seg || seg->n.cached_length <= 0) continue;
        seg->seq = seq;
        seg->local_seq = local_seq;
        seg->client_id = client_id;
        map_marker_id(d, seg); /* blockInsert: Marker.is(newSegment) && getId() (mergeTree.ts:2200-2205) */
        ICtx ctx = {LEAF_INSERT, seg, 1};
        Block *sn = inserting_walk(d, d->root, insert_pos, ref_seq, client_id, seq, &ctx);
        if (seg->n.parent) bump_bounds(seg);
        if (seg->n.parent == NULL)
            fail(d, MTO_INVALID_POS, "MergeTree insert failed: {\"currentSeq\":%d,\"minSeq\":%d,\"segSeq\":%d}",
                 d->cw.current_seq, d->cw.min_seq, seg->seq);
        update_root(d, sn);
        /* saveIfLocal (2164-2179) */
        if (d->cw.collaborating) {
            if (seg->seq == UNASSIGNED_SEQ && client_id == d->cw.client_id) {
                group = add_to_pending_list(d, seg, group, local_seq);
            } else if (seg->seq > d->cw.min_seq) {
                add_to_lru_set(d, seg, seg->seq);
            }
        }
        insert_pos += seg->n.cached_length;
    }
    if (d->cw.collaborating && seq != UNASSIGNED_SEQ) zamboni_segments(d);
}

static void insert_segment(mto_doc *d, int pos, Seg *seg, int ref_seq, int client_id, int seq) {
    insert_segments(d, pos, &seg, 1, ref_seq, client_id, seq);
}

/* ------------------------------------------------------------------ marker ids, relative positions */
static int jv_int(const jv *v, int *out);
/* String(v) of a JSON value as an object key (idToSegment[id]) */
static u16 *js_key_of(const jv *v, int *n) {
    u16buf b = {NULL, 0, 0};
    js_to_string(v, &b);
    if (!b.p) b.p = (u16 *)malloc(sizeof(u16));
    *n = b.n;
    return b.p;
}
/* Marker.getId (mergeTree.ts:690-695): properties.markerId when truthy */
static const jv *marker_id(const Seg *s) {
    if (s->kind != SEG_MARKER || !s->props) return NULL;
    static const u16 MID[8] = {'m', 'a', 'r', 'k', 'e', 'r', 'I', 'd'};
    const jv *v = jv_obj_get(s->props, MID, 8);
    return jv_truthy(v) ? v : NULL;
}
static uint32_t key_hash(const u16 *k, int kl) {
    uint32_t h = 2166136261u;
    for (int i = 0; i < kl; i++) h = (h ^ k[i]) * 16777619u;
    return h;
}
/* index of key k in the id map, or -1 */
static int id_find(mto_doc *d, const u16 *k, int kl) {
    if (!d->id_hcap) return -1;
    for (uint32_t h = key_hash(k, kl) & (uint32_t)(d->id_hcap - 1);; h = (h + 1) & (uint32_t)(d->id_hcap - 1)) {
        const int e = d->id_hash[h];
        if (!e) return -1;
        if (u16_eq(d->id_keys[e - 1], d->id_klens[e - 1], k, kl)) return e - 1;
    }
}
static Seg *id_lookup(mto_doc *d, const u16 *k, int kl) {
    const int i = id_find(d, k, kl);
    return i < 0 ? NULL : d->id_segs[i];
}
static void id_rehash(mto_doc *d) {
    d->id_hcap = d->id_hcap ? 2 * d->id_hcap : 16;
    free(d->id_hash);
    d->id_hash = (int *)calloc((size_t)d->id_hcap, sizeof(int));
    for (int i = 0; i < d->n_ids_map; i++) {
        uint32_t h = key_hash(d->id_keys[i], d->id_klens[i]) & (uint32_t)(d->id_hcap - 1);
        while (d->id_hash[h]) h = (h + 1) & (uint32_t)(d->id_hcap - 1);
        d->id_hash[h] = i + 1;
    }
}
/* mapIdToSegment (mergeTree.ts:1185-1187) */
static void map_marker_id(mto_doc *d, Seg *s) {
    const jv *id = marker_id(s);
    if (!id) return;
    if (s->id_jv == id) { /* same id object as last time: same entry */
        d->id_segs[s->id_idx] = s;
        return;
    }
    int kl;
    u16 *k = js_key_of(id, &kl);
    int i = id_find(d, k, kl);
    if (i >= 0) {
        free(k);
    } else {
        if (d->n_ids_map == d->cap_ids_map) {
            d->cap_ids_map = d->cap_ids_map ? 2 * d->cap_ids_map : 8;
            d->id_keys = (u16 **)realloc(d->id_keys, sizeof(u16 *) * (size_t)d->cap_ids_map);
            d->id_klens = (int *)realloc(d->id_klens, sizeof(int) * (size_t)d->cap_ids_map);
            d->id_segs = (Seg **)realloc(d->id_segs, sizeof(Seg *) * (size_t)d->cap_ids_map);
        }
        i = d->n_ids_map++;
        d->id_keys[i] = k;
        d->id_klens[i] = kl;
        if (2 * d->n_ids_map > d->id_hcap) id_rehash(d);
        else {
            uint32_t h = key_hash(k, kl) & (uint32_t)(d->id_hcap - 1);
            while (d->id_hash[h]) h = (h + 1) & (uint32_t)(d->id_hcap - 1);
            d->id_hash[h] = i + 1;
        }
    }
    d->id_segs[i] = s;
    jv_unref((jv *)s->id_jv);
    s->id_jv = jv_ref((jv *)id); /* held: the cached address cannot be reused by another value */
    s->id_idx = i;
}
/* getPosition (mergeTree.ts:1586-1603): view lengths of everything before `node` on its path to the
   root (an unlinked node has no parent: 0) */
static int get_position(mto_doc *d, Node *node, int ref_seq, int client_id) {
    int total = 0;
    Block *prev = NULL;
    for (Block *p = node->parent; p; prev = p, p = p->n.parent)
        for (int i = 0; i < p->child_count; i++) {
            Node *c = p->children[i];
            if ((prev && c == &prev->n) || c == node) break;
            total += node_length(d, c, ref_seq, client_id);
        }
    return total;
}
/* posFromRelativePos (mergeTree.ts:1942-1966): -1 when the id names no marker */
static int pos_from_relative_pos(mto_doc *d, const jv *rel, int ref_seq, int client_id) {
    int pos = -1;
    const jv *id = rel && rel->kind == JV_OBJ ? jv_obj_get_ascii(rel, "id") : NULL;
    Seg *m = NULL;
    if (jv_truthy(id)) {
        int kl;
        u16 *k = js_key_of(id, &kl);
        m = id_lookup(d, k, kl);
        free(k);
    }
    if (m) {
        pos = get_position(d, &m->n, ref_seq, client_id);
        const jv *before = jv_obj_get_ascii(rel, "before"), *off = jv_obj_get_ascii(rel, "offset");
        int o = 0;
        if (off && off->kind != JV_UNDEF && !jv_int(off, &o)) fail(d, MTO_UNSUPPORTED, "non-integer offset");
        if (!jv_truthy(before)) {
            pos += m->n.cached_length;
            if (off) pos += o;
        } else if (off) {
            pos -= o;
        }
    }
    return pos;
}

typedef struct {
    int seq;
    int client_id;
    int overwrite;
    int local_seq;
    Group *group;
} RemoveCtx;

/* markRangeRemoved.markRemoved (mergeTree.ts:2614-2660), single branch */
static int mark_removed(mto_doc *d, Seg *s, int pos, int r, int c, int st, int en, void *vctx) {
    (void)pos; (void)r; (void)c; (void)st; (void)en;
    RemoveCtx *ctx = (RemoveCtx *)vctx;
    if (s->removed) {
        ctx->overwrite = 1;
        if (s->removed_seq == UNASSIGNED_SEQ) { /* a pending local remove: the sequenced one replaces it */
            s->removed_client = ctx->client_id;
            s->removed_seq = ctx->seq;
            s->local_removed_seq = 0;
            bump_bounds(s);
        } else {
            if (s->novl == s->covl) {
                s->covl = s->covl ? s->covl * 2 : 4;
                s->ovl = (int *)realloc(s->ovl, sizeof(int) * (size_t)s->covl);
            }
            s->ovl[s->novl++] = ctx->client_id; /* addOverlappingClient, 2544-2552 */
        }
    } else {
        s->removed_client = ctx->client_id;
        s->removed_seq = ctx->seq;
        s->local_removed_seq = ctx->local_seq;
        s->removed = 1;
        bump_bounds(s);
    }
    if (d->cw.collaborating) {
        if (s->removed_seq == UNASSIGNED_SEQ && ctx->client_id == d->cw.client_id) {
            ctx->group = add_to_pending_list(d, s, ctx->group, ctx->local_seq);
        } else {
            add_to_lru_set(d, s, ctx->seq);
        }
    }
    return 1;
}
static int after_mark_removed(mto_doc *d, Block *b, void *ctx) {
    (void)d; (void)ctx;
    block_update_length(b); /* or nodeUpdateLengthNewStructure: same cachedLength */
    return 1;
}

static void mark_range_removed(mto_doc *d, int start, int end, int ref_seq, int client_id, int seq) {
    ensure_interval_boundary(d, start, ref_seq, client_id);
    ensure_interval_boundary(d, end, ref_seq, client_id);
    RemoveCtx ctx = {seq, client_id, 0, seq == UNASSIGNED_SEQ ? ++d->local_seq : 0, NULL}; /* mergeTree.ts:2613 */
    MapActions a = {mark_removed, after_mark_removed, &ctx};
    node_map(d, d->root, &a, 0, ref_seq, client_id, start, end, 1);
    if (d->cw.collaborating && seq != UNASSIGNED_SEQ) zamboni_segments(d);
}

typedef struct {
    const jv *props;
    int rewrite;
    int seq;
    const CombineOp *co;
    int local_seq;
    Group *group;
} AnnotateCtx;

static int annotate_segment(mto_doc *d, Seg *s, int pos, int r, int c, int st, int en, void *vctx) {
    (void)pos; (void)r; (void)c; (void)st; (void)en;
    AnnotateCtx *ctx = (AnnotateCtx *)vctx;
    seg_add_properties(d, s, ctx->props, ctx->rewrite, ctx->co, ctx->seq, d->cw.collaborating);
    if (d->cw.collaborating) {
        if (ctx->seq == UNASSIGNED_SEQ) ctx->group = add_to_pending_list(d, s, ctx->group, ctx->local_seq);
        else add_to_lru_set(d, s, ctx->seq);
    }
    return 1;
}

/* annotateRange, mergeTree.ts:2565-2605 */
static void annotate_range(mto_doc *d, int start, int end, const jv *props, int rewrite, const CombineOp *co,
                           int ref_seq, int client_id, int seq) {
    ensure_interval_boundary(d, start, ref_seq, client_id);
    ensure_interval_boundary(d, end, ref_seq, client_id);
    AnnotateCtx ctx = {props, rewrite, seq, co, seq == UNASSIGNED_SEQ ? ++d->local_seq : 0, NULL}; /* 2571 */
    MapActions a = {annotate_segment, NULL, &ctx};
    node_map(d, d->root, &a, 0, ref_seq, client_id, start, end, 1);
    if (d->cw.collaborating && seq != UNASSIGNED_SEQ) zamboni_segments(d);
}

static u16 *utf8_to_u16(const char *s, int *n);
/* ------------------------------------------------------------------ tiles (findTile) */
static void tm_clear(struct TileMap *m) {
    for (int i = 0; i < m->n; i++) free(m->keys[i]);
    m->n = 0;
}
static void tm_free(struct TileMap *m) {
    tm_clear(m);
    free(m->keys);
    free(m->klens);
    free(m->segs);
}
static int tm_find(const struct TileMap *m, const u16 *k, int kl) {
    for (int i = 0; i < m->n; i++)
        if (m->klens[i] == kl && !memcmp(m->keys[i], k, sizeof(u16) * (size_t)kl)) return i;
    return -1;
}
/* tiles[label] = seg (overwrite), or only if absent */
static void tm_set(struct TileMap *m, const u16 *k, int kl, Seg *seg, int only_if_absent) {
    int i = tm_find(m, k, kl);
    if (i >= 0) {
        if (!only_if_absent) m->segs[i] = seg;
        return;
    }
    if (m->n == m->cap) {
        m->cap = m->cap ? m->cap * 2 : 4;
        m->keys = (u16 **)realloc(m->keys, sizeof(u16 *) * (size_t)m->cap);
        m->klens = (int *)realloc(m->klens, sizeof(int) * (size_t)m->cap);
        m->segs = (Seg **)realloc(m->segs, sizeof(Seg *) * (size_t)m->cap);
    }
    m->keys[m->n] = (u16 *)malloc(sizeof(u16) * (size_t)(kl + 1));
    memcpy(m->keys[m->n], k, sizeof(u16) * (size_t)kl);
    m->klens[m->n] = kl;
    m->segs[m->n++] = seg;
}
/* refHasTileLabels (mergeTree.ts:580-582): refType & Tile and a truthy properties[referenceTileLabels] */
static const jv *tile_labels(const Seg *s) {
    if (s->kind != SEG_MARKER || !(s->ref_type & 1) || !s->props) return NULL;
    const jv *v = jv_obj_get_ascii(s->props, "referenceTileLabels");
    return jv_truthy(v) ? v : NULL;
}
/* for (const label of labels): array elements (as object keys: String(element)) or the code
   points of a string; anything else would throw */
typedef void (*LabelFn)(void *ctx, const u16 *k, int kl, const jv *elem);
static int each_label(const jv *v, LabelFn fn, void *ctx) {
    if (v->kind == JV_ARR) {
        for (int i = 0; i < v->n; i++) {
            int kl;
            u16 *k = js_key_of(v->vals[i], &kl);
            fn(ctx, k, kl, v->vals[i]);
            free(k);
        }
        return 1;
    }
    if (v->kind == JV_STR) {
        for (int i = 0; i < v->slen;) {
            int w = (v->s[i] >= 0xD800 && v->s[i] < 0xDC00 && i + 1 < v->slen && v->s[i + 1] >= 0xDC00 && v->s[i + 1] < 0xE000) ? 2 : 1;
            fn(ctx, v->s + i, w, NULL);
            i += w;
        }
        return 1;
    }
    return 0;
}
typedef struct {
    Block *b;
    Seg *seg;
} AddTileCtx;
static void add_tile_cb(void *vctx, const u16 *k, int kl, const jv *elem) {
    (void)elem;
    AddTileCtx *c = (AddTileCtx *)vctx;
    tm_set(&c->b->rt, k, kl, c->seg, 0); /* addTile */
    tm_set(&c->b->lt, k, kl, c->seg, 1); /* addTileIfNotPresent */
}
/* blockUpdate's rightmostTiles / leftmostTiles (mergeTree.ts:2751-2762 -> addNodeReferences) */
/* ------------------------------------------------------------------ range stacks (getStackContext) */
static void rm_clear(struct RangeMap *m) {
    for (int i = 0; i < m->n; i++) {
        free(m->s[i].key);
        free(m->s[i].items);
    }
    m->n = 0;
}
static void rm_free(struct RangeMap *m) {
    rm_clear(m);
    free(m->s);
    m->s = NULL;
    m->cap = 0;
}
/* rangeStacks[label], created empty at the end of the key order when absent */
static RStack *rm_get(struct RangeMap *m, const u16 *k, int kl) {
    for (int i = 0; i < m->n; i++)
        if (m->s[i].klen == kl && !memcmp(m->s[i].key, k, sizeof(u16) * (size_t)kl)) return &m->s[i];
    if (m->n == m->cap) {
        m->cap = m->cap ? 2 * m->cap : 4;
        m->s = (RStack *)realloc(m->s, sizeof(RStack) * (size_t)m->cap);
    }
    RStack *st = &m->s[m->n++];
    st->key = (u16 *)malloc(sizeof(u16) * (size_t)(kl + 1));
    memcpy(st->key, k, sizeof(u16) * (size_t)kl);
    st->klen = kl;
    st->items = NULL;
    st->n = st->cap = 0;
    return st;
}
static void rs_push(RStack *st, Seg *x) {
    if (st->n == st->cap) {
        st->cap = st->cap ? 2 * st->cap : 4;
        st->items = (Seg **)realloc(st->items, sizeof(Seg *) * (size_t)st->cap);
    }
    st->items[st->n++] = x;
}
/* applyRangeReference (mergeTree.ts:246-261): a NestBegin pushes; anything else (a NestEnd) pops a
   NestBegin on top, else is pushed ("TODO: match end with begin": labels are not compared) */
static void apply_range_ref(RStack *st, Seg *delta) {
    if (delta->ref_type & 2) {
        rs_push(st, delta);
        return;
    }
    if (st->n > 0 && (st->items[st->n - 1]->ref_type & 2)) st->n--;
    else rs_push(st, delta);
}
/* applyStackDelta (mergeTree.ts:229-244): every label of the delta with a non-empty stack, in the
   delta's key order, its items bottom to top */
static void apply_stack_delta(struct RangeMap *cur, const struct RangeMap *delta) {
    for (int i = 0; i < delta->n; i++) {
        const RStack *ds = &delta->s[i];
        if (ds->n == 0) continue;
        RStack *cs = rm_get(cur, ds->key, ds->klen);
        for (int j = 0; j < ds->n; j++) apply_range_ref(cs, ds->items[j]);
    }
}
/* refHasRangeLabels (mergeTree.ts:584-586): refType & (NestBegin | NestEnd) and a truthy
   properties[referenceRangeLabels] */
static const jv *range_labels(const Seg *s) {
    if (s->kind != SEG_MARKER || !(s->ref_type & 6) || !s->props) return NULL;
    const jv *v = jv_obj_get_ascii(s->props, "referenceRangeLabels");
    return jv_truthy(v) ? v : NULL;
}
typedef struct {
    Block *b;
    Seg *seg;
} AddRangeCtx;
static void add_range_cb(void *vctx, const u16 *k, int kl, const jv *elem) {
    (void)elem;
    AddRangeCtx *c = (AddRangeCtx *)vctx;
    apply_range_ref(rm_get(&c->b->rs, k, kl), c->seg); /* updateRangeInfo (mergeTree.ts:266-273) */
}

static void block_update_tiles(Block *b) {
    tm_clear(&b->rt);
    tm_clear(&b->lt);
    rm_clear(&b->rs);
    for (int i = 0; i < b->child_count; i++) {
        Node *c = b->children[i];
        if (c->is_leaf) {
            Seg *sg = (Seg *)c;
            if (local_net_length(sg) > 0 && sg->kind == SEG_MARKER && (sg->ref_type & 1)) {
                const jv *labels = tile_labels(sg);
                if (labels) { /* getTileLabels() -> [] otherwise */
                    AddTileCtx ctx = {b, sg};
                    if (!each_label(labels, add_tile_cb, &ctx) && b->doc) b->doc->tile_bad = 1;
                }
            }
            /* addNodeReferences (mergeTree.ts:289-293): NestBegin / NestEnd markers' range labels */
            if (local_net_length(sg) > 0 && sg->kind == SEG_MARKER && (sg->ref_type & 6)) {
                const jv *labels = range_labels(sg);
                if (labels) {
                    AddRangeCtx ctx = {b, sg};
                    if (!each_label(labels, add_range_cb, &ctx) && b->doc) b->doc->range_bad = 1;
                }
            }
        } else {
            const Block *cb = (const Block *)c;
            apply_stack_delta(&b->rs, &cb->rs); /* (mergeTree.ts:312-316) */
            for (int j = 0; j < cb->rt.n; j++) tm_set(&b->rt, cb->rt.keys[j], cb->rt.klens[j], cb->rt.segs[j], 0);
            for (int j = 0; j < cb->lt.n; j++) tm_set(&b->lt, cb->lt.keys[j], cb->lt.klens[j], cb->lt.segs[j], 1);
        }
    }
}
typedef struct {
    const u16 *label;
    int llen;
    int hit;
} HasLabelCtx;
static void has_label_cb(void *vctx, const u16 *k, int kl, const jv *elem) {
    HasLabelCtx *c = (HasLabelCtx *)vctx;
    /* refHasTileLabel (mergeTree.ts:588-597): label === refLabel (a string element, or a code point) */
    if (elem && elem->kind != JV_STR) return;
    if (kl == c->llen && !memcmp(k, c->label, sizeof(u16) * (size_t)kl)) c->hit = 1;
}
static int seg_has_tile_label(mto_doc *d, const Seg *s, const u16 *label, int llen) {
    const jv *labels = tile_labels(s);
    if (!labels) return 0;
    HasLabelCtx ctx = {label, llen, 0};
    if (!each_label(labels, has_label_cb, &ctx)) d->tile_bad = 1;
    return ctx.hit;
}

typedef struct {
    const u16 *label;
    int llen;
    int preceding;
    Seg *tile;
} TileSearch;
/* tileShift (mergeTree.ts:1012-1035) */
static void tile_shift(mto_doc *d, Node *node, TileSearch *ts) {
    if (node->is_leaf) {
        Seg *sg = (Seg *)node;
        if (local_net_length(sg) > 0 && sg->kind == SEG_MARKER && seg_has_tile_label(d, sg, ts->label, ts->llen))
            ts->tile = sg;
    } else {
        const Block *b = (const Block *)node;
        const struct TileMap *m = ts->preceding ? &b->rt : &b->lt;
        int i = tm_find(m, ts->label, ts->llen);
        if (i >= 0) ts->tile = m->segs[i];
    }
}
/* recordTileStart (mergeTree.ts:998-1010) */
static void record_tile_start(mto_doc *d, Seg *sg, TileSearch *ts) {
    if (sg->kind == SEG_MARKER && seg_has_tile_label(d, sg, ts->label, ts->llen)) ts->tile = sg;
}
/* searchBlock (mergeTree.ts:1797-1829) with the local client's view (refSeq UniversalSequenceNumber) */
static void search_block(mto_doc *d, Block *block, int pos, TileSearch *ts) {
    for (int ci = 0; ci < block->child_count; ci++) {
        Node *child = block->children[ci];
        const int len = node_length(d, child, UNIVERSAL_SEQ, d->cw.client_id);
        if (pos < len) {
            if (!child->is_leaf) search_block(d, (Block *)child, pos, ts);
            else record_tile_start(d, (Seg *)child, ts);
            return;
        }
        tile_shift(d, child, ts);
        pos -= len;
    }
}
/* backwardSearchBlock (mergeTree.ts:1841-1874) */
static void backward_search_block(mto_doc *d, Block *block, int pos, int seg_end, TileSearch *ts) {
    for (int ci = block->child_count - 1; ci >= 0; ci--) {
        Node *child = block->children[ci];
        const int len = node_length(d, child, UNIVERSAL_SEQ, d->cw.client_id);
        const int segpos = seg_end - len;
        if (pos >= segpos) {
            if (!child->is_leaf) backward_search_block(d, (Block *)child, pos, seg_end, ts);
            else record_tile_start(d, (Seg *)child, ts);
            return;
        }
        tile_shift(d, child, ts);
        seg_end = segpos;
    }
}
/* MergeTree.findTile (mergeTree.ts:1763-1789) for the local client (Client.findTile, client.ts:
   1073-1076): the tile's position, or -1 when there is none; -2 when the document holds a tile
   label list the reference could not iterate.  *props_json: the marker's properties (caller frees). */
long mto_find_tile(mto_doc *d, int start_pos, const char *label_utf8, int preceding, char **props_json) {
    if (props_json) *props_json = NULL;
    int llen;
    u16 *label = utf8_to_u16(label_utf8, &llen);
    TileSearch ts = {label, llen, preceding, NULL};
    if (preceding) {
        search_block(d, d->root, start_pos, &ts);
    } else {
        const int len = d->root->n.cached_length; /* getLength(UniversalSequenceNumber, local client) */
        if (start_pos <= len) backward_search_block(d, d->root, start_pos, len, &ts);
    }
    free(label);
    if (d->tile_bad) return -2;
    if (!ts.tile) return -1;
    /* getPosition(marker, UniversalSequenceNumber, clientId) (mergeTree.ts:1586-1603) */
    long pos = 0;
    Node *node = &ts.tile->n;
    for (Block *p = node->parent; p; node = &p->n, p = p->n.parent)
        for (int i = 0; i < p->child_count && p->children[i] != node; i++)
            pos += node_length(d, p->children[i], UNIVERSAL_SEQ, d->cw.client_id);
    if (props_json && ts.tile->props) {
        sb o;
        sb_init(&o);
        jv_stringify(ts.tile->props, &o);
        sb_putc(&o, 0);
        *props_json = o.p;
    }
    return pos;
}

/* refHasRangeLabel (mergeTree.ts:599-608) */
static int seg_has_range_label(mto_doc *d, const Seg *s, const u16 *label, int llen) {
    const jv *labels = range_labels(s);
    if (!labels) return 0;
    HasLabelCtx ctx = {label, llen, 0};
    if (!each_label(labels, has_label_cb, &ctx)) d->range_bad = 1;
    return ctx.hit;
}
typedef struct {
    u16 **labels;
    int *llens;
    int nl;
    struct RangeMap out; /* searchInfo.stacks */
} RangeSearch;
/* applyLeafRangeMarker (mergeTree.ts:953-964): only the requested labels, in request order */
static void apply_leaf_range_marker(mto_doc *d, Seg *m, RangeSearch *rs) {
    for (int i = 0; i < rs->nl; i++)
        if (seg_has_range_label(d, m, rs->labels[i], rs->llens[i])) apply_range_ref(rm_get(&rs->out, rs->labels[i], rs->llens[i]), m);
}
/* rangeShift (mergeTree.ts:978-994): a preceding leaf by its requested labels, a preceding block by
   its whole rangeStacks delta (every label) */
static void range_shift(mto_doc *d, Node *node, RangeSearch *rs) {
    if (node->is_leaf) {
        Seg *sg = (Seg *)node;
        if (local_net_length(sg) > 0 && sg->kind == SEG_MARKER && (sg->ref_type & 6)) apply_leaf_range_marker(d, sg, rs);
    } else {
        apply_stack_delta(&rs->out, &((Block *)node)->rs);
    }
}
/* searchBlock (mergeTree.ts:1797-1829) with { leaf: recordRangeLeaf (965-976), shift: rangeShift } */
static void range_search_block(mto_doc *d, Block *block, int pos, RangeSearch *rs) {
    for (int ci = 0; ci < block->child_count; ci++) {
        Node *child = block->children[ci];
        const int len = node_length(d, child, UNIVERSAL_SEQ, d->cw.client_id);
        if (pos < len) {
            if (!child->is_leaf) {
                range_search_block(d, (Block *)child, pos, rs);
            } else {
                Seg *sg = (Seg *)child;
                if (sg->kind == SEG_MARKER && (sg->ref_type & 6)) apply_leaf_range_marker(d, sg, rs);
            }
            return;
        }
        range_shift(d, child, rs);
        pos -= len;
    }
}
static long seg_position_local(mto_doc *d, Seg *s) { /* getPosition (mergeTree.ts:1586-1603), local view */
    long pos = 0;
    Node *node = &s->n;
    for (Block *p = node->parent; p; node = &p->n, p = p->n.parent)
        for (int i = 0; i < p->child_count && p->children[i] != node; i++)
            pos += node_length(d, p->children[i], UNIVERSAL_SEQ, d->cw.client_id);
    return pos;
}
/* canonical array index ("0", "17"; not "01"): JS object keys enumerate those first, ascending */
static int u16_index_key(const u16 *k, int kl, unsigned long *v) {
    if (kl < 1 || kl > 10 || (kl > 1 && k[0] == '0')) return 0;
    unsigned long x = 0;
    for (int i = 0; i < kl; i++) {
        if (k[i] < '0' || k[i] > '9') return 0;
        x = x * 10 + (unsigned long)(k[i] - '0');
    }
    if (x >= 4294967295ul) return 0;
    *v = x;
    return 1;
}
/* MergeTree.getStackContext(startPos, clientId, rangeLabels) (mergeTree.ts:1750-1760) via
   Client.getStackContext (client.ts:946-948: the local client): JSON of searchInfo.stacks —
   {label: [{"pos": P, "refType": T[, "props": {...}]}, ...]} in JS key order, each stack bottom to
   top.  NULL with *status MTO_UNSUPPORTED when the document holds a range label list the reference
   could not iterate. */
char *mto_stack_context(mto_doc *d, int start_pos, const char *const *labels_utf8, int n_labels, int *status) {
    RangeSearch rs;
    memset(&rs, 0, sizeof rs);
    rs.nl = n_labels;
    rs.labels = (u16 **)calloc((size_t)(n_labels + 1), sizeof(u16 *));
    rs.llens = (int *)calloc((size_t)(n_labels + 1), sizeof(int));
    for (int i = 0; i < n_labels; i++) rs.labels[i] = utf8_to_u16(labels_utf8[i], &rs.llens[i]);
    range_search_block(d, d->root, start_pos, &rs);
    char *res = NULL;
    *status = d->range_bad ? MTO_UNSUPPORTED : MTO_OK;
    if (!d->range_bad) {
        int *order = (int *)malloc(sizeof(int) * (size_t)(rs.out.n + 1));
        int no = 0;
        unsigned long iv[2];
        /* integer-like keys ascending, then the others in creation order */
        for (int i = 0; i < rs.out.n; i++)
            if (u16_index_key(rs.out.s[i].key, rs.out.s[i].klen, &iv[0])) {
                int j = no++;
                while (j > 0 && (u16_index_key(rs.out.s[order[j - 1]].key, rs.out.s[order[j - 1]].klen, &iv[1]), iv[1] > iv[0])) {
                    order[j] = order[j - 1];
                    j--;
                }
                order[j] = i;
            }
        for (int i = 0; i < rs.out.n; i++)
            if (!u16_index_key(rs.out.s[i].key, rs.out.s[i].klen, &iv[0])) order[no++] = i;
        sb o;
        sb_init(&o);
        sb_putc(&o, '{');
        for (int q = 0; q < no; q++) {
            const RStack *st = &rs.out.s[order[q]];
            if (q) sb_putc(&o, ',');
            jv key;
            memset(&key, 0, sizeof key);
            key.kind = JV_STR;
            key.s = st->key;
            key.slen = st->klen;
            jv_stringify(&key, &o);
            sb_puts(&o, ":[");
            for (int j = 0; j < st->n; j++) {
                Seg *m = st->items[j];
                char num[64];
                snprintf(num, sizeof num, "%s{\"pos\":%ld,\"refType\":%d", j ? "," : "", seg_position_local(d, m), m->ref_type);
                sb_puts(&o, num);
                if (m->props) {
                    sb_puts(&o, ",\"props\":");
                    jv_stringify(m->props, &o);
                }
                sb_putc(&o, '}');
            }
            sb_putc(&o, ']');
        }
        sb_putc(&o, '}');
        sb_putc(&o, 0);
        res = o.p;
        free(order);
    }
    for (int i = 0; i < n_labels; i++) free(rs.labels[i]);
    free(rs.labels);
    free(rs.llens);
    rm_free(&rs.out);
    return res;
}

/* ------------------------------------------------------------------ client */
static int get_short_client_id(mto_doc *d, const char *long_id) {
    for (int i = 0; i < d->n_ids; i++)
        if (!strcmp(d->long_ids[i], long_id)) return i;
    return -1;
}
static int add_long_client_id(mto_doc *d, const char *long_id) { /* client.ts:653-660 */
    if (d->n_ids == d->cap_ids) {
        d->cap_ids = d->cap_ids ? d->cap_ids * 2 : 16;
        d->long_ids = (char **)realloc(d->long_ids, sizeof(char *) * (size_t)d->cap_ids);
    }
    d->long_ids[d->n_ids] = strdup(long_id);
    return d->n_ids++;
}
static int get_or_add_short_client_id(mto_doc *d, const char *long_id) { /* client.ts:636-641 */
    int id = get_short_client_id(d, long_id);
    return id >= 0 ? id : add_long_client_id(d, long_id);
}
static const char *get_long_client_id(mto_doc *d, int short_id) { /* client.ts:645-652 */
    if (short_id >= 0) return short_id < d->n_ids ? d->long_ids[short_id] : "undefined";
    return "original";
}

mto_doc *mto_new(void) {
    mto_doc *d = (mto_doc *)calloc(1, sizeof(mto_doc));
    d->root = make_block(d, 0); /* initialNode, mergeTree.ts:1125-1129 */
    d->root->n.cached_length = 0;
    d->cw.client_id = LOCAL_CLIENT;
    heap_init(d);
    for (int i = 0; i < MT_MAX_CLIENTS + 2; i++) d->pk_map[i] = -1;
    return d;
}

static void free_blobs(mto_doc *d) {
    for (int i = 0; i < d->n_blobs; i++) {
        free(d->blob_names[i]);
        sb_free(&d->blobs[i]);
    }
    free(d->blob_names);
    free(d->blobs);
    d->blob_names = NULL;
    d->blobs = NULL;
    d->n_blobs = 0;
}

void mto_free(mto_doc *d) {
    if (!d) return;
    for (Seg *s = d->all_segs; s;) {
        Seg *n = s->all_next;
        free(s->text);
        free(s->ovl);
        free(s->sg);
        jv_unref(s->pend_keys);
        jv_unref(s->props);
        jv_unref((jv *)s->id_jv);
        free(s);
        s = n;
    }
    for (Block *b = d->all_blocks; b;) {
        Block *n = b->all_next;
        tm_free(&b->rt);
        tm_free(&b->lt);
        rm_free(&b->rs);
        free(b);
        b = n;
    }
    for (Group *g = d->all_groups; g;) {
        Group *n = g->all_next;
        free(g->segs);
        free(g);
        g = n;
    }
    free(d->pend);
    sb_free(&d->regen_cur);
    sb_free(&d->regen_all);
    for (int i = 0; i < d->n_cons; i++) free(d->cons_keys[i]);
    free(d->cons_keys);
    free(d->cons_marks);
    for (int i = 1; i <= d->n_lis; i++) free(d->cons_lis[i].key);
    free(d->cons_lis);
    sb_free(&d->cons_events);
    free(d->ntf_key);
    for (int i = 0; i < d->n_ids; i++) free(d->long_ids[i]);
    free(d->long_ids);
    for (int i = 0; i < d->n_ids_map; i++) free(d->id_keys[i]);
    free(d->id_keys);
    free(d->id_klens);
    free(d->id_segs);
    free(d->id_hash);
    free(d->long_client_id);
    free(d->heap);
    free_blobs(d);
    free(d);
}

int mto_status(const mto_doc *d) { return d->status; }
const char *mto_error(const mto_doc *d) { return d->err; }

#define GUARD(d)                                       \
    if ((d)->status != MTO_OK) return (d)->status;     \
    (d)->jb_armed = 1;                                 \
    if (setjmp((d)->jb)) {                             \
        (d)->jb_armed = 0;                             \
        return (d)->status;                            \
    }
#define UNGUARD(d) ((d)->jb_armed = 0)

/* Client.startOrUpdateCollaboration (client.ts:1051-1071) → MergeTree.startCollaboration (1254-1271) */
int mto_start_collab(mto_doc *d, const char *long_id, int min_seq, int cur_seq) {
    GUARD(d);
    if (d->long_client_id == NULL) {
        d->long_client_id = strdup(long_id);
        int sid = add_long_client_id(d, long_id);
        d->cw.client_id = sid;
        d->cw.min_seq = min_seq;
        d->cw.collaborating = 1;
        d->cw.current_seq = cur_seq;
        heap_init(d);
    } else {
        int sid = get_short_client_id(d, d->long_client_id);
        free(d->long_ids[sid]);
        d->long_ids[sid] = strdup(long_id);
        free(d->long_client_id);
        d->long_client_id = strdup(long_id);
    }
    UNGUARD(d);
    return d->status;
}

/* completeAndLogOp asserts for remote ops (client.ts:461-464) */
static void complete_remote_op(mto_doc *d, int seq, int msn) {
    if (!(d->cw.current_seq < seq)) fail(d, MTO_SEQ_ORDER, "Incoming remote op sequence# <= local collabWindow's currentSequence#");
    if (!(d->cw.min_seq <= msn)) fail(d, MTO_MSN_ORDER, "Incoming remote op minSequence# < local collabWindow's minSequence#");
}

/* Client.updateSeqNumbers (client.ts:821-828) */
static void update_seq_numbers(mto_doc *d, int min, int seq) {
    if (!(d->cw.current_seq <= seq)) fail(d, MTO_SEQ_ORDER, "Incoming op sequence# < local collabWindow's currentSequence#");
    d->cw.current_seq = seq;
    if (!(min <= seq)) fail(d, MTO_MSN_ORDER, "Incoming op sequence# < minSequence#");
    set_min_seq(d, min);
}

static int jv_int(const jv *v, int *out) {
    if (!v || v->kind != JV_NUM) return 0;
    *out = (int)v->num;
    return 1;
}

/* specToSegment (sequence/src/sequenceFactory.ts:31-37): TextSegment.fromJSONObject
   (textSegment.ts:30-39) then Marker.fromJSONObject (mergeTree.ts:658-665) */
static Seg *spec_to_segment(mto_doc *d, const jv *spec) {
    if (spec && spec->kind == JV_STR) return new_text_seg(d, spec->s, spec->slen);
    if (spec && spec->kind == JV_OBJ) {
        const jv *t = jv_obj_get_ascii(spec, "text");
        if (t) {
            if (t->kind != JV_STR) fail(d, MTO_BAD_INPUT, "text is not a string");
            Seg *s = new_text_seg(d, t->s, t->slen);
            seg_init_props(d, s, jv_obj_get_ascii(spec, "props"));
            return s;
        }
        const jv *m = jv_obj_get_ascii(spec, "marker");
        if (m) {
            int rt = 0;
            if (m->kind == JV_OBJ) jv_int(jv_obj_get_ascii(m, "refType"), &rt);
            Seg *s = new_marker(d, rt);
            seg_init_props(d, s, jv_obj_get_ascii(spec, "props"));
            return s;
        }
    }
    fail(d, MTO_BAD_INPUT, "unrecognized segment spec");
    return NULL;
}

/* MergeTree.ackPendingSegment (mergeTree.ts:1893-1920) with BaseSegment.ack (487-522): one op of
   the replica's own sequenced message (Client.ackPendingSegment, client.ts:588-625) assigns `seq`
   to the segments of the oldest pending group, in the group's order */
static void ack_pending_segment(mto_doc *d, int type, const jv *op_props, int rewrite, int seq) {
    Group *g = NULL;
    if (d->pend_n > 0) {
        g = d->pend[d->pend_head++];
        d->pend_n--;
    }
    if (g) {
        Block *nodes[64];
        int nn = 0;
        Block **more = NULL;
        for (int i = 0; i < g->n; i++) {
            Seg *s = g->segs[i];
            if (seg_group_dequeue(s) != g) fail(d, MTO_BAD_INPUT, "ack: segment group not at the head");
            switch (type) {
                case MT_OP_ANNOTATE: seg_ack_pending_properties(d, s, op_props, rewrite); break;
                case MT_OP_INSERT:
                    if (s->seq != UNASSIGNED_SEQ) fail(d, MTO_BAD_INPUT, "ack: insert of a sequenced segment");
                    s->seq = seq;
                    s->local_seq = 0;
                    break;
                case MT_OP_REMOVE:
                    if (!s->removed) fail(d, MTO_BAD_INPUT, "ack: remove of a segment not removed");
                    s->local_removed_seq = 0;
                    if (s->removed_seq == UNASSIGNED_SEQ) s->removed_seq = seq;
                    break;
                default: fail(d, MTO_BAD_INPUT, "ack: op type %d", type);
            }
            add_to_lru_set(d, s, seq);
            Block *p = s->n.parent; /* nodesToUpdate, first appearance order */
            int seen = 0;
            for (int j = 0; j < nn && !seen; j++) seen = (j < 64 ? nodes[j] : more[j - 64]) == p;
            if (!seen) {
                if (nn < 64) nodes[nn] = p;
                else {
                    more = (Block **)realloc(more, sizeof(Block *) * (size_t)(nn - 63));
                    more[nn - 64] = p;
                }
                nn++;
            }
        }
        for (int j = 0; j < nn; j++) block_update_path_lengths(j < 64 ? nodes[j] : more[j - 64]);
        free(more);
    }
    zamboni_segments(d);
}

/* an annotate's combiningOp (segmentPropertiesManager.ts:53-54): "rewrite" when op.name is
   "rewrite", else any truthy combiningOp goes through Properties.combine */
static void combine_of(const jv *op, int *rewrite, CombineOp *co) {
    const jv *cop = jv_obj_get_ascii(op, "combiningOp");
    *rewrite = 0;
    co->kind = MT_COMBINE_NONE;
    co->def = co->min = NULL;
    if (!jv_truthy(cop)) return;
    const jv *nm = cop->kind == JV_OBJ ? jv_obj_get_ascii(cop, "name") : NULL;
    static const u16 RW[7] = {'r', 'e', 'w', 'r', 'i', 't', 'e'};
    static const u16 INCR[4] = {'i', 'n', 'c', 'r'};
    static const u16 CONS[9] = {'c', 'o', 'n', 's', 'e', 'n', 's', 'u', 's'};
    const int str = nm && nm->kind == JV_STR;
    if (str && u16_eq(nm->s, nm->slen, RW, 7)) {
        *rewrite = 1;
        return;
    }
    co->kind = str && u16_eq(nm->s, nm->slen, INCR, 4)   ? MT_COMBINE_INCR
               : str && u16_eq(nm->s, nm->slen, CONS, 9) ? MT_COMBINE_CONSENSUS
                                                         : MT_COMBINE_OTHER;
    if (cop->kind == JV_OBJ) {
        co->def = jv_obj_get_ascii(cop, "defaultValue");
        co->min = jv_obj_get_ascii(cop, "minValue");
    }
}

/* Client.applyRemoteOp (client.ts:768-795) */
static void apply_remote_op(mto_doc *d, const jv *op, int short_id, int seq, int ref_seq, int msn) {
    int type = -1;
    if (!op || op->kind != JV_OBJ || !jv_int(jv_obj_get_ascii(op, "type"), &type)) fail(d, MTO_BAD_INPUT, "bad op");
    int pos1 = 0, pos2 = 0;
    int has1 = jv_int(jv_obj_get_ascii(op, "pos1"), &pos1);
    int has2 = jv_int(jv_obj_get_ascii(op, "pos2"), &pos2);
    /* getValidOpRange (client.ts:485-502): pos undefined and relativePos given -> posFromRelativePos */
    if (type != 3 && !jv_obj_get_ascii(op, "pos1") && jv_truthy(jv_obj_get_ascii(op, "relativePos1"))) {
        pos1 = pos_from_relative_pos(d, jv_obj_get_ascii(op, "relativePos1"), ref_seq, short_id);
        has1 = 1;
    }
    if ((type == 1 || type == 2) && !jv_obj_get_ascii(op, "pos2") && jv_truthy(jv_obj_get_ascii(op, "relativePos2"))) {
        pos2 = pos_from_relative_pos(d, jv_obj_get_ascii(op, "relativePos2"), ref_seq, short_id);
        has2 = 1;
    }
    if (type != 3 && !has1) fail(d, MTO_UNSUPPORTED, "op without a position");
    switch (type) {
        case 0: { /* applyInsertOp, client.ts:393-441 */
            const jv *segspec = jv_obj_get_ascii(op, "seg");
            if (!segspec) fail(d, MTO_UNSUPPORTED, "register insert");
            Seg *s = spec_to_segment(d, segspec);
            insert_segment(d, pos1, s, ref_seq, short_id, seq);
            complete_remote_op(d, seq, msn);
            break;
        }
        case 1: /* applyRemoveRangeOp, client.ts:320-351 */
            if (jv_obj_get_ascii(op, "register")) fail(d, MTO_UNSUPPORTED, "register remove");
            if (!has2) pos2 = 0; /* undefined end: nodeMap never matches (end > 0 fails) */
            mark_range_removed(d, pos1, pos2, ref_seq, short_id, seq);
            complete_remote_op(d, seq, msn);
            break;
        case 2: { /* applyAnnotateRangeOp, client.ts:358-386 */
            const jv *props = jv_obj_get_ascii(op, "props");
            int rewrite = 0;
            CombineOp co;
            combine_of(op, &rewrite, &co);
            if (!has2) pos2 = 0;
            annotate_range(d, pos1, pos2, props, rewrite, co.kind ? &co : NULL, ref_seq, short_id, seq);
            complete_remote_op(d, seq, msn);
            break;
        }
        case 3: { /* GROUP */
            const jv *ops = jv_obj_get_ascii(op, "ops");
            if (!ops || ops->kind != JV_ARR) fail(d, MTO_BAD_INPUT, "group without ops");
            for (int i = 0; i < ops->n; i++) apply_remote_op(d, ops->vals[i], short_id, seq, ref_seq, msn);
            break;
        }
        default: break;
    }
}

/* Client.ackPendingSegment (client.ts:588-625): a GROUP acks each member */
static void ack_op_json(mto_doc *d, const jv *op, int seq) {
    int type = -1;
    if (!op || op->kind != JV_OBJ || !jv_int(jv_obj_get_ascii(op, "type"), &type)) fail(d, MTO_BAD_INPUT, "bad op");
    if (type == 3) {
        const jv *ops = jv_obj_get_ascii(op, "ops");
        if (!ops || ops->kind != JV_ARR) fail(d, MTO_BAD_INPUT, "group without ops");
        for (int i = 0; i < ops->n; i++) ack_op_json(d, ops->vals[i], seq);
        return;
    }
    int rewrite = 0;
    CombineOp co = {MT_COMBINE_NONE, NULL, NULL};
    if (type == 2) combine_of(op, &rewrite, &co);
    ack_pending_segment(d, type, type == 2 ? jv_obj_get_ascii(op, "props") : NULL, rewrite, seq);
    /* Client.ackPendingSegment -> updateConsensusProperty (client.ts:596-600) */
    if (type == 2 && co.kind == MT_COMBINE_CONSENSUS)
        update_consensus_property(d, jv_obj_get_ascii(op, "relativePos1"), jv_obj_get_ascii(op, "props"), &co, seq);
}

/* a local op of a collaborating replica: Client.insertSegmentLocal / removeRangeLocal /
   annotateRangeLocal (client.ts:201-291) -> applyXOp with getClientSequenceArgs' local args
   (currentSeq, clientId, UnassignedSequenceNumber; 553-563).  getValidOpRange's local check
   (504-543): an invalid range is logged (InvalidOpRange) and the op is not applied; returns 0 then. */
static int local_range_valid(mto_doc *d, int type, int start, int has_end, int end) {
    const int len = d->root->n.cached_length; /* getLength() */
    if (start < 0 || start > len || (start == len && type != 0)) return 0;
    if (type != 0 || has_end) {
        if (!has_end || end <= start) return 0;
    }
    return 1;
}
static int apply_local_op_json(mto_doc *d, const jv *op) {
    int type = -1;
    if (!op || op->kind != JV_OBJ || !jv_int(jv_obj_get_ascii(op, "type"), &type)) fail(d, MTO_BAD_INPUT, "bad op");
    const int ref = d->cw.current_seq, cid = d->cw.client_id;
    const int seq = d->cw.collaborating ? UNASSIGNED_SEQ : UNIVERSAL_SEQ; /* getLocalSequenceNumber (client.ts:949-955) */
    if (type == 3) {
        const jv *ops = jv_obj_get_ascii(op, "ops");
        if (!ops || ops->kind != JV_ARR) fail(d, MTO_BAD_INPUT, "group without ops");
        int any = 0;
        for (int i = 0; i < ops->n; i++) any |= apply_local_op_json(d, ops->vals[i]);
        return any;
    }
    int pos1 = 0, pos2 = 0;
    int has1 = jv_int(jv_obj_get_ascii(op, "pos1"), &pos1);
    int has2 = jv_int(jv_obj_get_ascii(op, "pos2"), &pos2);
    /* getValidOpRange (client.ts:485-502) in the local view: relative positions (-1: no marker) */
    if (!jv_obj_get_ascii(op, "pos1") && jv_truthy(jv_obj_get_ascii(op, "relativePos1"))) {
        pos1 = pos_from_relative_pos(d, jv_obj_get_ascii(op, "relativePos1"), ref, cid);
        has1 = 1;
    }
    if (!jv_obj_get_ascii(op, "pos2") && jv_truthy(jv_obj_get_ascii(op, "relativePos2"))) {
        pos2 = pos_from_relative_pos(d, jv_obj_get_ascii(op, "relativePos2"), ref, cid);
        has2 = 1;
    }
    if (!has1) fail(d, MTO_UNSUPPORTED, "local op without pos1");
    if (!local_range_valid(d, type, pos1, has2, pos2)) return 0;
    switch (type) {
        case 0: {
            const jv *segspec = jv_obj_get_ascii(op, "seg");
            if (!segspec) fail(d, MTO_UNSUPPORTED, "register insert");
            Seg *s = spec_to_segment(d, segspec);
            insert_segment(d, pos1, s, ref, cid, seq);
            break;
        }
        case 1: mark_range_removed(d, pos1, pos2, ref, cid, seq); break;
        case 2: {
            int rewrite = 0;
            CombineOp co;
            combine_of(op, &rewrite, &co);
            annotate_range(d, pos1, pos2, jv_obj_get_ascii(op, "props"), rewrite, co.kind ? &co : NULL, ref, cid, seq);
            break;
        }
        default: break;
    }
    return 1;
}

int mto_local_op_json(mto_doc *d, const char *op_json) { return mto_local_op_notify_json(d, op_json, 0); }

/* notify: Client.annotateMarkerNotifyConsensus(marker, props, callback) (client.ts:113-134) made
   the op (createAnnotateMarkerOp: relativePos1 {id, before: true}); the marker is
   getMarkerFromId(id), registered in pendingConsensus when the annotate applies */
int mto_local_op_notify_json(mto_doc *d, const char *op_json, int notify) {
    GUARD(d);
    jv *op = jv_parse(op_json, strlen(op_json));
    if (!op) fail(d, MTO_BAD_INPUT, "op is not JSON");
    char *key = NULL;
    Seg *m = NULL;
    if (notify) {
        const jv *r1 = op->kind == JV_OBJ ? jv_obj_get_ascii(op, "relativePos1") : NULL;
        const jv *id = r1 && r1->kind == JV_OBJ ? jv_obj_get_ascii(r1, "id") : NULL;
        if (!jv_truthy(id) || id->kind == JV_OBJ || id->kind == JV_ARR) {
            jv_unref(op);
            fail(d, MTO_BAD_INPUT, "notifyConsensus without a marker id");
        }
        int kl;
        u16 *k = js_key_of(id, &kl);
        m = id_lookup(d, k, kl);
        free(k);
        key = jv_json_text(id);
    }
    const int applied = apply_local_op_json(d, op);
    if (notify && applied && m) cons_register(d, key, m);
    free(key);
    jv_unref(op);
    UNGUARD(d);
    return d->status;
}

/* test helper: the local position of the marker mapped to `id_json`'s key, -1 when there is none
   or it is removed in the local view */
int mto_local_marker_pos(mto_doc *d, const char *id_json) {
    jv *id = jv_parse(id_json, strlen(id_json));
    int pos = -1;
    if (id && jv_truthy(id)) {
        int kl;
        u16 *k = js_key_of(id, &kl);
        Seg *m = id_lookup(d, k, kl);
        free(k);
        if (m && m->n.parent && local_net_length(m) > 0) pos = get_position(d, &m->n, d->cw.current_seq, d->cw.client_id);
    }
    jv_unref(id);
    return pos;
}

/* the consensus callbacks made so far, in call order: [{"markerId", "seq", "minSeq"}, ...] */
char *mto_consensus_events(mto_doc *d) {
    sb o;
    sb_init(&o);
    sb_putc(&o, '[');
    if (d->cons_events.p) sb_putn(&o, d->cons_events.p, d->cons_events.n);
    sb_puts(&o, "]");
    sb_putc(&o, 0);
    return o.p;
}

int mto_pending_groups(const mto_doc *d) { return d->pend_n; }
static long copy_out(const sb *s, char *buf, long cap);
long mto_regenerated_ops(mto_doc *d, char *buf, long cap) {
    sb o;
    sb_init(&o);
    sb_putc(&o, '[');
    if (d->regen_all.n) sb_putn(&o, d->regen_all.p, d->regen_all.n);
    sb_putc(&o, ']');
    long n = copy_out(&o, buf, cap);
    sb_free(&o);
    return n;
}

static void seg_json(sb *out, int kind, const u16 *text, int len, int ref_type, const jv *props);
/* ------------------------------------------------------------------ regeneratePendingOp */
/* document order of every linked segment (the ordinal order resetPendingDeltaToOps sorts by) */
typedef struct {
    Seg **segs;
    int n, cap;
} SegList;
static void collect_segs(Block *b, SegList *l) {
    for (int i = 0; i < b->child_count; i++) {
        Node *c = b->children[i];
        if (!c->is_leaf) collect_segs((Block *)c, l);
        else {
            if (l->n == l->cap) {
                l->cap = l->cap ? 2 * l->cap : 64;
                l->segs = (Seg **)realloc(l->segs, sizeof(Seg *) * (size_t)l->cap);
            }
            l->segs[l->n++] = (Seg *)c;
        }
    }
}
static int seg_index(const SegList *l, const Seg *s) {
    for (int i = 0; i < l->n; i++)
        if (l->segs[i] == s) return i;
    return -1;
}
/* Client.findReconnectionPostition (client.ts:674-706) */
static int reconnection_position(const SegList *l, const Seg *seg, int local_seq) {
    int pos = 0;
    for (int i = 0; i < l->n && l->segs[i] != seg; i++) {
        const Seg *s = l->segs[i];
        const int inserted = s->local_seq == 0 || s->local_seq <= local_seq;
        const int not_removed = !s->removed || (s->local_removed_seq != 0 && s->local_removed_seq > local_seq);
        if (inserted && not_removed) pos += s->n.cached_length;
    }
    return pos;
}
/* Client.resetPendingDeltaToOps (client.ts:708-766): the oldest pending group regenerated against
   the current tree, one op (and one new group, queued last) per segment; ops appended to `out` as
   JSON (comma separated), returns how many */
static int reset_pending_delta_to_ops(mto_doc *d, const jv *reset_op, sb *out, int n_prev) {
    int type = -1;
    if (!reset_op || reset_op->kind != JV_OBJ || !jv_int(jv_obj_get_ascii(reset_op, "type"), &type))
        fail(d, MTO_BAD_INPUT, "regeneratePendingOp: bad op");
    if (d->pend_n == 0) fail(d, MTO_BAD_INPUT, "regeneratePendingOp: no pending segment group");
    Group *g = d->pend[d->pend_head++];
    d->pend_n--;
    SegList all = {NULL, 0, 0};
    collect_segs(d->root, &all);
    /* segmentGroup.segments.sort by ordinal (document order) */
    int *ord = (int *)malloc(sizeof(int) * (size_t)(g->n + 1));
    for (int i = 0; i < g->n; i++) ord[i] = seg_index(&all, g->segs[i]);
    for (int i = 1; i < g->n; i++) { /* insertion sort of (index, seg) pairs */
        int k = ord[i];
        Seg *sk = g->segs[i];
        int j = i - 1;
        while (j >= 0 && ord[j] > k) {
            ord[j + 1] = ord[j];
            g->segs[j + 1] = g->segs[j];
            j--;
        }
        ord[j + 1] = k;
        g->segs[j + 1] = sk;
    }
    free(ord);
    int n = n_prev;
    for (int i = 0; i < g->n; i++) {
        Seg *seg = g->segs[i];
        if (seg_group_dequeue(seg) != g) fail(d, MTO_BAD_INPUT, "Segment group not at head of segment pending queue");
        const int pos = reconnection_position(&all, seg, g->local_seq);
        char t[96];
        int made = 0;
        switch (type) {
            case 2: { /* createAnnotateRangeOp(pos, pos + len, props, combiningOp) */
                if (n++) sb_putc(out, ',');
                sb_puts(out, "{");
                const jv *co = jv_obj_get_ascii(reset_op, "combiningOp");
                if (co && co->kind != JV_UNDEF) {
                    sb_puts(out, "\"combiningOp\":");
                    jv_stringify(co, out);
                    sb_putc(out, ',');
                }
                snprintf(t, sizeof t, "\"pos1\":%d,\"pos2\":%d,\"props\":", pos, pos + seg->n.cached_length);
                sb_puts(out, t);
                const jv *pr = jv_obj_get_ascii(reset_op, "props");
                if (pr) jv_stringify(pr, out);
                else sb_puts(out, "null");
                sb_puts(out, ",\"type\":2}");
                made = 1;
                break;
            }
            case 0: /* createInsertSegmentOp(pos, segment) */
                if (seg->seq != UNASSIGNED_SEQ) fail(d, MTO_BAD_INPUT, "regenerate: insert of a sequenced segment");
                if (n++) sb_putc(out, ',');
                snprintf(t, sizeof t, "{\"pos1\":%d,\"seg\":", pos);
                sb_puts(out, t);
                seg_json(out, seg->kind, seg->text, seg->n.cached_length, seg->ref_type, seg->props);
                sb_puts(out, ",\"type\":0}");
                made = 1;
                break;
            case 1: /* createRemoveRangeOp, only while the local remove is still pending */
                if (seg->local_removed_seq != 0) {
                    if (n++) sb_putc(out, ',');
                    snprintf(t, sizeof t, "{\"pos1\":%d,\"pos2\":%d,\"type\":1}", pos, pos + seg->n.cached_length);
                    sb_puts(out, t);
                    made = 1;
                }
                break;
            default: fail(d, MTO_BAD_INPUT, "Invalid op type");
        }
        if (made) { /* a new group of this segment alone, queued last (same localSeq) */
            Group *ng = NULL;
            ng = add_to_pending_list(d, seg, NULL, g->local_seq);
            (void)ng;
        }
    }
    free(all.segs);
    return n;
}
/* regeneratePendingOp's result: the op, or createGroupOp(...opList) (client.ts:885) */
static void wrap_regenerated(sb *res, const sb *ops, int n) {
    if (n == 1) {
        sb_putn(res, ops->p, ops->n);
    } else {
        sb_puts(res, "{\"ops\":[");
        if (ops->n) sb_putn(res, ops->p, ops->n);
        sb_puts(res, "],\"type\":3}");
    }
}
/* Client.regeneratePendingOp(resetOp, segmentGroup) (client.ts:855-893) with segmentGroup = the
   oldest pending group(s): the regenerated op as JSON (a GROUP when it is more than one op), in
   *out_json (malloc'd) */
int mto_regenerate_pending_op_json(mto_doc *d, const char *reset_op_json, char **out_json) {
    *out_json = NULL;
    GUARD(d);
    jv *op = jv_parse(reset_op_json, strlen(reset_op_json));
    if (!op) fail(d, MTO_BAD_INPUT, "op is not JSON");
    sb ops;
    sb_init(&ops);
    int n = 0;
    int type = -1;
    jv_int(jv_obj_get_ascii(op, "type"), &type);
    if (type == 3) {
        const jv *members = jv_obj_get_ascii(op, "ops");
        if (!members || members->kind != JV_ARR) fail(d, MTO_BAD_INPUT, "group without ops");
        for (int i = 0; i < members->n; i++) n = reset_pending_delta_to_ops(d, members->vals[i], &ops, n);
    } else {
        n = reset_pending_delta_to_ops(d, op, &ops, 0);
    }
    sb res;
    sb_init(&res);
    wrap_regenerated(&res, &ops, n);
    if (d->regen_all_n++) sb_putc(&d->regen_all, ',');
    sb_putn(&d->regen_all, res.p, res.n);
    sb_putc(&res, 0);
    *out_json = res.p;
    sb_free(&ops);
    jv_unref(op);
    UNGUARD(d);
    return d->status;
}


int mto_apply_msg_json(mto_doc *d, const char *msg_json) {
    GUARD(d);
    jv *msg = jv_parse(msg_json, strlen(msg_json));
    if (!msg || msg->kind != JV_OBJ) fail(d, MTO_BAD_INPUT, "message is not a JSON object");
    const jv *cid = jv_obj_get_ascii(msg, "clientId");
    if (!cid || cid->kind != JV_STR) fail(d, MTO_BAD_INPUT, "clientId");
    sb name;
    sb_init(&name);
    sb_put_u16_utf8(&name, cid->s, cid->slen);
    int seq = 0, ref = 0, msn = 0;
    if (!jv_int(jv_obj_get_ascii(msg, "sequenceNumber"), &seq) ||
        !jv_int(jv_obj_get_ascii(msg, "referenceSequenceNumber"), &ref) ||
        !jv_int(jv_obj_get_ascii(msg, "minimumSequenceNumber"), &msn)) {
        sb_free(&name);
        fail(d, MTO_BAD_INPUT, "sequence numbers");
    }
    int short_id = get_or_add_short_client_id(d, name.p ? name.p : "");
    const jv *type = jv_obj_get_ascii(msg, "type");
    static const u16 OP[2] = {'o', 'p'};
    if (type && type->kind == JV_STR && u16_eq(type->s, type->slen, OP, 2)) {
        if (d->long_client_id && !strcmp(name.p ? name.p : "", d->long_client_id)) {
            ack_op_json(d, jv_obj_get_ascii(msg, "contents"), seq); /* client.ts:810-812 */
        } else {
            apply_remote_op(d, jv_obj_get_ascii(msg, "contents"), short_id, seq, ref, msn);
        }
    }
    sb_free(&name);
    update_seq_numbers(d, msn, seq);
    jv_unref(msg);
    UNGUARD(d);
    return d->status;
}

/* ------------------------------------------------------------------ SnapshotLoader */
/* SnapshotLoader.specToSegment (snapshotLoader.ts:94-125): merge info when the spec has "json" */
static Seg *spec_to_loaded_segment(mto_doc *d, const jv *spec) {
    const jv *json = (spec && spec->kind == JV_OBJ) ? jv_obj_get_ascii(spec, "json") : NULL;
    Seg *s;
    if (json) {
        s = spec_to_segment(d, json);
        const jv *cl = jv_obj_get_ascii(spec, "client");
        const jv *sq = jv_obj_get_ascii(spec, "seq");
        const jv *rs = jv_obj_get_ascii(spec, "removedSeq");
        const jv *rc = jv_obj_get_ascii(spec, "removedClient");
        sb name;
        if (cl && cl->kind != JV_UNDEF) {
            if (cl->kind != JV_STR) fail(d, MTO_BAD_INPUT, "client is not a string");
            sb_init(&name);
            sb_put_u16_utf8(&name, cl->s, cl->slen);
            s->client_id = get_or_add_short_client_id(d, name.p ? name.p : "");
            sb_free(&name);
        } else {
            s->client_id = NONCOLLAB_CLIENT;
        }
        s->seq = UNIVERSAL_SEQ;
        if (sq && sq->kind != JV_UNDEF && !jv_int(sq, &s->seq)) fail(d, MTO_BAD_INPUT, "seq");
        if (rs && rs->kind != JV_UNDEF) {
            if (!jv_int(rs, &s->removed_seq)) fail(d, MTO_BAD_INPUT, "removedSeq");
            s->removed = 1;
        }
        if (rc && rc->kind != JV_UNDEF) {
            if (rc->kind != JV_STR) fail(d, MTO_BAD_INPUT, "removedClient is not a string");
            sb_init(&name);
            sb_put_u16_utf8(&name, rc->s, rc->slen);
            s->removed_client = get_or_add_short_client_id(d, name.p ? name.p : "");
            sb_free(&name);
        }
    } else {
        s = spec_to_segment(d, spec);
        s->seq = UNIVERSAL_SEQ;
        s->client_id = NONCOLLAB_CLIENT;
    }
    return s;
}

/* MergeTree.reloadFromSegments (mergeTree.ts:1195-1251): bottom-up, MaxNodesInBlock - 1 children */
static Block *build_merge_block(mto_doc *d, Node **nodes, int n) {
    const int max_children = MAX_NODES - 1;
    const int nb = (n + max_children - 1) / max_children;
    Node **blocks = (Node **)malloc(sizeof(Node *) * (size_t)nb);
    for (int bi = 0, ni = 0; bi < nb; bi++) {
        Block *b = make_block(d, 0);
        for (int c = 0; c < max_children && ni < n; c++, ni++) {
            const int idx = b->child_count++; /* addNode, mergeTree.ts:1189-1193 */
            assign_child(b, nodes[ni], idx);
        }
        block_update(b);
        blocks[bi] = &b->n;
    }
    Block *r = nb == 1 ? (Block *)blocks[0] : build_merge_block(d, blocks, nb);
    free(blocks);
    return r;
}

static const jv *chunk_segments(mto_doc *d, const jv *chunk) {
    const jv *segs = (chunk && chunk->kind == JV_OBJ) ? jv_obj_get_ascii(chunk, "segments") : NULL;
    if (!segs || segs->kind != JV_ARR) fail(d, MTO_BAD_INPUT, "chunk without segments");
    const jv *ver = jv_obj_get_ascii(chunk, "version");
    static const u16 V1[1] = {'1'};
    if (!ver || ver->kind != JV_STR || !u16_eq(ver->s, ver->slen, V1, 1)) fail(d, MTO_UNSUPPORTED, "chunk version");
    return segs;
}

/* SnapshotLoader.initialize (snapshotLoader.ts:36-205): loadHeader -> reloadFromSegments +
   startOrUpdateCollaboration(long_id, minSeq, seq), then loadBody: body segments appended at
   the end with insertSegments, consecutive NonCollab/Universal ones in one batch */
int mto_load_snapshot_v1(mto_doc *d, const char *const *blobs, const long *blob_len, int n_blobs,
                         const char *long_id) {
    GUARD(d);
    jv *parsed[256] = {0};
    Seg **body = NULL;
    int nbody = 0;
    if (n_blobs < 1 || n_blobs > 256) fail(d, MTO_BAD_INPUT, "blob count");
    for (int i = 0; i < n_blobs; i++) {
        parsed[i] = jv_parse(blobs[i], (size_t)blob_len[i]);
        if (!parsed[i]) fail(d, MTO_BAD_INPUT, "blob %d is not JSON", i);
    }
    const jv *h = parsed[0];
    const jv *hsegs = chunk_segments(d, h);
    const jv *meta = jv_obj_get_ascii(h, "headerMetadata");
    if (!meta || meta->kind != JV_OBJ) fail(d, MTO_BAD_INPUT, "header metadata not available");
    int seq = 0, min_seq = 0, seg_count = 0, total_count = 0;
    if (!jv_int(jv_obj_get_ascii(meta, "sequenceNumber"), &seq)) fail(d, MTO_BAD_INPUT, "sequenceNumber");
    if (!jv_int(jv_obj_get_ascii(meta, "minSequenceNumber"), &min_seq)) min_seq = seq;
    jv_int(jv_obj_get_ascii(h, "segmentCount"), &seg_count);
    jv_int(jv_obj_get_ascii(meta, "totalSegmentCount"), &total_count);
    const jv *order = jv_obj_get_ascii(meta, "orderedChunkMetadata");
    const int n_chunks = (order && order->kind == JV_ARR) ? order->n : 1;
    /* loadHeader */
    Node **hn = (Node **)malloc(sizeof(Node *) * (size_t)(hsegs->n + 1));
    for (int i = 0; i < hsegs->n; i++) hn[i] = &spec_to_loaded_segment(d, hsegs->vals[i])->n;
    if (hsegs->n > 0) {
        d->root = build_merge_block(d, hn, hsegs->n);
    } else {
        d->root = make_block(d, 0);
        d->root->n.cached_length = 0;
    }
    free(hn);
    d->root->n.parent = NULL;
    d->root->n.index = 0;
    /* startOrUpdateCollaboration (client.ts:1051-1071) -> startCollaboration (1254-1271) */
    if (d->long_client_id == NULL) {
        d->long_client_id = strdup(long_id);
        d->cw.client_id = get_or_add_short_client_id(d, long_id);
        d->cw.min_seq = min_seq;
        d->cw.collaborating = 1;
        d->cw.current_seq = seq;
        heap_init(d);
    }
    /* loadBody */
    if (seg_count < total_count) {
        if (n_blobs < n_chunks) fail(d, MTO_BAD_INPUT, "missing body chunks");
        int cap = 64;
        body = (Seg **)malloc(sizeof(Seg *) * (size_t)cap);
        for (int ci = 1; ci < n_chunks; ci++) {
            const jv *segs = chunk_segments(d, parsed[ci]);
            for (int i = 0; i < segs->n; i++) {
                if (nbody == cap) {
                    cap *= 2;
                    body = (Seg **)realloc(body, sizeof(Seg *) * (size_t)cap);
                }
                body[nbody++] = spec_to_loaded_segment(d, segs->vals[i]);
            }
        }
        int bstart = 0;
        for (int i = 0; i <= nbody; i++) {
            const int batchable = i < nbody && body[i]->client_id == NONCOLLAB_CLIENT && body[i]->seq == UNIVERSAL_SEQ;
            if (batchable) continue;
            if (i > bstart)  /* flushBatch */
                insert_segments(d, d->root->n.cached_length, body + bstart, i - bstart, UNIVERSAL_SEQ,
                                NONCOLLAB_CLIENT, UNIVERSAL_SEQ);
            if (i < nbody) {
                Seg *sg = body[i];
                insert_segments(d, d->root->n.cached_length, &sg, 1, UNIVERSAL_SEQ, sg->client_id, sg->seq);
            }
            bstart = i + 1;
        }
    }
    free(body);
    for (int i = 0; i < n_blobs; i++) jv_unref(parsed[i]);
    UNGUARD(d);
    return d->status;
}

/* Client.insertSegmentLocal on a non-collaborating client (client.ts:201-210, 393-441, 485-547) */
int mto_insert_local_json(mto_doc *d, int pos, const char *seg_json) {
    GUARD(d);
    jv *spec = jv_parse(seg_json, strlen(seg_json));
    if (!spec) fail(d, MTO_BAD_INPUT, "segment spec");
    Seg *s = spec_to_segment(d, spec);
    jv_unref(spec);
    if (s->n.cached_length <= 0) {
        UNGUARD(d);
        return d->status;
    }
    if (d->cw.collaborating) fail(d, MTO_UNSUPPORTED, "local edits on a collaborating client");
    int len = d->root->n.cached_length;
    if (pos < 0 || pos > len) fail(d, MTO_INVALID_POS, "InvalidOpRange");
    insert_segment(d, pos, s, d->cw.current_seq, d->cw.client_id, UNIVERSAL_SEQ);
    UNGUARD(d);
    return d->status;
}

int mto_annotate_local_json(mto_doc *d, int start, int end, const char *props_json) {
    GUARD(d);
    if (d->cw.collaborating) fail(d, MTO_UNSUPPORTED, "local edits on a collaborating client");
    int len = d->root->n.cached_length;
    if (start < 0 || start >= len || end <= start) fail(d, MTO_INVALID_POS, "InvalidOpRange");
    jv *props = jv_parse(props_json, strlen(props_json));
    if (!props) fail(d, MTO_BAD_INPUT, "props");
    annotate_range(d, start, end, props, 0, NULL, d->cw.current_seq, d->cw.client_id, UNIVERSAL_SEQ);
    jv_unref(props);
    UNGUARD(d);
    return d->status;
}

int mto_remove_local(mto_doc *d, int start, int end) {
    GUARD(d);
    if (d->cw.collaborating) fail(d, MTO_UNSUPPORTED, "local edits on a collaborating client");
    int len = d->root->n.cached_length;
    if (start < 0 || start >= len || end <= start) fail(d, MTO_INVALID_POS, "InvalidOpRange");
    mark_range_removed(d, start, end, d->cw.current_seq, d->cw.client_id, UNIVERSAL_SEQ);
    UNGUARD(d);
    return d->status;
}

int mto_get_length(mto_doc *d) { return d->root->n.cached_length; }
int mto_view_length(mto_doc *d, int ref_seq, int short_client) { return block_length(d, d->root, ref_seq, short_client); }
int mto_current_seq(mto_doc *d) { return d->cw.current_seq; }
int mto_min_seq(mto_doc *d) { return d->cw.min_seq; }

/* ------------------------------------------------------------------ read-out */
typedef struct {
    sb *out;
} TextCtx;
/* MergeTreeTextHelper.gatherText (textSegment.ts:188-275) with placeholder "" over the
   full local view */
static int gather_text(mto_doc *d, Seg *s, int pos, int r, int c, int start, int end, void *vctx) {
    (void)d; (void)pos; (void)r; (void)c;
    TextCtx *ctx = (TextCtx *)vctx;
    if (s->kind == SEG_TEXT) {
        int len = s->n.cached_length;
        int a = start < 0 ? 0 : start;
        int b = end >= len ? len : end;
        if (start <= 0 && end >= len) { a = 0; b = len; }
        sb_put_u16_utf8(ctx->out, s->text + a, b - a);
    }
    return 1;
}

static void build_text(mto_doc *d, sb *out) {
    TextCtx ctx = {out};
    MapActions a = {gather_text, NULL, &ctx};
    int len = block_length(d, d->root, d->cw.current_seq, d->cw.client_id);
    node_map(d, d->root, &a, 0, d->cw.current_seq, d->cw.client_id, 0, len, 1);
}

static long copy_out(const sb *s, char *buf, long cap) {
    long n = (long)s->n;
    if (buf && cap > 0) {
        long m = n < cap - 1 ? n : cap - 1;
        if (m > 0) memcpy(buf, s->p, (size_t)m);
        buf[m] = 0;
    }
    return n;
}

long mto_get_text(mto_doc *d, char *buf, long cap) {
    sb s;
    sb_init(&s);
    build_text(d, &s);
    long n = copy_out(&s, buf, cap);
    sb_free(&s);
    return n;
}

static void seg_props_json(const Seg *s, sb *out) {
    if (!s->props) sb_puts(out, "null");
    else {
        sb t;
        sb_init(&t);
        jv_stringify(s->props, &t);
        /* re-quote the JSON text as a JSON string (UTF-8 bytes pass through as-is below) */
        sb_putc(out, '"');
        for (size_t i = 0; i < t.n; i++) {
            char ch = t.p[i];
            if (ch == '"' || ch == '\\') sb_putc(out, '\\');
            sb_putc(out, ch);
        }
        sb_putc(out, '"');
        sb_free(&t);
    }
}

typedef struct {
    sb *out;
    int pos;
    int run_start, run_len;
    sb run_props;
    int first;
} RunCtx;

static void flush_run(RunCtx *c) {
    if (c->run_len <= 0) return;
    if (!c->first) sb_putc(c->out, ',');
    c->first = 0;
    char t[64];
    snprintf(t, sizeof t, "[%d,%d,", c->run_start, c->run_len);
    sb_puts(c->out, t);
    sb_putn(c->out, c->run_props.p, c->run_props.n);
    sb_putc(c->out, ']');
}

static int gather_runs(mto_doc *d, Seg *s, int pos, int r, int cl, int start, int end, void *vctx) {
    (void)d; (void)pos; (void)r; (void)cl; (void)start; (void)end;
    RunCtx *c = (RunCtx *)vctx;
    int len = s->n.cached_length;
    sb pj;
    sb_init(&pj);
    seg_props_json(s, &pj);
    if (c->run_len > 0 && pj.n == c->run_props.n && !memcmp(pj.p, c->run_props.p, pj.n)) {
        c->run_len += len;
    } else {
        flush_run(c);
        sb_free(&c->run_props);
        c->run_props = pj;
        c->run_start = c->pos;
        c->run_len = len;
        pj.p = NULL;
    }
    sb_free(&pj);
    c->pos += len;
    return 1;
}

long mto_props_runs(mto_doc *d, char *buf, long cap) {
    sb out;
    sb_init(&out);
    sb_putc(&out, '[');
    RunCtx c;
    memset(&c, 0, sizeof c);
    c.out = &out;
    c.first = 1;
    sb_init(&c.run_props);
    MapActions a = {gather_runs, NULL, &c};
    int len = block_length(d, d->root, d->cw.current_seq, d->cw.client_id);
    node_map(d, d->root, &a, 0, d->cw.current_seq, d->cw.client_id, 0, len, 1);
    flush_run(&c);
    sb_free(&c.run_props);
    sb_putc(&out, ']');
    long n = copy_out(&out, buf, cap);
    sb_free(&out);
    return n;
}

/* UTF-8 -> UTF-16 code units (invalid sequences -> U+FFFD) */
static u16 *utf8_to_u16(const char *s, int *n) {
    size_t L = strlen(s);
    u16 *out = (u16 *)malloc(sizeof(u16) * (L * 2 + 1));
    int k = 0;
    const unsigned char *q = (const unsigned char *)s;
    size_t i = 0;
    while (i < L) {
        uint32_t c = q[i];
        int len = 1;
        if (c < 0x80) len = 1;
        else if ((c & 0xE0) == 0xC0) { len = 2; c &= 0x1F; }
        else if ((c & 0xF0) == 0xE0) { len = 3; c &= 0x0F; }
        else if ((c & 0xF8) == 0xF0) { len = 4; c &= 0x07; }
        else { out[k++] = 0xFFFD; i++; continue; }
        if (i + (size_t)len > L) { out[k++] = 0xFFFD; break; }
        int bad = 0;
        for (int m = 1; m < len; m++) {
            if ((q[i + m] & 0xC0) != 0x80) { bad = 1; break; }
            c = (c << 6) | (q[i + m] & 0x3F);
        }
        if (bad) { out[k++] = 0xFFFD; i++; continue; }
        i += (size_t)len;
        if (c >= 0x10000) {
            c -= 0x10000;
            out[k++] = (u16)(0xD800 + (c >> 10));
            out[k++] = (u16)(0xDC00 + (c & 0x3FF));
        } else {
            out[k++] = (u16)c;
        }
    }
    *n = k;
    return out;
}

static void put_json_string_utf8(sb *out, const char *s) {
    int n;
    u16 *u = utf8_to_u16(s, &n);
    js_quote(out, u, n);
    free(u);
}

/* ------------------------------------------------------------------ SnapshotV1 (snapshotV1.ts) */
typedef struct {
    sb json; /* serialized JsonSegmentSpecs */
    int len;
} SnapSeg;

typedef struct {
    SnapSeg *p;
    int n, cap;
} SnapVec;

static void snap_push(SnapVec *v, sb json, int len) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 64;
        v->p = (SnapSeg *)realloc(v->p, sizeof(SnapSeg) * (size_t)v->cap);
    }
    v->p[v->n].json = json;
    v->p[v->n].len = len;
    v->n++;
}

/* segment.toJSONObject(): TextSegment (textSegment.ts:48-54), Marker (mergeTree.ts:652-656) */
static void seg_json(sb *out, int kind, const u16 *text, int len, int ref_type, const jv *props) {
    if (kind == SEG_TEXT) {
        if (props) {
            sb_puts(out, "{\"text\":");
            js_quote(out, text, len);
            sb_puts(out, ",\"props\":");
            jv_stringify(props, out);
            sb_putc(out, '}');
        } else {
            js_quote(out, text, len);
        }
    } else {
        char t[64];
        snprintf(t, sizeof t, "{\"marker\":{\"refType\":%d}", ref_type);
        sb_puts(out, t);
        if (props) {
            sb_puts(out, ",\"props\":");
            jv_stringify(props, out);
        }
        sb_putc(out, '}');
    }
}

/* coalescing candidate `prev` (a clone when coalesced: snapshotV1.ts:191-210) */
typedef struct {
    int active;
    int kind, ref_type;
    u16 *text;
    int len, cap;
    const jv *props;
} Prev;

static void prev_push(SnapVec *v, Prev *p) {
    if (!p->active) return;
    sb j;
    sb_init(&j);
    seg_json(&j, p->kind, p->text, p->len, p->ref_type, p->props);
    snap_push(v, j, p->len);
    p->active = 0;
}

static void prev_set(Prev *p, const Seg *s) {
    p->active = 1;
    p->kind = s->kind;
    p->ref_type = s->ref_type;
    p->len = 0;
    if (s->kind == SEG_TEXT) {
        if (p->cap < s->n.cached_length) {
            p->cap = s->n.cached_length + 64;
            p->text = (u16 *)realloc(p->text, sizeof(u16) * (size_t)p->cap);
        }
        memcpy(p->text, s->text, sizeof(u16) * (size_t)s->n.cached_length);
    }
    p->len = s->n.cached_length;
    p->props = s->props;
}

typedef struct {
    mto_doc *d;
    SnapVec *segs;
    Prev prev;
    int min_seq;
} ExtractCtx;

static void extract_segment(ExtractCtx *c, const Seg *s) { /* snapshotV1.ts:175-240 */
    int min_seq = c->min_seq;
    if (s->seq == UNASSIGNED_SEQ || (s->removed && s->removed_seq <= min_seq)) return;
    if (s->seq <= min_seq && (!s->removed || s->removed_seq == UNASSIGNED_SEQ)) {
        if (!c->prev.active) {
            prev_set(&c->prev, s);
        } else {
            /* prev.canAppend(segment) && matchProperties(prev.properties, segment.properties) */
            int can = c->prev.kind == SEG_TEXT && s->kind == SEG_TEXT &&
                      !(c->prev.len > 0 && c->prev.text[c->prev.len - 1] == '\n') &&
                      (c->prev.len <= TEXT_GRANULARITY || s->n.cached_length <= TEXT_GRANULARITY);
            if (can && jv_match_properties(c->prev.props, s->props)) {
                int need = c->prev.len + s->n.cached_length;
                if (need > c->prev.cap) {
                    c->prev.cap = need * 2;
                    c->prev.text = (u16 *)realloc(c->prev.text, sizeof(u16) * (size_t)c->prev.cap);
                }
                memcpy(c->prev.text + c->prev.len, s->text, sizeof(u16) * (size_t)s->n.cached_length);
                c->prev.len = need;
            } else {
                prev_push(c->segs, &c->prev);
                prev_set(&c->prev, s);
            }
        }
    } else {
        prev_push(c->segs, &c->prev);
        sb j;
        sb_init(&j);
        sb_puts(&j, "{\"json\":");
        seg_json(&j, s->kind, s->text, s->n.cached_length, s->ref_type, s->props);
        char t[64];
        if (s->seq > min_seq) {
            snprintf(t, sizeof t, ",\"seq\":%d,\"client\":", s->seq);
            sb_puts(&j, t);
            put_json_string_utf8(&j, get_long_client_id(c->d, s->client_id));
        }
        if (s->removed) {
            snprintf(t, sizeof t, ",\"removedSeq\":%d,\"removedClient\":", s->removed_seq);
            sb_puts(&j, t);
            put_json_string_utf8(&j, get_long_client_id(c->d, s->removed_client));
        }
        sb_putc(&j, '}');
        snap_push(c->segs, j, s->n.cached_length);
    }
}

static void walk_all_segments(Block *b, ExtractCtx *c) { /* mergeTree.ts:2969-2983 */
    for (int i = 0; i < b->child_count; i++) {
        Node *n = b->children[i];
        if (n->is_leaf) extract_segment(c, (Seg *)n);
        else walk_all_segments((Block *)n, c);
    }
}

static void add_blob(mto_doc *d, const char *name, sb content) {
    d->blob_names = (char **)realloc(d->blob_names, sizeof(char *) * (size_t)(d->n_blobs + 1));
    d->blobs = (sb *)realloc(d->blobs, sizeof(sb) * (size_t)(d->n_blobs + 1));
    d->blob_names[d->n_blobs] = strdup(name);
    d->blobs[d->n_blobs] = content;
    d->n_blobs++;
}

int mto_snapshot_v1(mto_doc *d, int chunk_size) {
    if (chunk_size <= 0) chunk_size = 10000; /* SnapshotV1.chunkSize, snapshotV1.ts:40 */
    free_blobs(d);
    SnapVec segs = {0, 0, 0};
    ExtractCtx c;
    memset(&c, 0, sizeof c);
    c.d = d;
    c.segs = &segs;
    c.min_seq = d->cw.min_seq;
    walk_all_segments(d->root, &c);
    prev_push(&segs, &c.prev);
    free(c.prev.text);

    /* emit (snapshotV1.ts:85-149) + getSeqLengthSegs (57-79) */
    typedef struct { int start, count, length; } Chunk;
    Chunk *chunks = NULL;
    int nch = 0;
    int total_count = 0, total_length = 0;
    do {
        int length = 0, count = 0;
        while (length < chunk_size && total_count + count < segs.n) {
            length += segs.p[total_count + count].len;
            count++;
        }
        chunks = (Chunk *)realloc(chunks, sizeof(Chunk) * (size_t)(nch + 1));
        chunks[nch].start = total_count;
        chunks[nch].count = count;
        chunks[nch].length = length;
        nch++;
        total_count += count;
        total_length += length;
    } while (total_count < segs.n);

    for (int ci = 0; ci < nch; ci++) {
        sb j;
        sb_init(&j);
        char t[128];
        snprintf(t, sizeof t, "{\"version\":\"1\",\"segmentCount\":%d,\"length\":%d,\"segments\":[", chunks[ci].count,
                 chunks[ci].length);
        sb_puts(&j, t);
        for (int k = 0; k < chunks[ci].count; k++) {
            if (k) sb_putc(&j, ',');
            SnapSeg *s = &segs.p[chunks[ci].start + k];
            sb_putn(&j, s->json.p, s->json.n);
        }
        snprintf(t, sizeof t, "],\"startIndex\":%d", chunks[ci].start);
        sb_puts(&j, t);
        if (ci == 0) {
            snprintf(t, sizeof t, ",\"headerMetadata\":{\"minSequenceNumber\":%d,\"sequenceNumber\":%d,"
                                  "\"orderedChunkMetadata\":[{\"id\":\"header\"}",
                     d->cw.min_seq, d->cw.current_seq);
            sb_puts(&j, t);
            for (int b = 1; b < nch; b++) {
                snprintf(t, sizeof t, ",{\"id\":\"body_%d\"}", b - 1);
                sb_puts(&j, t);
            }
            snprintf(t, sizeof t, "],\"totalLength\":%d,\"totalSegmentCount\":%d}", total_length, total_count);
            sb_puts(&j, t);
        }
        sb_putc(&j, '}');
        if (ci == 0) add_blob(d, "header", j);
        else {
            snprintf(t, sizeof t, "body_%d", ci - 1);
            add_blob(d, t, j);
        }
    }
    free(chunks);
    for (int i = 0; i < segs.n; i++) sb_free(&segs.p[i].json);
    free(segs.p);
    return d->n_blobs;
}

long mto_snapshot_blob(mto_doc *d, int i, char *name, long name_cap, char *buf, long cap) {
    if (i < 0 || i >= d->n_blobs) return -1;
    if (name && name_cap > 0) {
        snprintf(name, (size_t)name_cap, "%s", d->blob_names[i]);
    }
    return copy_out(&d->blobs[i], buf, cap);
}

/* ------------------------------------------------------------------ shape / dump / digest */
static int tree_depth(const Block *b) {
    int depth = 1;
    while (b->child_count > 0 && !b->children[0]->is_leaf) {
        b = (const Block *)b->children[0];
        depth++;
    }
    return depth;
}

typedef struct {
    sb *out;
    int first;
} ShapeCtx;
static void shape_walk(const Block *b, int level, int leaf_level, ShapeCtx *c) {
    if (level == leaf_level) {
        char t[16];
        snprintf(t, sizeof t, "%s%d", c->first ? "" : ",", b->child_count);
        sb_puts(c->out, t);
        c->first = 0;
        return;
    }
    for (int i = 0; i < b->child_count; i++) shape_walk((const Block *)b->children[i], level + 1, leaf_level, c);
}

long mto_shape(mto_doc *d, char *buf, long cap) {
    sb out;
    sb_init(&out);
    int depth = tree_depth(d->root);
    char t[32];
    snprintf(t, sizeof t, "D%d:", depth);
    sb_puts(&out, t);
    ShapeCtx c = {&out, 1};
    shape_walk(d->root, 1, depth, &c);
    long n = copy_out(&out, buf, cap);
    sb_free(&out);
    return n;
}

typedef struct {
    uint64_t h;
} Fnv;
static void fnv_bytes(Fnv *f, const void *p, size_t n) {
    const unsigned char *q = (const unsigned char *)p;
    for (size_t i = 0; i < n; i++) {
        f->h ^= q[i];
        f->h *= 0x100000001b3ull;
    }
}
static void fnv_u32(Fnv *f, uint32_t x) {
    unsigned char b[4] = {(unsigned char)x, (unsigned char)(x >> 8), (unsigned char)(x >> 16), (unsigned char)(x >> 24)};
    fnv_bytes(f, b, 4);
}

static uint64_t fnv_name(const char *name) {
    Fnv f = {0xcbf29ce484222325ull};
    fnv_bytes(&f, name, strlen(name));
    return f.h;
}
static void fnv_u64(Fnv *f, uint64_t x) {
    fnv_u32(f, (uint32_t)x);
    fnv_u32(f, (uint32_t)(x >> 32));
}

/* State digest (DESIGN.md "State digest"): client ids enter by long name, so the digest does
   not depend on how short ids were numbered. */
static void digest_walk(mto_doc *d, const Block *b, int level, int leaf_level, Fnv *f) {
    if (level == leaf_level) {
        fnv_u32(f, 0xB10CB10Cu);
        fnv_u32(f, (uint32_t)b->child_count);
        for (int i = 0; i < b->child_count; i++) {
            const Seg *s = (const Seg *)b->children[i];
            uint64_t ovl = 0;
            for (int k = 0; k < s->novl; k++) ovl += fnv_name(get_long_client_id(d, s->ovl[k]));
            fnv_u32(f, (uint32_t)s->kind);
            fnv_u32(f, (uint32_t)s->n.cached_length);
            fnv_u32(f, (uint32_t)s->seq);
            fnv_u64(f, fnv_name(get_long_client_id(d, s->client_id)));
            fnv_u32(f, s->removed ? (uint32_t)s->removed_seq : 0xFFFFFFFFu);
            fnv_u64(f, s->removed ? fnv_name(get_long_client_id(d, s->removed_client)) : 0ull);
            fnv_u64(f, ovl);
            if (!s->props) {
                fnv_u32(f, 0xFFFFFFFFu);
            } else {
                sb t;
                sb_init(&t);
                jv_stringify(s->props, &t);
                fnv_u32(f, (uint32_t)t.n);
                fnv_bytes(f, t.p, t.n);
                sb_free(&t);
            }
            if (s->kind == SEG_TEXT) {
                for (int k = 0; k < s->n.cached_length; k++) {
                    unsigned char b2[2] = {(unsigned char)s->text[k], (unsigned char)(s->text[k] >> 8)};
                    fnv_bytes(f, b2, 2);
                }
            } else {
                fnv_u32(f, (uint32_t)s->ref_type);
            }
        }
        return;
    }
    for (int i = 0; i < b->child_count; i++) digest_walk(d, (const Block *)b->children[i], level + 1, leaf_level, f);
}

uint64_t mto_state_digest(mto_doc *d) {
    Fnv f = {0xcbf29ce484222325ull};
    int depth = tree_depth(d->root);
    fnv_u32(&f, (uint32_t)depth);
    digest_walk(d, d->root, 1, depth, &f);
    fnv_u32(&f, (uint32_t)d->cw.min_seq);
    fnv_u32(&f, (uint32_t)d->cw.current_seq);
    fnv_u32(&f, (uint32_t)d->status);
    return f.h;
}

static void dump_walk(mto_doc *d, const Block *b, sb *out, int depth) {
    for (int i = 0; i < b->child_count; i++) {
        const Node *n = b->children[i];
        if (!n->is_leaf) {
            char t[64];
            snprintf(t, sizeof t, "%*sB(%d)\n", depth * 2, "", ((const Block *)n)->child_count);
            sb_puts(out, t);
            dump_walk(d, (const Block *)n, out, depth + 1);
        } else {
            const Seg *s = (const Seg *)n;
            char t[160];
            char rs[16] = "none";
            if (s->removed) snprintf(rs, sizeof rs, "%d", s->removed_seq);
            snprintf(t, sizeof t, "%*sS len=%d seq=%d cli=%d rseq=%s rcli=%d novl=%d ", depth * 2, "",
                     s->n.cached_length, s->seq, s->client_id, rs, s->removed ? s->removed_client : -1, s->novl);
            sb_puts(out, t);
            if (s->sg_n > 0) {
                snprintf(t, sizeof t, "grp=%d ", s->sg_n);
                sb_puts(out, t);
            }
            if (s->kind == SEG_MARKER) {
                snprintf(t, sizeof t, "rt=%d ", s->ref_type);
                sb_puts(out, t);
            }
            sb_putc(out, '\'');
            if (s->kind == SEG_TEXT) sb_put_u16_utf8(out, s->text, s->n.cached_length);
            sb_puts(out, "'");
            if (s->props) {
                sb_putc(out, ' ');
                jv_stringify(s->props, out);
            }
            sb_putc(out, '\n');
        }
    }
}

long mto_dump(mto_doc *d, char *buf, long cap) {
    sb out;
    sb_init(&out);
    char t[96];
    snprintf(t, sizeof t, "root(%d) min=%d cur=%d heap=%d\n", d->root->child_count, d->cw.min_seq, d->cw.current_seq,
             heap_count(d));
    sb_puts(&out, t);
    dump_walk(d, d->root, &out, 1);
    long n = copy_out(&out, buf, cap);
    sb_free(&out);
    return n;
}

/* ------------------------------------------------------------------ packed logs */
mto_tables *mto_tables_new(const char *const *key_names, int n_keys, const char *const *value_json, int n_values) {
    mto_tables *t = (mto_tables *)calloc(1, sizeof(mto_tables));
    t->n_keys = n_keys;
    t->keys = (char **)calloc((size_t)n_keys + 1, sizeof(char *));
    t->keys16 = (u16 **)calloc((size_t)n_keys + 1, sizeof(u16 *));
    t->keylen16 = (int *)calloc((size_t)n_keys + 1, sizeof(int));
    for (int i = 0; i < n_keys; i++) {
        t->keys[i] = strdup(key_names[i]);
        t->keys16[i] = utf8_to_u16(key_names[i], &t->keylen16[i]);
    }
    t->n_values = n_values;
    t->values = (jv **)calloc((size_t)n_values + 1, sizeof(jv *));
    for (int i = 0; i < n_values; i++) {
        if (i == 0 || !value_json[i]) t->values[i] = jv_new(JV_NULL);
        else {
            t->values[i] = jv_parse(value_json[i], strlen(value_json[i]));
            if (!t->values[i]) t->values[i] = jv_new(JV_NULL);
        }
    }
    return t;
}

void mto_tables_free(mto_tables *t) {
    if (!t) return;
    for (int i = 0; i < t->n_keys; i++) {
        free(t->keys[i]);
        free(t->keys16[i]);
    }
    for (int i = 0; i < t->n_values; i++) jv_unref(t->values[i]);
    free(t->keys);
    free(t->keys16);
    free(t->keylen16);
    free(t->values);
    free(t);
}

/* a value of a packed record as the message's JSON.parse would give it: objects are per-op objects
   (consensus may update one in place), so they are copied, not shared through the table */
static jv *value_from_record(mto_doc *d, uint32_t v, const mto_tables *t) {
    if (v == MT_VALUE_UNDEFINED) return NULL;
    if ((int)v >= t->n_values) fail(d, MTO_BAD_INPUT, "prop id out of range");
    return jv_deep_clone(t->values[v]);
}
static jv *props_from_records(mto_doc *d, const mt_prop *p, uint32_t n, const mto_tables *t) {
    jv *o = jv_new(JV_OBJ);
    for (uint32_t i = 0; i < n; i++) {
        if ((int)p[i].key >= t->n_keys || (int)p[i].value >= t->n_values) {
            jv_unref(o);
            fail(d, MTO_BAD_INPUT, "prop id out of range");
        }
        jv_obj_set(o, t->keys16[p[i].key], t->keylen16[p[i].key], value_from_record(d, p[i].value, t));
    }
    return o;
}

/* an annotate record's combiningOp (mt_oplog.h: defaultValue / minValue records after the props) */
static void combine_of_records(mto_doc *d, const mt_op *op, const mt_prop *props, const mto_tables *t, CombineOp *co) {
    co->kind = (int)MT_OPF_COMBINE(op->flags);
    co->def = co->min = NULL;
    if (!co->kind) return;
    const mt_prop *x = props + op->payload + op->payload_len;
    if (x[0].key != MT_KEY_COMBINE || x[1].key != MT_KEY_COMBINE) fail(d, MTO_BAD_INPUT, "combiningOp records");
    co->def = value_from_record(d, x[0].value, t);
    co->min = value_from_record(d, x[1].value, t);
}
/* a packed RELPOS: posFromRelativePos of the next record's positions (client.ts:485-502) */
static void relpos_packed(mto_doc *d, const mt_op *op, const mto_tables *t, int ref_seq, int client_id) {
    d->rel_pending = 0;
    for (int k = 0; k < 2; k++) {
        const uint32_t f = op->flags;
        if (!(f & (k ? MT_RELF_POS2 : MT_RELF_POS1))) continue;
        const uint32_t idv = (uint32_t)(k ? op->pos2 : op->pos1);
        jv *rel = jv_new(JV_OBJ);
        if (idv) jv_obj_set_ascii(rel, "id", value_from_record(d, idv, t));
        if (f & (k ? MT_RELF_BEFORE2 : MT_RELF_BEFORE1)) jv_obj_set_ascii(rel, "before", jv_new(JV_TRUE));
        if (f & (k ? MT_RELF_OFF2 : MT_RELF_OFF1))
            jv_obj_set_ascii(rel, "offset", jv_new_num((double)(int32_t)(k ? op->payload_len : op->payload)));
        const int pos = pos_from_relative_pos(d, rel, ref_seq, client_id);
        jv_unref(rel);
        if (k) d->rel_pos2 = pos;
        else d->rel_pos1 = pos;
        d->rel_pending |= 1 << k;
    }
}

/* a packed local op (seq == -1, client 0): see apply_local_op_json */
static void apply_local_packed(mto_doc *d, const mt_op *op, const uint16_t *text, const mt_prop *props,
                               const mto_tables *t) {
    const uint32_t bits = MT_OPF_BITS(op->flags);
    const int ref = d->cw.current_seq, cid = d->cw.client_id;
    if (op->type == MT_OP_RELPOS) {
        relpos_packed(d, op, t, ref, cid);
        free(d->ntf_key);
        d->ntf_key = NULL;
        d->ntf_marker = NULL;
        if (op->flags & MT_RELF_NOTIFY) { /* annotateMarkerNotifyConsensus: getMarkerFromId(id) */
            jv *id = value_from_record(d, op->payload, t);
            if (!jv_truthy(id)) fail(d, MTO_BAD_INPUT, "notifyConsensus without a marker id");
            int kl;
            u16 *k = js_key_of(id, &kl);
            d->ntf_marker = id_lookup(d, k, kl);
            free(k);
            d->ntf_key = jv_json_text(id);
            jv_unref(id);
        }
        return;
    }
    char *ntf_key = d->ntf_key;
    Seg *ntf_marker = d->ntf_marker;
    d->ntf_key = NULL;
    d->ntf_marker = NULL;
    mt_op rop;
    if (d->rel_pending) {
        rop = *op;
        if (d->rel_pending & 1) rop.pos1 = d->rel_pos1;
        if (d->rel_pending & 2) rop.pos2 = d->rel_pos2;
        d->rel_pending = 0;
        op = &rop;
    }
    if (ntf_key && !(op->type == MT_OP_ANNOTATE && MT_OPF_COMBINE(op->flags) == MT_COMBINE_CONSENSUS)) {
        free(ntf_key);
        fail(d, MTO_BAD_INPUT, "notifyConsensus on an op that is not a consensus annotate");
    }
    switch (op->type) {
        case MT_OP_INSERT: {
            if (!local_range_valid(d, 0, op->pos1, 0, 0)) return;
            Seg *s;
            if (bits & MT_OPF_MARKER) s = new_marker(d, (int)op->payload);
            else s = new_text_seg(d, text + op->payload, (int)op->payload_len);
            if (bits & MT_OPF_HAS_PROPS) {
                uint32_t p0 = 0;
                const uint32_t np = mt_insert_props(op, props, &p0); /* MT_OPF_NPROPS_EXT: any count */
                jv *pr = props_from_records(d, props + p0, (int)np, t);
                seg_add_properties(d, s, pr, 0, NULL, 0, 0);
                jv_unref(pr);
            }
            insert_segment(d, op->pos1, s, ref, cid, UNASSIGNED_SEQ);
            break;
        }
        case MT_OP_REMOVE:
            if (!local_range_valid(d, 1, op->pos1, 1, op->pos2)) return;
            mark_range_removed(d, op->pos1, op->pos2, ref, cid, UNASSIGNED_SEQ);
            break;
        case MT_OP_ANNOTATE: {
            if (!local_range_valid(d, 2, op->pos1, 1, op->pos2)) {
                free(ntf_key);
                return;
            }
            jv *pr = props_from_records(d, props + op->payload, op->payload_len, t);
            CombineOp co;
            combine_of_records(d, op, props, t, &co);
            annotate_range(d, op->pos1, op->pos2, pr, (bits & MT_OPF_REWRITE) ? 1 : 0, co.kind ? &co : NULL, ref, cid,
                           UNASSIGNED_SEQ);
            jv_unref(pr);
            jv_unref(co.def);
            jv_unref(co.min);
            if (ntf_key && ntf_marker) cons_register(d, ntf_key, ntf_marker);
            free(ntf_key);
            break;
        }
        case MT_OP_REGENERATE: { /* regeneratePendingOp of one reset op (member) */
            jv *reset = jv_new(JV_OBJ);
            jv_obj_set_ascii(reset, "type", jv_new_num(op->ref_seq));
            if (op->ref_seq == MT_OP_ANNOTATE) {
                if (bits & MT_OPF_REWRITE) {
                    jv *co = jv_new(JV_OBJ);
                    jv_obj_set_ascii(co, "name", jv_new_str_ascii("rewrite"));
                    jv_obj_set_ascii(reset, "combiningOp", co);
                }
                jv_obj_set_ascii(reset, "props", props_from_records(d, props + op->payload, op->payload_len, t));
            }
            d->regen_cur_n = reset_pending_delta_to_ops(d, reset, &d->regen_cur, d->regen_cur_n);
            jv_unref(reset);
            if (!(bits & MT_OPF_GROUP_CONT)) {
                if (d->regen_all_n++) sb_putc(&d->regen_all, ',');
                wrap_regenerated(&d->regen_all, &d->regen_cur, d->regen_cur_n);
                d->regen_cur.n = 0;
                d->regen_cur_n = 0;
            }
            break;
        }
        default: fail(d, MTO_BAD_INPUT, "local op type %d", op->type);
    }
}

static void apply_packed_one(mto_doc *d, const mt_op *op, const uint16_t *text, const mt_prop *props,
                             const mto_tables *t, const char *const *client_names, int n_clients) {
    const int oc = (int)MT_OP_CLIENT(*op); /* 15-bit short id: high bits in flags 11-13 (mt_oplog.h) */
    if (oc >= n_clients || oc >= MT_MAX_CLIENTS + 2) fail(d, MTO_BAD_INPUT, "client index out of range");
    int sid = d->pk_map[oc];
    if (sid < 0) {
        sid = get_or_add_short_client_id(d, client_names[oc]); /* applyMsg registration */
        d->pk_map[oc] = sid;
    }
    uint32_t bits = MT_OPF_BITS(op->flags);
    if (op->seq == UNASSIGNED_SEQ) { /* a local op of this replica (mt_oplog.h "local ops") */
        if (sid != d->cw.client_id) fail(d, MTO_BAD_INPUT, "local op of another client");
        apply_local_packed(d, op, text, props, t);
        return;
    }
    if (op->type != MT_OP_NOOP && d->long_client_id && sid == d->cw.client_id) {
        /* the replica's own sequenced message: ack (client.ts:810-812); positions are not read */
        if (op->type != MT_OP_RELPOS) {
            jv *pr = NULL;
            if (op->type == MT_OP_ANNOTATE) pr = props_from_records(d, props + op->payload, op->payload_len, t);
            ack_pending_segment(d, op->type, pr, op->type == MT_OP_ANNOTATE && (bits & MT_OPF_REWRITE), op->seq);
            if (op->type == MT_OP_ANNOTATE && MT_OPF_COMBINE(op->flags) == MT_COMBINE_CONSENSUS) {
                /* updateConsensusProperty: pos1 = relativePos1.id's value id (0: none to match) */
                CombineOp co;
                combine_of_records(d, op, props, t, &co);
                jv *rel = jv_new(JV_OBJ);
                if (op->pos1) jv_obj_set_ascii(rel, "id", value_from_record(d, (uint32_t)op->pos1, t));
                update_consensus_property(d, rel, pr, &co, op->seq);
                jv_unref(rel);
                jv_unref(co.def);
                jv_unref(co.min);
            }
            jv_unref(pr);
        }
        if (!(bits & MT_OPF_GROUP_CONT)) update_seq_numbers(d, op->msn, op->seq);
        return;
    }
    mt_op rop;
    if (d->rel_pending && op->type != MT_OP_RELPOS) { /* positions resolved by the RELPOS record */
        rop = *op;
        if (d->rel_pending & 1) rop.pos1 = d->rel_pos1;
        if (d->rel_pending & 2) rop.pos2 = d->rel_pos2;
        d->rel_pending = 0;
        op = &rop;
    }
    switch (op->type) {
        case MT_OP_INSERT: {
            Seg *s;
            if (bits & MT_OPF_MARKER) s = new_marker(d, (int)op->payload);
            else s = new_text_seg(d, text + op->payload, (int)op->payload_len);
            if (bits & MT_OPF_HAS_PROPS) {
                uint32_t p0 = 0;
                const uint32_t np = mt_insert_props(op, props, &p0); /* MT_OPF_NPROPS_EXT: any count */
                jv *pr = props_from_records(d, props + p0, (int)np, t);
                seg_add_properties(d, s, pr, 0, NULL, 0, 0);
                jv_unref(pr);
            }
            insert_segment(d, op->pos1, s, op->ref_seq, sid, op->seq);
            complete_remote_op(d, op->seq, op->msn);
            break;
        }
        case MT_OP_REMOVE:
            mark_range_removed(d, op->pos1, op->pos2, op->ref_seq, sid, op->seq);
            complete_remote_op(d, op->seq, op->msn);
            break;
        case MT_OP_ANNOTATE: {
            jv *pr = props_from_records(d, props + op->payload, op->payload_len, t);
            CombineOp co;
            combine_of_records(d, op, props, t, &co);
            annotate_range(d, op->pos1, op->pos2, pr, (bits & MT_OPF_REWRITE) ? 1 : 0, co.kind ? &co : NULL,
                           op->ref_seq, sid, op->seq);
            jv_unref(pr);
            jv_unref(co.def);
            jv_unref(co.min);
            complete_remote_op(d, op->seq, op->msn);
            break;
        }
        case MT_OP_RELPOS: /* getValidOpRange of the next record (client.ts:485-502) */
            relpos_packed(d, op, t, op->ref_seq, sid);
            break;
        case MT_OP_NOOP: break;
        default: fail(d, MTO_BAD_INPUT, "op type %d", op->type);
    }
    if (!(bits & MT_OPF_GROUP_CONT)) update_seq_numbers(d, op->msn, op->seq);
}

int mto_apply_packed(mto_doc *d, const mt_op *ops, long n_ops, const uint16_t *text, const mt_prop *props,
                     const mto_tables *t, const char *const *client_names, int n_clients) {
    if (d->status != MTO_OK) return d->status;
    if (!d->cw.collaborating) {
        mto_start_collab(d, client_names[0], 0, 0);
        d->pk_map[0] = d->cw.client_id;
    }
    GUARD(d);
    for (long i = 0; i < n_ops; i++) apply_packed_one(d, &ops[i], text, props, t, client_names, n_clients);
    UNGUARD(d);
    return d->status;
}

/* ------------------------------------------------------------------ generator */
static const char *GEN_KEYS[MT_GEN_N_KEYS] = {"bold", "italic", "color", "size"};
static const char *GEN_COLORS[3] = {"\"red\"", "\"green\"", "\"blue\""};
static const char *GEN_CLIENTS[] = {"readonly", "A", "B", "C", "D", "E", "F", "G", "H", "I", "J", "K", "L", "M",
                                    "N", "O", "P", "Q", "R", "S", "T", "U", "V", "W", "X", "Y", "Z"};
static char GEN_SIZES[17][4];

const char *mto_gen_key_name(int k) { return (k >= 0 && k < MT_GEN_N_KEYS) ? GEN_KEYS[k] : NULL; }
const char *mto_gen_value_json(int v) {
    if (v == 0) return "null";
    if (v == 1) return "true";
    if (v >= 2 && v <= 4) return GEN_COLORS[v - 2];
    if (v >= 5 && v < MT_GEN_N_VALUES) {
        snprintf(GEN_SIZES[v - 5], sizeof GEN_SIZES[0], "%d", v - 5 + 8);
        return GEN_SIZES[v - 5];
    }
    return NULL;
}
const char *mto_gen_client_name(int i) {
    return (i >= 0 && i < (int)(sizeof GEN_CLIENTS / sizeof GEN_CLIENTS[0])) ? GEN_CLIENTS[i] : NULL;
}

static const char GEN_ALPHABET[] = "abcdefghijklmnopqrstuvwxyz ";

int mto_gen_doc(const mt_gen_params *p, long doc, mt_op *ops_out, uint16_t *text_out, long text_cap, long *text_len,
                mt_prop *props_out, long props_cap, long *n_props) {
    if (p->n_clients < 1 || p->n_clients > 26) return MTO_BAD_INPUT;
    static mto_tables *tables = NULL;
    static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    pthread_mutex_lock(&mu);
    if (!tables) {
        const char *vals[MT_GEN_N_VALUES];
        for (int v = 0; v < MT_GEN_N_VALUES; v++) vals[v] = mto_gen_value_json(v);
        tables = mto_tables_new(GEN_KEYS, MT_GEN_N_KEYS, vals, MT_GEN_N_VALUES);
    }
    pthread_mutex_unlock(&mu);

    mto_doc *d = mto_new();
    mto_start_collab(d, GEN_CLIENTS[0], 0, 0);
    d->pk_map[0] = d->cw.client_id;
    uint64_t x = mt_rng_seed(p->seed, (uint64_t)doc);
    int last_ref[64];
    for (int c = 0; c <= p->n_clients; c++) last_ref[c] = 0;
    long tl = 0, np = 0;
    int st = MTO_OK;
    for (int k = 1; k <= p->n_ops; k++) {
        mt_op op;
        memset(&op, 0, sizeof op);
        int seq = k;
        int c = 1 + (int)mt_rng_below(&x, (uint32_t)p->n_clients);
        int lag = (int)mt_rng_below(&x, (uint32_t)p->max_lag + 1);
        int ref = seq - 1 - lag;
        if (ref < last_ref[c]) ref = last_ref[c];
        last_ref[c] = ref;
        int msn = last_ref[1];
        for (int i = 2; i <= p->n_clients; i++)
            if (last_ref[i] < msn) msn = last_ref[i];
        /* view length of the issuer: MergeTree.getLength(refSeq, clientId) */
        int sid = d->pk_map[c];
        int len;
        if (sid < 0) {
            /* not yet registered: nodeLength compares ids only; an unknown id sees no own segments */
            len = block_length(d, d->root, ref, 1000 + c);
        } else {
            len = block_length(d, d->root, ref, sid);
        }
        uint32_t u = mt_rng_below(&x, 100);
        int type;
        if (len < p->min_len || (int)u < p->pct_insert) type = MT_OP_INSERT;
        else if ((int)u < p->pct_insert + p->pct_remove) type = MT_OP_REMOVE;
        else type = MT_OP_ANNOTATE;
        op.type = (uint16_t)type;
        op.client = (uint16_t)c;
        op.seq = seq;
        op.ref_seq = ref;
        op.msn = msn;
        if (type == MT_OP_INSERT) {
            int pos = (int)mt_rng_below(&x, (uint32_t)len + 1);
            int n = 1 + (int)mt_rng_below(&x, (uint32_t)p->max_insert);
            if (tl + n > text_cap) { st = MTO_BAD_INPUT; break; }
            op.pos1 = pos;
            op.pos2 = 0;
            op.payload = (uint32_t)tl;
            op.payload_len = (uint32_t)n;
            for (int i = 0; i < n; i++) {
                uint32_t r = mt_rng_below(&x, 100);
                u16 ch = (int)r < p->pct_newline ? (u16)'\n' : (u16)GEN_ALPHABET[mt_rng_below(&x, 27)];
                text_out[tl++] = ch;
            }
        } else {
            int rl = 1;
            while (rl < len && mt_rng_below(&x, 4) != 0) rl++;
            int start = (int)mt_rng_below(&x, (uint32_t)(len - rl + 1));
            op.pos1 = start;
            op.pos2 = start + rl;
            if (type == MT_OP_ANNOTATE) {
                int nk = 1 + (int)mt_rng_below(&x, 2);
                int k0 = (int)mt_rng_below(&x, 4);
                int keys[2] = {k0, (k0 + 1 + (int)mt_rng_below(&x, 3)) % 4};
                if (np + nk > props_cap) { st = MTO_BAD_INPUT; break; }
                op.payload = (uint32_t)np;
                op.payload_len = (uint32_t)nk;
                for (int i = 0; i < nk; i++) {
                    uint32_t v;
                    if (mt_rng_below(&x, 10) == 0) v = 0;
                    else if (keys[i] <= 1) v = 1;
                    else if (keys[i] == 2) v = 2 + mt_rng_below(&x, 3);
                    else v = 5 + mt_rng_below(&x, 17);
                    props_out[np].key = (uint32_t)keys[i];
                    props_out[np].value = v;
                    np++;
                }
            }
        }
        ops_out[k - 1] = op;
        /* replay as the observer (text/props arrays are the doc-relative buffers) */
        const char *const *names = GEN_CLIENTS;
        mto_apply_packed(d, &op, 1, text_out, props_out, tables, names, p->n_clients + 1);
        if (d->status != MTO_OK) { st = d->status; break; }
    }
    *text_len = tl;
    *n_props = np;
    mto_free(d);
    return st;
}

/* ------------------------------------------------------------------ batch replay (CPU baseline) */
typedef struct {
    const mt_op *ops;
    const int64_t *off;
    long n_docs;
    const uint16_t *text;
    const mt_prop *props;
    const mto_tables *t;
    const char *const *names;
    int n_clients;
    uint64_t *digests;
    int32_t *status;
    long next;
    pthread_mutex_t mu;
} BatchJob;

static void *batch_worker(void *arg) {
    BatchJob *j = (BatchJob *)arg;
    for (;;) {
        long dd = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (dd >= j->n_docs) break;
        mto_doc *d = mto_new();
        mto_apply_packed(d, j->ops + j->off[dd], (long)(j->off[dd + 1] - j->off[dd]), j->text, j->props, j->t, j->names,
                         j->n_clients);
        if (j->digests) j->digests[dd] = mto_state_digest(d);
        if (j->status) j->status[dd] = d->status;
        mto_free(d);
    }
    return NULL;
}

double mto_replay_batch(const mt_op *ops, const int64_t *doc_op_off, long n_docs, const uint16_t *text,
                        const mt_prop *props, const mto_tables *t, const char *const *client_names, int n_clients,
                        int n_threads, uint64_t *digests_out, int32_t *status_out) {
    BatchJob j;
    memset(&j, 0, sizeof j);
    j.ops = ops;
    j.off = doc_op_off;
    j.n_docs = n_docs;
    j.text = text;
    j.props = props;
    j.t = t;
    j.names = client_names;
    j.n_clients = n_clients;
    j.digests = digests_out;
    j.status = status_out;
    if (n_threads < 1) n_threads = 1;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)n_threads);
    for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, batch_worker, &j);
    for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

void mto_free_string(char *p) { free(p); }
