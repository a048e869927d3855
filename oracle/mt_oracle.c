/*
 * TEST INFRASTRUCTURE ONLY -- CPU restatement of the reference merge-tree observer replay.
 *
 * This is the checker for the HIP path, not part of the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.  It deliberately keeps
 * the reference's *pointer B-tree* structure (blocks of <= MaxNodesInBlock-1 children,
 * recursive walks, binary-heap zamboni) so that it is an independent restatement of the
 * algorithm the GPU path re-derives as flat scans.  Every function cites the reference
 * (paths relative to /root/reference/packages/dds/merge-tree/src/, "MT/").
 *
 * Parity pin: oracle/ref_harness.mjs runs the reference itself (transpiled by
 * oracle/build_ref.py) and tests/golden/ holds its outputs; tests/test_oracle.py checks
 * this file against them.
 *
 * Scope: the replica of SURVEY.md Appendix A as a participant whose own short id is 0 --
 * remote messages, and (live-client path) the local client's own unsequenced
 * ops (MT_F_LOCAL records) and their acks (MT_F_ACK); an observer is the participant that
 * submits nothing; reconnects regenerate the pending ops (orc_regenerate).  All branch ids
 * 0, no local references, no tracking groups.
 */
#include "mt_oracle.h"

#include <limits.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define MAXN 8                 /* MaxNodesInBlock               MT/mergeTree.ts:333 */
#define TEXT_GRANULARITY 256   /* MergeTree.TextSegmentGranularity MT/mergeTree.ts:1093 */
#define ZAMBONI_MAX 2          /* MergeTree.zamboniSegmentsMaxCount MT/mergeTree.ts:1095 */
#define RSEQ_NONE INT32_MIN    /* removedSeq === undefined */
#define OBSERVER 0             /* collabWindow.clientId of the observer */
#define UNASSIGNED (-1)        /* UnassignedSequenceNumber       MT/constants.ts:12 */
#define SCOUR_UNDEF (-1)       /* needsScour === undefined */

typedef struct Props {
    int n, cap;
    uint32_t *key, *val;
} Props;

struct Block;
typedef struct Node {
    int leaf;
    struct Block *parent;
    int index;
} Node;

struct Group;
typedef struct Seg {
    Node n;
    int32_t len, seq, client, rseq, rclient;
    int novl, ovlcap;
    int32_t *ovl;          /* removedClientOverlap, push order */
    int32_t marker;        /* -1: TextSegment, else Marker refType */
    uint16_t *text;
    int tcap;
    Props *props;          /* NULL == properties undefined */
    /* SegmentPropertiesManager (MT/segmentPropertiesManager.ts:12-14): pendingKeyUpdateCount
       (key -> count) and pendingRewriteCount; allocated with the property set */
    Props *pk;
    int32_t prw;
    /* segmentGroups (SegmentGroupCollection, MT/segmentGroupCollection.ts): FIFO of the
       pending local-op groups the segment belongs to, oldest at ghead */
    struct Group **grp;
    int ghead, gn, gcap;
    int32_t lseq, lrseq;   /* localSeq / localRemovedSeq (RSEQ_NONE: undefined) */
    int32_t ord;           /* document order (regeneration's ordinal sort) */
} Seg;

/* SegmentGroup {segments, localSeq} (MT/mergeTree.ts:96-99); pendingSegments is a FIFO of
   them (the doc's pend_head .. pend_tail) */
typedef struct Group {
    Seg **segs;
    int n, cap;
    int32_t local_seq;
    struct Group *next;
} Group;

typedef struct Block {
    Node n;
    int count;
    Node *ch[MAXN + 1];
    int needs_scour;       /* -1 undefined, 0 false, 1 true */
    /* cached aggregates of the subtree (the restatement's stand-in for the reference's
       cachedLength + PartialSequenceLengths, MT/mergeTree.ts:1692-1732, partialLengths.ts):
       c_obs = its length in the local client's view (sum of localNetLength), c_chg = the
       largest seq / removedSeq in it (INT32_MAX for an unacked one), so every view with
       refSeq >= c_chg sees exactly c_obs; valid while c_ok (cleared up the parent chain by
       every change below, blk_dirty) */
    int32_t c_obs, c_chg;
    int c_ok;
} Block;

typedef struct HeapEnt {
    int32_t max_seq;
    Seg *seg;
} HeapEnt;

typedef struct Vec {
    void **p;
    int n, cap;
} Vec;

typedef struct IVec {
    int32_t *p;
    int64_t n, cap;
} IVec;

struct orc_doc {
    Block *root;
    int32_t min_seq, current_seq;
    int32_t status;
    HeapEnt *heap;         /* 1-based like Collections.Heap MT/collections.ts:212-265 */
    int heap_n, heap_cap;
    Vec allocs;
    int record;
    IVec dlog;             /* optional flattened delta records */
    uint64_t delta_hash;
    uint32_t maint[3];     /* mergeTreeMaintenanceCallback events: SPLIT, APPEND, UNLINK */
    int32_t local_seq;     /* collabWindow.localSeq */
    Group *pend_head, *pend_tail;   /* pendingSegments */
    int32_t n_pend;
    int64_t ovl_units, ovl_peak;   /* sum over segments in the tree of removedClientOverlap
                                      lists as [n, ids...] (n + 1 units each) and its maximum
                                      after a message (tests: the device's overflow arena) */
    Seg **segv;            /* the segments in document order (read-outs by index), valid while */
    int32_t segv_n, segv_cap, segv_ok;   /* segv_ok: cleared by every mutating entry point */
};

typedef void (*seg_fn)(Seg *, void *);
static void walk_segs(Node *n, seg_fn fn, void *arg);

/* ------------------------------------------------------------------ utilities */
static void vec_push(Vec *v, void *x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 64;
        v->p = (void **)realloc(v->p, sizeof(void *) * v->cap);
    }
    v->p[v->n++] = x;
}
static void ivec_push(IVec *v, int32_t x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 256;
        v->p = (int32_t *)realloc(v->p, sizeof(int32_t) * v->cap);
    }
    v->p[v->n++] = x;
}
static void *dalloc(orc_doc *d, size_t sz) {
    void *p = calloc(1, sz);
    vec_push(&d->allocs, p);
    return p;
}

#define FNV_OFF 1469598103934665603ULL
#define FNV_PRIME 1099511628211ULL
static inline uint64_t fnv_u32(uint64_t h, uint32_t x) {
    for (int i = 0; i < 4; i++) {
        h ^= (x >> (8 * i)) & 0xFF;
        h *= FNV_PRIME;
    }
    return h;
}

/* ------------------------------------------------------------------ properties */
static Props *props_new(orc_doc *d) {
    Props *p = (Props *)dalloc(d, sizeof(Props));
    return p;
}
static int props_find(const Props *p, uint32_t key) {
    for (int i = 0; i < p->n; i++)
        if (p->key[i] == key) return i;
    return -1;
}
static void props_set(orc_doc *d, Props *p, uint32_t key, uint32_t val) {
    int i = props_find(p, key);
    if (i >= 0) {
        p->val[i] = val;
        return;
    }
    if (p->n == p->cap) {
        int nc = p->cap ? p->cap * 2 : 4;
        uint32_t *k = (uint32_t *)dalloc(d, sizeof(uint32_t) * nc);
        uint32_t *v = (uint32_t *)dalloc(d, sizeof(uint32_t) * nc);
        if (p->n) {
            memcpy(k, p->key, sizeof(uint32_t) * p->n);
            memcpy(v, p->val, sizeof(uint32_t) * p->n);
        }
        p->key = k;
        p->val = v;
        p->cap = nc;
    }
    p->key[p->n] = key;
    p->val[p->n] = val;
    p->n++;
}
static void props_del(Props *p, uint32_t key) {  /* `delete obj[key]` keeps order of rest */
    int i = props_find(p, key);
    if (i < 0) return;
    for (int j = i + 1; j < p->n; j++) {
        p->key[j - 1] = p->key[j];
        p->val[j - 1] = p->val[j];
    }
    p->n--;
}
static Props *props_clone(orc_doc *d, const Props *src) {
    if (!src) return NULL;
    Props *p = props_new(d);
    for (int i = 0; i < src->n; i++) props_set(d, p, src->key[i], src->val[i]);
    return p;
}
/* Properties.matchProperties MT/properties.ts:61-92 (value ids are canonical, so deep
   equality of values == id equality). */
static int match_props(const Props *a, const Props *b) {
    if (a) {
        if (!b) return 0;
        for (int i = 0; i < a->n; i++) {
            int j = props_find(b, a->key[i]);
            /* NaN !== NaN; an undefined member fails `b[key] === undefined` */
            if (j < 0 || b->val[j] != a->val[i] || (a->val[i] & MT_VAL_NOMATCH_BIT)) return 0;
        }
        for (int j = 0; j < b->n; j++)
            if (props_find(a, b->key[j]) < 0) return 0;
        return 1;
    }
    return b ? 0 : 1;
}

/* ------------------------------------------------------------------ tree nodes */
static Block *make_block(orc_doc *d, int count) {   /* MergeTree.makeBlock :1148-1157 */
    Block *b = (Block *)dalloc(d, sizeof(Block));
    b->n.leaf = 0;
    b->count = count;
    b->needs_scour = SCOUR_UNDEF;
    return b;
}
static Seg *make_text_seg(orc_doc *d, const uint16_t *text, int32_t len) {
    Seg *s = (Seg *)dalloc(d, sizeof(Seg));
    s->n.leaf = 1;
    s->len = len;
    s->seq = 0;               /* UniversalSequenceNumber  MT/mergeTree.ts:433 */
    s->client = -1;           /* LocalClientId            MT/mergeTree.ts:432 */
    s->rseq = RSEQ_NONE;
    s->lseq = s->lrseq = RSEQ_NONE;
    s->marker = -1;
    s->tcap = len > 0 ? len : 1;
    s->text = (uint16_t *)malloc(sizeof(uint16_t) * s->tcap);
    vec_push(&d->allocs, s->text);
    if (len) memcpy(s->text, text, sizeof(uint16_t) * len);
    return s;
}
/* a block's children or a leaf below it changed: its cached aggregates and its ancestors'
   are stale (a stale block's ancestors are always stale, so the walk stops at the first one) */
static void blk_dirty(Block *b) {
    for (; b && b->c_ok; b = b->n.parent) b->c_ok = 0;
}
static inline void seg_dirty(Seg *s) { blk_dirty(s->n.parent); }
static void assign_child(Block *b, Node *child, int index) {  /* assignChild :374-381 */
    blk_dirty(b);
    child->parent = b;
    child->index = index;
    b->ch[index] = child;
}
static int ovl_has(const Seg *s, int32_t c) {
    for (int i = 0; i < s->novl; i++)
        if (s->ovl[i] == c) return 1;
    return 0;
}
static void ovl_push(orc_doc *d, Seg *s, int32_t c) {   /* addOverlappingClient :2577-2585 */
    if (s->novl == s->ovlcap) {
        int nc = s->ovlcap ? s->ovlcap * 2 : 4;
        int32_t *p = (int32_t *)dalloc(d, sizeof(int32_t) * nc);
        if (s->novl) memcpy(p, s->ovl, sizeof(int32_t) * s->novl);
        s->ovl = p;
        s->ovlcap = nc;
    }
    s->ovl[s->novl++] = c;
    if (s->n.parent) d->ovl_units += s->novl == 1 ? 2 : 1;   /* (a split's right half: parent set first) */
}

/* SegmentGroupCollection.enqueue MT/segmentGroupCollection.ts:26-29: the group joins the
   segment's FIFO and the segment the group's list */
static void group_enqueue(orc_doc *d, Seg *s, Group *g) {
    if (s->ghead + s->gn == s->gcap) {
        int nc = s->gcap ? s->gcap * 2 : 4;
        Group **p = (Group **)dalloc(d, sizeof(Group *) * nc);
        if (s->gn) memcpy(p, s->grp + s->ghead, sizeof(Group *) * s->gn);
        s->grp = p;
        s->gcap = nc;
        s->ghead = 0;
    }
    s->grp[s->ghead + s->gn++] = g;
    if (g->n == g->cap) {
        int nc = g->cap ? g->cap * 2 : 8;
        Seg **p = (Seg **)dalloc(d, sizeof(Seg *) * nc);
        if (g->n) memcpy(p, g->segs, sizeof(Seg *) * g->n);
        g->segs = p;
        g->cap = nc;
    }
    g->segs[g->n++] = s;
}

/* addToPendingList :1955-1962: the op's first segment opens its group at the queue's tail */
static void add_to_pending(orc_doc *d, Seg *s, Group **g, int32_t local_seq) {
    if (!*g) {
        Group *ng = (Group *)dalloc(d, sizeof(Group));
        ng->local_seq = local_seq;
        if (d->pend_tail)
            d->pend_tail->next = ng;
        else
            d->pend_head = ng;
        d->pend_tail = ng;
        d->n_pend++;
        *g = ng;
    }
    group_enqueue(d, s, *g);
}

/* localNetLength :1195-1206 */
static inline int32_t local_net_length(const Seg *s) {
    return s->rseq != RSEQ_NONE ? 0 : s->len;
}

/* A leaf's term in its ancestors' PartialSequenceLengths for a remote view (client, refSeq).
   The partials (MT/partialLengths.ts fromLeaves :208-259 / insertSegment :286-336 / combine
   :88-207) record +len at the segment's seq and -len at its removedSeq under the remover, and
   under every overlapping remover in clientSeqNumbers (addClientSeqNumberFromPartial
   :581-590); getBranchPartialLength (:455-486) takes every entry at or below refSeq (latestLEQ
   :31-47) plus the client's own entries above it.  So a segment adds len when it is inserted
   in the view (seq <= refSeq or its own client) and subtracts len when it is removed in the
   view (removedSeq <= refSeq, or removed / overlap-removed by the client) -- independently:
   a segment the view sees removed but not inserted counts -len.  That happens only in views
   below the client's latest refSeq ("stale"); elsewhere a removal implies the insert, and the
   term equals the leaf's nodeLength. */
static int32_t seg_partial(const Seg *s, int32_t ref_seq, int32_t client) {
    const int ins = s->client == client || (s->seq != UNASSIGNED && s->seq <= ref_seq);
    const int rem = s->rseq != RSEQ_NONE && (s->rclient == client || ovl_has(s, client) ||
                                             (s->rseq != UNASSIGNED && s->rseq <= ref_seq));
    return s->len * (ins - rem);
}
static inline int32_t seg_chg(const Seg *s) {
    int32_t c = s->seq == UNASSIGNED ? INT32_MAX : s->seq;
    if (s->rseq != RSEQ_NONE) {
        const int32_t r = s->rseq == UNASSIGNED ? INT32_MAX : s->rseq;
        if (r > c) c = r;
    }
    return c;
}
static void blk_refresh(Block *b) {
    if (b->c_ok) return;
    int32_t obs = 0, chg = INT32_MIN;
    for (int i = 0; i < b->count; i++) {
        const Node *c = b->ch[i];
        if (c->leaf) {
            const Seg *s = (const Seg *)c;
            obs += local_net_length(s);
            const int32_t x = seg_chg(s);
            if (x > chg) chg = x;
        } else {
            Block *cb = (Block *)c;
            blk_refresh(cb);
            obs += cb->c_obs;
            if (cb->c_chg > chg) chg = cb->c_chg;
        }
    }
    b->c_obs = obs;
    b->c_chg = chg;
    b->c_ok = 1;
}
/* A block's partial length for a remote view: the sum of its leaves' terms -- equal to its
   local length when every segment below was inserted (and removed, if it is) at or below
   refSeq: then each term is len * (1 - removed) = localNetLength. */
static int32_t block_partial(const Block *b, int32_t ref_seq, int32_t client) {
    blk_refresh((Block *)b);
    if (b->c_chg <= ref_seq) return b->c_obs;
    int32_t sum = 0;
    for (int i = 0; i < b->count; i++)
        sum += b->ch[i]->leaf ? seg_partial((const Seg *)b->ch[i], ref_seq, client)
                              : block_partial((const Block *)b->ch[i], ref_seq, client);
    return sum;
}

#ifdef ORC_CACHE_CHECK
/* the aggregates recomputed from the leaves (cache check builds: tests of the caching) */
static int32_t node_len_slow(const Node *n, int32_t ref_seq, int32_t client) {
    if (n->leaf) {
        const Seg *s = (const Seg *)n;
        return client == OBSERVER ? local_net_length(s) : seg_partial(s, ref_seq, client);
    }
    const Block *b = (const Block *)n;
    int32_t sum = 0;
    for (int i = 0; i < b->count; i++) sum += node_len_slow(b->ch[i], ref_seq, client);
    return sum;
}
#endif
/* nodeLength :1692-1732.  Interior nodes read PartialSequenceLengths.getPartialLength
   (blockLength :1664-1670): the sum of their leaves' partial terms (seg_partial); leaves
   their visibility in the view. */
static int32_t node_len(const Node *n, int32_t ref_seq, int32_t client) {
    if (!n->leaf) {
        const Block *b = (const Block *)n;
        int32_t r;
        if (client != OBSERVER) {
            r = block_partial(b, ref_seq, client);
        } else {
            blk_refresh((Block *)b);
            r = b->c_obs;
        }
#ifdef ORC_CACHE_CHECK
        if (r != node_len_slow(n, ref_seq, client)) abort();
#endif
        return r;
    }
    const Seg *s = (const Seg *)n;
    if (client == OBSERVER) return local_net_length(s);
    if (s->client == client || (s->seq != UNASSIGNED && s->seq <= ref_seq)) {
        if (s->rseq != RSEQ_NONE) {
            if (s->rclient == client || ovl_has(s, client) ||
                (s->rseq != UNASSIGNED && s->rseq <= ref_seq))
                return 0;
            return s->len;
        }
        return s->len;
    }
    return 0;
}

/* getPosition :1619-1636 (always in the observer's view here) */
static int32_t get_position(const Node *node) {
    int32_t total = 0;
    const Block *parent = node->parent;
    const Node *prev = node;
    while (parent) {
        for (int i = 0; i < parent->count; i++) {
            const Node *c = parent->ch[i];
            if (c == prev) break;
            total += node_len(c, 0, OBSERVER);
        }
        prev = &parent->n;
        parent = parent->n.parent;
    }
    return total;
}

/* ------------------------------------------------------------------ zamboni heap */
static void heap_swap(HeapEnt *a, HeapEnt *b) {
    HeapEnt t = *a;
    *a = *b;
    *b = t;
}
static void heap_add(orc_doc *d, Seg *s, int32_t max_seq) {   /* Heap.add/fixup */
    if (d->heap_n + 2 > d->heap_cap) {
        d->heap_cap = d->heap_cap ? d->heap_cap * 2 : 64;
        d->heap = (HeapEnt *)realloc(d->heap, sizeof(HeapEnt) * d->heap_cap);
    }
    int k = ++d->heap_n;
    d->heap[k].max_seq = max_seq;
    d->heap[k].seg = s;
    while (k > 1 && d->heap[k >> 1].max_seq - d->heap[k].max_seq > 0) {
        heap_swap(&d->heap[k >> 1], &d->heap[k]);
        k >>= 1;
    }
}
static HeapEnt heap_get(orc_doc *d) {   /* Heap.get/fixdown MT/collections.ts:227-262 */
    HeapEnt x = d->heap[1];
    d->heap[1] = d->heap[d->heap_n];
    d->heap_n--;
    int k = 1;
    while ((k << 1) <= d->heap_n) {
        int j = k << 1;
        if (j < d->heap_n && d->heap[j].max_seq - d->heap[j + 1].max_seq > 0) j++;
        if (d->heap[k].max_seq - d->heap[j].max_seq <= 0) break;
        heap_swap(&d->heap[k], &d->heap[j]);
        k = j;
    }
    return x;
}

/* addToLRUSet :1306-1316 */
static void add_to_lru(orc_doc *d, Seg *s, int32_t seq) {
    if (s->n.parent->needs_scour != 1 && seq > d->current_seq) {
        s->n.parent->needs_scour = 1;
        heap_add(d, s, seq);
    }
}

/* TextSegment.canAppend MT/textSegment.ts:63-68 (Marker.canAppend is false :827-829) */
static int can_append(const Seg *prev, const Seg *s) {
    if (prev->marker >= 0) return 0;
    if (prev->len > 0 && prev->text[prev->len - 1] == '\n') return 0;
    if (s->marker >= 0) return 0;
    return prev->len <= TEXT_GRANULARITY || s->len <= TEXT_GRANULARITY;
}
/* TextSegment.append :74-85 */
static void seg_append(orc_doc *d, Seg *prev, const Seg *s) {
    if (prev->len + s->len > prev->tcap) {
        int nc = (prev->len + s->len) * 2;
        uint16_t *t = (uint16_t *)dalloc(d, sizeof(uint16_t) * nc);
        memcpy(t, prev->text, sizeof(uint16_t) * prev->len);
        prev->text = t;
        prev->tcap = nc;
    }
    memcpy(prev->text + prev->len, s->text, sizeof(uint16_t) * s->len);
    prev->len += s->len;
    seg_dirty(prev);
}

/* scourNode :1322-1398 */
static void scour_node(orc_doc *d, Block *node, Node **hold, int *nhold) {
    Seg *prev = NULL;
    for (int k = 0; k < node->count; k++) {
        Node *child = node->ch[k];
        if (child->leaf) {
            Seg *s = (Seg *)child;
            if (s->gn) {                           /* a pending segment stays :1328 */
                hold[(*nhold)++] = child;
                prev = NULL;
            } else if (s->rseq != RSEQ_NONE) {
                if (s->rseq > d->min_seq) {
                    hold[(*nhold)++] = child;
                } else {
                    blk_dirty(s->n.parent);
                    if (s->novl) d->ovl_units -= s->novl + 1;
                    s->n.parent = NULL;            /* unlink */
                    d->maint[2]++;                 /* UNLINK :1343-1348 */
                }
                prev = NULL;
            } else if (s->seq <= d->min_seq) {
                int ok = prev && can_append(prev, s) && match_props(prev->props, s->props) &&
                         local_net_length(s) > 0;
                if (ok) {
                    seg_append(d, prev, s);
                    blk_dirty(s->n.parent);
                    s->n.parent = NULL;
                    d->maint[1]++;                 /* APPEND :1368-1373 */
                } else {
                    hold[(*nhold)++] = child;
                    prev = local_net_length(s) > 0 ? s : NULL;
                }
            } else {
                hold[(*nhold)++] = child;
                prev = NULL;
            }
        } else {
            hold[(*nhold)++] = child;
            prev = NULL;
        }
    }
}

/* pack :1401-1453 */
static void pack(orc_doc *d, Block *block) {
    Block *parent = block->n.parent;
    Node *hold[MAXN * MAXN + 8];
    int nhold = 0;
    for (int ci = 0; ci < parent->count; ci++) {
        Block *cb = (Block *)parent->ch[ci];
        scour_node(d, cb, hold, &nhold);
        blk_dirty(parent);
        cb->n.parent = NULL;
    }
    int total = nhold;
    int half = MAXN / 2;
    int child_count = total / half;
    if (child_count > MAXN - 1) child_count = MAXN - 1;
    if (child_count < 1) child_count = 1;
    int base = total / child_count;
    int extra = total % child_count;
    int read = 0;
    for (int ni = 0; ni < child_count; ni++) {
        int cnt = base;
        if (extra > 0) {
            cnt++;
            extra--;
        }
        Block *pb = make_block(d, cnt);
        for (int j = 0; j < cnt; j++) assign_child(pb, hold[read++], j);
        pb->n.parent = parent;
        assign_child(parent, &pb->n, ni);
    }
    parent->count = child_count;
    blk_dirty(parent);
    if (parent->count < MAXN / 2 && parent->n.parent) pack(d, parent);
}

/* zamboniSegments :1455-1511 */
static void zamboni(orc_doc *d) {
    for (int i = 0; i < ZAMBONI_MAX; i++) {
        if (d->heap_n == 0 || d->heap[1].max_seq > d->min_seq) break;
        HeapEnt e = heap_get(d);
        Block *block = e.seg->n.parent;
        if (block && block->needs_scour != 0) {
            Node *hold[MAXN + 1];
            int nhold = 0;
            scour_node(d, block, hold, &nhold);
            block->needs_scour = 0;
            if (nhold < block->count) {
                blk_dirty(block);
                block->count = nhold;
                for (int j = 0; j < nhold; j++) assign_child(block, hold[j], j);
                if (block->count < MAXN / 2 && block->n.parent) pack(d, block);
            }
        }
    }
}

static Block theUnfinishedNode;   /* MergeTree.theUnfinishedNode */
#define UNFINISHED (&theUnfinishedNode)

/* split :2509-2522 */
static Block *split_block(orc_doc *d, Block *node) {
    int half = MAXN / 2;
    Block *nb = make_block(d, half);
    blk_dirty(node);
    node->count = half;
    for (int i = 0; i < half; i++) {
        assign_child(nb, node->ch[half + i], i);
        node->ch[half + i] = NULL;
    }
    return nb;
}
/* updateRoot :1909-1920 */
static void update_root(orc_doc *d, Block *split_node) {
    if (split_node && split_node != UNFINISHED) {
        Block *nr = make_block(d, 2);
        assign_child(nr, &d->root->n, 0);
        assign_child(nr, &split_node->n, 1);
        nr->n.parent = NULL;
        d->root = nr;
    }
}

/* BaseSegment.splitAt :523-567 + TextSegment.createSplitSegmentAt MT/textSegment.ts:103-111
   + SegmentPropertiesManager.copyTo MT/segmentPropertiesManager.ts:113-128 */
static Seg *split_at(orc_doc *d, Seg *s, int32_t pos) {
    if (!(pos > 0) || s->marker >= 0) return NULL;
    Seg *r = make_text_seg(d, s->text + pos, s->len - pos);
    s->len = pos;
    seg_dirty(s);
    r->props = props_clone(d, s->props);
    if (s->props) {                                  /* copyTo: the pending counts too */
        r->pk = props_clone(d, s->pk);
        r->prw = s->prw;
    }
    r->n.parent = s->n.parent;
    r->rclient = s->rclient;
    r->rseq = s->rseq;
    r->seq = s->seq;
    r->client = s->client;
    r->lseq = s->lseq;
    r->lrseq = s->lrseq;
    for (int i = 0; i < s->novl; i++) ovl_push(d, r, s->ovl[i]);
    /* segmentGroups.copyTo :26-38: the right half joins every group of the left one */
    for (int i = 0; i < s->gn; i++) group_enqueue(d, r, s->grp[s->ghead + i]);
    return r;
}

/* breakTie :2281-2310 (remote client: never the collab window's own client) */
static int break_tie(int32_t pos, const Node *node, int32_t ref_seq, int32_t client) {
    if (node->leaf) {
        if (pos == 0) {
            const Seg *s = (const Seg *)node;
            if (s->rseq != RSEQ_NONE && s->rseq != 0 && s->rseq <= ref_seq && s->rseq != UNASSIGNED)
                return 0;
            if (client == OBSERVER) return 1;
            if (s->seq != UNASSIGNED) return 1;
        }
        return 0;
    }
    return 1;
}

enum { WALK_SPLIT = 0, WALK_INSERT = 1 };

/* the first segment the local client sees inside a block: nodeMap(block, 0,
   UniversalSequenceNumber, collab client) stopping at its first leaf action (:2936-2998) */
static Seg *first_visible(Block *b) {
    for (int i = 0; i < b->count; i++) {
        Node *c = b->ch[i];
        if (node_len(c, 0, OBSERVER) <= 0) continue;
        if (c->leaf) return (Seg *)c;
        Seg *s = first_visible((Block *)c);
        if (s) return s;
    }
    return NULL;
}
/* blockInsert's continuePredicate continueFrom (:2176-2194) = rightExcursion (:2346-2376)
   with checkSegmentIsLocal: the first segment after `node` -- a following sibling leaf
   whatever its length, else the first one the local client sees in a following block,
   climbing the parents -- is an unacked local insert */
static int continue_from(Block *node) {
    Node *start = &node->n;
    Block *parent = node->n.parent;
    while (parent) {
        int matched = 0;
        for (int i = 0; i < parent->count; i++) {
            Node *c = parent->ch[i];
            if (matched) {
                if (c->leaf) return ((Seg *)c)->seq == UNASSIGNED;
                Seg *s = first_visible((Block *)c);
                if (s) return s->seq == UNASSIGNED;
            } else {
                matched = c == start;
            }
        }
        start = &parent->n;
        parent = parent->n.parent;
    }
    return 0;
}


/* insertingWalk :2378-2507 with leaf = splitLeafSegment (:2258-2272) or onLeaf
   (:2213-2223); a sequenced insert that reaches a block's end at pos 0 continues past it
   when the next segment is an unacked local insert (continuePredicate). */
static Block *inserting_walk(orc_doc *d, Block *block, int32_t pos, int32_t ref_seq,
                             int32_t client, int mode, Seg *cand, int32_t seq) {
    int ci;
    Node *new_node = NULL;
    for (ci = 0; ci < block->count; ci++) {
        Node *child = block->ch[ci];
        int32_t len = node_len(child, ref_seq, client);
        if (pos < len || (pos == len && break_tie(pos, child, ref_seq, client))) {
            if (!child->leaf) {
                Block *sn = inserting_walk(d, (Block *)child, pos, ref_seq, client, mode, cand, seq);
                if (sn == UNFINISHED) {   /* act as if shifted past the child */
                    pos -= len;
                    continue;
                }
                if (!sn) return NULL;
                new_node = &sn->n;
                ci++;
            } else {
                Seg *s = (Seg *)child;
                if (mode == WALK_INSERT) {
                    assign_child(block, &cand->n, ci);
                    new_node = &s->n;
                    ci++;
                } else {
                    Seg *next = split_at(d, s, pos);
                    if (!next) return NULL;
                    d->maint[0]++;   /* splitLeafSegment SPLIT :2264-2269 */
                    new_node = &next->n;
                    ci++;
                }
            }
            break;
        } else {
            pos -= len;
        }
    }
    if (!new_node && pos == 0 && mode == WALK_INSERT) {
        if (seq != UNASSIGNED && continue_from(block)) return UNFINISHED;
        new_node = &cand->n;
    }
    if (new_node) {
        blk_dirty(block);
        for (int i = block->count; i > ci; i--) {
            block->ch[i] = block->ch[i - 1];
            block->ch[i]->index = i;
        }
        assign_child(block, new_node, ci);
        block->count++;
        if (block->count < MAXN) return NULL;
        return split_block(d, block);
    }
    return NULL;
}

/* ensureIntervalBoundary :2274-2278 */
static void ensure_boundary(orc_doc *d, int32_t pos, int32_t ref_seq, int32_t client) {
    Block *sn = inserting_walk(d, d->root, pos, ref_seq, client, WALK_SPLIT, NULL, 0);
    update_root(d, sn);
}

/* ------------------------------------------------------------------ delta callbacks */
typedef struct DeltaSeg {
    Seg *seg;
    int npd;
    uint32_t *pd;   /* (key, old) pairs */
} DeltaSeg;

static inline uint64_t fnv_u64(uint64_t h, uint64_t x) {
    h = fnv_u32(h, (uint32_t)x);
    return fnv_u32(h, (uint32_t)(x >> 32));
}

/* Delta hash (DESIGN.md "Checksums"), streamable so the GPU can fold lane-parallel:
     seg_hash = FNV(pos, len [, (key, old)*, npd])            per delta segment
     cb       = FNV(seq, kind) <- seg_hash_0 .. seg_hash_{n-1} <- n   per callback
     H        = fnv_u64(H, cb)                                  per document */
static void emit_deltas(orc_doc *d, int32_t seq, int kind, DeltaSeg *ds, int n) {
    uint64_t cb = FNV_OFF;
    cb = fnv_u32(cb, (uint32_t)seq);
    cb = fnv_u32(cb, (uint32_t)kind);
    if (d->record) {
        ivec_push(&d->dlog, seq);
        ivec_push(&d->dlog, kind);
        ivec_push(&d->dlog, n);
    }
    for (int i = 0; i < n; i++) {
        Seg *s = ds[i].seg;
        int32_t pos = s->n.parent ? get_position(&s->n) : -1;
        uint64_t sh = FNV_OFF;
        sh = fnv_u32(sh, (uint32_t)pos);
        sh = fnv_u32(sh, (uint32_t)s->len);
        if (d->record) {
            ivec_push(&d->dlog, pos);
            ivec_push(&d->dlog, s->len);
        }
        if (kind == MT_OP_ANNOTATE && ds[i].npd < 0) {
            /* propertyDeltas undefined (a pending local rewrite blocked the op) */
            if (d->record) ivec_push(&d->dlog, -1);
            sh = fnv_u32(sh, 0xFFFFFFFFu);
        } else if (kind == MT_OP_ANNOTATE) {
            if (d->record) ivec_push(&d->dlog, ds[i].npd);
            for (int j = 0; j < ds[i].npd; j++) {
                sh = fnv_u32(sh, ds[i].pd[2 * j]);
                sh = fnv_u32(sh, ds[i].pd[2 * j + 1]);
                if (d->record) {
                    ivec_push(&d->dlog, (int32_t)ds[i].pd[2 * j]);
                    ivec_push(&d->dlog, (int32_t)ds[i].pd[2 * j + 1]);
                }
            }
            sh = fnv_u32(sh, (uint32_t)ds[i].npd);
        }
        cb = fnv_u64(cb, sh);
    }
    cb = fnv_u32(cb, (uint32_t)n);
    d->delta_hash = fnv_u64(d->delta_hash, cb);
}

/* ------------------------------------------------------------------ nodeMap */
typedef struct MapCtx {
    int kind;
    int32_t seq, client, local_seq;
    Group *group;          /* the local op's segment group, opened by its first segment */
    const uint32_t *props_rec;
    DeltaSeg *ds;
    int nds, cap;
    orc_doc *d;
} MapCtx;

static void ds_push(MapCtx *m, Seg *s, int npd, uint32_t *pd) {
    if (m->nds == m->cap) {
        m->cap = m->cap ? m->cap * 2 : 16;
        m->ds = (DeltaSeg *)realloc(m->ds, sizeof(DeltaSeg) * m->cap);
    }
    m->ds[m->nds].seg = s;
    m->ds[m->nds].npd = npd;
    m->ds[m->nds].pd = pd;
    m->nds++;
}

/* pendingKeyUpdateCount[key] !== undefined */
static int key_pending(const Seg *s, uint32_t key) { return s->pk && props_find(s->pk, key) >= 0; }

/* SegmentPropertiesManager.addProperties MT/segmentPropertiesManager.ts:35-111 while
   collaborating: seq UNASSIGNED is the local client's own annotate (every key modified, its
   keys counted pending), otherwise a sequenced op, which an outstanding local rewrite blocks
   (returns -1: propertyDeltas undefined) and which skips keys with a pending local update
   unless it carries a combining op (shouldModifyKey :56-63). */
static int add_properties(orc_doc *d, Seg *s, const uint32_t *rec, int32_t seq, uint32_t **pd_out) {
    uint32_t count = rec[0] & 0xFFFF, combine = rec[0] >> 16;
    if (!s->props) s->props = props_new(d);
    Props *p = s->props;
    const int local = seq == UNASSIGNED;
    *pd_out = NULL;
    if (s->prw > 0 && !local) return -1;
    if (!s->pk) s->pk = props_new(d);
    const int combining = combine == MT_COMBINE_TABLE;
#define MODIFY(k) (local || combining || !key_pending(s, (k)))
    if (combine == MT_COMBINE_REWRITE && local) s->prw++;
    /* deltas: ordered map key -> previous value (insertion order, overwrite in place) */
    uint32_t *pd = (uint32_t *)dalloc(d, sizeof(uint32_t) * 2 * (p->n + count + 1));
    int npd = 0;
#define PD_SET(k, v)                                   \
    do {                                               \
        int f_ = -1;                                   \
        for (int q_ = 0; q_ < npd; q_++)               \
            if (pd[2 * q_] == (k)) f_ = q_;            \
        if (f_ < 0) {                                  \
            pd[2 * npd] = (k);                         \
            pd[2 * npd + 1] = (v);                     \
            npd++;                                     \
        } else                                         \
            pd[2 * f_ + 1] = (v);                      \
    } while (0)
    if (combine == MT_COMBINE_REWRITE) {
        /* delete all keys not (truthily) present in newProps  :66-79 */
        for (int i = 0; i < p->n;) {
            uint32_t key = p->key[i];
            int truthy = 0;
            for (uint32_t j = 0; j < count; j++) {
                if (rec[1 + 2 * j] == key) {
                    uint32_t v = rec[2 + 2 * j];
                    truthy = (v != MT_VAL_NULL) && !(v & MT_VAL_FALSY_BIT);
                }
            }
            if (!truthy && MODIFY(key)) {
                PD_SET(key, p->val[i]);
                props_del(p, key);
            } else {
                i++;
            }
        }
    }
    for (uint32_t j = 0; j < count; j++) {
        uint32_t key = rec[1 + 2 * j], val = rec[2 + 2 * j];
        if (local) {
            int q = props_find(s->pk, key);
            props_set(d, s->pk, key, q >= 0 ? s->pk->val[q] + 1 : 1);
        } else if (!MODIFY(key)) {
            continue;
        }
        int i = props_find(p, key);
        /* deltas[key] = previousValue === undefined ? null : previousValue */
        const int absent = i < 0 || p->val[i] == MT_VAL_UNDEF;
        PD_SET(key, absent ? MT_VAL_NULL : p->val[i]);
        if (combine == MT_COMBINE_TABLE) {
            /* newValue = combine(op, previousValue, undefined, seq) :93-99 */
            const uint32_t *tab = rec + 1 + 2 * count;
            val = tab[1];
            if (!absent) {
                int hit = 0;
                for (uint32_t q = 0; q < tab[0]; q++)
                    if (tab[2 + 2 * q] == p->val[i]) {
                        val = tab[3 + 2 * q];
                        hit = 1;
                    }
                if (!hit) {          /* the host tabulated every value: cannot happen */
                    d->status = MT_DOC_INTERNAL;
                    *pd_out = pd;
                    return 0;
                }
            }
        }
        if (val == MT_VAL_NULL)
            props_del(p, key);
        else
            props_set(d, p, key, val);
    }
#undef PD_SET
#undef MODIFY
    *pd_out = pd;
    return npd;
}

/* ackPendingProperties MT/segmentPropertiesManager.ts:19-33 */
static void ack_pending_properties(Seg *s, const uint32_t *rec) {
    uint32_t count = rec[0] & 0xFFFF, combine = rec[0] >> 16;
    if (combine == MT_COMBINE_REWRITE) s->prw--;
    for (uint32_t j = 0; j < count && s->pk; j++) {
        int q = props_find(s->pk, rec[1 + 2 * j]);
        if (q < 0) continue;
        if (--s->pk->val[q] == 0) props_del(s->pk, rec[1 + 2 * j]);
    }
}

/* markRemoved / annotateSegment leaf actions :2647-2693, :2607-2620 */
static void map_leaf(MapCtx *m, Seg *s) {
    orc_doc *d = m->d;
    if (m->kind == MT_OP_REMOVE) {
        seg_dirty(s);
        if (s->rseq == UNASSIGNED) {          /* a pending local removal: replaced :2657-2662 */
            s->rclient = m->client;
            s->rseq = m->seq;
            s->lrseq = RSEQ_NONE;
        } else if (s->rseq != RSEQ_NONE) {
            ovl_push(d, s, m->client);
        } else {
            s->rclient = m->client;
            s->rseq = m->seq;
            s->lrseq = m->seq == UNASSIGNED ? m->local_seq : RSEQ_NONE;
            ds_push(m, s, 0, NULL);
        }
        if (s->rseq == UNASSIGNED && m->client == OBSERVER)
            add_to_pending(d, s, &m->group, m->local_seq);
        else
            add_to_lru(d, s, m->seq);
    } else {
        uint32_t *pd;
        int npd = add_properties(d, s, m->props_rec, m->seq, &pd);
        ds_push(m, s, npd, pd);
        if (m->seq == UNASSIGNED)
            add_to_pending(d, s, &m->group, m->local_seq);
        else
            add_to_lru(d, s, m->seq);
    }
}

/* nodeMap :2936-2998 */
static void node_map(MapCtx *m, Block *node, int32_t ref_seq, int32_t client, int32_t start,
                     int32_t end) {
    for (int ci = 0; ci < node->count; ci++) {
        Node *child = node->ch[ci];
        int32_t len = node_len(child, ref_seq, client);
        if (end > 0 && len > 0 && start < len) {
            if (!child->leaf)
                node_map(m, (Block *)child, ref_seq, client, start, end);
            else
                map_leaf(m, (Seg *)child);
        }
        start -= len;
        end -= len;
    }
}

/* ------------------------------------------------------------------ op application */
static Seg *segment_from_op(orc_doc *d, const mt_op_rec *op, const uint16_t *text_arena,
                            const uint32_t *props_arena) {
    Seg *s;
    if (op->flags & MT_F_MARKER) {           /* Marker.make  MT/mergeTree.ts:676-688 */
        s = make_text_seg(d, NULL, 0);
        s->marker = (int32_t)op->payload;
        s->len = 1;
    } else {                                 /* TextSegment.make MT/textSegment.ts:23-29 */
        s = make_text_seg(d, text_arena + op->payload, op->pos2);
    }
    if (op->props != MT_NO_PROPS) {
        /* addProperties(props) without op/seq: keys with null dropped, {} kept (Q5) */
        const uint32_t *rec = props_arena + op->props;
        uint32_t count = rec[0] & 0xFFFF;
        s->props = props_new(d);
        for (uint32_t j = 0; j < count; j++)
            if (rec[2 + 2 * j] != MT_VAL_NULL) props_set(d, s->props, rec[1 + 2 * j], rec[2 + 2 * j]);
    }
    return s;
}

/* updateSeqNumbers / updateMinSeq / setMinSeq  MT/client.ts:821-828, 991-1004;
   MT/mergeTree.ts:1751-1769 */
static int update_seq_numbers(orc_doc *d, int32_t msn, int32_t seq) {
    if (!(d->current_seq <= seq)) return MT_DOC_SEQ_BACKWARDS;   /* client.ts:824 */
    d->current_seq = seq;
    if (!(msn <= seq)) return MT_DOC_MSN_ABOVE_SEQ;              /* client.ts:826 */
    if (!(d->min_seq <= msn)) return MT_DOC_MSN_BACKWARDS;        /* mergeTree.ts:1755 */
    if (msn > d->min_seq) {
        d->min_seq = msn;
        zamboni(d);
    }
    return MT_DOC_OK;
}

/* ackPendingSegment MT/client.ts:589-626 (one GROUP member) -> MergeTree.ackPendingSegment
   :1926-1953 with ISegment.ack :486-521 */
static void ack_pending(orc_doc *d, const mt_op_rec *op, const uint32_t *props_arena) {
    Group *g = d->pend_head;
    const int32_t seq = op->seq;
    if (g) {
        d->pend_head = g->next;
        if (!d->pend_head) d->pend_tail = NULL;
        d->n_pend--;
        for (int i = 0; i < g->n; i++) {
            Seg *s = g->segs[i];
            if (s->gn == 0 || s->grp[s->ghead] != g) {   /* assert.equal(currentSegmentGroup, ..) */
                d->status = MT_DOC_INTERNAL;
                return;
            }
            s->ghead++;
            s->gn--;
            seg_dirty(s);
            if (op->kind == MT_OP_ANNOTATE) {
                static const uint32_t empty_rec[1] = {0};
                ack_pending_properties(s, op->props != MT_NO_PROPS ? props_arena + op->props : empty_rec);
            } else if (op->kind == MT_OP_INSERT) {
                s->seq = seq;
                s->lseq = RSEQ_NONE;
            } else if (op->kind == MT_OP_REMOVE) {
                s->lrseq = RSEQ_NONE;
                if (s->rseq == UNASSIGNED) s->rseq = seq;   /* else a remote removal replaced it */
            }
            add_to_lru(d, s, seq);
        }
    }
    zamboni(d);
}

static void ord_fn(Seg *s, void *arg) { s->ord = (*(int32_t *)arg)++; }
typedef struct ReconAcc {
    const Seg *target;
    int32_t local_seq, pos, done;
} ReconAcc;
/* findReconnectionPostition MT/client.ts:675-707: the segments before `target` that are
   inserted and not removed as of the group's localSeq */
static void recon_fn(Seg *s, void *arg) {
    ReconAcc *a = (ReconAcc *)arg;
    if (a->done || s == a->target) {
        a->done = 1;
        return;
    }
    if ((s->lseq == RSEQ_NONE || s->lseq <= a->local_seq) &&
        (s->rseq == RSEQ_NONE || (s->lrseq != RSEQ_NONE && s->lrseq > a->local_seq)))
        a->pos += s->len;
}
static int cmp_ord(const void *a, const void *b) {
    const Seg *x = *(Seg *const *)a, *y = *(Seg *const *)b;
    return x->ord < y->ord ? -1 : x->ord > y->ord;
}

/* getValidOpRange MT/client.ts:486-548 for the local client's own op (its length view) */
static int local_range_ok(orc_doc *d, const mt_op_rec *op) {
    const int32_t len = orc_length(d), start = op->pos1;
    if (start < 0 || start > len || (start == len && op->kind != MT_OP_INSERT)) return 0;
    if (op->kind != MT_OP_INSERT && op->pos2 <= start) return 0;
    return 1;
}

static int32_t orc_apply_impl(orc_doc *d, const mt_op_rec *op, const uint16_t *text_arena,
                              const uint32_t *props_arena);
int32_t orc_apply(orc_doc *d, const mt_op_rec *op, const uint16_t *text_arena,
                  const uint32_t *props_arena) {
    const int32_t r = orc_apply_impl(d, op, text_arena, props_arena);
    if (d->ovl_units > d->ovl_peak) d->ovl_peak = d->ovl_units;
    return r;
}
void orc_overlap_units(const orc_doc *d, int64_t *out) {
    out[0] = d->ovl_units;
    out[1] = d->ovl_peak;
}
static int32_t orc_apply_impl(orc_doc *d, const mt_op_rec *op, const uint16_t *text_arena,
                              const uint32_t *props_arena) {
    d->segv_ok = 0;
    if (d->status) return d->status;
    int32_t r = op->ref_seq, c = op->client, seq = op->seq;
    if (op->flags & MT_F_ACK) {             /* applyMsg of our own op's echo :805-813 */
        if (op->kind != MT_OP_NOOP) ack_pending(d, op, props_arena);
        if (!d->status && !(op->flags & MT_F_GROUP_MORE)) {
            int st = update_seq_numbers(d, op->min_seq, seq);
            if (st) d->status = st;
        }
        return d->status;
    }
    int32_t local_seq = 0;
    if (op->flags & MT_F_LOCAL) {
        /* insertSegmentLocal / removeRangeLocal / annotateRangeLocal MT/client.ts:164-211:
           getClientSequenceArgs (:559-575) -- the collab client at refSeq = currentSeq,
           UnassignedSequenceNumber; an invalid range applies nothing */
        if (op->kind == MT_OP_NOOP || !local_range_ok(d, op)) return d->status;
        if (op->kind == MT_OP_INSERT && !(op->flags & MT_F_MARKER) && op->pos2 <= 0) return d->status;
        r = d->current_seq;
        c = OBSERVER;
        seq = UNASSIGNED;
    }
    if (op->kind == MT_OP_INSERT) {
        /* Client.applyInsertOp MT/client.ts:394-442 -> MergeTree.insertSegments :2001-2031 */
        Seg *s = segment_from_op(d, op, text_arena, props_arena);
        ensure_boundary(d, op->pos1, r, c);
        if (seq == UNASSIGNED) local_seq = ++d->local_seq;
        if (s->len > 0) {                   /* blockInsert :2227-2256 */
            s->seq = seq;
            s->client = c;
            s->lseq = seq == UNASSIGNED ? local_seq : RSEQ_NONE;
            Block *sn = inserting_walk(d, d->root, op->pos1, r, c, WALK_INSERT, s, seq);
            if (s->n.parent == NULL) {
                d->status = MT_DOC_INSERT_FAILED;
                return d->status;
            }
            update_root(d, sn);
            if (seq == UNASSIGNED && c == OBSERVER) {   /* saveIfLocal :2197-2212 */
                Group *g = NULL;
                add_to_pending(d, s, &g, local_seq);
            } else if (seq > d->min_seq) {
                add_to_lru(d, s, seq);
            }
        }
        DeltaSeg ds = {s, 0, NULL};
        emit_deltas(d, seq, MT_OP_INSERT, &ds, 1);
        if (seq != UNASSIGNED) zamboni(d);
    } else if (op->kind == MT_OP_REMOVE || op->kind == MT_OP_ANNOTATE) {
        /* markRangeRemoved :2640-2752 / annotateRange :2598-2638 */
        if (op->kind == MT_OP_ANNOTATE && op->props != MT_NO_PROPS &&
            (props_arena[op->props] >> 16) == MT_COMBINE_OTHER) {
            d->status = MT_DOC_UNSUPPORTED;
            return d->status;
        }
        ensure_boundary(d, op->pos1, r, c);
        ensure_boundary(d, op->pos2, r, c);
        MapCtx m;
        memset(&m, 0, sizeof(m));
        m.kind = op->kind;
        m.seq = seq;
        m.client = c;
        m.d = d;
        if (seq == UNASSIGNED) m.local_seq = ++d->local_seq;
        m.props_rec = op->props != MT_NO_PROPS ? props_arena + op->props : NULL;
        static const uint32_t empty_rec[1] = {0};
        if (!m.props_rec) m.props_rec = empty_rec;
        node_map(&m, d->root, r, c, op->pos1, op->pos2);
        emit_deltas(d, seq, op->kind, m.ds, m.nds);
        free(m.ds);
        if (seq != UNASSIGNED) zamboni(d);
    }
    if (seq == UNASSIGNED) return d->status;   /* local: no completeAndLogOp asserts, no seq update */
    if (op->kind != MT_OP_NOOP) {
        /* completeAndLogOp asserts MT/client.ts:451-479 */
        if (!(d->current_seq < seq)) return d->status = MT_DOC_SEQ_ORDER;
        if (!(d->min_seq <= op->min_seq)) return d->status = MT_DOC_MINSEQ_ORDER;
    }
    if (!(op->flags & MT_F_GROUP_MORE)) {
        int st = update_seq_numbers(d, op->min_seq, seq);
        if (st) d->status = st;
    }
    return d->status;
}

/* ------------------------------------------------------------------ summary load (C5) */
/* SnapshotLoader.specToSegment MT/snapshotLoader.ts:86-118 (the host resolved client ids) */
static Seg *seg_from_rec(orc_doc *d, const mt_seg_rec *r, const uint16_t *text_arena,
                         const uint32_t *props_arena) {
    Seg *s;
    if (r->flags & MT_F_MARKER) {
        s = make_text_seg(d, NULL, 0);
        s->marker = (int32_t)r->payload;
        s->len = 1;
    } else {
        s = make_text_seg(d, text_arena + r->payload, r->len);
    }
    if (r->props != MT_NO_PROPS) {          /* TextSegment.make(text, props): nulls dropped */
        const uint32_t *rec = props_arena + r->props;
        uint32_t count = rec[0] & 0xFFFF;
        s->props = props_new(d);
        for (uint32_t j = 0; j < count; j++)
            if (rec[2 + 2 * j] != MT_VAL_NULL) props_set(d, s->props, rec[1 + 2 * j], rec[2 + 2 * j]);
    }
    s->seq = r->seq;
    s->client = r->client;
    if (r->removed_seq != RSEQ_NONE) {
        s->rseq = r->removed_seq;
        s->rclient = r->removed_client;
    }
    return s;
}

/* reloadFromSegments :1229-1284: blocks of MaxNodesInBlock - 1 children, bottom-up */
static Block *build_merge_block(orc_doc *d, Node **nodes, int n) {
    const int max_children = MAXN - 1;
    const int nb = (n + max_children - 1) / max_children;
    Node **blocks = (Node **)malloc(sizeof(Node *) * (nb > 0 ? nb : 1));
    for (int bi = 0, ni = 0; bi < nb; bi++) {
        Block *b = make_block(d, 0);
        for (int ci = 0; ci < max_children && ni < n; ci++, ni++) {
            assign_child(b, nodes[ni], ci);
            b->count++;
        }
        blocks[bi] = &b->n;
    }
    Block *root = nb == 1 ? (Block *)blocks[0] : build_merge_block(d, blocks, nb);
    free(blocks);
    return root;
}

/* loadBody's append helper :197-205: insertSegments(root.cachedLength, segs, refSeq 0,
   cli, seq, opArgs undefined) -- insertSegments :2001-2031 with blockInsert :2174-2257 */
static int load_append(orc_doc *d, Seg **segs, int n, int32_t cli, int32_t seq) {
    const int32_t pos = orc_length(d);
    ensure_boundary(d, pos, 0, cli);
    int32_t ins = pos;
    for (int i = 0; i < n; i++) {
        Seg *s = segs[i];
        if (s->len <= 0) continue;
        s->seq = seq;
        s->client = cli;
        Block *sn = inserting_walk(d, d->root, ins, 0, cli, WALK_INSERT, s, seq);
        if (s->n.parent == NULL) return d->status = MT_DOC_INSERT_FAILED;
        update_root(d, sn);
        if (seq > d->min_seq) add_to_lru(d, s, seq);   /* saveIfLocal :2197-2212 */
        ins += s->len;
    }
    zamboni(d);                                         /* collaborating :2027-2030 */
    return 0;
}

/* Client.load -> SnapshotLoader.initialize (MT/snapshotLoader.ts:36-228) for one decoded
   summary: loadHeader (reloadFromSegments + startOrUpdateCollaboration(minSeq, seq)), then
   loadBody (plain below-MSN specs appended in batches, the others one by one). */
orc_doc *orc_load(const mt_seg_rec *recs, int32_t n_header, int32_t n_total, const uint16_t *text_arena,
                  const uint32_t *props_arena, int32_t min_seq, int32_t cur_seq) {
    orc_doc *d = (orc_doc *)calloc(1, sizeof(orc_doc));
    d->delta_hash = FNV_OFF;
    if (n_header > 0) {
        Node **nodes = (Node **)malloc(sizeof(Node *) * n_header);
        for (int i = 0; i < n_header; i++) nodes[i] = &seg_from_rec(d, &recs[i], text_arena, props_arena)->n;
        d->root = build_merge_block(d, nodes, n_header);
        free(nodes);
    } else {
        d->root = make_block(d, 0);
    }
    d->root->n.parent = NULL;
    d->min_seq = min_seq;                   /* startCollaboration :1287-1304 */
    d->current_seq = cur_seq;
    int nb = n_total - n_header;
    Seg **batch = (Seg **)malloc(sizeof(Seg *) * (nb > 0 ? nb : 1));
    int nbatch = 0;
    /* the batch is never emptied (:207-227): once flushed holding a segment of non-zero
       length, the next flush re-inserts it -- the reference's tree then holds one segment
       object twice; the restatement stops there (MT_DOC_ALIASED) */
    int batch_len = 0, flushed = 0;
    for (int i = n_header; i < n_total && !d->status; i++) {
        Seg *s = seg_from_rec(d, &recs[i], text_arena, props_arena);
        if (s->client == -2 && s->seq == 0) {
            if (flushed) continue;
            batch[nbatch++] = s;
            batch_len |= s->len > 0;
        } else {
            if (batch_len && flushed) {
                d->status = MT_DOC_ALIASED;
                break;
            }
            if (nbatch) load_append(d, batch, nbatch, -2, 0);
            if (batch_len) flushed = 1;
            nbatch = 0;
            if (!d->status) load_append(d, &s, 1, s->client, s->seq);
        }
    }
    if (!d->status && batch_len && flushed) d->status = MT_DOC_ALIASED;   /* the final flushBatch() */
    if (nbatch && !d->status) load_append(d, batch, nbatch, -2, 0);
    free(batch);
    return d;
}

/* ------------------------------------------------------------------ lifecycle / output */
orc_doc *orc_new(const uint16_t *seed_text, int32_t seed_len) {
    orc_doc *d = (orc_doc *)calloc(1, sizeof(orc_doc));
    d->root = make_block(d, 0);             /* initialNode :1159-1163 */
    d->delta_hash = FNV_OFF;
    if (seed_len > 0) {
        /* insertSegmentLocal before collaboration: seq 0, client LocalClientId (-1) */
        Seg *s = make_text_seg(d, seed_text, seed_len);
        assign_child(d->root, &s->n, 0);
        d->root->count = 1;
    }
    return d;
}
void orc_free(orc_doc *d) {
    if (!d) return;
    for (int i = 0; i < d->allocs.n; i++) free(d->allocs.p[i]);
    free(d->allocs.p);
    free(d->heap);
    free(d->segv);
    free(d->dlog.p);
    free(d);
}
int32_t orc_status(const orc_doc *d) { return d->status; }
/* regeneratePendingOp MT/client.ts:855-893 for one (non-GROUP) pending op of kind `kind`:
   resetPendingDeltaToOps (:709-767) on the oldest segment group -- its segments in document
   order (the ordinal sort), each at findReconnectionPostition, one op each (a remove whose
   removal a remote replaced: none), each joining a new group at the queue's tail.  Outputs
   mt_regen_rec records (include/mt_replay.h); returns their count, -1 without a pending
   group, -2 when an output buffer is too small (the document is then left unusable). */
int32_t orc_regenerate(orc_doc *d, int32_t kind, orc_regen_rec *out, int32_t cap, uint16_t *text,
                       int32_t text_cap, uint32_t *props, int32_t props_cap) {
    d->segv_ok = 0;
    Group *g = d->pend_head;
    if (!g) return -1;
    d->pend_head = g->next;
    if (!d->pend_head) d->pend_tail = NULL;
    d->n_pend--;
    int32_t ord = 0;
    walk_segs(&d->root->n, ord_fn, &ord);
    Seg **segs = (Seg **)malloc(sizeof(Seg *) * (g->n > 0 ? g->n : 1));
    memcpy(segs, g->segs, sizeof(Seg *) * g->n);
    qsort(segs, g->n, sizeof(Seg *), cmp_ord);
    int32_t n = 0, tu = 0, pu = 0;
    for (int i = 0; i < g->n; i++) {
        Seg *s = segs[i];
        if (s->gn == 0 || s->grp[s->ghead] != g) {
            d->status = MT_DOC_INTERNAL;
            break;
        }
        s->ghead++;
        s->gn--;
        ReconAcc ra = {s, g->local_seq, 0, 0};
        walk_segs(&d->root->n, recon_fn, &ra);
        if (kind == MT_OP_REMOVE && s->lrseq == RSEQ_NONE) continue;
        if (n >= cap) {
            n = -2;
            break;
        }
        orc_regen_rec *r = &out[n++];
        memset(r, 0, sizeof(*r));
        r->kind = kind;
        r->pos1 = ra.pos;
        r->pos2 = kind == MT_OP_INSERT ? 0 : ra.pos + s->len;
        r->local_seq = g->local_seq;
        r->props_off = MT_NO_PROPS;
        if (kind == MT_OP_INSERT) {   /* createInsertSegmentOp: the segment's JSON as it is now */
            if (s->marker >= 0) {
                r->flags = MT_F_MARKER;
                r->text_off = (uint32_t)s->marker;
                r->text_len = 1;
            } else {
                if (tu + s->len > text_cap) {
                    n = -2;
                    break;
                }
                memcpy(text + tu, s->text, sizeof(uint16_t) * s->len);
                r->text_off = (uint32_t)tu;
                r->text_len = (uint32_t)s->len;
                tu += s->len;
            }
            if (s->props) {
                if (pu + 1 + 2 * s->props->n > props_cap) {
                    n = -2;
                    break;
                }
                r->props_off = (uint32_t)pu;
                props[pu++] = (uint32_t)s->props->n;
                for (int k = 0; k < s->props->n; k++) {
                    props[pu++] = s->props->key[k];
                    props[pu++] = s->props->val[k];
                }
            }
        }
        Group *ng = NULL;
        add_to_pending(d, s, &ng, g->local_seq);
    }
    free(segs);
    return d->status ? -3 : n;
}

void orc_pending_counts(const orc_doc *d, int32_t *out) {
    out[0] = d->local_seq;   /* collabWindow.localSeq */
    out[1] = d->n_pend;      /* pendingSegments.count() */
}
void orc_set_record_deltas(orc_doc *d, int32_t on) { d->record = on; }
int32_t orc_view_length(orc_doc *d, int32_t ref_seq, int32_t client) {
    return node_len(&d->root->n, ref_seq, client);
}
int32_t orc_length(orc_doc *d) { return node_len(&d->root->n, 0, OBSERVER); }

/* getPosition :1619-1636 in view (client, refSeq): the nodeLength of every earlier sibling of
   the node and of each of its ancestors */
static int32_t get_position_view(const Node *node, int32_t ref_seq, int32_t client) {
    int32_t total = 0;
    const Block *parent = node->parent;
    const Node *prev = node;
    while (parent) {
        for (int i = 0; i < parent->count; i++) {
            const Node *c = parent->ch[i];
            if (c == prev) break;
            total += node_len(c, ref_seq, client);
        }
        prev = &parent->n;
        parent = parent->n.parent;
    }
    return total;
}
typedef struct IdxAcc {
    const Seg *want;
    int32_t idx, hit;
} IdxAcc;
static void idx_fn(Seg *s, void *arg) {
    IdxAcc *a = (IdxAcc *)arg;
    if (s == a->want) a->hit = a->idx;
    a->idx++;
}
/* getContainingSegment :1656-1667 -> searchBlock :1830-1862 in view (client, refSeq): at
   every level the first child with pos < nodeLength(child) (interior children by their partial
   lengths), descending without backtracking -- a block whose leaves do not hold pos yields no
   segment.  out = {document-order index, offset, getPosition in the view, observer position}
   (index -1: undefined). */
void orc_containing(orc_doc *d, int32_t pos, int32_t ref_seq, int32_t client, int32_t *out) {
    const Block *b = d->root;
    out[0] = -1;
    out[1] = out[2] = out[3] = 0;
    for (;;) {
        const Node *hit = NULL;
        for (int i = 0; i < b->count; i++) {
            const int32_t len = node_len(b->ch[i], ref_seq, client);
            if (pos < len) {
                hit = b->ch[i];
                break;
            }
            pos -= len;
        }
        if (!hit) return;
        if (!hit->leaf) {
            b = (const Block *)hit;
            continue;
        }
        IdxAcc a = {(const Seg *)hit, 0, -1};
        walk_segs(&d->root->n, idx_fn, &a);
        out[0] = a.hit;
        out[1] = pos;
        out[2] = get_position_view(hit, ref_seq, client);
        out[3] = get_position_view(hit, 0, OBSERVER);
        return;
    }
}
/* getPosition of the seg_index-th segment (document order) in view (client, refSeq); -1: none */
static Seg *seg_at(orc_doc *d, int32_t seg_index);
int32_t orc_position(orc_doc *d, int32_t seg_index, int32_t ref_seq, int32_t client) {
    const Seg *hit = seg_at(d, seg_index);
    return hit ? get_position_view(&hit->n, ref_seq, client) : -1;
}

typedef void (*seg_fn)(Seg *, void *);
static void walk_segs(Node *n, seg_fn fn, void *arg) {   /* walkAllSegments :3002-3016 */
    if (n->leaf) {
        fn((Seg *)n, arg);
        return;
    }
    Block *b = (Block *)n;
    for (int i = 0; i < b->count; i++) walk_segs(b->ch[i], fn, arg);
}

typedef struct TextAcc {
    uint16_t *out;
    int32_t cap, n;
} TextAcc;
static void text_fn(Seg *s, void *arg) {   /* gatherText MT/textSegment.ts:188-275 */
    TextAcc *a = (TextAcc *)arg;
    if (s->rseq != RSEQ_NONE || s->marker >= 0) return;
    for (int i = 0; i < s->len; i++) {
        if (a->n < a->cap) a->out[a->n] = s->text[i];
        a->n++;
    }
}
int32_t orc_text(orc_doc *d, uint16_t *out, int32_t cap) {
    TextAcc a = {out, cap, 0};
    walk_segs(&d->root->n, text_fn, &a);
    return a.n;
}

typedef struct SegAcc {
    int32_t *out;
    int32_t cap, n;
} SegAcc;
static void seg_fn_dump(Seg *s, void *arg) {
    SegAcc *a = (SegAcc *)arg;
    if (a->n < a->cap) {
        int32_t *r = a->out + 8 * a->n;
        r[0] = s->len;
        r[1] = s->seq;
        r[2] = s->client;
        r[3] = s->rseq;
        r[4] = s->rseq == RSEQ_NONE ? INT32_MIN : s->rclient;
        r[5] = s->novl;
        r[6] = s->marker;
        r[7] = s->props ? 1 : 0;
    }
    a->n++;
}
int32_t orc_segments(orc_doc *d, int32_t *out, int32_t cap_rows) {
    SegAcc a = {out, cap_rows, 0};
    walk_segs(&d->root->n, seg_fn_dump, &a);
    return a.n;
}
static void segv_fn(Seg *s, void *arg) {
    orc_doc *d = (orc_doc *)arg;
    if (d->segv_n == d->segv_cap) {
        d->segv_cap = d->segv_cap ? 2 * d->segv_cap : 1024;
        d->segv = (Seg **)realloc(d->segv, sizeof(Seg *) * d->segv_cap);
    }
    d->segv[d->segv_n++] = s;
}
/* segment seg_index in document order (NULL: none) */
static Seg *seg_at(orc_doc *d, int32_t seg_index) {
    if (!d->segv_ok) {
        d->segv_n = 0;
        walk_segs(&d->root->n, segv_fn, d);
        d->segv_ok = 1;
    }
    return seg_index >= 0 && seg_index < d->segv_n ? d->segv[seg_index] : NULL;
}
int32_t orc_segment_props(orc_doc *d, int32_t seg_index, uint32_t *out, int32_t cap_pairs) {
    const Seg *hit = seg_at(d, seg_index);
    if (!hit || !hit->props) return -1;
    for (int i = 0; i < hit->props->n && i < cap_pairs; i++) {
        out[2 * i] = hit->props->key[i];
        out[2 * i + 1] = hit->props->val[i];
    }
    return hit->props->n;
}

static void leaves_rec(Block *b, int32_t *out, int32_t cap, int32_t *n) {
    if (b->count == 0 || b->ch[0]->leaf) {
        if (*n < cap) out[*n] = b->count;
        (*n)++;
        return;
    }
    for (int i = 0; i < b->count; i++) leaves_rec((Block *)b->ch[i], out, cap, n);
}
int32_t orc_leaves(orc_doc *d, int32_t *out, int32_t cap) {
    int32_t n = 0;
    leaves_rec(d->root, out, cap, &n);
    return n;
}

typedef struct SumAcc {
    uint64_t ph;
    uint32_t len, nseg;
    Seg *run;          /* current props run representative */
    int32_t run_len;
    int have;
} SumAcc;
static int same_ordered(const Props *a, const Props *b) {
    if (!a || !b) return a == b;
    if (a->n != b->n) return 0;
    for (int i = 0; i < a->n; i++)
        if (a->key[i] != b->key[i] || a->val[i] != b->val[i]) return 0;
    return 1;
}
/* props hash: FNV over maximal runs of observer-visible segments with identical
   (ordered) property sets: (len, has, n, (key, val)*) per run. */
static uint64_t fold_run(uint64_t h, const Props *p, int32_t len) {
    h = fnv_u32(h, (uint32_t)len);
    h = fnv_u32(h, p ? 1u : 0u);
    if (p) {
        h = fnv_u32(h, (uint32_t)p->n);
        for (int i = 0; i < p->n; i++) {
            h = fnv_u32(h, p->key[i]);
            h = fnv_u32(h, p->val[i]);
        }
    }
    return h;
}
static void sum_fn(Seg *s, void *arg) {
    SumAcc *a = (SumAcc *)arg;
    a->nseg++;
    if (s->rseq != RSEQ_NONE) return;
    a->len += s->len;
    if (a->have && same_ordered(a->run->props, s->props)) {
        a->run_len += s->len;
    } else {
        if (a->have) a->ph = fold_run(a->ph, a->run->props, a->run_len);
        a->run = s;
        a->run_len = s->len;
        a->have = 1;
    }
}
/* text hash: H = FNV(n) folded with h_k = FNV-1a over the UTF-16LE bytes of characters
   [64k, 64k+64) of the getText() string (markers contribute nothing). */
uint64_t orc_text_hash(const uint16_t *t, int32_t n) {
    uint64_t h = fnv_u32(FNV_OFF, (uint32_t)n);
    for (int32_t k = 0; k < n; k += 64) {
        uint64_t hk = FNV_OFF;
        for (int32_t i = k; i < n && i < k + 64; i++) {
            hk ^= t[i] & 0xFF;
            hk *= FNV_PRIME;
            hk ^= t[i] >> 8;
            hk *= FNV_PRIME;
        }
        h = fnv_u64(h, hk);
    }
    return h;
}
void orc_maintenance(orc_doc *d, uint32_t *out) {
    for (int i = 0; i < 3; i++) out[i] = d->maint[i];
}

void orc_checksum(orc_doc *d, mt_checksum *out) {
    SumAcc a;
    memset(&a, 0, sizeof(a));
    a.ph = FNV_OFF;
    walk_segs(&d->root->n, sum_fn, &a);
    if (a.have) a.ph = fold_run(a.ph, a.run->props, a.run_len);
    int32_t n = orc_text(d, NULL, 0);
    uint16_t *t = (uint16_t *)malloc(sizeof(uint16_t) * (n > 0 ? n : 1));
    orc_text(d, t, n);
    out->length = a.len;
    out->n_segments = a.nseg;
    out->text_hash = orc_text_hash(t, n);
    out->props_hash = a.ph;
    out->delta_hash = d->delta_hash;
    free(t);
}
int32_t orc_deltas(orc_doc *d, int32_t *out, int32_t cap) {
    for (int64_t i = 0; i < d->dlog.n && i < cap; i++) out[i] = d->dlog.p[i];
    return (int32_t)d->dlog.n;
}

/* ------------------------------------------------------------------ generator */
static __thread int32_t *g_trace = NULL;
void orc_set_gen_trace(int32_t *trace) { g_trace = trace; }
typedef struct Rng {
    uint32_t s[4];
} Rng;
static uint32_t splitmix32(uint32_t *x) {
    *x += 0x9E3779B9u;
    uint32_t z = *x;
    z = (z ^ (z >> 16)) * 0x85EBCA6Bu;
    z = (z ^ (z >> 13)) * 0xC2B2AE35u;
    return z ^ (z >> 16);
}
static void rng_init(Rng *r, uint32_t seed, int32_t doc) {
    uint32_t x = seed ^ ((uint32_t)(doc + 1) * 0x9E3779B9u);
    for (int i = 0; i < 4; i++) r->s[i] = splitmix32(&x);
}
static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
static uint32_t rng_next(Rng *r) {   /* xoshiro128** */
    uint32_t *s = r->s;
    uint32_t result = rotl32(s[1] * 5u, 7) * 9u;
    uint32_t t = s[1] << 9;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl32(s[3], 11);
    return result;
}
static inline uint32_t rng_uniform(Rng *r, uint32_t n) {
    return (uint32_t)(((uint64_t)rng_next(r) * n) >> 32);
}
static int gen_text(Rng *r, uint16_t *out, int n, uint64_t p_nl) {
    for (int i = 0; i < n; i++) {
        uint32_t v = rng_next(r);
        out[i] = ((uint64_t)v < p_nl) ? (uint16_t)'\n' : (uint16_t)(97 + rng_uniform(r, 26));
    }
    return n;
}
/* writes [count, (key, val)*] ; returns words used */
static int gen_props(Rng *r, const orc_gen_cfg *cfg, uint32_t *out) {
    uint32_t nk = 1 + rng_uniform(r, (uint32_t)cfg->max_keys_per_op);
    uint32_t count = 0;
    for (uint32_t j = 0; j < nk; j++) {
        uint32_t key = rng_uniform(r, (uint32_t)cfg->n_keys);
        int is_null = (uint64_t)rng_next(r) < cfg->p_null;
        uint32_t val = rng_uniform(r, (uint32_t)cfg->n_values);
        int dup = 0;
        for (uint32_t q = 0; q < count; q++)
            if (out[1 + 2 * q] == key) dup = 1;
        if (dup) continue;
        out[1 + 2 * count] = key;
        out[2 + 2 * count] = is_null ? MT_VAL_NULL : (val | (val == 0 ? MT_VAL_FALSY_BIT : 0));
        count++;
    }
    out[0] = count;
    return 1 + 2 * (int)count;
}

int32_t orc_generate(const orc_gen_cfg *cfg_in, int32_t doc, mt_op_rec *ops, int32_t ops_cap,
                     uint16_t *text, int32_t text_cap, int32_t *text_used, uint32_t *props,
                     int32_t props_cap, int32_t *props_used, uint16_t *seed_out,
                     int32_t *seed_len_out, orc_doc **keep) {
    const orc_gen_cfg *cfg = cfg_in;
    Rng rng;
    rng_init(&rng, cfg->seed, doc);
    gen_text(&rng, seed_out, cfg->seed_len, 0);
    *seed_len_out = cfg->seed_len;
    orc_doc *d = orc_new(seed_out, cfg->seed_len);
    int W = cfg->writers;
    int32_t *last_ref = (int32_t *)calloc(W + 1, sizeof(int32_t));
    int32_t *short_id = (int32_t *)calloc(W + 1, sizeof(int32_t));
    int32_t next_short = 1;
    int32_t tu = 0, pu = 0, n = 0;
    uint64_t p_ins = cfg->p_insert, p_ir = cfg->p_insert_remove;
    for (int32_t t = 1; t <= cfg->ops; t++) {
        int k = 1 + (int)rng_uniform(&rng, (uint32_t)W);
        int32_t lo = last_ref[k] > t - 1 - cfg->lag ? last_ref[k] : t - 1 - cfg->lag;
        if (lo < 0) lo = 0;
        int32_t r = lo + (int32_t)rng_uniform(&rng, (uint32_t)(t - 1 - lo + 1));
        last_ref[k] = r;
        int32_t msn = INT32_MAX;
        for (int j = 1; j <= W; j++)
            if (last_ref[j] < msn) msn = last_ref[j];
        if (!short_id[k]) short_id[k] = next_short++;
        int32_t c = short_id[k];
        int32_t len = orc_view_length(d, r, c);
        if (g_trace) g_trace[t - 1] = len;
        uint32_t u = rng_next(&rng);
        if (n >= ops_cap) goto fail;
        mt_op_rec *op = &ops[n];
        memset(op, 0, sizeof(*op));
        op->seq = t;
        op->ref_seq = r;
        op->min_seq = msn;
        op->client = (uint16_t)c;
        op->props = MT_NO_PROPS;
        if (len == 0 || (uint64_t)u < p_ins) {
            int32_t pos = (int32_t)rng_uniform(&rng, (uint32_t)(len + 1));
            int32_t tl = 1 + (int32_t)rng_uniform(&rng, (uint32_t)cfg->text_max);
            if (tu + tl > text_cap) goto fail;
            gen_text(&rng, text + tu, tl, cfg->p_newline);
            op->kind = MT_OP_INSERT;
            op->pos1 = pos;
            op->pos2 = tl;
            op->payload = (uint32_t)tu;
            tu += tl;
            if (cfg->p_insert_props > 0 && (uint64_t)rng_next(&rng) < cfg->p_insert_props) {
                if (pu + 1 + 2 * cfg->max_keys_per_op > props_cap) goto fail;
                op->props = (uint32_t)pu;
                pu += gen_props(&rng, cfg, props + pu);
            }
        } else {
            int32_t p1 = (int32_t)rng_uniform(&rng, (uint32_t)len);
            int32_t m = 1;
            while (m < 64 && (uint64_t)rng_next(&rng) < cfg->p_len_continue) m++;
            int32_t p2 = p1 + m < len ? p1 + m : len;
            op->pos1 = p1;
            op->pos2 = p2;
            if ((uint64_t)u < p_ir) {
                op->kind = MT_OP_REMOVE;
            } else {
                if (pu + 1 + 2 * cfg->max_keys_per_op > props_cap) goto fail;
                op->kind = MT_OP_ANNOTATE;
                op->props = (uint32_t)pu;
                pu += gen_props(&rng, cfg, props + pu);
            }
        }
        if (orc_apply(d, op, text, props) != MT_DOC_OK) goto fail;
        n++;
    }
    free(last_ref);
    free(short_id);
    *text_used = tu;
    *props_used = pu;
    if (keep)
        *keep = d;
    else
        orc_free(d);
    return n;
fail:
    free(last_ref);
    free(short_id);
    orc_free(d);
    if (keep) *keep = NULL;
    return -1;
}

/* ------------------------------------------------------------------ batch replay */
typedef struct BatchArg {
    int32_t d0, d1;
    int32_t *next;   /* shared: the next document to take (dynamic: documents differ in length) */
    const int64_t *doc_op_off;
    const mt_op_rec *ops;
    const uint16_t *text;
    const uint32_t *props;
    const int64_t *seed_off;
    const uint16_t *seed;
    mt_checksum *sum;
    int32_t *status;
} BatchArg;

static void *batch_worker(void *p) {
    BatchArg *a = (BatchArg *)p;
    for (;;) {
        const int32_t doc = __atomic_fetch_add(a->next, 1, __ATOMIC_RELAXED);
        if (doc >= a->d1) break;
        orc_doc *d = orc_new(a->seed + a->seed_off[doc], (int32_t)(a->seed_off[doc + 1] - a->seed_off[doc]));
        for (int64_t i = a->doc_op_off[doc]; i < a->doc_op_off[doc + 1]; i++)
            if (orc_apply(d, &a->ops[i], a->text, a->props)) break;
        orc_checksum(d, &a->sum[doc]);
        a->status[doc] = d->status;
        orc_free(d);
    }
    return NULL;
}

int32_t orc_replay_batch(int32_t n_docs, const int64_t *doc_op_off, const mt_op_rec *ops,
                         const uint16_t *text_arena, const uint32_t *props_arena,
                         const int64_t *seed_off, const uint16_t *seed_arena,
                         mt_checksum *out_sum, int32_t *out_status, int32_t threads) {
    if (threads < 1) threads = 1;
    if (threads > n_docs) threads = n_docs > 0 ? n_docs : 1;
    pthread_t *th = (pthread_t *)calloc(threads, sizeof(pthread_t));
    BatchArg *args = (BatchArg *)calloc(threads, sizeof(BatchArg));
    int32_t next = 0;   /* documents are taken in index order as threads free up */
    for (int t = 0; t < threads; t++) {
        BatchArg *a = &args[t];
        a->d0 = 0;
        a->d1 = n_docs;
        a->next = &next;
        a->doc_op_off = doc_op_off;
        a->ops = ops;
        a->text = text_arena;
        a->props = props_arena;
        a->seed_off = seed_off;
        a->seed = seed_arena;
        a->sum = out_sum;
        a->status = out_status;
        pthread_create(&th[t], NULL, batch_worker, a);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    free(args);
    return 0;
}

/* ------------------------------------------------------------------ batch load + replay (C5) */
typedef struct LoadArg {
    int32_t d0, d1;
    const int64_t *seg_off;
    const int32_t *n_header;
    const mt_seg_rec *segs;
    const uint16_t *stext;
    const uint32_t *sprops;
    const int32_t *min_seq, *cur_seq;
    const int64_t *doc_op_off;
    const mt_op_rec *ops;
    const uint16_t *text;
    const uint32_t *props;
    mt_checksum *sum;
    int32_t *status;
} LoadArg;

static void *load_worker(void *p) {
    LoadArg *a = (LoadArg *)p;
    for (int32_t doc = a->d0; doc < a->d1; doc++) {
        const int64_t s0 = a->seg_off[doc];
        orc_doc *d = orc_load(a->segs + s0, a->n_header[doc], (int32_t)(a->seg_off[doc + 1] - s0), a->stext,
                              a->sprops, a->min_seq[doc], a->cur_seq[doc]);
        for (int64_t i = a->doc_op_off[doc]; i < a->doc_op_off[doc + 1] && !d->status; i++)
            if (orc_apply(d, &a->ops[i], a->text, a->props)) break;
        orc_checksum(d, &a->sum[doc]);
        a->status[doc] = d->status;
        orc_free(d);
    }
    return NULL;
}

int32_t orc_load_replay_batch(int32_t n_docs, const int64_t *seg_off, const int32_t *n_header,
                              const mt_seg_rec *segs, const uint16_t *seg_text, const uint32_t *seg_props,
                              const int32_t *min_seq, const int32_t *cur_seq, const int64_t *doc_op_off,
                              const mt_op_rec *ops, const uint16_t *text_arena, const uint32_t *props_arena,
                              mt_checksum *out_sum, int32_t *out_status, int32_t threads) {
    if (threads < 1) threads = 1;
    if (threads > n_docs) threads = n_docs > 0 ? n_docs : 1;
    pthread_t *th = (pthread_t *)calloc(threads, sizeof(pthread_t));
    LoadArg *args = (LoadArg *)calloc(threads, sizeof(LoadArg));
    for (int t = 0; t < threads; t++) {
        LoadArg *a = &args[t];
        a->d0 = (int32_t)((int64_t)n_docs * t / threads);
        a->d1 = (int32_t)((int64_t)n_docs * (t + 1) / threads);
        a->seg_off = seg_off;
        a->n_header = n_header;
        a->segs = segs;
        a->stext = seg_text;
        a->sprops = seg_props;
        a->min_seq = min_seq;
        a->cur_seq = cur_seq;
        a->doc_op_off = doc_op_off;
        a->ops = ops;
        a->text = text_arena;
        a->props = props_arena;
        a->sum = out_sum;
        a->status = out_status;
        pthread_create(&th[t], NULL, load_worker, a);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    free(args);
    return 0;
}
