// mt_engine.h -- the per-document replay engine executed by one wavefront.
//
// Every function here is called by all 64 lanes with wave-uniform arguments; scalar
// document state lives in the (uniform) Doc struct, the segment table in HBM, and the
// B-tree counts in LDS.  The semantics follow the reference observer replica
//  -- see oracle/mt_oracle.c for the function-by-function
// restatement this engine is tested against.  Reference paths below are relative to
// /root/reference/packages/dds/merge-tree/src/ ("MT/").
#pragma once
#include "mt_device.h"

#define WSYNC() __syncthreads()

__device__ static const uint32_t kEmptyPropsRec = 0u;

struct Doc {
    DocHdr *hp;
    int4 *A;
    u64 *O;
    uint4 *Bv;
    uint8_t *gcnt;
    int8_t *gflg;
    int2 *heap;
    uint16_t *text;
    uint32_t *props;
    int32_t *dlog;
    int32_t S_cap, B_cap, H_cap, T_cap, P_cap, DL_cap;
    // LDS
    uint8_t *cnt;      // [MT_LV][B_cap]
    int8_t *flg;       // [B_cap]
    uint16_t *ends;    // [B_cap] scratch: level-0 block end indices
    int32_t *scr;      // small scratch (scour plans)
    // scalars (uniform)
    int n, depth, heap_n, cur_seq, min_seq, text_top, text_half, props_top, props_half, next_uid,
        status, dlog_n;
    int nb[MT_LV];
    u64 dhash;
};

__device__ __forceinline__ void fail(Doc &d, int code) {
    if (d.status == 0) d.status = code;
}
__device__ __forceinline__ uint8_t *lvl(Doc &d, int l) { return d.cnt + l * d.B_cap; }
__device__ __forceinline__ uint16_t *text_base(Doc &d, int half) {
    return d.text + (size_t)half * d.T_cap;
}
__device__ __forceinline__ uint32_t *prec(Doc &d, int half, uint32_t h) {
    return d.props + ((size_t)half * d.P_cap + h) * MT_PREC;
}

// ------------------------------------------------------------------ load / store
__device__ void load_doc(Doc &d, const DevState &st, int doc, uint8_t *smem) {
    const size_t S = st.S, B = st.B;
    d.hp = st.hdr + doc;
    d.A = st.segA + doc * S;
    d.O = st.segO + doc * S;
    d.Bv = st.segB + doc * S;
    d.gcnt = st.cnt + doc * (size_t)MT_LV * B;
    d.gflg = st.flg + doc * B;
    d.heap = st.heap + doc * (size_t)(st.H + 1);
    d.text = st.text + doc * (size_t)2 * st.T;
    d.props = st.props + doc * (size_t)2 * st.P * MT_PREC;
    d.dlog = st.DL ? st.dlog + doc * (size_t)st.DL : nullptr;
    d.S_cap = st.S;
    d.B_cap = st.B;
    d.H_cap = st.H;
    d.T_cap = st.T;
    d.P_cap = st.P;
    d.DL_cap = st.DL;
    d.cnt = smem;
    d.flg = (int8_t *)(smem + MT_LV * st.B);
    d.ends = (uint16_t *)(smem + (MT_LV + 1) * st.B);
    d.scr = (int32_t *)(smem + (MT_LV + 3) * st.B);
    DocHdr h = *d.hp;
    d.n = h.n_seg;
    d.depth = h.depth;
    d.heap_n = h.heap_n;
    d.cur_seq = h.cur_seq;
    d.min_seq = h.min_seq;
    d.text_top = h.text_top;
    d.text_half = h.text_half;
    d.props_top = h.props_top;
    d.props_half = h.props_half;
    d.next_uid = h.next_uid;
    d.status = h.status;
    d.dlog_n = h.dlog_n;
    for (int l = 0; l < MT_LV; l++) d.nb[l] = h.n_blk[l];
    d.dhash = h.delta_hash;
    for (int l = 0; l < d.depth; l++)
        for (int b = lane(); b < d.nb[l]; b += MT_WAVE) lvl(d, l)[b] = d.gcnt[l * B + b];
    for (int b = lane(); b < d.nb[0]; b += MT_WAVE) d.flg[b] = d.gflg[b];
    WSYNC();
}

__device__ void store_doc(Doc &d) {
    WSYNC();
    const int B = d.B_cap;
    for (int l = 0; l < d.depth; l++)
        for (int b = lane(); b < d.nb[l]; b += MT_WAVE) d.gcnt[l * B + b] = lvl(d, l)[b];
    for (int b = lane(); b < d.nb[0]; b += MT_WAVE) d.gflg[b] = d.flg[b];
    if (lane() == 0) {
        DocHdr h;
        h.n_seg = d.n;
        h.depth = d.depth;
        h.heap_n = d.heap_n;
        h.cur_seq = d.cur_seq;
        h.min_seq = d.min_seq;
        h.text_top = d.text_top;
        h.text_half = d.text_half;
        h.props_top = d.props_top;
        h.props_half = d.props_half;
        h.next_uid = d.next_uid;
        h.status = d.status;
        h.dlog_n = d.dlog_n;
        for (int l = 0; l < MT_LV; l++) h.n_blk[l] = d.nb[l];
        h.delta_hash = d.dhash;
        h.n_ops = d.hp->n_ops;
        h.pad0 = 0;
        for (int i = 0; i < 8; i++) h.pad[i] = 0;
        *d.hp = h;
    }
}

// ------------------------------------------------------------------ segment table moves
// [from, n) -> [from + k, n + k)
__device__ void seg_move_right(Doc &d, int from, int k) {
    for (int hi = d.n; hi > from; hi -= MT_WAVE) {
        const int lo = max(from, hi - MT_WAVE);
        const int i = lo + lane();
        if (i < hi) {
            int4 a = d.A[i];
            u64 o = d.O[i];
            uint4 b = d.Bv[i];
            d.A[i + k] = a;
            d.O[i + k] = o;
            d.Bv[i + k] = b;
        }
    }
    WSYNC();
}
// [from, n) -> [from - k, n - k)
__device__ void seg_move_left(Doc &d, int from, int k) {
    for (int lo = from; lo < d.n; lo += MT_WAVE) {
        const int i = lo + lane();
        if (i < d.n) {
            int4 a = d.A[i];
            u64 o = d.O[i];
            uint4 b = d.Bv[i];
            d.A[i - k] = a;
            d.O[i - k] = o;
            d.Bv[i - k] = b;
        }
    }
    WSYNC();
}

// ------------------------------------------------------------------ B-tree counts (LDS)
// First block b of level l whose end (prefix of counts) is > x (strict) or >= x.
__device__ int blk_find(Doc &d, int l, int x, bool strict, int &start) {
    const uint8_t *c = lvl(d, l);
    const int nb = d.nb[l];
    int carry = 0;
    for (int base = 0; base < nb; base += MT_WAVE) {
        const int b = base + lane();
        const int v = b < nb ? c[b] : 0;
        const int inc = wave_scan_incl(v);
        const int end = carry + inc;
        const u64 m = ballot(b < nb && (strict ? end > x : end >= x));
        if (m) {
            const int fl = first_lane(m);
            start = bcast(end - v, fl);
            return base + fl;
        }
        carry += bcast(inc, MT_WAVE - 1);
    }
    start = carry;
    return -1;
}
// sum of counts of blocks [0, b) at level l
__device__ int blk_prefix(Doc &d, int l, int b) {
    const uint8_t *c = lvl(d, l);
    int s = 0;
    for (int base = 0; base < b; base += MT_WAVE) {
        const int i = base + lane();
        s += wave_sum(i < b ? c[i] : 0);
    }
    return s;
}
// shift entries [from, nb) of level l by delta (right if > 0), flags too at level 0
__device__ void blk_shift(Doc &d, int l, int from, int delta) {
    uint8_t *c = lvl(d, l);
    const int nb = d.nb[l];
    if (delta > 0) {
        for (int hi = nb; hi > from; hi -= MT_WAVE) {
            const int lo = max(from, hi - MT_WAVE);
            const int i = lo + lane();
            uint8_t v = 0;
            int8_t f = 0;
            if (i < hi) {
                v = c[i];
                if (l == 0) f = d.flg[i];
            }
            __syncthreads();
            if (i < hi) {
                c[i + delta] = v;
                if (l == 0) d.flg[i + delta] = f;
            }
            __syncthreads();
        }
    } else if (delta < 0) {
        for (int lo = from; lo < nb; lo += MT_WAVE) {
            const int i = lo + lane();
            uint8_t v = 0;
            int8_t f = 0;
            if (i < nb) {
                v = c[i];
                if (l == 0) f = d.flg[i];
            }
            __syncthreads();
            if (i < nb) {
                c[i + delta] = v;
                if (l == 0) d.flg[i + delta] = f;
            }
            __syncthreads();
        }
    }
    d.nb[l] += delta;
}

// A block at level l reached MaxNodesInBlock: split 4|4 and propagate (insertingWalk
// :2479-2503, split :2509-2522, updateRoot :1909-1920).  New blocks have needsScour
// undefined; the original keeps its flag.
__device__ void blk_split_up(Doc &d, int l, int b) {
    while (true) {
        if (d.nb[l] + 1 > d.B_cap) {
            fail(d, MT_DOC_CAPACITY);
            return;
        }
        const bool has_parent = l + 1 < d.depth;
        int pstart = 0, P = -1;
        if (has_parent) {
            P = blk_find(d, l + 1, b, true, pstart);
            if (P < 0) {
                fail(d, MT_DOC_INTERNAL);
                return;
            }
        }
        blk_shift(d, l, b + 1, 1);
        if (lane() == 0) {
            lvl(d, l)[b] = MT_HALF;
            lvl(d, l)[b + 1] = MT_HALF;
            if (l == 0) d.flg[b + 1] = MT_SCOUR_UNDEF;
        }
        WSYNC();
        if (!has_parent) {
            const int nl = d.depth;
            if (nl >= MT_LV) {
                fail(d, MT_DOC_CAPACITY);
                return;
            }
            d.depth++;
            d.nb[nl] = 1;
            if (lane() == 0) lvl(d, nl)[0] = 2;
            WSYNC();
            return;
        }
        const int pc = lvl(d, l + 1)[P] + 1;
        WSYNC();
        if (lane() == 0) lvl(d, l + 1)[P] = (uint8_t)pc;
        WSYNC();
        if (pc < MT_MAXN) return;
        l = l + 1;
        b = P;
    }
}

// Replace entries [b0, b0 + nold) of level l with k entries sized base (+1 for the first
// `extra`), as pack :1414-1446 does; new level-0 blocks have needsScour undefined.
__device__ void blk_replace(Doc &d, int l, int b0, int nold, int k, int base, int extra) {
    if (d.nb[l] + (k - nold) > d.B_cap) {
        fail(d, MT_DOC_CAPACITY);
        return;
    }
    blk_shift(d, l, b0 + nold, k - nold);
    uint8_t *c = lvl(d, l);
    for (int j = lane(); j < k; j += MT_WAVE) {
        c[b0 + j] = (uint8_t)(base + (j < extra ? 1 : 0));
        if (l == 0) d.flg[b0 + j] = MT_SCOUR_UNDEF;
    }
    WSYNC();
}

// level-0 end indices into LDS (for per-lane block lookups)
__device__ void compute_ends(Doc &d) {
    const uint8_t *c = lvl(d, 0);
    int carry = 0;
    for (int base = 0; base < d.nb[0]; base += MT_WAVE) {
        const int b = base + lane();
        const int v = b < d.nb[0] ? c[b] : 0;
        const int inc = wave_scan_incl(v);
        if (b < d.nb[0]) d.ends[b] = (uint16_t)(carry + inc);
        carry += bcast(inc, MT_WAVE - 1);
    }
    WSYNC();
}
// first block with end > i (binary search over d.ends; per-lane)
__device__ __forceinline__ int block_of(Doc &d, int i) {
    int lo = 0, hi = d.nb[0] - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (d.ends[mid] > i)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}

// ------------------------------------------------------------------ zamboni heap
// Collections.Heap add/get (MT/collections.ts:212-265); touched by lane 0 only.
__device__ void heap_add(Doc &d, int max_seq, int uid) {
    if (d.heap_n + 1 > d.H_cap) {
        fail(d, MT_DOC_CAPACITY);
        return;
    }
    d.heap_n++;
    if (lane() == 0) {
        int2 *h = d.heap;
        int k = d.heap_n;
        h[k] = make_int2(max_seq, uid);
        while (k > 1 && h[k >> 1].x - h[k].x > 0) {
            int2 t = h[k >> 1];
            h[k >> 1] = h[k];
            h[k] = t;
            k >>= 1;
        }
    }
}
__device__ int2 heap_top(Doc &d) {
    int x = 0, y = 0;
    if (lane() == 0) {
        int2 t = d.heap[1];
        x = t.x;
        y = t.y;
    }
    return make_int2(bcast(x, 0), bcast(y, 0));
}
__device__ void heap_pop(Doc &d) {
    if (lane() == 0) {
        int2 *h = d.heap;
        int n = d.heap_n;
        h[1] = h[n];
        n--;
        int k = 1;
        while ((k << 1) <= n) {
            int j = k << 1;
            if (j < n && h[j].x - h[j + 1].x > 0) j++;
            if (h[k].x - h[j].x <= 0) break;
            int2 t = h[k];
            h[k] = h[j];
            h[j] = t;
            k = j;
        }
    }
    d.heap_n--;
}

__device__ int find_uid(Doc &d, uint32_t uid) {
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        const u64 m = ballot(i < d.n && (d.Bv[i].z & ~MT_MARKER_BIT) == uid);
        if (m) return base + first_lane(m);
    }
    return -1;
}

// sum of observer lengths over [0, x)  (getPosition :1619-1636 in the observer view)
__device__ int obs_prefix(Doc &d, int x) {
    int s = 0;
    for (int base = 0; base < x; base += MT_WAVE) {
        const int i = base + lane();
        s += wave_sum(i < x ? obs_len(d.A[i]) : 0);
    }
    return s;
}

// ------------------------------------------------------------------ text arena
__device__ void wave_copy16(uint16_t *dst, const uint16_t *src, int n) {
    for (int j = lane(); j < n; j += MT_WAVE) dst[j] = src[j];
}
// Compact all live text (non-removed TextSegments) into the other half, document order.
__device__ void text_gc(Doc &d) {
    WSYNC();
    const int dh = 1 - d.text_half;
    uint16_t *dst = text_base(d, dh), *src = text_base(d, d.text_half);
    int carry = 0;
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        int4 a = make_int4(0, 0, 0, 0);
        uint4 b = make_uint4(0, 0, 0, 0);
        if (i < d.n) {
            a = d.A[i];
            b = d.Bv[i];
        }
        const bool live = i < d.n && a.z == MT_RSEQ_NONE && !(b.z & MT_MARKER_BIT);
        const int len = live ? a.x : 0;
        const int inc = wave_scan_incl(len);
        const int off = carry + inc - len;
        u64 m = ballot(live && len > 0);
        while (m) {
            const int j = first_lane(m);
            m &= m - 1;
            const int lj = bcast(len, j), oj = bcast(off, j), sj = bcast((int)b.x, j);
            wave_copy16(dst + oj, src + sj, lj);
        }
        if (live) d.Bv[i].x = (uint32_t)off;
        carry += bcast(inc, MT_WAVE - 1);
    }
    d.text_half = dh;
    d.text_top = carry;
    WSYNC();
}
__device__ bool text_ensure(Doc &d, int need) {
    if (d.text_top + need <= d.T_cap) return true;
    text_gc(d);
    if (d.text_top + need <= d.T_cap) return true;
    fail(d, MT_DOC_CAPACITY);
    return false;
}

// ------------------------------------------------------------------ property records
__device__ void props_gc(Doc &d) {
    WSYNC();
    const int dh = 1 - d.props_half;
    int carry = 1;
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        uint32_t h = i < d.n ? d.Bv[i].y : 0;
        const int has = h != 0;
        const int inc = wave_scan_incl(has);
        const uint32_t nh = (uint32_t)(carry + inc - has);
        if (has) {
            const uint32_t *s = prec(d, d.props_half, h);
            uint32_t *t = prec(d, dh, nh);
            const uint32_t n = s[0];
            t[0] = n;
            for (uint32_t k = 0; k < 2 * n; k++) t[1 + k] = s[1 + k];
            d.Bv[i].y = nh;
        }
        carry += bcast(inc, MT_WAVE - 1);
    }
    d.props_half = dh;
    d.props_top = carry;
    WSYNC();
}
__device__ bool props_ensure(Doc &d, int need) {
    if (d.props_top + need <= d.P_cap) return true;
    props_gc(d);
    if (d.props_top + need <= d.P_cap) return true;
    fail(d, MT_DOC_CAPACITY);
    return false;
}
// Properties.matchProperties MT/properties.ts:61-92 over interned ids
__device__ bool match_props(Doc &d, uint32_t ha, uint32_t hb) {
    if (ha == 0 || hb == 0) return ha == hb;
    if (ha == hb) return true;
    const uint32_t *a = prec(d, d.props_half, ha), *b = prec(d, d.props_half, hb);
    const uint32_t na = a[0], nbb = b[0];
    if (na != nbb) return false;
    for (uint32_t i = 0; i < na; i++) {
        bool ok = false;
        for (uint32_t j = 0; j < nbb; j++)
            if (b[1 + 2 * j] == a[1 + 2 * i]) ok = b[2 + 2 * j] == a[2 + 2 * i];
        if (!ok) return false;
    }
    return true;
}

// ------------------------------------------------------------------ delta callbacks
struct Cb {
    u64 h;
    int n;
    int log_hdr;  // dlog index of the record header, -1 if not logging
};
__device__ Cb cb_begin(Doc &d, int seq, int kind) {
    Cb cb;
    cb.h = fnv_u32(fnv_u32(MT_FNV_OFF, (uint32_t)seq), (uint32_t)kind);
    cb.n = 0;
    cb.log_hdr = -1;
    if (d.dlog && d.dlog_n + 3 <= d.DL_cap) {
        cb.log_hdr = d.dlog_n;
        if (lane() == 0) {
            d.dlog[d.dlog_n] = seq;
            d.dlog[d.dlog_n + 1] = kind;
        }
        d.dlog_n += 3;
    }
    return cb;
}
__device__ void cb_end(Doc &d, Cb &cb) {
    cb.h = fnv_u32(cb.h, (uint32_t)cb.n);
    d.dhash = fnv_u64(d.dhash, cb.h);
    if (cb.log_hdr >= 0 && lane() == 0) d.dlog[cb.log_hdr + 2] = cb.n;
}
__device__ void cb_log(Doc &d, int32_t v) {
    if (d.dlog && d.dlog_n + 1 <= d.DL_cap) {
        if (lane() == 0) d.dlog[d.dlog_n] = v;
        d.dlog_n++;
    }
}

// ------------------------------------------------------------------ splitting
// BaseSegment.splitAt :523-567 (right half inserted right after the left half in the same
// leaf block, which may then split).  Property records are immutable, so both halves share.
__device__ void split_seg(Doc &d, int i, int q) {
    if (d.n + 1 > d.S_cap) {
        fail(d, MT_DOC_CAPACITY);
        return;
    }
    int bstart;
    const int b = blk_find(d, 0, i, true, bstart);
    if (b < 0) {
        fail(d, MT_DOC_INTERNAL);
        return;
    }
    seg_move_right(d, i + 1, 1);
    if (lane() == 0) {
        int4 a = d.A[i];
        uint4 bb = d.Bv[i];
        int4 r = a;
        r.x = a.x - q;
        a.x = q;
        uint4 rb = bb;
        rb.x = bb.x + (uint32_t)q;
        rb.z = (uint32_t)d.next_uid | (bb.z & MT_MARKER_BIT);
        d.A[i] = a;
        d.A[i + 1] = r;
        d.O[i + 1] = d.O[i];
        d.Bv[i + 1] = rb;
    }
    d.next_uid++;
    d.n++;
    const int c = lvl(d, 0)[b] + 1;
    WSYNC();
    if (lane() == 0) lvl(d, 0)[b] = (uint8_t)c;
    WSYNC();
    if (c == MT_MAXN) blk_split_up(d, 0, b);
}

// ensureIntervalBoundary :2274-2278 -- split the leaf strictly containing view position p
__device__ void boundary(Doc &d, int p, int r, int c) {
    int carry = 0;
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        const bool v = i < d.n;
        int4 a = v ? d.A[i] : make_int4(0, 0, MT_RSEQ_NONE, 0);
        const u64 o = v ? d.O[i] : 0ull;
        const int vl = v ? view_len(a, o, r, c) : 0;
        const int inc = wave_scan_incl(vl);
        const int pex = carry + inc - vl, pin = carry + inc;
        const u64 m = ballot(v && pex < p && p < pin);
        if (m) {
            const int l = first_lane(m);
            split_seg(d, base + l, p - bcast(pex, l));
            return;
        }
        if (ballot(v && pex >= p)) return;
        carry += bcast(inc, MT_WAVE - 1);
    }
}

// addToLRUSet :1306-1316 for the segment at index i in leaf block b
__device__ void add_to_lru_block(Doc &d, int b, uint32_t uid, int seq) {
    const int f = d.flg[b];
    WSYNC();
    if (f != 1 && seq > d.cur_seq) {
        if (lane() == 0) d.flg[b] = 1;
        WSYNC();
        heap_add(d, seq, (int)uid);
    }
}

// ------------------------------------------------------------------ zamboni
// TextSegment.canAppend MT/textSegment.ts:63-68 (Marker.canAppend false :827-829)
__device__ __forceinline__ bool can_append(int plen, bool pmarker, bool p_nl, int slen,
                                           bool smarker) {
    if (pmarker || smarker) return false;
    if (p_nl) return false;
    return plen <= MT_GRAN || slen <= MT_GRAN;
}

// scourNode :1322-1398 over leaf block [s, e); compacts the table.  Returns survivors.
__device__ int scour_block(Doc &d, int s, int e) {
    // plan (lane 0): scr[k] = -2 keep, -1 unlink, >=0 append into that local index
    int *plan = d.scr;
    int *glen = d.scr + 16;  // merged length per keeper
    const int cntb = e - s;
    int need = 0;
    if (lane() == 0) {
        const uint16_t *tb = text_base(d, d.text_half);
        int prev = -1;
        int plen = 0;
        bool pmark = false, pnl = false;
        uint32_t pprops = 0;
        int pend = 0;  // arena end of prev's current contiguous text (-1 if not contiguous)
        for (int k = 0; k < cntb; k++) {
            const int4 a = d.A[s + k];
            const uint4 b = d.Bv[s + k];
            const bool mk = (b.z & MT_MARKER_BIT) != 0;
            glen[k] = a.x;
            if (a.z != MT_RSEQ_NONE) {
                plan[k] = (a.z > d.min_seq) ? -2 : -1;
                prev = -1;
            } else if (a.y <= d.min_seq) {
                const bool ok = prev >= 0 && can_append(plen, pmark, pnl, a.x, mk) &&
                                match_props(d, pprops, b.y) && a.x > 0;
                if (ok) {
                    plan[k] = prev;
                    if (pend != (int)b.x) need += 1;  // needs a copy (flag)
                    pend = pend == (int)b.x ? (int)b.x + a.x : -1;
                    plen += a.x;
                    glen[prev] = plen;
                    pnl = tb[b.x + a.x - 1] == '\n';
                } else {
                    plan[k] = -2;
                    prev = k;
                    plen = a.x;
                    pmark = mk;
                    pnl = !mk && a.x > 0 && tb[b.x + a.x - 1] == '\n';
                    pprops = b.y;
                    pend = (int)b.x + a.x;
                }
            } else {
                plan[k] = -2;
                prev = -1;
            }
        }
    }
    WSYNC();
    need = bcast(need, 0);
    if (need) {
        // total bytes of groups that are not contiguous
        int tot = 0;
        for (int k = 0; k < cntb; k++)
            if (plan[k] == -2) tot += glen[k];
        if (!text_ensure(d, tot)) return cntb;
    }
    // execute text merges group by group (uniform loops; cntb <= 8)
    for (int k = 0; k < cntb; k++) {
        if (plan[k] != -2 || glen[k] == d.A[s + k].x) continue;
        // keeper k with appended followers
        uint4 bk = d.Bv[s + k];
        int4 ak = d.A[s + k];
        bool contig = true;
        int endp = (int)bk.x + ak.x;
        for (int j = k + 1; j < cntb && plan[j] == k; j++) {
            const uint4 bj = d.Bv[s + j];
            if ((int)bj.x != endp) contig = false;
            endp += d.A[s + j].x;
        }
        uint16_t *tb = text_base(d, d.text_half);
        uint32_t newoff = bk.x;
        if (!contig) {
            int dst;
            if ((int)bk.x + ak.x == d.text_top) {
                dst = d.text_top + 0;
                newoff = bk.x;
                dst = d.text_top;
            } else {
                newoff = (uint32_t)d.text_top;
                wave_copy16(tb + d.text_top, tb + bk.x, ak.x);
                dst = d.text_top + ak.x;
            }
            for (int j = k + 1; j < cntb && plan[j] == k; j++) {
                const uint4 bj = d.Bv[s + j];
                const int lj = d.A[s + j].x;
                wave_copy16(tb + dst, tb + bj.x, lj);
                dst += lj;
            }
            d.text_top = dst;
        }
        WSYNC();
        if (lane() == 0) {
            d.A[s + k].x = glen[k];
            d.Bv[s + k].x = newoff;
        }
        WSYNC();
    }
    // compaction: survivors to the front of the block, tail moved left
    int keep = 0;
    for (int k = 0; k < cntb; k++) keep += plan[k] == -2 ? 1 : 0;
    if (keep < cntb) {
        int4 a;
        u64 o;
        uint4 b;
        int dst = -1;
        if (lane() < cntb && plan[lane()] == -2) {
            a = d.A[s + lane()];
            o = d.O[s + lane()];
            b = d.Bv[s + lane()];
            int r = 0;
            for (int k = 0; k < lane(); k++) r += plan[k] == -2 ? 1 : 0;
            dst = s + r;
        }
        WSYNC();
        if (dst >= 0) {
            d.A[dst] = a;
            d.O[dst] = o;
            d.Bv[dst] = b;
        }
        WSYNC();
        const int from = e, k = cntb - keep;
        seg_move_left(d, from, k);
        d.n -= k;
    }
    return keep;
}

// pack :1401-1453 starting from the underflowing block b of level l
__device__ void pack(Doc &d, int l, int b) {
    while (true) {
        int c0;
        const int P = blk_find(d, l + 1, b, true, c0);
        if (P < 0) {
            fail(d, MT_DOC_INTERNAL);
            return;
        }
        const int nch = lvl(d, l + 1)[P];
        int total = 0;
        if (l == 0) {
            int pos = blk_prefix(d, 0, c0);
            for (int cb = c0; cb < c0 + nch; cb++) {
                const int old = lvl(d, 0)[cb];
                const int kept = scour_block(d, pos, pos + old);
                if (d.status) return;
                WSYNC();
                if (lane() == 0) lvl(d, 0)[cb] = (uint8_t)kept;
                WSYNC();
                pos += kept;
                total += kept;
            }
        } else {
            for (int cb = c0; cb < c0 + nch; cb++) total += lvl(d, l)[cb];
        }
        int k = total / MT_HALF;
        if (k > MT_MAXN - 1) k = MT_MAXN - 1;
        if (k < 1) k = 1;
        const int base = total / k, extra = total % k;
        blk_replace(d, l, c0, nch, k, base, extra);
        if (lane() == 0) lvl(d, l + 1)[P] = (uint8_t)k;
        WSYNC();
        if (k < MT_HALF && l + 2 < d.depth) {
            l = l + 1;
            b = P;
            continue;
        }
        return;
    }
}

// zamboniSegments :1455-1511
__device__ void zamboni(Doc &d) {
    for (int it = 0; it < MT_ZAMBONI && d.status == 0; it++) {
        if (d.heap_n == 0) break;
        const int2 top = heap_top(d);
        if (top.x > d.min_seq) break;
        heap_pop(d);
        const int i = find_uid(d, (uint32_t)top.y);
        if (i < 0) continue;
        int bstart;
        const int b = blk_find(d, 0, i, true, bstart);
        if (b < 0) {
            fail(d, MT_DOC_INTERNAL);
            return;
        }
        const int f = d.flg[b];
        const int old = lvl(d, 0)[b];
        WSYNC();
        if (f == 0) continue;
        const int kept = scour_block(d, bstart, bstart + old);
        if (d.status) return;
        WSYNC();
        if (lane() == 0) {
            d.flg[b] = 0;
            lvl(d, 0)[b] = (uint8_t)kept;
        }
        WSYNC();
        if (kept < old && kept < MT_HALF && d.depth > 1) pack(d, 0, b);
    }
}

// ------------------------------------------------------------------ ops
// Client.applyInsertOp MT/client.ts:394-442 -> MergeTree.insertSegments :2001-2031
__device__ void op_insert(Doc &d, const mt_op_rec &op, const uint16_t *tin, const uint32_t *pin) {
    const int r = op.ref_seq, c = op.client, seq = op.seq, p = op.pos1;
    const bool marker = (op.flags & MT_F_MARKER) != 0;
    const int slen = marker ? 1 : op.pos2;
    // pass: split point, first index with prefix >= p, first tie-able index at prefix == p
    int carry = 0, split_i = -1, split_q = 0, ip = -1, js = -1;
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        const bool v = i < d.n;
        const int4 a = v ? d.A[i] : make_int4(0, 0, MT_RSEQ_NONE, 0);
        const u64 o = v ? d.O[i] : 0ull;
        const int vl = v ? view_len(a, o, r, c) : 0;
        const int inc = wave_scan_incl(vl);
        const int pex = carry + inc - vl, pin_ = carry + inc;
        const u64 ms = ballot(v && pex < p && p < pin_);
        if (ms) {
            const int l = first_lane(ms);
            split_i = base + l;
            split_q = p - bcast(pex, l);
            break;
        }
        const u64 mi = ballot(v && pex >= p);
        if (ip < 0 && mi) ip = base + first_lane(mi);
        const u64 mj = ballot(v && pex == p && (vl > 0 || tie(a, r)));
        if (mj) {
            js = base + first_lane(mj);
            break;
        }
        carry += bcast(inc, MT_WAVE - 1);
        if (ballot(v && pex > p)) break;
    }
    if (split_i >= 0) {
        split_seg(d, split_i, split_q);
        if (d.status) return;
        ip = js = split_i + 1;
    } else if (ip < 0 && carry == p) {
        ip = d.n;
    }
    Cb cb = cb_begin(d, seq, MT_OP_INSERT);
    if (slen == 0) {  // zero-length segment: boundary only, not inserted (:2229)
        cb.n = 1;
        cb_log(d, -1);
        cb_log(d, 0);
        cb.h = fnv_u64(cb.h, fnv_u32(fnv_u32(MT_FNV_OFF, (uint32_t)-1), 0u));
        cb_end(d, cb);
        zamboni(d);
        return;
    }
    if (ip < 0) {
        fail(d, MT_DOC_INSERT_FAILED);  // :2243-2249
        return;
    }
    if (d.n + 1 > d.S_cap) {
        fail(d, MT_DOC_CAPACITY);
        return;
    }
    if (!marker && !text_ensure(d, slen)) return;
    uint32_t ph = 0;
    if (op.props != MT_NO_PROPS) {
        if (!props_ensure(d, 1)) return;
        ph = (uint32_t)d.props_top;
        d.props_top++;
        const uint32_t *rec = pin + op.props;
        const uint32_t cntk = rec[0] & 0xFFFF;
        if (lane() == 0) {
            uint32_t *t = prec(d, d.props_half, ph);
            uint32_t n = 0;
            for (uint32_t j = 0; j < cntk; j++) {
                if (rec[2 + 2 * j] == MT_VAL_NULL) continue;  // null dropped (Q5)
                if (n < MT_KMAX) {
                    t[1 + 2 * n] = rec[1 + 2 * j];
                    t[2 + 2 * n] = rec[2 + 2 * j];
                }
                n++;
            }
            t[0] = n;
        }
        int cn = 0;
        for (uint32_t j = 0; j < cntk; j++) cn += rec[2 + 2 * j] != MT_VAL_NULL;
        if (cn > MT_KMAX) {
            fail(d, MT_DOC_CAPACITY);
            return;
        }
    }
    int bstart;
    const int B = blk_find(d, 0, ip, false, bstart);
    if (B < 0) {
        fail(d, MT_DOC_INTERNAL);
        return;
    }
    const int bend = bstart + lvl(d, 0)[B];
    const int x = (js >= 0 && js < bend) ? js : bend;
    uint32_t toff;
    if (marker) {
        toff = op.payload;
    } else {
        toff = (uint32_t)d.text_top;
        wave_copy16(text_base(d, d.text_half) + d.text_top, tin + op.payload, slen);
        d.text_top += slen;
    }
    seg_move_right(d, x, 1);
    const uint32_t uid = (uint32_t)d.next_uid;
    if (lane() == 0) {
        d.A[x] = make_int4(slen, seq, MT_RSEQ_NONE, pack_cli(c, 0));
        d.O[x] = 0ull;
        d.Bv[x] = make_uint4(toff, ph, uid | (marker ? MT_MARKER_BIT : 0u), 0u);
    }
    d.next_uid++;
    d.n++;
    const int nc = lvl(d, 0)[B] + 1;
    WSYNC();
    if (lane() == 0) lvl(d, 0)[B] = (uint8_t)nc;
    WSYNC();
    int lb = B;
    if (nc == MT_MAXN) {
        blk_split_up(d, 0, B);
        if (d.status) return;
        if (x - bstart >= MT_HALF) lb = B + 1;
    }
    if (seq > d.min_seq) add_to_lru_block(d, lb, uid, seq);  // saveIfLocal :2197-2212
    // delta callback: position of the new segment in the observer view
    const int pos = obs_prefix(d, x);
    cb.n = 1;
    cb_log(d, pos);
    cb_log(d, slen);
    cb.h = fnv_u64(cb.h, fnv_u32(fnv_u32(MT_FNV_OFF, (uint32_t)pos), (uint32_t)slen));
    cb_end(d, cb);
    zamboni(d);
}

// SegmentPropertiesManager.addProperties MT/segmentPropertiesManager.ts:35-111 applied by
// one lane to its segment: writes the new record nh, returns the seg hash contribution of
// the propertyDeltas (and logs them when `log` is set).  Returns false on key overflow.
__device__ bool annotate_record(Doc &d, uint32_t oh, uint32_t nh, const uint32_t *rec,
                                u64 &sh, int32_t *logp, int &nlog) {
    const uint32_t cntk = rec[0] & 0xFFFF, comb = rec[0] >> 16;
    const uint32_t *o = oh ? prec(d, d.props_half, oh) : nullptr;
    uint32_t *t = prec(d, d.props_half, nh);
    const uint32_t on = o ? o[0] : 0;
    uint32_t n = 0;
    int npd = 0;
    // rewrite: delete keys whose new value is not truthy (:66-79)
    for (uint32_t i = 0; i < on; i++) {
        const uint32_t k = o[1 + 2 * i], v = o[2 + 2 * i];
        bool in_new = false, truthy = false;
        if (comb == MT_COMBINE_REWRITE) {
            for (uint32_t j = 0; j < cntk; j++)
                if (rec[1 + 2 * j] == k) {
                    in_new = true;
                    const uint32_t nv = rec[2 + 2 * j];
                    truthy = nv != MT_VAL_NULL && !(nv & MT_VAL_FALSY_BIT);
                }
        }
        if (comb == MT_COMBINE_REWRITE && !truthy) {
            const uint32_t dv = in_new ? MT_VAL_NULL : v;
            sh = fnv_u32(fnv_u32(sh, k), dv);
            if (logp) {
                logp[nlog++] = (int32_t)k;
                logp[nlog++] = (int32_t)dv;
            }
            npd++;
        } else {
            t[1 + 2 * n] = k;
            t[2 + 2 * n] = v;
            n++;
        }
    }
    for (uint32_t j = 0; j < cntk; j++) {
        const uint32_t k = rec[1 + 2 * j], v = rec[2 + 2 * j];
        int idx = -1;
        for (uint32_t q = 0; q < n; q++)
            if (t[1 + 2 * q] == k) idx = (int)q;
        bool deleted_by_rewrite = false;
        if (comb == MT_COMBINE_REWRITE && idx < 0) {
            for (uint32_t i = 0; i < on; i++)
                if (o[1 + 2 * i] == k) deleted_by_rewrite = true;
        }
        if (!deleted_by_rewrite) {
            const uint32_t dv = idx >= 0 ? t[2 + 2 * idx] : MT_VAL_NULL;
            sh = fnv_u32(fnv_u32(sh, k), dv);
            if (logp) {
                logp[nlog++] = (int32_t)k;
                logp[nlog++] = (int32_t)dv;
            }
            npd++;
        }
        if (v == MT_VAL_NULL) {
            if (idx >= 0) {
                for (uint32_t q = (uint32_t)idx + 1; q < n; q++) {
                    t[2 * q - 1] = t[2 * q + 1];
                    t[2 * q] = t[2 * q + 2];
                }
                n--;
            }
        } else if (idx >= 0) {
            t[2 + 2 * idx] = v;
        } else {
            if (n >= MT_KMAX) return false;
            t[1 + 2 * n] = k;
            t[2 + 2 * n] = v;
            n++;
        }
    }
    t[0] = n;
    sh = fnv_u32(sh, (uint32_t)npd);
    return true;
}

// markRangeRemoved :2640-2752 / annotateRange :2598-2638.  After the two boundary splits
// the visited leaves are exactly those with view length > 0 inside [p1, p2) (nodeMap
// :2936-2998 is tree-shape independent), processed in document order.
__device__ void op_range(Doc &d, const mt_op_rec &op, const uint32_t *pin) {
    const int r = op.ref_seq, c = op.client, seq = op.seq, p1 = op.pos1, p2 = op.pos2;
    const bool rem = op.kind == MT_OP_REMOVE;
    const uint32_t *rec = (!rem && op.props != MT_NO_PROPS) ? pin + op.props : nullptr;
    if (rec && (rec[0] >> 16) == MT_COMBINE_OTHER) {
        fail(d, MT_DOC_UNSUPPORTED);
        return;
    }
    boundary(d, p1, r, c);
    if (d.status) return;
    boundary(d, p2, r, c);
    if (d.status) return;
    compute_ends(d);
    Cb cb = cb_begin(d, seq, op.kind);
    int carry = 0, ocarry = 0, last_b = -1;
    const int L = lane();
    for (int base = 0; base < d.n; base += MT_WAVE) {
        if (!rem && !props_ensure(d, MT_WAVE)) return;
        const int i = base + L;
        const bool v = i < d.n;
        int4 a = v ? d.A[i] : make_int4(0, 0, MT_RSEQ_NONE, 0);
        const u64 o = v ? d.O[i] : 0ull;
        const uint4 bv = v ? d.Bv[i] : make_uint4(0, 0, 0, 0);
        const int vl = v ? view_len(a, o, r, c) : 0;
        const int inc = wave_scan_incl(vl);
        const int pex = carry + inc - vl, pin_ = carry + inc;
        const bool sel = v && vl > 0 && pex < p2 && pin_ > p1;
        const u64 sel_m = ballot(sel);
        bool newly = false, bad = false;
        if (rem && sel) {
            if (a.z != MT_RSEQ_NONE) {          // addOverlappingClient :2577-2585
                if (c < 1 || c > 64)
                    bad = true;
                else
                    d.O[i] = o | (1ull << (c - 1));
            } else {
                newly = true;
                a.z = seq;
                a.w = pack_cli(seg_cli(a), c);
                d.A[i] = a;
            }
        }
        uint32_t nh = 0;
        if (!rem && sel) nh = (uint32_t)(d.props_top + __popcll(sel_m & ((1ull << L) - 1ull)));
        // observer positions after marking (getPosition at callback time)
        const int ol = v ? obs_len(a) : 0;
        const int oinc = wave_scan_incl(ol);
        const int opos = ocarry + oinc - ol;
        const bool entry = rem ? newly : sel;
        u64 sh = fnv_u32(fnv_u32(MT_FNV_OFF, (uint32_t)opos), (uint32_t)a.x);
        if (!rem && sel) {
            int unused = 0;
            if (!annotate_record(d, bv.y, nh, rec ? rec : &kEmptyPropsRec, sh, nullptr, unused)) bad = true;
            d.Bv[i].y = nh;
        }
        if (ballot(bad)) {
            fail(d, MT_DOC_CAPACITY);
            return;
        }
        if (!rem) d.props_top += __popcll(sel_m);
        WSYNC();
        // fold the callback records in document order
        u64 em = ballot(entry);
        while (em) {
            const int j = first_lane(em);
            em &= em - 1;
            cb.h = fnv_u64(cb.h, bcast64(sh, j));
            cb.n++;
            if (d.dlog) {
                cb_log(d, bcast(opos, j));
                cb_log(d, bcast(a.x, j));
                if (!rem) {
                    // re-derive this segment's propertyDeltas into the log (debug only)
                    const uint32_t ohj = (uint32_t)bcast((int)bv.y, j), nhj = (uint32_t)bcast((int)nh, j);
                    (void)ohj;
                    int nl = 0;
                    u64 dummy = 0;
                    const int at = d.dlog_n + 1;
                    if (L == 0 && at + 4 * MT_KMAX + 2 <= d.DL_cap) {
                        // old record is untouched (new record went to a fresh handle)
                        annotate_record(d, ohj, nhj, rec ? rec : &kEmptyPropsRec, dummy, d.dlog + at, nl);
                        d.dlog[at - 1] = nl / 2;
                    }
                    nl = bcast(nl, 0);
                    d.dlog_n += 1 + nl;
                }
            }
        }
        // addToLRUSet for every visited segment, first one per leaf block (:2680-2689)
        const int b = sel ? block_of(d, i) : -1;
        const u64 below = sel_m & ((1ull << L) - 1ull);
        const int prevl = below ? 63 - __clzll((long long)below) : -1;
        const int pb = __shfl(b, prevl < 0 ? 0 : prevl, MT_WAVE);
        const int prev_b = prevl < 0 ? last_b : pb;
        u64 fm = ballot(sel && b != prev_b);
        while (fm) {
            const int j = first_lane(fm);
            fm &= fm - 1;
            add_to_lru_block(d, bcast(b, j), (uint32_t)bcast((int)(bv.z & ~MT_MARKER_BIT), j), seq);
        }
        if (sel_m) last_b = bcast(b, 63 - __clzll((long long)sel_m));
        carry += bcast(inc, MT_WAVE - 1);
        ocarry += bcast(oinc, MT_WAVE - 1);
        if (ballot(v && pex >= p2)) break;
    }
    cb_end(d, cb);
    zamboni(d);
}

// updateSeqNumbers / updateMinSeq / setMinSeq  MT/client.ts:821-828, 991-1004,
// MT/mergeTree.ts:1751-1769
__device__ void update_seq(Doc &d, int msn, int seq) {
    if (!(d.cur_seq <= seq)) {
        fail(d, MT_DOC_SEQ_ORDER);
        return;
    }
    d.cur_seq = seq;
    if (!(msn <= seq) || !(d.min_seq <= msn)) {
        fail(d, MT_DOC_MINSEQ_ORDER);
        return;
    }
    if (msn > d.min_seq) {
        d.min_seq = msn;
        zamboni(d);
    }
}

// Client.applyMsg MT/client.ts:797-819 for one encoded record
__device__ void apply_op(Doc &d, const mt_op_rec &op, const uint16_t *tin, const uint32_t *pin) {
    if (op.kind == MT_OP_INSERT) {
        op_insert(d, op, tin, pin);
    } else if (op.kind == MT_OP_REMOVE || op.kind == MT_OP_ANNOTATE) {
        op_range(d, op, pin);
    }
    if (d.status) return;
    if (op.kind != MT_OP_NOOP) {   // completeAndLogOp asserts MT/client.ts:451-479
        if (!(d.cur_seq < op.seq)) {
            fail(d, MT_DOC_SEQ_ORDER);
            return;
        }
        if (!(d.min_seq <= op.min_seq)) {
            fail(d, MT_DOC_MINSEQ_ORDER);
            return;
        }
    }
    if (!(op.flags & MT_F_GROUP_MORE)) update_seq(d, op.min_seq, op.seq);
}
