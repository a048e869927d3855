// mt_engine.h -- the per-document replay engine executed by one wavefront.
//
// Every function here is called by all 64 lanes with wave-uniform arguments; scalar
// document state lives in the (uniform) Doc struct, the B-tree counts in LDS, and the
// segment table + zamboni heap in the storage tier the engine is instantiated for:
//
//   TierLds  the whole segment table and heap are staged into LDS for the launch (the
//            common case: C2 documents hold <= ~100 live segments).  A document that
//            outgrows the LDS capacities is *not* written back: it is flagged for retry
//            and the same batch is replayed for it by the TierGlb instantiation.
//   TierGlb  the segment table and heap stay in HBM (fallback for large documents).
//
// Text and property records always live in HBM.  The semantics follow the reference
// observer replica; oracle/mt_oracle.c is the function-by-function
// CPU restatement this engine is tested against.  Reference paths below are relative to
// /root/reference/packages/dds/merge-tree/src/ ("MT/").
#pragma once
#include <type_traits>

#include "mt_device.h"

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

// kLog: the delta log (a debug/verification feature) is compiled in only when a handle asks
// for one, so the replay fast path does not carry its registers.
template <bool kLogT> struct TierLdsT {
    static constexpr bool kLds = true;
    static constexpr bool kLog = kLogT;
    static constexpr bool kPaged = false;
    static constexpr bool kLive = false;
    // removedClientOverlap masks of short ids 1..32 (4 bytes per segment in LDS); a
    // document that needs ids 33..64 continues in the next tier (lds_room / load_doc)
    static constexpr int kOvlBits = 32;
    static constexpr bool kMayGrow = false;
    static constexpr bool kOvf = false;
    typedef uint32_t O_v;
    typedef LDS_AS v4i *A_t;
    typedef LDS_AS uint32_t *O_t;
    typedef LDS_AS v4u *B_t;
    typedef LDS_AS v2i *H_t;
};
template <bool kLogT> struct TierGlbT {
    static constexpr bool kLds = false;
    static constexpr bool kLog = kLogT;
    static constexpr bool kPaged = false;
    static constexpr bool kLive = false;
    static constexpr int kOvlBits = 64;
    static constexpr bool kMayGrow = false;
    static constexpr bool kOvf = false;
    typedef u64 O_v;
    typedef GLB_AS v4i *A_t;
    typedef GLB_AS u64 *O_t;
    typedef GLB_AS v4u *B_t;
    typedef GLB_AS v2i *H_t;
};
// Live-client documents (mt_device.h MT_LOCAL_BASE): the HBM tier plus the local client's
// unacked ops and segment groups (MT/client.ts:164-274, 589-626, 709-893); every segment also
// carries its segment-group FIFO (DocT.P, moved with the segment).
template <bool kLogT> struct TierLiveT {
    static constexpr bool kLds = false;
    static constexpr bool kLog = kLogT;
    static constexpr bool kPaged = false;
    static constexpr bool kLive = true;
    static constexpr int kOvlBits = 64;
    static constexpr bool kMayGrow = false;
    static constexpr bool kOvf = false;
    typedef u64 O_v;
    typedef GLB_AS v4i *A_t;
    typedef GLB_AS u64 *O_t;
    typedef GLB_AS v4u *B_t;
    typedef GLB_AS v2i *H_t;
};

// Live-client documents staged in LDS: the LDS tier's storage with the live semantics; the
// segment-group FIFOs (DocT.P), the group table and the queue stay in HBM at the same
// segment indices, so a document that outgrows the LDS capacities spills and continues in
// TierLiveT exactly as an observer continues in TierGlbT.
template <bool kLogT> struct TierLiveLdsT {
    static constexpr bool kLds = true;
    static constexpr bool kLog = kLogT;
    static constexpr bool kPaged = false;
    static constexpr bool kLive = true;
    static constexpr int kOvlBits = 32;
    static constexpr bool kMayGrow = false;
    static constexpr bool kOvf = false;
    typedef uint32_t O_v;
    typedef LDS_AS v4i *A_t;
    typedef LDS_AS uint32_t *O_t;
    typedef LDS_AS v4u *B_t;
    typedef LDS_AS v2i *H_t;
};

// The paged layout (mt_paged.h): LDS-staged window and upper levels.  kPaged compiles the
// page bookkeeping in; the flat tiers carry none of it.  kNarrow: removedClientOverlap masks
// of short ids 1..32 in LDS (window and unsettled table: 4 bytes per segment instead of 8) --
// a tight tier for documents with few writers; one whose clients above 32 remove overlapping
// ranges continues in the full tier.
// kBigT: the instantiation the growth step launches for documents in the big region (their
// paged arrays at DevState.big[bslot[doc]], mt_replay.hip "growth step"); every other
// launch reads the main arrays and never sees such a document.
// kPackedT: 12-byte unsettled-table entries in LDS (mt_paged.h "packed table"; a tight tier
// whose table dominates its LDS footprint, e.g. C4: 64 writers, minSeq ~1k messages behind).
// kPPT / kPHT / kUTT (0: from PagedCaps at run time): LDS capacities fixed at compile time --
// the launch's LDS layout becomes constant offsets and the capacities immediates, so the
// kernel keeps none of them in registers (the bench's C3 tight tier, mt_replay.hip launch_paged).
// kHMT: the page metadata (observer length, leaf-block counts, needsScour flags) stays in HBM
// (mt_paged.h "page metadata accessors"): no LDS per page instead of 12 bytes, for documents
// of thousands of pages (the skewed bench's long classes); with or without the delta log
// (kLogT: P_HM_LOG, round 6), not with segment ordinals (their per-page characters follow the
// LDS page metadata: mt_replay.hip use_hm).
template <bool kLogT, bool kNarrowT = false, bool kBigT = false, bool kPackedT = false, int kPPT = 0, int kPHT = 0,
          int kUTT = 0, bool kHMT = false>
struct TierPagedT {
    static constexpr int kPP = kPPT, kPH = kPHT, kUT = kUTT;
    static constexpr bool kHM = kHMT;
    static constexpr bool kBig = kBigT;
    static constexpr bool kPacked = kPackedT;
    // a last-tier instantiation (runtime capacities, wide masks, full table entries): the
    // launches the growth step may serve (PagedCaps.grow)
    static constexpr bool kMayGrow = !kNarrowT && !kPackedT && kPPT == 0;
    // 64-bit overlap masks: the tier keeps overflow overlap sets (MT_OVF_BIT)
    static constexpr bool kOvf = !kNarrowT;
    static constexpr bool kLds = true;
    static constexpr bool kLog = kLogT;
    static constexpr bool kPaged = true;
    static constexpr bool kLive = false;
    static constexpr int kOvlBits = kNarrowT ? 32 : 64;
    typedef typename std::conditional<kNarrowT, uint32_t, u64>::type O_v;
    typedef LDS_AS v4i *A_t;
    typedef LDS_AS O_v *O_t;
    typedef LDS_AS v4u *B_t;
    typedef LDS_AS v2i *H_t;
};

// Cross-lane ordering inside one wavefront.  LDS instructions of a wave execute in order,
// so the LDS tier only needs the compiler not to reorder; global memory written by one
// lane and read by another waits for the stores to complete.
__device__ __forceinline__ void gsync() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// Before a lane reads global data (text, property records) that another lane of the same
// wavefront stored earlier: a workgroup-scope acquire-release fence, the memory model's own
// form for this.  The AMDGPU memory model gives lanes of one wavefront (and waves of one
// workgroup, outside tgsplit mode) a single coherent vector L1 on gfx950, so the backend
// lowers this fence to an ordering constraint with no wait; -DMT_STRICT_GSYNC adds
// s_waitcnt vmcnt(0) anyway (measured: no difference on the C3 bench, r2 A/B).
__device__ __forceinline__ void gsync_rd() {
#ifdef MT_STRICT_GSYNC
    gsync();
#endif
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
}
template <class T> __device__ __forceinline__ void wsync() {
    if constexpr (T::kLds && !T::kLive)   // live: the HBM-resident group FIFOs move too
        asm volatile("" ::: "memory");
    else
        gsync();
}

// segB.w flags
#define SEGF_NL_KNOWN 1u   // SEGF_NL is valid
#define SEGF_NL 2u         // the segment's text ends with '\n' (TextSegment.canAppend :63-68)
#define SEGF_NOMATCH 4u    // its property set holds a value matchProperties never finds equal
                           // (MT_VAL_NOMATCH_BIT: NaN / undefined from a combining op, Q4)
#define SEGF_NONL 8u       // its text holds no '\n' at all: every piece a split makes ends
                           // without one (the trailing-'\n' flag is known without a text read)
#define SEGF_SLACK_SHIFT 16 // bits 16..31: arena units reserved after the text for appends
__device__ __forceinline__ int text_slack(int len) { return min((len >> 1) + 8, 4096); }

__device__ static const uint32_t kEmptyPropsRec = 0u;

template <class T> struct DocT {
    DocHdr *hp;   // generic: POD struct copies
    typename T::A_t A;
    typename T::O_t O;
    typename T::B_t Bv;
    typename T::H_t heap;
    GLB_AS uint16_t *text;
    GLB_AS uint32_t *props;
    GLB_AS int32_t *dlog;
    int32_t S_cap, B_cap, H_cap, T_cap, P_cap, DL_cap;
    // LDS
    LDS_AS uint8_t *cnt;    // [MT_LV][B_cap]
    LDS_AS int8_t *flg;     // [B_cap]
    LDS_AS uint16_t *ends;  // [B_cap] scratch: level-0 block end indices
    LDS_AS int32_t *scr;    // [64] scratch (scour plans)
    LDS_AS int32_t *nb;     // [MT_LV] blocks per level
    // scalars (uniform)
    int n, depth, heap_n, cur_seq, min_seq, text_top, text_half, props_top, props_half, next_uid,
        status, dlog_n, text_gcs, props_gcs, cap_cause;
    u64 dhash;
    int m_split, m_append, m_unlink;   // maintenance events (kept only when T::kLog)
    int dlog_rec, dlog_ovf;            // open log record header (-1: none), log overflowed
    int rich;                          // rich delta log (segments' state, maintenance events)
    // paged windows (segment_ordinals): the insert callback's [uid, position, ordinal] entry
    // is written after the op's page split (pg_op_insert), as the reference reads it once the
    // whole insertingWalk is done; dfr_rec = its record's first word (-1: none pending)
    int dfr_rec, dfr_uid, dfr_pos;
    // segment ordinals (logging handles with segment_ordinals): each segment's and each
    // block's own ordinal character, in HBM -- DevState.ordS / ordB for flat documents; for a
    // paged window the current page's slot / leaf-block characters, for the paged upper
    // instance the characters of levels >= 1 by level position (mt_paged.h "ordinals")
    int ord;
    int obst;                          // per-level stride of ob (st.B)
    GLB_AS uint16_t *os;               // [S]
    GLB_AS uint16_t *ob;               // [MT_LV][obst]
    int wide;               // an overlap mask holds a slot above 32 (DocHdr.pad0 bit 0)
    // overlap slots (mt_device.h ovl_has): lane i holds the client owning slot i + 1
    // (MT_OSLOT_FREE); ocs = the current message's client's slot (0: none)
    int ocli;
    int ocs;
    GLB_AS int32_t *oslot;  // this document's [64][2] {client, last seq} in HBM
    int dlo;                // paged window: lowest slot written since the page was loaded /
                            // written back (only [dlo, n) goes back to HBM)
    // paged documents (mt_paged.h): this DocT is a window onto one page, or the instance
    // holding the levels >= 1 of the tree (dir != nullptr); all zero for flat documents
    int paged;              // 1: window onto one page
    int obs_base;           // observer position of the window's first segment
    int pend_split;         // the page reached MaxNodesInBlock leaf blocks: split it after the op
    int pend_second;        // leaf block split while a page split was pending (-1: none)
    LDS_AS uint16_t *dir;   // upper instance: page ids in level-1 order (moved with level 1)
    int sp_pg, sp_l, sp_r;  // upper instance, segment ordinals: the page split blk_split_up links in
                            // at level 1 (new page id, blocks of the two halves; pg_split_page)
    // live-client documents (T::kLive): collabWindow.localSeq, the segment-group queue
    // (head id, length; MT/mergeTree.ts pendingSegments) and the current message's group
    int local_seq, g_head, g_n;
    int lop;                // the current message is the local client's own op
    int lg;                 // its segment group id
    GLB_AS int32_t *grp;    // [LG + 1][MT_GRP_WORDS] group table (index = id)
    GLB_AS u64 *P;          // [S][4] each segment's pending segment groups (mt_device.h PendQ)
    int LG;                 // group ids 1..LG
#ifdef MT_PROF
    LDS_AS u64 *prof;       // [128] section timers: ticks [0, 64), calls / counts [64, 128)
#endif
};

#define TD template <class T> __device__ __forceinline__
// live documents: segment i's pending-group FIFO in HBM (4 words)
TD PendQ pq_get(DocT<T> &d, int i) {
    const GLB_AS u64 *w = d.P + 4 * (size_t)i;
    return PendQ{{w[0], w[1], w[2], w[3]}};
}
TD void pq_put(DocT<T> &d, int i, const PendQ &q) {
    GLB_AS u64 *w = d.P + 4 * (size_t)i;
    w[0] = q.w[0];
    w[1] = q.w[1];
    w[2] = q.w[2];
    w[3] = q.w[3];
}

#ifdef MT_PROF
// per-wave accumulators live in LDS (no global atomics inside the timed sections: they
// would be waited for by the engine's s_waitcnt vmcnt(0)); added to DevState.prof at the end
#define PROF_WRAP_BEGIN const unsigned long long _t0 = __builtin_amdgcn_s_memtime();
#define PROF_WRAP_END(k)                                                              \
    if (lane() == 0) {                                                                \
        d.prof[k] += __builtin_amdgcn_s_memtime() - _t0;                              \
        d.prof[64 + k] += 1ull;                                                       \
    }
#endif

// MT_PROF2 (with MT_PROF): finer timers, P2 slot k (9..15) in slot k + 17
#if defined(MT_PROF) && defined(MT_PROF2)
#define P2_T0(k) const unsigned long long _p2##k = __builtin_amdgcn_s_memtime();
#define P2_T1(k)                                                         \
    if (lane() == 0) {                                                   \
        d.prof[k + 17] += __builtin_amdgcn_s_memtime() - _p2##k;         \
        d.prof[64 + k + 17] += 1ull;                                     \
    }
#else
#define P2_T0(k)
#define P2_T1(k)
#endif

// Makes the document's uniform state opaque to the optimiser at the top of every message:
// nothing derived from it is hoisted across messages (hoisted loop invariants of the fully
// inlined engine were spilling hundreds of SGPRs).
template <class P> __device__ __forceinline__ void opq_ptr(P &p) {
    if constexpr (sizeof(P) == 8) {
        uint64_t v = (uint64_t)p;
        uint32_t lo = (uint32_t)uni((int)(uint32_t)v), hi = (uint32_t)uni((int)(uint32_t)(v >> 32));
        asm volatile("" : "+s"(lo), "+s"(hi));
        p = (P)(((uint64_t)hi << 32) | lo);
    } else {
        uint32_t v = (uint32_t)(uintptr_t)p;
        v = (uint32_t)uni((int)v);
        asm volatile("" : "+s"(v));
        p = (P)(uintptr_t)v;
    }
}
__device__ __forceinline__ void opq(int &x) {
    x = uni(x);
    asm volatile("" : "+s"(x));
}
TD void opaque(DocT<T> &d) {
    opq(d.n); opq(d.depth); opq(d.heap_n); opq(d.cur_seq); opq(d.min_seq); opq(d.text_top);
    opq(d.text_half); opq(d.props_top); opq(d.props_half); opq(d.next_uid); opq(d.status);
    opq(d.dlog_n); opq(d.S_cap); opq(d.B_cap); opq(d.H_cap); opq(d.T_cap); opq(d.P_cap); opq(d.DL_cap);
    opq_ptr(d.text); opq_ptr(d.props); opq_ptr(d.dlog); opq_ptr(d.hp);
    opq_ptr(d.cnt); opq_ptr(d.flg); opq_ptr(d.ends); opq_ptr(d.scr); opq_ptr(d.nb);
    opq_ptr(d.A); opq_ptr(d.O); opq_ptr(d.Bv); opq_ptr(d.heap);
}

// B-tree counts of the flat tiers: level 0 holds up to B blocks, level 1 B/2, higher
// levels B/4 (each level has at most ~1/4 of the blocks below plus the lds_room margin); the
// paged upper instance keeps MT_LV x B (its level 1 = pages).
static __host__ __device__ inline int cnt_cap(int B, int l) { return l == 0 ? B : (l == 1 ? B / 2 : B / 4); }
static __host__ __device__ inline int cnt_off(int B, int l) { return l == 0 ? 0 : (l == 1 ? B : B + B / 2 + (l - 2) * (B / 4)); }
static __host__ __device__ inline int cnt_bytes(int B) { return cnt_off(B, MT_LV); }
// level-0 block ends alias the 256-byte scratch when they fit (range_mark only)
static __host__ __device__ inline bool ends_in_scr(bool seg_in_lds, int B) { return seg_in_lds && 2 * B <= 256; }

// Per-launch LDS layout of one document (host and device agree on it).
struct LdsLayout {
    uint32_t offA, offO, offB, offH, offCnt, offFlg, offEnds, offScr, offNb, offGen, offProf, total;
};
static __host__ __device__ inline LdsLayout lds_layout(bool seg_in_lds, int S, int B, int H, int gen_words) {
    LdsLayout L;
    uint32_t o = 0;
    if (seg_in_lds) {
        L.offA = o; o += 16u * S;
        L.offB = o; o += 16u * S;
        L.offO = o; o += 4u * S;   // u32 overlap masks (TierLdsT::kOvlBits)
        L.offH = o; o += 8u * (H + 1);
    } else {
        L.offA = L.offB = L.offO = L.offH = 0;
    }
    L.offScr = o; o += 64u * 4;
    L.offNb = o; o += MT_LV * 4;
    L.offGen = o; o += 4u * gen_words;
    L.offEnds = ends_in_scr(seg_in_lds, B) ? L.offScr : o;
    if (!ends_in_scr(seg_in_lds, B)) o += 2u * B;
    L.offCnt = o; o += (uint32_t)cnt_bytes(B);
    L.offFlg = o; o += (uint32_t)B;
#ifdef MT_PROF
    o = (o + 7u) & ~7u;
    L.offProf = o; o += 128u * 8;
#else
    L.offProf = 0;
#endif
    L.total = (o + 15u) & ~15u;
    return L;
}

TD void fail(DocT<T> &d, int code) {
    if (d.status == 0) d.status = code;
}
// an inconsistent tree: the source line is kept in cap_cause (diagnostic; paged documents
// store it in their header)
#define FAIL_INTERNAL(d)                                    \
    do {                                                    \
        if ((d).status == 0) (d).cap_cause = 10000 + __LINE__; \
        fail(d, MT_DOC_INTERNAL);                           \
    } while (0)
// Out of a capacity: the LDS tier hands the document to the HBM tier, which reports it.
// cause (diagnostic): 1 segments, 2 blocks, 3 heap, 4 text, 5 property records
TD void fail_cap(DocT<T> &d, int cause) {
    if (d.status == 0) d.cap_cause = cause;
    fail(d, T::kLds ? MT_DOC_RETRY : MT_DOC_CAPACITY);
}

// ------------------------------------------------------------------ overlap slots
// removedClientOverlap (MT/mergeTree.ts:2577-2585) is an unbounded list of client ids; a
// segment's overlap set only matters while the segment is unsettled (a view with refSeq >=
// minSeq sees a segment removed at <= minSeq as removed anyway).  So the masks index slots,
// not ids: a client takes a slot at its first overlapping remove and keeps it while a segment
// it marked may be unsettled (the slot's last use > minSeq); after that the slot is reused.
// Bits a reused slot left on settled segments are never consulted.  Slots 1..63: bit 63 marks
// an overflow set (MT_OVF_BIT): when every slot is taken, a last-tier paged document keeps the
// segment's whole list in its overflow arena instead (ovf_member / ovf_mark, mt_paged.h), so
// the number of clients overlapping at once is bounded only by that arena, which the growth
// step raises; the other tiers hand such a document on (pg_room, pg_load).
#define MT_SLOTS_OF(T) (T::kOvlBits < MT_OSLOT_USE ? T::kOvlBits : MT_OSLOT_USE)
TD int oslot_of(DocT<T> &d, int c) {
    const u64 m = ballot(d.ocli == c);
    return m ? first_lane(m) + 1 : 0;
}
// A slot for client c (the current message's remover) within T::kOvlBits; 0: none free.
TD int oslot_take(DocT<T> &d, int c) {
    const int last = d.oslot[2 * lane() + 1];
    const u64 m = ballot(lane() < MT_SLOTS_OF(T) && (d.ocli == MT_OSLOT_FREE || last <= d.min_seq));
    if (!m) return 0;
    const int s = first_lane(m);
    if (lane() == s) d.ocli = c;
    if (lane() == 0) d.oslot[2 * s] = c;
    return s + 1;
}
// Would a remove by client c need a slot none of the first T::kOvlBits can give?
TD bool oslot_short(DocT<T> &d, int c) {
    if (oslot_of(d, c)) return false;
    if (ballot(lane() < MT_SLOTS_OF(T) && d.ocli == MT_OSLOT_FREE)) return false;
    const int last = d.oslot[2 * lane() + 1];
    return !ballot(lane() < MT_SLOTS_OF(T) && last <= d.min_seq);
}
// overflow overlap sets of paged documents (mt_paged.h)
TD bool ovf_member(DocT<T> &d, u64 o, int c);
TD bool ovf_mark(DocT<T> &d, bool need, int i, u64 o, int c, int seq);
// nodeLength of a leaf in the remote view (c, r) of document d: view_len, with the segment's
// overflow set consulted instead of the slot bits when its mask carries MT_OVF_BIT (last-tier
// paged instantiations with 64-bit masks; the narrow tier never loads such a document)
TD int vlen(DocT<T> &d, v4i a, u64 o, int r, int c) {
    if constexpr (T::kPaged && T::kOvf) {
        if (o & MT_OVF_BIT) return ovf_member(d, o, c) ? 0 : view_len(a, 0, r, c, 0);
    }
    return view_len(a, o, r, c, d.ocs);
}

// paged instances (window: levels 0-1; upper levels: 1.. with level 1 = pages): B entries
// for levels 0 and 1, B / 4^(l-1) + 8 above (growth is checked against bcap)
// paged instances: a node above level 1 holds >= 4 children once split or repacked (pack
// regroups a parent's children max(1, min(7, n/4)) to a node), so level l >= 2 has at most
// B / 4^(l-1) nodes -- plus 8 for the few a repack leaves short (pg_room keeps 4 free per level;
// a document that needs more is handed to the growth step, which doubles B)
static __host__ __device__ inline int pcnt_cap(int B, int l) { return l <= 1 ? B : (B >> (2 * (l - 1))) + 8; }
static __host__ __device__ inline int pcnt_off(int B, int l) {
    if (l <= 1) return l * B;
    int o = 2 * B;
#pragma unroll
    for (int j = 2; j < MT_LV; j++)
        if (j < l) o += pcnt_cap(B, j);
    return o;
}
static __host__ __device__ inline int pcnt_bytes(int B) { return pcnt_off(B, MT_LV); }
TD LDS_AS uint8_t *lvl(DocT<T> &d, int l) {
    if constexpr (T::kPaged)
        return d.cnt + pcnt_off(d.B_cap, l);
    else
        return d.cnt + cnt_off(d.B_cap, l);
}
// capacity of level l
TD int bcap(DocT<T> &d, int l) {
    if constexpr (T::kPaged)
        return pcnt_cap(d.B_cap, l);
    else
        return cnt_cap(d.B_cap, l);
}
// wave-uniform reads of LDS state (kept in SGPRs)
TD int nbr(DocT<T> &d, int l) { return uni(d.nb[l]); }
TD int cntr(DocT<T> &d, int l, int b) { return uni(lvl(d, l)[b]); }
TD int flgr(DocT<T> &d, int b) { return uni(d.flg[b]); }
__device__ __forceinline__ v4i uni4(v4i a) { return v4i{uni(a.x), uni(a.y), uni(a.z), uni(a.w)}; }
__device__ __forceinline__ v2i uni2(v2i a) { return v2i{uni(a.x), uni(a.y)}; }
__device__ __forceinline__ v4u uni4(v4u a) {
    return v4u{(uint32_t)uni((int)a.x), (uint32_t)uni((int)a.y), (uint32_t)uni((int)a.z), (uint32_t)uni((int)a.w)};
}
TD GLB_AS uint16_t *text_base(DocT<T> &d, int half) { return d.text + (size_t)half * d.T_cap; }
TD GLB_AS uint32_t *prec(DocT<T> &d, int half, uint32_t h) {
    return d.props + ((size_t)half * d.P_cap + h) * MT_PREC;
}

// ------------------------------------------------------------------ load / store
// Binds the document's HBM state; for TierLds stages the segment table and heap into LDS.
// Returns false (status MT_DOC_RETRY) when the document does not fit the LDS capacities.
TD bool load_doc(DocT<T> &d, const DevState &st, int doc, LDS_AS uint8_t *smem, const LdsLayout &L,
                 int S_l, int B_l, int H_l) {
    const size_t S = st.S, B = st.B;
    d.hp = st.hdr + doc;
    d.text = (GLB_AS uint16_t *)(st.text + doc * (size_t)2 * st.T);
    d.props = (GLB_AS uint32_t *)(st.props + doc * (size_t)2 * st.P * MT_PREC);
    d.dlog = st.DL ? (GLB_AS int32_t *)(st.dlog + doc * (size_t)st.DL) : nullptr;
    d.T_cap = st.T;
    d.P_cap = st.P;
    d.DL_cap = st.DL;
    d.rich = st.DLR;
    if constexpr (T::kLog && !T::kPaged) {
        d.ord = 0;
        d.obst = 0;
        d.os = nullptr;
        d.ob = nullptr;
        if (st.ordS) {
            d.ord = 1;
            d.obst = st.B;
            d.os = (GLB_AS uint16_t *)(st.ordS + doc * (size_t)st.S);
            d.ob = (GLB_AS uint16_t *)(st.ordB + doc * (size_t)MT_LV * st.B);
        }
    }
    d.oslot = (GLB_AS int32_t *)(st.oslot + doc * (size_t)(2 * MT_OSLOTS));
    d.ocli = d.oslot[2 * lane()];
    d.ocs = 0;
    d.scr = (LDS_AS int32_t *)(smem + L.offScr);
    d.nb = (LDS_AS int32_t *)(smem + L.offNb);
    d.ends = (LDS_AS uint16_t *)(smem + L.offEnds);
    d.cnt = smem + L.offCnt;
    d.flg = (LDS_AS int8_t *)(smem + L.offFlg);
#ifdef MT_PROF
    d.prof = (LDS_AS u64 *)(smem + L.offProf);
    d.prof[lane()] = 0;
    d.prof[64 + lane()] = 0;
#endif
    GLB_AS const uint8_t *gcnt = (GLB_AS const uint8_t *)(st.cnt + doc * (size_t)MT_LV * B);
    GLB_AS const int8_t *gflg = (GLB_AS const int8_t *)(st.flg + doc * B);
    const DocHdr h = *d.hp;
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
    d.dhash = h.delta_hash;
    d.wide = h.pad0 & 1;
    if (T::kLog) {
        d.m_split = h.pad[HDR_MSPLIT];
        d.m_append = h.pad[HDR_MAPPEND];
        d.m_unlink = h.pad[HDR_MUNLINK];
        d.dlog_ovf = h.pad[HDR_DLOG_OVF];
        d.dlog_rec = -1;
    }
    d.text_gcs = 0;
    d.props_gcs = 0;
    d.cap_cause = 0;
    d.paged = 0;
    d.obs_base = 0;
    d.pend_split = 0;
    d.pend_second = -1;
    d.dir = nullptr;
    d.lop = 0;
    d.lg = 0;
    if constexpr (T::kLive) {
        const GLB_AS int32_t *lv = (const GLB_AS int32_t *)(st.live + 4 * (size_t)doc);
        d.local_seq = lv[0];
        d.g_head = lv[1];
        d.g_n = lv[2];
        d.LG = st.LG;
        d.grp = (GLB_AS int32_t *)(st.grp + (size_t)doc * (st.LG + 1) * MT_GRP_WORDS);
        d.P = (GLB_AS u64 *)(st.segP + (size_t)doc * st.S);
    }
    if (d.status) return true;   // failed earlier: the caller leaves it untouched
    if (h.pad[HDR_PAGED]) {      // lives in the paged layout: the paged kernel replays it
        d.status = MT_DOC_RETRY;
        d.cap_cause = 6;
        return false;
    }
    bool over = false;
#pragma unroll
    for (int l = 0; l < MT_LV; l++) over = over || h.n_blk[l] > cnt_cap(T::kLds ? B_l : st.B, l);
    if (!T::kLds && over) {   // cannot happen: the HBM tier's levels are sized for st.B
        d.status = MT_DOC_CAPACITY;
        d.cap_cause = 2;
        return true;
    }
    if (T::kLds) {
        d.S_cap = S_l;
        d.B_cap = B_l;
        d.H_cap = H_l;
        if (d.n > S_l || over || d.heap_n > H_l) {
            d.status = MT_DOC_RETRY;
            d.cap_cause = 6;
            return false;
        }
        d.A = (typename T::A_t)(smem + L.offA);
        d.Bv = (typename T::B_t)(smem + L.offB);
        d.O = (typename T::O_t)(smem + L.offO);
        d.heap = (typename T::H_t)(smem + L.offH);
        GLB_AS const v4i *gA = (GLB_AS const v4i *)(st.segA + doc * S);
        GLB_AS const v4u *gB = (GLB_AS const v4u *)(st.segB + doc * S);
        GLB_AS const u64 *gO = (GLB_AS const u64 *)(st.segO + doc * S);
        GLB_AS const v2i *gH = (GLB_AS const v2i *)(st.heap + doc * (size_t)(st.H + 1));
        bool wide = false;
        for (int i = lane(); i < d.n; i += MT_WAVE) {
            d.A[i] = gA[i];
            d.Bv[i] = gB[i];
            const u64 o = gO[i];
            wide = wide || (o >> T::kOvlBits) != 0ull;
            d.O[i] = (typename T::O_v)o;
        }
        if (ballot(wide)) {   // overlap ids above the LDS tier's masks
            d.status = MT_DOC_RETRY;
            d.cap_cause = 6;
            return false;
        }
        for (int i = 1 + lane(); i <= d.heap_n; i += MT_WAVE) d.heap[i] = gH[i];
    } else {
        d.S_cap = st.S;
        d.B_cap = st.B;
        d.H_cap = st.H;
        d.A = (typename T::A_t)(st.segA + doc * S);
        d.Bv = (typename T::B_t)(st.segB + doc * S);
        d.O = (typename T::O_t)(st.segO + doc * S);
        d.heap = (typename T::H_t)(st.heap + doc * (size_t)(st.H + 1));
    }
    if (lane() < MT_LV) d.nb[lane()] = d.hp->n_blk[lane()];
    wsync<T>();
    for (int l = 0; l < d.depth; l++) {
        const int nbl = nbr(d, l);
        for (int b = lane(); b < nbl; b += MT_WAVE) lvl(d, l)[b] = gcnt[l * B + b];
    }
    for (int b = lane(); b < h.n_blk[0]; b += MT_WAVE) d.flg[b] = gflg[b];
    wsync<T>();
    return true;
}

TD void store_doc(DocT<T> &d, const DevState &st, int doc) {
    wsync<T>();
    const size_t S = st.S, B = st.B;
    GLB_AS uint8_t *gcnt = (GLB_AS uint8_t *)(st.cnt + doc * (size_t)MT_LV * B);
    GLB_AS int8_t *gflg = (GLB_AS int8_t *)(st.flg + doc * B);
    if (T::kLds) {
        GLB_AS v4i *gA = (GLB_AS v4i *)(st.segA + doc * S);
        GLB_AS v4u *gB = (GLB_AS v4u *)(st.segB + doc * S);
        GLB_AS u64 *gO = (GLB_AS u64 *)(st.segO + doc * S);
        GLB_AS v2i *gH = (GLB_AS v2i *)(st.heap + doc * (size_t)(st.H + 1));
        for (int i = lane(); i < d.n; i += MT_WAVE) {
            gA[i] = d.A[i];
            gB[i] = d.Bv[i];
            gO[i] = d.O[i];
        }
        for (int i = 1 + lane(); i <= d.heap_n; i += MT_WAVE) gH[i] = d.heap[i];
    }
    d.oslot[2 * lane()] = d.ocli;
    if constexpr (T::kLive) {
        if (lane() == 0) {
            GLB_AS int32_t *lv = (GLB_AS int32_t *)(st.live + 4 * (size_t)doc);
            lv[0] = d.local_seq;
            lv[1] = d.g_head;
            lv[2] = d.g_n;
        }
    }
    for (int l = 0; l < d.depth; l++)
        for (int b = lane(); b < nbr(d, l); b += MT_WAVE) gcnt[l * B + b] = lvl(d, l)[b];
    for (int b = lane(); b < nbr(d, 0); b += MT_WAVE) gflg[b] = d.flg[b];
    int nbl[MT_LV];
#pragma unroll
    for (int l = 0; l < MT_LV; l++) nbl[l] = nbr(d, l);
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
#pragma unroll
        for (int l = 0; l < MT_LV; l++) h.n_blk[l] = nbl[l];
        h.delta_hash = d.dhash;
        h.n_ops = d.hp->n_ops;
        h.pad0 = d.wide;
#pragma unroll
        for (int i = 0; i < 8; i++) h.pad[i] = 0;
        h.pad[HDR_DIAG] = d.status ? d.cap_cause : 0;
        if (T::kLog) {
            h.pad[HDR_MSPLIT] = d.m_split;
            h.pad[HDR_MAPPEND] = d.m_append;
            h.pad[HDR_MUNLINK] = d.m_unlink;
            h.pad[HDR_DLOG_OVF] = d.dlog_ovf;
        }
        *d.hp = h;
    }
}

// A paged window records the lowest slot an engine step writes (mark_dirty); the flat
// tiers compile it out.
TD void mark_dirty(DocT<T> &d, int i) {
#if defined(MT_NO_DIRTY)
#elif defined(MT_FULL_WRITEBACK)
    if constexpr (T::kPaged) d.dlo = 0;
#else
    if constexpr (T::kPaged) d.dlo = min(d.dlo, i);
#endif
}

// Segment ordinals are kept by the logging instantiations only (the replay fast path
// compiles them out).
TD bool ordon(DocT<T> &d) {
    if constexpr (T::kLog)
        return d.ord != 0;
    else
        return false;
}
// paged layout (mt_paged.h): nodeUpdateOrdinals below the upper instance's block b of level l
// (its pages' leaf blocks and segments are in HBM), and the ordinal of a window segment
TD void pg_ord_canon_up(DocT<T> &up, int l, int b);
TD int pg_ord_of_win(DocT<T> &w, int i, int *codes);
// setOrdinal's width for a block of c children (mt_engine.h "segment ordinals")
__device__ __forceinline__ int ord_w(int c) { return 1 << (7 - min(max(c, 1), 7)); }
// lane 0 writes one ordinal character (a global store other lanes read after gsync)
__device__ __forceinline__ void ord_put(GLB_AS uint16_t *p, int v) {
    if (lane() == 0) *p = (uint16_t)v;
    gsync();
}

// ------------------------------------------------------------------ segment table moves
// [from, n) -> [from + k, n + k)
TD void seg_move_right(DocT<T> &d, int from, int k) {
    mark_dirty(d, from);
    const bool om = ordon(d);
    for (int hi = d.n; hi > from; hi -= MT_WAVE) {
        const int lo = max(from, hi - MT_WAVE);
        const int i = lo + lane();
        v4i a;
        u64 o;
        PendQ pq = pq_zero();
        v4u b;
        uint16_t oc = 0;
        if (i < hi) {
            a = d.A[i];
            o = d.O[i];
            b = d.Bv[i];
            if constexpr (T::kLive) pq = pq_get(d, i);
            if (om) oc = d.os[i];
        }
        wsync<T>();
        if (i < hi) {
            d.A[i + k] = a;
            d.O[i + k] = o;
            d.Bv[i + k] = b;
            if constexpr (T::kLive) pq_put(d, i + k, pq);
            if (om) d.os[i + k] = oc;
        }
        wsync<T>();
    }
    if (om) gsync();
}
// [from, n) -> [from - k, n - k)
TD void seg_move_left(DocT<T> &d, int from, int k) {
    mark_dirty(d, from - k);
    const bool om = ordon(d);
    for (int lo = from; lo < d.n; lo += MT_WAVE) {
        const int i = lo + lane();
        v4i a;
        u64 o;
        PendQ pq = pq_zero();
        v4u b;
        uint16_t oc = 0;
        if (i < d.n) {
            a = d.A[i];
            o = d.O[i];
            b = d.Bv[i];
            if constexpr (T::kLive) pq = pq_get(d, i);
            if (om) oc = d.os[i];
        }
        wsync<T>();
        if (i < d.n) {
            d.A[i - k] = a;
            d.O[i - k] = o;
            d.Bv[i - k] = b;
            if constexpr (T::kLive) pq_put(d, i - k, pq);
            if (om) d.os[i - k] = oc;
        }
        wsync<T>();
    }
    if (om) gsync();
}

// Loads a segment's {A, O} for a scan lane.  The load is unconditional (inactive lanes read
// slot 0) and pinned in registers: a 64-bit LDS/global load that the compiler sinks into a
// divergent branch was observed to return wrong masks on gfx950 / ROCm 7.2.
TD void load_ao(DocT<T> &d, int i, bool v, v4i &a, u64 &o) {
    const int ic = v ? i : 0;
    a = d.A[ic];
    o = d.O[ic];
    asm volatile("" : "+v"(a), "+v"(o));
    if (!v) {
        a = v4i{0, 0, MT_RSEQ_NONE, 0};
        o = 0ull;
    }
}

// ------------------------------------------------------------------ B-tree counts (LDS)
// First block b of level l whose end (prefix of counts) is > x (strict) or >= x.
TD int blk_find(DocT<T> &d, int l, int x, bool strict, int &start) {
    const LDS_AS uint8_t *c = lvl(d, l);
    const int nb = nbr(d, l);
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
TD int blk_prefix(DocT<T> &d, int l, int b) {
    const LDS_AS uint8_t *c = lvl(d, l);
    int s = 0;
    for (int base = 0; base < b; base += MT_WAVE) {
        const int i = base + lane();
        s += wave_sum(i < b ? c[i] : 0);
    }
    return s;
}
// shift entries [from, nb) of level l by delta (right if > 0), flags too at level 0
TD void blk_shift(DocT<T> &d, int l, int from, int delta) {
    LDS_AS uint8_t *c = lvl(d, l);
    const int nb = nbr(d, l);
    if (T::kPaged && d.dir && l == 1 && delta) {   // paged upper instance: page ids move with level 1
        LDS_AS uint16_t *dr = d.dir;
        if (delta > 0) {
            for (int hi = nb; hi > from; hi -= MT_WAVE) {
                const int lo = max(from, hi - MT_WAVE);
                const int i = lo + lane();
                uint16_t v = 0;
                if (i < hi) v = dr[i];
                wsync<T>();
                if (i < hi) dr[i + delta] = v;
                wsync<T>();
            }
        } else {
            for (int lo = from; lo < nb; lo += MT_WAVE) {
                const int i = lo + lane();
                uint16_t v = 0;
                if (i < nb) v = dr[i];
                wsync<T>();
                if (i < nb) dr[i + delta] = v;
                wsync<T>();
            }
        }
    }
    const bool om = ordon(d);
    GLB_AS uint16_t *oc = om ? d.ob + (size_t)l * d.obst : nullptr;   // block ordinal characters
    if (delta > 0) {
        for (int hi = nb; hi > from; hi -= MT_WAVE) {
            const int lo = max(from, hi - MT_WAVE);
            const int i = lo + lane();
            uint8_t v = 0;
            int8_t f = 0;
            uint16_t ov = 0;
            if (i < hi) {
                v = c[i];
                if (l == 0) f = d.flg[i];
                if (om) ov = oc[i];
            }
            wsync<T>();
            if (i < hi) {
                c[i + delta] = v;
                if (l == 0) d.flg[i + delta] = f;
                if (om) oc[i + delta] = ov;
            }
            wsync<T>();
        }
    } else if (delta < 0) {
        for (int lo = from; lo < nb; lo += MT_WAVE) {
            const int i = lo + lane();
            uint8_t v = 0;
            int8_t f = 0;
            uint16_t ov = 0;
            if (i < nb) {
                v = c[i];
                if (l == 0) f = d.flg[i];
                if (om) ov = oc[i];
            }
            wsync<T>();
            if (i < nb) {
                c[i + delta] = v;
                if (l == 0) d.flg[i + delta] = f;
                if (om) oc[i + delta] = ov;
            }
            wsync<T>();
        }
    }
    if (om) gsync();
    wsync<T>();
    if (lane() == 0) d.nb[l] = nb + delta;
    wsync<T>();
}

// A block at level l reached MaxNodesInBlock: split 4|4 and propagate (insertingWalk
// :2479-2503, split :2509-2522, updateRoot :1909-1920).  New blocks have needsScour
// undefined; the original keeps its flag.
TD void blk_split_up(DocT<T> &d, int l, int b) {
    // paged window: level 1 is the page itself; its split (a new level-1 node) is done by
    // the paged driver after the op.  A second leaf split while it is pending is recorded:
    // it decides which half ends up with 5 blocks (reference order: split page, then leaf).
    if (T::kPaged && d.paged && l == 0 && d.pend_split) d.pend_second = b;
    while (true) {
        if (T::kPaged && d.paged && l == 1) {
            d.pend_split = 1;
            return;
        }
        if (nbr(d, l) + 1 > bcap(d, l)) {
            fail_cap(d, 2);
            return;
        }
        const bool has_parent = l + 1 < d.depth;
        int pstart = 0, P = -1;
        if (has_parent) {
            P = blk_find(d, l + 1, b, true, pstart);
            if (P < 0) {
                FAIL_INTERNAL(d);
                return;
            }
        }
        blk_shift(d, l, b + 1, 1);
        if (lane() == 0) {
            lvl(d, l)[b] = MT_HALF;
            lvl(d, l)[b + 1] = MT_HALF;
            if (l == 0) d.flg[b + 1] = MT_SCOUR_UNDEF;
            // the paged upper instance's page split: its halves' real leaf-block counts and the
            // new page id are in place before any re-derivation reads them (pg_ord_canon_up)
            if (T::kPaged && ordon(d) && d.dir && l == 1) {
                lvl(d, 1)[b] = (uint8_t)d.sp_l;
                lvl(d, 1)[b + 1] = (uint8_t)d.sp_r;
                d.dir[b + 1] = (uint16_t)d.sp_pg;
            }
        }
        wsync<T>();
        if (!has_parent) {
            const int nl = d.depth;
            if (nl >= MT_LV) {
                fail_cap(d, 2);
                return;
            }
            d.depth++;
            if (lane() == 0) {
                d.nb[nl] = 1;
                lvl(d, nl)[0] = 2;
            }
            wsync<T>();
            if (ordon(d)) ord_canon_all(d);   // updateRoot: nodeUpdateOrdinals(root)
            return;
        }
        const int pc = cntr(d, l + 1, P) + 1;
        wsync<T>();
        if (lane() == 0) lvl(d, l + 1)[P] = (uint8_t)pc;
        wsync<T>();
        if (pc < MT_MAXN) {
            // the propagation stops here: the new half is linked after the old one
            // (setOrdinal) and re-derived (nodeUpdateOrdinals(fromSplit)); the old half was
            // re-derived by its split -- each re-derivation covers every split below
            if (ordon(d)) {
                ord_put(ordl(d, l) + b + 1, uni((int)ordl(d, l)[b]) + ord_w(pc));
                ord_canon(d, l, b);
                ord_canon(d, l, b + 1);
            }
            return;
        }
        l = l + 1;
        b = P;
    }
}

// Replace entries [b0, b0 + nold) of level l with k entries sized base (+1 for the first
// `extra`), as pack :1414-1446 does; new level-0 blocks have needsScour undefined.
TD void blk_replace(DocT<T> &d, int l, int b0, int nold, int k, int base, int extra) {
    if (nbr(d, l) + (k - nold) > bcap(d, l)) {
        fail_cap(d, 2);
        return;
    }
    blk_shift(d, l, b0 + nold, k - nold);
    LDS_AS uint8_t *c = lvl(d, l);
    for (int j = lane(); j < k; j += MT_WAVE) {
        c[b0 + j] = (uint8_t)(base + (j < extra ? 1 : 0));
        if (l == 0) d.flg[b0 + j] = MT_SCOUR_UNDEF;
    }
    wsync<T>();
}

// level-0 end indices into LDS (for per-lane block lookups)
TD void compute_ends(DocT<T> &d) {
    const LDS_AS uint8_t *c = lvl(d, 0);
    const int nb = nbr(d, 0);
    int carry = 0;
    for (int base = 0; base < nb; base += MT_WAVE) {
        const int b = base + lane();
        const int v = b < nb ? c[b] : 0;
        const int inc = wave_scan_incl(v);
        if (b < nb) d.ends[b] = (uint16_t)(carry + inc);
        carry += bcast(inc, MT_WAVE - 1);
    }
    wsync<T>();
}
// first block with end > i (binary search over d.ends; per-lane)
TD int block_of(DocT<T> &d, int i, int nb) {
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (d.ends[mid] > i)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}

// ------------------------------------------------------------------ segment ordinals
// MergeBlock.setOrdinal (MT/mergeTree.ts:347-372): a child's ordinal is its parent's plus one
// character -- at index 0 width - 1, otherwise the previous sibling's last character + width,
// width = 1 << (MaxNodesInBlock - (childCount + 1)) with childCount capped at 7 -- and
// nodeUpdateOrdinals (:2553-2575) re-derives a whole subtree that way (child q of a block
// with c children: (q + 1) * width(c) - 1).  Only these two write ordinals, and between
// messages every node's ordinal is its parent's plus its own last character (checked on the
// reference over C2/C3/C4 streams: oracle/ref_harness.mjs ordprobe, tests/test_events.py; a
// loaded summary whose body re-inserts segments breaks it -- MT_DOC_ALIASED), so
// the engine keeps one character per node (DocT.os / DocT.ob) and spells an ordinal out
// only to log it.
// Where the reference writes them (Q8: the characters are not unique, SequenceDeltaEvent
// drops ranges whose ordinals collide):
//   insert before an existing segment (blockInsert's onLeaf replaceCurrent :2437-2441): the
//     new segment takes the existing one's character, which gets its own + width;
//   insert at a block end, or a split's right half (:2483-2486): previous sibling's + width;
//   a block that overflows (:2487-2503, split :2509-2522): every split half's subtree is
//     re-derived; the level where the propagation stops gives the new half previous + width;
//     a new root (updateRoot :1909-1920) re-derives the whole tree;
//   zamboni's shrunk block (:1486-1501) and pack's topmost parent (:1444-1450) are re-derived.
TD GLB_AS uint16_t *ordl(DocT<T> &d, int l) { return d.ob + (size_t)l * d.obst; }

// nodeUpdateOrdinals(block b of level l): every node below it gets its canonical character
TD void ord_canon(DocT<T> &d, int l, int b) {
    if constexpr (T::kPaged) {
        if (d.dir) {   // the paged upper instance: levels 1 and 0 are pages in HBM
            pg_ord_canon_up(d, l, b);
            return;
        }
    }
    int lo = b, hi = b + 1;
    for (int j = l; j >= 0; j--) {
        const int c0 = blk_prefix(d, j, lo);
        int carry = c0;
        GLB_AS uint16_t *dst = j == 0 ? d.os : ordl(d, j - 1);
        const LDS_AS uint8_t *cnt = lvl(d, j);
        for (int base = lo; base < hi; base += MT_WAVE) {
            const int p = base + lane();
            const int c = p < hi ? (int)cnt[p] : 0;
            const int inc = wave_scan_incl(c);
            const int first = carry + inc - c;
            const int w = ord_w(c);
            for (int q = 0; q < c; q++) dst[first + q] = (uint16_t)((q + 1) * w - 1);
            carry += bcast(inc, MT_WAVE - 1);
        }
        lo = c0;
        hi = carry;
    }
    gsync();
}
// the whole tree (updateRoot, reloadFromSegments)
TD void ord_canon_all(DocT<T> &d) { ord_canon(d, d.depth - 1, 0); }

// the ordinal of segment i: its ancestors' characters below the root, then its own
// (codes[0 .. depth)); returns the length
TD int ord_of(DocT<T> &d, int i, int *codes) {
    if constexpr (T::kPaged) return pg_ord_of_win(d, i, codes);
    const int dep = d.depth;
    gsync();
    codes[dep - 1] = uni((int)d.os[i]);
    int x = i;
    for (int l = 0; l + 1 < dep; l++) {
        int st;
        const int b = blk_find(d, l, x, true, st);
        if (b < 0) return -1;
        codes[dep - 2 - l] = uni((int)ordl(d, l)[b]);
        x = b;
    }
    return dep;
}

// ------------------------------------------------------------------ zamboni heap
// Collections.Heap add/get (MT/collections.ts:212-265), comparer maxSeq (LRUSegmentComparer
// MT/mergeTree.ts:957-960); touched by lane 0 only.  (A wave-parallel fixdown -- five levels
// loaded at once, the path followed with readlane -- measured slower: 1.8k -> 2.9k cycles
// per pop on C3, profiles/r2/sections_c3_v2.log.)
TD void heap_add(DocT<T> &d, int max_seq, int uid) {
    if (d.heap_n + 1 > d.H_cap) {
        fail_cap(d, 3);
        return;
    }
    d.heap_n++;
    if (lane() == 0) {
        typename T::H_t h = d.heap;
        int k = d.heap_n;
        const v2i e = v2i{max_seq, uid};
        while (k > 1) {
            const v2i p = h[k >> 1];
            if (!(p.x - e.x > 0)) break;
            h[k] = p;
            k >>= 1;
        }
        h[k] = e;
    }
}
TD v2i heap_top(DocT<T> &d) {
    int x = 0, y = 0;
    if (lane() == 0) {
        const v2i t = d.heap[1];
        x = t.x;
        y = t.y;
    }
    return v2i{bcast(x, 0), bcast(y, 0)};
}
TD void heap_pop(DocT<T> &d) {
    if (lane() == 0) {
        typename T::H_t h = d.heap;
        const int n = d.heap_n - 1;
        const v2i e = h[d.heap_n];
        int k = 1;
        while ((k << 1) <= n) {
            int j = k << 1;
            // both children in one LDS round trip (h[n + 1] is the entry being moved: in bounds)
            v2i cj = h[j];
            const v2i cj1 = h[j + 1];
            if (j < n && cj.x - cj1.x > 0) {
                j++;
                cj = cj1;
            }
            if (e.x - cj.x <= 0) break;
            h[k] = cj;
            k = j;
        }
        h[k] = e;
    }
    d.heap_n--;
}

TD int find_uid(DocT<T> &d, uint32_t uid) {
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        const u64 m = ballot(i < d.n && (d.Bv[i].z & ~MT_MARKER_BIT) == uid);
        if (m) return base + first_lane(m);
    }
    return -1;
}

// sum of observer lengths over [0, x)  (getPosition :1619-1636 in the observer view)
#ifdef MT_PROF
TD int obs_prefix_impl(DocT<T> &d, int x);
TD int obs_prefix(DocT<T> &d, int x) {
    PROF_WRAP_BEGIN
    auto _r = obs_prefix_impl(d, x);
    PROF_WRAP_END(8)
    return _r;
}
TD int obs_prefix_impl(DocT<T> &d, int x) {
#else
TD int obs_prefix(DocT<T> &d, int x) {
#endif
    int s = 0;
    for (int base = 0; base < x; base += MT_WAVE) {
        const int i = base + lane();
        s += i < x ? obs_len(d.A[i]) : 0;
    }
    return wave_sum(s);
}

// ------------------------------------------------------------------ text arena
// dst/src in the same arena half; callers gsync() before reading text written this launch
TD void copy_text(GLB_AS uint16_t *dst, const GLB_AS uint16_t *src, int n) {
    for (int j = lane(); j < n; j += MT_WAVE) dst[j] = src[j];
}
// Compact all live text (non-removed TextSegments) into the other half, document order.
#ifdef MT_PROF
TD void text_gc_impl(DocT<T> &d);
TD void text_gc(DocT<T> &d) {
    PROF_WRAP_BEGIN
    text_gc_impl(d);
    PROF_WRAP_END(5)
    
}
TD void text_gc_impl(DocT<T> &d) {
#else
TD void text_gc(DocT<T> &d) {
#endif
    d.text_gcs++;
    gsync_rd();
    const int dh = 1 - d.text_half;
    GLB_AS uint16_t *dst = text_base(d, dh);
    const GLB_AS uint16_t *src = text_base(d, d.text_half);
    int carry = 0;
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        v4i a = v4i{0, 0, 0, 0};
        v4u b = v4u{0, 0, 0, 0};
        if (i < d.n) {
            a = d.A[i];
            b = d.Bv[i];
        }
        // (a rich delta log keeps removed segments' text: their UNLINK event reports it)
        // (a live document keeps the text of segments in a pending group: regeneratePendingOp
        // re-creates an unacked insert the local client has removed since)
        bool keep = a.z == MT_RSEQ_NONE || (T::kLog && d.rich);
        if constexpr (T::kLive) keep = keep || (i < d.n && pq_any(pq_get(d, i)));
        const bool live = i < d.n && keep && !(b.z & MT_MARKER_BIT);
        const int len = live ? a.x : 0;
        const int inc = wave_scan_incl(len);
        const int off = carry + inc - len;
        u64 m = ballot(live && len > 0);
        while (m) {
            const int j = first_lane(m);
            m &= m - 1;
            const int lj = bcast(len, j), oj = bcast(off, j), sj = bcast((int)b.x, j);
            copy_text<T>(dst + oj, src + sj, lj);
        }
        wsync<T>();
        if (live) {
            v4u nb = b;
            nb.x = (uint32_t)off;
            nb.w &= 0xFFFFu;   // compaction drops the append slack
            d.Bv[i] = nb;
        }
        carry += bcast(inc, MT_WAVE - 1);
    }
    d.text_half = dh;
    d.text_top = carry;
    wsync<T>();
}
TD bool paged_text_ensure(DocT<T> &d, int need);
TD bool paged_props_ensure(DocT<T> &d, int need);
TD bool text_ensure(DocT<T> &d, int need) {
    if (d.text_top + need <= d.T_cap) return true;
    if constexpr (T::kPaged) {
        if (d.paged) return paged_text_ensure(d, need);
    }
    text_gc(d);
    if (d.status) return false;
    if (d.text_top + need <= d.T_cap) return true;
    fail_cap(d, 4);
    return false;
}

// ------------------------------------------------------------------ property records
TD void props_gc(DocT<T> &d) {
    d.props_gcs++;
    gsync_rd();
    const int dh = 1 - d.props_half;
    int carry = 1;
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        uint32_t h = i < d.n ? d.Bv[i].y : 0;
        const int has = h != 0;
        const int inc = wave_scan_incl(has);
        const uint32_t nh = (uint32_t)(carry + inc - has);
        if (has) {
            const GLB_AS uint32_t *s = prec(d, d.props_half, h);
            GLB_AS uint32_t *t = prec(d, dh, nh);
            const uint32_t n = s[0];
            t[0] = n;
            for (uint32_t k = 0; k < 2 * n; k++) t[1 + k] = s[1 + k];
        }
        wsync<T>();
        if (has) d.Bv[i].y = nh;
        carry += bcast(inc, MT_WAVE - 1);
    }
    d.props_half = dh;
    d.props_top = carry;
    gsync_rd();
    wsync<T>();
}
TD bool props_ensure(DocT<T> &d, int need) {
    if (d.props_top + need <= d.P_cap) return true;
    if constexpr (T::kPaged) {
        if (d.paged) return paged_props_ensure(d, need);
    }
    props_gc(d);
    if (d.status) return false;
    if (d.props_top + need <= d.P_cap) return true;
    fail_cap(d, 5);
    return false;
}
// Properties.matchProperties MT/properties.ts:61-92 over interned ids; nm: either set holds a
// NaN / undefined value (SEGF_NOMATCH), which no comparison finds equal
TD bool match_props(DocT<T> &d, uint32_t ha, uint32_t hb, bool nm) {
    if (ha == 0 || hb == 0) return ha == hb;
    if (nm) return false;
    if (ha == hb) return true;
    const GLB_AS uint32_t *a = prec(d, d.props_half, ha), *b = prec(d, d.props_half, hb);
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
// Every mergeTreeDeltaCallback folds into the document's delta hash.  Delta-logging handles
// (T::kLog) also append the record [seq, kind, n, entries...] to the document's log.  A
// record is written whole or not at all: when the next words of the open record do not fit,
// the partial record is dropped and the log is marked overflowed (sticky until
// mt_delta_log_reset), so a reader never sees a count without its entries.
struct Cb {
    u64 h;
    int n;
};
TD Cb cb_begin(DocT<T> &d, int seq, int kind) {
    Cb cb;
    cb.h = fnv_u32(fnv_u32(MT_FNV_OFF, (uint32_t)seq), (uint32_t)kind);
    cb.n = 0;
    if constexpr (T::kLog) {
        d.dlog_rec = -1;
        if (d.dlog) {
            if (!d.dlog_ovf && d.dlog_n + 3 <= d.DL_cap) {
                d.dlog_rec = d.dlog_n;
                if (lane() == 0) {
                    d.dlog[d.dlog_n] = seq;
                    d.dlog[d.dlog_n + 1] = kind;
                }
                d.dlog_n += 3;
            } else {
                d.dlog_ovf = 1;
            }
        }
    }
    return cb;
}
// Room for `words` more words of the open record; on overflow the record is dropped.
TD bool cb_room(DocT<T> &d, int words) {
    if constexpr (T::kLog) {
        if (!d.dlog || d.dlog_rec < 0) return false;
        if (d.dlog_n + words <= d.DL_cap) return true;
        d.dlog_n = d.dlog_rec;
        d.dlog_rec = -1;
        d.dlog_ovf = 1;
    }
    return false;
}
TD void cb_end(DocT<T> &d, Cb &cb) {
    cb.h = fnv_u32(cb.h, (uint32_t)cb.n);
    d.dhash = fnv_u64(d.dhash, cb.h);
    if constexpr (T::kLog) {
        if (d.dlog && d.dlog_rec >= 0 && lane() == 0) d.dlog[d.dlog_rec + 2] = cb.n;
        d.dlog_rec = -1;
    }
}
TD void cb_log(DocT<T> &d, int32_t v) {
    if (cb_room(d, 1)) {
        if (lane() == 0) d.dlog[d.dlog_n] = v;
        d.dlog_n++;
    }
}

// Rich delta log (handles with delta_log_mode 1): every logged segment also carries its
// state at the event -- [flags (1 marker, 2 has properties), marker: refType | text: the
// UTF-16 units two per word, n (-1: no properties), (key, value) x n] -- and the
// mergeTreeMaintenanceCallback events are records of their own (kind SPLIT -2, APPEND -1,
// UNLINK -3; MT/mergeTreeDeltaCallback.ts:15-30): [seq, kind, n, (cachedLength, state) x n].
// A segment's text is the concatenation of np pieces (an APPEND's merged segment).
struct TextPieces {
    uint32_t off[8];
    int len[8];
    int np;
};
TD void cb_log_state(DocT<T> &d, bool marker, uint32_t ref_type, const TextPieces &tp, const GLB_AS uint32_t *pr) {
    if constexpr (T::kLog) {
        int tot = 0;
        for (int q = 0; q < tp.np; q++) tot += tp.len[q];
        const int words = marker ? 1 : (tot + 1) / 2;
        if (pr) gsync_rd();   // a record another lane may just have written
        const int np = pr ? (int)pr[0] : -1;
        if (!cb_room(d, 2 + words + 2 * max(np, 0))) return;
        GLB_AS int32_t *o = d.dlog + d.dlog_n;
        if (lane() == 0) {
            o[0] = (marker ? 1 : 0) | (pr ? 2 : 0) | (ordon(d) ? 4 : 0);
            if (marker) o[1] = (int32_t)ref_type;
            o[1 + words] = np;
        }
        if (!marker && tot > 0) {
            gsync_rd();
            const GLB_AS uint16_t *tb = text_base(d, d.text_half);
            for (int w = lane(); w < words; w += MT_WAVE) {
                uint32_t u[2] = {0u, 0u};
                for (int h = 0; h < 2; h++) {
                    int t = 2 * w + h, pre = 0;
                    for (int q = 0; q < tp.np; q++) {
                        if (t >= pre && t < pre + tp.len[q]) u[h] = tb[tp.off[q] + (t - pre)];
                        pre += tp.len[q];
                    }
                }
                o[1 + w] = (int32_t)(u[0] | (u[1] << 16));
            }
        }
        for (int q = lane(); q < 2 * np; q += MT_WAVE) o[2 + words + q] = (int32_t)pr[1 + q];
        d.dlog_n += 2 + words + 2 * max(np, 0);
    }
}
// After a rich entry's state on a segment_ordinals handle (flags bit 4): [uid, observer
// position of the segment at the event as Client.getPosition reads it then, ordinal length
// (-1: the segment has none -- never linked), ordinal characters].  zero_suffix: the SPLIT
// event's right half, whose ordinal is the left half's + "\0" until it is linked
// (BaseSegment.splitAt :531-535).
TD void cb_log_ext(DocT<T> &d, uint32_t uid, int pos, int seg_i, bool zero_suffix) {
    if constexpr (T::kLog) {
        if (!ordon(d) || !d.rich) return;
        int codes[MT_LV + 1];
        int olen = seg_i >= 0 ? ord_of(d, seg_i, codes) : -1;
        if (olen >= 0 && zero_suffix) codes[olen++] = 0;
        if (!cb_room(d, 3 + max(olen, 0))) return;
        GLB_AS int32_t *o = d.dlog + d.dlog_n;
        if (lane() == 0) {
            o[0] = (int32_t)uid;
            o[1] = pos;
            o[2] = olen;
            for (int q = 0; q < olen; q++) o[3 + q] = codes[q];
        }
        d.dlog_n += 3 + max(olen, 0);
    }
}
TD void cb_log_seg(DocT<T> &d, v4i a, v4u b) {
    if constexpr (T::kLog) {
        if (!d.rich) return;
        TextPieces tp;
        tp.np = 1;
        tp.off[0] = b.x;
        tp.len[0] = a.x;
        cb_log_state(d, (b.z & MT_MARKER_BIT) != 0, b.x, tp, b.y ? prec(d, d.props_half, b.y) : nullptr);
    }
}
// a maintenance record of one or two segments
// (uid / pos / seg index of each segment for cb_log_ext; i1z: the second one is a split's
// unlinked right half)
struct MaintExt {
    uint32_t uid0, uid1;
    int pos0, pos1, i0, i1;
    bool z1;
};
TD void cb_maint(DocT<T> &d, int kind, int len0, bool mk0, uint32_t ref0, const TextPieces &t0, uint32_t ph0,
                 int len1, const TextPieces *t1, uint32_t ph1, const MaintExt &ex) {
    if constexpr (T::kLog) {
        if (!d.rich || !d.dlog) return;
        Cb cb = cb_begin(d, d.cur_seq, kind);
        cb_log(d, len0);
        cb_log_state(d, mk0, ref0, t0, ph0 ? prec(d, d.props_half, ph0) : nullptr);
        cb_log_ext(d, ex.uid0, ex.pos0, ex.i0, false);
        cb.n = 1;
        if (t1) {
            cb_log(d, len1);
            cb_log_state(d, false, 0u, *t1, ph1 ? prec(d, d.props_half, ph1) : nullptr);
            cb_log_ext(d, ex.uid1, ex.pos1, ex.i1, ex.z1);
            cb.n = 2;
        }
        // maintenance events are not part of the delta hash (the hash pins the delta callbacks)
        if (d.dlog && d.dlog_rec >= 0 && lane() == 0) d.dlog[d.dlog_rec + 2] = cb.n;
        d.dlog_rec = -1;
    }
}

// ------------------------------------------------------------------ splitting
// BaseSegment.splitAt :523-567 (right half inserted right after the left half in the same
// leaf block, which may then split).  Property records are immutable, so both halves share.
// The left half's last character is unknown until a scour needs it.
#ifdef MT_PROF
TD void split_seg_impl(DocT<T> &d, int i, int q);
TD void split_seg(DocT<T> &d, int i, int q) {
    PROF_WRAP_BEGIN
    split_seg_impl(d, i, q);
    PROF_WRAP_END(0)
    
}
TD void split_seg_impl(DocT<T> &d, int i, int q) {
#else
TD void split_seg(DocT<T> &d, int i, int q) {
#endif
    if (d.n + 1 > d.S_cap) {
        fail_cap(d, 1);
        return;
    }
    int bstart;
    const int b = blk_find(d, 0, i, true, bstart);
    if (b < 0) {
        FAIL_INTERNAL(d);
        return;
    }
    // SPLIT event positions as getPosition reads them inside the callback (segment_ordinals
    // handles): the left half's is its own; the right half is not linked yet (its parent is
    // the leaf block, which does not list it), so getPosition sums every child of the block
    // -- the block's observer end with the left half already trimmed (:1619-1636)
    MaintExt ex{0u, 0u, 0, 0, i, i, true};
    if (ordon(d) && d.rich) {
        const v4i ai = uni4(d.A[i]);
        const int ob = T::kPaged ? d.obs_base : 0;   // a paged window's observer start
        ex.pos0 = ob + obs_prefix(d, i);
        ex.pos1 = ob + obs_prefix(d, bstart + cntr(d, 0, b)) - (ai.z == MT_RSEQ_NONE ? ai.x - q : 0);
        ex.uid0 = uni((int)(d.Bv[i].z & ~MT_MARKER_BIT));
        ex.uid1 = (uint32_t)d.next_uid;
    }
    seg_move_right(d, i + 1, 1);
    mark_dirty(d, i);
    if (T::kLog) d.m_split++;   // splitLeafSegment's SPLIT event :2264-2269
    if constexpr (T::kLog) {   // SPLIT [left, right] (splitLeafSegment :2260-2272), rich log
        if (d.rich) {
            const v4i a0 = uni4(d.A[i]);
            const v4u b0 = uni4(d.Bv[i]);
            TextPieces l, rt;
            l.np = rt.np = 1;
            l.off[0] = b0.x;
            l.len[0] = q;
            rt.off[0] = b0.x + (uint32_t)q;
            rt.len[0] = a0.x - q;
            cb_maint(d, -2, q, false, 0u, l, b0.y, a0.x - q, &rt, b0.y, ex);
        }
    }
    if (lane() == 0) {
        v4i a = d.A[i];
        v4u bb = d.Bv[i];
        v4i r = a;
        r.x = a.x - q;
        a.x = q;
        v4u rb = bb;
        rb.x = bb.x + (uint32_t)q;
        rb.z = (uint32_t)d.next_uid | (bb.z & MT_MARKER_BIT);
        bb.w &= ~(SEGF_NL_KNOWN | SEGF_NL | (0xFFFFu << SEGF_SLACK_SHIFT));
#ifndef MT_NO_NONL
        if (bb.w & SEGF_NONL) bb.w |= SEGF_NL_KNOWN;   // a newline-free text's left part ends without one
#endif
        d.A[i] = a;
        d.Bv[i] = bb;
        d.A[i + 1] = r;
        d.O[i + 1] = d.O[i];
        d.Bv[i + 1] = rb;
        if constexpr (T::kLive) pq_put(d, i + 1, pq_get(d, i));   // the right half joins the left one's groups
    }
    d.next_uid++;
    d.n++;
    const int c = cntr(d, 0, b) + 1;
    wsync<T>();
    if (lane() == 0) lvl(d, 0)[b] = (uint8_t)c;
    wsync<T>();
    // the right half is linked after the left one: setOrdinal (:2483-2486)
    if (ordon(d)) ord_put(d.os + i + 1, uni((int)d.os[i]) + ord_w(c));
    if (c == MT_MAXN) blk_split_up(d, 0, b);
}

// ensureIntervalBoundary :2274-2278 -- split the leaf strictly containing view position p
#ifdef MT_PROF
TD void boundary_impl(DocT<T> &d, int p, int r, int c);
TD void boundary(DocT<T> &d, int p, int r, int c) {
    PROF_WRAP_BEGIN
    boundary_impl(d, p, r, c);
    PROF_WRAP_END(1)
    
}
TD void boundary_impl(DocT<T> &d, int p, int r, int c) {
#else
TD void boundary(DocT<T> &d, int p, int r, int c) {
#endif
    int carry = 0;
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        const bool v = i < d.n;
        v4i a;
        u64 o;
        load_ao(d, i, v, a, o);
        const int vl = v ? vlen(d, a, o, r, c) : 0;
        const int inc = wave_scan_incl(vl);
        const int pex = carry + inc - vl, pin = carry + inc;
        const u64 m = ballot(v && pex < p && p < pin);
#ifdef MT_DEBUG_BOUNDARY
        if (T::kLog && d.dlog) {
            cb_log(d, 0x7777); cb_log(d, p); cb_log(d, r); cb_log(d, c); cb_log(d, base);
            for (int q = 0; q < 16; q++) { cb_log(d, bcast(vl, q)); cb_log(d, bcast(a.z, q)); cb_log(d, bcast(a.w, q)); cb_log(d, (int)bcast64(o, q)); }
        }
#endif
        if (m) {
            const int l = first_lane(m);
            split_seg(d, base + l, p - bcast(pex, l));
            return;
        }
        if (ballot(v && pex >= p)) return;
        carry += bcast(inc, MT_WAVE - 1);
    }
}

// addToLRUSet :1306-1316 for a segment in leaf block b
TD void add_to_lru_block(DocT<T> &d, int b, uint32_t uid, int seq) {
    const int f = flgr(d, b);
    if (f != 1 && seq > d.cur_seq) {
        wsync<T>();
        if (lane() == 0) d.flg[b] = 1;
        wsync<T>();
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

// Rich delta log: scourNode's UNLINK / APPEND events (MT/mergeTree.ts:1343-1373) of a scour,
// in child order, before any text moves.  Lane j holds entry j (a: lengths, b: text offset /
// marker refType, props); m_app: entries appended to the run before them, whose keeper is
// the nearest kept entry below (m_keep).
//
// Positions (segment_ordinals handles), as getPosition reads them inside each callback
// (:1619-1636): the scoured block's children array is untouched until the scour ends, a
// keeper has already absorbed the segments appended to it up to the current one, and an
// appended segment keeps its own length -- so for entry k of a block starting at observer
// position S, with base(j) its observer length and app(j) "appended":
//   UNLINK k, APPEND's keeper k:  S + D(k),  D(k) = sum over earlier entries j of the block
//                                             of base(j) * (1 + app(j))
//   APPEND's appended segment k:  S + D(k) + base(k)
// (pack scours several blocks; the ones before keep their cachedLength, so S is the
// pre-scour observer start).  s: table index of entry 0; ntot: entries; start: the first
// entry of this lane's block.
TD void scour_events(DocT<T> &d, v4i a, v4u b, u64 m_unlink, u64 m_app, u64 m_keep, int s, int ntot, int start) {
    if constexpr (T::kLog) {
        if (!d.rich) return;
        int pos_k = 0, base_k = 0;
        if (ordon(d) && (m_unlink | m_app)) {
            const int k = lane();
            base_k = (k < ntot && a.z == MT_RSEQ_NONE) ? a.x : 0;
            const int val = base_k * (((m_app >> k) & 1ull) ? 2 : 1);
            const int dex = wave_scan_incl(val) - val;
            const int bex = wave_scan_incl(base_k) - base_k;
            const int s0 = (T::kPaged ? d.obs_base : 0) + obs_prefix(d, s);
            pos_k = s0 + __shfl(bex, start, MT_WAVE) + dex - __shfl(dex, start, MT_WAVE);
        }
        for (u64 ev = m_unlink | m_app; ev; ev &= ev - 1) {
            const int j = first_lane(ev);
            const int lj = bcast(a.x, j);
            TextPieces tj;
            tj.np = 1;
            tj.off[0] = (uint32_t)bcast((int)b.x, j);
            tj.len[0] = lj;
            const uint32_t pj = (uint32_t)bcast((int)b.y, j);
            if ((m_app >> j) & 1ull) {
                const int kk = 63 - __clzll((long long)(m_keep & ((1ull << j) - 1ull)));
                TextPieces tk;
                tk.np = 0;
                int tot = 0;
                for (int q = kk; q <= j && tk.np < 8; q++) {
                    tk.off[tk.np] = (uint32_t)bcast((int)b.x, q);
                    tk.len[tk.np] = bcast(a.x, q);
                    tot += tk.len[tk.np];
                    tk.np++;
                }
                const MaintExt ex{(uint32_t)bcast((int)(b.z & ~MT_MARKER_BIT), kk),
                                  (uint32_t)bcast((int)(b.z & ~MT_MARKER_BIT), j), bcast(pos_k, kk),
                                  bcast(pos_k, j) + bcast(base_k, j), s + kk, s + j, false};
                cb_maint(d, -1, tot, false, 0u, tk, (uint32_t)bcast((int)b.y, kk), lj, &tj, pj, ex);
            } else {
                const bool mk = (bcast((int)b.z, j) & MT_MARKER_BIT) != 0;
                const MaintExt ex{(uint32_t)bcast((int)(b.z & ~MT_MARKER_BIT), j), 0u, bcast(pos_k, j), 0, s + j, -1,
                                  false};
                cb_maint(d, -3, lj, mk, tj.off[0], tj, pj, 0, (const TextPieces *)nullptr, 0u, ex);
            }
        }
    }
}

// scourNode :1322-1398 over leaf block [s, e); compacts the table.  Returns survivors.
#ifdef MT_PROF
TD int scour_block_impl(DocT<T> &d, int s, int e);
TD int scour_block(DocT<T> &d, int s, int e) {
    PROF_WRAP_BEGIN
    auto _r = scour_block_impl(d, s, e);
    PROF_WRAP_END(2)
    return _r;
}
TD int scour_block_impl(DocT<T> &d, int s, int e) {
#else
TD int scour_block(DocT<T> &d, int s, int e) {
#endif
    const int cntb = e - s;   // <= MaxNodesInBlock
    const int k = lane();
    const bool in = k < cntb;
    v4i a = d.A[in ? s + k : s];
    v4u b = d.Bv[in ? s + k : s];
    const bool removed = a.z != MT_RSEQ_NONE;
    const bool marker = (b.z & MT_MARKER_BIT) != 0;
    // a segment in a pending segment group is held (scourNode :1328, :1389-1392)
    bool pend = false;
    if constexpr (T::kLive) pend = in && pq_any(pq_get(d, in ? s + k : s));
    const bool settled = in && !pend && !removed && a.y <= d.min_seq;   // merge candidate
    // resolve unknown trailing-newline flags of merge candidates (lanes in parallel)
    const bool need_nl = settled && !marker && a.x > 0 && !(b.w & SEGF_NL_KNOWN);
    if (ballot(need_nl)) {
        gsync_rd();
        if (need_nl) {
            const uint16_t ch = text_base(d, d.text_half)[b.x + a.x - 1];
            b.w = (b.w & ~SEGF_NL) | SEGF_NL_KNOWN | (ch == '\n' ? SEGF_NL : 0u);
            d.Bv[s + k].w = b.w;
        }
        wsync<T>();
    }
    const u64 m_unlink = ballot(in && !pend && removed && a.z <= d.min_seq);
    const u64 m_settled = ballot(settled);
    const u64 m_mark = ballot(in && marker);
    const u64 m_nl = ballot(in && (b.w & SEGF_NL) != 0);
    // plan (scalar): owner of each entry, 4 bits per entry: its own index = survivor,
    // another index = appended to that keeper, 0xF = unlinked
    uint32_t owners = 0;
    int prev = -1, plen = 0;
    bool pmark = false, pnl = false, pnm = false;
    uint32_t pprops = 0;
    for (int j = 0; j < cntb; j++) {
        uint32_t own = (uint32_t)j;
        if ((m_unlink >> j) & 1ull) {
            own = 0xF;
            prev = -1;
        } else if (!((m_settled >> j) & 1ull)) {
            prev = -1;
        } else {
            const int lj = bcast(a.x, j);
            const bool mk = (m_mark >> j) & 1ull, nl = (m_nl >> j) & 1ull;
            const uint32_t pj = (uint32_t)bcast((int)b.y, j);
            const bool nmj = (bcast((int)b.w, j) & SEGF_NOMATCH) != 0;
            const bool ok = prev >= 0 && lj > 0 && can_append(plen, pmark, pnl, lj, mk) &&
                            match_props(d, pprops, pj, pnm || nmj);
            if (ok) {
                own = (uint32_t)prev;
                plen += lj;
                pnl = nl;
            } else {
                prev = j;
                plen = lj;
                pmark = mk;
                pnl = !mk && lj > 0 && nl;
                pprops = pj;
                pnm = nmj;
            }
        }
        owners |= own << (4 * j);
    }
    const uint32_t myown = in ? (owners >> (4 * k)) & 0xFu : 0xFu;
    const u64 m_keep = ballot(in && myown == (uint32_t)k);
    const u64 m_app = ballot(in && myown != 0xFu && myown != (uint32_t)k);
    scour_events(d, a, b, m_unlink, m_app, m_keep, s, cntb, 0);
    if (T::kLog) {   // scourNode's UNLINK / APPEND events :1343-1373
        d.m_unlink += __popcll(m_unlink);
        d.m_append += __popcll(m_app);
    }
    if (m_app) {
        mark_dirty(d, s);
        // group length per keeper (lanes that are keepers sum their members)
        int glen = 0;
        if (in && myown == (uint32_t)k) {
            for (int j = 0; j < cntb; j++) glen += ((owners >> (4 * j)) & 0xFu) == (uint32_t)k ? bcast(a.x, j) : 0;
        }
        // keepers with appended members
        u64 m_grp = 0;
        for (int j = 0; j < cntb; j++)
            if ((m_app >> j) & 1ull) m_grp |= 1ull << ((owners >> (4 * j)) & 0xFu);
        // upper bound of what the merges allocate (group text + slack)
        int tot = 0;
        for (u64 g = m_grp; g; g &= g - 1) {
            const int gl = bcast(glen, first_lane(g));
            tot += gl + text_slack(gl);
        }
        if (!text_ensure(d, tot)) return cntb;
        gsync_rd();
        // execute text merges group by group.  A keeper copied to the arena top reserves
        // slack after its text so that later appends land in place (TextSegment.append
        // :70-85 is a string concatenation; this keeps it amortised O(1)).
        LDS_AS int *psrc = d.scr + 48;   // gather pieces of one group: source offset, length
        LDS_AS int *plen_ = d.scr + 56;
        for (u64 g = m_grp; g; g &= g - 1) {
            const int kk = first_lane(g);
            const int gk = bcast(glen, kk);
            const v4u bk = uni4(d.Bv[s + kk]);   // fresh: text_ensure may have compacted
            const int ak = uni(d.A[s + kk].x);
            const uint32_t kslack = bk.w >> SEGF_SLACK_SHIFT;
            bool contig = true;
            int endp = (int)bk.x + ak, add = 0;
            uint32_t lastw = 0, nonl = bk.w & SEGF_NONL;
            for (int j = kk + 1; j < cntb && ((owners >> (4 * j)) & 0xFu) == (uint32_t)kk; j++) {
                const v4u bj = uni4(d.Bv[s + j]);
                const int lj = bcast(a.x, j);
                if ((int)bj.x != endp) contig = false;
                endp += lj;
                add += lj;
                lastw = bj.w;
                nonl &= bj.w;
            }
            uint32_t newoff = bk.x, newslack = lastw >> SEGF_SLACK_SHIFT;
            if (!contig) {
                int dst, np = 0, ntot = 0;
                if ((uint32_t)add <= kslack) {                       // append into the slack
                    dst = (int)bk.x + ak;
                    newslack = kslack - (uint32_t)add;
                } else if ((int)bk.x + ak == d.text_top) {          // keeper ends at the top
                    dst = d.text_top;
                    newslack = (uint32_t)text_slack(gk);
                    d.text_top += add + (int)newslack;
                } else {                                            // move keeper + appends
                    newoff = (uint32_t)d.text_top;
                    dst = d.text_top;
                    newslack = (uint32_t)text_slack(gk);
                    d.text_top += gk + (int)newslack;
                    if (lane() == 0) {
                        psrc[0] = (int)bk.x;
                        plen_[0] = ak;
                    }
                    np = 1;
                    ntot = ak;
                }
                for (int j = kk + 1; j < cntb && ((owners >> (4 * j)) & 0xFu) == (uint32_t)kk; j++) {
                    const int lj = bcast(a.x, j);
                    if (lane() == 0) {
                        psrc[np] = (int)d.Bv[s + j].x;
                        plen_[np] = lj;
                    }
                    ntot += lj;
                    np++;
                }
                wsync<T>();
                GLB_AS uint16_t *tb = text_base(d, d.text_half);
                for (int base = 0; base < ntot; base += MT_WAVE) {   // one gather per 64 units
                    const int t = base + lane();
                    int src = -1, pre = 0;
                    for (int q = 0; q < np; q++) {
                        const int lq = plen_[q];
                        if (src < 0 && t < pre + lq) src = psrc[q] + (t - pre);
                        pre += lq;
                    }
                    uint16_t ch = 0;
                    if (t < ntot) ch = tb[src];
                    if (t < ntot) tb[dst + t] = ch;
                }
            }
            if (lane() == 0) {
                d.A[s + kk].x = gk;
                v4u nb = bk;
                nb.x = newoff;
                nb.w = (lastw & (SEGF_NL_KNOWN | SEGF_NL)) | nonl | (newslack << SEGF_SLACK_SHIFT);
                d.Bv[s + kk] = nb;
            }
            wsync<T>();
        }
    }
    const int keep = __popcll(m_keep);
    if (keep < cntb) {
        mark_dirty(d, s);
        // compaction: survivors to the front of the block, tail moved left
        const bool surv = (m_keep >> k) & 1ull;
        v4i sa;
        u64 so;
        PendQ sp = pq_zero();
        v4u sb;
        uint16_t soc = 0;   // ordinal character: a pack re-scours before re-deriving them
        if (surv) {
            sa = d.A[s + k];
            so = d.O[s + k];
            sb = d.Bv[s + k];
            if constexpr (T::kLive) sp = pq_get(d, s + k);
            if (ordon(d)) soc = d.os[s + k];
        }
        const int dst = s + __popcll(m_keep & ((1ull << k) - 1ull));
        wsync<T>();
        if (surv) {
            d.A[dst] = sa;
            d.O[dst] = so;
            d.Bv[dst] = sb;
            if constexpr (T::kLive) pq_put(d, dst, sp);
            if (ordon(d)) d.os[dst] = soc;
        }
        wsync<T>();
        if (ordon(d)) gsync();
        seg_move_left(d, e, cntb - keep);
        d.n -= cntb - keep;
    }
    return keep;
}

// scourNode :1322-1398 applied, in order, to the consecutive leaf blocks [b0, b0 + nbk)
// whose segments start at index s -- one block for zamboniSegments, every child of the
// parent for pack.  Lane-parallel: entry j is appended to the run before it iff both are
// settled (seq <= minSeq, not removed), j is not the first of its block, neither is a
// Marker, j-1 does not end with '\n' and their property sets match (matchProperties is an
// equivalence, so comparing with j-1 equals comparing with the run's keeper).  The only
// order-dependent rule -- canAppend's 256-unit granularity (MT/textSegment.ts:63-68) --
// can only refuse an entry longer than 256 units: such ranges take the serial per-block
// plan.  Updates the level-0 counts of the blocks; returns the survivors.
TD int scour_range(DocT<T> &d, int s, int b0, int nbk) {
    int tot = 0;
    for (int q = 0; q < nbk; q++) tot += cntr(d, 0, b0 + q);
    const int k = lane();
    bool serial = tot > MT_WAVE;
    const bool in = k < tot;
    v4i a = d.A[in ? s + k : s];
    v4u b = d.Bv[in ? s + k : s];
    int start = 0;   // first index of this lane's block (relative)
    {
        int st = 0;
        for (int q = 0; q < nbk; q++) {
            if (k >= st) start = st;
            st += cntr(d, 0, b0 + q);
        }
    }
    const bool removed = a.z != MT_RSEQ_NONE;
    const bool marker = (b.z & MT_MARKER_BIT) != 0;
    bool pend = false;   // held: in a pending segment group (scourNode :1328)
    if constexpr (T::kLive) pend = in && pq_any(pq_get(d, in ? s + k : s));
    const bool cand = in && !pend && !removed && a.y <= d.min_seq;
    if (!serial) {
        // resolve unknown trailing-newline flags of merge candidates (lanes in parallel)
        const bool need_nl = cand && !marker && a.x > 0 && !(b.w & SEGF_NL_KNOWN);
        if (ballot(need_nl)) {
            P2_T0(9)
            gsync_rd();
            if (need_nl) {
                const uint16_t ch = text_base(d, d.text_half)[b.x + a.x - 1];
                b.w = (b.w & ~SEGF_NL) | SEGF_NL_KNOWN | (ch == '\n' ? SEGF_NL : 0u);
                d.Bv[s + k].w = b.w;
            }
            wsync<T>();
            P2_T1(9)
        }
    }
    const u64 m_cand = ballot(cand);
    const u64 m_mark = ballot(in && marker);
    const u64 m_nl = ballot(in && (b.w & SEGF_NL) != 0);
    const uint32_t pprops = (uint32_t)__shfl_up((int)b.y, 1, MT_WAVE);
    const bool pc = k > 0 && ((m_cand >> (k - 1)) & 1ull);
    const bool pm = k > 0 && ((m_mark >> (k - 1)) & 1ull);
    const bool pn = k > 0 && ((m_nl >> (k - 1)) & 1ull);
#ifdef MT_NO_Q4
    const u64 m_nm = 0;
#else
    const u64 m_nm = ballot(in && (b.w & SEGF_NOMATCH) != 0);
#endif
    const bool nm = ((m_nm >> k) & 1ull) || (k > 0 && ((m_nm >> (k - 1)) & 1ull));
    bool join = cand && pc && k != start && !marker && !pm && !pn && a.x > 0;
    if (join && (nm || pprops != b.y)) join = match_props(d, pprops, b.y, nm);
    const u64 m_join = ballot(join);
    if (!serial && ballot(join && a.x > MT_GRAN)) serial = true;
    if (serial) {   // rare: per-block serial plan (scour_block)
        int pos = s, kept_all = 0;
        for (int q = 0; q < nbk; q++) {
            const int old = cntr(d, 0, b0 + q);
            const int kept = scour_block(d, pos, pos + old);
            if (d.status) return kept_all;
            wsync<T>();
            if (lane() == 0) lvl(d, 0)[b0 + q] = (uint8_t)kept;
            wsync<T>();
            pos += kept;
            kept_all += kept;
        }
        return kept_all;
    }
    const bool unlink = in && !pend && removed && a.z <= d.min_seq;
    const bool surv = in && !unlink && !join;
    if (T::kLog) {   // scourNode's UNLINK / APPEND events :1343-1373
        d.m_unlink += __popcll(ballot(unlink));
        d.m_append += __popcll(m_join);
    }
    const u64 m_surv = ballot(surv);
    scour_events(d, a, b, ballot(unlink), m_join, m_surv, s, tot, start);
    const u64 above = (k < 63) ? (m_join >> (k + 1)) : 0ull;
    const u64 m_grp = ballot(surv && (above & 1ull));
    P2_T0(10)
    if (m_grp) {
        mark_dirty(d, s);
        // group length of each keeper: inclusive lengths up to the group's last member
        const int L = wave_scan_incl(in ? a.x : 0);
        const int gend = k + __ffsll((long long)~above) - 1;   // last member (above has a 0)
        const int Lend = __shfl(L, gend < MT_WAVE ? gend : MT_WAVE - 1, MT_WAVE);
        const int glen = Lend - L + (in ? a.x : 0);
        int totc = 0;
        for (u64 g = m_grp; g; g &= g - 1) {
            const int gl = bcast(glen, first_lane(g));
            totc += gl + text_slack(gl);
        }
        if (!text_ensure(d, totc)) return tot;
        gsync_rd();
        // text merges group by group.  A keeper copied to the arena top reserves slack after
        // its text so that later appends land in place (TextSegment.append :70-85 is a
        // string concatenation; this keeps it amortised O(1)).
        for (u64 g = m_grp; g; g &= g - 1) {
            const int kk = first_lane(g);
            const int gk = bcast(glen, kk);
            const int ge = bcast(gend, kk);
            const v4u bk = uni4(d.Bv[s + kk]);   // fresh: text_ensure may have compacted
            const int ak = uni(d.A[s + kk].x);
            const uint32_t kslack = bk.w >> SEGF_SLACK_SHIFT;
            // members kk+1..ge: contiguity of their text after the keeper's
            const bool mem = k > kk && k <= ge;
            const v4u bm = d.Bv[mem ? s + k : s];   // fresh offsets after a possible gc
            const int Lm = L - (in ? a.x : 0);        // exclusive prefix of lengths
            const int Lk = bcast(L, kk) - ak;         // keeper's exclusive prefix
            const int rel = Lm - Lk;                  // member's offset inside the merged text
            const bool contig_lane = !mem || (int)bm.x == (int)bk.x + rel;
            const bool contig = !ballot(!contig_lane);
            const int add = gk - ak;
            const uint32_t lastw = (uint32_t)bcast((int)bm.w, ge);
            // the merged text is newline-free when the keeper's and every member's are
            const uint32_t nonl = (bk.w & SEGF_NONL) && !ballot(mem && !(bm.w & SEGF_NONL)) ? SEGF_NONL : 0u;
            uint32_t newoff = bk.x, newslack = lastw >> SEGF_SLACK_SHIFT;
            if (!contig) {
                int dst;
                bool move_keeper = false;
                if ((uint32_t)add <= kslack) {                       // append into the slack
                    dst = (int)bk.x + ak;
                    newslack = kslack - (uint32_t)add;
                } else if ((int)bk.x + ak == d.text_top) {          // keeper ends at the top
                    dst = d.text_top;
                    newslack = (uint32_t)text_slack(gk);
                    d.text_top += add + (int)newslack;
                } else {                                            // move keeper + appends
                    newoff = (uint32_t)d.text_top;
                    dst = d.text_top + ak;
                    move_keeper = true;
                    newslack = (uint32_t)text_slack(gk);
                    d.text_top += gk + (int)newslack;
                }
                GLB_AS uint16_t *tb = text_base(d, d.text_half);
                // gather: unit t of the merged text (t < gk); units < ak come from the keeper
                const int t0 = move_keeper ? 0 : ak;
                for (int base = t0; base < gk; base += MT_WAVE) {
                    const int t = base + lane();
                    int src = 0;
                    if (t < ak) {
                        src = (int)bk.x + t;
                    } else {
                        // member whose exclusive prefix (relative) is <= t: scan members
                        for (int j = kk + 1; j <= ge; j++) {
                            const int rj = bcast(Lm, j) - Lk;
                            if (t >= rj) src = bcast((int)bm.x, j) + (t - rj);
                        }
                    }
                    uint16_t ch = 0;
                    if (t < gk) ch = tb[src];
                    if (t < gk) tb[(move_keeper ? (int)newoff : dst - ak) + t] = ch;
                }
            }
            if (lane() == 0) {
                d.A[s + kk].x = gk;
                v4u nb = bk;
                nb.x = newoff;
                nb.w = (lastw & (SEGF_NL_KNOWN | SEGF_NL)) | nonl | (newslack << SEGF_SLACK_SHIFT);
                d.Bv[s + kk] = nb;
            }
            wsync<T>();
        }
    }
    P2_T1(10)
    P2_T0(11)
    const int keep = __popcll(m_surv);
    if (keep < tot) {
        mark_dirty(d, s);
        // compaction: survivors to the front, tail moved left
        v4i sa;
        u64 so;
        PendQ sp = pq_zero();
        v4u sb;
        uint16_t soc = 0;   // ordinal character: a pack re-scours before re-deriving them
        if (surv) {
            sa = d.A[s + k];
            so = d.O[s + k];
            sb = d.Bv[s + k];
            if constexpr (T::kLive) sp = pq_get(d, s + k);
            if (ordon(d)) soc = d.os[s + k];
        }
        const int dst = s + __popcll(m_surv & ((1ull << k) - 1ull));
        wsync<T>();
        if (surv) {
            d.A[dst] = sa;
            d.O[dst] = so;
            d.Bv[dst] = sb;
            if constexpr (T::kLive) pq_put(d, dst, sp);
            if (ordon(d)) d.os[dst] = soc;
        }
        wsync<T>();
        if (ordon(d)) gsync();
        seg_move_left(d, s + tot, tot - keep);
        d.n -= tot - keep;
    }
    P2_T1(11)
    // survivors per block
    {
        int st = 0;
        for (int q = 0; q < nbk; q++) {
            const int c = cntr(d, 0, b0 + q);
            const u64 bm = c ? (((c >= 64) ? ~0ull : ((1ull << c) - 1ull)) << st) : 0ull;
            if (lane() == 0) lvl(d, 0)[b0 + q] = (uint8_t)__popcll(m_surv & bm);
            st += c;
        }
        wsync<T>();
    }
    return keep;
}

// pack :1401-1453 starting from the underflowing block b of level l
#ifdef MT_PROF
TD void pack_impl(DocT<T> &d, int l, int b);
TD void pack(DocT<T> &d, int l, int b) {
    PROF_WRAP_BEGIN
    pack_impl(d, l, b);
    PROF_WRAP_END(3)
    
}
TD void pack_impl(DocT<T> &d, int l, int b) {
#else
TD void pack(DocT<T> &d, int l, int b) {
#endif
    while (true) {
        int c0;
        const int P = blk_find(d, l + 1, b, true, c0);
        if (P < 0) {
            FAIL_INTERNAL(d);
            return;
        }
        const int nch = cntr(d, l + 1, P);
        int total = 0;
        if (l == 0) {
            total = scour_range(d, blk_prefix(d, 0, c0), c0, nch);
            if (d.status) return;
        } else {
            for (int cb = c0; cb < c0 + nch; cb++) total += cntr(d, l, cb);
        }
        int k = total / MT_HALF;
        if (k > MT_MAXN - 1) k = MT_MAXN - 1;
        if (k < 1) k = 1;
        const int base = total / k, extra = total % k;
        blk_replace(d, l, c0, nch, k, base, extra);
        if (d.status) return;
        if (lane() == 0) lvl(d, l + 1)[P] = (uint8_t)k;
        wsync<T>();
        if (k < MT_HALF && l + 2 < d.depth) {
            l = l + 1;
            b = P;
            continue;
        }
        if (ordon(d)) ord_canon(d, l + 1, P);   // nodeUpdateOrdinals(parent) :1449-1450
        return;
    }
}

// pack :1401-1453 above the leaf level only (no scour): the paged upper instance.  top_l /
// top_b: the block whose subtree nodeUpdateOrdinals re-derives at the end (:1449-1450).
TD void pack_counts(DocT<T> &d, int l, int b, int &top_l, int &top_b) {
    while (true) {
        int c0;
        const int P = blk_find(d, l + 1, b, true, c0);
        if (P < 0) {
            FAIL_INTERNAL(d);
            return;
        }
        const int nch = cntr(d, l + 1, P);
        int total = 0;
        for (int cb = c0; cb < c0 + nch; cb++) total += cntr(d, l, cb);
        int k = total / MT_HALF;
        if (k > MT_MAXN - 1) k = MT_MAXN - 1;
        if (k < 1) k = 1;
        blk_replace(d, l, c0, nch, k, total / k, total % k);
        if (d.status) return;
        if (lane() == 0) lvl(d, l + 1)[P] = (uint8_t)k;
        wsync<T>();
        if (k < MT_HALF && l + 2 < d.depth) {
            l = l + 1;
            b = P;
            continue;
        }
        top_l = l + 1;
        top_b = P;
        return;
    }
}

// zamboniSegments :1455-1511
#ifdef MT_PROF
TD void zamboni_impl(DocT<T> &d);
TD void zamboni(DocT<T> &d) {
    PROF_WRAP_BEGIN
    zamboni_impl(d);
    PROF_WRAP_END(4)
    
}
TD void zamboni_impl(DocT<T> &d) {
#else
TD void zamboni(DocT<T> &d) {
#endif
    for (int it = 0; it < MT_ZAMBONI && d.status == 0; it++) {
        if (d.heap_n == 0) break;
        const v2i top = heap_top(d);
        if (top.x > d.min_seq) break;
        heap_pop(d);
        wsync<T>();
        P2_T0(12)
        const int i = find_uid(d, (uint32_t)top.y);
        if (i < 0) continue;
        int bstart;
        const int b = blk_find(d, 0, i, true, bstart);
        P2_T1(12)
        if (b < 0) {
            FAIL_INTERNAL(d);
            return;
        }
        const int f = flgr(d, b);
        const int old = cntr(d, 0, b);
        if (f == 0) continue;
        const int kept = scour_range(d, bstart, b, 1);
        if (d.status) return;
        wsync<T>();
        if (lane() == 0) d.flg[b] = 0;
        wsync<T>();
        if (kept < old && kept < MT_HALF && d.depth > 1)
            pack(d, 0, b);
        else if (kept < old && ordon(d))
            ord_canon(d, 0, b);   // nodeUpdateOrdinals(block) :1500-1501
    }
}

// ------------------------------------------------------------------ ops
// LDS tier: is there room for one more message of this kind without overflowing the LDS
// capacities mid-message?  Bounds: an op adds <= 3 segments (2 boundary splits + 1
// insert), each of which may split one block per level; every pack (<= 2 zamboni scours
// per call, <= 2 calls per message) can grow a level by <= 6 blocks; an insert adds <= 1
// heap entry, a range op <= one per leaf block.  A message that fails this check is handed
// to the HBM tier *before* it is applied (the LDS state is spilled first), so the LDS tier
// never has to roll back.
TD bool lds_room(DocT<T> &d, const mt_op_rec &op) {
    if (d.n + 3 > d.S_cap) return false;
    if (d.depth + 2 > MT_LV) return false;
    const int nb0 = nbr(d, 0);
    int need_heap = op.kind == MT_OP_INSERT ? 1 : nb0 + 3;
    if (d.heap_n + need_heap > d.H_cap) return false;
    bool ok = true;
    for (int l = 0; l < d.depth; l++) ok = ok && nbr(d, l) + 3 + 24 <= bcap(d, l);
    // an overlapping remove that would need a slot above the LDS tier's u32 masks
    if (op.kind == MT_OP_REMOVE && oslot_short(d, op_cli(op))) ok = false;
    return ok;
}

// Live documents on the flat HBM tier (TierLiveT with TierCaps.grow): can this message be
// applied within the handle's capacities?  0: yes; else the capacity the growth step must raise
// (1 segments, 2 blocks, 3 heap, 4 text, 5 property records, 12 segment groups) -- checked,
// with the text / property arenas compacted first, before the message, so that a message never
// fails half applied (segmentGroups and the pending queue are unbounded in the reference,
// MT/mergeTree.ts:1955-1962, MT/segmentGroupCollection.ts).  The bounds are lds_room's for the
// tree (a message adds <= 2 segments); an insert's text plus the slack a zamboni merge may copy
// (1/8 of the arena, >= 4096 units); a range op's records (one per segment it reaches: <= its
// span, <= the segments) plus an insert's one; one group for a local op.
TD int live_room(DocT<T> &d, const mt_op_rec &op) {
    if (d.n + 3 > d.S_cap) return 1;
    for (int l = 0; l < d.depth; l++)
        if (nbr(d, l) + 3 + 24 > bcap(d, l)) return 2;
    const int nb0 = nbr(d, 0);
    if (d.heap_n + (op.kind == MT_OP_INSERT ? 1 : nb0 + 3) > d.H_cap) return 3;
    const int nt = op.kind == MT_OP_INSERT && !(op.flags & MT_F_MARKER) ? max(op.pos2, 0) : 0;
    const int tslack = max(d.T_cap / 8, 4096);
    if (d.text_top + nt + tslack > d.T_cap) {
        text_gc(d);
        if (d.text_top + nt + tslack > d.T_cap) return 4;
    }
    const int span = op.kind == MT_OP_ANNOTATE ? min(max(op.pos2 - op.pos1, 0), d.n) + 2 : 0;
    const int np = span + (op.props != MT_NO_PROPS ? 1 : 0) + MT_WAVE;
    if (d.props_top + np > d.P_cap) {
        props_gc(d);
        if (d.props_top + np > d.P_cap) return 5;
    }
    if ((op.flags & MT_F_LOCAL) && d.g_n + 1 > d.LG) return 12;
    return 0;
}

// One sequenced message as the engine consumes it: the record plus (prefetched) the first
// 8 UTF-16 units of an insert's payload and whether the payload ends with '\n'.
struct OpIn {
    mt_op_rec op;
    u64 pay_lo, pay_hi;   // units 0..3 / 4..7 when pay_ok
    bool pay_ok;
    bool nl;
    bool pay_lane = false;   // pay_ok, with lane j's unit in pay_v (a load issued with the message)
    uint32_t pay_v = 0;
};

__device__ __forceinline__ uint16_t pay_unit(const OpIn &in, int j) {
    const u64 w = j < 4 ? (in.pay_lo >> (16 * j)) : (in.pay_hi >> (16 * (j - 4)));
    return (uint16_t)(w & 0xFFFF);
}

// Live documents: first segment at or after index `from` visible in view
// (UniversalSequenceNumber, local client) -- the leaf rightExcursion's nodeMap reaches first
// (MT/mergeTree.ts:2346-2376, nodeMap :2936-2998 visits leaves of length > 0).  The local
// client's view of a node is its local net length whatever the refSeq (nodeLength
// :1692-1698): a segment not removed at all.  -1: none.
TD int first_v0(DocT<T> &d, int from) {
    for (int base = from; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        const bool v = i < d.n;
        v4i a;
        u64 o;
        load_ao(d, i, v, a, o);
        const u64 m = ballot(v && obs_len(a) > 0);
        if (m) return base + first_lane(m);
    }
    return -1;
}

// Client.applyInsertOp MT/client.ts:394-442 -> MergeTree.insertSegments :2001-2031
#ifdef MT_PROF
TD void op_insert_impl(DocT<T> &d, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin);
TD void op_insert(DocT<T> &d, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin) {
    PROF_WRAP_BEGIN
    op_insert_impl(d, in, tin, pin);
    PROF_WRAP_END(6)
    
}
TD void op_insert_impl(DocT<T> &d, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin) {
#else
TD void op_insert(DocT<T> &d, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin) {
#endif
    const mt_op_rec &op = in.op;
    const int r = op.ref_seq, c = op_cli(op), seq = op.seq, p = op.pos1;
    const bool quiet = (op.flags & MT_F_LOAD) != 0;   // SnapshotLoader.loadBody append
    const bool marker = (op.flags & MT_F_MARKER) != 0;
    const int slen = marker ? 1 : op.pos2;
    // arena room first (a compaction changes no structure, so doing it before the boundary
    // split is equivalent; a paged window must not be flushed with a page split pending)
    if (slen > 0 && !marker && !text_ensure(d, slen)) return;
    if (slen > 0 && op.props != MT_NO_PROPS && !props_ensure(d, 1)) return;
    // pass: split point, first index with prefix >= p, first tie-able index at prefix == p
    P2_T0(13)
    int carry = 0, split_i = -1, split_q = 0, ip = -1, js = -1;
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        const bool v = i < d.n;
        v4i a;
        u64 o;
        load_ao(d, i, v, a, o);
        const int vl = v ? vlen(d, a, o, r, c) : 0;
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
        bool tj;
        if constexpr (T::kLive)
            tj = d.lop ? tie_local(a, r) : tie_remote_live(a, r);
        else
            tj = tie(a, r);
        const u64 mj = ballot(v && pex == p && (vl > 0 || tj));
        if (mj) {
            js = base + first_lane(mj);
            break;
        }
        carry += bcast(inc, MT_WAVE - 1);
        if (ballot(v && pex > p)) break;
    }
    P2_T1(13)
    if (split_i >= 0) {
        split_seg(d, split_i, split_q);
        if (d.status) return;
        ip = js = split_i + 1;
    } else if (ip < 0 && carry == p) {
        ip = d.n;
    }
    Cb cb;
    if (!quiet) cb = cb_begin(d, (T::kLive && d.lop) ? -1 : seq, MT_OP_INSERT);
    if (slen == 0) {  // zero-length segment: boundary only, not inserted (:2229)
        if (quiet) return;
        cb.n = 1;
        cb_log(d, -1);
        cb_log(d, 0);
        if constexpr (T::kLog) {   // rich: the (never linked) empty segment, props nulls dropped
            if (d.rich && cb_room(d, 2 + (op.props != MT_NO_PROPS ? 2 * (int)(pin[op.props] & 0xFFFF) : 0))) {
                int np = -1;
                if (op.props != MT_NO_PROPS) {
                    const GLB_AS uint32_t *rec = pin + op.props;
                    np = 0;
                    for (uint32_t j = 0; j < (rec[0] & 0xFFFF); j++) {
                        if (rec[2 + 2 * j] == MT_VAL_NULL) continue;
                        if (lane() == 0) {
                            d.dlog[d.dlog_n + 2 + 2 * np] = (int32_t)rec[1 + 2 * j];
                            d.dlog[d.dlog_n + 3 + 2 * np] = (int32_t)rec[2 + 2 * j];
                        }
                        np++;
                    }
                }
                if (lane() == 0) {
                    d.dlog[d.dlog_n] = (np >= 0 ? 2 : 0) | (ordon(d) ? 4 : 0);
                    d.dlog[d.dlog_n + 1] = np;
                }
                d.dlog_n += 2 + 2 * max(np, 0);
                // never linked: no ordinal, getPosition walks no parent (0)
                cb_log_ext(d, 0u, 0, -1, false);
            }
        }
        cb.h = fnv_u64(cb.h, fnv_u32(fnv_u32(MT_FNV_OFF, (uint32_t)-1), 0u));
        cb_end(d, cb);
        // zamboni runs in apply_op (single inlined site)
        return;
    }
    if (ip < 0) {
        fail(d, MT_DOC_INSERT_FAILED);  // :2243-2249
        return;
    }
    if (d.n + 1 > d.S_cap) {
        fail_cap(d, 1);
        return;
    }
    uint32_t ph = 0, nomatch = 0;
    if (op.props != MT_NO_PROPS) {
        ph = (uint32_t)d.props_top;
        d.props_top++;
        const GLB_AS uint32_t *rec = pin + op.props;
        const uint32_t cntk = rec[0] & 0xFFFF;
        int cn = 0;
        for (uint32_t j = 0; j < cntk; j++) cn += rec[2 + 2 * j] != MT_VAL_NULL;
        if (cn > MT_KMAX) {
            fail(d, MT_DOC_CAPACITY);
            return;
        }
        if (lane() == 0) {
            GLB_AS uint32_t *t = prec(d, d.props_half, ph);
            uint32_t n = 0;
            for (uint32_t j = 0; j < cntk; j++) {
                if (rec[2 + 2 * j] == MT_VAL_NULL) continue;  // null dropped (Q5)
                t[1 + 2 * n] = rec[1 + 2 * j];
                t[2 + 2 * n] = rec[2 + 2 * j];
                n++;
            }
            t[0] = n;
        }
#ifndef MT_NO_Q4
        bool nm = false;
        for (uint32_t j = 0; j < cntk; j++) {
            const uint32_t v = rec[2 + 2 * j];
            nm = nm || (v != MT_VAL_NULL && (v & MT_VAL_NOMATCH_BIT));
        }
        if (nm) nomatch = SEGF_NOMATCH;
#endif
    }
    int bstart;
    int B = blk_find(d, 0, ip, false, bstart);
    if (B < 0) {
        FAIL_INTERNAL(d);
        return;
    }
    int bend = bstart + cntr(d, 0, B);
    int x = (js >= 0 && js < bend) ? js : bend;
    if constexpr (T::kLive) {
        // A remote insert that reaches the end of leaf block B continues into the next block
        // when the first segment after B visible in view (UniversalSequenceNumber, local
        // client) is an unacked local insert (insertingWalk's continuePredicate,
        // MT/mergeTree.ts:2464-2469 with blockInsert's checkSegmentIsLocal :2176-2194; the
        // unfinished node makes the parent walk on with pos 0, :2419-2424).
        while (!d.lop && x == bend) {
            const int s0 = first_v0(d, bend);
            if (s0 < 0 || !is_local_seq(uni(d.A[s0].y)) || B + 1 >= nbr(d, 0)) break;
            B++;
            bstart = bend;
            bend += cntr(d, 0, B);
            x = (js >= 0 && js < bend) ? js : bend;
        }
    }
    uint32_t toff, segw = 0;
    if (marker) {
        toff = op.payload;
    } else {
        toff = (uint32_t)d.text_top;
        GLB_AS uint16_t *dst = text_base(d, d.text_half) + d.text_top;
        // the payload (<= 8 units prefetched with the record, else read from the batch); its last
        // unit decides TextSegment.canAppend's trailing-'\n' rule
        bool anynl = false, lastnl = false;
        if (in.pay_ok) {
            const uint16_t u = lane() < slen ? (in.pay_lane ? (uint16_t)in.pay_v : pay_unit(in, lane())) : (uint16_t)0;
            if (lane() < slen) dst[lane()] = u;
            anynl = ballot(lane() < slen && u == (uint16_t)'\n') != 0ull;
            lastnl = ballot(lane() == slen - 1 && u == (uint16_t)'\n') != 0ull;
        } else {
            for (int j = lane(); j < slen; j += MT_WAVE) {
                const uint16_t u = tin[op.payload + j];
                dst[j] = u;
                anynl = anynl || u == (uint16_t)'\n';
                lastnl = lastnl || (j == slen - 1 && u == (uint16_t)'\n');
            }
            anynl = ballot(anynl) != 0ull;
            lastnl = ballot(lastnl) != 0ull;
        }
#ifdef MT_NO_NONL
        anynl = true;
#endif
        d.text_top += slen;
        segw = SEGF_NL_KNOWN | (lastnl ? SEGF_NL : 0u) | (anynl ? 0u : SEGF_NONL);
    }
    P2_T0(15)
    seg_move_right(d, x, 1);
    P2_T1(15)
    mark_dirty(d, x);
    const uint32_t uid = (uint32_t)d.next_uid;
    if (lane() == 0) {
        d.A[x] = v4i{slen, seq, MT_RSEQ_NONE, pack_cli(c, 0)};
        d.O[x] = 0ull;
        if constexpr (T::kLive) {   // addToPendingList :2128
            PendQ q = pq_zero();
            q.w[0] = d.lop ? (u64)(uint32_t)d.lg : 0ull;
            pq_put(d, x, q);
        }
        d.Bv[x] = v4u{toff, ph, uid | (marker ? MT_MARKER_BIT : 0u), segw | nomatch};
    }
    d.next_uid++;
    d.n++;
    const int nc = cntr(d, 0, B) + 1;
    if (ordon(d)) {
        const int w = ord_w(nc);
        if (x < bend) {
            // insert before a segment (blockInsert's onLeaf, :2218-2225): the new segment
            // replaces it in the block with its ordinal (replaceCurrent, :2437-2441), and it is
            // linked after the new one (setOrdinal :2486)
            const int oc = uni((int)d.os[x + 1]);
            if (lane() == 0) {
                d.os[x] = (uint16_t)oc;
                d.os[x + 1] = (uint16_t)(oc + w);
            }
            gsync();
        } else {   // at the block end
            ord_put(d.os + x, x > bstart ? uni((int)d.os[x - 1]) + w : w - 1);
        }
    }
    wsync<T>();
    if (lane() == 0) lvl(d, 0)[B] = (uint8_t)nc;
    wsync<T>();
    int lb = B;
    if (nc == MT_MAXN) {
        blk_split_up(d, 0, B);
        if (d.status) return;
        if (x - bstart >= MT_HALF) lb = B + 1;
    }
    if (!(T::kLive && d.lop) && seq > d.min_seq) add_to_lru_block(d, lb, uid, seq);  // saveIfLocal :2197-2212
    if (d.status) return;
    if (quiet) return;   // insertSegments with opArgs undefined fires no callback (:2013-2021)
    // delta callback: position of the new segment in the observer view
    const int pos = (T::kPaged ? d.obs_base : 0) + obs_prefix(d, x);
    cb.n = 1;
    cb_log(d, pos);
    cb_log(d, slen);
    if constexpr (T::kLog) {
        if (d.rich) {
            wsync<T>();
            cb_log_seg(d, uni4(d.A[x]), uni4(d.Bv[x]));
            if (T::kPaged && ordon(d)) {   // after the page split (pg_op_insert)
                d.dfr_rec = d.dlog_rec;
                d.dfr_uid = (int)uid;
                d.dfr_pos = pos;
            } else {
                cb_log_ext(d, uid, pos, x, false);
            }
        }
    }
    cb.h = fnv_u64(cb.h, fnv_u32(fnv_u32(MT_FNV_OFF, (uint32_t)pos), (uint32_t)slen));
    cb_end(d, cb);
    // zamboni runs in apply_op (single inlined site)
}

// SegmentPropertiesManager.addProperties MT/segmentPropertiesManager.ts:35-111 applied by
// one lane to its segment: writes the new record nh, returns the seg hash contribution of
// the propertyDeltas (and logs them when `logp` is set).  Returns false on key overflow.
// Live documents: the pending-property state of a segment (SegmentPropertiesManager
// pendingKeyUpdateCount / pendingRewriteCount, MT/segmentPropertiesManager.ts:13-14, 19-33)
// is the set of unacked local annotate groups in its segment-group FIFO (word pw).
TD bool grp_pending_rewrite(DocT<T> &d, const PendQ &pw) {
    for (int q = 0; q < MT_PQ_IDS; q++) {
        const int id = pq_at(pw, q);
        if (id == 0) break;
        const int w1 = d.grp[id * MT_GRP_WORDS + 1];
        if ((w1 & 0xFF) == MT_OP_ANNOTATE && ((w1 >> 8) & 0xFF)) return true;
    }
    return false;
}
TD bool grp_pending_key(DocT<T> &d, const PendQ &pw, uint32_t k) {
    for (int q = 0; q < MT_PQ_IDS; q++) {
        const int id = pq_at(pw, q);
        if (id == 0) break;
        const GLB_AS int32_t *g = d.grp + id * MT_GRP_WORDS;
        if ((g[1] & 0xFF) != MT_OP_ANNOTATE) continue;
        const int nk = (g[1] >> 16) & 0xFF;
        for (int j = 0; j < nk; j++)
            if ((uint32_t)g[2 + j] == k) return true;
    }
    return false;
}

// pw (live documents, remote ops): the segment's pending-group FIFO -- keys with a pending
// local update are not modified (shouldModifyKey :56-63), an outstanding local rewrite blocks
// the whole op (:48-51: *undef = true, propertyDeltas undefined, the set unchanged).
TD bool annotate_record(DocT<T> &d, uint32_t oh, uint32_t nh, const GLB_AS uint32_t *rec, u64 &sh,
                        GLB_AS int32_t *logp, int &nlog, bool *nomatch = nullptr, PendQ pw = pq_zero(),
                        bool *undef = nullptr) {
    const uint32_t cntk = rec[0] & 0xFFFF, comb = rec[0] >> 16;
    const GLB_AS uint32_t *o = oh ? prec(d, d.props_half, oh) : nullptr;
    GLB_AS uint32_t *t = prec(d, d.props_half, nh);
    const uint32_t on = o ? o[0] : 0;
    uint32_t n = 0;
    int npd = 0;
    if constexpr (T::kLive) {
        if (pq_any(pw) && grp_pending_rewrite(d, pw)) {
            for (uint32_t i = 0; i < 2 * on; i++) t[1 + i] = o[1 + i];
            t[0] = on;
            sh = fnv_u32(sh, 0xFFFFFFFFu);
            if (undef) *undef = true;
            return true;
        }
        if (comb == MT_COMBINE_TABLE) pw = pq_zero();   // a combining op modifies every key
    }
    // rewrite: delete keys whose new value is not truthy (:66-79)
    for (uint32_t i = 0; i < on; i++) {
        const uint32_t k = o[1 + 2 * i], v = o[2 + 2 * i];
        bool in_new = false, truthy = false;
        if constexpr (T::kLive) {
            if (pq_any(pw) && grp_pending_key(d, pw, k)) {   // kept: a pending local update
                t[1 + 2 * n] = k;
                t[2 + 2 * n] = v;
                n++;
                continue;
            }
        }
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
        if constexpr (T::kLive) {
            if (pq_any(pw) && grp_pending_key(d, pw, k)) continue;
        }
        int idx = -1;
        for (uint32_t q = 0; q < n; q++)
            if (t[1 + 2 * q] == k) idx = (int)q;
        bool deleted_by_rewrite = false;
        if (comb == MT_COMBINE_REWRITE && idx < 0) {
            for (uint32_t i = 0; i < on; i++)
                if (o[1 + 2 * i] == k) deleted_by_rewrite = true;
        }
        // a key set to undefined reads as absent: deltas[key] = previousValue ?? null
        const bool absent = idx < 0 || t[2 + 2 * idx] == MT_VAL_UNDEF;
        if (!deleted_by_rewrite) {
            const uint32_t dv = absent ? MT_VAL_NULL : t[2 + 2 * idx];
            sh = fnv_u32(fnv_u32(sh, k), dv);
            if (logp) {
                logp[nlog++] = (int32_t)k;
                logp[nlog++] = (int32_t)dv;
            }
            npd++;
        }
        uint32_t nv = v;
#ifndef MT_NO_Q4
        if (comb == MT_COMBINE_TABLE) {
            // newValue = combine(op, previousValue, undefined, seq) (:93-99): the
            // host tabulated it for every value that can be present
            const GLB_AS uint32_t *tab = rec + 1 + 2 * cntk;
            nv = tab[1];
            if (!absent) {
                const uint32_t old = t[2 + 2 * idx];
                bool hit = false;
                for (uint32_t q = 0; q < tab[0]; q++)
                    if (tab[2 + 2 * q] == old) {
                        nv = tab[3 + 2 * q];
                        hit = true;
                    }
                if (!hit) return false;
            }
        }
#endif
        if (nv == MT_VAL_NULL) {
            if (idx >= 0) {
                for (uint32_t q = (uint32_t)idx + 1; q < n; q++) {
                    t[2 * q - 1] = t[2 * q + 1];
                    t[2 * q] = t[2 * q + 2];
                }
                n--;
            }
        } else if (idx >= 0) {
            t[2 + 2 * idx] = nv;
        } else {
            if (n >= MT_KMAX) return false;
            t[1 + 2 * n] = k;
            t[2 + 2 * n] = nv;
            n++;
        }
    }
    t[0] = n;
    sh = fnv_u32(sh, (uint32_t)npd);
    // *nomatch in: the new set can hold a NaN / undefined value at all; out: it does
    if (nomatch && *nomatch) {
        bool nm = false;
        for (uint32_t q = 0; q < n; q++) nm = nm || (t[2 + 2 * q] & MT_VAL_NOMATCH_BIT) != 0;
        *nomatch = nm;
    }
    return true;
}

// The marking pass of markRangeRemoved :2640-2752 / annotateRange :2598-2638 over the
// segments of d (after the boundary splits).  carry / ocarry: view / observer position of
// d's first segment (advanced past it); the callback record cb accumulates across calls.
// Returns true when the range ended inside d (or on failure: check d.status).
TD bool range_mark(DocT<T> &d, const mt_op_rec &op, const GLB_AS uint32_t *rec, int &carry, int &ocarry,
                   Cb &cb) {
    const int r = op.ref_seq, c = op_cli(op), seq = op.seq, p1 = op.pos1, p2 = op.pos2;
    const bool rem = op.kind == MT_OP_REMOVE;
    compute_ends(d);
    if (!rem) gsync_rd();   // property records written earlier in this launch are read below
    int last_b = -1;
    const int L = lane();
    const int nblk = nbr(d, 0);
    // can this op leave a NaN / undefined value in a set?
    bool rec_nm = false;
#ifndef MT_NO_Q4
    if (!rem) {
        rec_nm = (rec[0] >> 16) == MT_COMBINE_TABLE;
        for (uint32_t j = 0; j < (rec[0] & 0xFFFFu); j++) {
            const uint32_t v = rec[2 + 2 * j];
            rec_nm = rec_nm || (v != MT_VAL_NULL && (v & MT_VAL_NOMATCH_BIT));
        }
    }
#endif
    for (int base = 0; base < d.n; base += MT_WAVE) {
        if (!rem && !props_ensure(d, MT_WAVE)) return true;
        const int i = base + L;
        const bool v = i < d.n;
        v4i a;
        u64 o;
        load_ao(d, i, v, a, o);
        const v4u bv = d.Bv[v ? i : 0];
        const int vl = v ? vlen(d, a, o, r, c) : 0;
        const int inc = wave_scan_incl(vl);
        const int pex = carry + inc - vl, pin_ = carry + inc;
        const bool sel = v && vl > 0 && pex < p2 && pin_ > p1;
        const u64 sel_m = ballot(sel);
        if (sel_m) mark_dirty(d, base + first_lane(sel_m));
        bool newly = false, bad = false, spill = false, want_ovf = false;
        // live documents: a remote remove of a segment the local client removed (unacked)
        // replaces that removal (:2657-2662): no overlap slot, no callback entry
        bool lrem = false;
        if constexpr (T::kLive) lrem = rem && sel && !d.lop && is_local_seq(a.z);
        const bool ovl_any = rem && ballot(sel && a.z != MT_RSEQ_NONE && !lrem);
        if (ovl_any) {   // this client's slot (taken at its first overlapping remove)
            if (d.ocs == 0) d.ocs = oslot_take(d, c);
            if (d.ocs > 32) d.wide = 1;
            if (d.ocs && lane() == 0) d.oslot[2 * (d.ocs - 1) + 1] = seq;
        }
        if (rem && sel) {
            if (lrem) {
                a.z = seq;
                a.w = pack_cli(seg_cli(a), c);
                d.A[i] = a;
            } else if (a.z != MT_RSEQ_NONE) {          // addOverlappingClient :2577-2585
                bool ovf = false;
                if constexpr (T::kPaged && T::kOvf) ovf = d.ocs == 0 || (o & MT_OVF_BIT);
                if (ovf) {
                    want_ovf = true;   // (ovf_mark below)
                } else if (d.ocs == 0) {
                    if (T::kOvlBits < 64)
                        spill = true;
                    else
                        bad = true;
                } else {
                    d.O[i] = (typename T::O_v)(o | (1ull << (d.ocs - 1)));
                }
            } else {
                newly = true;
                a.z = seq;
                a.w = pack_cli(seg_cli(a), c);
                d.A[i] = a;
                if constexpr (T::kLive) {   // the local client's remove: addToPendingList :2683-2684
                    if (d.lop) {
                        PendQ pq = pq_get(d, i);
                        if (pq_push(pq, d.lg))
                            pq_put(d, i, pq);
                        else
                            bad = true;
                    }
                }
            }
        }
        if constexpr (T::kPaged && T::kOvf) {   // overflow sets: the whole list, in the arena
            // (want_ovf: decided on the segment's removal state before this message marked it)
            if (ballot(want_ovf) && !ovf_mark(d, want_ovf, i, o, c, seq)) bad = true;
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
            bool nm = rec_nm || (bv.w & SEGF_NOMATCH) != 0;
            PendQ pw = pq_zero();
            if constexpr (T::kLive) {
                PendQ pq = pq_get(d, i);
                if (d.lop) {   // the local client's annotate: addToPendingList :2611-2612
                    if (pq_push(pq, d.lg))
                        pq_put(d, i, pq);
                    else
                        bad = true;
                } else {
                    pw = pq;
                }
            }
            if (!annotate_record(d, bv.y, nh, rec, sh, (GLB_AS int32_t *)nullptr, unused, &nm, pw)) bad = true;
            v4u nb = bv;
            nb.y = nh;
            nb.w = (bv.w & ~SEGF_NOMATCH) | (nm ? SEGF_NOMATCH : 0u);
            d.Bv[i] = nb;
        }
        if (ballot(bad)) {
            // diagnostic 11: more than 63 clients' overlapping removes unsettled at once (or a
            // full overflow arena)
            if (ovl_any && d.ocs == 0 && d.status == 0) d.cap_cause = 11;
            fail(d, MT_DOC_CAPACITY);
            return true;
        }
        if (ballot(spill)) {   // (the generator's LDS tier: the document restarts in HBM)
            fail_cap(d, 1);
            return true;
        }
        if (!rem) d.props_top += __popcll(sel_m);
        wsync<T>();
        // fold the callback records in document order
        u64 em = ballot(entry);
        while (em) {
            const int j = first_lane(em);
            em &= em - 1;
            cb.h = fnv_u64(cb.h, bcast64(sh, j));
            cb.n++;
            if (T::kLog && d.dlog) {
                cb_log(d, bcast(opos, j));
                cb_log(d, bcast(a.x, j));
                if (!rem) {
                    // re-derive this segment's propertyDeltas into the log (debug only)
                    const uint32_t ohj = (uint32_t)bcast((int)bv.y, j), nhj = (uint32_t)bcast((int)nh, j);
                    int nl = 0;
                    u64 dummy = 0;
                    gsync_rd();
                    // propertyDeltas: <= one per old key (rewrite) plus one per op key
                    if (cb_room(d, 1 + 2 * (MT_KMAX + (int)(rec[0] & 0xFFFF)))) {
                        const int at = d.dlog_n + 1;
                        PendQ pwj = pq_zero();
                        if constexpr (T::kLive) {
                            if (!d.lop) pwj = pq_bcast(pq_get(d, v ? i : 0), j);
                        }
                        if (L == 0) {
                            // old record is untouched (new record went to a fresh handle)
                            bool undef = false;
                            annotate_record(d, ohj, nhj, rec, dummy, d.dlog + at, nl, nullptr, pwj, &undef);
                            d.dlog[at - 1] = undef ? -1 : nl / 2;   // -1: propertyDeltas undefined
                        }
                        nl = bcast(nl, 0);
                        d.dlog_n += 1 + nl;
                    }
                }
                if (d.rich) {   // the segment after the op (annotate: its new property set)
                    const v4i aj = v4i{bcast(a.x, j), bcast(a.y, j), bcast(a.z, j), bcast(a.w, j)};
                    v4u bj = v4u{(uint32_t)bcast((int)bv.x, j), (uint32_t)bcast((int)bv.y, j),
                                 (uint32_t)bcast((int)bv.z, j), (uint32_t)bcast((int)bv.w, j)};
                    if (!rem) bj.y = (uint32_t)bcast((int)nh, j);
                    cb_log_seg(d, aj, bj);
                    cb_log_ext(d, bj.z & ~MT_MARKER_BIT, bcast(opos, j), base + j, false);
                }
            }
        }
        // addToLRUSet for every visited segment, first one per leaf block (:2680-2689)
        const int b = sel ? block_of(d, i, nblk) : -1;
        const u64 below = sel_m & ((1ull << L) - 1ull);
        const int prevl = below ? 63 - __clzll((long long)below) : -1;
        const int pb = __shfl(b, prevl < 0 ? 0 : prevl, MT_WAVE);
        const int prev_b = prevl < 0 ? last_b : pb;
        // (the local client's own op: its segments join the pending group instead, :2610-2617, 2680-2689)
        u64 fm = ballot(sel && b != prev_b && !(T::kLive && d.lop));
        while (fm) {
            const int j = first_lane(fm);
            fm &= fm - 1;
            add_to_lru_block(d, bcast(b, j), (uint32_t)bcast((int)(bv.z & ~MT_MARKER_BIT), j), seq);
        }
        if (d.status) return true;
        if (sel_m) last_b = bcast(b, 63 - __clzll((long long)sel_m));
        carry += bcast(inc, MT_WAVE - 1);
        ocarry += bcast(oinc, MT_WAVE - 1);
        if (ballot(v && pex >= p2)) return true;
    }
    return false;
}


// markRangeRemoved :2640-2752 / annotateRange :2598-2638.  After the two boundary splits
// the visited leaves are exactly those with view length > 0 inside [p1, p2) (nodeMap
// :2936-2998 is tree-shape independent), processed in document order.
#ifdef MT_PROF
TD void op_range_impl(DocT<T> &d, const mt_op_rec &op, const GLB_AS uint32_t *pin);
TD void op_range(DocT<T> &d, const mt_op_rec &op, const GLB_AS uint32_t *pin) {
    PROF_WRAP_BEGIN
    op_range_impl(d, op, pin);
    PROF_WRAP_END(7)
    
}
TD void op_range_impl(DocT<T> &d, const mt_op_rec &op, const GLB_AS uint32_t *pin) {
#else
TD void op_range(DocT<T> &d, const mt_op_rec &op, const GLB_AS uint32_t *pin) {
#endif
    const int r = op.ref_seq, c = op_cli(op), seq = op.seq, p1 = op.pos1, p2 = op.pos2;
    const bool rem = op.kind == MT_OP_REMOVE;
    const GLB_AS uint32_t *rec = (!rem && op.props != MT_NO_PROPS) ? pin + op.props : nullptr;
    if (rec && (rec[0] >> 16) == MT_COMBINE_OTHER) {
        fail(d, MT_DOC_UNSUPPORTED);
        return;
    }
    if (!rec) rec = (const GLB_AS uint32_t *)&kEmptyPropsRec;
    boundary(d, p1, r, c);
    if (d.status) return;
    boundary(d, p2, r, c);
    if (d.status) return;
    Cb cb = cb_begin(d, (T::kLive && d.lop) ? -1 : seq, op.kind);
    int carry = 0, ocarry = 0;
    P2_T0(14)
    range_mark(d, op, rec, carry, ocarry, cb);
    P2_T1(14)
    if (d.status) return;
    cb_end(d, cb);
    // zamboni runs in apply_op (single inlined site)
}

// Client.applyMsg MT/client.ts:797-819 for one encoded record: the op (insertSegments /
// markRangeRemoved / annotateRange each end with zamboniSegments), completeAndLogOp's
// asserts (:451-479), then updateSeqNumbers -> setMinSeq (:821-828, 991-1004,
// MT/mergeTree.ts:1751-1769) whose zamboni runs when minSeq advances.  Both zamboni passes
// share one call site so the (large) zamboni/scour/pack code is inlined once.
// Summary load: the removal info of the body segment the preceding MT_F_LOAD insert
// appended (specToSegment sets removedSeq/removedClientId before insertion,
// MT/snapshotLoader.ts:102-107; the segment's own insertion walk never reads them).
TD void load_removed(DocT<T> &d, const mt_op_rec &op) {
    const int i = find_uid(d, (uint32_t)(d.next_uid - 1));
    if (i < 0) {
        FAIL_INTERNAL(d);
        return;
    }
    mark_dirty(d, i);
    if (lane() == 0) {
        v4i a = d.A[i];
        a.z = op.seq;
        a.w = pack_cli(seg_cli(a), op_cli(op));
        d.A[i] = a;
    }
    wsync<T>();
}

// ---------------------------------------------------------------- live-client documents
// The local client's own op (insertSegmentLocal / removeRangeLocal / annotateRangeLocal,
// MT/client.ts:164-211 -> applyInsertOp / applyRemoveRangeOp / applyAnnotateRangeOp with no
// sequencedMessage): refSeq = currentSeq, seq = UnassignedSequenceNumber with
// ++collabWindow.localSeq (MT/mergeTree.ts:2009, 2604, 2646), one new segment group at the
// tail of the pending queue (addToPendingList :1955-1962); no zamboni, no seq update
// (completeAndLogOp's asserts are for sequenced messages only, MT/client.ts:456-471).
TD void live_local(DocT<T> &d, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin) {
    const mt_op_rec &op = in.op;
    if (op.kind != MT_OP_INSERT && op.kind != MT_OP_REMOVE && op.kind != MT_OP_ANNOTATE) return;
    const GLB_AS uint32_t *rec = (op.kind == MT_OP_ANNOTATE && op.props != MT_NO_PROPS) ? pin + op.props : nullptr;
    const int nk = rec ? (int)(rec[0] & 0xFFFFu) : 0;
    if (d.g_n >= d.LG || nk > MT_KMAX) {
        if (d.status == 0) d.cap_cause = nk > MT_KMAX ? 13 : 12;
        fail(d, MT_DOC_CAPACITY);
        return;
    }
    const int ls = ++d.local_seq;
    const int g = (d.g_head - 1 + d.g_n) % d.LG + 1;
    GLB_AS int32_t *ge = d.grp + g * MT_GRP_WORDS;
    const int rw = rec && (rec[0] >> 16) == MT_COMBINE_REWRITE ? 1 : 0;
    if (lane() == 0) {
        ge[0] = ls;
        ge[1] = (int)op.kind | (rw << 8) | (nk << 16);
    }
    if (lane() < nk) ge[2 + lane()] = (int)rec[1 + 2 * lane()];
    d.g_n++;
    d.lop = 1;
    d.lg = g;
    OpIn lin = in;
    lin.op.seq = MT_LOCAL_BASE + ls;
    lin.op.ref_seq = d.cur_seq;
    if (op.kind == MT_OP_INSERT)
        op_insert(d, lin, tin, pin);
    else
        op_range(d, lin.op, pin);
    // segment ids below this joined the group in the op's walk (document order); a later split
    // appends its right half -- a new id -- to every group of the left one (SegmentGroup
    // segments order, segmentGroupCollection.ts copyTo)
    if (lane() == 0) ge[10] = d.next_uid;
    d.lop = 0;
    d.lg = 0;
}

// ackPendingSegment (MT/client.ts:589-626 -> MT/mergeTree.ts:1926-1953, ISegment.ack
// :486-521) for one member op: the head group's segments get the sequence number (insert:
// seq; remove: removedSeq unless a remote remove replaced it), leave the group and enter
// the zamboni LRU set (addToLRUSet :1306-1316, in document order).
TD void live_ack(DocT<T> &d, const mt_op_rec &op) {
    if (d.g_n == 0) return;   // nothing pending: ackPendingSegment dequeues undefined (:1931)
    const int g = d.g_head;
    const int kind = d.grp[g * MT_GRP_WORDS + 1] & 0xFF;
    if (kind != (int)op.kind) {   // the echo does not match the pending op (ack's assert)
        if (d.status == 0) d.cap_cause = 14;
        fail(d, MT_DOC_INTERNAL);
        return;
    }
    const uint32_t ustamp = (uint32_t)d.grp[g * MT_GRP_WORDS + 10];
    compute_ends(d);
    const int nblk = nbr(d, 0);
    // The group's segments in its own order (SegmentGroup.segments): first the ones its op
    // walked, in document order (their ids are below the stamp), then the right halves later
    // splits appended (segmentGroupCollection.ts copyTo), in split order = id order.
    int n_late = 0;
    for (int pass = 0; pass < 2; pass++) {
        const int rounds = pass == 0 ? 1 : n_late;
        uint32_t last = ustamp;
        for (int q = 0; q < rounds; q++) {
            uint32_t pick = 0xFFFFFFFFu;
            if (pass == 1) {   // the late member with the smallest id above the previous one
                for (int base = 0; base < d.n; base += MT_WAVE) {
                    const int i = base + lane();
                    const bool v = i < d.n;
                    const uint32_t uid = v ? (d.Bv[i].z & ~MT_MARKER_BIT) : 0xFFFFFFFFu;
                    const bool c = v && pq_first(pq_get(d, i)) == g && uid >= last;
                    uint32_t mn = c ? uid : 0xFFFFFFFFu;
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, MT_WAVE));
                    pick = min(pick, (uint32_t)uni((int)mn));
                }
                last = pick;
            }
            for (int base = 0; base < d.n; base += MT_WAVE) {
                const int i = base + lane();
                const bool v = i < d.n;
                v4i a;
                u64 o;
                load_ao(d, i, v, a, o);
                const v4u bv = d.Bv[v ? i : 0];
                const uint32_t uid = bv.z & ~MT_MARKER_BIT;
                const PendQ pq = pq_get(d, v ? i : 0);
                const bool mem0 = v && pq_first(pq) == g;
                const bool late = mem0 && uid >= ustamp;
                if (pass == 0) n_late += __popcll(ballot(late));
                const bool mem = pass == 0 ? (mem0 && !late) : (mem0 && uid == pick);
                bool bad = false;
                if (mem) {
                    if (kind == MT_OP_INSERT) {
                        bad = !is_local_seq(a.y);
                        a.y = op.seq;
                    } else if (kind == MT_OP_REMOVE && is_local_seq(a.z)) {
                        a.z = op.seq;   // else a remote remove replaced it: ack returns false
                    }
                    d.A[i] = a;
                    pq_put(d, i, pq_pop(pq));
                }
                if (ballot(bad)) {
                    FAIL_INTERNAL(d);
                    return;
                }
                wsync<T>();
                const int b = mem ? block_of(d, i, nblk) : -1;
                for (u64 m = ballot(mem); m; m &= m - 1) {
                    const int j = first_lane(m);
                    add_to_lru_block(d, bcast(b, j), (uint32_t)bcast((int)uid, j), op.seq);
                    if (d.status) return;
                }
            }
        }
    }
    d.g_head = g % d.LG + 1;
    d.g_n--;
}

TD void apply_op(DocT<T> &d, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin) {
    const mt_op_rec &op = in.op;
    d.ocs = oslot_of(d, op_cli(op));
    bool ack = false;
    if constexpr (T::kLive) {
        if (op.flags & MT_F_LOCAL) {
            live_local(d, in, tin, pin);
            return;
        }
        ack = (op.flags & MT_F_ACK) != 0;
    }
    if (op.flags & MT_F_LOAD) {
        // SnapshotLoader.loadBody (MT/snapshotLoader.ts:195-227): insertSegments at
        // root.cachedLength in view (client, refSeq 0), no callback, no seq/msn update.  Its
        // zamboniSegments has nothing to do: the heap is new (startCollaboration) and body
        // segments are never newer than currentSeq (addToLRUSet :1312).  No events.
        const int rich = d.rich;
        d.rich = 0;
        if (op.kind == MT_OP_INSERT)
            op_insert(d, in, tin, pin);
        else if (op.kind == MT_OP_LOAD_REMOVED)
            load_removed(d, op);
        else if (op.kind == MT_OP_LOAD_ALIASED)
            fail(d, MT_DOC_ALIASED);
        d.rich = rich;
        return;
    }
    const bool is_op = op.kind == MT_OP_INSERT || op.kind == MT_OP_REMOVE || op.kind == MT_OP_ANNOTATE;
    if constexpr (T::kLive) {
        if (ack && is_op) live_ack(d, op);
    }
    if (ack) {
    } else if (op.kind == MT_OP_INSERT) {
        op_insert(d, in, tin, pin);
    } else if (is_op) {
        op_range(d, op, pin);
    }
    if (d.status) return;
    bool z = is_op;
    for (int pass = 0; pass < 2; pass++) {
        if (z) {
            zamboni(d);
            if (d.status) return;
        }
        if (pass == 1) break;
        if (op.kind != MT_OP_NOOP && !ack) {
            if (!(d.cur_seq < op.seq)) {
                fail(d, MT_DOC_SEQ_ORDER);
                return;
            }
            if (!(d.min_seq <= op.min_seq)) {
                fail(d, MT_DOC_MINSEQ_ORDER);
                return;
            }
        }
        z = false;
        if (!(op.flags & MT_F_GROUP_MORE)) {
            if (!(d.cur_seq <= op.seq)) {   // updateSeqNumbers MT/client.ts:824
                fail(d, MT_DOC_SEQ_BACKWARDS);
                return;
            }
            d.cur_seq = op.seq;
            if (!(op.min_seq <= op.seq)) {    // MT/client.ts:826
                fail(d, MT_DOC_MSN_ABOVE_SEQ);
                return;
            }
            if (!(d.min_seq <= op.min_seq)) {   // setMinSeq MT/mergeTree.ts:1755
                fail(d, MT_DOC_MSN_BACKWARDS);
                return;
            }
            if (op.min_seq > d.min_seq) {
                d.min_seq = op.min_seq;
                z = true;
            }
        }
        if (!z) break;
    }
}
