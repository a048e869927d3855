// mt_paged.h -- paged layout for documents that outgrow the LDS tier (configs C3/C4:
// 3.5-4.5 k live segments, annotates keep property sets apart).
//
// A page is a level-1 node of the reference B-tree (MT/mergeTree.ts:333 MaxNodesInBlock=8):
// <= 7 leaf blocks of <= 7 segments, stored in HBM as 64 segment slots in document order
// plus a PageMeta (leaf-block counts, needsScour flags, observer length).  Levels >= 1 of
// the tree live in LDS for the launch (level 1 = pages in document order, counted in leaf
// blocks; `dir` maps level-1 positions to page ids).  An op costs O(pages/64 + unsettled/64)
// to find its page plus one page of work, instead of the flat engine's O(segments):
//
//  * page view lengths for a remote view (c, r): settled segments (seq <= minSeq and not
//    removed after minSeq) look the same in every view (refSeq >= minSeq), so a page's view
//    length is its observer length plus the (view - observer) difference of its unsettled
//    segments, kept in a per-document table (~200 entries on C3, each naming its page's
//    level-1 position).  Positions are grouped in chunks of 64: the chunks' observer lengths
//    are kept up to date, so a search sums the table's differences per chunk, picks the chunk
//    and then the page inside it -- O(table / 64 + pages / 4096) per op, not O(pages);
//  * the page is staged in a "window" DocT and the flat engine's own functions (op_insert,
//    boundary, range_mark, scour_range, pack at level 0) run on it unchanged; a page that
//    reaches MaxNodesInBlock leaf blocks is split 4|4 after the op (blk_split_up records it),
//    a page that underflows is repacked with its siblings (pack at level 1) in HBM;
//  * the zamboni heap is the flat one (LDS); a uid -> page map in HBM locates its segments;
//  * documents of thousands of pages (T::kHM) keep every PageMeta in HBM: the window's page
//    has its own in registers, searches read a chunk's 64 observer lengths once (sob).
#pragma once
#include "mt_engine.h"

// MT_PROF section timers of the paged driver (slots 9..15; the engine uses 0..8)
#ifdef MT_PROF
#define PG_T0(k) const unsigned long long _pt##k = __builtin_amdgcn_s_memtime();
#define PG_T1(k)                                                         \
    if (lane() == 0) {                                                   \
        pd.w.prof[k] += __builtin_amdgcn_s_memtime() - _pt##k;           \
        pd.w.prof[64 + k] += 1ull;                                       \
    }
#define PG_CNT(k)                                                        \
    if (lane() == 0) pd.w.prof[64 + k] += 1ull;
#else
#define PG_T0(k)
#define PG_T1(k)
#define PG_CNT(k)
#endif

template <class T> struct PagedDoc {
    DocT<T> w;    // window: one page staged in LDS (first member: see pdoc)
    DocT<T> up;   // levels >= 1 of the tree (level 1 = pages, counted in leaf blocks)
    LDS_AS PageMeta *meta;    // [PP] by page id (T::kHM: null -- gmeta instead)
    GLB_AS PageMeta *gmeta;   // T::kHM: the page metadata in HBM, where it lives for the launch
                              // (observer length, leaf-block counts, needsScour flags)
    LDS_AS int *pvl;          // [PP] by level-1 position: view length in the cached view (vr, vc)
    LDS_AS int *cob;          // T::kHM (no pvl): [PP / 64] observer length of each chunk of 64
    LDS_AS int *cdl;          //   level-1 positions, and its (view - observer) in the cached view
    int vgen, scr_ch;         // T::kHM: views computed so far; the chunk whose per-position
                              //   differences w.scr holds for view number vgen (-1: none)
    LDS_AS uint16_t *upage;   // [UT] unsettled-segment table: level-1 position, {len, seq, rseq, cli}, overlap
    LDS_AS v4i *uA;
    LDS_AS typename T::O_v *uO;
    LDS_AS uint32_t *uL, *uS, *uP;   // T::kPacked: len | seq, rseq (16 bits each, from sbase) |
    int sbase;                       // page, mask index, cli, rcli (8 bits each) -- tab_get / tab_put
    LDS_AS u64 *uM;                  // T::kPacked: the overlap masks of the entries that have one
    LDS_AS uint32_t *mbm;            // [MT_PK_MASKS] by index (0: none), and their use bitmap
    GLB_AS v4i *gA;           // this document's pages (slot 0 of page 0)
    GLB_AS u64 *gO;
    GLB_AS v4u *gB;
    GLB_AS uint16_t *gumap;   // (the bases used only at load / store are PgCold's: fewer live SGPRs)
    GLB_AS uint16_t *goS;     // segment ordinals (T::kLog handles with them): page slot / leaf-block
    GLB_AS uint16_t *goL;     // characters by page id (the window's os / ob point into them)
    int doc;
    int PP, PH, UT, UM;       // LDS capacities of this launch (pages, heap, table); uid map size
    int PPh;                  // page capacity of the HBM arrays (stride; >= PP)
    int ut_n;
    int cur;                  // page id staged in the window (-1: none)
    int cur_pos;              // its level-1 position (-1: not known yet)
    int dirty;                // the window differs from the page in HBM (slots, uid map, table)
    int tdirty;               // an op changed the window since it was loaded: its unsettled-table
                              // entries are rebuilt at the flush (zamboni's scours / packs change
                              // settled segments only, whose entries contribute nothing to a view)
    int uid_lo;               // next_uid when the window was loaded: older segments of the
                              // window are already mapped to its page
    int vvalid, vr, vc;       // cdl holds the chunk view differences of view (vr, vc): boundary
                              // splits keep them (lengths are preserved), any other change drops them
    int zuid, zpv;            // zamboni's first pop of the current message (known before the op:
                              // the op only adds heap entries above minSeq) and its page from the
                              // uid map, loaded at the message's start (zuid 0: none)
    GLB_AS uint16_t *govf;    // overflow overlap sets (MT_OVF_BIT; last-tier instantiations)
    int ovf_top, ovf_last, OA;   // its fill, the last message that made a set, its capacity
    int ovf_maxn, ovf_half;      // the largest set made; the half sets are appended in (the
                                 // other one receives the live sets at a compaction)
    uint32_t ovf_made;           // units of every set made (diagnostic: reclamation)
    int ovf_peak;                // the most units the half in use has held (diagnostic)
    int press;                // a compaction left the text (4) / record (5) arena more than 7/8
                              // full: a tight launch hands the document on (pg_arena_room)
    int wgrow, opbound;       // tight tier: bound on the table's growth not yet in ut_n (the
                              // window's entries since they were last rebuilt); the current
                              // message's bound (pg_room)
    LDS_AS int *sob;          // T::kHM: observer lengths of chunk sob_ch's 64 positions (a
    int sob_ch;               //   cache of the HBM values, kept in step by pg_win_sync; -1: none)
    int wnb, wobs;            // T::kHM: leaf blocks / observer length of the window's page as
                              //   its meta in HBM holds them (uniform)
};

// LDS capacities of one paged launch.  The HBM arrays are sized for the handle's paged
// capacities; a "tight" launch stages documents at smaller LDS capacities (more documents per
// CU) and hands a document over to the next launch, at full capacities, before a message
// that could outgrow them (pg_room) -- or at load, when it no longer fits.
struct PagedCaps {
    int PP, PH, UT;
    int tight;   // 1: hand over instead of failing; 0: the HBM capacities (last tier)
    int stage;   // retry[doc] value this launch serves (1: from the LDS tier, 2: from the tight
                 // tier, 3: from the growth step)
    int narrow;  // TierPagedT<., true>: 32-bit overlap masks in LDS (tight tier only)
    int grow;    // last tier: a document that does not fit at load, or whose next message could
                 // outgrow these capacities, is handed to the host's growth step (retry = 3)
                 // instead of failing -- re-tiered to a larger HBM region, it continues there;
                 // 2: only the HBM arenas and the uid map can still grow (pg_arena_room)
    int packed;  // TierPagedT<., ., ., true>: 12-byte unsettled-table entries (tight tier only)
};

#define PW_B 16   // window leaf-block capacity (a page holds <= 9 transiently)
#define MT_PK_MASKS 256   // packed table: overlap-mask slots (index 0: no mask)

struct PagedLayout {
    uint32_t offWA, offWB, offWO, offWcnt, offWflg, offWends, offWscr, offWnb;
    uint32_t offUcnt, offUnb, offDir, offMeta, offCob, offHeap, offUpage, offUA, offUO, offGen, offProf,
        total;
};
// ob: bytes per overlap mask in LDS (8, or 4 for a narrow tier)
// packed: the table's entries are 12 bytes (three u32 arrays at offUA) and carry their page
// hm: T::kHM (no per-page metadata in LDS: it stays in HBM)
static __host__ __device__ inline PagedLayout paged_layout(int PP, int PH, int UT, int gen_words, int ob,
                                                           bool packed = false, bool hm = false) {
    PagedLayout L;
    uint32_t o = 0;
    L.offWA = o; o += 16u * MT_PG_SLOTS;
    L.offWB = o; o += 16u * MT_PG_SLOTS;
    L.offWO = o; o += (uint32_t)ob * MT_PG_SLOTS;
    L.offUA = o; o += (packed ? 12u : 16u) * UT;
    // packed: a sparse mask table instead of one mask per entry (few unsettled segments carry
    // an overlap: C4 peaks at ~70 of ~1000)
    o = (o + 7u) & ~7u;
    L.offUO = o; o += packed ? 8u * MT_PK_MASKS + MT_PK_MASKS / 8 : ((((uint32_t)ob * UT) + 7u) & ~7u);
    L.offHeap = o; o += 8u * (PH + 1);
    L.offMeta = o; o += hm ? 0u : (uint32_t)sizeof(PageMeta) * PP;
    L.offUpage = o; o += packed ? 0u : (2u * UT + 3u) & ~3u;
    L.offCob = o; o += hm ? 8u * (uint32_t)((PP + 63) / 64) + 4u * 64 : 4u * PP;   // cob + cdl + sob, or pvl
    L.offWscr = o; o += 64u * 4;
    L.offWnb = o; o += MT_LV * 4;
    L.offUnb = o; o += MT_LV * 4;
    L.offGen = o; o += 4u * gen_words;
    L.offDir = o; o += 2u * PP;
    L.offWends = o; o += 2u * PW_B;
    L.offWcnt = o; o += (uint32_t)MT_LV * PW_B;
    L.offWflg = o; o += PW_B;
    L.offUcnt = o; o += (uint32_t)(pcnt_bytes(PP) - PP);   // levels >= 1 (level 0 is the window's)
#ifdef MT_PROF
    o = (o + 7u) & ~7u;
    L.offProf = o; o += 128u * 8;
#else
    L.offProf = 0;
#endif
    L.total = (o + 15u) & ~15u;
    return L;
}

// the window is PagedDoc's first member (standard layout: pointer-interconvertible); no
// pointer to the PagedDoc is stored, so the whole struct stays in registers
TD PagedDoc<T> &pdoc(DocT<T> &w) { return *reinterpret_cast<PagedDoc<T> *>(&w); }
// the launch's capacities with those the tier fixes at compile time (T::kPP ...) substituted
template <class T> __device__ __forceinline__ PagedCaps eff_caps(PagedCaps pc) {
    if constexpr (T::kPP > 0) pc.PP = T::kPP;
    if constexpr (T::kPH > 0) pc.PH = T::kPH;
    if constexpr (T::kUT > 0) pc.UT = T::kUT;
    return pc;
}
// a paged-layout capacity (cause: 4 text, 5 property records, 7 pages, 8 unsettled table,
// 9 uid map, 3 heap; kept in the header's HDR_DIAG word)
TD void pg_fail_cap(DocT<T> &w, int cause) {
    if (w.status == 0) w.cap_cause = cause;
    fail(w, MT_DOC_CAPACITY);
}
__device__ __forceinline__ PageMeta pm_load(const LDS_AS PageMeta *m) {
    PageMeta r;
    r.nseg = m->nseg;
    r.nblk = m->nblk;
    r.flg2 = m->flg2;
    r.bc = m->bc;
    r.obs = m->obs;
    return r;
}
__device__ __forceinline__ int pm_bcnt_l(const LDS_AS PageMeta *m, int q) { return (int)((m->bc >> (4 * q)) & 15u); }
__device__ __forceinline__ int8_t pm_flg_l(const LDS_AS PageMeta *m, int q) {
    return (int8_t)((int)((m->flg2 >> (2 * q)) & 3u) - 1);
}
// Page metadata accessors.  A tier with T::kHM (documents of thousands of pages: LDS per page
// sets how many share a CU) keeps only each page's segment / leaf-block counts and observer
// length in LDS; its leaf-block counts and needsScour flags stay in HBM (read when the page is
// staged, written back when it changes -- once per window move, not per op).
// T::kHM: no per-page LDS at all; the fields are global loads (after gsync_rd() where another
// lane wrote them) -- the window's page has them in registers (pg_win_fetch_blocks).
TD int pm_nseg(const PagedDoc<T> &pd, int pg) {
    if constexpr (T::kHM) {
        gsync_rd();
        return pd.gmeta[pg].nseg;
    } else {
        return pd.meta[pg].nseg;
    }
}
TD int pm_nblk(const PagedDoc<T> &pd, int pg) {
    if constexpr (T::kHM) {
        gsync_rd();
        return pd.gmeta[pg].nblk;
    } else {
        return pd.meta[pg].nblk;
    }
}
TD int pm_obs(const PagedDoc<T> &pd, int pg) {
    if constexpr (T::kHM) {
        gsync_rd();
        return pd.gmeta[pg].obs;
    } else {
        return pd.meta[pg].obs;
    }
}
TD void pm_set_ns(PagedDoc<T> &pd, int pg, int ns, int nb) {
    if constexpr (T::kHM) {
        pd.gmeta[pg].nseg = (uint8_t)ns;
        pd.gmeta[pg].nblk = (uint8_t)nb;
    } else {
        pd.meta[pg].nseg = (uint8_t)ns;
        pd.meta[pg].nblk = (uint8_t)nb;
    }
}
TD void pm_set_nblk(PagedDoc<T> &pd, int pg, int nb) {
    if constexpr (T::kHM) {
        pd.gmeta[pg].nblk = (uint8_t)nb;
    } else {
        pd.meta[pg].nblk = (uint8_t)nb;
    }
}
TD void pm_set_obs(PagedDoc<T> &pd, int pg, int obs) {
    if constexpr (T::kHM) pd.gmeta[pg].obs = obs;
    else pd.meta[pg].obs = obs;
}
// page pg's leaf-block counts and needsScour flags (any lane; T::kHM: a global load -- after
// gsync() + gsync_rd() when another lane may have written them)
TD void pm_blocks(const PagedDoc<T> &pd, int pg, uint32_t &bc, uint32_t &f2) {
    if constexpr (T::kHM) {
        bc = pd.gmeta[pg].bc;
        f2 = pd.gmeta[pg].flg2;
    } else {
        bc = pd.meta[pg].bc;
        f2 = pd.meta[pg].flg2;
    }
}
// the whole PageMeta of page pg (ordinal code paths)
TD PageMeta pm_page(const PagedDoc<T> &pd, int pg) {
    PageMeta m;
    m.nseg = (uint8_t)pm_nseg(pd, pg);
    m.nblk = (uint8_t)pm_nblk(pd, pg);
    uint32_t bc, f2;
    pm_blocks(pd, pg, bc, f2);
    m.bc = bc;
    m.flg2 = (uint16_t)f2;
    m.obs = pm_obs(pd, pg);
    return m;
}
__device__ __forceinline__ int pm_bc_of(uint32_t bc, int q) { return (int)((bc >> (4 * q)) & 15u); }
__device__ __forceinline__ int8_t pm_fl_of(uint32_t f2, int q) { return (int8_t)((int)((f2 >> (2 * q)) & 3u) - 1); }
// Packs the leaf-block counts / needsScour flags of page pg from lanes holding block q (v):
// all lanes call it (wave-uniform control flow); fields are disjoint, so the sum is an OR.
TD void pm_set_blocks(PagedDoc<T> &pd, int pg, int q, bool v, int cnt, int flg) {
    const uint32_t bc = (uint32_t)wave_sum(v ? (int)((uint32_t)cnt << (4 * q)) : 0);
    const uint32_t f2 = (uint32_t)wave_sum(v ? (flg + 1) << (2 * q) : 0);
    if (lane() == 0) {
        if constexpr (T::kHM) {
            pd.gmeta[pg].bc = bc;
            pd.gmeta[pg].flg2 = (uint16_t)f2;
        } else {
            pd.meta[pg].bc = bc;
            pd.meta[pg].flg2 = (uint16_t)f2;
        }
    }
}
TD bool unsettled(const v4i a, int min_seq) {
    return a.y > min_seq || (a.z != MT_RSEQ_NONE && a.z > min_seq);
}
// Lowest page id not in use (-1: none).  Pages in the directory always hold >= 1 leaf block,
// free ones none; the id is marked taken (its meta is written by the caller).  Allocation
// is rare (page split, repack), so a scan of the meta replaces a free list.
TD int pg_alloc(PagedDoc<T> &pd) {
    for (int base = 0; base < pd.PP; base += MT_WAVE) {
        const int pg = base + lane();
        const u64 m = ballot(pg < pd.PP && pm_nblk(pd, pg) == 0);
        if (m) {
            const int r = base + first_lane(m);
            if (lane() == 0) pm_set_nblk(pd, r, 1);
            wsync<T>();
            return r;
        }
    }
    return -1;
}

// dir position of page id pg (-1 if not in the directory)
TD int pg_pos(PagedDoc<T> &pd, int pg) {
    const int np = nbr(pd.up, 1);
    for (int base = 0; base < np; base += MT_WAVE) {
        const int q = base + lane();
        const u64 m = ballot(q < np && pd.up.dir[q] == pg);
        if (m) return base + first_lane(m);
    }
    return -1;
}

TD int pg_cur_pos(PagedDoc<T> &pd) {
    if (pd.cur_pos < 0) pd.cur_pos = pg_pos(pd, pd.cur);
    return pd.cur_pos;
}
// observer position of the window page's first segment (the pages before it in the directory:
// whole chunks, then the chunk's pages before it)
TD int pg_obs_start(PagedDoc<T> &pd) {
    const int pos = pg_cur_pos(pd);
    int s = 0;
    if constexpr (T::kHM) {
        gsync_rd();
        const int c = pos >> 6;
        for (int base = 0; base < c; base += MT_WAVE) s += base + lane() < c ? pd.cob[base + lane()] : 0;
        const int q = (c << 6) + lane();
        s += q < pos ? pm_obs(pd, pd.up.dir[q]) : 0;
    } else {
        for (int base = 0; base < pos; base += MT_WAVE) {
            const int q = base + lane();
            s += q < pos ? pm_obs(pd, pd.up.dir[q]) : 0;
        }
    }
    return wave_sum(s);
}
// Chunk observer lengths from the pages (after the directory changed: page split, pack at
// level 1, load, conversion): one wave sum per chunk of 64 positions.
TD void pg_cob_rebuild(PagedDoc<T> &pd) {
    pd.vvalid = 0;
    if constexpr (!T::kHM) return;
    pd.sob_ch = -1;
    gsync_rd();
    const int np = nbr(pd.up, 1);
    for (int base = 0; base < np; base += MT_WAVE) {
        const int q = base + lane();
        const int s = wave_sum(q < np ? pm_obs(pd, pd.up.dir[q]) : 0);
        if (lane() == 0) pd.cob[base >> 6] = s;
    }
    pd.vvalid = 0;
    wsync<T>();
}
// Table positions at or after `from` move by delta (a page inserted / pages replaced there).
TD void pg_table_shift(PagedDoc<T> &pd, int from, int delta) {
    for (int e = lane(); e < pd.ut_n; e += MT_WAVE) {
        if constexpr (T::kPacked) {
            const uint32_t pc = pd.uP[e];
            const int pos = (int)(pc & 0xFFu);
            if (pos >= from) pd.uP[e] = (pc & ~0xFFu) | (uint32_t)((pos + delta) & 0xFF);
        } else {
            const int pos = pd.upage[e];
            if (pos >= from) pd.upage[e] = (uint16_t)(pos + delta);
        }
    }
    wsync<T>();
}

// ------------------------------------------------------------------ segment ordinals
// The flat engine's representation (mt_engine.h "segment ordinals": one character per node,
// an ordinal is the ancestors' characters below the root then the node's own) over the paged
// layout, in HBM: each page keeps its slots' characters (PagedDoc.goS, 64 per page) and its
// leaf blocks' (goL), and the upper instance keeps levels >= 1 by level position (DocT.ob,
// level 1 = pages in directory order, moved with the directory by blk_shift).  The window's
// os / ob point at its page's arrays, so every engine step inside a page (inserts, splits,
// leaf-block splits, scours, pack of the page's leaf blocks) writes them as for a flat
// document; the steps that cross pages re-derive from the upper instance (pg_ord_canon_up):
// a page split (blk_split_up of the upper instance, whose page-level link is pg_split_page's
// sp_*), pack at level 1 (pg_pack1: the topmost parent, :1444-1450), a new root (updateRoot
// :1909-1920) and a converted document without characters (reloadFromSegments).
// The PagedDoc of its upper instance (the second member)
TD PagedDoc<T> &updoc(DocT<T> &up) {
    return *reinterpret_cast<PagedDoc<T> *>(reinterpret_cast<char *>(&up) - offsetof(PagedDoc<T>, up));
}
// canonical characters of page pg's leaf blocks and slots (nodeUpdateOrdinals of the page):
// leaf block q of nb gets (q + 1) * width(nb) - 1, slot k of block q's c_q the same in c_q
TD void pg_ord_canon_page(PagedDoc<T> &pd, int pg, bool root_leaf) {
    const PageMeta m = pm_page(pd, pg);
    const int nb = root_leaf ? 1 : (int)m.nblk;
    const int t = lane();
    int q = 0, st = 0, c = root_leaf ? (int)m.nseg : pm_bcnt(m, 0);
    while (q + 1 < nb && t >= st + c) {
        st += c;
        q++;
        c = pm_bcnt(m, q);
    }
    if (t < (int)m.nseg) pd.goS[(size_t)pg * MT_PG_SLOTS + t] = (uint16_t)((t - st + 1) * ord_w(c) - 1);
    if (!root_leaf && t < nb) pd.goL[(size_t)pg * MT_PG_OLB + t] = (uint16_t)((t + 1) * ord_w(nb) - 1);
}
TD void pg_ord_canon_up(DocT<T> &up, int l, int b) {
    PagedDoc<T> &pd = updoc(up);
    if (l == 0) {   // a one-level tree: the root is page dir[0]'s only leaf block
        pg_ord_canon_page(pd, uni((int)up.dir[0]), true);
        gsync();
        return;
    }
    int lo = b, hi = b + 1;
    for (int j = l; j >= 2; j--) {   // children of [lo, hi) at level j: nodes of level j - 1
        const int c0 = blk_prefix(up, j, lo);
        int carry = c0;
        GLB_AS uint16_t *dst = up.ob + (size_t)(j - 1) * up.obst;
        const LDS_AS uint8_t *cnt = lvl(up, j);
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
    for (int q = lo; q < hi; q++) pg_ord_canon_page(pd, uni((int)up.dir[q]), false);   // level-1 nodes
    gsync();
}
// The ordinal of slot i of page pg (codes[0 .. depth)): window counts for the current page,
// the page metadata otherwise.
TD int pg_ord_of_page(PagedDoc<T> &pd, int pg, int i, int *codes) {
    DocT<T> &w = pd.w;
    DocT<T> &up = pd.up;
    gsync();
    // a root leaf block split inside this step: the page is the root (pg_win_sync sets up.depth)
    const int D = (up.depth == 1 && pg == pd.cur && w.depth == 2) ? 2 : up.depth;
    codes[D - 1] = uni((int)pd.goS[(size_t)pg * MT_PG_SLOTS + i]);
    if (D == 1) return 1;
    int q;
    if (pg == pd.cur) {
        int st;
        q = blk_find(w, 0, i, true, st);
    } else {
        const PageMeta m = pm_page(pd, pg);
        int st = 0;
        q = 0;
        while (q + 1 < (int)m.nblk && i >= st + pm_bcnt(m, q)) st += pm_bcnt(m, q++);
        q = uni(q);
    }
    if (q < 0) return -1;
    codes[D - 2] = uni((int)pd.goL[(size_t)pg * MT_PG_OLB + q]);
    if (D == 2) return 2;
    int x = pg == pd.cur ? pg_cur_pos(pd) : pg_pos(pd, pg);
    if (x < 0) return -1;
    codes[D - 3] = uni((int)up.ob[(size_t)up.obst + x]);
    for (int l = 2; l + 1 < D; l++) {
        int st;
        const int b = blk_find(up, l, x, true, st);
        if (b < 0) return -1;
        codes[D - 2 - l] = uni((int)up.ob[(size_t)l * up.obst + b]);
        x = b;
    }
    return D;
}
TD int pg_ord_of_win(DocT<T> &w, int i, int *codes) { return pg_ord_of_page(pdoc(w), pdoc(w).cur, i, codes); }
// The insert callback's [uid, position, ordinal] entry once the op's page split is done
// (op_insert deferred it: DocT.dfr_*); the segment is in the window or in the new page.
TD void pg_log_deferred(PagedDoc<T> &pd) {
    if constexpr (T::kLog) {
        DocT<T> &w = pd.w;
        const int rec = w.dfr_rec;
        w.dfr_rec = -1;
        const uint32_t uid = (uint32_t)w.dfr_uid;
        int pg = pd.cur, i = find_uid(w, uid);
        if (i < 0 && uid < (uint32_t)pd.UM) {
            gsync();
            pg = uni((int)pd.gumap[uid]);
            const bool hit = lane() < pm_nseg(pd, pg) &&
                             (pd.gB[(size_t)pg * MT_PG_SLOTS + lane()].z & ~MT_MARKER_BIT) == uid;
            const u64 m = ballot(hit);
            i = m ? first_lane(m) : -1;
        }
        int codes[MT_LV + 1];
        const int olen = i >= 0 ? pg_ord_of_page(pd, pg, i, codes) : -1;
        if (olen < 0) {
            FAIL_INTERNAL(w);
            return;
        }
        if (!w.dlog || w.dlog_n + 3 + olen > w.DL_cap) {   // the whole record goes (cb_room)
            if (w.dlog) {
                w.dlog_n = rec;
                w.dlog_ovf = 1;
            }
            return;
        }
        GLB_AS int32_t *o = w.dlog + w.dlog_n;
        if (lane() == 0) {
            o[0] = (int32_t)uid;
            o[1] = w.dfr_pos;
            o[2] = olen;
            for (int q = 0; q < olen; q++) o[3 + q] = codes[q];
        }
        w.dlog_n += 3 + olen;
    }
}

// ------------------------------------------------------------------ window load / store
TD void pg_win_load_impl(PagedDoc<T> &pd, int pg);
TD void pg_win_load(PagedDoc<T> &pd, int pg) {
    PG_T0(10)
    pg_win_load_impl(pd, pg);
    PG_T1(10)
}
// page pg's slots into registers (lane i: slot i)
TD void pg_win_fetch(PagedDoc<T> &pd, int pg, v4i &a, u64 &o, v4u &b) {
    // (T::kHM: every slot -- the page's count arrives with its meta, pg_win_fetch_blocks, so
    // the rows do not wait for it; slots past the count are never placed)
    const int n = T::kHM ? MT_PG_SLOTS : uni(pm_nseg(pd, pg));
    const int i = lane();
    if (i < n) {
        a = pd.gA[(size_t)pg * MT_PG_SLOTS + i];
        o = pd.gO[(size_t)pg * MT_PG_SLOTS + i];
        b = pd.gB[(size_t)pg * MT_PG_SLOTS + i];
    }
}
// the page's leaf-block words: from LDS, or (T::kHM) loaded beside its slots with its
// leaf-block count (f2 bits 16..23), segment count (bits 24..31) and observer length (ob), lane 0
TD void pg_win_fetch_blocks(PagedDoc<T> &pd, int pg, uint32_t &bc, uint32_t &f2, int &ob) {
    if constexpr (T::kHM) {
        bc = f2 = 0;
        ob = 0;
        if (lane() == 0) {
            gsync_rd();
            const GLB_AS PageMeta *m = pd.gmeta + pg;
            bc = m->bc;
            f2 = (uint32_t)m->flg2 | ((uint32_t)m->nblk << 16) | ((uint32_t)m->nseg << 24);
            ob = m->obs;
        }
    }
}
TD void pg_win_place(PagedDoc<T> &pd, int pg, const v4i &a, const u64 &o, const v4u &b, uint32_t bc, uint32_t f2,
                     int ob);
TD void pg_win_load_impl(PagedDoc<T> &pd, int pg) {
    v4i a = v4i{0, 0, 0, 0};
    u64 o = 0;
    v4u b = v4u{0, 0, 0, 0};
    uint32_t bc = 0, f2 = 0;
    int ob = 0;
    pg_win_fetch(pd, pg, a, o, b);
    pg_win_fetch_blocks(pd, pg, bc, f2, ob);
    pg_win_place(pd, pg, a, o, b, bc, f2, ob);
}
TD void pg_win_place(PagedDoc<T> &pd, int pg, const v4i &a, const u64 &o, const v4u &b, uint32_t bc, uint32_t f2,
                     int ob) {
    DocT<T> &w = pd.w;
    int n, nb;
    if constexpr (T::kHM) {
        bc = (uint32_t)bcast((int)bc, 0);
        f2 = (uint32_t)bcast((int)f2, 0);
        n = (int)(f2 >> 24);
        nb = (int)((f2 >> 16) & 0xFFu);
        f2 &= 0xFFFFu;
        pd.wnb = nb;
        pd.wobs = bcast(ob, 0);
    } else {
        n = uni(pm_nseg(pd, pg));
        nb = uni(pm_nblk(pd, pg));
        pm_blocks(pd, pg, bc, f2);
    }
    const int i = lane();
    if (i < n) {
        w.A[i] = a;
        w.O[i] = o;
        w.Bv[i] = b;
    }
    if (i < PW_B) {
        lvl(w, 0)[i] = i < nb ? (uint8_t)pm_bc_of(bc, i & 7) : 0;
        w.flg[i] = i < nb ? pm_fl_of(f2, i & 7) : (int8_t)0;
    }
    if (i == 0) {
        w.nb[0] = nb;
        w.nb[1] = 1;
        lvl(w, 1)[0] = (uint8_t)nb;
    }
    w.n = n;
    w.depth = pd.up.depth == 1 ? 1 : 2;
    if (ordon(w)) {   // the page's own ordinal characters (its slots, its leaf blocks)
        w.os = pd.goS + (size_t)pg * MT_PG_SLOTS;
        w.ob = pd.goL + (size_t)pg * MT_PG_OLB;
    }
    w.pend_split = 0;
    w.pend_second = -1;
    w.dlo = MT_PG_SLOTS;
    pd.cur = pg;
    pd.cur_pos = -1;
    pd.dirty = 0;
    pd.tdirty = 0;
    pd.uid_lo = w.next_uid;
    // the table holds >= as many entries for this page as it has unsettled segments now
    pd.wgrow = max(pd.wgrow, pd.opbound);
    wsync<T>();
}

// ------------------------------------------------------------------ table entries
// Packed table (T::kPacked): seq / removedSeq as 16-bit offsets from sbase = the document's
// currentSeq at load - 32000 (0xFFFF: not removed).  A value below sbase is stored as sbase:
// the tier only takes documents whose collab window is under 30000 messages (pg_load), so
// such a segment's value is below minSeq and compares the same way in every view (refSeq >=
// minSeq) and in unsettled(); messages more than 65000 above sbase go to the next tier
// (pg_room).  Short client ids are 8-bit signed (the host packs only when every id of the
// handle fits).
__device__ __forceinline__ uint32_t sq_enc(int v, int sbase) {
    return v == MT_RSEQ_NONE ? 0xFFFFu : (uint32_t)min(max(v - sbase, 0), 0xFFFE);
}
__device__ __forceinline__ int sq_dec(uint32_t v, int sbase) { return v == 0xFFFFu ? MT_RSEQ_NONE : (int)v + sbase; }
TD void tab_get(PagedDoc<T> &pd, int e, int &pg, v4i &a, u64 &o) {
    if constexpr (T::kPacked) {
        const uint32_t l = pd.uL[e], sq = pd.uS[e], pc = pd.uP[e];
        pg = (int)(pc & 0xFFu);
        a = v4i{(int)l, sq_dec(sq & 0xFFFFu, pd.sbase), sq_dec(sq >> 16, pd.sbase),
                pack_cli((int)(int8_t)(pc >> 16), (int)(int8_t)(pc >> 24))};
        const uint32_t mi = (pc >> 8) & 0xFFu;
        o = pd.uM[mi];   // (slot 0 holds 0: an unconditional load, see pg_load)
    } else {
        pg = pd.upage[e];
        a = pd.uA[e];
        o = pd.uO[e];
    }
}
// mi: the entry's mask slot (tab_midx; packed tables only)
TD void tab_put(PagedDoc<T> &pd, int e, int pg, const v4i &a, u64 o, int mi = 0) {
    if constexpr (T::kPacked) {
        pd.uL[e] = (uint32_t)a.x;
        pd.uS[e] = sq_enc(a.y, pd.sbase) | (sq_enc(a.z, pd.sbase) << 16);
        pd.uP[e] = (uint32_t)(pg & 0xFF) | ((uint32_t)mi << 8) | ((uint32_t)(seg_cli(a) & 0xFF) << 16) |
                   ((uint32_t)(seg_rcli(a) & 0xFF) << 24);
        if (mi) pd.uM[mi] = o;
    } else {
        pd.upage[e] = (uint16_t)pg;
        pd.uA[e] = a;
        pd.uO[e] = (typename T::O_v)o;
    }
}
// Packed tables move an entry as it is (its mask slot goes with it).
TD v4i tab_raw(PagedDoc<T> &pd, int e) { return v4i{(int)pd.uL[e], (int)pd.uS[e], (int)pd.uP[e], 0}; }
TD void tab_raw_put(PagedDoc<T> &pd, int e, const v4i &r) {
    pd.uL[e] = (uint32_t)r.x;
    pd.uS[e] = (uint32_t)r.y;
    pd.uP[e] = (uint32_t)r.z;
}
// Mask slots of a packed table: lanes with `need` get distinct free slots (1..255), marked used
// in the bitmap; a slot dropped with its entry stays marked until a collection (tab_mgc) when
// too few are free.  -1 (every lane): not enough slots even after one.  Wave-uniform call.
TD void tab_mgc(PagedDoc<T> &pd) {
    if (lane() < MT_PK_MASKS / 32) pd.mbm[lane()] = lane() == 0 ? 1u : 0u;   // (slot 0: no mask)
    wsync<T>();
    for (int e = lane(); e < pd.ut_n; e += MT_WAVE) {
        const uint32_t mi = (pd.uP[e] >> 8) & 0xFFu;
        if (mi) atomicOr((uint32_t *)&pd.mbm[mi >> 5], 1u << (mi & 31));
    }
    wsync<T>();
}
TD int tab_mfree(PagedDoc<T> &pd) {
    const int f = lane() < MT_PK_MASKS / 32 ? __popc(~pd.mbm[lane()]) : 0;
    return wave_sum(f);
}
TD int tab_midx(PagedDoc<T> &pd, bool need) {
    if constexpr (!T::kPacked) {
        return 0;
    } else {
        const u64 m = ballot(need);
        if (!m) return 0;
        const int k = __popcll(m);
        if (tab_mfree(pd) < k) {
            tab_mgc(pd);
            if (tab_mfree(pd) < k) return -1;
        }
        int mi = 0;
        if (need) {
            int r = __popcll(m & ((1ull << lane()) - 1ull));
            for (int wd = 0; wd < MT_PK_MASKS / 32; wd++) {
                uint32_t f = ~pd.mbm[wd];
                const int c = __popc(f);
                if (r < c) {
                    for (; r > 0; r--) f &= f - 1;
                    mi = wd * 32 + __ffs(f) - 1;
                    break;
                }
                r -= c;
            }
        }
        wsync<T>();
        if (need) atomicOr((uint32_t *)&pd.mbm[mi >> 5], 1u << (mi & 31));
        wsync<T>();
        return mi;
    }
}

// Removes the table entries of level-1 position pg (and every settled entry); pg_table_add
// appends the unsettled segments of window slots [lo, hi) under position pg2.
TD void pg_table_purge(PagedDoc<T> &pd, int pg) {
    const int ms = pd.w.min_seq;
    int dst = 0;
    for (int base = 0; base < pd.ut_n; base += MT_WAVE) {
        const int e = base + lane();
        const bool v = e < pd.ut_n;
        int p = -1;
        v4i a = v4i{0, 0, MT_RSEQ_NONE, 0};
        u64 o = 0;
        v4i raw = v4i{0, 0, 0, 0};
        if (v) {
            tab_get(pd, e, p, a, o);
            if constexpr (T::kPacked) raw = tab_raw(pd, e);
        }
        const bool keep = v && p != pg && unsettled<T>(a, ms);
        const u64 km = ballot(keep);
        const int at = dst + __popcll(km & ((1ull << lane()) - 1ull));
        wsync<T>();
        if (keep) {
            if constexpr (T::kPacked)
                tab_raw_put(pd, at, raw);
            else
                tab_put(pd, at, p, a, o);
        }
        wsync<T>();
        dst += __popcll(km);
    }
    pd.ut_n = dst;
}
TD void pg_table_add(PagedDoc<T> &pd, int lo, int hi, int pg2) {
    DocT<T> &w = pd.w;
    const int i = lane() + lo;
    const bool v = i < hi;
    v4i a;
    u64 o;
    load_ao(w, i, v, a, o);
    const bool add = v && unsettled<T>(a, w.min_seq);
    const u64 m = ballot(add);
    if (pd.ut_n + __popcll(m) > pd.UT) {
        pg_fail_cap(w, 8);
        return;
    }
    const int mi = tab_midx(pd, add && o != 0);
    if (mi < 0) {
        pg_fail_cap(w, 8);
        return;
    }
    const int at = pd.ut_n + __popcll(m & ((1ull << lane()) - 1ull));
    if (add) tab_put(pd, at, pg2, a, o, mi);
    pd.ut_n += __popcll(m);
    wsync<T>();
}

// Writes window slots [lo, hi) to page pg (slot 0 = lo) with its meta (blocks [b0, b1) of
// the window) and the uid -> page map.  Slots below `from` (relative to lo) are unchanged
// in HBM and are not written.
TD void pg_write_page(PagedDoc<T> &pd, int pg, int lo, int hi, int b0, int b1, int from = 0) {
    DocT<T> &w = pd.w;
    const int i = lane();
    GLB_AS v4i *gA = pd.gA + (size_t)pg * MT_PG_SLOTS;
    GLB_AS u64 *gO = pd.gO + (size_t)pg * MT_PG_SLOTS;
    GLB_AS v4u *gB = pd.gB + (size_t)pg * MT_PG_SLOTS;
    int ol = 0;
    if (lo + i < hi) {
        const v4i a = w.A[lo + i];
        if (i >= from) {
            const v4u b = w.Bv[lo + i];
            gA[i] = a;
            gO[i] = w.O[lo + i];
            gB[i] = b;
            const uint32_t uid = b.z & ~MT_MARKER_BIT;
            // the uid -> page map changes only for segments created since the window was
            // loaded, or moved to another page (scattered 2-byte writes: one sector each)
            if (uid < (uint32_t)pd.UM && (pg != pd.cur || uid >= (uint32_t)pd.uid_lo)) pd.gumap[uid] = (uint16_t)pg;
        }
        ol = obs_len(a);
    }
    const int obs = wave_sum(ol);
    const bool vb = i < 8 && b0 + i < b1;
    pm_set_blocks(pd, pg, i, vb, vb ? lvl(w, 0)[b0 + i] : 0, vb ? w.flg[b0 + i] : 0);
    if (i == 0) {
        pm_set_ns(pd, pg, hi - lo, b1 - b0);
        pm_set_obs(pd, pg, obs);
    }
    if constexpr (T::kHM) {
        if (pg == pd.cur) {
            if (obs != pd.wobs) pd.sob_ch = -1;   // (pg_win_sync keeps the cache otherwise)
            pd.wnb = b1 - b0;
            pd.wobs = obs;
        } else {
            pd.sob_ch = -1;
        }
    }
    wsync<T>();
}

// Page split: the window's page reached MaxNodesInBlock leaf blocks during the op
// (insertingWalk :2479-2503 / split :2509-2522 at level 1, updateRoot :1909-1920).  The
// reference splits 4|4 at once; a second leaf split of the same op then lands in one half.
TD void pg_split_page(PagedDoc<T> &pd) {
    DocT<T> &w = pd.w;
    DocT<T> &up = pd.up;
    const int nbk = nbr(w, 0);
    const int sp = (nbk == MT_MAXN + 1 && w.pend_second >= 0 && w.pend_second < MT_HALF) ? MT_HALF + 1 : MT_HALF;
    int s0 = 0;
    for (int q = 0; q < sp; q++) s0 += cntr(w, 0, q);
    const int np = pg_alloc(pd);
    if (np < 0) {
        pg_fail_cap(w, 7);
        return;
    }
    PG_CNT(25)
    pd.zuid = 0;   // zamboni's prefetched page may be the moved half's
    const int pos = pg_cur_pos(pd);
    // table: the window's entries are rebuilt now (first half at this position, second half
    // at the new page's, pos + 1, after the later positions moved up), so it never holds both
    // a stale and a fresh copy of a segment
    pg_table_purge(pd, pos);
    pg_table_shift(pd, pos + 1, 1);
    pg_table_add(pd, 0, s0, pos);
    if (w.status) return;
    pg_table_add(pd, s0, w.n, pos + 1);
    if (w.status) return;
    pd.wgrow = pd.opbound;
    pg_write_page(pd, np, s0, w.n, sp, nbk);
    pd.vvalid = 0;   // (the chunks are rebuilt once the directory holds the new page)
    if (ordon(w)) {
        // segment ordinals: blk_split_up re-derives the split halves' subtrees from the page
        // metadata, so this page's holds its first sp blocks already, and level 1 links the
        // new page in with the real counts (blk_split_up: sp_*)
        const bool vb = lane() < sp;
        pm_set_blocks(pd, pd.cur, lane(), vb, vb ? lvl(w, 0)[lane()] : 0, vb ? w.flg[lane()] : 0);
        if (lane() == 0) pm_set_ns(pd, pd.cur, s0, sp);
        up.sp_pg = np;
        up.sp_l = sp;
        up.sp_r = nbk - sp;
        wsync<T>();
    }
    // level 1: new node after cur (blk_split_up grows the parents / the root)
    blk_split_up(up, 1, pos);
    if (up.status) {
        pg_fail_cap(w, 7);
        return;
    }
    if (lane() == 0) {
        lvl(up, 1)[pos] = (uint8_t)sp;
        lvl(up, 1)[pos + 1] = (uint8_t)(nbk - sp);
        up.dir[pos + 1] = (uint16_t)np;
    }
    // the window keeps the first sp blocks
    w.n = s0;
    if (lane() == 0) {
        w.nb[0] = sp;
        lvl(w, 1)[0] = (uint8_t)sp;
    }
    w.pend_split = 0;
    w.pend_second = -1;
    wsync<T>();
}

// After a step that modified the window: resolves a pending page split and brings the
// page's metadata and level-1 count up to date (LDS only; the slots stay in the window).
TD void pg_win_sync(PagedDoc<T> &pd) {
    DocT<T> &w = pd.w;
    DocT<T> &up = pd.up;
    if (pd.cur < 0) return;
    if (w.depth == 2 && up.depth == 1) {   // the root leaf block split: the page is the root now
        up.depth = 2;
        if (lane() == 0) up.nb[2] = 0;
    }
    const bool split = w.pend_split != 0;
    if (split) {
        pg_split_page(pd);
        if (w.status) return;
    }
    const int nbk = nbr(w, 0);
    const int i = lane();
    int ol = 0;
    if (i < w.n) ol = obs_len(w.A[i]);
    const int obs = wave_sum(ol);
    const int pg = pd.cur;
    // the level-1 count (== meta nblk) changes only with the page's leaf-block count, the
    // chunk's observer length only with the page's: its directory position is looked up only
    // then (an op's window knows it)
    int old_nb, old_obs;
    if constexpr (T::kHM) {
        old_nb = pd.wnb;
        old_obs = pd.wobs;
    } else {
        old_nb = uni(pm_nblk(pd, pg));
        old_obs = uni(pm_obs(pd, pg));
    }
    const bool vb = i < 8 && i < nbk;
    pm_set_blocks(pd, pg, i, vb, vb ? lvl(w, 0)[i] : 0, vb ? w.flg[i] : 0);
    const int pos = (nbk != old_nb || (T::kHM && obs != old_obs)) ? pg_cur_pos(pd) : -1;
    if (i == 0) {
        pm_set_ns(pd, pg, w.n, nbk);
        pm_set_obs(pd, pg, obs);
        if (pos >= 0) lvl(up, 1)[pos] = (uint8_t)nbk;
        if (T::kHM && pos >= 0 && !split) {
            pd.cob[pos >> 6] += obs - old_obs;
            if ((pos >> 6) == pd.sob_ch) pd.sob[pos & 63] = obs;
        }
    }
    if constexpr (T::kHM) {
        pd.wnb = nbk;
        pd.wobs = obs;
    }
    pd.dirty = 1;
    wsync<T>();
    if (split) pg_cob_rebuild(pd);
}

// Writes a dirty window back: slots and uid map to HBM, its unsettled-table entries rebuilt.
TD void pg_win_flush_impl(PagedDoc<T> &pd);
TD void pg_win_flush(PagedDoc<T> &pd) {
    PG_T0(11)
    pg_win_flush_impl(pd);
    PG_T1(11)
}
TD void pg_win_flush_impl(PagedDoc<T> &pd) {
    DocT<T> &w = pd.w;
    if (pd.cur < 0 || !pd.dirty) return;
#ifdef MT_NO_DIRTY
    w.dlo = 0;
#endif
    if (w.dlo < w.n) {   // some slot changed: its table entries and the slots from dlo on
        PG_CNT(23)
#ifndef MT_FLUSH_TABLE_ALWAYS
        if (pd.tdirty) {
#endif
            const int pos = pg_cur_pos(pd);   // (an op's window: known)
            PG_T0(33)
            pg_table_purge(pd, pos);
            PG_T1(33)
            PG_T0(34)
            pg_table_add(pd, 0, w.n, pos);
            PG_T1(34)
            if (w.status) return;
#ifndef MT_FLUSH_TABLE_ALWAYS
        }
#endif
        PG_T0(35)
        pg_write_page(pd, pd.cur, 0, w.n, 0, nbr(w, 0), w.dlo);
        PG_T1(35)
    }
    w.dlo = MT_PG_SLOTS;
    pd.dirty = 0;
    pd.wgrow = pd.opbound;   // exact again, up to the rest of the current message
}

// Replaces the window by page pg: its loads are issued before the current window is
// written back, so their latency hides behind the flush.
TD void pg_win_switch(PagedDoc<T> &pd, int pg) {
    v4i a = v4i{0, 0, 0, 0};
    u64 o = 0;
    v4u b = v4u{0, 0, 0, 0};
    uint32_t bc = 0, f2 = 0;
    int ob = 0;
    pg_win_fetch(pd, pg, a, o, b);
    pg_win_fetch_blocks(pd, pg, bc, f2, ob);
    pg_win_flush(pd);
    if (pd.w.status) return;
    PG_T0(10)
    pg_win_place(pd, pg, a, o, b, bc, f2, ob);
    PG_T1(10)
}

// ------------------------------------------------------------------ page view lengths
// A page's length in view (c, r) is its observer length (PageMeta.obs) plus the (view -
// observer) difference of its unsettled segments: their table entries, or -- when an op has
// changed the window since it was loaded (tdirty) -- the window's own slots for its page (its
// entries are rebuilt only at the flush; zamboni's scours change settled segments only, so a
// window they alone touched keeps exact entries).  Level-1 positions are grouped in chunks of
// 64 whose observer lengths (cob) are kept up to date; a view sums the differences per chunk
// (cdl, O(table / 64)), and a search picks the chunk, then the page inside it.
TD int pg_win_delta(PagedDoc<T> &pd, int r, int c) {
    DocT<T> &w = pd.w;
    const int i = lane();
    v4i a;
    u64 o;
    load_ao(w, i, i < w.n, a, o);
    return wave_sum(i < w.n ? vlen(w, a, o, r, c) - obs_len(a) : 0);
}
// cdl for view (r, c); returns the total length when asked (the generator draws positions
// from it; replay only needs cdl).
TD int pg_views_impl(PagedDoc<T> &pd, int r, int c, bool total);
TD int pg_views(PagedDoc<T> &pd, int r, int c, bool total = true) {
    PG_T0(9)
    const int r_ = pg_views_impl(pd, r, c, total);
    PG_T1(9)
    pd.vvalid = 1;
    pd.vr = r;
    pd.vc = c;
    return r_;
}
// cdl for view (r, c): recomputed only if a change other than a boundary split happened
TD void pg_views_cached(PagedDoc<T> &pd, int r, int c) {
    if (!(pd.vvalid && pd.vr == r && pd.vc == c)) pg_views(pd, r, c, false);
}
TD int pg_views_impl(PagedDoc<T> &pd, int r, int c, bool total) {
    const int np = nbr(pd.up, 1);
    const bool win = pd.cur >= 0 && pd.tdirty;
    const int wpos = win ? pg_cur_pos(pd) : -1;
    if constexpr (!T::kHM) {   // pvl[position] = observer length + differences
        for (int base = 0; base < np; base += MT_WAVE) {
            const int q = base + lane();
            if (q < np) pd.pvl[q] = pm_obs(pd, pd.up.dir[q]);
        }
        wsync<T>();
        PG_T0(36)
        for (int base = 0; base < pd.ut_n; base += MT_WAVE) {
            const int e = base + lane();
            if (e < pd.ut_n) {
                int pos;
                v4i a;
                u64 o;
                tab_get(pd, e, pos, a, o);
                const int dlt = vlen(pd.w, a, o, r, c) - obs_len(a);
                if (dlt && pos != wpos) atomicAdd((int *)(pd.pvl + pos), dlt);
            }
        }
        PG_T1(36)
        if (win) {
            const int dlt = pg_win_delta(pd, r, c);
            if (lane() == 0) pd.pvl[wpos] += dlt;
        }
        wsync<T>();
#ifndef MT_VIEWS_TOTAL
        if (!total) return 0;
#endif
        int tot = 0;
        for (int base = 0; base < np; base += MT_WAVE) tot += base + lane() < np ? pd.pvl[base + lane()] : 0;
        return wave_sum(tot);
    } else {   // cdl[chunk] = differences
        const int nch = (np + 63) >> 6;
        pd.vgen = (pd.vgen + 1) & 0x7FFF;
        for (int base = 0; base < nch; base += MT_WAVE)
            if (base + lane() < nch) pd.cdl[base + lane()] = 0;
        wsync<T>();
        PG_T0(36)
        for (int base = 0; base < pd.ut_n; base += MT_WAVE) {
            const int e = base + lane();
            if (e < pd.ut_n) {
                int pos;
                v4i a;
                u64 o;
                tab_get(pd, e, pos, a, o);
                const int dlt = vlen(pd.w, a, o, r, c) - obs_len(a);
                if (dlt && pos != wpos) atomicAdd((int *)(pd.cdl + (pos >> 6)), dlt);
            }
        }
        PG_T1(36)
        if (win) {
            const int dlt = pg_win_delta(pd, r, c);
            if (lane() == 0) pd.cdl[wpos >> 6] += dlt;
        }
        wsync<T>();
#ifndef MT_VIEWS_TOTAL
        if (!total) return 0;
#endif
        int tot = 0;
        for (int base = 0; base < nch; base += MT_WAVE) {
            const int ch = base + lane();
            tot += ch < nch ? pd.cob[ch] + pd.cdl[ch] : 0;
        }
        return wave_sum(tot);
    }
}
// First level-1 position whose cumulative view end is >= p (strict: > p); start = its
// view start.  -1 (start = total) if none.
TD int pg_find_impl(PagedDoc<T> &pd, int p, bool strict, int &start, int &ostart);
TD int pg_find(PagedDoc<T> &pd, int p, bool strict, int &start, int &ostart) {
    PG_T0(13)
    const int r_ = pg_find_impl(pd, p, strict, start, ostart);
    PG_T1(13)
    return r_;
}
// ... and ostart = its observer start.  The chunk first (cob + cdl), then the chunk's pages:
// their differences from the table entries at those positions (and the window), summed in the
// window's scratch.  Views are never negative here (a writer's view at its op's refSeq), so
// the cumulative lengths grow with the position and the page lies in the chunk found.
TD int pg_find_impl(PagedDoc<T> &pd, int p, bool strict, int &start, int &ostart) {
    DocT<T> &w = pd.w;
    const int np = nbr(pd.up, 1);
    if constexpr (!T::kHM) {   // pvl by position
        int carry = 0, ocarry = 0;
        int b0 = 0, b1 = np;
        if constexpr (T::kPP == 0 || T::kPP > 4 * MT_WAVE) {
            if (np > 4 * MT_WAVE) {
                // a long directory: each lane first sums a contiguous run of ceil(np / 64) pages
                // (plain adds), one pair of wave scans picks the run holding p, and only that run
                // is scanned page by page below
                const int chunk = (np + MT_WAVE - 1) / MT_WAVE;
                const int lo = min(lane() * chunk, np), hi = min(lo + chunk, np);
                int v = 0, ov = 0;
                for (int q = lo; q < hi; q++) {
                    v += pd.pvl[q];
                    ov += pm_obs(pd, pd.up.dir[q]);
                }
                const int inc = wave_scan_incl(v), oinc = wave_scan_incl(ov);
                const u64 m = ballot(hi > lo && (strict ? inc > p : inc >= p));
                if (!m) {
                    start = bcast(inc, MT_WAVE - 1);
                    ostart = bcast(oinc, MT_WAVE - 1);
                    return -1;
                }
                const int fl = first_lane(m);
                carry = bcast(inc - v, fl);
                ocarry = bcast(oinc - ov, fl);
                b0 = bcast(lo, fl);
                b1 = bcast(hi, fl);
            }
        }
        for (int base = b0; base < b1; base += MT_WAVE) {
            const int q = base + lane();
            int v = 0, ov = 0;
            if (q < b1) {
                v = pd.pvl[q];
                ov = pm_obs(pd, pd.up.dir[q]);
            }
            const int inc = wave_scan_incl(v);
            const int end = carry + inc;
            const u64 m = ballot(q < b1 && (strict ? end > p : end >= p));
            const int oinc = wave_scan_incl(ov);
            if (m) {
                const int fl = first_lane(m);
                start = bcast(end - v, fl);
                ostart = ocarry + bcast(oinc - ov, fl);
                return base + fl;
            }
            carry += bcast(inc, MT_WAVE - 1);
            ocarry += bcast(oinc, MT_WAVE - 1);
        }
        start = carry;
        ostart = ocarry;
        return -1;
    } else {   // chunks, then the chunk's pages
        const int nch = (np + 63) >> 6;
        int carry = 0, ocarry = 0, cf = -1;
        for (int base = 0; base < nch; base += MT_WAVE) {
            const int ch = base + lane();
            int v = 0, ov = 0;
            if (ch < nch) {
                ov = pd.cob[ch];
                v = ov + pd.cdl[ch];
            }
            const int inc = wave_scan_incl(v), oinc = wave_scan_incl(ov);
            const int end = carry + inc;
            const u64 m = ballot(ch < nch && (strict ? end > p : end >= p));
            if (m) {
                const int fl = first_lane(m);
                cf = base + fl;
                carry += bcast(inc - v, fl);
                ocarry += bcast(oinc - ov, fl);
                break;
            }
            carry += bcast(inc, MT_WAVE - 1);
            ocarry += bcast(oinc, MT_WAVE - 1);
        }
        if (cf < 0) {
            start = carry;
            ostart = ocarry;
            return -1;
        }
        // the chunk's pages: differences per position in w.scr (64 entries), kept for the
        // view's next search in the same chunk (boundary splits preserve them)
        const int key = cf | ((pd.vgen & 0x7FFF) << 16);
        if (pd.scr_ch != key) {
            const int r = pd.vr, c = pd.vc;
            w.scr[lane()] = 0;
            wsync<T>();
            const bool win = pd.cur >= 0 && pd.tdirty;
            const int wpos = win ? pg_cur_pos(pd) : -1;
            for (int base = 0; base < pd.ut_n; base += MT_WAVE) {
                const int e = base + lane();
                if (e < pd.ut_n) {
                    int pos;
                    v4i a;
                    u64 o;
                    tab_get(pd, e, pos, a, o);
                    if ((pos >> 6) == cf && pos != wpos) {
                        const int dlt = vlen(pd.w, a, o, r, c) - obs_len(a);
                        if (dlt) atomicAdd((int *)(w.scr + (pos & 63)), dlt);
                    }
                }
            }
            if (win && (wpos >> 6) == cf) {
                const int dlt = pg_win_delta(pd, r, c);
                if (lane() == 0) w.scr[wpos & 63] += dlt;
            }
            wsync<T>();
            pd.scr_ch = key;
        }
        const int q = (cf << 6) + lane();
        if (pd.sob_ch != cf) {   // the chunk's observer lengths from HBM, kept for its next search
            pd.sob[lane()] = q < np ? pm_obs(pd, pd.up.dir[q]) : 0;
            pd.sob_ch = cf;
            wsync<T>();
        }
        int v = 0, ov = 0;
        if (q < np) {
            ov = pd.sob[lane()];
            v = ov + w.scr[lane()];
        }
        const int inc = wave_scan_incl(v), oinc = wave_scan_incl(ov);
        const int end = carry + inc;
        const u64 m = ballot(q < np && (strict ? end > p : end >= p));
        if (!m) {   // (the chunk's sum and its pages' disagree: cannot happen)
            FAIL_INTERNAL(w);
            start = carry;
            ostart = ocarry;
            return -1;
        }
        const int fl = first_lane(m);
        start = carry + bcast(inc - v, fl);
        ostart = ocarry + bcast(oinc - ov, fl);
        return (cf << 6) + fl;
    }
}
// The length of level-1 position pos in the cached view (pg_views first).
TD int pg_page_view(PagedDoc<T> &pd, int pos) {
    if constexpr (!T::kHM) return uni(pd.pvl[pos]);
    const int pg = uni((int)pd.up.dir[pos]);
    const bool win = pd.cur >= 0 && pd.tdirty;
    const int wpos = win ? pg_cur_pos(pd) : -1;
    int d = 0;
    for (int base = 0; base < pd.ut_n; base += MT_WAVE) {
        const int e = base + lane();
        if (e < pd.ut_n) {
            int ep;
            v4i a;
            u64 o;
            tab_get(pd, e, ep, a, o);
            if (ep == pos && pos != wpos) d += vlen(pd.w, a, o, pd.vr, pd.vc) - obs_len(a);
        }
    }
    d = wave_sum(d);
    if (pos == wpos) d = pg_win_delta(pd, pd.vr, pd.vc);
    if ((pos >> 6) == pd.sob_ch) return uni(pd.sob[pos & 63]) + d;
    return uni(pm_obs(pd, pg)) + d;
}
// the window onto level-1 position pos, whose observer start is obs_base
// L2 warm-up of zamboni's page (the message's first pop, pd.zuid / zpv): one dword load per
// 128-byte line of its slots, lanes 0-7 / 8-15 / 16-19 -> A / B / O.  Issued between the op
// page's fetch and the flush: the place step waits for the fetch, and so (in-order vmcnt) for
// this load too, before `touch` dies -- its register is never reused while the load is out.
__device__ __forceinline__ int pg_touch_lines(const GLB_AS void *a, const GLB_AS void *b, const GLB_AS void *o) {
    const int l = lane();
    const GLB_AS char *p = l < 8 ? (const GLB_AS char *)a + 128 * l
                                 : (l < 16 ? (const GLB_AS char *)b + 128 * (l - 8)
                                           : (const GLB_AS char *)o + 128 * (l < 20 ? l - 16 : 0));
    int x;
    asm volatile("global_load_dword %0, %1, off" : "=v"(x) : "v"(p) : "memory");
    return x;
}
TD void pg_load_pos(PagedDoc<T> &pd, int pos, int obs_base) {
    const int pg = uni(pd.up.dir[pos]);
    if (pd.cur != pg) {
        PG_CNT(24)
#ifdef MT_ZPF
        v4i a = v4i{0, 0, 0, 0};
        u64 o = 0;
        v4u b = v4u{0, 0, 0, 0};
        pg_win_fetch(pd, pg, a, o, b);
        int touch = 0;
        const int zp = pd.zuid ? uni(pd.zpv) : -1;
        if (pd.zuid) pd.zpv = zp;   // uniform from here on
        if (zp >= 0 && zp != pg && zp < pd.PP)
            touch = pg_touch_lines(pd.gA + (size_t)zp * MT_PG_SLOTS, pd.gB + (size_t)zp * MT_PG_SLOTS,
                                   pd.gO + (size_t)zp * MT_PG_SLOTS);
        uint32_t bc = 0, f2 = 0;
        int ob = 0;
        pg_win_fetch_blocks(pd, pg, bc, f2, ob);
        pg_win_flush(pd);
        if (pd.w.status) return;
        pg_win_place(pd, pg, a, o, b, bc, f2, ob);
        asm volatile("" ::"v"(touch));
#else
        pg_win_switch(pd, pg);
#endif
    }
    pd.cur_pos = pos;
    pd.w.obs_base = obs_base;
}

// ------------------------------------------------------------------ pack at level 1
// pack :1401-1453 for the underflowing page at level-1 position pos: the leaf blocks of
// every child of its parent are regrouped into max(1, min(7, n/4)) pages (copied in HBM
// into fresh pages); then the parent may underflow in turn (counts only above level 1).
TD void pg_pack1_impl(PagedDoc<T> &pd, int pos);
TD void pg_pack1(PagedDoc<T> &pd, int pos) {
    PG_T0(14)
    pg_pack1_impl(pd, pos);
    PG_T1(14)
}
TD void pg_pack1_impl(PagedDoc<T> &pd, int pos) {
    DocT<T> &w = pd.w;
    DocT<T> &up = pd.up;
    pg_win_flush(pd);
    pd.cur = -1;
    pd.zuid = 0;   // (zamboni's prefetched page may be one of the repacked ones)
    int c0;
    const int P = blk_find(up, 2, pos, true, c0);
    if (P < 0) {
        FAIL_INTERNAL(w);
        return;
    }
    const int nch = cntr(up, 2, P);
    int TB = 0, TS = 0;
    for (int j = 0; j < nch; j++) {
        TB += cntr(up, 1, c0 + j);
        TS += uni(pm_nseg(pd, up.dir[c0 + j]));
    }
    int k = TB / MT_HALF;
    if (k > MT_MAXN - 1) k = MT_MAXN - 1;
    if (k < 1) k = 1;
    const int base = TB / k, extra = TB % k;
    if (nbr(up, 1) + k > pd.PP) {   // the new pages are taken before the old ones are freed
        pg_fail_cap(w, 7);
        return;
    }
    // per lane: one leaf block of the concatenation (TB <= 49): its old page / index
    if constexpr (T::kHM) {   // the block words lane 0 wrote to HBM are read by every lane
        gsync();
        gsync_rd();
    }
    const int bl = lane();
    int opg = -1, ob = 0, bseg0 = 0;   // old page, block index in it, first segment (concat)
    uint32_t obc = 0, of2 = 0;         // its block words
    {
        int acc_b = 0, acc_s = 0;
        for (int j = 0; j < nch; j++) {
            const int pg = uni(up.dir[c0 + j]);
            const int nb = uni(pm_nblk(pd, pg));
            if (bl >= acc_b && bl < acc_b + nb) {
                opg = pg;
                ob = bl - acc_b;
                pm_blocks(pd, pg, obc, of2);
                int s = acc_s;
                for (int q = 0; q < ob; q++) s += pm_bc_of(obc, q);
                bseg0 = s;
            }
            acc_b += nb;
            acc_s += uni(pm_nseg(pd, pg));
        }
    }
    const int bcnt = opg >= 0 ? pm_bc_of(obc, ob) : 0;
    const int8_t bflg = opg >= 0 ? pm_fl_of(of2, ob) : (int8_t)0;
    // new page m gets blocks [nb0(m), nb0(m) + base + (m < extra))
    auto nb0 = [&](int m) { return m * base + min(m, extra); };
    LDS_AS int32_t *newp = w.scr;   // scratch: the new page ids
    for (int m = 0; m < k; m++) {
        const int pg = pg_alloc(pd);
        if (pg < 0) {
            pg_fail_cap(w, 7);
            return;
        }
        if (lane() == 0) newp[m] = pg;
    }
    wsync<T>();
    // table entries of the old pages go (and the later positions move by k - nch); the copy
    // pass re-adds the unsettled ones at the new pages' positions c0 .. c0 + k - 1
    for (int j = 0; j < nch; j++) pg_table_purge(pd, c0 + j);
    if (k != nch) pg_table_shift(pd, c0 + nch, k - nch);
    // copy, one new page at a time (<= 7 * 8 segments each)
    for (int m = 0; m < k; m++) {
        const int npg = uni(newp[m]);
        const int blo = nb0(m), bhi = nb0(m + 1);
        const int s_lo = bcast(bseg0, blo);
        const int s_hi = bhi < TB ? bcast(bseg0, bhi) : TS;
        const int t = lane();
        const int g = s_lo + t;
        int ol = 0;
        bool add = false;
        v4i a = v4i{0, 0, MT_RSEQ_NONE, 0};
        u64 o = 0;
        if (g < s_hi) {
            // source: old page j and slot
            int acc = 0, spg = 0, slot = 0;
            for (int j = 0; j < nch; j++) {
                const int pg = uni(up.dir[c0 + j]);
                const int ns = uni(pm_nseg(pd, pg));
                if (g >= acc && g < acc + ns) {
                    spg = pg;
                    slot = g - acc;
                }
                acc += ns;
            }
            a = pd.gA[(size_t)spg * MT_PG_SLOTS + slot];
            o = pd.gO[(size_t)spg * MT_PG_SLOTS + slot];
            const v4u b = pd.gB[(size_t)spg * MT_PG_SLOTS + slot];
            pd.gA[(size_t)npg * MT_PG_SLOTS + t] = a;
            pd.gO[(size_t)npg * MT_PG_SLOTS + t] = o;
            pd.gB[(size_t)npg * MT_PG_SLOTS + t] = b;
            const uint32_t uid = b.z & ~MT_MARKER_BIT;
            if (uid < (uint32_t)pd.UM) pd.gumap[uid] = (uint16_t)npg;
            ol = obs_len(a);
            add = unsettled<T>(a, w.min_seq);
        }
        const u64 am = ballot(add);
        if (pd.ut_n + __popcll(am) > pd.UT) {
            pg_fail_cap(w, 8);
            return;
        }
        const int mi = tab_midx(pd, add && o != 0);
        if (mi < 0) {
            pg_fail_cap(w, 8);
            return;
        }
        if (add) tab_put(pd, pd.ut_n + __popcll(am & ((1ull << lane()) - 1ull)), c0 + m, a, o, mi);
        pd.ut_n += __popcll(am);
        const int obs = wave_sum(ol);
        // meta of the new page: blocks blo..bhi of the concatenation
        const bool vb = lane() >= blo && lane() < bhi;
        pm_set_blocks(pd, npg, lane() - blo, vb, bcnt, bflg);
        if (lane() == 0) {
            pm_set_ns(pd, npg, s_hi - s_lo, bhi - blo);
            pm_set_obs(pd, npg, obs);
        }
        wsync<T>();
    }
    // free the old pages (their meta marks them empty)
    for (int j = 0; j < nch; j++) {
        const int pg = uni(up.dir[c0 + j]);
        if (lane() == 0) pm_set_ns(pd, pg, 0, 0);
        wsync<T>();
    }
    // level 1: nch entries -> k entries of base (+1) blocks; then the page ids
    blk_replace(up, 1, c0, nch, k, base, extra);
    if (up.status) {
        pg_fail_cap(w, 7);
        return;
    }
    for (int m = 0; m < k; m++)
        if (lane() == 0) up.dir[c0 + m] = (uint16_t)newp[m];
    if (lane() == 0) lvl(up, 2)[P] = (uint8_t)k;
    wsync<T>();
    pg_cob_rebuild(pd);
    int top_l = 2, top_b = P;
    if (k < MT_HALF && 3 < up.depth) pack_counts(up, 2, P, top_l, top_b);   // counts only above level 1
    if (up.status) {
        if (w.status == 0) w.cap_cause = up.cap_cause;
        fail(w, MT_DOC_INTERNAL);
        return;
    }
    if (ordon(w)) ord_canon(up, top_l, top_b);   // nodeUpdateOrdinals(the topmost parent) :1449-1450
}

// ------------------------------------------------------------------ zamboni (paged)
// zamboniSegments :1455-1511 with the heap in LDS and the uid -> page map in HBM.
TD void pg_zamboni_impl(PagedDoc<T> &pd);
TD void pg_zamboni(PagedDoc<T> &pd) {
    PG_T0(12)
    pg_zamboni_impl(pd);
    PG_T1(12)
}
TD void pg_zamboni_impl(PagedDoc<T> &pd) {
    DocT<T> &w = pd.w;
    pd.vvalid = 0;
    for (int it = 0; it < MT_ZAMBONI && w.status == 0; it++) {
        if (w.heap_n == 0) break;
        const v2i top = heap_top(w);
        if (top.x > w.min_seq) break;
        const uint32_t uid = (uint32_t)top.y;
        if (uid >= (uint32_t)pd.UM) {   // ids stay below the map size (pg_renumber)
            FAIL_INTERNAL(w);
            return;
        }
        // the segment's page from the uid map: issued before the heap pop so that its
        // latency hides behind it; needed only if the segment is not in the window (the
        // message's first pop: loaded at the message's start)
#ifdef MT_ZPF
        const int gpg = uid == (uint32_t)pd.zuid ? pd.zpv : (int)pd.gumap[uid];
        pd.zuid = 0;
#else
        const int gpg = pd.gumap[uid];
#endif
        PG_T0(5)
        heap_pop(w);
        wsync<T>();
        PG_T1(5)
        PG_CNT(16)
        PG_T0(4)
        if (uid == 0) {   // its segment was merged or unlinked before a renumbering
            PG_CNT(17)
            continue;
        }
        // the window first (its uid map entries are written when it is flushed)
        int i = pd.cur >= 0 ? find_uid(w, uid) : -1;
        if (i < 0) {
            const int pg = uni(gpg);
            if constexpr (T::kHM) {   // the page's count arrives with its rows: an empty page is
                                      // skipped before the window moves
                if (pg == pd.cur || pg >= pd.PP) {
                    PG_CNT(19)
                    continue;
                }
                v4i a = v4i{0, 0, 0, 0};
                u64 o = 0;
                v4u b = v4u{0, 0, 0, 0};
                uint32_t bc = 0, f2 = 0;
                int ob = 0;
                pg_win_fetch(pd, pg, a, o, b);
                pg_win_fetch_blocks(pd, pg, bc, f2, ob);
                if ((((uint32_t)bcast((int)f2, 0)) >> 24) == 0) {
                    PG_CNT(19)
                    continue;
                }
                PG_CNT(18)
                pg_win_flush(pd);
                if (w.status) return;
                pg_win_place(pd, pg, a, o, b, bc, f2, ob);
            } else {
                if (pg == pd.cur || pg >= pd.PP || uni(pm_nseg(pd, pg)) == 0) {
                    PG_CNT(19)
                    continue;
                }
                PG_CNT(18)
                pg_win_switch(pd, pg);
                if (w.status) return;
            }
            i = find_uid(w, uid);
            if (i < 0) {
                PG_CNT(19)
                continue;
            }
        }
        PG_T1(4)
        int bstart;
        const int b = blk_find(w, 0, i, true, bstart);
        if (b < 0) {
            FAIL_INTERNAL(w);
            return;
        }
        const int f = flgr(w, b);
        const int old = cntr(w, 0, b);
        if (f == 0) {
            PG_CNT(20)
            continue;
        }
        PG_CNT(21)
        if (ordon(w) && w.rich) w.obs_base = pg_obs_start(pd);   // scour event positions
        PG_T0(2)
        const int kept = scour_range(w, bstart, b, 1);
        PG_T1(2)
        if (w.status) return;
        wsync<T>();
        if (lane() == 0) w.flg[b] = 0;
        wsync<T>();
        bool pk = false;
        if (kept < old && kept < MT_HALF && w.depth > 1) {
            pack(w, 0, b);   // regroups this page's leaf blocks (stops at the window top)
            if (w.status) return;
            pk = nbr(w, 0) < MT_HALF && pd.up.depth > 2;
        } else if (kept < old && ordon(w)) {
            ord_canon(w, 0, b);   // nodeUpdateOrdinals(block) :1500-1501
        }
        pg_win_sync(pd);
        if (w.status) return;
        if (pk) {
            PG_CNT(22)
            pg_pack1(pd, pg_cur_pos(pd));
            if (w.status) return;
        }
    }
}

// ------------------------------------------------------------------ ops (paged)
TD void pg_boundary(PagedDoc<T> &pd, int p, int r, int c);
TD void pg_log_deferred(PagedDoc<T> &pd);
TD void pg_op_insert(PagedDoc<T> &pd, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin) {
    DocT<T> &w = pd.w;
    const mt_op_rec &op = in.op;
    const int slen = (op.flags & MT_F_MARKER) ? 1 : op.pos2;
    if (ordon(w)) {
        // insertSegments splits at the position in a walk of its own first
        // (ensureIntervalBoundary, MT/mergeTree.ts:2004): a page split it causes re-derives
        // ordinals before the new segment takes its character
        pg_boundary(pd, op.pos1, op.ref_seq, op_cli(op));
        if (w.status) return;
    }
    pg_views_cached(pd, op.ref_seq, op_cli(op));
    int start;
    int ostart;
    int pos = pg_find(pd, op.pos1, false, start, ostart);
    if constexpr (T::kLog) {
        // a zero-length insert past the end logs its (never linked) segment like the flat
        // engine: the last page's window runs it
        const int np = nbr(pd.up, 1);
        if (pos < 0 && slen == 0 && np > 0 && !(op.flags & MT_F_LOAD)) {
            pos = np - 1;
            const int lp = uni((int)pd.up.dir[pos]);
            start -= pg_page_view(pd, pos);
            ostart -= uni(pm_obs(pd, lp));
        }
    }
    if (pos < 0) {
        if (slen == 0) {   // boundary only; nothing splits past the end
            if (op.flags & MT_F_LOAD) return;
            Cb cb = cb_begin(w, op.seq, MT_OP_INSERT);
            cb.n = 1;
            cb_log(w, -1);
            cb_log(w, 0);
            cb.h = fnv_u64(cb.h, fnv_u32(fnv_u32(MT_FNV_OFF, (uint32_t)-1), 0u));
            cb_end(w, cb);
            return;
        }
        fail(w, MT_DOC_INSERT_FAILED);
        return;
    }
    pg_load_pos(pd, pos, ostart);
    if (w.status) return;
    OpIn rel = in;
    rel.op.pos1 = op.pos1 - start;
    pd.vvalid = 0;
    pd.tdirty = 1;
    op_insert(w, rel, tin, pin);
    if (w.status) return;
    pg_win_sync(pd);
    if (T::kLog && w.dfr_rec >= 0) pg_log_deferred(pd);
}

TD void pg_boundary(PagedDoc<T> &pd, int p, int r, int c) {
    pg_views_cached(pd, r, c);
    int start;
    int ostart;
    const int pos = pg_find(pd, p, true, start, ostart);
    if (pos < 0 || start >= p) return;   // p is at a page boundary or past the end
    pg_load_pos(pd, pos, ostart);
    if (pd.w.status) return;
    pd.tdirty = 1;
    boundary(pd.w, p - start, r, c);
    if (pd.w.status) return;
    pg_win_sync(pd);
}

TD void pg_op_range(PagedDoc<T> &pd, const mt_op_rec &op, const GLB_AS uint32_t *pin) {
    DocT<T> &w = pd.w;
    const int r = op.ref_seq, c = op_cli(op), p1 = op.pos1, p2 = op.pos2;
    const bool rem = op.kind == MT_OP_REMOVE;
    const GLB_AS uint32_t *rec = (!rem && op.props != MT_NO_PROPS) ? pin + op.props : nullptr;
    if (rec && (rec[0] >> 16) == MT_COMBINE_OTHER) {
        fail(w, MT_DOC_UNSUPPORTED);
        return;
    }
    if (!rec) rec = (const GLB_AS uint32_t *)&kEmptyPropsRec;
    pg_boundary(pd, p1, r, c);
    if (w.status) return;
    pg_boundary(pd, p2, r, c);
    if (w.status) return;
    Cb cb = cb_begin(w, op.seq, op.kind);
    pg_views_cached(pd, r, c);
    pd.vvalid = 0;   // range_mark changes view lengths
    int start;
    int ostart;
    int pos = pg_find(pd, p1, true, start, ostart);
    if (pos >= 0) {
        int carry = start, ocarry = ostart;
        const int np = nbr(pd.up, 1);
        while (pos < np && carry < p2) {
            pg_load_pos(pd, pos, ocarry);
            if (w.status) return;
            pd.tdirty = 1;
            const bool done = range_mark(w, op, rec, carry, ocarry, cb);
            if (w.status) return;
            pg_win_sync(pd);
            if (w.status) return;
            if (done) break;
            pos = pg_cur_pos(pd) + 1;
        }
    }
    cb_end(w, cb);
}

// ------------------------------------------------------------------ segment ids
// Renumbers the document's segment ids densely in document order.  Every split and insert
// creates an id, so a long-lived document creates far more ids than it ever holds; the
// uid -> page map (zamboni's only way to find a segment's page) has pd.UM entries, and ids are
// compacted when they run out.  Zamboni heap entries follow their segments; an entry whose
// segment is gone (merged or unlinked: the reference skips it, its parent is undefined)
// gets id 0, which matches nothing.  Runs between messages, from the pages in HBM.
TD void pg_renumber(PagedDoc<T> &pd, bool soft = false) {
    DocT<T> &w = pd.w;
    pg_win_flush(pd);
    if (w.status) return;
    pd.cur = -1;
    pd.cur_pos = -1;
    pd.vvalid = 0;
    gsync();
    const int np = nbr(pd.up, 1);
    // first new id of every page (segments before it + 1), by page id, in the text arena's
    // idle half (scratch: only a compaction writes it, and none runs here)
    if (2 * pd.PP > w.T_cap) {
        pg_fail_cap(w, 4);
        return;
    }
    GLB_AS int32_t *first = (GLB_AS int32_t *)text_base(w, 1 - w.text_half);
    int carry = 1;
    for (int base = 0; base < np; base += MT_WAVE) {
        const int q = base + lane();
        const int pg = q < np ? (int)pd.up.dir[q] : 0;
        const int ns = q < np ? pm_nseg(pd, pg) : 0;
        const int inc = wave_scan_incl(ns);
        if (q < np) first[pg] = carry + inc - ns;
        carry += bcast(inc, MT_WAVE - 1);
    }
    gsync();
    gsync_rd();
    // heap entries: old id -> page (map) -> slot -> new id.  Ids at or above the map size
    // (a document converted from the flat tiers after many creations) are searched for.
    const int i = lane();
    for (int e = 1; e <= w.heap_n; e++) {
        const uint32_t uid = (uint32_t)uni(w.heap[e].y);
        int nid = 0;
        if (uid != 0) {
            const int mp = uid < (uint32_t)pd.UM ? uni((int)pd.gumap[uid]) : -1;
            for (int q = (mp >= 0 ? -1 : 0); q < (mp >= 0 ? 0 : np); q++) {
                const int pg = q < 0 ? mp : uni((int)pd.up.dir[q]);
                if (pg >= pd.PP) continue;
                const int ns = uni(pm_nseg(pd, pg));
                const bool hit = i < ns && (pd.gB[(size_t)pg * MT_PG_SLOTS + i].z & ~MT_MARKER_BIT) == uid;
                const u64 m = ballot(hit);
                if (m) {
                    nid = uni((int)first[pg]) + first_lane(m);
                    break;
                }
            }
        }
        if (lane() == 0) w.heap[e].y = nid;
    }
    // every slot gets its new id; the map follows
    for (int q = 0; q < np; q++) {
        const int pg = uni((int)pd.up.dir[q]);
        const int ns = uni(pm_nseg(pd, pg));
        if (i < ns) {
            GLB_AS v4u *b = pd.gB + (size_t)pg * MT_PG_SLOTS + i;
            const uint32_t nid = (uint32_t)(uni((int)first[pg]) + i);
            v4u bv = *b;
            bv.z = nid | (bv.z & MT_MARKER_BIT);
            *b = bv;
            if (nid < (uint32_t)pd.UM) pd.gumap[nid] = (uint16_t)pg;
        }
    }
    w.next_uid = carry;
    // more live segments than map entries (soft: the caller hands the document to the growth step)
    if (w.next_uid + 8 > pd.UM && !soft) pg_fail_cap(w, 9);
    gsync();
    wsync<T>();
}

// Tight paged tier: can this message be applied without outgrowing the launch's LDS
// capacities?  Bounds per message: the unsettled table grows by <= 3 for an insert (the two
// halves of a split unsettled segment and the new one) and by <= 2 + (pos2 - pos1) for a
// range op (two splits and the marked segments: only segments of positive view length are
// marked); the heap by <= 1 / <= 1 + (pos2 - pos1) (one entry per touched leaf block); a
// message splits or repacks a few pages (8 kept in reserve).  pd.wgrow bounds what the
// window added since its table entries were last rebuilt.
TD bool pg_room(PagedDoc<T> &pd, const mt_op_rec &op) {
    const bool range = op.kind == MT_OP_REMOVE || op.kind == MT_OP_ANNOTATE;
    const int span = range ? min(max(op.pos2 - op.pos1, 0), 1 << 20) : 0;
    const int ut_b = op.kind == MT_OP_INSERT ? 3 : (range ? 2 + span : (op.kind == MT_OP_LOAD_REMOVED ? 1 : 0));
    const int hp_b = op.kind == MT_OP_INSERT ? 1 : (range ? 1 + span : 0);
    // a narrow tier holds overlap slots 1..32 only
    if (T::kOvlBits < 64 && op.kind == MT_OP_REMOVE && oslot_short(pd.w, op_cli(op))) return false;
    if (T::kPacked && op.seq - pd.sbase > 65000) return false;   // the packed table's seq offsets
    if (pd.ut_n + pd.wgrow + ut_b > pd.UT) return false;
    if constexpr (T::kPacked) {
        // the sparse mask table: every entry this message (and the window's rebuild) may add
        // could carry a mask; a shortage hands the document on here instead of failing a
        // table add mid-message (a collection runs only when the bound is not met outright)
        const int need = pd.wgrow + ut_b;
        if (tab_mfree(pd) < need) {
            tab_mgc(pd);
            if (tab_mfree(pd) < need) return false;
        }
    }
    if (pd.w.heap_n + hp_b > pd.PH) return false;
    if (nbr(pd.up, 1) + 8 > pd.PP) return false;
    for (int l = 2; l < pd.up.depth; l++)
        if (nbr(pd.up, l) + 4 > bcap(pd.up, l)) return false;
    pd.opbound = ut_b;
    pd.wgrow += ut_b;
    return true;
}
// Client.applyMsg (MT/client.ts:797-819) for a paged document; mirrors apply_op.
TD void pg_apply_op_impl(PagedDoc<T> &pd, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin);
TD void pg_apply_op(PagedDoc<T> &pd, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin) {
    PG_T0(15)
    pg_apply_op_impl(pd, in, tin, pin);
    PG_T1(15)
}
// load_removed for a paged document: the appended segment is in the window, or (after a
// page split) in the page the uid map names.
TD void pg_load_removed(PagedDoc<T> &pd, const mt_op_rec &op) {
    DocT<T> &w = pd.w;
    pd.vvalid = 0;
    const uint32_t uid = (uint32_t)(w.next_uid - 1);
    int i = pd.cur >= 0 ? find_uid(w, uid) : -1;
    if (i < 0) {
        const int pg = uid < (uint32_t)pd.UM ? uni(pd.gumap[uid]) : -1;
        if (pg < 0 || pg >= pd.PP) {
            FAIL_INTERNAL(w);
            return;
        }
        pg_win_switch(pd, pg);
        if (w.status) return;
        i = find_uid(w, uid);
        if (i < 0) {
            FAIL_INTERNAL(w);
            return;
        }
    }
    pd.tdirty = 1;
    load_removed(w, op);
    if (w.status) return;
    pg_win_sync(pd);
}

TD void pg_apply_op_impl(PagedDoc<T> &pd, const OpIn &in, const GLB_AS uint16_t *tin, const GLB_AS uint32_t *pin) {
    DocT<T> &w = pd.w;
    const mt_op_rec &op = in.op;
    w.ocs = oslot_of(w, op_cli(op));
    // a message creates <= 3 ids (load_removed finds the id its insert just created)
    if (w.next_uid + 4 > pd.UM && op.kind != MT_OP_LOAD_REMOVED) {
        pg_renumber(pd);
        if (w.status) return;
    }
#ifdef MT_ZPF
    {   // zamboni's first pop of this message and its page (the op adds entries above minSeq only)
        pd.zuid = 0;
        if (w.heap_n > 0 && op.kind != MT_OP_NOOP) {
            const v2i top = heap_top(w);
            if (top.x <= max(w.min_seq, op.min_seq) && top.y > 0 && top.y < pd.UM) {
                pd.zuid = top.y;
                pd.zpv = pd.gumap[top.y];
            }
        }
    }
#endif
    if (op.flags & MT_F_LOAD) {   // summary body append (apply_op); no events
        const int rich = w.rich;
        w.rich = 0;
        if (op.kind == MT_OP_INSERT)
            pg_op_insert(pd, in, tin, pin);
        else if (op.kind == MT_OP_LOAD_REMOVED)
            pg_load_removed(pd, op);
        else if (op.kind == MT_OP_LOAD_ALIASED)
            fail(w, MT_DOC_ALIASED);
        w.rich = rich;
        return;
    }
    const bool is_op = op.kind == MT_OP_INSERT || op.kind == MT_OP_REMOVE || op.kind == MT_OP_ANNOTATE;
    if (op.kind == MT_OP_INSERT) {
        pg_op_insert(pd, in, tin, pin);
    } else if (is_op) {
        pg_op_range(pd, op, pin);
    }
    if (w.status) return;
    bool z = is_op;
    for (int pass = 0; pass < 2; pass++) {
        if (z) {
            pg_zamboni(pd);
            if (w.status) return;
        }
        if (pass == 1) break;
        if (op.kind != MT_OP_NOOP) {
            if (!(w.cur_seq < op.seq)) {
                fail(w, MT_DOC_SEQ_ORDER);
                return;
            }
            if (!(w.min_seq <= op.min_seq)) {
                fail(w, MT_DOC_MINSEQ_ORDER);
                return;
            }
        }
        z = false;
        if (!(op.flags & MT_F_GROUP_MORE)) {
            if (!(w.cur_seq <= op.seq)) {   // updateSeqNumbers MT/client.ts:824
                fail(w, MT_DOC_SEQ_BACKWARDS);
                return;
            }
            w.cur_seq = op.seq;
            if (!(op.min_seq <= op.seq)) {    // MT/client.ts:826
                fail(w, MT_DOC_MSN_ABOVE_SEQ);
                return;
            }
            if (!(w.min_seq <= op.min_seq)) {   // setMinSeq MT/mergeTree.ts:1755
                fail(w, MT_DOC_MSN_BACKWARDS);
                return;
            }
            if (op.min_seq > w.min_seq) {
                w.min_seq = op.min_seq;
                z = true;
            }
        }
        if (!z) break;
    }
}

// ------------------------------------------------------------------ text / props gc (paged)
// Compacts the live text of every page into the other arena half, page by page.
TD void paged_text_compact(DocT<T> &w) {
    PagedDoc<T> &pd = pdoc(w);
    const int keep = pd.cur, keep_pos = pd.cur_pos, keep_td = pd.tdirty;
    if (keep >= 0) pd.dirty = 1;   // a scour may have updated flags in the window since its sync
    pg_win_flush(pd);
    if (w.status) return;
    gsync_rd();
    const int dh = 1 - w.text_half;
    GLB_AS uint16_t *dst = text_base(w, dh);
    const GLB_AS uint16_t *src = text_base(w, w.text_half);
    int carry = 0;
    const int np = nbr(pd.up, 1);
    for (int q = 0; q < np; q++) {
        pg_win_load(pd, uni(pd.up.dir[q]));
        const int i = lane();
        const bool v = i < w.n;
        v4i a = v4i{0, 0, 0, 0};
        v4u b = v4u{0, 0, 0, 0};
        if (v) {
            a = w.A[i];
            b = w.Bv[i];
        }
        const bool live = v && (a.z == MT_RSEQ_NONE || (T::kLog && w.rich)) && !(b.z & MT_MARKER_BIT);
        const int len = live ? a.x : 0;
        const int inc = wave_scan_incl(len);
        const int off = carry + inc - len;
        u64 m = ballot(live && len > 0);
        while (m) {
            const int j = first_lane(m);
            m &= m - 1;
            copy_text<T>(dst + bcast(off, j), src + bcast((int)b.x, j), bcast(len, j));
        }
        wsync<T>();
        if (live) {
            v4u nb = b;
            nb.x = (uint32_t)off;
            nb.w &= 0xFFFFu;
            w.Bv[i] = nb;
        }
        carry += bcast(inc, MT_WAVE - 1);
        wsync<T>();
        pg_write_page(pd, pd.cur, 0, w.n, 0, nbr(w, 0));
    }
    w.text_half = dh;
    w.text_top = carry;
    pd.cur = -1;
    if (keep >= 0) {   // the step that asked for room goes on in the same page
        pg_win_load(pd, keep);
        pd.cur_pos = keep_pos;
        pd.tdirty = keep_td;
    }
}
TD bool paged_text_ensure(DocT<T> &w, int need) {
    paged_text_compact(w);
    if (w.status) return false;
    if (8 * (w.text_top + need) > 7 * w.T_cap) pdoc(w).press = 4;
    if (w.text_top + need <= w.T_cap) return true;
    pg_fail_cap(w, 4);
    return false;
}

TD void paged_props_compact(DocT<T> &w) {
    PagedDoc<T> &pd = pdoc(w);
    const int keep = pd.cur, keep_pos = pd.cur_pos, keep_td = pd.tdirty;
    if (keep >= 0) pd.dirty = 1;   // a scour may have updated flags in the window since its sync
    pg_win_flush(pd);
    if (w.status) return;
    gsync_rd();
    const int dh = 1 - w.props_half;
    int carry = 1;
    const int np = nbr(pd.up, 1);
    for (int q = 0; q < np; q++) {
        pg_win_load(pd, uni(pd.up.dir[q]));
        const int i = lane();
        const uint32_t h = i < w.n ? w.Bv[i].y : 0;
        const int has = h != 0;
        const int inc = wave_scan_incl(has);
        const uint32_t nh = (uint32_t)(carry + inc - has);
        if (has) {
            const GLB_AS uint32_t *s = prec(w, w.props_half, h);
            GLB_AS uint32_t *t = prec(w, dh, nh);
            const uint32_t n = s[0];
            t[0] = n;
            for (uint32_t k = 0; k < 2 * n; k++) t[1 + k] = s[1 + k];
        }
        wsync<T>();
        if (has) w.Bv[i].y = nh;
        carry += bcast(inc, MT_WAVE - 1);
        wsync<T>();
        pg_write_page(pd, pd.cur, 0, w.n, 0, nbr(w, 0));
    }
    w.props_half = dh;
    w.props_top = carry;
    pd.cur = -1;
    gsync_rd();
    if (keep >= 0) {   // the step that asked for room goes on in the same page
        pg_win_load(pd, keep);
        pd.cur_pos = keep_pos;
        pd.tdirty = keep_td;
    }
}
TD bool paged_props_ensure(DocT<T> &w, int need) {
    paged_props_compact(w);
    if (w.status) return false;
    if (8 * (w.props_top + need) > 7 * w.P_cap) pdoc(w).press = 5;
    if (w.props_top + need <= w.P_cap) return true;
    pg_fail_cap(w, 5);
    return false;
}

// ------------------------------------------------------------------ overflow overlap sets
// removedClientOverlap beyond the 63 slots (MT/mergeTree.ts:2577-2585, read at :1717): a
// segment's mask MT_OVF_BIT | off points at [n, client...] in the document's overflow arena.
// Sets are written once; a segment that gains a client gets a new set (copy + the client), so
// the halves of a split share theirs.  vlen reads a set only for a removal the view has not
// seen; the sets of settled segments stay for their rows (mt_get_segments: n_overlap).
TD bool ovf_member(DocT<T> &d, u64 o, int c) {
    PagedDoc<T> &pd = pdoc(d);
    const GLB_AS uint16_t *s = pd.govf + (uint32_t)o;
    const int n = s[0];
    bool in = false;
    for (int k = 1; k <= n; k++) in = in || s[k] == (uint16_t)c;
    return in;
}
// The arena is used in two halves of one size, [MT_OVF_HDR, mid) and [mid, 2 mid - MT_OVF_HDR)
// (mt_ovf_mid): sets are appended in
// one, and a compaction (pg_ovf_compact) copies the live ones -- those a segment row still
// names -- into the other, as the text arena's halves are compacted.  Masks hold offsets from
// the arena's start, so a set is read the same wherever it lies.
TD int ovf_half_lo(const PagedDoc<T> &pd, int half) { return half ? mt_ovf_mid(pd.OA) : MT_OVF_HDR; }
TD int ovf_half_hi(const PagedDoc<T> &pd, int half) {
    return half ? 2 * mt_ovf_mid(pd.OA) - MT_OVF_HDR : mt_ovf_mid(pd.OA);
}
TD int ovf_half_end(const PagedDoc<T> &pd) { return ovf_half_hi(pd, pd.ovf_half); }
// Adds client c to the overlap list of the window's segment i (lanes with need; wave-uniform
// call): its overflow set, or the clients of its slot bits, copied with c into a new set.
// false: the arena is full (the caller fails the document, diagnostic 11).
TD bool ovf_mark(DocT<T> &d, bool need, int i, u64 o, int c, int seq) {
    PagedDoc<T> &pd = pdoc(d);
    const bool isset = (o & MT_OVF_BIT) != 0;
    const int n_old = !need ? 0 : (isset ? (int)pd.govf[(uint32_t)o] : __popcll(o));
    const int sz = need ? n_old + 2 : 0;
    const int inc = wave_scan_incl(sz);
    const int tot = bcast(inc, MT_WAVE - 1), top = pd.ovf_top;
    if (!pd.govf || top + tot > ovf_half_end(pd)) return false;
    pd.ovf_maxn = max(pd.ovf_maxn, wave_max(need ? n_old + 1 : 0));
    if (need) {
        const int off = top + inc - sz;
        GLB_AS uint16_t *t = pd.govf + off;
        t[0] = (uint16_t)(n_old + 1);
        if (isset) {
            const GLB_AS uint16_t *s = pd.govf + (uint32_t)o;
            for (int k = 1; k <= n_old; k++) t[k] = s[k];
        } else {
            u64 m = o;
            for (int k = 1; m; k++) {
                const int b = __ffsll((long long)m) - 1;
                m &= m - 1;
                t[k] = (uint16_t)d.oslot[2 * b];   // slot b + 1's client (unsettled: not reused)
            }
        }
        t[n_old + 1] = (uint16_t)c;
        d.O[i] = (typename T::O_v)(MT_OVF_BIT | (u64)(uint32_t)off);
    }
    pd.ovf_top = top + tot;
    pd.ovf_peak = max(pd.ovf_peak, pd.ovf_top - ovf_half_lo(pd, pd.ovf_half));
    pd.ovf_made = (uint32_t)min((u64)pd.ovf_made + (u64)tot, (u64)0xFFFFFFFFu);
    pd.ovf_last = seq;
    d.wide = 1;
    gsync_rd();   // the new sets are read by other lanes
    return true;
}

// Reclaims the overflow sets no segment names any more (removedClientOverlap lists go with
// their segments: the reference drops them when zamboni unlinks or merges the segment,
// MT/mergeTree.ts:1322-1398): every page's sets are copied into the other half of the arena,
// each row's mask re-pointed, and the pages' unsettled-table entries (which copy the masks)
// rebuilt.  Runs between messages, page by page from HBM, like paged_text_compact.
TD void pg_ovf_compact(PagedDoc<T> &pd) {
    DocT<T> &w = pd.w;
    const int keep = pd.cur, keep_pos = pd.cur_pos;
    if (keep >= 0) pd.dirty = 1;
    pg_win_flush(pd);
    if (w.status) return;
    gsync_rd();
    const int nh = 1 - pd.ovf_half;
    const int lo = ovf_half_lo(pd, nh), hi = ovf_half_hi(pd, nh);
    int top = lo;
    const int np = nbr(pd.up, 1);
    for (int q = 0; q < np; q++) {
        pg_win_load(pd, uni(pd.up.dir[q]));
        const int i = lane();
        const u64 o = i < w.n ? (u64)w.O[i] : 0ull;
        const bool isset = (o & MT_OVF_BIT) != 0;
        const int n = isset ? (int)pd.govf[(uint32_t)o] : 0;
        const int sz = isset ? n + 1 : 0;
        const int inc = wave_scan_incl(sz);
        const int tot = bcast(inc, MT_WAVE - 1);
        if (!ballot(isset)) continue;
        if (top + tot > hi) {   // (cannot happen: the live sets fit the half they came from, of the same size)
            FAIL_INTERNAL(w);
            return;
        }
        if (isset) {
            const int off = top + inc - sz;
            const GLB_AS uint16_t *src = pd.govf + (uint32_t)o;
            GLB_AS uint16_t *dst = pd.govf + off;
            for (int k = 0; k <= n; k++) dst[k] = src[k];
            w.O[i] = (typename T::O_v)(MT_OVF_BIT | (u64)(uint32_t)off);
        }
        top += tot;
        wsync<T>();
        pd.dirty = 1;
        pd.tdirty = 1;   // the table's copies of the masks are rebuilt at the flush
        w.dlo = 0;
        pg_win_flush(pd);
        if (w.status) return;
    }
    gsync_rd();
    pd.ovf_half = nh;
    pd.ovf_top = top;
    pd.ovf_peak = max(pd.ovf_peak, top - lo);
    pd.cur = -1;
    if (keep >= 0) {
        pg_win_load(pd, keep);
        pd.cur_pos = keep_pos;
    }
}
// Arena units one message may take for new overflow sets: a remove makes at most one set per
// segment it marks (<= its span), each a copy of the segment's list -- an existing set (<= the
// largest made) or the clients of its slot bits (<= the slots in use) -- plus the remover and
// the count.  0 when no set can be made (no set exists yet and the remover has or can take an
// overlap slot).
TD int pg_ovf_need(PagedDoc<T> &pd, const mt_op_rec &op) {
    if (op.kind != MT_OP_REMOVE) return 0;
    DocT<T> &w = pd.w;
    if (!w.wide && !oslot_short(w, op_cli(op))) return 0;
    const int used = __popcll(ballot(lane() < MT_OSLOT_USE && w.ocli != MT_OSLOT_FREE));
    const int span = min(max(op.pos2 - op.pos1, 0), 1 << 16);
    return (int)min((int64_t)span * (max(pd.ovf_maxn, used) + 2), (int64_t)1 << 30);
}
// The same bound counted instead of assumed, for when the first would not fit: a set is made
// only for a segment some concurrent remover already removed (removedSeq above the remover's
// refSeq >= minSeq, so an unsettled segment: an unsettled-table entry, or a row of the page in
// the window when that page changed since its entries were written) that the remover still
// sees (its view length > 0), so on a page its view [pos1, pos2) reaches; at most one per
// segment (a split segment's set goes to the piece inside the range), of its list's size + 2.
TD int ovf_units_of(PagedDoc<T> &pd, const v4i &a, u64 o, int r, int c) {
    if (a.z == MT_RSEQ_NONE || vlen(pd.w, a, o, r, c) <= 0) return 0;
    return ((o & MT_OVF_BIT) ? (int)pd.govf[(uint32_t)o] : __popcll(o)) + 2;
}
TD int pg_ovf_need_counted(PagedDoc<T> &pd, const mt_op_rec &op) {
    DocT<T> &w = pd.w;
    const int r = op.ref_seq, c = op_cli(op);
    w.ocs = oslot_of(w, c);   // (as pg_apply_op_impl sets it: the view's own slot)
    pg_views_cached(pd, r, c);
    int start, ostart;
    const int np = nbr(pd.up, 1);
    const int p1 = pg_find(pd, op.pos1, true, start, ostart);
    int p2 = pg_find(pd, op.pos2, false, start, ostart);
    if (w.status) return 1 << 30;
    if (p1 < 0) return 0;   // (the range starts past the end: nothing to mark)
    if (p2 < 0) p2 = np - 1;
    const int wpos = pd.cur >= 0 && pd.tdirty ? pg_cur_pos(pd) : -1;   // (as pg_views_impl)
    int s = 0;
    for (int e = lane(); e < pd.ut_n; e += MT_WAVE) {
        int pos;
        v4i a;
        u64 o;
        tab_get(pd, e, pos, a, o);
        if (pos >= p1 && pos <= p2 && pos != wpos) s += ovf_units_of(pd, a, o, r, c);
    }
    if (wpos >= p1 && wpos <= p2) {
        v4i a;
        u64 o;
        load_ao(w, lane(), lane() < w.n, a, o);
        if (lane() < w.n) s += ovf_units_of(pd, a, o, r, c);
    }
    return wave_sum(s);
}

// Can this message's text / property records be placed without running out of the arenas?
// (TextSegment.append and property sets are unbounded in the reference, MT/textSegment.ts:74-85.)
// A tight launch compacts inside messages, as every tier does, and hands the document on when a
// compaction left an arena nearly full (press); a growing launch compacts here, between
// messages, and hands the document to the
// growth step (cause 4 text / 5 records / 9 uid map, kept in HDR_DIAG with status 0) when the
// live text / records / segments then leave less than 1/8 of it free (and at least 4096 text
// units / 128 records / 64 ids, for a message's merges; 11: the overflow overlap
// sets, never reclaimed, half of it) -- so a message never fails half applied, and a document
// whose live data fits is compacted, not moved.  The
// bound covers an insert's own text and one range step's records (props_ensure(d, MT_WAVE));
// a zamboni merge's copy is served by the half kept free.
TD bool pg_arena_room(PagedDoc<T> &pd, const mt_op_rec &op, const PagedCaps &pc) {
    DocT<T> &w = pd.w;
    const int nt = op.kind == MT_OP_INSERT && !(op.flags & MT_F_MARKER) ? max(op.pos2, 0) : 0;
    const int np = MT_WAVE + 1;
    const bool t_ok = w.text_top + nt <= w.T_cap, p_ok = w.props_top + np <= w.P_cap;
    const bool u_ok = w.next_uid + 4 <= pd.UM || op.kind == MT_OP_LOAD_REMOVED;
    if constexpr (T::kOvf) {
        if (pd.govf) {   // the overflow overlap arena (cause 11; a tight launch hands the document on)
            // this message's new sets must fit the current half: the live sets are compacted
            // into the other half first when they would not, and the document is handed to
            // the growth step (which doubles the arena) when even that leaves too little room
            // -- so ovf_mark never runs out in the middle of a message
            int need = pg_ovf_need(pd, op);
            if (need > 0 && pd.ovf_top + need > ovf_half_end(pd)) need = min(need, pg_ovf_need_counted(pd, op));
            if (need > 0 && pd.ovf_top + need > ovf_half_end(pd)) {
                pg_ovf_compact(pd);
                if (w.status) return true;   // (failed: the loop stops)
                if (pd.ovf_top + need > ovf_half_end(pd)) {
                    w.cap_cause = 11;
                    return false;
                }
            }
        }
    }
    // a tight launch compacts inside the message (text_ensure) and hands the document on once
    // a compaction leaves an arena nearly full (press); the uid map is renumbered at the next
    // tier's message start
    if (pc.tight) return u_ok && !pd.press;
    if (t_ok && p_ok && u_ok) return true;
    if constexpr (T::kMayGrow) {
        {
            if (!u_ok) {   // (the renumbering pg_apply_op would do, done here; cause 9)
                pg_renumber(pd, true);
                if (w.status) return true;
                if (w.next_uid + 8 > pd.UM - max(pd.UM / 8, 64)) {
                    w.cap_cause = 9;
                    return false;
                }
            }
            if (!t_ok) {
                paged_text_compact(w);
                if (w.status) return true;   // (failed: the loop stops)
                if (w.text_top + nt > w.T_cap - max(w.T_cap / 8, 4096)) {   // (slack: merges' copies)
                    w.cap_cause = 4;
                    return false;
                }
            }
            if (!p_ok) {
                paged_props_compact(w);
                if (w.status) return true;
                if (w.props_top + np > w.P_cap - max(w.P_cap / 8, 2 * MT_WAVE)) {
                    w.cap_cause = 5;
                    return false;
                }
            }
            return true;
        }
    }
    return false;
}

// ------------------------------------------------------------------ bind / store / convert
// Per-document HBM bases of the paged arrays the op path uses (pages, uid map).
// (the main arrays, or the document's slot in the big region after a growth step)
TD void pg_bases(PagedDoc<T> &pd, const DevState &st, int doc) {
    const PagedBase b = tier_paged<T::kBig>(st, doc);
    pd.gA = (GLB_AS v4i *)b.A;
    pd.gO = (GLB_AS u64 *)b.O;
    pd.gB = (GLB_AS v4u *)b.B;
    pd.gumap = (GLB_AS uint16_t *)b.umap;
    pd.govf = (GLB_AS uint16_t *)b.ovf;
    pd.OA = b.OA;
    pd.goS = (GLB_AS uint16_t *)b.oS;
    pd.goL = (GLB_AS uint16_t *)b.oL;
    pd.PPh = b.PP;
    pd.UM = b.UM;
    pd.doc = doc;
}

// The bases only pg_load / pg_store touch, recomputed there from the kernel arguments.
struct PgCold {
    GLB_AS PageMeta *gmeta;
    GLB_AS uint16_t *gdir;
    GLB_AS uint8_t *gcnt;
    GLB_AS v2i *gheap;
    GLB_AS int *gupage;
    GLB_AS v4i *guA;
    GLB_AS u64 *guO;
};
template <class T> __device__ __forceinline__ PgCold pg_cold(const DevState &st, int doc) {
    const PagedBase b = tier_paged<T::kBig>(st, doc);
    PgCold c;
    c.gmeta = (GLB_AS PageMeta *)b.meta;
    c.gdir = (GLB_AS uint16_t *)b.dir;
    c.gcnt = (GLB_AS uint8_t *)b.cnt;
    c.gheap = (GLB_AS v2i *)b.heap;
    c.gupage = (GLB_AS int *)b.upage;
    c.guA = (GLB_AS v4i *)b.uA;
    c.guO = (GLB_AS u64 *)b.uO;
    return c;
}

// Window + upper DocT instances over the LDS layout; scalars from the document header.
TD void pg_setup(PagedDoc<T> &pd, const DevState &st, int doc, LDS_AS uint8_t *smem, const PagedLayout &L,
              const PagedCaps &pc) {
    DocT<T> &w = pd.w;
    DocT<T> &up = pd.up;
    pg_bases(pd, st, doc);
    pd.PP = pc.PP;
    pd.PH = pc.PH;
    pd.UT = pc.UT;
    w.hp = st.hdr + doc;
    {   // the arenas of the document's region (the big region's grow with the growth step)
        const PagedBase b = tier_paged<T::kBig>(st, doc);
        w.text = (GLB_AS uint16_t *)b.text;
        w.props = (GLB_AS uint32_t *)b.props;
        w.T_cap = b.T;
        w.P_cap = b.P;
    }
    w.dlog = st.DL ? (GLB_AS int32_t *)(st.dlog + doc * (size_t)st.DL) : nullptr;
    w.DL_cap = st.DL;
    w.rich = st.DLR;
    w.oslot = (GLB_AS int32_t *)(st.oslot + doc * (size_t)(2 * MT_OSLOTS));
    w.ocli = w.oslot[2 * lane()];
    w.ocs = 0;
    w.S_cap = MT_PG_SLOTS;
    w.B_cap = PW_B;
    w.H_cap = pc.PH;
    w.A = (typename T::A_t)(smem + L.offWA);
    w.Bv = (typename T::B_t)(smem + L.offWB);
    w.O = (typename T::O_t)(smem + L.offWO);
    w.heap = (typename T::H_t)(smem + L.offHeap);
    w.cnt = smem + L.offWcnt;
    w.flg = (LDS_AS int8_t *)(smem + L.offWflg);
    w.ends = (LDS_AS uint16_t *)(smem + L.offWends);
    w.scr = (LDS_AS int32_t *)(smem + L.offWscr);
    w.nb = (LDS_AS int32_t *)(smem + L.offWnb);
#ifdef MT_PROF
    w.prof = (LDS_AS u64 *)(smem + L.offProf);
    w.prof[lane()] = 0;
    w.prof[64 + lane()] = 0;
#endif
    const DocHdr h = *w.hp;
    w.n = 0;
    w.depth = h.depth;
    w.heap_n = h.heap_n;
    w.cur_seq = h.cur_seq;
    w.min_seq = h.min_seq;
    w.text_top = h.text_top;
    w.text_half = h.text_half;
    w.props_top = h.props_top;
    w.props_half = h.props_half;
    w.next_uid = h.next_uid;
    w.status = h.status;
    w.dlog_n = h.dlog_n;
    w.dhash = h.delta_hash;
    w.wide = h.pad0 & 1;
    if (T::kLog) {
        w.m_split = h.pad[HDR_MSPLIT];
        w.m_append = h.pad[HDR_MAPPEND];
        w.m_unlink = h.pad[HDR_MUNLINK];
        w.dlog_ovf = h.pad[HDR_DLOG_OVF];
        w.dlog_rec = -1;
    }
    w.text_gcs = w.props_gcs = w.cap_cause = 0;
    w.ord = 0;
    w.obst = 0;
    w.os = nullptr;
    w.ob = nullptr;
    w.dfr_rec = -1;
    if constexpr (T::kLog) {
        if (pd.goS) {   // segment ordinals: the window's pointers follow its page (pg_win_place)
            w.ord = 1;
            w.obst = 16;   // level 1 of a window (the page itself) lands in the scratch half of goL
        }
    }
    w.dlo = MT_PG_SLOTS;
    w.paged = 1;
    w.obs_base = 0;
    w.pend_split = 0;
    w.pend_second = -1;
    w.dir = nullptr;
    up = w;
    up.paged = 0;
    up.cnt = smem + L.offUcnt - pc.PP;   // lvl(up, l) for l >= 1 only
    up.nb = (LDS_AS int32_t *)(smem + L.offUnb);
    up.dir = (LDS_AS uint16_t *)(smem + L.offDir);
    up.B_cap = pc.PP;
    up.status = 0;
    if (ordon(w)) {   // levels >= 1 by level position (PagedBase.oU)
        up.ob = (GLB_AS uint16_t *)tier_paged<T::kBig>(st, doc).oU;
        up.obst = pd.PPh;
    }
    pd.pvl = (LDS_AS int *)(smem + L.offCob);
    pd.cob = pd.pvl;
    pd.cdl = pd.cob + (pc.PP + 63) / 64;
    if constexpr (T::kHM) {
        pd.meta = nullptr;
        pd.gmeta = (GLB_AS PageMeta *)tier_paged<T::kBig>(st, doc).meta;
        pd.sob = pd.cdl + (pc.PP + 63) / 64;
        pd.sob_ch = -1;
        pd.wnb = pd.wobs = 0;
    } else {
        pd.meta = (LDS_AS PageMeta *)(smem + L.offMeta);
    }
    pd.vgen = 0;
    pd.scr_ch = -1;
    pd.upage = (LDS_AS uint16_t *)(smem + L.offUpage);
    pd.uA = (LDS_AS v4i *)(smem + L.offUA);
    pd.uO = (LDS_AS typename T::O_v *)(smem + L.offUO);
    if constexpr (T::kPacked) {
        pd.uL = (LDS_AS uint32_t *)(smem + L.offUA);
        pd.uS = pd.uL + pc.UT;
        pd.uP = pd.uS + pc.UT;
        pd.sbase = h.cur_seq - 32000;
        pd.uM = (LDS_AS u64 *)(smem + L.offUO);
        pd.mbm = (LDS_AS uint32_t *)(smem + L.offUO + 8u * MT_PK_MASKS);
        if (lane() < MT_PK_MASKS / 32) pd.mbm[lane()] = lane() == 0 ? 1u : 0u;
        if (lane() == 0) pd.uM[0] = 0;
    }
    pd.cur = -1;
    pd.cur_pos = -1;
    pd.dirty = 0;
    pd.tdirty = 0;
    pd.vvalid = 0;
    pd.wgrow = 0;
    pd.opbound = 0;
    pd.zuid = 0;
    pd.zpv = 0;
    pd.press = 0;
    pd.ovf_top = MT_OVF_HDR;
    pd.ovf_last = 0;
    pd.ovf_maxn = 0;
    pd.ovf_half = 0;
    pd.ovf_made = 0;
    pd.ovf_peak = 0;
    if constexpr (T::kOvf) {
        if (pd.govf) {
            const GLB_AS uint32_t *hw = (const GLB_AS uint32_t *)pd.govf;
            pd.ovf_top = max((int)hw[0], MT_OVF_HDR);
            pd.ovf_last = (int)hw[1];
            pd.ovf_maxn = (int)hw[2];
            pd.ovf_made = hw[4];
            pd.ovf_peak = (int)hw[5];
            // the upper half only while the fill is above the midpoint: after a growth step
            // (the arena doubled, its contents copied at the same offsets) the sets lie in the
            // new lower half
            pd.ovf_half = ((int)hw[3] & 1) && pd.ovf_top > mt_ovf_mid(pd.OA) ? 1 : 0;
        }
    }
}

// Pages not in the directory are free (meta cleared; a tag bit in nblk marks them first): the
// HBM meta of ids above a narrower launch's capacity may never have been written.
TD void pg_mark_free(PagedDoc<T> &pd) {
    const int np = nbr(pd.up, 1);
    pd.vvalid = 0;
    for (int base = 0; base < pd.PP; base += MT_WAVE)
        if (base + lane() < pd.PP) pm_set_nblk(pd, base + lane(), pm_nblk(pd, base + lane()) | 0x80);
    wsync<T>();
    for (int base = 0; base < np; base += MT_WAVE)
        if (base + lane() < np) {
            const int pg = pd.up.dir[base + lane()];
            pm_set_nblk(pd, pg, pm_nblk(pd, pg) & 0x7F);
        }
    wsync<T>();
    for (int base = 0; base < pd.PP; base += MT_WAVE) {
        const int pg = base + lane();
        if (pg < pd.PP && (pm_nblk(pd, pg) & 0x80)) pm_set_ns(pd, pg, 0, 0);
    }
    wsync<T>();
}

// Loads a paged document's directory, meta, upper counts, heap and table into LDS.  Returns
// false (nothing staged) when the document does not fit this launch's LDS capacities.
TD bool pg_load(PagedDoc<T> &pd, const DevState &st) {
    const PgCold g = pg_cold<T>(st, pd.doc);
    DocT<T> &w = pd.w;
    DocT<T> &up = pd.up;
    const DocHdr h = *w.hp;
    const int np = h.n_blk[1];
    if (np > pd.PP || h.pad[HDR_UTN] > pd.UT || h.heap_n > pd.PH) return false;
    for (int l = 2; l < h.depth; l++)
        if (h.n_blk[l] + 4 > pcnt_cap(pd.PP, l)) return false;   // (the upper levels' room, pg_room)
    if (T::kOvlBits < 64 && w.wide) return false;
    if constexpr (!T::kOvf) {   // overflow overlap sets still consulted: a 64-bit tier's
        if (pd.govf) {
            const GLB_AS uint32_t *hw = (const GLB_AS uint32_t *)pd.govf;
            if ((int)hw[0] > MT_OVF_HDR && (int)hw[1] > w.min_seq) return false;
        }
    }
    if (T::kPacked && w.cur_seq - w.min_seq > 30000) return false;   // the packed table's seq offsets
    int mx = 0;
    for (int q = lane(); q < np; q += MT_WAVE) mx = max(mx, (int)g.gdir[q]);
    if (wave_max(mx) >= pd.PP) return false;   // a page id allocated by a wider launch
    if (lane() < MT_LV) up.nb[lane()] = w.hp->n_blk[lane()];
    wsync<T>();
    for (int q = lane(); q < np; q += MT_WAVE) up.dir[q] = g.gdir[q];
    if constexpr (!T::kHM) {   // (T::kHM: the metadata stays in HBM; pg_mark_free clears the free pages')
        GLB_AS const uint32_t *gm = (GLB_AS const uint32_t *)g.gmeta;
        LDS_AS uint32_t *lm = (LDS_AS uint32_t *)pd.meta;
        for (int i = lane(); i < pd.PP * (int)(sizeof(PageMeta) / 4); i += MT_WAVE) lm[i] = gm[i];
    }
    for (int l = 1; l < up.depth; l++) {
        const int nl = nbr(up, l);
        for (int b = lane(); b < nl; b += MT_WAVE) lvl(up, l)[b] = g.gcnt[l * pd.PPh + b];
    }
    for (int i = 1 + lane(); i <= w.heap_n; i += MT_WAVE) w.heap[i] = g.gheap[i];
    // the HBM table names page ids; LDS entries name level-1 positions: each page's position
    // in its meta obs word for the conversion (restored from HBM below) -- T::kHM: in the text
    // arena's idle half (scratch, as pg_renumber), or found in the directory when it is short
    wsync<T>();
    GLB_AS int32_t *posof = T::kHM ? (GLB_AS int32_t *)text_base(w, 1 - w.text_half) : nullptr;
    const bool pscr = T::kHM && 2 * pd.PP <= w.T_cap;
    if constexpr (T::kHM) {
        if (pscr)
            for (int q = lane(); q < np; q += MT_WAVE) posof[up.dir[q]] = q;
        gsync();
        gsync_rd();
    } else {
        for (int q = lane(); q < np; q += MT_WAVE) pm_set_obs(pd, up.dir[q], q);
    }
    wsync<T>();
    // ut_n follows the fill, so that a mask collection inside tab_midx (tab_mgc) scans only
    // the entries written so far, not stale LDS of an earlier workgroup
    const int utn = h.pad[HDR_UTN];
    pd.ut_n = 0;
    for (int base = 0; base < utn; base += MT_WAVE) {   // (uniform: tab_midx is collective)
        const int e = base + lane();
        const bool v = e < utn;
        // unconditional loads (a 64-bit load under a per-lane select miscompiles: DESIGN.md
        // section 10); entry 0 exists whenever the loop runs
        const int ec = v ? e : 0;
        int p;   // (its position)
        if constexpr (T::kHM) {
            const int pg = g.gupage[ec];
            if (pscr) {
                p = posof[pg];
            } else {
                p = 0;
                for (int q = 0; q < np; q++)
                    if (up.dir[q] == pg) {
                        p = q;
                        break;
                    }
            }
        } else {
            p = pm_obs(pd, g.gupage[ec]);
        }
        const v4i a = g.guA[ec];
        const u64 o = g.guO[ec];
        const int mi = tab_midx(pd, v && o != 0);
        if (mi < 0) return false;   // (more masked entries than the packed table keeps)
        if (v) tab_put(pd, e, p, a, o, mi);
        pd.ut_n = min(base + MT_WAVE, utn);
    }
    wsync<T>();
    if constexpr (!T::kHM) {
        for (int q = lane(); q < np; q += MT_WAVE) pm_set_obs(pd, up.dir[q], g.gmeta[up.dir[q]].obs);
        wsync<T>();
    }
    pg_mark_free(pd);
    pg_cob_rebuild(pd);
    return true;
}

TD void pg_store(PagedDoc<T> &pd, const DevState &st) {
    const PgCold g = pg_cold<T>(st, pd.doc);
    DocT<T> &w = pd.w;
    DocT<T> &up = pd.up;
    // a document that failed keeps the state it had at the failure (the reference's state at
    // its throw): the window is written back regardless of the status
    const int failed = w.status;
    w.status = 0;
    pg_win_flush(pd);
    if (failed) w.status = failed;
    w.oslot[2 * lane()] = w.ocli;
    if constexpr (T::kOvf) {
        if (pd.govf && lane() < MT_OVF_HDR / 2)
            ((GLB_AS uint32_t *)pd.govf)[lane()] =
                lane() == 0 ? (uint32_t)pd.ovf_top
                            : (lane() == 1 ? (uint32_t)pd.ovf_last
                                           : (lane() == 2 ? (uint32_t)pd.ovf_maxn
                                                          : (lane() == 3 ? (uint32_t)pd.ovf_half
                                                                         : (lane() == 4 ? pd.ovf_made
                                                                                        : (uint32_t)pd.ovf_peak))));
    }
    wsync<T>();
    const int np = nbr(up, 1);
    for (int q = lane(); q < np; q += MT_WAVE) g.gdir[q] = up.dir[q];
    if constexpr (!T::kHM) {   // (T::kHM: the metadata is in HBM already)
        GLB_AS uint32_t *gm = (GLB_AS uint32_t *)g.gmeta;
        LDS_AS const uint32_t *lm = (LDS_AS const uint32_t *)pd.meta;
        for (int i = lane(); i < pd.PP * (int)(sizeof(PageMeta) / 4); i += MT_WAVE) gm[i] = lm[i];
    }
    for (int l = 1; l < up.depth; l++) {
        const int nl = nbr(up, l);
        for (int b = lane(); b < nl; b += MT_WAVE) g.gcnt[l * pd.PPh + b] = lvl(up, l)[b];
    }
    for (int i = 1 + lane(); i <= w.heap_n; i += MT_WAVE) g.gheap[i] = w.heap[i];
    for (int e = lane(); e < pd.ut_n; e += MT_WAVE) {
        int p;
        v4i a;
        u64 o;
        tab_get(pd, e, p, a, o);
        g.gupage[e] = up.dir[p];   // (LDS entries name positions; HBM ones page ids)
        g.guA[e] = a;
        g.guO[e] = o;
    }
    int nbl[MT_LV];
#pragma unroll
    for (int l = 0; l < MT_LV; l++) nbl[l] = nbr(up, l);
    int nseg = 0;
    for (int q = lane(); q < np; q += MT_WAVE) nseg += pm_nseg(pd, up.dir[q]);
    nseg = wave_sum(nseg);
    if (lane() == 0) {
        DocHdr h;
        memset(&h, 0, sizeof(h));
        h.n_seg = nseg;
        h.depth = up.depth;
        h.heap_n = w.heap_n;
        h.cur_seq = w.cur_seq;
        h.min_seq = w.min_seq;
        h.text_top = w.text_top;
        h.text_half = w.text_half;
        h.props_top = w.props_top;
        h.props_half = w.props_half;
        h.next_uid = w.next_uid;
        h.status = w.status;
        h.dlog_n = w.dlog_n;
#pragma unroll
        for (int l = 0; l < MT_LV; l++) h.n_blk[l] = nbl[l];
        h.delta_hash = w.dhash;
        h.n_ops = w.hp->n_ops;
        h.pad0 = w.wide;
        h.pad[HDR_PAGED] = 1;
        h.pad[HDR_NPAGES] = np;
        h.pad[HDR_UTN] = pd.ut_n;
        // (status 0: an arena hand-over's cause for the growth step, pg_arena_room)
        h.pad[HDR_DIAG] =
            w.status || w.cap_cause == 4 || w.cap_cause == 5 || w.cap_cause == 9 || w.cap_cause == 11 ? w.cap_cause : 0;
        if (T::kLog) {
            h.pad[HDR_MSPLIT] = w.m_split;
            h.pad[HDR_MAPPEND] = w.m_append;
            h.pad[HDR_MUNLINK] = w.m_unlink;
            h.pad[HDR_DLOG_OVF] = w.dlog_ovf;
        }
        *w.hp = h;
    }
}

// A flat document's state: segment table, per-level child counts (level stride B), leaf
// needsScour flags and heap -- in the flat HBM arrays, or a summary load's staging buffers.
struct FlatSrc {
    GLB_AS const v4i *A;
    GLB_AS const u64 *O;
    GLB_AS const v4u *Bv;
    GLB_AS const uint8_t *cnt;
    GLB_AS const int8_t *flg;
    GLB_AS const v2i *heap;
    size_t B;
    GLB_AS const uint16_t *os, *ob;   // ordinal characters (DevState.ordS / ordB; null: none kept)
};
__device__ __forceinline__ FlatSrc flat_src(const DevState &st, int doc) {
    const size_t S = st.S, B = st.B;
    FlatSrc f;
    f.A = (GLB_AS const v4i *)(st.segA + doc * S);
    f.O = (GLB_AS const u64 *)(st.segO + doc * S);
    f.Bv = (GLB_AS const v4u *)(st.segB + doc * S);
    f.cnt = (GLB_AS const uint8_t *)(st.cnt + doc * (size_t)MT_LV * B);
    f.flg = (GLB_AS const int8_t *)(st.flg + doc * B);
    f.heap = (GLB_AS const v2i *)(st.heap + doc * (size_t)(st.H + 1));
    f.B = B;
    f.os = st.ordS ? (GLB_AS const uint16_t *)(st.ordS + doc * S) : nullptr;
    f.ob = st.ordS ? (GLB_AS const uint16_t *)(st.ordB + doc * (size_t)MT_LV * B) : nullptr;
    return f;
}

// Converts a flat document (state in the flat HBM arrays: initial contents, or spilled by
// the LDS tier; or a large summary header staged by k_load_header) into the paged layout:
// page j = level-1 node j (the whole tree when the root is a leaf block).  Leaves the paged
// state staged in LDS (pg_store writes it).
TD bool pg_convert(PagedDoc<T> &pd, const FlatSrc &src) {
    DocT<T> &w = pd.w;
    DocT<T> &up = pd.up;
    const DocHdr h = *w.hp;
    const size_t B = src.B;
    GLB_AS const v4i *fA = src.A;
    GLB_AS const u64 *fO = src.O;
    GLB_AS const v4u *fB = src.Bv;
    GLB_AS const uint8_t *fc = src.cnt;
    GLB_AS const int8_t *ff = src.flg;
    GLB_AS const v2i *fH = src.heap;
    const int depth = h.depth;
    const int np = depth == 1 ? 1 : h.n_blk[1];
    bool up_ok = true;
    for (int l = 2; l < depth; l++) up_ok = up_ok && h.n_blk[l] + 4 <= pcnt_cap(pd.PP, l);
    if (np + 8 > pd.PP || !up_ok || h.heap_n > pd.PH) {
        pg_fail_cap(w, np + 8 > pd.PP || !up_ok ? 7 : 3);
        return false;
    }
    // the packed table stores seq / removedSeq as 16-bit offsets from currentSeq - 32000: a
    // wider collab window goes to the next tier (as pg_load refuses it)
    if (T::kPacked && w.cur_seq - w.min_seq > 30000) {
        pg_fail_cap(w, 8);
        return false;
    }
    up.depth = depth;
    if (lane() < MT_LV) up.nb[lane()] = lane() == 0 ? 0 : (lane() == 1 ? np : (lane() < depth ? h.n_blk[lane()] : 0));
    wsync<T>();
    for (int l = 2; l < depth; l++) {
        const int nl = h.n_blk[l];
        for (int b = lane(); b < nl; b += MT_WAVE) lvl(up, l)[b] = fc[l * B + b];
    }
    for (int i = 1 + lane(); i <= h.heap_n; i += MT_WAVE) w.heap[i] = fH[i];
    for (int pg = lane(); pg < pd.PP; pg += MT_WAVE) pm_set_ns(pd, pg, 0, 0);
    pd.ut_n = 0;
    wsync<T>();
    int lb = 0, s = 0;
    for (int j = 0; j < np; j++) {
        const int nbk = depth == 1 ? 1 : (int)uni(fc[B + j]);   // level-1 count: leaf blocks
        int ns = 0;
        for (int q = 0; q < nbk; q++) ns += depth == 1 ? h.n_seg : (int)uni(fc[lb + q]);
        if (nbk > MT_MAXN || ns > MT_PG_SLOTS) {
            FAIL_INTERNAL(w);
            return false;
        }
        // stage the page in the window, then write it like any other page
        const int i = lane();
        bool wide = false;
        if (i < ns) {
            w.A[i] = fA[s + i];
            const u64 o = fO[s + i];
            wide = T::kOvlBits < 64 && (o >> T::kOvlBits) != 0ull;
            w.O[i] = (typename T::O_v)o;
            w.Bv[i] = fB[s + i];
        }
        if (ballot(wide)) {   // overlap ids above a narrow tier's masks
            pg_fail_cap(w, 10);
            return false;
        }
        if (i < PW_B) {
            lvl(w, 0)[i] = i < nbk ? (depth == 1 ? (uint8_t)h.n_seg : fc[lb + i]) : 0;
            w.flg[i] = i < nbk ? ff[lb + i] : (int8_t)0;
        }
        if (i == 0) {
            up.dir[j] = (uint16_t)j;
            lvl(up, 1)[j] = (uint8_t)nbk;
        }
        w.n = ns;
        if (ordon(w) && src.os) {   // the flat document's characters: slots, leaf blocks, the page
            if (i < ns) pd.goS[(size_t)j * MT_PG_SLOTS + i] = src.os[s + i];
            if (i < nbk) pd.goL[(size_t)j * MT_PG_OLB + i] = src.ob[lb + i];
            if (i == 0) up.ob[(size_t)up.obst + j] = src.ob[B + j];
        }
        wsync<T>();
        pg_table_add(pd, 0, ns, j);
        if (w.status) return false;
        pg_write_page(pd, j, 0, ns, 0, nbk);
        lb += nbk;
        s += ns;
    }
    pg_mark_free(pd);
    pg_cob_rebuild(pd);
    pd.cur = -1;
    pd.wgrow = pd.opbound = 0;
    if (ordon(w)) {
        if (src.os) {   // levels >= 2 keep their positions
            for (int l = 2; l < depth; l++)
                for (int b = lane(); b < h.n_blk[l]; b += MT_WAVE) up.ob[(size_t)l * up.obst + b] = src.ob[l * B + b];
            gsync();
        } else {   // a loaded summary: reloadFromSegments ends with nodeUpdateOrdinals(root) (:1273-1276)
            ord_canon_all(up);
        }
    }
    // the flat tiers number ids without bound: compact them for the uid -> page map
    if (w.next_uid + 4 > pd.UM) pg_renumber(pd);
    return w.status == 0;
}
