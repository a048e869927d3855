// mt_device.h -- device-side data layout and wave primitives of the MI355X merge-tree
// replay engine.  One wavefront (64 lanes, one workgroup) owns one document for the whole
// launch and applies that document's ops in sequence order.
//
// Per-document state in HBM (struct-of-arrays, document-major, fixed per-doc strides):
//   segA[S]  int4  {cachedLength, seq, removedSeq (INT_MIN = undefined), client|rclient<<16}
//   segO[S]  u64   removedClientOverlap as a bit mask over short client ids 1..64
//   segB[S]  uint4 {text offset (marker: refType), props record handle, uid|MARKER, 0}
//            -- all in *document order*: the flat order of the reference's leaves
//   cnt[LV][B] u8  child counts of every B-tree level in order (level 0 = leaf blocks);
//            the reference's tree (MT/mergeTree.ts:333 MaxNodesInBlock=8) is exactly
//            determined by these counts because every leaf sits at the same depth
//   flg[B]   i8    leaf-block needsScour tri-state (-1 undefined, 0 false, 1 true)
//   heap[H]  int2  zamboni LRU heap {maxSeq, uid} (1-based, MT/collections.ts:212-265)
//   text[2][T] u16 UTF-16 arena, two halves for compaction
//   props[2][P][PREC] u32 property-set records {n, (key, value) x KMAX}
// During a launch the B-tree counts and flags are staged in LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mt_types.h"

#define MT_WAVE 64
#define MT_LV 8                 // max B-tree levels (7^8 leaves >> any capacity)
#define MT_MAXN 8               // MaxNodesInBlock           MT/mergeTree.ts:333
#define MT_HALF 4               // MaxNodesInBlock / 2       MT/mergeTree.ts:2510
#define MT_GRAN 256             // TextSegmentGranularity    MT/mergeTree.ts:1093
#define MT_ZAMBONI 2            // zamboniSegmentsMaxCount   MT/mergeTree.ts:1095
#define MT_KMAX 8               // max keys in one segment's property set
#define MT_PREC (1 + 2 * MT_KMAX)
#define MT_RSEQ_NONE ((int32_t)0x80000000)
#define MT_MARKER_BIT 0x80000000u
#define MT_SCOUR_UNDEF ((int8_t)-1)
#define MT_DOC_RETRY 100        // internal: document outgrew the LDS tier, replay it in HBM

typedef unsigned long long u64;
// clang ext-vector types (not HIP_vector_type): usable through LDS / global pointers
typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

struct DocHdr {               // 128 bytes per document
    int32_t n_seg, depth, heap_n, cur_seq;
    int32_t min_seq, text_top, text_half, props_top;
    int32_t props_half, next_uid, status, dlog_n;
    int32_t n_blk[MT_LV];
    u64 delta_hash;
    int32_t n_ops, pad0;
    int32_t pad[8];
};
static_assert(sizeof(DocHdr) == 128, "DocHdr size");

// Paged documents (mt_paged.h): a document that outgrows the LDS tier is kept as pages =
// level-1 nodes of the reference B-tree (<= 7 leaf blocks, <= 64 segment slots each).
struct PageMeta {             // 12 bytes, indexed by page id (LDS footprint: documents per CU)
    uint8_t nseg, nblk;
    uint16_t flg2;            // needsScour per leaf block, 2 bits each (value + 1: -1/0/1 -> 0/1/2)
    uint32_t bc;              // segments per leaf block, 4 bits each (<= MaxNodesInBlock)
    int32_t obs;              // observer length of the page
};
static_assert(sizeof(PageMeta) == 12, "PageMeta size");
static __host__ __device__ inline int pm_bcnt(const PageMeta &m, int q) { return (int)((m.bc >> (4 * q)) & 15u); }
static __host__ __device__ inline int8_t pm_flg(const PageMeta &m, int q) { return (int8_t)((int)((m.flg2 >> (2 * q)) & 3u) - 1); }
#define MT_OSLOTS 64
// Overlap masks use slots 1..63; bit 63 marks an *overflow set* (the last-tier paged
// instantiations with 64-bit masks, TierPagedT::kOvf, once every slot is taken): the mask's low 32 bits are
// then the offset of the segment's whole removedClientOverlap list in the document's overflow
// arena ([count, short ids...], u16), which starts with a 4-unit header {top (u32), last seq
// that made a set (u32)}
#define MT_OSLOT_USE 63
#define MT_OVF_BIT (1ull << 63)
// overflow arena header (u16 units): u32 {top, last message that made a set, largest set
// made, current half (0: [MT_OVF_HDR, mid), 1: [mid, MT_OVF_HDR + 2 (mid - MT_OVF_HDR))), units of
// every set made, high-water mark of the half in use (units)}
#define MT_OVF_HDR 12
// the overflow arena's two halves are the same size, so the live sets of either always fit the
// other (pg_ovf_compact)
static __host__ __device__ inline int mt_ovf_mid(int OA) { return MT_OVF_HDR + (((OA - MT_OVF_HDR) / 2) & ~7); }
#define MT_OVF_ARENA 8192      // overflow-arena units per document in the main arrays (the growth step raises it)
#define MT_OSLOT_FREE 0x7FFFFFFF
#define MT_PG_SLOTS 64
#define MT_PG_OLB 32          // ordinal characters kept per page for its leaf blocks (16 + scratch)
// DocHdr.pad[] words used by paged documents
#define HDR_PAGED 0           // 1: the document lives in the paged layout
#define HDR_NPAGES 1          // pages in the directory
#define HDR_UTN 2             // entries of the unsettled-segment table
#define HDR_DIAG 3            // failure diagnostic (source line of an internal error)
// DocHdr.pad[] words of every document kept by delta-logging handles (T::kLog):
// mergeTreeMaintenanceCallback event counts (MT/mergeTree.ts:2264-2269, :1368-1373, :1343-1348)
#define HDR_MSPLIT 4
#define HDR_MAPPEND 5
#define HDR_MUNLINK 6
#define HDR_DLOG_OVF 7        // the delta log overflowed (records dropped since the last reset)

// A set of paged arrays with its per-document capacities (strides).  The handle's main set
// is sized by mt_options; documents that outgrow it move to a second, larger set -- the
// *big region* -- in the growth step of mt_sync ("Growth").
struct PagedRegion {
    v4i *A;                   // [slots][PP][64]
    u64 *O;
    v4u *B;
    PageMeta *meta;           // [slots][PP]
    uint16_t *dir;            // [slots][PP]
    uint8_t *cnt;             // [slots][MT_LV][PP]
    v2i *heap;                // [slots][PH + 1]
    int32_t *upage;           // [slots][UT]
    v4i *uA;
    u64 *uO;
    // segment ordinals (segment_ordinals handles; null otherwise): each node's own ordinal
    // character -- per page slot, per leaf block of a page (16 + 16 scratch), and per node of
    // the upper levels by level position (level 1 = pages in directory order)
    uint16_t *oS;             // [slots][PP][64]
    uint16_t *oL;             // [slots][PP][32]
    uint16_t *oU;             // [slots][MT_LV][PP]
    int32_t PP, PH, UT, slots;
    // text / property arenas (two halves each, DocT text_base / prec): the main set's are the
    // handle's (DevState.text / props); the big region's are sized by the growth step too
    uint16_t *text;           // [slots][2][T]
    uint32_t *props;          // [slots][2][P][MT_PREC]
    uint16_t *umap;           // [slots][UM] uid -> page (pg_renumber keeps ids below UM)
    uint16_t *ovf;            // [slots][OA] overflow overlap sets (MT_OVF_BIT masks)
    int32_t T, P, UM, OA;
};
// document doc's paged arrays, arenas and uid map (bslot: its slot in the big region, -1: the
// main set)
struct PagedBase {
    v4i *A;
    u64 *O;
    v4u *B;
    PageMeta *meta;
    uint16_t *dir;
    uint8_t *cnt;
    v2i *heap;
    int32_t *upage;
    v4i *uA;
    u64 *uO;
    uint16_t *oS, *oL, *oU;   // ordinal characters (null: none)
    int32_t PP, PH, UT;
    uint16_t *text;           // [2][T]
    uint32_t *props;          // [2][P][MT_PREC]
    uint16_t *umap;           // [UM]
    uint16_t *ovf;            // [OA]
    int32_t T, P, UM, OA;
};
__host__ __device__ inline PagedBase paged_base(const PagedRegion &R, size_t i) {
    PagedBase b;
    const size_t PP = (size_t)R.PP;
    b.A = R.A + i * PP * MT_PG_SLOTS;
    b.O = R.O + i * PP * MT_PG_SLOTS;
    b.B = R.B + i * PP * MT_PG_SLOTS;
    b.meta = R.meta + i * PP;
    b.dir = R.dir + i * PP;
    b.cnt = R.cnt + i * MT_LV * PP;
    b.heap = R.heap + i * (size_t)(R.PH + 1);
    b.upage = R.upage + i * (size_t)R.UT;
    b.uA = R.uA + i * (size_t)R.UT;
    b.uO = R.uO + i * (size_t)R.UT;
    b.oS = R.oS ? R.oS + i * PP * MT_PG_SLOTS : nullptr;
    b.oL = R.oL ? R.oL + i * PP * MT_PG_OLB : nullptr;
    b.oU = R.oU ? R.oU + i * MT_LV * PP : nullptr;
    b.PP = R.PP;
    b.PH = R.PH;
    b.UT = R.UT;
    b.text = R.text + i * 2 * (size_t)R.T;
    b.props = R.props + i * 2 * (size_t)R.P * MT_PREC;
    b.umap = R.umap + i * (size_t)R.UM;
    b.ovf = R.ovf ? R.ovf + i * (size_t)R.OA : nullptr;
    b.T = R.T;
    b.P = R.P;
    b.UM = R.UM;
    b.OA = R.OA;
    return b;
}

struct DevState {
    DocHdr *hdr;
    v4i *segA;
    u64 *segO;
    v4u *segB;
    uint8_t *cnt;
    int8_t *flg;
    v2i *heap;
    uint16_t *text;
    uint32_t *props;
    int32_t *dlog;
    int32_t *oslot;           // [n_docs][64][2] overlap slots: {client (MT_OSLOT_FREE), last seq}
    int32_t *retry;           // per document: replay (the rest of) this batch in the HBM tier
    int64_t *resume;          // per document: first op the HBM tier replays
    uint32_t *stats;          // [0]: documents replayed in the HBM tier by the last launch
    // paged layout (PP == 0: disabled)
    v4i *pgA;                 // [n_docs][PP][64]
    u64 *pgO;
    v4u *pgB;
    PageMeta *pgMeta;         // [n_docs][PP]
    uint16_t *pgDir;          // [n_docs][PP] page ids in document (level-1) order
    uint8_t *pgCnt;           // [n_docs][MT_LV][PP] counts of levels >= 1 (level 1 = blocks per page)
    v2i *pgHeap;              // [n_docs][PH + 1] zamboni heap
    int32_t *pgUtPage;        // [n_docs][UT] unsettled-segment table: page, {len, seq, rseq, cli}, overlap
    v4i *pgUtA;
    u64 *pgUtO;
    uint16_t *pgUmap;         // [n_docs][UM] uid -> page
    uint16_t *pgOvf;          // [n_docs][OA] overflow overlap sets (MT_OVF_BIT)
    uint16_t *pgOS, *pgOL, *pgOU;   // ordinal characters of the paged layout (PagedRegion oS / oL / oU)
    int32_t PP, PH, UT, UM, OA;
    int32_t *bslot;           // [n_docs] slot in the big region (-1: main arrays); null: no big region
    PagedRegion big;          // documents re-tiered by the growth step (larger PP / PH / UT)
    int32_t S, B, H, T, P, DL;
    int32_t DLR;              // rich delta log: segment text / properties + maintenance events
    // segment ordinals (mt_options.segment_ordinals; null otherwise) of flat documents: every
    // node's own ordinal character (MergeBlock.setOrdinal, MT/mergeTree.ts:347-372); a
    // node's ordinal is its ancestors' characters then its own (mt_engine.h "ordinals")
    uint16_t *ordS;           // [n_docs][S] per segment
    uint16_t *ordB;           // [n_docs][MT_LV][B] per block of every level
    int32_t n_docs;
    // live-client handles (mt_options.live_client; null otherwise)
    int32_t *live;            // [n_docs][4] {collabWindow.localSeq, group queue head id, length, 0}
    int32_t *grp;             // [n_docs][LG + 1][MT_GRP_WORDS] segment-group table (index = id)
    struct PendQ *segP;       // [n_docs][S] per segment: its pending segment groups
    int32_t LG;               // group ids per document (outstanding segment groups)
    unsigned long long *prof; // [128] section timers of a -DMT_PROF build (null otherwise)
    const int64_t *gen_off;   // mt_generate_docs: [n_docs + 1] op offsets (per-document lengths);
                              // null: cfg.ops messages every document
    const int32_t *gen_ids;   // mt_generate_docs: [n_docs] global document indices (draws); null:
                              // doc_index_base + doc
    const int32_t *order;     // the applied batch's dispatch order (documents by message count,
                              // longest first); null: index order (equal lengths)
};
// The document replay workgroup i serves: the hardware dispatches workgroups in index order as
// slots free up, so a longest-first order is LPT scheduling of a skewed batch's documents
// (its serial tail is the longest document, not whichever came last).
__device__ __forceinline__ int doc_at(const DevState &st, int i) { return st.order ? st.order[i] : i; }

__host__ __device__ inline PagedRegion main_region(const DevState &st) {
    return PagedRegion{st.pgA,   st.pgO,    st.pgB,   st.pgMeta, st.pgDir, st.pgCnt, st.pgHeap, st.pgUtPage,
                       st.pgUtA, st.pgUtO, st.pgOS, st.pgOL,   st.pgOU,  st.PP,    st.PH,    st.UT,
                       st.n_docs, st.text, st.props, st.pgUmap, st.pgOvf, st.T, st.P, st.UM, st.OA};
}
// the paged arrays of document doc (device side: its slot from st.bslot; readers outside the
// replay kernels, which are instantiated per region)
__device__ inline PagedBase doc_paged(const DevState &st, int doc) {
    const int s = st.bslot ? st.bslot[doc] : -1;
    return s >= 0 ? paged_base(st.big, (size_t)s) : paged_base(main_region(st), (size_t)doc);
}
template <bool kBig> __device__ __forceinline__ PagedBase tier_paged(const DevState &st, int doc) {
    if constexpr (kBig)
        return paged_base(st.big, (size_t)st.bslot[doc]);
    else
        return paged_base(main_region(st), (size_t)doc);
}

// ------------------------------------------------------------------ wave primitives
// lane within the wavefront (the LDS-tier replay may hold several documents per workgroup,
// one per wave)
#ifdef MT_LANE_ASM
__device__ __forceinline__ int lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
#else
__device__ __forceinline__ int lane() { return (int)(threadIdx.x & (MT_WAVE - 1)); }
#endif

// Inclusive prefix sum over the wavefront with DPP row shifts + row broadcasts (6 VALU
// ops, no LDS traffic).  Lanes that have no source read the identity (bound_ctrl off,
// old = 0).
__device__ __forceinline__ int wave_scan_incl(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}
// Wave-uniform results come back through readlane/readfirstlane so that the compiler keeps
// them in SGPRs and branches on them uniformly.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int wave_sum(int v) { return __builtin_amdgcn_readlane(wave_scan_incl(v), 63); }
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, MT_WAVE));
    return uni(v);
}
// value of lane l (l wave-uniform)
__device__ __forceinline__ int bcast(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ u64 bcast64(u64 v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ u64 ballot(bool p) { return (u64)__ballot(p); }
__device__ __forceinline__ int first_lane(u64 m) { return __ffsll((long long)m) - 1; }

// ------------------------------------------------------------------ hashing
#define MT_FNV_OFF 1469598103934665603ULL
#define MT_FNV_PRIME 1099511628211ULL
__device__ __forceinline__ u64 fnv_u32(u64 h, uint32_t x) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        h ^= (x >> (8 * i)) & 0xFF;
        h *= MT_FNV_PRIME;
    }
    return h;
}
__device__ __forceinline__ u64 fnv_u64(u64 h, u64 x) {
    h = fnv_u32(h, (uint32_t)x);
    return fnv_u32(h, (uint32_t)(x >> 32));
}

// writer short id (sign-extended: loaded summaries append as NonCollabClient = -2)
__device__ __forceinline__ int op_cli(const mt_op_rec &op) { return (int)(int16_t)op.client; }

// ------------------------------------------------------------------ segment fields
__device__ __forceinline__ int seg_cli(v4i a) { return (int)(short)(a.w & 0xFFFF); }
__device__ __forceinline__ int seg_rcli(v4i a) { return (int)(short)((uint32_t)a.w >> 16); }
__device__ __forceinline__ int pack_cli(int cli, int rcli) {
    return (int)(((uint32_t)(uint16_t)cli) | (((uint32_t)(uint16_t)rcli) << 16));
}
// removedClientOverlap (MT/mergeTree.ts:2577-2585) as a bit mask over the document's overlap
// *slots*: a client that removes an already-removed segment takes a slot (1..63) for as long
// as a segment it marked is unsettled (DocT.ocli, mt_engine.h oslot_alloc); s = 0: no slot
__device__ __forceinline__ bool ovl_has(u64 o, int s) {
    const uint32_t sh = (uint32_t)(s - 1) & 63u;
    const uint32_t w = sh < 32 ? (uint32_t)o : (uint32_t)(o >> 32);
    return (s >= 1) & (s <= 64) & (((w >> (sh & 31u)) & 1u) != 0);
}

// nodeLength for a leaf in a remote view (c, r)   MT/mergeTree.ts:1692-1732; cs = c's overlap
// slot.  (branch-free: every term is evaluated, no shift depends on an unchecked slot)
__device__ __forceinline__ int view_len(v4i a, u64 o, int r, int c, int cs) {
    const int len = a.x, seq = a.y, rseq = a.z;
    const int cli = seg_cli(a), rcli = seg_rcli(a);
    const bool ins = (cli == c) | ((seq != -1) & (seq <= r));
    const bool gone = (rseq != MT_RSEQ_NONE) & ((rcli == c) | ovl_has(o, cs) | ((rseq != -1) & (rseq <= r)));
    return (ins & !gone) ? len : 0;
}
// localNetLength (observer view)   MT/mergeTree.ts:1195-1206
__device__ __forceinline__ int obs_len(v4i a) { return a.z == MT_RSEQ_NONE ? a.x : 0; }
// breakTie for a leaf at pos == len == 0, remote client   MT/mergeTree.ts:2281-2306
__device__ __forceinline__ bool tie(v4i a, int r) {
    const int rs = a.z;
    return !((rs != MT_RSEQ_NONE) & (rs != 0) & (rs <= r) & (rs != -1)) & (a.y != -1);
}

// ------------------------------------------------------------------ live-client documents
// A live handle (mt_options.live_client) backs a participant Client: the local client (short
// id 0) applies its own ops before they are sequenced (MT/client.ts:164-274).  Unacked
// sequence numbers are encoded above every real one: a pending insert has seq =
// MT_LOCAL_BASE + localSeq, a pending local remove removedSeq = MT_LOCAL_BASE +
// localRemovedSeq (UnassignedSequenceNumber + the segment's localSeq / localRemovedSeq,
// MT/mergeTree.ts:2102-2104, 2669-2670), so every `seq != Unassigned && seq <= refSeq` test
// of the observer engine holds unchanged.  Segment groups (MT/mergeTree.ts:1955-1962,
// segmentGroupCollection.ts) are a FIFO of up to 16 group ids per segment (DevState.segP,
// PendQ); the group table (a ring of DevState.LG ids) lives in HBM.
#define MT_LOCAL_BASE 0x40000000
#define MT_GRP_WORDS 12          // group entry {localSeq, kind | rewrite << 8 | nkeys << 16, keys[8], id stamp, 0}
#define MT_PQ_IDS 16             // pending groups a segment can be in at once
__device__ __forceinline__ bool is_local_seq(int s) { return s >= MT_LOCAL_BASE && s != MT_RSEQ_NONE; }
// A segment's pending segment groups: FIFO of group ids (1..DevState.LG, 16 bits each, the
// oldest in the low bits of w[0]); all zero: none.
struct PendQ {
    u64 w[4];
};
__device__ __forceinline__ PendQ pq_zero() { return PendQ{{0ull, 0ull, 0ull, 0ull}}; }
__device__ __forceinline__ bool pq_any(const PendQ &q) { return (q.w[0] | q.w[1] | q.w[2] | q.w[3]) != 0ull; }
__device__ __forceinline__ int pq_first(const PendQ &q) { return (int)(q.w[0] & 0xFFFFull); }
__device__ __forceinline__ int pq_at(const PendQ &q, int k) { return (int)((q.w[k >> 2] >> (16 * (k & 3))) & 0xFFFFull); }
__device__ __forceinline__ PendQ pq_pop(PendQ q) {
    PendQ r;
    r.w[0] = (q.w[0] >> 16) | (q.w[1] << 48);
    r.w[1] = (q.w[1] >> 16) | (q.w[2] << 48);
    r.w[2] = (q.w[2] >> 16) | (q.w[3] << 48);
    r.w[3] = q.w[3] >> 16;
    return r;
}
// enqueue group g at the tail; false when the FIFO is full
__device__ __forceinline__ bool pq_push(PendQ &q, int g) {
    for (int k = 0; k < MT_PQ_IDS; k++)
        if (pq_at(q, k) == 0) {
            q.w[k >> 2] |= (u64)(uint32_t)g << (16 * (k & 3));
            return true;
        }
    return false;
}
__device__ __forceinline__ PendQ pq_bcast(const PendQ &q, int l) {
    return PendQ{{bcast64(q.w[0], l), bcast64(q.w[1], l), bcast64(q.w[2], l), bcast64(q.w[3], l)}};
}
// breakTie for the local client's own insert (MT/mergeTree.ts:2290-2298: "local change see
// everything" after the removed-at-or-below-refSeq test)
__device__ __forceinline__ bool tie_local(v4i a, int r) {
    const int rs = a.z;
    return !((rs != MT_RSEQ_NONE) & (rs != 0) & (rs <= r) & (rs != -1));
}
// breakTie for a remote client on a live document: an unacked local segment never ties
__device__ __forceinline__ bool tie_remote_live(v4i a, int r) { return tie(a, r) & !is_local_seq(a.y); }
