// mt_replay.hip -- HIP kernels and the C-ABI boundary (include/mt_replay.h) of the MI355X
// merge-tree replay backend.  Build: see fluidframework_amd/build.py (hipcc --offload-arch=gfx950).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mt_replay.h"
#include "mt_kernels.h"
#include "mt_variants.h"
#ifdef MT_SINGLE_TU
#define MT_VARIANT_DEF(n, k) const void *mtk_##n() { return (const void *)k; }
MT_VARIANTS(MT_VARIANT_DEF)
#endif

__global__ void __launch_bounds__(MT_WAVE) k_init(DevState st, const int64_t *seed_off,
                                                  const uint16_t *seed) {
    const int doc = blockIdx.x;
    if (doc >= st.n_docs) return;
    oslot_reset(st, doc);
    if (st.bslot && lane() == 0) st.bslot[doc] = -1;   // back to the main arrays
    const int64_t s0 = seed_off ? seed_off[doc] : 0, s1 = seed_off ? seed_off[doc + 1] : 0;
    const int len = (int)(s1 - s0);
    uint16_t *text = st.text + (size_t)doc * 2 * st.T;
    for (int j = lane(); j < len && j < st.T; j += MT_WAVE) text[j] = seed[s0 + j];
    if (lane() == 0) {
        init_doc_hdr(st, doc, len);
        st.retry[doc] = 0;
        // the seed segment is the root's only child: setOrdinal(child, 0) with childCount 1
        if (st.ordS) st.ordS[(size_t)doc * st.S] = 63;
        if (st.live) {   // collabWindow.localSeq 0, empty pending queue (next group id 1)
            st.live[4 * doc] = 0;
            st.live[4 * doc + 1] = 1;
            st.live[4 * doc + 2] = 0;
            st.live[4 * doc + 3] = 0;
        }
    }
}

// ---------------------------------------------------------------- summary load (config C5)
// Client.load -> SnapshotLoader.loadHeader (MT/snapshotLoader.ts:120-159): the header's
// segments become the leaves of a tree built bottom-up in blocks of MaxNodesInBlock - 1 = 7
// (reloadFromSegments MT/mergeTree.ts:1229-1284; new blocks: needsScour undefined), then
// startOrUpdateCollaboration(minSeq, seq) (MT/mergeTree.ts:1287-1304: fresh zamboni heap).
// Body segments are appended afterwards by replaying MT_F_LOAD records (mt_load_snapshots).
__global__ void __launch_bounds__(MT_WAVE) k_load_header(DevState st, const int64_t *off, const int32_t *nh,
                                                         const mt_seg_rec *segs, const uint16_t *tin,
                                                         const uint32_t *pin, const int32_t *min_seq,
                                                         const int32_t *cur_seq, LoadScratch sc, int lo) {
    // summary r of the set (off, nh, min_seq, cur_seq, sc.off index r) -> document lo + r
    const int r = blockIdx.x, doc = lo + r;
    if (doc >= st.n_docs) return;
    oslot_reset(st, doc);
    if (st.bslot && lane() == 0) st.bslot[doc] = -1;   // back to the main arrays
    const int n = nh[r];
    const mt_seg_rec *rs = segs + off[r];
    const bool big = sc.off && sc.off[2 * r] >= 0;
    uint16_t *text = st.text + (size_t)doc * 2 * st.T;
    uint32_t *props = st.props + (size_t)doc * 2 * st.P * MT_PREC;
    const int nb0 = n > 0 ? (n + MT_LOAD_FANOUT - 1) / MT_LOAD_FANOUT : 1;
    int status = !big && (n > st.S || nb0 > st.B) ? MT_DOC_CAPACITY : 0;
    const size_t B = big ? (size_t)nb0 : st.B;   // stride of a level's counts
    v4i *dA = big ? sc.A + sc.off[2 * r] : st.segA + doc * (size_t)st.S;
    u64 *dO = big ? sc.O + sc.off[2 * r] : st.segO + doc * (size_t)st.S;
    v4u *dB = big ? sc.B + sc.off[2 * r] : st.segB + doc * (size_t)st.S;
    int ttop = 0, ptop = 1;
    for (int base = 0; base < n && status == 0; base += MT_WAVE) {
        const int i = base + lane();
        const bool v = i < n;
        mt_seg_rec r;
        memset(&r, 0, sizeof(r));
        if (v) r = rs[i];
        const bool marker = (r.flags & MT_F_MARKER) != 0;
        const int tl = v && !marker ? r.len : 0;
        const int hp = v && r.props != MT_NO_PROPS ? 1 : 0;
        const int tinc = wave_scan_incl(tl), pinc = wave_scan_incl(hp);
        const int toff = ttop + tinc - tl, ph = ptop + pinc - hp;
        const int tend = ttop + bcast(tinc, MT_WAVE - 1), pend = ptop + bcast(pinc, MT_WAVE - 1);
        if (tend > st.T || pend > st.P) {
            status = MT_DOC_CAPACITY;
            break;
        }
        bool bad = false, nm = false;
        if (hp) {   // TextSegment.make / Marker.make(props): keys with null dropped (Q5)
            const uint32_t *rec = pin + r.props;
            const uint32_t cnt = rec[0] & 0xFFFF;
            uint32_t *t = props + (size_t)ph * MT_PREC;
            uint32_t k = 0;
            for (uint32_t j = 0; j < cnt; j++) {
                if (rec[2 + 2 * j] == MT_VAL_NULL) continue;
                if (k >= MT_KMAX) {
                    bad = true;
                    break;
                }
                t[1 + 2 * k] = rec[1 + 2 * j];
                t[2 + 2 * k] = rec[2 + 2 * j];
                nm = nm || (rec[2 + 2 * j] & MT_VAL_NOMATCH_BIT) != 0;
                k++;
            }
            t[0] = k;
        }
        if (ballot(bad)) {
            status = MT_DOC_CAPACITY;
            break;
        }
        // text: one wave-wide copy per segment of this chunk
        for (u64 m = ballot(tl > 0); m; m &= m - 1) {
            const int j = first_lane(m);
            const int lj = bcast(tl, j), oj = bcast(toff, j);
            const uint32_t sj = (uint32_t)bcast((int)r.payload, j);
            for (int q = lane(); q < lj; q += MT_WAVE) text[oj + q] = tin[sj + q];
        }
        if (v) {
            const bool rem = r.removed_seq != MT_RSEQ_NONE;
            uint32_t w = 0;
            if (tl > 0) w = SEGF_NL_KNOWN | (tin[r.payload + tl - 1] == '\n' ? SEGF_NL : 0u);
            if (nm) w |= SEGF_NOMATCH;
            dA[i] = v4i{r.len, r.seq, r.removed_seq, pack_cli(r.client, rem ? r.removed_client : 0)};
            dO[i] = 0ull;
            if (st.segP && !big) {   // no pending groups
                u64 *w = (u64 *)(st.segP + doc * (size_t)st.S + i);
                w[0] = w[1] = w[2] = w[3] = 0ull;
            }
            dB[i] = v4u{marker ? r.payload : (uint32_t)toff, hp ? (uint32_t)ph : 0u,
                        (uint32_t)(i + 1) | (marker ? MT_MARKER_BIT : 0u), w};
        }
        ttop = tend;
        ptop = pend;
    }
    // block counts, level by level (blocks of 7, the last one takes the rest)
    int nbl[MT_LV];
    int depth = 0, cnt_below = n > 0 ? n : 0, nl = nb0;
    uint8_t *cnt = big ? sc.cnt + MT_LV * sc.off[2 * r + 1] : st.cnt + (size_t)doc * MT_LV * B;
    int8_t *flg = big ? sc.flg + sc.off[2 * r + 1] : st.flg + (size_t)doc * B;
    for (int l = 0; l < MT_LV; l++) nbl[l] = 0;
    while (status == 0) {
        if (depth >= MT_LV) {
            status = MT_DOC_CAPACITY;
            break;
        }
        for (int b = lane(); b < nl; b += MT_WAVE)
            cnt[depth * B + b] = (uint8_t)min(MT_LOAD_FANOUT, cnt_below - MT_LOAD_FANOUT * b);
        nbl[depth] = nl;
        depth++;
        if (nl == 1) break;
        cnt_below = nl;
        nl = (nl + MT_LOAD_FANOUT - 1) / MT_LOAD_FANOUT;
    }
    for (int b = lane(); b < nb0 && (big || b < st.B); b += MT_WAVE) flg[b] = MT_SCOUR_UNDEF;
    if (st.ordS && !big && status == 0) {
        // reloadFromSegments ends with nodeUpdateOrdinals(root) (MT/mergeTree.ts:1273-1276):
        // child q of a block of c children gets (q + 1) * (1 << (7 - c)) - 1; children of
        // block p are [7p, 7p + c) one level down
        uint16_t *os = st.ordS + (size_t)doc * st.S;
        uint16_t *ob = st.ordB + (size_t)doc * MT_LV * st.B;
        for (int i = lane(); i < n; i += MT_WAVE) {
            const int c = cnt[i / MT_LOAD_FANOUT];
            os[i] = (uint16_t)((i % MT_LOAD_FANOUT + 1) * (1 << (7 - c)) - 1);
        }
        for (int l = 0; l + 1 < depth; l++)
            for (int b = lane(); b < nbl[l]; b += MT_WAVE) {
                const int c = cnt[(l + 1) * B + b / MT_LOAD_FANOUT];
                ob[(size_t)l * st.B + b] = (uint16_t)((b % MT_LOAD_FANOUT + 1) * (1 << (7 - c)) - 1);
            }
    }
    if (lane() == 0) {
        DocHdr h;
        memset(&h, 0, sizeof(h));
        h.n_seg = status ? 0 : n;
        h.depth = status ? 1 : depth;
        h.cur_seq = cur_seq[r];
        h.min_seq = min_seq[r];
        h.text_top = ttop;
        h.props_top = ptop;
        h.next_uid = n + 1;
        h.status = status;
        h.delta_hash = MT_FNV_OFF;
        for (int l = 0; l < MT_LV; l++) h.n_blk[l] = status ? (l == 0) : nbl[l];
        st.hdr[doc] = h;
        st.retry[doc] = 0;
    }
}

// ---------------------------------------------------------------- checksums
struct SumCtx {
    const uint32_t *props;
};
__device__ static bool same_ordered(const uint32_t *pr, uint32_t ha, uint32_t hb) {
    if (ha == 0 || hb == 0) return ha == hb;
    if (ha == hb) return true;
    const uint32_t *a = pr + (size_t)ha * MT_PREC, *b = pr + (size_t)hb * MT_PREC;
    if (a[0] != b[0]) return false;
    for (uint32_t i = 0; i < 2 * a[0]; i++)
        if (a[1 + i] != b[1 + i]) return false;
    return true;
}
__device__ static u64 fold_run(const uint32_t *pr, u64 h, uint32_t ph, int len) {
    h = fnv_u32(h, (uint32_t)len);
    h = fnv_u32(h, ph ? 1u : 0u);
    if (ph) {
        const uint32_t *p = pr + (size_t)ph * MT_PREC;
        h = fnv_u32(h, p[0]);
        for (uint32_t i = 0; i < 2 * p[0]; i++) h = fnv_u32(h, p[1 + i]);
    }
    return h;
}
// mt_checksum per document (definitions: DESIGN.md "Checksums", oracle/mt_oracle.c).
// Segment ranges of a document in document order: the flat table, or its pages.
struct SegRanges {
    const v4i *A;
    const v4u *B;
    int n;
    bool paged;
    const uint16_t *dir;
    const PageMeta *meta;
    int nr;
    __device__ int count() const { return nr; }
    __device__ void get(int r, const v4i *&a, const v4u *&b, int &cnt) const {
        if (!paged) {
            a = A;
            b = B;
            cnt = n;
            return;
        }
        const int pg = dir[r];
        a = A + (size_t)pg * MT_PG_SLOTS;
        b = B + (size_t)pg * MT_PG_SLOTS;
        cnt = meta[pg].nseg;
    }
};
__device__ static SegRanges seg_ranges(const DevState &st, int doc, const DocHdr &h) {
    SegRanges R;
    R.paged = h.pad[HDR_PAGED] != 0;
    if (R.paged) {
        const PagedBase b = doc_paged(st, doc);
        R.A = b.A;
        R.B = b.B;
        R.dir = b.dir;
        R.meta = b.meta;
        R.nr = h.pad[HDR_NPAGES];
        R.n = 0;
    } else {
        R.A = st.segA + doc * (size_t)st.S;
        R.B = st.segB + doc * (size_t)st.S;
        R.n = h.n_seg;
        R.nr = 1;
        R.dir = nullptr;
        R.meta = nullptr;
    }
    return R;
}

// SnapshotV1.extractSync (MT/snapshotV1.ts:156-252) of a document's current state: walk the
// leaves in order; drop unacked segments and those removed at or below minSeq; coalesce runs
// of below-minSeq, unremoved segments while TextSegment.canAppend and matchProperties hold
// (MT/textSegment.ts:62-67, MT/properties.ts:61-92: the run's text is copied out once, as
// the clone + append chain builds it); everything else is emitted with its merge info.
// mode 0 counts {records, text units, props words} per document into io[3*doc]; mode 1
// writes them at the offsets io holds (the host's prefix sums).  One wave per document; the
// per-segment decisions are uniform, text copies are wave-wide.
__device__ static bool props_equal_set(const uint32_t *pr, uint32_t ha, uint32_t hb) {
    if (ha == 0 || hb == 0) return ha == hb;
    const uint32_t *a = pr + (size_t)ha * MT_PREC, *b = pr + (size_t)hb * MT_PREC;
    for (uint32_t i = 0; i < a[0]; i++)   // NaN / undefined values never match
        if (a[2 + 2 * i] & MT_VAL_NOMATCH_BIT) return false;
    for (uint32_t j = 0; j < b[0]; j++)
        if (b[2 + 2 * j] & MT_VAL_NOMATCH_BIT) return false;
    if (ha == hb) return true;
    if (a[0] != b[0]) return false;
    for (uint32_t i = 0; i < a[0]; i++) {
        bool ok = false;
        for (uint32_t j = 0; j < b[0]; j++)
            if (b[1 + 2 * j] == a[1 + 2 * i]) ok = b[2 + 2 * j] == a[2 + 2 * i];
        if (!ok) return false;
    }
    return true;
}
__global__ void __launch_bounds__(MT_WAVE) k_extract(DevState st, int mode, int64_t *io, mt_seg_rec *recs,
                                                     uint16_t *text_out, uint32_t *props_out, int32_t *win) {
    const int doc = blockIdx.x;
    if (doc >= st.n_docs) return;
    const DocHdr h = st.hdr[doc];
    const SegRanges R = seg_ranges(st, doc, h);
    const PagedBase ar = doc_paged(st, doc);   // (the arenas of the document's region)
    const uint16_t *tb = ar.text + (size_t)h.text_half * ar.T;
    const uint32_t *pr = ar.props + (size_t)h.props_half * ar.P * MT_PREC;
    const int ms = h.min_seq;
    int64_t nrec = 0, ntext = 0, nprop = 0;
    const int64_t rbase = mode ? io[3 * doc] : 0, tbase = mode ? io[3 * doc + 1] : 0, pbase = mode ? io[3 * doc + 2] : 0;
    // the coalescing candidate ("prev"): an open record
    bool open = false, p_marker = false, p_nl = false;
    int p_len = 0;
    uint32_t p_props = 0;
    int64_t p_rec = 0;
    auto emit = [&](const v4i a, const v4u b, uint32_t flags, int seq, int cli) {
        // a new record for segment (a, b); returns nothing, advances the counters
        const bool marker = (b.z & MT_MARKER_BIT) != 0;
        const int len = a.x;
        if (mode && lane() == 0) {
            mt_seg_rec r;
            memset(&r, 0, sizeof(r));
            r.len = len;
            r.seq = seq;
            r.removed_seq = a.z;
            r.client = (int16_t)cli;
            r.removed_client = a.z != MT_RSEQ_NONE ? (int16_t)seg_rcli(a) : (int16_t)0;
            r.flags = (uint8_t)(flags | (marker ? MT_F_MARKER : 0));
            r.payload = marker ? b.x : (uint32_t)(ntext);
            r.props = MT_NO_PROPS;
            if (b.y) {
                const uint32_t *src = pr + (size_t)b.y * MT_PREC;
                r.props = (uint32_t)nprop;
                uint32_t *dst = props_out + pbase + nprop;
                dst[0] = src[0];
                for (uint32_t k = 0; k < 2 * src[0]; k++) dst[1 + k] = src[1 + k];
            }
            recs[rbase + nrec] = r;
        }
        if (b.y) nprop += 1 + 2 * (int64_t)pr[(size_t)b.y * MT_PREC];
        if (!marker) {
            if (mode)
                for (int q = lane(); q < len; q += MT_WAVE) text_out[tbase + ntext + q] = tb[b.x + q];
            ntext += len;
        }
        nrec++;
    };
    for (int rr = 0; rr < R.count(); rr++) {
        const v4i *A;
        const v4u *Bv;
        int n;
        R.get(rr, A, Bv, n);
        for (int i = 0; i < n; i++) {
            const v4i a = uni4(A[i]);
            const v4u b = uni4(Bv[i]);
            const int seq = a.y, rseq = a.z;
            const bool removed = rseq != MT_RSEQ_NONE;
            if (seq == -1 || (removed && rseq <= ms)) continue;            // :189-191
            const bool marker = (b.z & MT_MARKER_BIT) != 0;
            if (seq <= ms && (!removed || rseq == -1)) {                   // :196-215 coalesce
                const bool nl = !marker && a.x > 0 && tb[b.x + a.x - 1] == '\n';
                const bool can = open && !p_marker && !marker && !p_nl &&
                                 (p_len <= MT_GRAN || a.x <= MT_GRAN) && props_equal_set(pr, p_props, b.y);
                if (can) {   // prev.clone().append(segment.clone())
                    if (mode)
                        for (int q = lane(); q < a.x; q += MT_WAVE) text_out[tbase + ntext + q] = tb[b.x + q];
                    ntext += a.x;
                    p_len += a.x;
                    if (a.x > 0) p_nl = nl;   // "".endsWith("\n") leaves the run's ending
                    if (mode && lane() == 0) recs[rbase + p_rec].len = p_len;
                } else {     // pushSeg(prev); prev = segment
                    p_rec = nrec;
                    emit(a, b, 0u, 0, -2);
                    open = true;
                    p_marker = marker;
                    p_nl = nl;
                    p_len = a.x;
                    p_props = b.y;
                }
            } else {                                                        // :216-242 merge info
                open = false;
                const bool above = seq > ms;
                uint32_t f = MT_SEG_MERGE_INFO | (above ? MT_SEG_HAS_SEQ : 0u);
                emit(a, b, f, above ? seq : 0, above ? seg_cli(a) : -2);
            }
        }
    }
    if (mode == 0 && lane() == 0) {
        io[3 * doc] = nrec;
        io[3 * doc + 1] = ntext;
        io[3 * doc + 2] = nprop;
    }
    if (lane() == 0 && win) {
        win[2 * doc] = h.min_seq;
        win[2 * doc + 1] = h.cur_seq;
    }
}

// mt_checksum per document (definitions: DESIGN.md "Checksums", oracle/mt_oracle.c).
__global__ void __launch_bounds__(MT_WAVE) k_checksum(DevState st, mt_checksum *out) {
    const int doc = blockIdx.x;
    if (doc >= st.n_docs) return;
    const DocHdr h = st.hdr[doc];
    const SegRanges R = seg_ranges(st, doc, h);
    const PagedBase ar = doc_paged(st, doc);   // (the arenas of the document's region)
    const uint16_t *tb = ar.text + (size_t)h.text_half * ar.T;
    const uint32_t *pr = ar.props + (size_t)h.props_half * ar.P * MT_PREC;
    int len = 0, ntext = 0, nseg = 0;
    for (int r = 0; r < R.count(); r++) {
        const v4i *A;
        const v4u *Bv;
        int n;
        R.get(r, A, Bv, n);
        nseg += n;
        for (int base = 0; base < n; base += MT_WAVE) {
            const int i = base + lane();
            int l = 0, t = 0;
            if (i < n) {
                const v4i a = A[i];
                l = obs_len(a);
                t = (Bv[i].z & MT_MARKER_BIT) ? 0 : l;
            }
            len += wave_sum(l);
            ntext += wave_sum(t);
        }
    }
    if (lane() == 0) {
        u64 th = fnv_u32(MT_FNV_OFF, (uint32_t)ntext), hk = MT_FNV_OFF, ph = MT_FNV_OFF;
        int g = 0, run_len = 0;
        bool have = false;
        uint32_t run_p = 0;
        for (int r = 0; r < R.count(); r++) {
            const v4i *A;
            const v4u *Bv;
            int n;
            R.get(r, A, Bv, n);
            for (int i = 0; i < n; i++) {
                const v4i a = A[i];
                const v4u b = Bv[i];
                if (a.z != MT_RSEQ_NONE) continue;
                if (!(b.z & MT_MARKER_BIT)) {
                    for (int j = 0; j < a.x; j++) {
                        const uint16_t ch = tb[b.x + j];
                        hk ^= ch & 0xFF;
                        hk *= MT_FNV_PRIME;
                        hk ^= ch >> 8;
                        hk *= MT_FNV_PRIME;
                        g++;
                        if ((g & 63) == 0) {
                            th = fnv_u64(th, hk);
                            hk = MT_FNV_OFF;
                        }
                    }
                }
                if (have && same_ordered(pr, run_p, b.y)) {
                    run_len += a.x;
                } else {
                    if (have) ph = fold_run(pr, ph, run_p, run_len);
                    run_p = b.y;
                    run_len = a.x;
                    have = true;
                }
            }
        }
        if (g & 63) th = fnv_u64(th, hk);
        if (have) ph = fold_run(pr, ph, run_p, run_len);
        mt_checksum cs;
        cs.length = (uint32_t)len;
        cs.n_segments = (uint32_t)nseg;
        cs.text_hash = th;
        cs.props_hash = ph;
        cs.delta_hash = h.delta_hash;
        out[doc] = cs;
    }
}

// ============================================================================ host side
// ---------------------------------------------------------------- live-client reconnect
// regeneratePendingOp for the oldest pending segment group of one document (one wave):
// resetPendingDeltaToOps (MT/client.ts:709-766) with findReconnectionPostition (:675-707) --
// a segment counts towards the positions when it is inserted (acked, or localSeq <= the
// group's) and not removed (or removed by a local op newer than the group).  Members in
// document order (the reference sorts by ordinal); each one that yields an op joins a new
// group (same localSeq, kind, keys) at the tail of the queue.  io: [0] records written
// (-1: no pending group, -2: a capacity, -3: the document has failed), [1] text units,
// [2] props words.
__global__ void __launch_bounds__(MT_WAVE) k_regen(DevState st, int doc, mt_regen_rec *out, int cap, uint16_t *otext,
                                                   int tcap, uint32_t *oprops, int pcap, int32_t *io) {
    typedef TierLiveT<false> T;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const LdsLayout L = lds_layout(false, 0, st.B, 0, 0);
    DocT<T> d;
    load_doc(d, st, doc, (LDS_AS uint8_t *)smem_raw, L, 0, st.B, 0);
    if (d.status || d.g_n == 0) {
        if (lane() == 0) io[0] = d.status ? -3 : -1;
        return;
    }
    const int g = d.g_head;
    const int gw = lane() < MT_GRP_WORDS ? d.grp[g * MT_GRP_WORDS + lane()] : 0;   // the entry, lane j = word j
    const int ls = bcast(gw, 0), kind = bcast(gw, 1) & 0xFF;
    {   // sizing pass (reads only): output buffers too small leave the document untouched --
        // the caller retries with the sizes in io[1..3]
        int need_n = 0, need_t = 0, need_p = 0;
        for (int base = 0; base < d.n; base += MT_WAVE) {
            const int i = base + lane();
            const bool v = i < d.n;
            v4i a;
            u64 o;
            load_ao(d, i, v, a, o);
            const v4u b = d.Bv[v ? i : 0];
            const bool mem = v && pq_first(pq_get(d, v ? i : 0)) == g;
            const bool emit = mem && (kind != MT_OP_REMOVE || is_local_seq(a.z));
            const bool mk = (b.z & MT_MARKER_BIT) != 0;
            const int np = emit && kind == MT_OP_INSERT && b.y ? (int)prec(d, d.props_half, b.y)[0] : -1;
            need_n += __popcll(ballot(emit));
            need_t += wave_sum(emit && kind == MT_OP_INSERT && !mk ? a.x : 0);
            need_p += wave_sum(np >= 0 ? 1 + 2 * np : 0);
        }
        if (need_n > cap || need_t > tcap || need_p > pcap) {
            if (lane() == 0) {
                io[0] = -4;
                io[1] = need_n;
                io[2] = need_t;
                io[3] = need_p;
            }
            return;
        }
        if (d.g_n - 1 + need_n > d.LG) {   // the new groups need more ids: the live growth step first
            if (lane() == 0) {
                io[0] = -5;
                io[1] = d.g_n - 1 + need_n;
            }
            return;
        }
    }
    d.g_head = g % d.LG + 1;   // dequeue first: the new groups may reuse its table slot
    d.g_n--;
    int carry = 0, nout = 0, tu = 0, pw = 0;
    bool over = false;
    for (int base = 0; base < d.n && !over; base += MT_WAVE) {
        const int i = base + lane();
        const bool v = i < d.n;
        v4i a;
        u64 o;
        load_ao(d, i, v, a, o);
        const v4u b = d.Bv[v ? i : 0];
        const bool ins = !is_local_seq(a.y) || a.y - MT_LOCAL_BASE <= ls;
        const bool nrem = a.z == MT_RSEQ_NONE || (is_local_seq(a.z) && a.z - MT_LOCAL_BASE > ls);
        const int cl = v && ins && nrem ? a.x : 0;
        const int inc = wave_scan_incl(cl);
        const int pos = carry + inc - cl;
        const PendQ pq = pq_get(d, v ? i : 0);
        const bool mem = v && pq_first(pq) == g;
        for (u64 m = ballot(mem); m && !over; m &= m - 1) {
            const int j = first_lane(m);
            const int ij = base + j;
            PendQ oj = pq_pop(pq_bcast(pq, j));
            const int aj_x = bcast(a.x, j), aj_z = bcast(a.z, j);
            const bool emit = kind != MT_OP_REMOVE || is_local_seq(aj_z);
            if (emit) {
                const uint32_t bx = (uint32_t)bcast((int)b.x, j), by = (uint32_t)bcast((int)b.y, j);
                const bool mk = (bcast((int)b.z, j) & MT_MARKER_BIT) != 0;
                const int np = (kind == MT_OP_INSERT && by) ? (int)prec(d, d.props_half, by)[0] : -1;
                const int ng = (d.g_head - 1 + d.g_n) % d.LG + 1;
                const int tneed = kind == MT_OP_INSERT && !mk ? aj_x : 0;
                if (nout >= cap || d.g_n >= d.LG || !pq_push(oj, ng) || tu + tneed > tcap ||
                    pw + 1 + 2 * max(np, 0) > pcap) {
                    over = true;
                    break;
                }
                // same localSeq / kind / keys; joined now (its later splits append after it)
                if (lane() < MT_GRP_WORDS) d.grp[ng * MT_GRP_WORDS + lane()] = lane() == 10 ? d.next_uid : gw;
                d.g_n++;
                if (lane() == 0) {
                    mt_regen_rec r;
                    r.kind = kind;
                    r.pos1 = bcast(pos, j);
                    r.pos2 = kind == MT_OP_INSERT ? r.pos1 : r.pos1 + aj_x;
                    r.local_seq = ls;
                    r.text_off = mk ? bx : (uint32_t)tu;
                    r.text_len = (uint32_t)aj_x;
                    r.props_off = np >= 0 ? (uint32_t)pw : MT_NO_PROPS;
                    r.flags = mk ? MT_F_MARKER : 0u;
                    out[nout] = r;
                }
                if (kind == MT_OP_INSERT) {
                    gsync_rd();
                    if (!mk)
                        for (int q = lane(); q < aj_x; q += MT_WAVE) otext[tu + q] = text_base(d, d.text_half)[bx + q];
                    if (np >= 0) {
                        const GLB_AS uint32_t *pr = prec(d, d.props_half, by);
                        for (int q = lane(); q < 1 + 2 * np; q += MT_WAVE) oprops[pw + q] = pr[q];
                    }
                    tu += tneed;
                    pw += np >= 0 ? 1 + 2 * np : 0;
                }
                nout++;
            }
            if (lane() == 0) pq_put(d, ij, oj);
        }
        carry += bcast(inc, MT_WAVE - 1);
    }
    if (over) {   // the group table / a segment's FIFO is full (the buffers were sized above)
        d.status = MT_DOC_CAPACITY;
        d.cap_cause = 15;
    }
    store_doc(d, st, doc);
    if (lane() == 0) {
        io[0] = over ? -2 : nout;
        io[1] = tu;
        io[2] = pw;
    }
}

struct mt_handle {
    int device = 0;
    bool live = false;       // live-client handle (mt_options.live_client)
    bool ordinals = false;   // segment ordinals kept (mt_options.segment_ordinals)
    uint32_t n_docs = 0;
    DevState st{};
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_load = nullptr, ev_load1 = nullptr;
    bool load_timed = false;   // ev_load / ev_load1 bracket the last snapshot load's kernels
    // documents per workgroup of the LDS-tier replay (env MT_WPG=2 for two): measured on C2
    // the CU saturates at 16 resident documents (16 -> 18 per CU: 61.8 -> 64.6 ms)
    int wpg = 1;
    float last_ms = 0.f;
    bool timed = false;      // ev0/ev1 bracket a launch not yet read by mt_sync
    std::string err;
    mt_checksum *d_sums = nullptr;
    int64_t *d_seed_off = nullptr;   // initial contents kept on device for mt_reset
    uint16_t *d_seed = nullptr;
    TierCaps lds{0, 0, 0, 0};        // LDS-tier capacities (S == 0: tier disabled)
    PagedCaps pg_tight{0, 0, 0, 1, 1, 0};   // tight paged tier (PP == 0: off)
    PagedCaps pg_full{0, 0, 0, 0, 1, 0};    // paged tier at the HBM capacities
    int paged_slices = 0;                   // mt_options.paged_slices
    int pg_resident = 0;                    // documents resident at once in a tight paged launch
    // growth step (mt_settle): the batch whose launches may have handed documents to it, the
    // big region's capacities (PP == 0: none yet) and its slots, the documents moved there
    struct mt_batch *pending = nullptr;
    PagedCaps big_caps{0, 0, 0, 0, 3, 0, 1};
    std::vector<int32_t> bslot_h;           // host mirror of st.bslot
    uint32_t n_big = 0;                     // documents with a slot in the big region
    int max_cli = 0;                        // largest |short client id| any batch / load / generation used
                                            // (<= 127: the tight tier may pack its table, PagedCaps.packed)
    uint32_t grown_last = 0, grow_rounds_last = 0;
};
struct mt_batch {
    mt_handle *owner = nullptr;   // the handle whose growth step still needs this batch
    int device = 0;
    uint32_t n_docs = 0;
    uint64_t n_ops = 0, text_len = 0, props_len = 0;
    int64_t *off = nullptr;
    mt_op_rec *ops = nullptr;
    uint16_t *text = nullptr;
    uint32_t *props = nullptr;
    int32_t *order = nullptr;     // dispatch order (DevState.order), null when lengths are equal
};
// Longest-first dispatch order of a batch whose documents differ in length (stable: equal
// lengths keep index order); none when every document has the same number of messages.
static bool set_order(mt_batch *b, const int64_t *off) {
    const uint32_t n = b->n_docs;
    bool equal = true;
    for (uint32_t d = 1; d < n && equal; d++) equal = off[d + 1] - off[d] == off[1] - off[0];
    if (equal) return true;
    std::vector<int32_t> ord(n);
    for (uint32_t d = 0; d < n; d++) ord[d] = (int32_t)d;
    std::stable_sort(ord.begin(), ord.end(),
                     [&](int32_t x, int32_t y) { return off[x + 1] - off[x] > off[y + 1] - off[y]; });
    return hipMalloc(&b->order, (size_t)n * 4) == hipSuccess &&
           hipMemcpy(b->order, ord.data(), (size_t)n * 4, hipMemcpyHostToDevice) == hipSuccess;
}

#define HIPCHK(h, x)                                                               \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            if (h) (h)->err = std::string(#x) + ": " + hipGetErrorString(e_);      \
            return MT_E_HIP;                                                       \
        }                                                                          \
    } while (0)

// Launches through the kernel pointers of mt_variants.h (hipLaunchKernel with the kernels'
// exact parameter types; errors are read with hipGetLastError as for hipLaunchKernelGGL)
static void launch_replay(const void *k, dim3 g, dim3 b, size_t lds, hipStream_t s, DevState st, const mt_op_rec *ops,
                          const int64_t *off, const uint16_t *tin, const uint32_t *pin, TierCaps caps) {
    void *a[] = {&st, &ops, &off, &tin, &pin, &caps};
    (void)hipLaunchKernel(k, g, b, a, lds, s);
}
static void launch_replay_paged(const void *k, dim3 g, dim3 b, size_t lds, hipStream_t s, DevState st,
                                const mt_op_rec *ops, const int64_t *off, const uint16_t *tin, const uint32_t *pin,
                                int use_resume, PagedCaps pc, PagedSlice sl) {
    void *a[] = {&st, &ops, &off, &tin, &pin, &use_resume, &pc, &sl};
    (void)hipLaunchKernel(k, g, b, a, lds, s);
}
static void launch_generate(const void *k, dim3 g, dim3 b, size_t lds, hipStream_t s, DevState st, mt_gen_cfg cfg,
                            uint32_t doc_base, mt_op_rec *ops_out, uint16_t *text_out, uint32_t *props_out,
                            int64_t tstride, int64_t pstride, int32_t *fail_out, int32_t *dbg_len, int64_t *used_out,
                            TierCaps caps) {
    void *a[] = {&st, &cfg, &doc_base, &ops_out, &text_out, &props_out, &tstride, &pstride, &fail_out, &dbg_len,
                 &used_out, &caps};
    (void)hipLaunchKernel(k, g, b, a, lds, s);
}
static void launch_generate_paged(const void *k, dim3 g, dim3 b, size_t lds, hipStream_t s, DevState st,
                                  mt_gen_cfg cfg, uint32_t doc_base, mt_op_rec *ops_out, uint16_t *text_out,
                                  uint32_t *props_out, int64_t tstride, int64_t pstride, int32_t *fail_out,
                                  int32_t *dbg_len, int64_t *used_out, PagedCaps pc) {
    void *a[] = {&st, &cfg, &doc_base, &ops_out, &text_out, &props_out, &tstride, &pstride, &fail_out, &dbg_len,
                 &used_out, &pc};
    (void)hipLaunchKernel(k, g, b, a, lds, s);
}
static void launch_load_convert(const void *k, dim3 g, dim3 b, size_t lds, hipStream_t s, DevState st, LoadScratch sc,
                                PagedCaps pc, int lo) {
    void *a[] = {&st, &sc, &pc, &lo};
    (void)hipLaunchKernel(k, g, b, a, lds, s);
}

static int mt_settle(mt_handle *h);
// waits for the stream and finishes a pending growth step (API entry points that read state or
// enqueue work: a growth step's launches must come before anything else)
#define SETTLE(h)                          \
    do {                                   \
        const int rc_ = mt_settle(h);      \
        if (rc_) return rc_;               \
    } while (0)

static TierCaps glb_caps(const mt_handle *h) { return TierCaps{0, h->st.B, 0, h->lds.S > 0 ? 1 : 0}; }
// the live handle's HBM tier: documents that could outgrow it go to the live growth step
static TierCaps live_caps(const mt_handle *h) {
    TierCaps c = glb_caps(h);
    c.grow = 1;
    return c;
}

// A props record [count | combine << 16, (key, value) x count] lies inside the arena.
static bool props_rec_ok(const uint32_t *props, uint64_t props_len, uint32_t off) {
    if (off == MT_NO_PROPS) return true;
    if ((uint64_t)off >= props_len) return false;
    const uint64_t cnt = props[off] & 0xFFFFu;
    uint64_t end = (uint64_t)off + 1 + 2 * cnt;
    if ((props[off] >> 16) == MT_COMBINE_TABLE) {   // + [n, absent, (old, new) x n]
        if (end + 2 > props_len) return false;
        end += 2 + 2 * (uint64_t)props[end];
    }
    return end <= props_len;
}
// Host-side bounds check of a batch (MT_E_INVALID instead of a device fault): per-document
// offsets monotonic inside [0, n_ops], every insert payload inside the text arena, every
// props record inside the props arena, known op kinds.
// (one pass over the records: also the largest |short client id| they name, for max_cli)
static std::string validate_batch(uint32_t n_docs, const int64_t *off, const mt_op_rec *ops, uint64_t n_ops,
                                  uint64_t text_len, const uint32_t *props, uint64_t props_len, bool live,
                                  int &max_cli) {
    if (off[0] < 0) return "doc_op_off[0] < 0";
    for (uint32_t d = 0; d < n_docs; d++)
        if (off[d + 1] < off[d]) return "doc_op_off not monotonic at document " + std::to_string(d);
    if ((uint64_t)off[n_docs] > n_ops) return "doc_op_off exceeds n_ops";
    int mc = max_cli;
    for (uint64_t k = (uint64_t)off[0]; k < (uint64_t)off[n_docs]; k++) {
        const mt_op_rec &o = ops[k];
        mc = std::max(mc, std::abs((int)(int16_t)o.client));
        if (o.kind > MT_OP_LOAD_ALIASED) return "op " + std::to_string(k) + ": unknown kind";
        if (o.kind >= MT_OP_LOAD_REMOVED && !(o.flags & MT_F_LOAD))
            return "op " + std::to_string(k) + ": summary-load record without MT_F_LOAD";
        if ((o.flags & (MT_F_LOCAL | MT_F_ACK)) && !live)
            return "op " + std::to_string(k) + ": local / ack record on a handle without live_client";
        if ((o.flags & MT_F_LOCAL) && (o.flags & MT_F_ACK))
            return "op " + std::to_string(k) + ": both MT_F_LOCAL and MT_F_ACK";
        if ((o.flags & MT_F_LOCAL) && o.client != 0)
            return "op " + std::to_string(k) + ": a local op's client must be the local client (short id 0)";
        if (o.kind == MT_OP_INSERT && !(o.flags & MT_F_MARKER)) {
            if (o.pos2 < 0 || (uint64_t)o.payload + (uint64_t)o.pos2 > text_len)
                return "op " + std::to_string(k) + ": insert payload outside the text arena";
        }
        if ((o.kind == MT_OP_INSERT || o.kind == MT_OP_ANNOTATE) && !props_rec_ok(props, props_len, o.props))
            return "op " + std::to_string(k) + ": props record outside the props arena";
    }
    max_cli = mc;
    return std::string();
}
static size_t tier_lds_bytes(bool seg_in_lds, const TierCaps &c, int gen_words) {
    return lds_layout(seg_in_lds, c.S, c.B, c.H, gen_words).total;
}

extern "C" {

mt_handle *mt_create(uint32_t n_docs, const mt_options *opt) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return nullptr;
    mt_options o{};
    if (opt) o = *opt;
    // the default handle is unbounded: the paged layout with the growth step behind it, at
    // small starting capacities (a flat-only handle is opt-in: page_capacity < 0); live
    // handles stay flat
    const bool dflt_paged = o.page_capacity == 0 && o.live_client == 0;
    if (dflt_paged) {
        o.page_capacity = 64;
        if (o.page_heap_capacity <= 0) o.page_heap_capacity = 256;
        if (o.unsettled_capacity <= 0) o.unsettled_capacity = 256;
        if (o.uid_capacity <= 0) o.uid_capacity = 8192;
        if (o.seg_capacity <= 0) o.seg_capacity = 512;
    }
    if (o.page_capacity < 0) o.page_capacity = 0;
    auto *h = new mt_handle();
    h->device = o.device;
    h->n_docs = n_docs;
    if (hipSetDevice(h->device) != hipSuccess) {
        delete h;
        return nullptr;
    }
    DevState &st = h->st;
    st.n_docs = (int32_t)n_docs;
    st.S = o.seg_capacity > 0 ? o.seg_capacity : 2048;
    st.B = o.block_capacity > 0 ? o.block_capacity : std::max(64, st.S / 2);
    st.B = (st.B + 63) / 64 * 64;
    st.H = o.heap_capacity > 0 ? o.heap_capacity : 2 * st.S;
    st.T = o.text_capacity > 0 ? o.text_capacity : 32768;
    st.P = o.props_capacity > 0 ? o.props_capacity : st.S + 2 * MT_WAVE;
    st.DL = o.delta_log_capacity > 0 ? o.delta_log_capacity : 0;
    st.DLR = st.DL > 0 && o.delta_log_mode == 1 ? 1 : 0;
    h->ordinals = o.segment_ordinals != 0;
    if (h->ordinals && !st.DLR) {   // ordinals ride on the rich log
        delete h;
        return nullptr;
    }
    if (const char *e = getenv("MT_WPG")) h->wpg = atoi(e) == 1 ? 1 : 2;
    h->live = o.live_client != 0;
    if (h->live && o.page_capacity > 0) {   // live documents replay from the flat HBM tier
        delete h;
        return nullptr;
    }
    // live handles stage in LDS (TierLiveLdsT, then TierLiveT) only when asked for explicitly
    if (o.lds_seg_capacity > 0 || (o.lds_seg_capacity == 0 && !h->live)) {
        int S_l = o.lds_seg_capacity > 0 ? o.lds_seg_capacity : 192;
        S_l = std::min(S_l, st.S);
        h->lds.S = S_l;
        h->lds.B = std::min(st.B, std::max(64, (S_l / 2 + 32 + 15) / 16 * 16));
        // zamboni heap in LDS: entries older than minSeq are popped as ops arrive, so the
        // heap stays far below S_l (C2 needs < 96 at S_l 192: 0 hand-overs); a smaller heap
        // is a smaller LDS footprint = more documents per CU (profiles/r1 sweep: 74.9 -> 68.9 ms)
        h->lds.H = std::min(st.H, std::max(64, S_l / 2));
        if (tier_lds_bytes(true, h->lds, 0) > 60 * 1024) h->lds = TierCaps{0, 0, 0, 0};
    }
    if (o.page_capacity > 0) {
        st.PP = std::min(o.page_capacity, 65535);
        st.PH = o.page_heap_capacity > 0 ? o.page_heap_capacity : 1024;
        st.UT = o.unsettled_capacity > 0 ? o.unsettled_capacity : 256;
        st.UM = std::min(o.uid_capacity > 0 ? o.uid_capacity : 65536, 1 << 24);
        st.UM = std::max(st.UM, 256);
        h->pg_full = PagedCaps{st.PP, st.PH, st.UT, 0, 1, 0, 1};
        const PagedCaps t{o.lds_page_capacity > 0 ? std::min(o.lds_page_capacity, st.PP) : st.PP,
                          o.lds_page_heap_capacity > 0 ? std::min(o.lds_page_heap_capacity, st.PH) : st.PH,
                          o.lds_unsettled_capacity > 0 ? std::min(o.lds_unsettled_capacity, st.UT) : st.UT, 1, 1,
                          o.lds_narrow_overlap ? 1 : 0};
        if (t.PP < st.PP || t.PH < st.PH || t.UT < st.UT || t.narrow) {
            h->pg_tight = t;
            h->pg_full.stage = 2;
        }
        // one document's paged state staged in LDS: up to the CU's 160 KiB (fewer
        // documents per CU above 64 KiB)
        const size_t lb = paged_layout(st.PP, st.PH, st.UT, 2 * 65, 8).total;
        if (lb > 160 * 1024) {
            delete h;
            return nullptr;
        }
        if (lb > 64 * 1024) {
            const void *ks[] = {MTK(P_LOG), MTK(P_FULL), MTK(P_HM), MTK(P_HM_LOG),
                                MTK(GP_FULL),
                                MTK(P_NARROW_LOG),
                                MTK(P_NARROW),
                                MTK(GP_NARROW),
                                MTK(LC_FAST),
                                MTK(LC_LOG),
                                MTK(P_PACKED_LOG),
                                MTK(P_PACKED)};
            for (const void *k : ks)
                if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb) != hipSuccess) {
                    delete h;
                    return nullptr;
                }
        }
        // documents resident at once in the first paged launch (the sliced schedule's round)
        h->paged_slices = std::min(std::max(o.paged_slices, 0), 256);
        if (h->paged_slices > 1) {
            const PagedCaps &c = h->pg_tight.PP ? h->pg_tight : h->pg_full;
            const size_t lt = paged_layout(c.PP, c.PH, c.UT, 0, c.narrow ? 4 : 8).total;
            const void *k = st.DL ? (c.narrow ? MTK(P_NARROW_LOG)
                                              : MTK(P_LOG))
                                  : (c.narrow ? MTK(P_NARROW)
                                              : MTK(P_FULL));
            int per_cu = 0, cus = 0;
            hipDeviceProp_t prop;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, MT_WAVE, lt) == hipSuccess &&
                hipGetDeviceProperties(&prop, h->device) == hipSuccess)
                cus = prop.multiProcessorCount;
            h->pg_resident = per_cu * cus;
        }
    }
    const size_t N = n_docs;
    bool ok = true;
    auto alloc = [&](void **p, size_t bytes) {
        if (!ok) return;
        if (hipMalloc(p, bytes ? bytes : 16) != hipSuccess) ok = false;
    };
    alloc((void **)&st.hdr, N * sizeof(DocHdr));
    alloc((void **)&st.segA, N * st.S * sizeof(int4));
    alloc((void **)&st.segO, N * st.S * sizeof(u64));
    alloc((void **)&st.segB, N * st.S * sizeof(uint4));
    alloc((void **)&st.cnt, N * MT_LV * st.B);
    alloc((void **)&st.flg, N * st.B);
    alloc((void **)&st.heap, N * (size_t)(st.H + 1) * sizeof(int2));
    alloc((void **)&st.oslot, N * (size_t)(2 * MT_OSLOTS) * sizeof(int32_t));
    alloc((void **)&st.text, N * 2 * (size_t)st.T * sizeof(uint16_t));
    alloc((void **)&st.props, N * 2 * (size_t)st.P * MT_PREC * sizeof(uint32_t));
    if (st.DL) alloc((void **)&st.dlog, N * (size_t)st.DL * sizeof(int32_t));
    alloc((void **)&h->d_sums, N * sizeof(mt_checksum));
    alloc((void **)&st.retry, N * sizeof(int32_t));
    alloc((void **)&st.resume, N * sizeof(int64_t));
    alloc((void **)&st.stats, 16 * sizeof(uint32_t));
#ifdef MT_PROF
    alloc((void **)&st.prof, 128 * sizeof(unsigned long long));
    if (ok) ok = hipMemset(st.prof, 0, 128 * sizeof(unsigned long long)) == hipSuccess;
#endif
    if (h->ordinals) {
        alloc((void **)&st.ordS, N * (size_t)st.S * sizeof(uint16_t));
        alloc((void **)&st.ordB, N * (size_t)MT_LV * st.B * sizeof(uint16_t));
    }
    if (h->live) {
        alloc((void **)&st.live, N * 4 * sizeof(int32_t));
        st.LG = std::min(std::max(o.live_group_capacity > 0 ? o.live_group_capacity : 1024, 16), 65535);
        alloc((void **)&st.grp, N * (size_t)(st.LG + 1) * MT_GRP_WORDS * sizeof(int32_t));
        alloc((void **)&st.segP, N * (size_t)st.S * sizeof(PendQ));
    }
    if (st.PP > 0) {
        const size_t slots = N * (size_t)st.PP * MT_PG_SLOTS;
        alloc((void **)&st.pgA, slots * sizeof(int4));
        alloc((void **)&st.pgO, slots * sizeof(u64));
        alloc((void **)&st.pgB, slots * sizeof(uint4));
        alloc((void **)&st.pgMeta, N * st.PP * sizeof(PageMeta));
        alloc((void **)&st.pgDir, N * st.PP * sizeof(uint16_t));
        alloc((void **)&st.pgCnt, N * MT_LV * (size_t)st.PP);
        alloc((void **)&st.pgHeap, N * (size_t)(st.PH + 1) * sizeof(int2));
        alloc((void **)&st.pgUtPage, N * (size_t)st.UT * sizeof(int32_t));
        alloc((void **)&st.pgUtA, N * (size_t)st.UT * sizeof(int4));
        alloc((void **)&st.pgUtO, N * (size_t)st.UT * sizeof(u64));
        alloc((void **)&st.pgUmap, N * (size_t)st.UM * sizeof(uint16_t));
        st.OA = o.overlap_arena_capacity > 0 ? std::min(std::max(o.overlap_arena_capacity, 64), 1 << 30) & ~7
                                              : MT_OVF_ARENA;
        alloc((void **)&st.pgOvf, N * (size_t)st.OA * sizeof(uint16_t));
        if (st.pgOvf) hipMemset(st.pgOvf, 0, N * (size_t)st.OA * sizeof(uint16_t));
        if (h->ordinals) {
            alloc((void **)&st.pgOS, slots * sizeof(uint16_t));
            alloc((void **)&st.pgOL, N * (size_t)st.PP * MT_PG_OLB * sizeof(uint16_t));
            alloc((void **)&st.pgOU, N * (size_t)MT_LV * st.PP * sizeof(uint16_t));
        }
    }
    if (!ok || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
        hipEventCreate(&h->ev_load) != hipSuccess || hipEventCreate(&h->ev_load1) != hipSuccess) {
        mt_destroy(h);
        return nullptr;
    }
    if (mt_load_initial_text(h, nullptr, nullptr) != 0) {
        mt_destroy(h);
        return nullptr;
    }
    return h;
}

static void free_region(PagedRegion &R) {
    void *ps[] = {R.A, R.O, R.B, R.meta, R.dir, R.cnt, R.heap, R.upage, R.uA, R.uO, R.oS, R.oL, R.oU, R.text, R.props, R.umap, R.ovf};
    for (void *p : ps)
        if (p) hipFree(p);
    R = PagedRegion{};
}

void mt_destroy(mt_handle *h) {
    if (!h) return;
    hipSetDevice(h->device);
    if (h->pending) h->pending->owner = nullptr;
    free_region(h->st.big);
    if (h->st.bslot) hipFree(h->st.bslot);
    DevState &st = h->st;
    void *ps[] = {st.hdr, st.segA, st.segO, st.segB, st.cnt, st.flg, st.heap, st.text, st.props, st.dlog, h->d_sums,
                  h->d_seed_off, h->d_seed, st.retry, st.stats, st.resume, st.pgA, st.pgO, st.pgB, st.pgMeta,
                  st.pgDir, st.pgCnt, st.pgHeap, st.pgUtPage, st.pgUtA, st.pgUtO, st.pgUmap, st.pgOvf, st.oslot,
                  st.live, st.grp, st.segP, st.ordS, st.ordB, st.pgOS, st.pgOL, st.pgOU, st.prof};
    for (void *p : ps)
        if (p) hipFree(p);
    if (h->ev0) hipEventDestroy(h->ev0);
    if (h->ev1) hipEventDestroy(h->ev1);
    if (h->ev_load) hipEventDestroy(h->ev_load);
    if (h->ev_load1) hipEventDestroy(h->ev_load1);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
}

const char *mt_last_error(const mt_handle *h) { return h ? h->err.c_str() : "null handle"; }
uint32_t mt_num_docs(const mt_handle *h) { return h ? h->n_docs : 0; }

// startCollaboration's window for the listed documents (mt_start_collaboration)
__global__ void k_set_window(DevState st, const int32_t *ms, const int32_t *cs) {
    const uint32_t doc = blockIdx.x * blockDim.x + threadIdx.x;
    if (doc >= (uint32_t)st.n_docs || ms[doc] < 0) return;
    st.hdr[doc].min_seq = ms[doc];
    st.hdr[doc].cur_seq = cs[doc];
    st.hdr[doc].heap_n = 0;
}

int mt_start_collaboration(mt_handle *h, const int32_t *min_seq, const int32_t *cur_seq) {
    if (!h || !min_seq || !cur_seq) return MT_E_INVALID;
    for (uint32_t d = 0; d < h->n_docs; d++)
        if (min_seq[d] >= 0 && cur_seq[d] < min_seq[d]) {
            h->err = "mt_start_collaboration: document " + std::to_string(d) + " has currentSeq < minSeq";
            return MT_E_INVALID;
        }
    SETTLE(h);
    int32_t *d_w = nullptr;
    HIPCHK(h, hipMalloc(&d_w, (size_t)h->n_docs * 8 + 8));
    bool ok = hipMemcpyAsync(d_w, min_seq, (size_t)h->n_docs * 4, hipMemcpyHostToDevice, h->stream) == hipSuccess &&
              hipMemcpyAsync(d_w + h->n_docs, cur_seq, (size_t)h->n_docs * 4, hipMemcpyHostToDevice, h->stream) ==
                  hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_set_window, dim3((h->n_docs + 255) / 256), dim3(256), 0, h->stream, h->st, d_w,
                           d_w + h->n_docs);
        ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(h->stream) == hipSuccess;
    }
    hipFree(d_w);
    if (!ok) {
        h->err = "mt_start_collaboration failed";
        return MT_E_HIP;
    }
    return 0;
}

int mt_load_initial_text(mt_handle *h, const int64_t *seed_off, const uint16_t *seed_text) {
    if (!h) return MT_E_INVALID;
    SETTLE(h);
    if (h->d_seed_off) hipFree(h->d_seed_off);
    if (h->d_seed) hipFree(h->d_seed);
    h->d_seed_off = nullptr;
    h->d_seed = nullptr;
    if (seed_off) {
        if (seed_off[0] != 0) {
            h->err = "mt_load_initial_text: seed_off[0] != 0";
            return MT_E_INVALID;
        }
        for (uint32_t d = 0; d < h->n_docs; d++)
            if (seed_off[d + 1] < seed_off[d]) {
                h->err = "mt_load_initial_text: seed_off not monotonic";
                return MT_E_INVALID;
            }
        if (seed_off[h->n_docs] > 0 && !seed_text) {
            h->err = "mt_load_initial_text: null seed_text";
            return MT_E_INVALID;
        }
        const size_t n = seed_off[h->n_docs];
        HIPCHK(h, hipMalloc(&h->d_seed_off, (h->n_docs + 1) * sizeof(int64_t)));
        HIPCHK(h, hipMalloc(&h->d_seed, std::max<size_t>(n, 1) * sizeof(uint16_t)));
        HIPCHK(h, hipMemcpy(h->d_seed_off, seed_off, (h->n_docs + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
        if (n) HIPCHK(h, hipMemcpy(h->d_seed, seed_text, n * sizeof(uint16_t), hipMemcpyHostToDevice));
    }
    int rc = mt_reset(h);
    if (rc) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int mt_reset(mt_handle *h) {
    if (!h) return MT_E_INVALID;
    if (h->pending) SETTLE(h);
    HIPCHK(h, hipSetDevice(h->device));
    if (h->n_big > 0) {   // every document starts over in the main arrays (k_init clears bslot)
        HIPCHK(h, hipStreamSynchronize(h->stream));
        free_region(h->st.big);
        h->big_caps = PagedCaps{0, 0, 0, 0, 3, 0, 1};
        h->bslot_h.assign(h->n_docs, -1);
        h->n_big = 0;
    }
    if (h->st.DL) HIPCHK(h, hipMemsetAsync(h->st.dlog, 0, (size_t)h->n_docs * h->st.DL * 4, h->stream));
    hipLaunchKernelGGL(k_init, dim3(h->n_docs), dim3(MT_WAVE), 0, h->stream, h->st, h->d_seed_off, h->d_seed);
    HIPCHK(h, hipGetLastError());
    return 0;
}

mt_batch *mt_batch_upload(mt_handle *h, const int64_t *doc_op_off, const mt_op_rec *ops,
                          uint64_t n_ops, const uint16_t *text, uint64_t text_len,
                          const uint32_t *props, uint64_t props_len) {
    if (!h || !doc_op_off || (n_ops && !ops) || (text_len && !text) || (props_len && !props)) {
        if (h) h->err = "mt_batch_upload: null array";
        return nullptr;
    }
    // the kernels index ops, text and props straight from these values: reject anything
    // that would read outside the arrays (remote ops are trusted for their semantics, not
    // for memory safety)
    int max_cli = h->max_cli;
    std::string bad = validate_batch(h->n_docs, doc_op_off, ops, n_ops, text_len, props, props_len, h->live, max_cli);
    if (!bad.empty()) {
        h->err = "mt_batch_upload: " + bad;
        return nullptr;
    }
    h->max_cli = max_cli;   // (over the records the documents replay)
    if (hipSetDevice(h->device) != hipSuccess) return nullptr;
    auto *b = new mt_batch();
    b->device = h->device;
    b->n_docs = h->n_docs;
    b->n_ops = n_ops;
    b->text_len = text_len;
    b->props_len = props_len;
    bool ok = hipMalloc(&b->off, (h->n_docs + 1) * sizeof(int64_t)) == hipSuccess &&
              hipMalloc(&b->ops, std::max<uint64_t>(n_ops, 1) * sizeof(mt_op_rec)) == hipSuccess &&
              hipMalloc(&b->text, std::max<uint64_t>(text_len, 1) * sizeof(uint16_t)) == hipSuccess &&
              hipMalloc(&b->props, std::max<uint64_t>(props_len, 1) * sizeof(uint32_t)) == hipSuccess;
    if (ok) {
        ok = hipMemcpy(b->off, doc_op_off, (h->n_docs + 1) * sizeof(int64_t), hipMemcpyHostToDevice) == hipSuccess;
        if (ok && n_ops) ok = hipMemcpy(b->ops, ops, n_ops * sizeof(mt_op_rec), hipMemcpyHostToDevice) == hipSuccess;
        if (ok && text_len) ok = hipMemcpy(b->text, text, text_len * 2, hipMemcpyHostToDevice) == hipSuccess;
        if (ok && props_len) ok = hipMemcpy(b->props, props, props_len * 4, hipMemcpyHostToDevice) == hipSuccess;
        if (ok) ok = set_order(b, doc_op_off);
    }
    if (!ok) {
        h->err = "mt_batch_upload: device allocation/copy failed";
        mt_batch_free(b);
        return nullptr;
    }
    return b;
}

// documents in the big region that this batch's LDS tier flagged (retry 1) skip the tight and
// full launches: the growth step replays them at the big region's capacities (retry 3)
__global__ void k_mark_big(DevState st, const int64_t *off, int resume_set) {
    const int doc = blockIdx.x * blockDim.x + threadIdx.x;
    if (doc >= st.n_docs || st.bslot[doc] < 0 || st.retry[doc] != 1) return;
    st.retry[doc] = 3;
    if (!resume_set) st.resume[doc] = off[doc];
    atomicAdd(st.stats + 13, 1u);
}
// One paged launch over every document (those not at stage pc.stage exit at once); big: the
// documents of the big region (the growth step's launches).
// Documents of many pages replay with their page metadata in HBM (TierPagedT kHM: no LDS per
// page instead of 12 bytes, so more of them share a CU); the bench's C3 / C4 documents (< 300
// pages) keep it in LDS (no global load on their page searches).  Delta-logging handles take
// the kHM tier too (P_HM_LOG, P_BIG_HM_LOG); segment-ordinal handles keep the LDS metadata.
#ifndef MT_HM_PAGES
#define MT_HM_PAGES 512
#endif
static bool use_hm(const mt_handle *h, const PagedCaps &pc) {
    return !pc.packed && !pc.narrow && !h->ordinals && pc.PP >= MT_HM_PAGES;
}
static int launch_paged(mt_handle *h, const mt_batch *b, const PagedCaps &pc, int res, const PagedSlice &sl,
                        bool big = false) {
    const bool hm = use_hm(h, pc);
    const size_t lb = paged_layout(pc.PP, pc.PH, pc.UT, 0, pc.narrow ? 4 : 8, pc.packed != 0, hm).total;
    const dim3 g(h->n_docs), blk(MT_WAVE);
    // the bench's C3 tight tier with its capacities fixed at compile time (same code, constant
    // LDS layout: bench.capacities)
    if (!big && !pc.packed && pc.narrow && !h->st.DL && pc.PP == 192 && pc.PH == 192 && pc.UT == 220)
        launch_replay_paged(MTK(P_C3), g, blk, lb, h->stream,
                           h->st, b->ops, b->off, b->text, b->props, res, pc, sl);
    else if (!big && pc.packed && !h->st.DL && pc.PP == 224 && pc.PH == 900 && pc.UT == 1900)   // the bench's C4 tier
        launch_replay_paged(MTK(P_C4), g, blk, lb, h->stream,
                           h->st, b->ops, b->off, b->text, b->props, res, pc, sl);
    else if (pc.packed && h->st.DL)
        launch_replay_paged(MTK(P_PACKED_LOG), g, blk, lb, h->stream, h->st, b->ops,
                           b->off, b->text, b->props, res, pc, sl);
    else if (pc.packed)
        launch_replay_paged(MTK(P_PACKED), g, blk, lb, h->stream, h->st,
                           b->ops, b->off, b->text, b->props, res, pc, sl);
    else if (big && h->st.DL && hm)
        launch_replay_paged(MTK(P_BIG_HM_LOG), g, blk, lb, h->stream, h->st, b->ops,
                           b->off, b->text, b->props, res, pc, sl);
    else if (big && h->st.DL)
        launch_replay_paged(MTK(P_BIG_LOG), g, blk, lb, h->stream, h->st, b->ops,
                           b->off, b->text, b->props, res, pc, sl);
    else if (big && hm)
        launch_replay_paged(MTK(P_BIG_HM), g, blk, lb, h->stream, h->st, b->ops,
                           b->off, b->text, b->props, res, pc, sl);
    else if (big)
        launch_replay_paged(MTK(P_BIG), g, blk, lb, h->stream, h->st, b->ops,
                           b->off, b->text, b->props, res, pc, sl);
    else if (h->st.DL && hm)
        launch_replay_paged(MTK(P_HM_LOG), g, blk, lb, h->stream, h->st, b->ops, b->off, b->text,
                           b->props, res, pc, sl);
    else if (h->st.DL && pc.narrow)
        launch_replay_paged(MTK(P_NARROW_LOG), g, blk, lb, h->stream, h->st, b->ops, b->off,
                           b->text, b->props, res, pc, sl);
    else if (h->st.DL)
        launch_replay_paged(MTK(P_LOG), g, blk, lb, h->stream, h->st, b->ops, b->off, b->text,
                           b->props, res, pc, sl);
    else if (pc.narrow)
        launch_replay_paged(MTK(P_NARROW), g, blk, lb, h->stream, h->st, b->ops, b->off,
                           b->text, b->props, res, pc, sl);
    else if (hm)
        launch_replay_paged(MTK(P_HM), g, blk, lb, h->stream, h->st, b->ops, b->off, b->text,
                           b->props, res, pc, sl);
    else
        launch_replay_paged(MTK(P_FULL), g, blk, lb, h->stream, h->st, b->ops, b->off, b->text,
                           b->props, res, pc, sl);
    HIPCHK(h, hipGetLastError());
    return 0;
}

int mt_batch_apply_async(mt_handle *h, const mt_batch *b) {
    if (!h || !b || b->n_docs != h->n_docs) return MT_E_INVALID;
    if (h->pending) {   // the previous batch's growth step runs before anything else
        const int rc = mt_settle(h);
        if (rc) return rc;
    }
    h->st.order = b->order;   // (its launches and its growth step's)
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipMemsetAsync(h->st.stats, 0, 16 * sizeof(uint32_t), h->stream));
    HIPCHK(h, hipEventRecord(h->ev0, h->stream));
    if (h->lds.S > 0) {
        // LDS tier for every document; the ones that outgrow it are flagged and replayed
        // from HBM by the second launch (whose other workgroups exit at once)
        if (h->live && h->st.DL)
            launch_replay(MTK(R_LIVELDS_LOG), dim3(h->n_docs), dim3(MT_WAVE),
                               tier_lds_bytes(true, h->lds, 0), h->stream, h->st, b->ops, b->off, b->text, b->props,
                               h->lds);
        else if (h->live)
            launch_replay(MTK(R_LIVELDS), dim3(h->n_docs), dim3(MT_WAVE),
                               tier_lds_bytes(true, h->lds, 0), h->stream, h->st, b->ops, b->off, b->text, b->props,
                               h->lds);
        else if (h->st.DL)
            launch_replay(MTK(R_LDS_LOG), dim3(h->n_docs), dim3(MT_WAVE), tier_lds_bytes(true, h->lds, 0),
                               h->stream, h->st, b->ops, b->off, b->text, b->props, h->lds);
        else if (h->wpg == 2)
            launch_replay(MTK(R_LDS2), dim3((h->n_docs + 1) / 2), dim3(2 * MT_WAVE),
                               2 * tier_lds_bytes(true, h->lds, 0), h->stream, h->st, b->ops, b->off, b->text, b->props,
                               h->lds);
        else
            launch_replay(MTK(R_LDS), dim3(h->n_docs), dim3(MT_WAVE), tier_lds_bytes(true, h->lds, 0),
                               h->stream, h->st, b->ops, b->off, b->text, b->props, h->lds);
        HIPCHK(h, hipGetLastError());
    } else {
        HIPCHK(h, hipMemsetD32Async((hipDeviceptr_t)h->st.retry, 1, h->n_docs, h->stream));
    }
    if (h->st.PP > 0) {
        // documents that outgrew the LDS tier continue in the paged layout: the tight tier
        // first (when configured), then the full capacities for the documents it handed over
        const int use_resume = h->lds.S > 0 ? 1 : 0;
        if (h->n_big > 0) {   // documents of the big region go straight to the growth step's launch
            hipLaunchKernelGGL(k_mark_big, dim3((h->n_docs + 255) / 256), dim3(256), 0, h->stream, h->st, b->off,
                               use_resume);
            HIPCHK(h, hipGetLastError());
        }
        const PagedCaps *tiers[2] = {h->pg_tight.PP ? &h->pg_tight : nullptr, &h->pg_full};
        const int n = (int)h->n_docs;
        for (const PagedCaps *pc : tiers) {
            if (!pc) continue;
            const int res = pc->stage == 2 ? 1 : use_resume;
            // the launches of this tier: one over every document, or (paged_slices, first
            // tier) m slices each leaving out a window of the r = n mod resident left-over
            // documents -- every launch is then whole rounds -- and a last one without limits
            std::vector<PagedSlice> sls;
            const int S = h->pg_resident, m = h->paged_slices;
            const int r = S > 0 ? n % S : 0;
            if (pc == tiers[0] && m > 1 && S > 0 && n > S && r > 0 && (int64_t)m * r <= n) {
                const int64_t q = ((int64_t)b->n_ops / n + m - 1) / m;
                for (int j = 0; j < m; j++) {
                    PagedSlice sl{q, j * r, (j + 1) * r, 0, 0};
                    if (j == 0) sl.cnt_lo = r, sl.cnt_hi = n;   // counted once: window 0 in launch 1
                    if (j == 1) sl.cnt_lo = 0, sl.cnt_hi = r;
                    sls.push_back(sl);
                }
                sls.push_back(PagedSlice{0, 0, 0, 0, 0});
            } else {
                sls.push_back(PagedSlice{0, 0, 0, 0, n});
            }
            // a sliced tier resumes every launch after its first from resume[doc]; without
            // the LDS tier nothing has written it yet, so seed it with each document's first
            // message and resume from the first launch on (a slice must never restart at off)
            int res_k = res;
            if (sls.size() > 1 && !res) {
                HIPCHK(h, hipMemcpyAsync(h->st.resume, b->off, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToDevice,
                                         h->stream));
                res_k = 1;
            }
            PagedCaps pcx = *pc;   // a wide tight tier packs its table when every client id fits 8 bits
            pcx.packed = pc->tight && !pc->narrow && h->max_cli <= 127 && pc->PP <= 255 ? 1 : 0;   // (8-bit pages)
            for (const PagedSlice &sl : sls) {
                const int rc = launch_paged(h, b, pcx, res_k, sl, false);
                if (rc) return rc;
            }
        }
    } else if (h->live && h->st.DL)
        launch_replay(MTK(R_LIVE_LOG), dim3(h->n_docs), dim3(MT_WAVE), tier_lds_bytes(false, live_caps(h), 0),
                           h->stream, h->st, b->ops, b->off, b->text, b->props, live_caps(h));
    else if (h->live)
        launch_replay(MTK(R_LIVE), dim3(h->n_docs), dim3(MT_WAVE), tier_lds_bytes(false, live_caps(h), 0),
                           h->stream, h->st, b->ops, b->off, b->text, b->props, live_caps(h));
    else if (h->st.DL)
        launch_replay(MTK(R_GLB_LOG), dim3(h->n_docs), dim3(MT_WAVE), tier_lds_bytes(false, glb_caps(h), 0),
                           h->stream, h->st, b->ops, b->off, b->text, b->props, glb_caps(h));
    else
        launch_replay(MTK(R_GLB), dim3(h->n_docs), dim3(MT_WAVE), tier_lds_bytes(false, glb_caps(h), 0),
                           h->stream, h->st, b->ops, b->off, b->text, b->props, glb_caps(h));
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipEventRecord(h->ev1, h->stream));
    h->timed = true;
    if (h->st.PP > 0 || h->live) {   // its last paged / live tier may hand documents to a growth step
        h->pending = const_cast<mt_batch *>(b);
        h->pending->owner = h;
    }
    return 0;
}

uint64_t mt_batch_num_ops(const mt_batch *b) { return b ? b->n_ops : 0; }

// ---------------------------------------------------------------- growth step
// The paged capacities of mt_options (page_capacity, unsettled_capacity, page_heap_capacity)
// are a starting point, not a limit.  The last paged tier (PagedCaps.grow) hands a document
// that does not fit it at load, or whose next message could outgrow it (pg_room), to this
// step with the message index (retry = 3); mt_settle then moves every such document into
// the *big region* -- a second set of paged arrays whose capacities are doubled where the
// documents ran out (bounded by the 160 KiB a paged launch may stage in LDS) -- and replays
// the rest of their messages there, round after round, before anything else runs on the
// stream.  Only documents beyond the handle's sizing pay for it; the others never move.
struct MigItem {
    int32_t doc, src, dst;   // src: slot in the old big region (-1: the main arrays)
};
__global__ void __launch_bounds__(MT_WAVE) k_migrate_paged(DevState st, PagedRegion old_big, PagedRegion dst_r,
                                                           const MigItem *items) {
    const MigItem it = items[blockIdx.x];
    const DocHdr h = st.hdr[it.doc];
    const PagedBase s = it.src < 0 ? paged_base(main_region(st), (size_t)it.doc) : paged_base(old_big, (size_t)it.src);
    const PagedBase d = paged_base(dst_r, (size_t)it.dst);
    {   // the live half of the text / property arenas (same half, same offsets): every record
        // below text_top / props_top
        const uint16_t *ts = s.text + (size_t)h.text_half * s.T;
        uint16_t *td = d.text + (size_t)h.text_half * d.T;
        for (int i = lane(); i < h.text_top; i += MT_WAVE) td[i] = ts[i];
        const uint32_t *ps = s.props + (size_t)h.props_half * s.P * MT_PREC;
        uint32_t *pd = d.props + (size_t)h.props_half * d.P * MT_PREC;
        for (size_t i = lane(); i < (size_t)h.props_top * MT_PREC; i += MT_WAVE) pd[i] = ps[i];
        // the uid map's entries below next_uid (a flat document has none yet)
        if (h.pad[HDR_PAGED])
            for (int i = lane(); i < min(h.next_uid, s.UM); i += MT_WAVE) d.umap[i] = s.umap[i];
        // the overflow overlap arena up to its fill (sets keep their offsets)
        if (s.ovf && d.ovf) {
            const int top = min(max((int)((const uint32_t *)s.ovf)[0], MT_OVF_HDR), s.OA);
            for (int i = lane(); i < top; i += MT_WAVE) d.ovf[i] = s.ovf[i];
        }
    }
    if (!h.pad[HDR_PAGED]) return;   // still flat: pg_convert pages it at the new capacities
    const size_t ns = (size_t)s.PP * MT_PG_SLOTS;   // page p slot k sits at p * 64 + k in both
    for (size_t i = lane(); i < ns; i += MT_WAVE) {
        d.A[i] = s.A[i];
        d.O[i] = s.O[i];
        d.B[i] = s.B[i];
    }
    for (int i = lane(); i < s.PP; i += MT_WAVE) {
        d.meta[i] = s.meta[i];
        d.dir[i] = s.dir[i];
    }
    for (int l = 0; l < MT_LV; l++)
        for (int b = lane(); b < s.PP; b += MT_WAVE) d.cnt[(size_t)l * d.PP + b] = s.cnt[(size_t)l * s.PP + b];
    for (int i = lane(); i <= s.PH; i += MT_WAVE) d.heap[i] = s.heap[i];
    for (int i = lane(); i < s.UT; i += MT_WAVE) {
        d.upage[i] = s.upage[i];
        d.uA[i] = s.uA[i];
        d.uO[i] = s.uO[i];
    }
    if (s.oS && d.oS) {   // segment ordinals: per page (same page ids), levels by position
        for (size_t i = lane(); i < ns; i += MT_WAVE) d.oS[i] = s.oS[i];
        for (size_t i = lane(); i < (size_t)s.PP * MT_PG_OLB; i += MT_WAVE) d.oL[i] = s.oL[i];
        for (int l = 0; l < MT_LV; l++)
            for (int b = lane(); b < s.PP; b += MT_WAVE) d.oU[(size_t)l * d.PP + b] = s.oU[(size_t)l * s.PP + b];
    }
}
// documents the growth step cannot serve (out of device memory) fail as before the step existed
__global__ void k_fail_grow(DevState st) {
    const int doc = blockIdx.x * blockDim.x + threadIdx.x;
    if (doc >= st.n_docs || st.retry[doc] != 3) return;
    st.retry[doc] = 0;
    if (st.hdr[doc].status == 0) {
        st.hdr[doc].status = MT_DOC_CAPACITY;
        st.hdr[doc].pad[HDR_DIAG] = 12;
    }
}

static bool alloc_region(PagedRegion &R, int slots, const PagedCaps &c, bool ordinals, int T, int P, int UM, int OA) {
    R = PagedRegion{};
    R.PP = c.PP;
    R.PH = c.PH;
    R.UT = c.UT;
    R.T = T;
    R.P = P;
    R.UM = UM;
    R.OA = OA;
    R.slots = slots;
    const size_t n = (size_t)slots, pages = n * c.PP;
    bool ok = hipMalloc(&R.A, pages * MT_PG_SLOTS * sizeof(int4)) == hipSuccess &&
              hipMalloc(&R.O, pages * MT_PG_SLOTS * sizeof(u64)) == hipSuccess &&
              hipMalloc(&R.B, pages * MT_PG_SLOTS * sizeof(uint4)) == hipSuccess &&
              hipMalloc(&R.meta, pages * sizeof(PageMeta)) == hipSuccess &&
              hipMalloc(&R.dir, pages * sizeof(uint16_t)) == hipSuccess &&
              hipMalloc(&R.cnt, pages * MT_LV) == hipSuccess &&
              hipMalloc(&R.heap, n * (size_t)(c.PH + 1) * sizeof(int2)) == hipSuccess &&
              hipMalloc(&R.upage, n * (size_t)c.UT * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&R.uA, n * (size_t)c.UT * sizeof(int4)) == hipSuccess &&
              hipMalloc(&R.uO, n * (size_t)c.UT * sizeof(u64)) == hipSuccess &&
              hipMalloc(&R.text, n * 2 * (size_t)T * sizeof(uint16_t)) == hipSuccess &&
              hipMalloc(&R.props, n * 2 * (size_t)P * MT_PREC * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&R.umap, n * (size_t)UM * sizeof(uint16_t)) == hipSuccess &&
              hipMalloc(&R.ovf, n * (size_t)OA * sizeof(uint16_t)) == hipSuccess &&
              hipMemset(R.ovf, 0, n * (size_t)OA * sizeof(uint16_t)) == hipSuccess;
    if (ok && ordinals)
        ok = hipMalloc(&R.oS, pages * MT_PG_SLOTS * sizeof(uint16_t)) == hipSuccess &&
             hipMalloc(&R.oL, pages * MT_PG_OLB * sizeof(uint16_t)) == hipSuccess &&
             hipMalloc(&R.oU, pages * MT_LV * sizeof(uint16_t)) == hipSuccess;
    if (!ok) free_region(R);
    return ok;
}


// Moves the documents of `moving` (and every document already there) into a new big region at
// capacities c, text / property arenas of T units / P records per half, UM uid-map entries
// and OA overflow-arena units; synchronous.
static int regrow(mt_handle *h, const std::vector<uint32_t> &moving, const PagedCaps &c, int T, int P, int UM,
                  int OA) {
    DevState &st = h->st;
    const uint32_t n = h->n_docs;
    if (!st.bslot) {
        HIPCHK(h, hipMalloc(&st.bslot, (size_t)n * sizeof(int32_t)));
        HIPCHK(h, hipMemset(st.bslot, 0xFF, (size_t)n * sizeof(int32_t)));
        h->bslot_h.assign(n, -1);
    }
    std::vector<int32_t> nb(n, -1);
    std::vector<MigItem> items;
    std::vector<uint8_t> mv(n, 0);
    for (uint32_t d : moving) mv[d] = 1;
    int slots = 0;
    for (uint32_t d = 0; d < n; d++)
        if (h->bslot_h[d] >= 0 || mv[d]) {
            nb[d] = slots;
            items.push_back(MigItem{(int32_t)d, h->bslot_h[d], slots});
            slots++;
        }
    PagedRegion R;
    if (!alloc_region(R, std::max(slots, 1), c, h->ordinals, T, P, UM, OA)) {
        (void)hipGetLastError();
        h->err = "growth step: device allocation of the big region failed";
        return MT_E_NOMEM;
    }
    MigItem *d_items = nullptr;
    if (hipMalloc(&d_items, items.size() * sizeof(MigItem)) != hipSuccess) {
        free_region(R);
        return MT_E_NOMEM;
    }
    HIPCHK(h, hipMemcpy(d_items, items.data(), items.size() * sizeof(MigItem), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_migrate_paged, dim3((uint32_t)items.size()), dim3(MT_WAVE), 0, h->stream, st, st.big, R,
                       (const MigItem *)d_items);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    hipFree(d_items);
    HIPCHK(h, hipMemcpy(st.bslot, nb.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice));
    free_region(st.big);
    st.big = R;
    h->bslot_h = nb;
    h->n_big = (uint32_t)slots;
    h->big_caps = PagedCaps{c.PP, c.PH, c.UT, 0, 3, 0, 1};
    const size_t lb = paged_layout(c.PP, c.PH, c.UT, 0, 8).total;
    if (lb > 64 * 1024) {
        const void *ks[] = {MTK(P_BIG_LOG), MTK(P_BIG_HM_LOG),
                            MTK(P_BIG), MTK(P_BIG_HM)};
        for (const void *k : ks) HIPCHK(h, hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lb));
    }
    return 0;
}

// After the launches of batch b: re-tiers and replays the documents they handed to the
// growth step until none is left (synchronous).
static int grow_loop(mt_handle *h, const mt_batch *b) {
    DevState &st = h->st;
    st.order = b->order;
    const uint32_t n = h->n_docs;
    h->grown_last = 0;
    h->grow_rounds_last = 0;
    PagedCaps launched = h->pg_full;   // the capacities of the launch that handed them over
    bool launched_big = false;         // ... and whether it was the big region's launch
    std::vector<int32_t> retry(n);
    std::vector<DocHdr> hdr(n);
    for (int round = 0; round < 32; round++) {
        uint32_t g = 0;
        HIPCHK(h, hipMemcpy(&g, st.stats + 13, sizeof(g), hipMemcpyDeviceToHost));
        if (g == 0) return 0;
        HIPCHK(h, hipMemset(st.stats + 13, 0, sizeof(g)));
        HIPCHK(h, hipMemcpy(retry.data(), st.retry, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemcpy(hdr.data(), st.hdr, (size_t)n * sizeof(DocHdr), hipMemcpyDeviceToHost));
        std::vector<uint32_t> moving;
        // what ran out, read from the handed-over documents' state: a capacity they fill to
        // more than half is doubled (the kernel's bound is per message, pg_room); documents
        // of the big region marked for this batch (k_mark_big) only need its capacities
        bool t = false, hp = false, pg = false, tx = false, pr = false, um = false, ov = false;
        int judged = 0;
        for (uint32_t d = 0; d < n; d++) {
            if (retry[d] != 3) continue;
            moving.push_back(d);
            const bool in_big = !h->bslot_h.empty() && h->bslot_h[d] >= 0;
            if (in_big && !launched_big) continue;
            judged++;
            const DocHdr &x = hdr[d];
            const int np = x.pad[HDR_PAGED] ? x.pad[HDR_NPAGES] : (x.depth > 1 ? x.n_blk[1] : 1);
            t = t || 2 * x.pad[HDR_UTN] > launched.UT;
            hp = hp || 2 * x.heap_n > launched.PH;
            pg = pg || 2 * (np + 8) > launched.PP;
            if (x.pad[HDR_PAGED])   // an upper level near its room (pcnt_cap scales with the pages)
                for (int l = 2; l < x.depth && l < MT_LV; l++) pg = pg || 2 * (x.n_blk[l] + 4) > pcnt_cap(launched.PP, l);
            const int cause = x.status == 0 ? x.pad[HDR_DIAG] : 0;   // an arena hand-over (pg_arena_room)
            tx = tx || cause == 4;
            pr = pr || cause == 5;
            um = um || cause == 9;
            ov = ov || cause == 11;
        }
        if (moving.empty()) return 0;
        if (!t && !hp && !pg && !tx && !pr && !um && !ov) t = hp = true;   // a single message's bound (a long range): its table / heap terms
        h->grown_last += (uint32_t)moving.size();
        h->grow_rounds_last++;
        // the new capacities: doubled where the documents ran out, never below the big
        // region's, within the LDS one paged launch may stage
        const bool have = h->big_caps.PP > 0;
        auto fits = [](const PagedCaps &c) { return paged_layout(c.PP, c.PH, c.UT, 0, 8).total <= 160 * 1024; };
        auto same = [](const PagedCaps &a, const PagedCaps &b) { return a.PP == b.PP && a.PH == b.PH && a.UT == b.UT; };
        auto doubled = [&](const PagedCaps &c) {   // c doubled where needed, one capacity at a time while it fits
            PagedCaps r = c, x = c;
            if (t) x.UT = std::min(2 * x.UT, 1 << 20);
            if (fits(x)) r = x;
            x = r;
            if (hp) x.PH = std::min(2 * x.PH, 1 << 20);
            if (fits(x)) r = x;
            x = r;
            if (pg) x.PP = std::min(2 * x.PP, 65535);
            if (fits(x)) r = x;
            return r;
        };
        PagedCaps nc = judged ? doubled(launched) : h->big_caps;   // (judged == 0: only marked documents)
        if (have) {
            nc.PP = std::max(nc.PP, h->big_caps.PP);
            nc.PH = std::max(nc.PH, h->big_caps.PH);
            nc.UT = std::max(nc.UT, h->big_caps.UT);
        }
        // the text / property arenas and the uid map (HBM only): doubled when a document's live
        // text / records / segments fill more than half of them after a compaction
        const int lT = launched_big ? st.big.T : st.T, lP = launched_big ? st.big.P : st.P;
        const int lU = launched_big ? st.big.UM : st.UM, lO = launched_big ? st.big.OA : st.OA;
        int nT = judged && tx ? (int)std::min<int64_t>(2LL * lT, 1 << 28) : lT;
        int nP = judged && pr ? (int)std::min<int64_t>(2LL * lP, 1 << 26) : lP;
        int nU = judged && um ? (int)std::min<int64_t>(2LL * lU, 1 << 24) : lU;
        int nO = judged && ov ? (int)std::min<int64_t>(2LL * lO, 1 << 30) : lO;
        if (have) {
            nT = std::max(nT, st.big.T);
            nP = std::max(nP, st.big.P);
            nU = std::max(nU, st.big.UM);
            nO = std::max(nO, st.big.OA);
        }
        int rc = 0;
        PagedCaps pc = nc;
        bool big = true;
        if (same(nc, launched) && nT == lT && nP == lP && nU == lU && nO == lO) {
            // no LDS capacity can grow: the documents run to their end at the capacities they
            // were handed over at (in their own region) and fail as before the step existed
            // only if they do outgrow them -- the arenas and the uid map still grow
            pc = launched;
            pc.grow = 2;
            big = launched_big;
        } else {
            bool all_big = have;
            for (uint32_t d : moving) all_big = all_big && !h->bslot_h.empty() && h->bslot_h[d] >= 0;
            if (!(all_big && same(nc, h->big_caps) && nT == st.big.T && nP == st.big.P && nU == st.big.UM &&
                  nO == st.big.OA))
                rc = regrow(h, moving, nc, nT, nP, nU, nO);
            pc.grow = 1;   // (the arenas can always grow; a round that raises nothing runs with grow 0)
        }
        if (rc) {
            hipLaunchKernelGGL(k_fail_grow, dim3((n + 255) / 256), dim3(256), 0, h->stream, st);
            HIPCHK(h, hipStreamSynchronize(h->stream));
            return rc;
        }
        pc.tight = 0;
        pc.stage = 3;
        pc.narrow = 0;
        rc = launch_paged(h, b, pc, 1, PagedSlice{0, 0, 0, 0, 0}, big);
        if (rc) return rc;
        HIPCHK(h, hipStreamSynchronize(h->stream));
        launched = pc;
        launched_big = big;
    }
    h->err = "growth step: no progress after 32 rounds";
    return MT_E_HIP;
}

// ---------------------------------------------------------------- live growth step
// Live (participant) documents replay on the flat HBM tier, whose per-document capacities
// (segments, blocks, heap, text and property arenas, segment groups) are the handle's.  They
// are a starting point, not a limit: a document whose next message could outgrow them
// (live_room) stops before it and is handed here; the step doubles what ran out for the whole
// handle -- every document's arrays are copied to the new strides (k_live_regrow) -- and
// replays the rest of the handed-over documents' messages, round after round.  Group ids are
// a ring of st.LG: growing it renumbers each document's outstanding groups from 1 (the
// segments' pending-group FIFOs with them).
struct LiveArrays {
    int32_t S, B, H, T, P, LG;
    int4 *segA;
    u64 *segO;
    uint4 *segB;
    uint8_t *cnt;
    int8_t *flg;
    int2 *heap;
    uint16_t *text;
    uint32_t *props;
    PendQ *segP;
    int32_t *grp;
    uint16_t *ordS, *ordB;
};
__global__ void __launch_bounds__(MT_WAVE) k_live_regrow(const DocHdr *hdr, int32_t *live, LiveArrays a, LiveArrays b) {
    const size_t doc = blockIdx.x;
    const DocHdr h = hdr[doc];
    const int n = h.n_seg;
    for (int i = lane(); i < n; i += MT_WAVE) {
        b.segA[doc * b.S + i] = a.segA[doc * a.S + i];
        b.segO[doc * b.S + i] = a.segO[doc * a.S + i];
        b.segB[doc * b.S + i] = a.segB[doc * a.S + i];
        if (a.ordS) b.ordS[doc * b.S + i] = a.ordS[doc * a.S + i];
    }
    for (int l = 0; l < MT_LV; l++)
        for (int q = lane(); q < h.n_blk[l]; q += MT_WAVE) {
            b.cnt[doc * MT_LV * b.B + (size_t)l * b.B + q] = a.cnt[doc * MT_LV * a.B + (size_t)l * a.B + q];
            if (a.ordB) b.ordB[doc * MT_LV * b.B + (size_t)l * b.B + q] = a.ordB[doc * MT_LV * a.B + (size_t)l * a.B + q];
        }
    for (int q = lane(); q < h.n_blk[0]; q += MT_WAVE) b.flg[doc * b.B + q] = a.flg[doc * a.B + q];
    for (int i = 1 + lane(); i <= h.heap_n; i += MT_WAVE) b.heap[doc * (b.H + 1) + i] = a.heap[doc * (a.H + 1) + i];
    {   // the live half of the arenas, same offsets
        const uint16_t *ts = a.text + doc * 2 * a.T + (size_t)h.text_half * a.T;
        uint16_t *td = b.text + doc * 2 * b.T + (size_t)h.text_half * b.T;
        for (int i = lane(); i < h.text_top; i += MT_WAVE) td[i] = ts[i];
        const uint32_t *ps = a.props + doc * 2 * a.P * MT_PREC + (size_t)h.props_half * a.P * MT_PREC;
        uint32_t *pd = b.props + doc * 2 * b.P * MT_PREC + (size_t)h.props_half * b.P * MT_PREC;
        for (size_t i = lane(); i < (size_t)h.props_top * MT_PREC; i += MT_WAVE) pd[i] = ps[i];
    }
    // segment groups: outstanding ids g_head .. (ring of a.LG) -> 1 .. g_n
    const int g_head = live[4 * doc + 1], g_n = live[4 * doc + 2];
    const bool renum = b.LG != a.LG;
    auto nid = [&](int x) { return x == 0 ? 0 : (renum ? (x - g_head + a.LG) % a.LG + 1 : x); };
    for (int i = lane(); i < n; i += MT_WAVE) {
        PendQ q = a.segP[doc * a.S + i];
        if (renum)
            for (int k = 0; k < 4; k++) {
                u64 w = 0;
                for (int j = 0; j < 4; j++) w |= (u64)(uint32_t)nid((int)((q.w[k] >> (16 * j)) & 0xFFFFull)) << (16 * j);
                q.w[k] = w;
            }
        b.segP[doc * b.S + i] = q;
    }
    const size_t ga = doc * (size_t)(a.LG + 1) * MT_GRP_WORDS, gb = doc * (size_t)(b.LG + 1) * MT_GRP_WORDS;
    if (!renum) {
        for (int i = lane(); i < (a.LG + 1) * MT_GRP_WORDS; i += MT_WAVE) b.grp[gb + i] = a.grp[ga + i];
    } else {
        for (int k = 0; k < g_n; k++) {
            const int x = (g_head - 1 + k) % a.LG + 1;
            if (lane() < MT_GRP_WORDS)
                b.grp[gb + (size_t)(k + 1) * MT_GRP_WORDS + lane()] = a.grp[ga + (size_t)x * MT_GRP_WORDS + lane()];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane() == 0) live[4 * doc + 1] = 1;
    }
}
static LiveArrays live_arrays(const DevState &st) {
    return LiveArrays{st.S, st.B, st.H, st.T, st.P, st.LG, (int4 *)st.segA, (u64 *)st.segO, (uint4 *)st.segB,
                      (uint8_t *)st.cnt, (int8_t *)st.flg, (int2 *)st.heap, (uint16_t *)st.text, (uint32_t *)st.props,
                      (PendQ *)st.segP, (int32_t *)st.grp, (uint16_t *)st.ordS, (uint16_t *)st.ordB};
}
// every document's flat arrays at the new capacities
static int live_regrow(mt_handle *h, int S2, int B2, int H2, int T2, int P2, int LG2) {
    DevState &st = h->st;
    const size_t N = h->n_docs;
    LiveArrays a = live_arrays(st), b = a;
    b.S = S2, b.B = B2, b.H = H2, b.T = T2, b.P = P2, b.LG = LG2;
    bool ok = true;
    auto alloc = [&](auto **p, size_t bytes) {
        *p = nullptr;
        if (ok && hipMalloc((void **)p, bytes ? bytes : 16) != hipSuccess) ok = false;
    };
    alloc(&b.segA, N * S2 * sizeof(int4));
    alloc(&b.segO, N * S2 * sizeof(u64));
    alloc(&b.segB, N * S2 * sizeof(uint4));
    alloc(&b.cnt, N * MT_LV * (size_t)B2);
    alloc(&b.flg, N * (size_t)B2);
    alloc(&b.heap, N * (size_t)(H2 + 1) * sizeof(int2));
    alloc(&b.text, N * 2 * (size_t)T2 * sizeof(uint16_t));
    alloc(&b.props, N * 2 * (size_t)P2 * MT_PREC * sizeof(uint32_t));
    alloc(&b.segP, N * (size_t)S2 * sizeof(PendQ));
    alloc(&b.grp, N * (size_t)(LG2 + 1) * MT_GRP_WORDS * sizeof(int32_t));
    if (a.ordS) {
        alloc(&b.ordS, N * (size_t)S2 * sizeof(uint16_t));
        alloc(&b.ordB, N * (size_t)MT_LV * B2 * sizeof(uint16_t));
    }
    void *nb[] = {b.segA, b.segO, b.segB, b.cnt, b.flg, b.heap, b.text, b.props, b.segP, b.grp, b.ordS, b.ordB};
    if (!ok) {
        for (void *p : nb)
            if (p) hipFree(p);
        h->err = "live growth step: device allocation failed (HBM exhausted)";
        return MT_E_HIP;
    }
    hipLaunchKernelGGL(k_live_regrow, dim3((unsigned)N), dim3(MT_WAVE), 0, h->stream, st.hdr, st.live, a, b);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    void *old[] = {a.segA, a.segO, a.segB, a.cnt, a.flg, a.heap, a.text, a.props, a.segP, a.grp, a.ordS, a.ordB};
    for (void *p : old)
        if (p) hipFree(p);
    st.S = S2, st.B = B2, st.H = H2, st.T = T2, st.P = P2, st.LG = LG2;
    st.segA = (decltype(st.segA))b.segA;
    st.segO = (decltype(st.segO))b.segO;
    st.segB = (decltype(st.segB))b.segB;
    st.cnt = (decltype(st.cnt))b.cnt;
    st.flg = (decltype(st.flg))b.flg;
    st.heap = (decltype(st.heap))b.heap;
    st.text = (decltype(st.text))b.text;
    st.props = (decltype(st.props))b.props;
    st.segP = (decltype(st.segP))b.segP;
    st.grp = (decltype(st.grp))b.grp;
    st.ordS = (decltype(st.ordS))b.ordS;
    st.ordB = (decltype(st.ordB))b.ordB;
    return 0;
}
__global__ void k_live_fail_flagged(DevState st, int cause) {
    const int doc = blockIdx.x * blockDim.x + threadIdx.x;
    if (doc >= st.n_docs || !st.retry[doc]) return;
    st.retry[doc] = 0;
    st.hdr[doc].status = MT_DOC_CAPACITY;
    st.hdr[doc].pad[HDR_DIAG] = cause;
}
static int live_grow_loop(mt_handle *h, const mt_batch *b) {
    DevState &st = h->st;
    st.order = b->order;
    h->grown_last = 0;
    h->grow_rounds_last = 0;
    for (int round = 0; round < 40; round++) {
        uint32_t s[2];
        HIPCHK(h, hipMemcpy(s, st.stats + 13, sizeof(s), hipMemcpyDeviceToHost));
        if (s[0] == 0) return 0;
        HIPCHK(h, hipMemset(st.stats + 13, 0, sizeof(s)));
        const uint32_t c = s[1];
        int S2 = st.S, B2 = st.B, H2 = st.H, T2 = st.T, P2 = st.P, LG2 = st.LG;
        if (c & (1u << 1)) S2 = 2 * st.S;
        B2 = std::max(st.B * ((c & (1u << 2)) ? 2 : 1), (std::max(64, S2 / 2) + 63) / 64 * 64);
        H2 = std::max(st.H * ((c & (1u << 3)) ? 2 : 1), (int)((int64_t)st.H * S2 / st.S));
        if (c & (1u << 4)) T2 = 2 * st.T;
        P2 = std::max(st.P * ((c & (1u << 5)) ? 2 : 1), st.P + (S2 - st.S));
        if (c & (1u << 12)) LG2 = std::min(2 * st.LG, 65535);
        if (S2 == st.S && B2 == st.B && H2 == st.H && T2 == st.T && P2 == st.P && LG2 == st.LG) {
            // nothing left to grow (group ids are 16 bits): the documents fail as before
            hipLaunchKernelGGL(k_live_fail_flagged, dim3((h->n_docs + 255) / 256), dim3(256), 0, h->stream, st, 12);
            HIPCHK(h, hipGetLastError());
            HIPCHK(h, hipStreamSynchronize(h->stream));
            return 0;
        }
        const int rc = live_regrow(h, S2, B2, H2, T2, P2, LG2);
        if (rc) return rc;
        h->grown_last += s[0];
        h->grow_rounds_last++;
        TierCaps caps = glb_caps(h);
        caps.resume = 1;
        caps.grow = 1;
        if (st.DL)
            launch_replay(MTK(R_LIVE_LOG), dim3(h->n_docs), dim3(MT_WAVE), tier_lds_bytes(false, caps, 0), h->stream,
                          st, b->ops, b->off, b->text, b->props, caps);
        else
            launch_replay(MTK(R_LIVE), dim3(h->n_docs), dim3(MT_WAVE), tier_lds_bytes(false, caps, 0), h->stream, st,
                          b->ops, b->off, b->text, b->props, caps);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipStreamSynchronize(h->stream));
    }
    h->err = "live growth step: no progress after 40 rounds";
    return MT_E_HIP;
}

// Waits for the stream, then runs the growth step of the last applied batch.
static int mt_settle(mt_handle *h) {
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (!h->pending) return 0;
    mt_batch *b = h->pending;
    h->pending = nullptr;
    const int rc = h->live ? live_grow_loop(h, b) : grow_loop(h, b);
    b->owner = nullptr;
    // the growth step's launches belong to the batch: the batch's timing (mt_last_kernel_ms)
    // ends after them
    if (h->grown_last > 0 && h->timed) {
        HIPCHK(h, hipEventRecord(h->ev1, h->stream));
        HIPCHK(h, hipEventSynchronize(h->ev1));
    }
    return rc;
}

void mt_batch_free(mt_batch *b) {
    if (!b) return;
    if (b->owner && b->owner->pending == b) mt_settle(b->owner);   // its growth step still reads it
    hipSetDevice(b->device);
    if (b->off) hipFree(b->off);
    if (b->ops) hipFree(b->ops);
    if (b->text) hipFree(b->text);
    if (b->props) hipFree(b->props);
    if (b->order) hipFree(b->order);
    delete b;
}

void *mt_host_alloc(uint64_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}
void mt_host_free(void *p) {
    if (p) hipHostFree(p);
}

int mt_sync(mt_handle *h) {
    if (!h) return MT_E_INVALID;
    const int rc = mt_settle(h);
    if (rc) return rc;
    if (h->timed) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, h->ev0, h->ev1) == hipSuccess) h->last_ms = ms;
        (void)hipGetLastError();   // never leave a sticky error for the next launch check
        h->timed = false;
    }
    return 0;
}

float mt_last_kernel_ms(const mt_handle *h) { return h ? h->last_ms : 0.f; }

// The handle's stream again, at a scheduling priority: > 0 the device's highest, < 0 its
// lowest, 0 the default.  Handles sharing the GPU (the skewed bench's size classes, each on its
// own stream) dispatch the high-priority stream's waiting workgroups first as CUs free up.
int mt_set_stream_priority(mt_handle *h, int priority) {
    if (!h) return MT_E_INVALID;
    const int rc = mt_sync(h);
    if (rc) return rc;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    int least = 0, greatest = 0;
    HIPCHK(h, hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t s = nullptr;
    HIPCHK(h, hipStreamCreateWithPriority(&s, hipStreamNonBlocking,
                                          priority > 0 ? greatest : (priority < 0 ? least : 0)));
    hipStreamDestroy(h->stream);
    h->stream = s;
    return 0;
}

int mt_last_hbm_docs(mt_handle *h, uint32_t *out) {
    if (!h || !out) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    SETTLE(h);
    HIPCHK(h, hipMemcpy(out, h->st.stats, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return 0;
}

int mt_last_grown(mt_handle *h, uint32_t *out) {
    if (!h || !out) return MT_E_INVALID;
    SETTLE(h);
    uint32_t in_big = 0;
    for (int32_t x : h->bslot_h) in_big += x >= 0;
    out[0] = h->grown_last;
    out[1] = h->grow_rounds_last;
    out[2] = in_big;
    out[3] = (uint32_t)h->big_caps.PP;
    out[4] = (uint32_t)h->big_caps.UT;
    out[5] = (uint32_t)h->big_caps.PH;
    return 0;
}

int mt_last_paged_peaks(mt_handle *h, uint32_t *out) {
    if (!h || !out) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    SETTLE(h);
    HIPCHK(h, hipMemcpy(out, h->st.stats + 8, 5 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return 0;
}

int mt_apply_ops(mt_handle *h, const int64_t *doc_op_off, const mt_op_rec *ops, uint64_t n_ops,
                 const uint16_t *text, uint64_t text_len, const uint32_t *props,
                 uint64_t props_len) {
    if (!h) return MT_E_INVALID;
    h->err.clear();
    mt_batch *b = mt_batch_upload(h, doc_op_off, ops, n_ops, text, text_len, props, props_len);
    if (!b) return h->err.rfind("mt_batch_upload: device", 0) == 0 ? MT_E_NOMEM : MT_E_INVALID;
    int rc = mt_batch_apply_async(h, b);
    if (rc == 0) rc = mt_sync(h);
    mt_batch_free(b);
    return rc;
}

struct mt_snapshots {
    int device = 0;
    uint32_t doc_lo = 0, n_docs = 0;   // summary d loads into document doc_lo + d
    int64_t *off = nullptr;
    int32_t *nh = nullptr, *min_seq = nullptr, *cur_seq = nullptr;
    mt_seg_rec *segs = nullptr;
    uint16_t *text = nullptr;
    uint32_t *props = nullptr;
    mt_batch *body = nullptr;   // loadBody appends as MT_F_LOAD records (nullptr: none)
    // headers larger than the flat capacities on a paged handle (k_load_convert)
    LoadScratch sc = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    int64_t *sc_off = nullptr;
    bool any_big = false;
};

void mt_snapshots_free(mt_snapshots *s) {
    if (!s) return;
    hipSetDevice(s->device);
    void *ps[] = {s->off, s->nh, s->min_seq, s->cur_seq, s->segs, s->text, s->props, s->sc.A, s->sc.O, s->sc.B,
                  s->sc.cnt, s->sc.flg, s->sc_off};
    for (void *p : ps)
        if (p) hipFree(p);
    mt_batch_free(s->body);
    delete s;
}

mt_snapshots *mt_snapshots_upload_range(mt_handle *h, uint32_t doc_lo, uint32_t n_docs, const int64_t *doc_seg_off,
                                        const int32_t *n_header, const mt_seg_rec *segs, uint64_t n_segs,
                                        const uint16_t *text, uint64_t text_len, const uint32_t *props,
                                        uint64_t props_len, const int32_t *min_seq, const int32_t *cur_seq) {
    if (!h || !doc_seg_off || !n_header || !min_seq || !cur_seq || (n_segs && !segs)) return nullptr;
    if (n_docs == 0 || doc_lo > h->n_docs || n_docs > h->n_docs - doc_lo) {
        h->err = "mt_snapshots_upload_range: documents [doc_lo, doc_lo + n_docs) outside the handle (or empty)";
        return nullptr;
    }
    const uint32_t N = n_docs;   // summary d of this set loads into document doc_lo + d
    for (uint32_t d = 0; d < N; d++)
        if (n_header[d] < 0 || doc_seg_off[d] + n_header[d] > doc_seg_off[d + 1] ||
            doc_seg_off[d + 1] > (int64_t)n_segs) {
            h->err = "mt_snapshots_upload: bad document segment ranges";
            return nullptr;
        }
    for (uint64_t i = 0; i < (uint64_t)doc_seg_off[N]; i++) {
        const mt_seg_rec &r = segs[i];
        h->max_cli = std::max({h->max_cli, std::abs((int)r.client), std::abs((int)r.removed_client)});
        const bool marker = (r.flags & MT_F_MARKER) != 0;
        if (r.len < 0 || (!marker && (uint64_t)r.payload + (uint64_t)r.len > text_len) ||
            !props_rec_ok(props, props_len, r.props)) {
            h->err = "mt_snapshots_upload: segment record " + std::to_string(i) + " outside the arenas";
            return nullptr;
        }
    }
    if (hipSetDevice(h->device) != hipSuccess) return nullptr;
    auto *s = new mt_snapshots();
    s->device = h->device;
    s->n_docs = N;
    s->doc_lo = doc_lo;
    bool ok = hipMalloc(&s->off, (N + 1) * 8) == hipSuccess && hipMalloc(&s->nh, N * 4) == hipSuccess &&
              hipMalloc(&s->min_seq, N * 4) == hipSuccess && hipMalloc(&s->cur_seq, N * 4) == hipSuccess &&
              hipMalloc(&s->segs, std::max<uint64_t>(n_segs, 1) * sizeof(mt_seg_rec)) == hipSuccess &&
              hipMalloc(&s->text, std::max<uint64_t>(text_len, 1) * 2) == hipSuccess &&
              hipMalloc(&s->props, std::max<uint64_t>(props_len, 1) * 4) == hipSuccess;
    ok = ok && hipMemcpy(s->off, doc_seg_off, (N + 1) * 8, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(s->nh, n_header, N * 4, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(s->min_seq, min_seq, N * 4, hipMemcpyHostToDevice) == hipSuccess &&
         hipMemcpy(s->cur_seq, cur_seq, N * 4, hipMemcpyHostToDevice) == hipSuccess &&
         (!n_segs || hipMemcpy(s->segs, segs, n_segs * sizeof(mt_seg_rec), hipMemcpyHostToDevice) == hipSuccess) &&
         (!text_len || hipMemcpy(s->text, text, text_len * 2, hipMemcpyHostToDevice) == hipSuccess) &&
         (!props_len || hipMemcpy(s->props, props, props_len * 4, hipMemcpyHostToDevice) == hipSuccess);
    // a header beyond the flat capacities is staged and paged (handles with a paged layout)
    if (ok && h->st.PP > 0) {
        std::vector<int64_t> so((size_t)N * 2, -1);
        int64_t ns = 0, nb = 0;
        for (uint32_t d = 0; d < N; d++) {
            const int64_t n = n_header[d], nb0 = n > 0 ? (n + MT_LOAD_FANOUT - 1) / MT_LOAD_FANOUT : 1;
            if (n > h->st.S || nb0 > h->st.B) {
                so[2 * d] = ns;
                so[2 * d + 1] = nb;
                ns += n;
                nb += nb0;
            }
        }
        if (ns > 0) {
            s->any_big = true;
            ok = hipMalloc(&s->sc.A, ns * sizeof(int4)) == hipSuccess &&
                 hipMalloc(&s->sc.O, ns * sizeof(u64)) == hipSuccess &&
                 hipMalloc(&s->sc.B, ns * sizeof(uint4)) == hipSuccess &&
                 hipMalloc(&s->sc.cnt, (size_t)nb * MT_LV) == hipSuccess &&
                 hipMalloc(&s->sc.flg, (size_t)nb) == hipSuccess &&
                 hipMalloc(&s->sc_off, (size_t)N * 16) == hipSuccess &&
                 hipMemcpy(s->sc_off, so.data(), (size_t)N * 16, hipMemcpyHostToDevice) == hipSuccess;
            s->sc.off = s->sc_off;
        }
    }
    if (!ok) {
        h->err = "mt_snapshots_upload: device allocation/copy failed";
        mt_snapshots_free(s);
        return nullptr;
    }
    // loadBody (MT/snapshotLoader.ts:161-228): specs without merge info (NonCollabClient,
    // seq 0) are appended in batches -- one insertSegments: one boundary at the batch start
    // (root.cachedLength), then each segment at insertPos += cachedLength -- the others one
    // by one at root.cachedLength.  Each append becomes an MT_F_LOAD insert record (refSeq
    // 0, the append's client and seq) plus MT_OP_LOAD_REMOVED when the spec carries removal
    // info; the ordinary replay kernels apply them (every tier).
    std::vector<mt_op_rec> ops;
    std::vector<int64_t> ooff(h->n_docs + 1, 0);   // the body batch spans the handle's documents
    for (uint32_t d = 0; d < N; d++) {
        ooff[doc_lo + d] = (int64_t)ops.size();
        const int64_t s0 = doc_seg_off[d], sh = s0 + n_header[d], s1 = doc_seg_off[d + 1];
        int64_t obs = 0;   // root.cachedLength: observer length (removed segments count 0)
        for (int64_t i = s0; i < sh; i++)
            if (segs[i].removed_seq == MT_RSEQ_NONE) obs += (segs[i].flags & MT_F_MARKER) ? 1 : segs[i].len;
        bool in_batch = false;
        int64_t ins = 0;
        // loadBody's batch is never emptied (:207-227): once it was flushed holding a segment
        // (of non-zero length -- blockInsert skips the others), the next flush (before the
        // next merge-info spec, or the final one) re-inserts it -> MT_DOC_ALIASED there
        bool batch_len = false, flushed = false, aliased = false;
        auto alias = [&]() {
            mt_op_rec q;
            memset(&q, 0, sizeof(q));
            q.kind = MT_OP_LOAD_ALIASED;
            q.flags = MT_F_LOAD;
            ops.push_back(q);
            aliased = true;
        };
        for (int64_t i = sh; i < s1 && !aliased; i++) {
            const mt_seg_rec &r = segs[i];
            const int len = (r.flags & MT_F_MARKER) ? 1 : r.len;
            const bool plain = r.client == -2 && r.seq == 0;
            const bool removed = r.removed_seq != MT_RSEQ_NONE;
            if (plain) {
                if (flushed) continue;   // inserted by the next flush, after the re-insertion
                if (!in_batch) ins = obs;
                in_batch = true;
                batch_len = batch_len || len > 0;
            } else {
                if (batch_len) {   // flushBatch() before this spec
                    if (flushed) {
                        alias();
                        break;
                    }
                    flushed = true;
                }
                in_batch = false;
                ins = obs;
            }
            if (len > 0) {   // blockInsert skips empty segments (:2229)
                mt_op_rec o;
                memset(&o, 0, sizeof(o));
                o.seq = plain ? 0 : r.seq;
                o.pos1 = (int32_t)ins;
                o.pos2 = len;
                o.payload = r.payload;
                o.props = r.props;
                o.client = (uint16_t)(plain ? -2 : r.client);
                o.kind = MT_OP_INSERT;
                o.flags = (uint8_t)(MT_F_LOAD | (r.flags & MT_F_MARKER));
                ops.push_back(o);
                if (removed) {
                    mt_op_rec q;
                    memset(&q, 0, sizeof(q));
                    q.seq = r.removed_seq;
                    q.client = (uint16_t)r.removed_client;
                    q.kind = MT_OP_LOAD_REMOVED;
                    q.flags = MT_F_LOAD;
                    ops.push_back(q);
                }
                ins += len;
            }
            if (!removed) obs += len;
        }
        if (!aliased && batch_len && flushed) alias();   // the final flushBatch()
    }
    for (uint32_t d = doc_lo + N; d <= h->n_docs; d++) ooff[d] = (int64_t)ops.size();
    if (!ops.empty()) {
        s->body = mt_batch_upload(h, ooff.data(), ops.data(), ops.size(), text, text_len, props, props_len);
        if (!s->body) {
            mt_snapshots_free(s);
            return nullptr;
        }
    }
    return s;
}

mt_snapshots *mt_snapshots_upload(mt_handle *h, const int64_t *doc_seg_off, const int32_t *n_header,
                                  const mt_seg_rec *segs, uint64_t n_segs, const uint16_t *text, uint64_t text_len,
                                  const uint32_t *props, uint64_t props_len, const int32_t *min_seq,
                                  const int32_t *cur_seq) {
    if (!h) return nullptr;
    return mt_snapshots_upload_range(h, 0, h->n_docs, doc_seg_off, n_header, segs, n_segs, text, text_len, props,
                                     props_len, min_seq, cur_seq);
}

int mt_snapshots_load_async(mt_handle *h, const mt_snapshots *s) {
    if (!h || !s || s->doc_lo > h->n_docs || s->n_docs > h->n_docs - s->doc_lo) return MT_E_INVALID;
    if (h->pending) SETTLE(h);
    HIPCHK(h, hipSetDevice(h->device));
    if (h->n_big > 0) {   // loaded documents start over in the main arrays (k_load_header clears bslot)
        for (uint32_t d = s->doc_lo; d < s->doc_lo + s->n_docs; d++) {
            h->n_big -= h->bslot_h[d] >= 0;
            h->bslot_h[d] = -1;
        }
    }
    if (h->st.DL)
        HIPCHK(h, hipMemsetAsync(h->st.dlog + (size_t)s->doc_lo * h->st.DL, 0, (size_t)s->n_docs * h->st.DL * 4,
                                 h->stream));
    HIPCHK(h, hipEventRecord(h->ev_load, h->stream));
    hipLaunchKernelGGL(k_load_header, dim3(s->n_docs), dim3(MT_WAVE), 0, h->stream, h->st, s->off, s->nh, s->segs,
                       s->text, s->props, s->min_seq, s->cur_seq, s->sc, (int)s->doc_lo);
    HIPCHK(h, hipGetLastError());
    if (s->any_big) {
        const PagedCaps &pc = h->pg_full;
        const size_t lb = paged_layout(pc.PP, pc.PH, pc.UT, 0, 8).total;
        if (h->ordinals)   // canonical ordinals for the paged documents (reloadFromSegments)
            launch_load_convert(MTK(LC_LOG), dim3(s->n_docs), dim3(MT_WAVE), lb, h->stream, h->st,
                               s->sc, pc, (int)s->doc_lo);
        else
            launch_load_convert(MTK(LC_FAST), dim3(s->n_docs), dim3(MT_WAVE), lb, h->stream, h->st,
                               s->sc, pc, (int)s->doc_lo);
        HIPCHK(h, hipGetLastError());
    }
    HIPCHK(h, hipEventRecord(h->ev_load1, h->stream));
    h->load_timed = true;
    if (s->body) return mt_batch_apply_async(h, s->body);
    return 0;
}

float mt_last_load_ms(mt_handle *h) {
    if (!h || !h->load_timed) return 0.f;
    float ms = 0.f;
    if (hipEventSynchronize(h->ev_load1) != hipSuccess || hipEventElapsedTime(&ms, h->ev_load, h->ev_load1) != hipSuccess)
        return 0.f;
    return ms;
}

int mt_load_snapshots(mt_handle *h, const int64_t *doc_seg_off, const int32_t *n_header, const mt_seg_rec *segs,
                      uint64_t n_segs, const uint16_t *text, uint64_t text_len, const uint32_t *props,
                      uint64_t props_len, const int32_t *min_seq, const int32_t *cur_seq) {
    if (!h) return MT_E_INVALID;
    if (hipSetDevice(h->device) != hipSuccess || hipStreamSynchronize(h->stream) != hipSuccess) return MT_E_HIP;
    mt_snapshots *s = mt_snapshots_upload(h, doc_seg_off, n_header, segs, n_segs, text, text_len, props, props_len,
                                          min_seq, cur_seq);
    if (!s) return MT_E_INVALID;
    int rc = mt_snapshots_load_async(h, s);
    if (rc == 0) rc = mt_sync(h);
    if (rc == 0 && hipStreamSynchronize(h->stream) != hipSuccess) rc = MT_E_HIP;
    mt_snapshots_free(s);
    return rc;
}

int mt_extract_snapshots(mt_handle *h, int64_t *io, mt_seg_rec *recs, uint16_t *text, uint32_t *props,
                         int32_t *min_seq, int32_t *cur_seq) {
    if (!h || !io) return MT_E_INVALID;
    const uint32_t N = h->n_docs;
    HIPCHK(h, hipSetDevice(h->device));
    SETTLE(h);
    int64_t *d_io = nullptr;
    HIPCHK(h, hipMalloc(&d_io, (size_t)N * 3 * 8));
    const int mode = recs ? 1 : 0;
    uint64_t nr = 0, nt = 0, np = 0;
    std::vector<int64_t> off;
    if (mode) {   // io holds the counts of the first call: exclusive prefix sums
        off.resize((size_t)N * 3);
        for (uint32_t d = 0; d < N; d++) {
            off[3 * d] = (int64_t)nr;
            off[3 * d + 1] = (int64_t)nt;
            off[3 * d + 2] = (int64_t)np;
            nr += io[3 * d];
            nt += io[3 * d + 1];
            np += io[3 * d + 2];
        }
    }
    mt_seg_rec *d_recs = nullptr;
    uint16_t *d_text = nullptr;
    uint32_t *d_props = nullptr;
    int32_t *d_win = nullptr;
    bool ok = hipMalloc(&d_win, (size_t)N * 8) == hipSuccess;
    if (ok && mode)
        ok = hipMalloc(&d_recs, std::max<uint64_t>(nr, 1) * sizeof(mt_seg_rec)) == hipSuccess &&
             hipMalloc(&d_text, std::max<uint64_t>(nt, 1) * 2) == hipSuccess &&
             hipMalloc(&d_props, std::max<uint64_t>(np, 1) * 4) == hipSuccess &&
             hipMemcpy(d_io, off.data(), (size_t)N * 3 * 8, hipMemcpyHostToDevice) == hipSuccess;
    if (ok) {
        hipLaunchKernelGGL(k_extract, dim3(N), dim3(MT_WAVE), 0, h->stream, h->st, mode, d_io, d_recs, d_text, d_props,
                           d_win);
        ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(h->stream) == hipSuccess;
    }
    if (ok && !mode) ok = hipMemcpy(io, d_io, (size_t)N * 3 * 8, hipMemcpyDeviceToHost) == hipSuccess;
    if (ok && mode) {
        ok = (!nr || hipMemcpy(recs, d_recs, nr * sizeof(mt_seg_rec), hipMemcpyDeviceToHost) == hipSuccess) &&
             (!nt || !text || hipMemcpy(text, d_text, nt * 2, hipMemcpyDeviceToHost) == hipSuccess) &&
             (!np || !props || hipMemcpy(props, d_props, np * 4, hipMemcpyDeviceToHost) == hipSuccess);
    }
    std::vector<int32_t> win((size_t)N * 2);
    if (ok) ok = hipMemcpy(win.data(), d_win, (size_t)N * 8, hipMemcpyDeviceToHost) == hipSuccess;
    if (ok)
        for (uint32_t d = 0; d < N; d++) {
            if (min_seq) min_seq[d] = win[2 * d];
            if (cur_seq) cur_seq[d] = win[2 * d + 1];
        }
    void *ps[] = {d_io, d_recs, d_text, d_props, d_win};
    for (void *p : ps)
        if (p) hipFree(p);
    if (!ok) {
        h->err = "mt_extract_snapshots failed";
        return MT_E_HIP;
    }
    return 0;
}

// Packs the generated documents' text / property regions (allocated at fixed strides) back
// to back and rebases their op records, whose offsets the generator wrote local to the
// document's region: the wire format's u32 offsets address the whole batch, and the strided
// layout would pass 2^32 units (C3: at document ~53.7k).
__global__ void __launch_bounds__(256) k_gen_compact(mt_op_rec *ops, const int64_t *off, const uint16_t *text_in,
                                                     const uint32_t *props_in, int64_t text_max, int64_t prec_words,
                                                     const int64_t *used, const int64_t *base, uint16_t *text_out,
                                                     uint32_t *props_out, int n_docs) {
    const int doc = blockIdx.x;
    if (doc >= n_docs) return;
    const int64_t tu = used[2 * doc], pu = used[2 * doc + 1], tb = base[2 * doc], pb = base[2 * doc + 1];
    const int64_t o0 = off[doc], n = off[doc + 1] - o0;
    const uint16_t *ts = text_in + o0 * text_max + doc;   // the generator's region (gen_begin)
    const uint32_t *ps = props_in + o0 * prec_words + doc;
    for (int64_t i = threadIdx.x; i < tu; i += blockDim.x) text_out[tb + i] = ts[i];
    for (int64_t i = threadIdx.x; i < pu; i += blockDim.x) props_out[pb + i] = ps[i];
    mt_op_rec *o = ops + o0;
    for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
        mt_op_rec op = o[k];
        if (op.kind == MT_OP_INSERT && !(op.flags & MT_F_MARKER)) op.payload += (uint32_t)tb;
        if (op.props != MT_NO_PROPS) op.props += (uint32_t)pb;
        o[k] = op;
    }
}

mt_batch *mt_generate(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base,
                      int32_t *view_len_trace) {
    return mt_generate_docs(h, cfg, doc_index_base, nullptr, nullptr, view_len_trace);
}

mt_batch *mt_generate_docs(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base,
                           const int32_t *ops_per_doc, const int32_t *doc_ids, int32_t *view_len_trace) {
    if (!h || !cfg || cfg->writers < 1 || cfg->ops < 0) return nullptr;
    if (ops_per_doc)
        for (uint32_t d = 0; d < h->n_docs; d++)
            if (ops_per_doc[d] < 0) return nullptr;
    if (h->pending && mt_settle(h) != 0) return nullptr;
    h->max_cli = std::max(h->max_cli, cfg->writers);
    if (h->ordinals) {   // the generator's kernels keep no ordinals
        h->err = "mt_generate: not on a segment_ordinals handle";
        return nullptr;
    }
    if (hipSetDevice(h->device) != hipSuccess) return nullptr;
    auto *b = new mt_batch();
    b->device = h->device;
    b->n_docs = h->n_docs;
    const int64_t N = h->n_docs, ops = cfg->ops;
    // every document's region at fixed strides per message (gen_begin)
    const int64_t tstride = ops * cfg->text_max + 1;
    const int64_t pstride = ops * (1 + 2 * (int64_t)cfg->max_keys_per_op) + 1;
    std::vector<int64_t> off(N + 1);
    for (int64_t i = 0; i <= N; i++) off[i] = ops_per_doc ? (i ? off[i - 1] + ops_per_doc[i - 1] : 0) : i * ops;
    b->n_ops = off[N];
    b->text_len = off[N] * cfg->text_max + N;
    b->props_len = off[N] * (1 + 2 * (int64_t)cfg->max_keys_per_op) + N;
    int32_t *d_fail = nullptr, *d_trace = nullptr;
    int64_t *d_used = nullptr;
    if (view_len_trace && hipMalloc(&d_trace, std::max<int64_t>(b->n_ops, 1) * 16) != hipSuccess) {
        delete b;
        return nullptr;
    }
    bool ok = hipMalloc(&b->off, (N + 1) * sizeof(int64_t)) == hipSuccess &&
              hipMalloc(&b->ops, std::max<int64_t>(b->n_ops, 1) * sizeof(mt_op_rec)) == hipSuccess &&
              hipMalloc(&b->text, b->text_len * 2) == hipSuccess &&
              hipMalloc(&b->props, b->props_len * 4) == hipSuccess &&
              hipMalloc(&d_fail, N * 4) == hipSuccess && hipMalloc(&d_used, N * 16) == hipSuccess;
    if (ok) {
        ok = hipMemcpy(b->off, off.data(), (N + 1) * 8, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemset(d_fail, 0, N * 4) == hipSuccess && set_order(b, off.data());
        h->st.gen_off = ops_per_doc ? b->off : nullptr;   // (the generator kernels' lengths)
    }
    int32_t *d_ids = nullptr;   // the documents' global indices (their draws)
    if (ok && doc_ids)
        ok = hipMalloc(&d_ids, N * 4) == hipSuccess && hipMemcpy(d_ids, doc_ids, N * 4, hipMemcpyHostToDevice) == hipSuccess;
    h->st.gen_ids = d_ids;
    if (ok) ok = hipMemsetAsync(h->st.stats, 0, 16 * sizeof(uint32_t), h->stream) == hipSuccess;
    if (ok) {
        const int gw = 2 * (cfg->writers + 1);
        if (h->lds.S > 0) {
            launch_generate(MTK(G_LDS), dim3(h->n_docs), dim3(MT_WAVE), tier_lds_bytes(true, h->lds, gw),
                               h->stream, h->st, *cfg, doc_index_base, b->ops, b->text, b->props, tstride,
                               pstride, d_fail, d_trace, d_used, h->lds);
            ok = hipGetLastError() == hipSuccess;
        } else {
            ok = hipMemsetD32Async((hipDeviceptr_t)h->st.retry, 1, h->n_docs, h->stream) == hipSuccess;
        }
        if (ok && h->st.PP > 0) {
            const PagedCaps *tiers[2] = {h->pg_tight.PP ? &h->pg_tight : nullptr, &h->pg_full};
            for (const PagedCaps *pc : tiers) {
                if (!pc || !ok) continue;
                const size_t lb = paged_layout(pc->PP, pc->PH, pc->UT, gw, pc->narrow ? 4 : 8).total;
                if (pc->narrow)
                    launch_generate_paged(MTK(GP_NARROW), dim3(h->n_docs), dim3(MT_WAVE), lb,
                                       h->stream, h->st, *cfg, doc_index_base, b->ops, b->text, b->props, tstride,
                                       pstride, d_fail, d_trace, d_used, *pc);
                else
                    launch_generate_paged(MTK(GP_FULL), dim3(h->n_docs), dim3(MT_WAVE), lb,
                                       h->stream, h->st, *cfg, doc_index_base, b->ops, b->text, b->props, tstride,
                                       pstride, d_fail, d_trace, d_used, *pc);
                ok = hipGetLastError() == hipSuccess;
            }
            ok = ok && hipStreamSynchronize(h->stream) == hipSuccess;
        } else if (ok) {
            launch_generate(MTK(G_GLB), dim3(h->n_docs), dim3(MT_WAVE),
                               tier_lds_bytes(false, glb_caps(h), gw), h->stream, h->st, *cfg, doc_index_base,
                               b->ops, b->text, b->props, tstride, pstride, d_fail, d_trace, d_used, glb_caps(h));
            ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(h->stream) == hipSuccess;
        }
    }
    if (ok) {
        std::vector<int32_t> f(N);
        ok = hipMemcpy(f.data(), d_fail, N * 4, hipMemcpyDeviceToHost) == hipSuccess;
        for (int64_t i = 0; ok && i < N; i++)
            if (f[i]) {
                DocHdr hd;
                hipMemcpy(&hd, h->st.hdr + i, sizeof(DocHdr), hipMemcpyDeviceToHost);
                h->err = "mt_generate: document " + std::to_string(i) + " failed with status " + std::to_string(f[i]) +
                         " (diagnostic " + std::to_string(hd.pad[HDR_DIAG]) + ")";
                ok = false;
            }
    }
    if (ok) {   // pack the per-document regions (u32 offsets address the whole batch)
        std::vector<int64_t> used((size_t)N * 2), base((size_t)N * 2);
        ok = hipMemcpy(used.data(), d_used, N * 16, hipMemcpyDeviceToHost) == hipSuccess;
        int64_t tt = 0, tp = 0;
        for (int64_t i = 0; ok && i < N; i++) {
            base[2 * i] = tt;
            base[2 * i + 1] = tp;
            tt += used[2 * i];
            tp += used[2 * i + 1];
        }
        if (ok && (tt > (int64_t)UINT32_MAX || tp >= (int64_t)MT_NO_PROPS)) {
            h->err = "mt_generate: the batch's text / property arenas exceed 32-bit offsets";
            ok = false;
        }
        uint16_t *nt = nullptr;
        uint32_t *np = nullptr;
        if (ok)
            ok = hipMalloc(&nt, std::max<int64_t>(tt, 1) * 2) == hipSuccess &&
                 hipMalloc(&np, std::max<int64_t>(tp, 1) * 4) == hipSuccess;
        int64_t *d_base = nullptr;
        if (ok) ok = hipMalloc(&d_base, N * 16) == hipSuccess &&
                     hipMemcpy(d_base, base.data(), N * 16, hipMemcpyHostToDevice) == hipSuccess;
        if (ok) {
            hipLaunchKernelGGL(k_gen_compact, dim3(h->n_docs), dim3(256), 0, h->stream, b->ops, b->off, b->text,
                               b->props, (int64_t)cfg->text_max, 1 + 2 * (int64_t)cfg->max_keys_per_op, d_used,
                               d_base, nt, np, h->n_docs);
            ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(h->stream) == hipSuccess;
        }
        if (d_base) hipFree(d_base);
        if (ok) {
            hipFree(b->text);
            hipFree(b->props);
            b->text = nt;
            b->props = np;
            b->text_len = tt;
            b->props_len = tp;
        } else {
            if (nt) hipFree(nt);
            if (np) hipFree(np);
        }
    }
    h->st.gen_off = nullptr;
    h->st.gen_ids = nullptr;
    if (d_ids) hipFree(d_ids);
    if (ok && d_trace)
        ok = hipMemcpy(view_len_trace, d_trace, b->n_ops * 16, hipMemcpyDeviceToHost) == hipSuccess;
    if (d_trace) hipFree(d_trace);
    if (d_fail) hipFree(d_fail);
    if (d_used) hipFree(d_used);
    if (!ok) {
        if (h->err.empty()) h->err = "mt_generate failed";
        mt_batch_free(b);
        return nullptr;
    }
    return b;
}

int mt_generated_seeds(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base,
                       int64_t *seed_off, uint16_t *seed_text) {
    return mt_generated_seeds_docs(h, cfg, doc_index_base, nullptr, seed_off, seed_text);
}
int mt_generated_seeds_docs(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base, const int32_t *doc_ids,
                            int64_t *seed_off, uint16_t *seed_text) {
    if (!h || !cfg) return MT_E_INVALID;
    int64_t pos = 0;
    for (uint32_t doc = 0; doc < h->n_docs; doc++) {
        seed_off[doc] = pos;
        Rng r;
        rng_init(r, cfg->seed, doc_ids ? doc_ids[doc] : (int)(doc_index_base + doc));
        for (int i = 0; i < cfg->seed_len; i++) {
            (void)rng_next(r);
            const uint16_t ch = (uint16_t)(97 + rng_uniform(r, 26));
            if (seed_text) seed_text[pos] = ch;
            pos++;
        }
    }
    seed_off[h->n_docs] = pos;
    return 0;
}

int mt_batch_sizes(const mt_batch *b, uint64_t *n_ops, uint64_t *text_len, uint64_t *props_len) {
    if (!b) return MT_E_INVALID;
    if (n_ops) *n_ops = b->n_ops;
    if (text_len) *text_len = b->text_len;
    if (props_len) *props_len = b->props_len;
    return 0;
}

int mt_batch_download(const mt_batch *b, int64_t *doc_op_off, mt_op_rec *ops, uint16_t *text,
                      uint32_t *props) {
    if (!b) return MT_E_INVALID;
    if (hipSetDevice(b->device) != hipSuccess) return MT_E_HIP;
    if (doc_op_off && hipMemcpy(doc_op_off, b->off, (b->n_docs + 1) * 8, hipMemcpyDeviceToHost) != hipSuccess) return MT_E_HIP;
    if (ops && b->n_ops && hipMemcpy(ops, b->ops, b->n_ops * sizeof(mt_op_rec), hipMemcpyDeviceToHost) != hipSuccess) return MT_E_HIP;
    if (text && b->text_len && hipMemcpy(text, b->text, b->text_len * 2, hipMemcpyDeviceToHost) != hipSuccess) return MT_E_HIP;
    if (props && b->props_len && hipMemcpy(props, b->props, b->props_len * 4, hipMemcpyDeviceToHost) != hipSuccess) return MT_E_HIP;
    return 0;
}

// ---------------------------------------------------------------- read-out
struct HostDoc {
    DocHdr hdr;
    std::vector<int4> A;
    std::vector<u64> O;
    std::vector<uint4> B;
    std::vector<uint8_t> cnt;
    std::vector<uint16_t> text;
    std::vector<uint32_t> props;
    // paged documents: each row's page id, slot and directory position, and the page metadata
    std::vector<int32_t> rpage, rslot, rpos;
    std::vector<PageMeta> pmeta;
    int32_t oslot[2 * MT_OSLOTS];   // overlap slots {client, last seq}
    std::vector<uint16_t> ovf;      // paged: the overflow overlap arena (MT_OVF_BIT masks)
    // the B-tree's child counts by level (lv[0]: segments per leaf block, lv[depth - 1]: the
    // root's children), in order -- the shape the remote views' partial lengths follow
    std::vector<std::vector<int>> lv;
};
// document doc's paged arrays, host side (the growth step's slot mirror)
static PagedBase host_paged(const mt_handle *h, uint32_t doc) {
    const int s = h->bslot_h.empty() ? -1 : h->bslot_h[doc];
    return s >= 0 ? paged_base(h->st.big, (size_t)s) : paged_base(main_region(h->st), (size_t)doc);
}
static int fetch_doc(mt_handle *h, uint32_t doc, HostDoc &hd, bool with_text, bool with_props) {
    if (!h || doc >= h->n_docs) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    SETTLE(h);
    const DevState &st = h->st;
    HIPCHK(h, hipMemcpy(&hd.hdr, st.hdr + doc, sizeof(DocHdr), hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemcpy(hd.oslot, st.oslot + (size_t)doc * 2 * MT_OSLOTS, sizeof(hd.oslot), hipMemcpyDeviceToHost));
    if (hd.hdr.pad[HDR_PAGED]) {
        // paged layout: concatenate the pages in directory order; leaf-block counts from
        // the page metadata
        const PagedBase pb = host_paged(h, doc);
        const size_t PP = pb.PP, slots = PP * MT_PG_SLOTS;
        const int np = hd.hdr.pad[HDR_NPAGES];
        std::vector<uint16_t> dir(std::max(np, 1));
        std::vector<PageMeta> meta(PP);
        std::vector<int4> pA(slots);
        std::vector<u64> pO(slots);
        std::vector<uint4> pB(slots);
        HIPCHK(h, hipMemcpy(dir.data(), pb.dir, np * sizeof(uint16_t), hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemcpy(meta.data(), pb.meta, PP * sizeof(PageMeta), hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemcpy(pA.data(), pb.A, slots * sizeof(int4), hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemcpy(pO.data(), pb.O, slots * sizeof(u64), hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemcpy(pB.data(), pb.B, slots * sizeof(uint4), hipMemcpyDeviceToHost));
        hd.ovf.assign(pb.ovf ? pb.OA : 0, 0);
        if (pb.ovf) HIPCHK(h, hipMemcpy(hd.ovf.data(), pb.ovf, (size_t)pb.OA * 2, hipMemcpyDeviceToHost));
        hd.A.clear();
        hd.O.clear();
        hd.B.clear();
        hd.cnt.clear();
        hd.rpage.clear();
        hd.rslot.clear();
        hd.rpos.clear();
        for (int q = 0; q < np; q++) {
            const PageMeta &m = meta[dir[q]];
            const size_t b0 = (size_t)dir[q] * MT_PG_SLOTS;
            for (int i = 0; i < m.nseg; i++) {
                hd.A.push_back(pA[b0 + i]);
                hd.O.push_back(pO[b0 + i]);
                hd.B.push_back(pB[b0 + i]);
                hd.rpage.push_back(dir[q]);
                hd.rslot.push_back(i);
                hd.rpos.push_back(q);
            }
            for (int k = 0; k < m.nblk; k++) hd.cnt.push_back((uint8_t)pm_bcnt(m, k));
        }
        {   // the levels: leaf blocks from the pages, level 1 = the pages in directory order,
            // levels >= 2 from the upper count arrays
            const int D = std::max(hd.hdr.depth, 1);
            hd.lv.assign(D, {});
            hd.lv[0].assign(hd.cnt.begin(), hd.cnt.end());
            if (D >= 2)
                for (int q = 0; q < np; q++) hd.lv[1].push_back(meta[dir[q]].nblk);
            if (D >= 3) {
                std::vector<uint8_t> cn((size_t)MT_LV * PP);
                HIPCHK(h, hipMemcpy(cn.data(), pb.cnt, cn.size(), hipMemcpyDeviceToHost));
                for (int l = 2; l < D; l++)
                    for (int b = 0; b < hd.hdr.n_blk[l]; b++) hd.lv[l].push_back(cn[(size_t)l * PP + b]);
            }
        }
        hd.pmeta = std::move(meta);
        hd.hdr.n_seg = (int)hd.A.size();
        hd.hdr.n_blk[0] = (int)hd.cnt.size();
        hd.A.resize(std::max<size_t>(hd.A.size(), 1));
        hd.O.resize(std::max<size_t>(hd.O.size(), 1));
        hd.B.resize(std::max<size_t>(hd.B.size(), 1));
        hd.cnt.resize(std::max<size_t>(hd.cnt.size(), 1));
    } else {
    const int n = hd.hdr.n_seg;
    hd.A.resize(std::max(n, 1));
    hd.O.resize(std::max(n, 1));
    hd.B.resize(std::max(n, 1));
    if (n) {
        HIPCHK(h, hipMemcpy(hd.A.data(), st.segA + (size_t)doc * st.S, n * sizeof(int4), hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemcpy(hd.O.data(), st.segO + (size_t)doc * st.S, n * sizeof(u64), hipMemcpyDeviceToHost));
        HIPCHK(h, hipMemcpy(hd.B.data(), st.segB + (size_t)doc * st.S, n * sizeof(uint4), hipMemcpyDeviceToHost));
    }
    hd.cnt.resize((size_t)MT_LV * st.B);
    HIPCHK(h, hipMemcpy(hd.cnt.data(), st.cnt + (size_t)doc * MT_LV * st.B, MT_LV * st.B, hipMemcpyDeviceToHost));
    const int D = std::max(hd.hdr.depth, 1);
    hd.lv.assign(D, {});
    for (int l = 0; l < D; l++)
        for (int b = 0; b < hd.hdr.n_blk[l]; b++) hd.lv[l].push_back(hd.cnt[(size_t)l * st.B + b]);
    }
    const PagedBase ar = host_paged(h, doc);   // (the arenas of the document's region)
    if (with_text) {
        hd.text.resize(ar.T);
        HIPCHK(h, hipMemcpy(hd.text.data(), ar.text + (size_t)hd.hdr.text_half * ar.T, (size_t)ar.T * 2,
                            hipMemcpyDeviceToHost));
    }
    if (with_props) {
        const size_t words = (size_t)ar.P * MT_PREC;
        hd.props.resize(words);
        HIPCHK(h, hipMemcpy(hd.props.data(), ar.props + (size_t)hd.hdr.props_half * words, words * 4,
                            hipMemcpyDeviceToHost));
    }
    return 0;
}

int mt_get_status(mt_handle *h, int32_t *out_status) {
    if (!h || !out_status) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    SETTLE(h);
    std::vector<DocHdr> hs(h->n_docs);
    HIPCHK(h, hipMemcpy(hs.data(), h->st.hdr, h->n_docs * sizeof(DocHdr), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < h->n_docs; i++) out_status[i] = hs[i].status;
    return 0;
}

int mt_get_length(mt_handle *h, uint32_t doc, uint32_t *out) {
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, false, false);
    if (rc) return rc;
    uint32_t len = 0;
    for (int i = 0; i < hd.hdr.n_seg; i++)
        if (hd.A[i].z == MT_RSEQ_NONE) len += hd.A[i].x;
    *out = len;
    return 0;
}

int mt_get_text(mt_handle *h, uint32_t doc, uint16_t *out, uint32_t cap, uint32_t *out_len) {
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, true, false);
    if (rc) return rc;
    uint32_t n = 0;
    for (int i = 0; i < hd.hdr.n_seg; i++) {
        const int4 a = hd.A[i];
        const uint4 b = hd.B[i];
        if (a.z != MT_RSEQ_NONE || (b.z & MT_MARKER_BIT)) continue;
        for (int j = 0; j < a.x; j++) {
            if (out && n < cap) out[n] = hd.text[b.x + j];
            n++;
        }
    }
    if (out_len) *out_len = n;
    return 0;
}

int mt_get_prop_runs(mt_handle *h, uint32_t doc, uint32_t *runs, uint32_t cap_runs,
                     uint32_t *n_runs, uint32_t *records, uint32_t cap_words, uint32_t *n_words) {
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, false, true);
    if (rc) return rc;
    uint32_t nr = 0, nw = 0, pos = 0;
    uint32_t cur_h = 0xFFFFFFFFu, cur_start = 0, cur_len = 0, cur_rec = 0;
    auto same = [&](uint32_t a, uint32_t b) {
        if (a == 0 || b == 0) return a == b;
        const uint32_t *x = &hd.props[(size_t)a * MT_PREC], *y = &hd.props[(size_t)b * MT_PREC];
        if (x[0] != y[0]) return false;
        for (uint32_t i = 0; i < 2 * x[0]; i++)
            if (x[1 + i] != y[1 + i]) return false;
        return true;
    };
    auto flush = [&]() {
        if (cur_h == 0xFFFFFFFFu) return;
        if (runs && nr < cap_runs) {
            runs[3 * nr] = cur_start;
            runs[3 * nr + 1] = cur_len;
            runs[3 * nr + 2] = cur_rec;
        }
        nr++;
    };
    for (int i = 0; i < hd.hdr.n_seg; i++) {
        const int4 a = hd.A[i];
        if (a.z != MT_RSEQ_NONE) continue;
        const uint32_t ph = hd.B[i].y;
        if (cur_h != 0xFFFFFFFFu && same(cur_h, ph)) {
            cur_len += a.x;
        } else {
            flush();
            cur_h = ph;
            cur_start = pos;
            cur_len = a.x;
            if (ph == 0) {
                cur_rec = 0xFFFFFFFFu;
            } else {
                cur_rec = nw;
                const uint32_t *x = &hd.props[(size_t)ph * MT_PREC];
                for (uint32_t k = 0; k < 1 + 2 * x[0]; k++) {
                    if (records && nw < cap_words) records[nw] = x[k];
                    nw++;
                }
            }
        }
        pos += a.x;
    }
    flush();
    if (n_runs) *n_runs = nr;
    if (n_words) *n_words = nw;
    return 0;
}

int mt_get_segments(mt_handle *h, uint32_t doc, int32_t *rows, uint32_t cap_rows,
                    uint32_t *n_rows, int32_t *leaves, uint32_t cap_leaves, uint32_t *n_leaves) {
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, false, false);
    if (rc) return rc;
    const int n = hd.hdr.n_seg;
    for (int i = 0; i < n && rows && (uint32_t)i < cap_rows; i++) {
        const int4 a = hd.A[i];
        const uint4 b = hd.B[i];
        int32_t *r = rows + 8 * i;
        // live documents: an unacked insert / local remove reads UnassignedSequenceNumber (-1)
        const bool lins = a.y >= MT_LOCAL_BASE, lrem = a.z >= MT_LOCAL_BASE;
        r[0] = a.x;
        r[1] = lins ? -1 : a.y;
        r[2] = (int)(short)(a.w & 0xFFFF);
        r[3] = lrem ? -1 : a.z;
        r[4] = a.z == MT_RSEQ_NONE ? MT_RSEQ_NONE : (int)(short)((uint32_t)a.w >> 16);
        {   // removedClientOverlap's length: the slot bits, or an overflow set's count
            const u64 o = hd.O[i];
            const size_t off = (uint32_t)o;
            r[5] = !(o & MT_OVF_BIT) ? __builtin_popcountll(o) : (off < hd.ovf.size() ? (int)hd.ovf[off] : -1);
        }
        r[6] = (b.z & MT_MARKER_BIT) ? (int32_t)b.x : -1;
        r[7] = b.y ? 1 : 0;
    }
    if (n_rows) *n_rows = (uint32_t)n;
    const int nb0 = hd.hdr.n_blk[0];
    for (int b = 0; b < nb0 && leaves && (uint32_t)b < cap_leaves; b++) leaves[b] = hd.cnt[b];
    if (n_leaves) *n_leaves = (uint32_t)nb0;
    return 0;
}

// ---------------------------------------------------------------- segment read-outs
// Views of one fetched document for mt_get_containing_segment / mt_get_segment_by_uid /
// mt_get_view_lengths (the device's view_len, MT/mergeTree.ts:1692-1732; client 0 = this
// replica: its local net length whatever the refSeq).
struct HostView {
    int r, c, cs;   // refSeq, short client, c's overlap slot (0: none)
    bool local;
};
static int host_view_setup(mt_handle *h, uint32_t doc, const HostDoc &hd, int32_t ref_seq, int32_t client,
                           HostView &v) {
    (void)doc;
    v.r = ref_seq;
    v.c = client;
    v.cs = 0;
    v.local = client == 0;
    if (v.local) return 0;
    if (ref_seq < hd.hdr.min_seq || ref_seq > hd.hdr.cur_seq) {
        h->err = "remote view: refSeq outside the collab window [minSeq, currentSeq]";
        return MT_E_INVALID;
    }
    for (int i = 0; i < MT_OSLOTS; i++)
        if (hd.oslot[2 * i] == client) {
            v.cs = i + 1;
            break;
        }
    return 0;
}
// row i in view v: {inserted in the view, removed in the view} (nodeLength's two tests)
static void host_view_vis(const HostDoc &hd, const HostView &v, int i, bool &ins, bool &gone) {
    const int4 a = hd.A[i];
    const int cli = (int)(short)(a.w & 0xFFFF), rcli = (int)(short)((uint32_t)a.w >> 16);
    const u64 o = hd.O[i];
    bool ovl = v.cs >= 1 && ((o >> (v.cs - 1)) & 1ull);
    if (o & MT_OVF_BIT) {   // an overflow set: the segment's whole overlap list
        ovl = false;
        const size_t off = (uint32_t)o;
        const size_t n = off < hd.ovf.size() ? hd.ovf[off] : 0;
        for (size_t k = 1; k <= n && off + k < hd.ovf.size(); k++) ovl = ovl || hd.ovf[off + k] == (uint16_t)v.c;
    }
    ins = cli == v.c || (a.y != -1 && a.y <= v.r);
    gone = a.z != MT_RSEQ_NONE && (rcli == v.c || ovl || (a.z != -1 && a.z <= v.r));
}
// a leaf's nodeLength in the view
static int host_view_len(const HostDoc &hd, const HostView &v, int i) {
    const int4 a = hd.A[i];
    if (v.local) return a.z == MT_RSEQ_NONE ? a.x : 0;
    bool ins, gone;
    host_view_vis(hd, v, i, ins, gone);
    return ins && !gone ? a.x : 0;
}
// The leaf's term in its ancestors' PartialSequenceLengths (MT/partialLengths.ts): +len at its
// insert, -len at its removal, each counted when the view holds it (getBranchPartialLength
// :455-486 adds every entry at or below refSeq and the client's own later ones, overlap
// removes included via clientSeqNumbers :581-590).  The two are independent: a view below the
// client's latest refSeq can see a segment removed (by the client) but not inserted, and then
// the segment counts -len -- the reference's interior node lengths there differ from the sum
// of their leaves' nodeLength (oracle/mt_oracle.c seg_partial; pinned on every view of
// tests/golden/ref_readouts*).  In any other view it equals the leaf's nodeLength.
static int host_seg_partial(const HostDoc &hd, const HostView &v, int i) {
    const int4 a = hd.A[i];
    if (v.local) return a.z == MT_RSEQ_NONE ? a.x : 0;   // blockLength: cachedLength
    bool ins, gone;
    host_view_vis(hd, v, i, ins, gone);
    return a.x * ((int)ins - (int)gone);
}
// The tree's node lengths in view v: P[l][b] = node b of level l's length (partial lengths),
// first[l][b] = its first child (a segment row at level 0, a node of level l - 1 above).
struct HostTree {
    std::vector<std::vector<int>> P, first;
};
static void host_tree(const HostDoc &hd, const HostView &v, HostTree &t) {
    const int D = (int)hd.lv.size();
    t.P.assign(D, {});
    t.first.assign(D, {});
    for (int l = 0; l < D; l++) {
        int f = 0;
        for (int b = 0; b < (int)hd.lv[l].size(); b++) {
            t.first[l].push_back(f);
            int sum = 0;
            for (int k = f; k < f + hd.lv[l][b]; k++)
                sum += l == 0 ? (k < hd.hdr.n_seg ? host_seg_partial(hd, v, k) : 0)
                              : (k < (int)t.P[l - 1].size() ? t.P[l - 1][k] : 0);
            t.P[l].push_back(sum);
            f += hd.lv[l][b];
        }
    }
}
// MergeTree.getPosition(node, refSeq, clientId) (:1619-1636) of row i: the nodeLength of its
// earlier siblings and of each ancestor's earlier siblings (interior ones: partial lengths)
static int host_position(const HostDoc &hd, const HostView &v, const HostTree &t, int i) {
    const int D = (int)hd.lv.size();
    int x = i, p = 0;
    for (int l = 0; l < D; l++) {
        int b = 0;   // x's parent at level l
        while (b + 1 < (int)t.first[l].size() && t.first[l][b + 1] <= x) b++;
        for (int k = t.first[l].empty() ? x : t.first[l][b]; k < x; k++)
            p += l == 0 ? host_view_len(hd, v, k) : t.P[l - 1][k];
        x = b;
    }
    return p;
}
// the fields of row i (and, on a segment_ordinals handle, its ordinal from the per-node
// characters: ancestors below the root, then its own)
static int host_seg_info(mt_handle *h, uint32_t doc, const HostDoc &hd, int i, mt_seg_info *out, uint16_t *text,
                         uint32_t text_cap) {
    const int4 a = hd.A[i];
    const uint4 b = hd.B[i];
    const bool lins = a.y >= MT_LOCAL_BASE, lrem = a.z >= MT_LOCAL_BASE && a.z != MT_RSEQ_NONE;
    out->row = i;
    out->uid = b.z & ~MT_MARKER_BIT;
    out->length = a.x;
    out->seq = lins ? -1 : a.y;
    out->client = (int)(short)(a.w & 0xFFFF);
    out->removed_seq = lrem ? -1 : a.z;
    out->removed_client = a.z == MT_RSEQ_NONE ? MT_RSEQ_NONE : (int)(short)((uint32_t)a.w >> 16);
    const bool marker = (b.z & MT_MARKER_BIT) != 0;
    out->marker_ref_type = marker ? (int32_t)b.x : -1;
    out->text_len = 0;
    if (!marker && text) {
        for (int j = 0; j < a.x && (uint32_t)j < text_cap; j++) text[j] = hd.text[b.x + j];
        out->text_len = std::min<int>(a.x, (int)text_cap);
    }
    out->ordinal_len = -1;
    if (h->ordinals && !hd.hdr.pad[HDR_PAGED]) {
        const size_t S = h->st.S, B = h->st.B;
        uint16_t code = 0;
        HIPCHK(h, hipMemcpy(&code, h->st.ordS + doc * S + i, 2, hipMemcpyDeviceToHost));
        std::vector<uint16_t> ob((size_t)MT_LV * B);
        HIPCHK(h, hipMemcpy(ob.data(), h->st.ordB + doc * MT_LV * B, ob.size() * 2, hipMemcpyDeviceToHost));
        const int dep = hd.hdr.depth;
        out->ordinal[dep - 1] = code;
        int x = i;
        for (int l = 0; l + 1 < dep; l++) {
            int b_ = 0, end = 0;
            while (b_ < hd.hdr.n_blk[l]) {
                end += hd.cnt[(size_t)l * B + b_];
                if (end > x) break;
                b_++;
            }
            out->ordinal[dep - 2 - l] = ob[(size_t)l * B + b_];
            x = b_;
        }
        out->ordinal_len = dep;
    } else if (h->ordinals && h->st.pgOS) {
        // paged: the slot's character, its leaf block's (page metadata), then the upper levels'
        // by position (level 1: the page's directory position; mt_paged.h "segment ordinals")
        const PagedBase pb = host_paged(h, doc);
        const size_t PP = pb.PP;
        const int pg = hd.rpage[i], slot = hd.rslot[i], dep = hd.hdr.depth;
        uint16_t code = 0;
        HIPCHK(h, hipMemcpy(&code, pb.oS + (size_t)pg * MT_PG_SLOTS + slot, 2, hipMemcpyDeviceToHost));
        out->ordinal[dep - 1] = code;
        if (dep >= 2) {
            const PageMeta &m = hd.pmeta[pg];
            int q = 0, st = 0;
            while (q + 1 < m.nblk && slot >= st + pm_bcnt(m, q)) st += pm_bcnt(m, q++);
            HIPCHK(h, hipMemcpy(&code, pb.oL + (size_t)pg * MT_PG_OLB + q, 2, hipMemcpyDeviceToHost));
            out->ordinal[dep - 2] = code;
        }
        if (dep >= 3) {
            std::vector<uint16_t> ou((size_t)MT_LV * PP);
            std::vector<uint8_t> cn((size_t)MT_LV * PP);
            HIPCHK(h, hipMemcpy(ou.data(), pb.oU, ou.size() * 2, hipMemcpyDeviceToHost));
            HIPCHK(h, hipMemcpy(cn.data(), pb.cnt, cn.size(), hipMemcpyDeviceToHost));
            int x = hd.rpos[i];
            out->ordinal[dep - 3] = ou[PP + x];
            for (int l = 2; l + 1 < dep; l++) {
                int b_ = 0, end = 0;
                while (b_ < hd.hdr.n_blk[l]) {
                    end += cn[(size_t)l * PP + b_];
                    if (end > x) break;
                    b_++;
                }
                out->ordinal[dep - 2 - l] = ou[(size_t)l * PP + b_];
                x = b_;
            }
        }
        out->ordinal_len = dep;
    }
    return 0;
}

int mt_get_containing_segment(mt_handle *h, uint32_t doc, int32_t pos, int32_t ref_seq, int32_t client,
                              mt_seg_info *out, uint16_t *text, uint32_t text_cap) {
    if (!out) return MT_E_INVALID;
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, text != nullptr, false);
    if (rc) return rc;
    HostView v;
    if ((rc = host_view_setup(h, doc, hd, ref_seq, client, v))) return rc;
    memset(out, 0, sizeof(*out));
    out->row = -1;
    if (hd.hdr.n_seg == 0 || hd.lv.empty()) return 0;
    // searchBlock (:1830-1862): at every level the first child with pos < nodeLength(child),
    // interior children by their partial lengths; no backtracking (a block whose leaves do not
    // hold pos yields no segment)
    HostTree t;
    host_tree(hd, v, t);
    const int D = (int)hd.lv.size();
    int b = 0;
    for (int l = D - 1; l >= 1; l--) {
        int hit = -1;
        for (int k = t.first[l][b]; k < t.first[l][b] + hd.lv[l][b]; k++) {
            if (pos < t.P[l - 1][k]) {
                hit = k;
                break;
            }
            pos -= t.P[l - 1][k];
        }
        if (hit < 0) return 0;
        b = hit;
    }
    for (int i = t.first[0][b]; i < t.first[0][b] + hd.lv[0][b] && i < hd.hdr.n_seg; i++) {
        const int l = host_view_len(hd, v, i);
        if (pos < l) {
            host_seg_info(h, doc, hd, i, out, text, text_cap);
            out->position = host_position(hd, v, t, i);
            out->offset = pos;
            return 0;
        }
        pos -= l;
    }
    return 0;
}

int mt_get_segment_by_uid(mt_handle *h, uint32_t doc, uint32_t uid, int32_t ref_seq, int32_t client,
                          mt_seg_info *out, uint16_t *text, uint32_t text_cap) {
    if (!out) return MT_E_INVALID;
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, text != nullptr, false);
    if (rc) return rc;
    HostView v;
    if ((rc = host_view_setup(h, doc, hd, ref_seq, client, v))) return rc;
    memset(out, 0, sizeof(*out));
    out->row = -1;
    for (int i = 0; i < hd.hdr.n_seg; i++) {
        if ((hd.B[i].z & ~MT_MARKER_BIT) == uid) {
            HostTree t;
            host_tree(hd, v, t);
            host_seg_info(h, doc, hd, i, out, text, text_cap);
            out->position = host_position(hd, v, t, i);
            return 0;
        }
    }
    return 0;
}

int mt_get_view_lengths(mt_handle *h, uint32_t n, const uint32_t *docs, const int32_t *ref_seq,
                        const int32_t *client, int32_t *out) {
    if (!h || (n && (!docs || !ref_seq || !client || !out))) return MT_E_INVALID;
    HostDoc hd;
    int64_t have = -1;   // the document fetched last (queries of one document fetch it once)
    for (uint32_t q = 0; q < n; q++) {
        int rc;
        if ((int64_t)docs[q] != have) {
            if ((rc = fetch_doc(h, docs[q], hd, false, false))) return rc;
            have = docs[q];
        }
        HostView v;
        if ((rc = host_view_setup(h, docs[q], hd, ref_seq[q], client[q], v))) return rc;
        // blockLength(root) (:1664-1670): the root's partial length in a remote view
        int len = 0;
        for (int i = 0; i < hd.hdr.n_seg; i++) len += host_seg_partial(hd, v, i);
        out[q] = len;
    }
    return 0;
}

// Debug: raw segment records (segA, segB as 8 u32 per segment) and header words.
int mt_debug_raw(mt_handle *h, uint32_t doc, uint32_t *rows, uint32_t cap_rows, uint32_t *n_rows,
                 int32_t *hdr_words) {
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, false, false);
    if (rc) return rc;
    const int n = hd.hdr.n_seg;
    for (int i = 0; i < n && rows && (uint32_t)i < cap_rows; i++) {
        memcpy(rows + 8 * i, &hd.A[i], 16);
        memcpy(rows + 8 * i + 4, &hd.B[i], 16);
    }
    if (n_rows) *n_rows = (uint32_t)n;
    if (hdr_words) memcpy(hdr_words, &hd.hdr, sizeof(DocHdr));
    return 0;
}

// Debug (flat documents): the zamboni heap in array order as {maxSeq, leaf index of its
// segment or -1} and the leaf blocks' needsScour flags.
int mt_debug_heap(mt_handle *h, uint32_t doc, int32_t *heap, uint32_t cap, uint32_t *n_heap, int32_t *flags,
                  uint32_t cap_flags, uint32_t *n_flags) {
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, false, false);
    if (rc) return rc;
    if (hd.hdr.pad[HDR_PAGED]) return MT_E_INVALID;
    const DevState &st = h->st;
    std::vector<int2> hp((size_t)st.H + 1);
    std::vector<int8_t> fl((size_t)st.B);
    HIPCHK(h, hipMemcpy(hp.data(), st.heap + doc * (size_t)(st.H + 1), hp.size() * sizeof(int2), hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemcpy(fl.data(), st.flg + doc * (size_t)st.B, fl.size(), hipMemcpyDeviceToHost));
    const int n = hd.hdr.n_seg;
    for (int k = 1; k <= hd.hdr.heap_n && (uint32_t)(k - 1) < cap; k++) {
        int at = -1;
        for (int i = 0; i < n; i++)
            if ((hd.B[i].z & ~MT_MARKER_BIT) == (uint32_t)hp[k].y) at = i;
        heap[2 * (k - 1)] = hp[k].x;
        heap[2 * (k - 1) + 1] = at;
    }
    if (n_heap) *n_heap = (uint32_t)hd.hdr.heap_n;
    for (int b = 0; b < hd.hdr.n_blk[0] && (uint32_t)b < cap_flags; b++) flags[b] = fl[b];
    if (n_flags) *n_flags = (uint32_t)hd.hdr.n_blk[0];
    return 0;
}

int mt_get_overlap_arena(mt_handle *h, uint32_t doc, int32_t *out) {
    if (!out) return MT_E_INVALID;
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, false, false);
    if (rc) return rc;
    for (int k = 0; k < 7; k++) out[k] = 0;
    if (hd.ovf.size() < MT_OVF_HDR) return 0;
    uint32_t w[MT_OVF_HDR / 2];
    memcpy(w, hd.ovf.data(), sizeof(w));
    const int OA = (int)hd.ovf.size(), mid = mt_ovf_mid(OA);
    const int half = (w[3] & 1) && (int)w[0] > mid ? 1 : 0;
    out[0] = OA;
    out[1] = (int)w[0] - (half ? mid : MT_OVF_HDR);
    out[2] = half;
    out[3] = (int)w[2];
    std::vector<uint32_t> offs;
    for (int i = 0; i < hd.hdr.n_seg; i++)
        if (hd.O[i] & MT_OVF_BIT) offs.push_back((uint32_t)hd.O[i]);
    std::sort(offs.begin(), offs.end());
    offs.erase(std::unique(offs.begin(), offs.end()), offs.end());
    for (uint32_t off : offs) out[4] += off < hd.ovf.size() ? (int)hd.ovf[off] + 1 : 0;
    out[5] = (int)std::min<uint32_t>(w[4], INT32_MAX);
    out[6] = (int)w[5];
    return 0;
}

int mt_get_segment_props(mt_handle *h, uint32_t doc, uint32_t seg_index, uint32_t *pairs,
                         uint32_t cap_pairs, int32_t *n_pairs) {
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, false, true);
    if (rc) return rc;
    if ((int)seg_index >= hd.hdr.n_seg) return MT_E_INVALID;
    const uint32_t ph = hd.B[seg_index].y;
    if (ph == 0) {
        *n_pairs = -1;
        return 0;
    }
    const uint32_t *x = &hd.props[(size_t)ph * MT_PREC];
    for (uint32_t k = 0; k < x[0] && k < cap_pairs; k++) {
        pairs[2 * k] = x[1 + 2 * k];
        pairs[2 * k + 1] = x[2 + 2 * k];
    }
    *n_pairs = (int32_t)x[0];
    return 0;
}

int mt_get_all_segment_props(mt_handle *h, uint32_t doc, int32_t *out, uint64_t cap_words, uint64_t *n_words) {
    HostDoc hd;
    int rc = fetch_doc(h, doc, hd, false, true);
    if (rc) return rc;
    uint64_t w = 0;
    for (int i = 0; i < hd.hdr.n_seg; i++) {
        const uint32_t ph = hd.B[i].y;
        const uint32_t *x = ph ? &hd.props[(size_t)ph * MT_PREC] : nullptr;
        const int np = x ? (int)x[0] : -1;
        if (out && w < cap_words) out[w] = np;
        w++;
        for (int k = 0; k < np; k++, w += 2)
            if (out && w + 1 < cap_words) {
                out[w] = (int32_t)x[1 + 2 * k];
                out[w + 1] = (int32_t)x[2 + 2 * k];
            }
    }
    if (n_words) *n_words = w;
    return 0;
}

int mt_get_delta_log(mt_handle *h, uint32_t doc, int32_t *out, uint32_t cap, uint32_t *n) {
    if (!h || doc >= h->n_docs) return MT_E_INVALID;
    if (!h->st.DL) {
        if (n) *n = 0;
        return 0;
    }
    HIPCHK(h, hipSetDevice(h->device));
    SETTLE(h);
    DocHdr hdr;
    HIPCHK(h, hipMemcpy(&hdr, h->st.hdr + doc, sizeof(DocHdr), hipMemcpyDeviceToHost));
    // only whole records are ever counted; clamp anyway (never read past this document)
    const uint32_t have = (uint32_t)std::min<int64_t>(std::max<int32_t>(hdr.dlog_n, 0), h->st.DL);
    const uint32_t cnt = std::min<uint32_t>(have, cap);
    if (out && cnt) HIPCHK(h, hipMemcpy(out, h->st.dlog + (size_t)doc * h->st.DL, cnt * 4, hipMemcpyDeviceToHost));
    if (n) *n = have;
    if (hdr.pad[HDR_DLOG_OVF]) {
        h->err = "mt_get_delta_log: document " + std::to_string(doc) +
                 " overflowed its delta log (delta_log_capacity) since the last mt_delta_log_reset";
        return MT_E_OVERFLOW;
    }
    return 0;
}

__global__ void __launch_bounds__(MT_WAVE) k_dlog_reset(DevState st) {
    const int doc = blockIdx.x * MT_WAVE + threadIdx.x;
    if (doc >= st.n_docs) return;
    st.hdr[doc].dlog_n = 0;
    st.hdr[doc].pad[HDR_DLOG_OVF] = 0;
}

int mt_delta_log_reset(mt_handle *h) {
    if (!h) return MT_E_INVALID;
    if (h->pending) SETTLE(h);
    if (!h->st.DL) return 0;
    HIPCHK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(k_dlog_reset, dim3((h->n_docs + MT_WAVE - 1) / MT_WAVE), dim3(MT_WAVE), 0, h->stream, h->st);
    HIPCHK(h, hipGetLastError());
    return 0;
}

// Debug: section timers of an MT_PROF build (s_memtime ticks [0, 64) and call / event counts
// [64, 128)).
int mt_debug_prof(mt_handle *h, uint64_t *out, int reset) {
#ifdef MT_PROF
    if (!h || !h->st.prof) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipDeviceSynchronize());
    if (out) HIPCHK(h, hipMemcpy(out, h->st.prof, 128 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (reset) HIPCHK(h, hipMemset(h->st.prof, 0, 128 * sizeof(uint64_t)));
    return 0;
#else
    (void)h; (void)out; (void)reset;
    return MT_E_INVALID;
#endif
}

int mt_checksums_device(mt_handle *h, void *device_out) {
    if (!h || !device_out) return MT_E_INVALID;
    if (h->pending) SETTLE(h);
    HIPCHK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(k_checksum, dim3(h->n_docs), dim3(MT_WAVE), 0, h->stream, h->st,
                       (mt_checksum *)device_out);
    HIPCHK(h, hipGetLastError());
    SETTLE(h);
    return 0;
}

int mt_maintenance_counts(mt_handle *h, uint32_t *out) {
    if (!h || !out || !h->st.DL) return MT_E_INVALID;   // kept by delta-logging handles only
    HIPCHK(h, hipSetDevice(h->device));
    SETTLE(h);
    std::vector<DocHdr> hd(h->n_docs);
    HIPCHK(h, hipMemcpy(hd.data(), h->st.hdr, h->n_docs * sizeof(DocHdr), hipMemcpyDeviceToHost));
    for (uint32_t d = 0; d < h->n_docs; d++) {
        out[3 * d] = (uint32_t)hd[d].pad[HDR_MSPLIT];
        out[3 * d + 1] = (uint32_t)hd[d].pad[HDR_MAPPEND];
        out[3 * d + 2] = (uint32_t)hd[d].pad[HDR_MUNLINK];
    }
    return 0;
}

int mt_checksums(mt_handle *h, mt_checksum *out) {
    if (!h || !out) return MT_E_INVALID;
    int rc = mt_checksums_device(h, h->d_sums);
    if (rc) return rc;
    HIPCHK(h, hipMemcpy(out, h->d_sums, h->n_docs * sizeof(mt_checksum), hipMemcpyDeviceToHost));
    return 0;
}

int mt_regenerate_pending(mt_handle *h, uint32_t doc, mt_regen_rec *out, uint32_t cap, int32_t *n_out,
                          uint16_t *out_text, uint32_t text_cap, uint32_t *out_props, uint32_t props_cap) {
    if (!h || !h->live || doc >= h->n_docs || !n_out || (cap && !out) || (text_cap && !out_text) ||
        (props_cap && !out_props)) {
        if (h) h->err = "mt_regenerate_pending: needs a live_client handle, a document and output buffers";
        return MT_E_INVALID;
    }
    HIPCHK(h, hipSetDevice(h->device));
    SETTLE(h);
    mt_regen_rec *d_out = nullptr;
    uint16_t *d_text = nullptr;
    uint32_t *d_props = nullptr;
    int32_t *d_io = nullptr;
    bool ok = hipMalloc(&d_out, std::max<size_t>(cap, 1) * sizeof(mt_regen_rec)) == hipSuccess &&
              hipMalloc(&d_text, std::max<size_t>(text_cap, 1) * 2) == hipSuccess &&
              hipMalloc(&d_props, std::max<size_t>(props_cap, 1) * 4) == hipSuccess &&
              hipMalloc(&d_io, 16) == hipSuccess;
    int32_t io[4] = {0, 0, 0, 0};
    for (int round = 0; ok && round < 8; round++) {
        hipLaunchKernelGGL(k_regen, dim3(1), dim3(MT_WAVE), tier_lds_bytes(false, glb_caps(h), 0), h->stream, h->st,
                           (int)doc, d_out, (int)cap, d_text, (int)text_cap, d_props, (int)props_cap, d_io);
        ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(h->stream) == hipSuccess &&
             hipMemcpy(io, d_io, 16, hipMemcpyDeviceToHost) == hipSuccess;
        if (!ok || io[0] != -5) break;
        // more segment groups than the handle's ring holds (nothing changed yet): grow it
        const int lg2 = std::min(65535, std::max(2 * h->st.LG, io[1]));
        if (lg2 <= h->st.LG || live_regrow(h, h->st.S, h->st.B, h->st.H, h->st.T, h->st.P, lg2) != 0) {
            io[0] = -2;
            break;
        }
    }
    if (ok) {
        if (io[0] > 0)
            ok = hipMemcpy(out, d_out, (size_t)io[0] * sizeof(mt_regen_rec), hipMemcpyDeviceToHost) == hipSuccess &&
                 (io[1] == 0 || hipMemcpy(out_text, d_text, (size_t)io[1] * 2, hipMemcpyDeviceToHost) == hipSuccess) &&
                 (io[2] == 0 || hipMemcpy(out_props, d_props, (size_t)io[2] * 4, hipMemcpyDeviceToHost) == hipSuccess);
    }
    for (void *p : {(void *)d_out, (void *)d_text, (void *)d_props, (void *)d_io})
        if (p) hipFree(p);
    if (!ok) {
        h->err = "mt_regenerate_pending: device allocation / launch failed";
        return MT_E_HIP;
    }
    if (io[0] == -3) {
        h->err = "mt_regenerate_pending: the document has failed";
        return MT_E_INVALID;
    }
    if (io[0] == -2) {
        h->err = "mt_regenerate_pending: capacity (group table or a segment's group FIFO); document failed";
        return MT_E_INVALID;
    }
    if (io[0] == -4) {   // nothing changed: retry with buffers of these sizes
        h->err = "mt_regenerate_pending: output buffers too small: need " + std::to_string(io[1]) + " records, " +
                 std::to_string(io[2]) + " text units, " + std::to_string(io[3]) + " props words";
        *n_out = -2;
        return MT_E_OVERFLOW;
    }
    *n_out = io[0];
    return 0;
}

int mt_pending_counts(mt_handle *h, int32_t *out) {
    if (!h || !h->live || !out) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    SETTLE(h);
    std::vector<int32_t> lv((size_t)h->n_docs * 4);
    HIPCHK(h, hipMemcpy(lv.data(), h->st.live, lv.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t d = 0; d < h->n_docs; d++) {
        out[2 * d] = lv[4 * d];
        out[2 * d + 1] = lv[4 * d + 2];
    }
    return 0;
}

}  // extern "C"
