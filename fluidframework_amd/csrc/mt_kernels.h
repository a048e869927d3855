// mt_kernels.h -- the replay / generation kernel templates of the MI355X merge-tree backend
// (the storage tiers of mt_engine.h / mt_paged.h instantiated as __global__ kernels).
// Each instantiation the library launches is compiled in a translation unit of its own
// (fluidframework_amd/build.py, csrc/mt_variants.h) and reached through a kernel pointer,
// so the library builds in parallel; mt_replay.hip holds the host side and the small kernels.
#pragma once
#include "../../include/mt_replay.h"
#include "mt_paged.h"

// ============================================================================ kernels
// Initial document contents (Client.insertSegmentLocal before collaboration: seq 0,
// client LocalClientId -1; MT/client.ts:202-215) and collaboration start
// (MT/mergeTree.ts:1287-1304): one leaf block under the root.
__device__ static void init_doc_hdr(const DevState &st, int doc, int len) {
    DocHdr h;
    memset(&h, 0, sizeof(h));
    h.depth = 1;
    h.n_blk[0] = 1;
    h.text_top = len;
    h.props_top = 1;
    h.next_uid = 2;   // segment ids start at 1 (0 marks a heap entry whose segment is gone)
    h.delta_hash = MT_FNV_OFF;
    h.status = len > st.T ? MT_DOC_CAPACITY : 0;
    const size_t S = st.S;
    if (len > 0) {
        h.n_seg = 1;
        st.segA[doc * S] = v4i{len, 0, MT_RSEQ_NONE, pack_cli(-1, 0)};
        st.segO[doc * S] = 0ull;
        st.segB[doc * S] = v4u{0u, 0u, 1u, 0u};
        if (st.segP) {
            u64 *w = (u64 *)(st.segP + doc * S);
            w[0] = w[1] = w[2] = w[3] = 0ull;
        }
    }
    st.cnt[(size_t)doc * MT_LV * st.B] = len > 0 ? 1 : 0;
    st.flg[(size_t)doc * st.B] = MT_SCOUR_UNDEF;
    st.hdr[doc] = h;
}

// every overlap slot free (one wave: lane i clears slot i)
__device__ static void oslot_reset(const DevState &st, int doc) {
    int32_t *o = st.oslot + (size_t)doc * 2 * MT_OSLOTS;
    o[2 * lane()] = MT_OSLOT_FREE;
    o[2 * lane() + 1] = 0;
    if (st.pgOvf && lane() < MT_OVF_HDR / 2) ((uint32_t *)(st.pgOvf + (size_t)doc * st.OA))[lane()] = lane() ? 0u : (uint32_t)MT_OVF_HDR;
}

#define MT_LOAD_FANOUT (MT_MAXN - 1)
// Staging for summary headers larger than the flat capacities on a paged handle: the flat
// tree is built here (off[2d] = first segment, off[2d+1] = first leaf block of document d;
// -1: the document uses the flat HBM arrays), then k_load_convert pages it.
struct LoadScratch {
    v4i *A;
    u64 *O;
    v4u *B;
    uint8_t *cnt;   // [MT_LV][nb0] per document
    int8_t *flg;
    const int64_t *off;
};

// Per-launch LDS capacities of the tier (the HBM tier keeps only the B-tree counts in LDS).
struct TierCaps {
    int S, B, H;
    int resume;   // TierGlb: start from resume[doc] (documents handed over by the LDS tier)
    int grow;     // TierLiveT: a document whose next message could outgrow the handle's
                  // capacities (live_room) stops before it and is handed to the live growth
                  // step (retry[doc] = 1, resume[doc] = that message; stats[13] counts them,
                  // stats[14] ORs 1 << the capacity that ran out)
};

// Client.applyMsg for every record of this document (one wavefront per document).  The
// records are prefetched 64 at a time (lane l holds record k+l plus up to 8 payload units)
// and broadcast with readlane, so no op waits on HBM latency.
//
// TierLds: the document is staged in LDS; before each message lds_room() checks that the
// LDS capacities cannot overflow while applying it.  If they could, the LDS state is
// spilled to HBM and the document continues from that message in the TierGlb launch
// (retry[doc] = 1, resume[doc] = message index).
//
// WPG documents per workgroup, one per wave, each with its own LDS slice; the waves never
// synchronise (more documents per CU than its workgroup limit of 16 would allow).
// waves per SIMD the flat live tier (TierLiveT: its state in HBM, little LDS) is compiled for;
// 1 = no constraint (the compiler's choice: 192 VGPRs, 2 waves)
#ifndef MT_LIVE_WAVES
#define MT_LIVE_WAVES 1
#endif
template <class T> constexpr int replay_waves() { return T::kLive && !T::kLds ? MT_LIVE_WAVES : 1; }
template <class T, int WPG>
__global__ void __launch_bounds__(MT_WAVE * WPG) __attribute__((amdgpu_waves_per_eu(replay_waves<T>())))
k_replay(DevState st, const mt_op_rec *ops, const int64_t *off, const uint16_t *tin, const uint32_t *pin,
         TierCaps caps) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const LdsLayout L = lds_layout(T::kLds, caps.S, caps.B, caps.H, 0);
    // wave-uniform (SGPR) document index and LDS slice
    const int wv = WPG == 1 ? 0 : uni((int)(threadIdx.x >> 6));
    LDS_AS uint8_t *smem = (LDS_AS uint8_t *)smem_raw + (uint32_t)(wv * (int)L.total);
    const int di = (int)blockIdx.x * WPG + wv;
    if (di >= st.n_docs) return;
    const int doc = doc_at(st, di);
    if (!T::kLds && !st.retry[doc]) return;
    const int64_t k1 = off[doc + 1];
    const int64_t k0 = (T::kLds || !caps.resume) ? off[doc] : st.resume[doc];
    if (k0 >= k1) {   // no message for this document in the batch: its state stays as it is
        if (!T::kLds && lane() == 0) st.retry[doc] = 0;
        return;
    }
    if (!T::kLds && lane() == 0) atomicAdd(st.stats, 1u);
    DocT<T> d;
    if (!load_doc(d, st, doc, smem, L, caps.S, caps.B, caps.H)) {
        if (lane() == 0) {
            st.retry[doc] = 1;
            st.resume[doc] = k0;
            atomicAdd(st.stats + 1 + d.cap_cause, 1u);
        }
        return;
    }
    if (d.status) {
        if (!T::kLds && lane() == 0) st.retry[doc] = 0;
        return;
    }
    const GLB_AS v4i *o4 = (const GLB_AS v4i *)ops;
    const GLB_AS uint16_t *gt = (const GLB_AS uint16_t *)tin;
    const GLB_AS uint32_t *gp = (const GLB_AS uint32_t *)pin;
    int64_t spill_at = -1, grow_at = -1;
    int grow_cause = 0;
    for (int64_t kb = k0; kb < k1 && d.status == 0 && spill_at < 0 && grow_at < 0; kb += MT_WAVE) {
        const int64_t k = kb + lane();
        v4i r0 = v4i{0, 0, 0, 0}, r1 = v4i{0, 0, 0, 0};
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
        int nl = 0, pok = 0;
        if (k < k1) {
            r0 = o4[2 * k];
            r1 = o4[2 * k + 1];
            const int kind = (r1.w >> 16) & 0xFF, flags = ((uint32_t)r1.w >> 24) & 0xFF;
            const int len = r1.x;
            if (kind == MT_OP_INSERT && !(flags & MT_F_MARKER) && len > 0) {
                const GLB_AS uint16_t *src = gt + (uint32_t)r1.y;
                nl = src[len - 1] == '\n';
                if (len <= 8) {
                    pok = 1;
                    uint32_t u[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) u[j] = j < len ? src[j] : 0u;
                    w0 = u[0] | (u[1] << 16);
                    w1 = u[2] | (u[3] << 16);
                    w2 = u[4] | (u[5] << 16);
                    w3 = u[6] | (u[7] << 16);
                }
            }
        }
        const int cnt = (int)min((int64_t)MT_WAVE, k1 - kb);
        for (int j = 0; j < cnt && d.status == 0; j++) {
            OpIn in;
            in.op.seq = __builtin_amdgcn_readlane(r0.x, j);
            in.op.ref_seq = __builtin_amdgcn_readlane(r0.y, j);
            in.op.min_seq = __builtin_amdgcn_readlane(r0.z, j);
            in.op.pos1 = __builtin_amdgcn_readlane(r0.w, j);
            in.op.pos2 = __builtin_amdgcn_readlane(r1.x, j);
            in.op.payload = (uint32_t)__builtin_amdgcn_readlane(r1.y, j);
            in.op.props = (uint32_t)__builtin_amdgcn_readlane(r1.z, j);
            const uint32_t cw = (uint32_t)__builtin_amdgcn_readlane(r1.w, j);
            in.op.client = (uint16_t)(cw & 0xFFFF);
            in.op.kind = (uint8_t)((cw >> 16) & 0xFF);
            in.op.flags = (uint8_t)(cw >> 24);
            if (T::kLds && !lds_room(d, in.op)) {
                spill_at = kb + j;
                break;
            }
            if constexpr (T::kLive && !T::kLds) {
                if (caps.grow) {
                    grow_cause = live_room(d, in.op);
                    if (grow_cause) {
                        grow_at = kb + j;
                        break;
                    }
                }
            }
            in.pay_lo = (u64)(uint32_t)__builtin_amdgcn_readlane((int)w0, j) |
                        ((u64)(uint32_t)__builtin_amdgcn_readlane((int)w1, j) << 32);
            in.pay_hi = (u64)(uint32_t)__builtin_amdgcn_readlane((int)w2, j) |
                        ((u64)(uint32_t)__builtin_amdgcn_readlane((int)w3, j) << 32);
            in.pay_ok = __builtin_amdgcn_readlane(pok, j) != 0;
            in.nl = __builtin_amdgcn_readlane(nl, j) != 0;
            opaque(d);

            apply_op(d, in, gt, gp);
        }
    }
    if (T::kLds && d.status == MT_DOC_RETRY) {
        // an LDS capacity overflowed mid-message despite lds_room(): not resumable
        d.status = MT_DOC_CAPACITY;
        if (lane() == 0) atomicAdd(st.stats + 1 + d.cap_cause, 1u);
    }
    if (T::kLds && spill_at >= 0) {
        if (lane() == 0) {
            st.retry[doc] = 1;
            st.resume[doc] = spill_at;
            atomicAdd(st.stats + 1, 1u);
        }
    }
    if (!T::kLds && lane() == 0) {
        if (grow_at >= 0 && d.status == 0) {   // to the live growth step, from this message
            st.retry[doc] = 1;
            st.resume[doc] = grow_at;
            atomicAdd(st.stats + 13, 1u);
            atomicOr(st.stats + 14, 1u << grow_cause);
        } else {
            st.retry[doc] = 0;
        }
    }
#ifdef MT_PROF
    if (st.prof) {
        atomicAdd(&st.prof[lane()], d.prof[lane()]);
        atomicAdd(&st.prof[64 + lane()], d.prof[64 + lane()]);
    }
#endif
    store_doc(d, st, doc);
}

// ---------------------------------------------------------------- synthetic generator
struct Rng {
    uint32_t s[4];
};
__host__ __device__ static inline uint32_t sm32(uint32_t &x) {
    x += 0x9E3779B9u;
    uint32_t z = x;
    z = (z ^ (z >> 16)) * 0x85EBCA6Bu;
    z = (z ^ (z >> 13)) * 0xC2B2AE35u;
    return z ^ (z >> 16);
}
__host__ __device__ static inline void rng_init(Rng &r, uint32_t seed, int doc) {
    uint32_t x = seed ^ ((uint32_t)(doc + 1) * 0x9E3779B9u);
    for (int i = 0; i < 4; i++) r.s[i] = sm32(x);
}
__host__ __device__ static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
__host__ __device__ static inline uint32_t rng_next(Rng &r) {   // xoshiro128**
    uint32_t result = rotl32(r.s[1] * 5u, 7) * 9u;
    uint32_t t = r.s[1] << 9;
    r.s[2] ^= r.s[0];
    r.s[3] ^= r.s[1];
    r.s[1] ^= r.s[2];
    r.s[0] ^= r.s[3];
    r.s[2] ^= t;
    r.s[3] = rotl32(r.s[3], 11);
    return result;
}
__host__ __device__ static inline uint32_t rng_uniform(Rng &r, uint32_t n) {
    return (uint32_t)(((uint64_t)rng_next(r) * n) >> 32);
}
__device__ static __forceinline__ uint32_t gen_props(Rng &r, const mt_gen_cfg &cfg, uint32_t *out) {
    const uint32_t nk = 1 + rng_uniform(r, (uint32_t)cfg.max_keys_per_op);
    uint32_t count = 0;
    for (uint32_t j = 0; j < nk; j++) {
        const uint32_t key = rng_uniform(r, (uint32_t)cfg.n_keys);
        const bool is_null = (uint64_t)rng_next(r) < cfg.p_null;
        const uint32_t val = rng_uniform(r, (uint32_t)cfg.n_values);
        bool dup = false;
        gsync();
        for (uint32_t q = 0; q < count; q++)
            if (out[1 + 2 * q] == key) dup = true;   // lane 0 wrote these
        if (dup) continue;
        if (lane() == 0) {
            out[1 + 2 * count] = key;
            out[2 + 2 * count] = is_null ? MT_VAL_NULL : (val | (val == 0 ? MT_VAL_FALSY_BIT : 0u));
        }
        count++;
    }
    if (lane() == 0) out[0] = count;
    gsync();
    return 1 + 2 * count;
}

// Per-document generator state (DESIGN.md "Synthetic op streams"), shared by the flat and
// the paged generators.  Every lane draws the same numbers (uniform state).
struct GenCtx {
    Rng rng;
    LDS_AS int32_t *last_ref;
    LDS_AS int32_t *short_id;
    int next_short;
    int64_t tu, pu, tb, pb;
    int64_t ob;   // the document's first op record in the batch
    int n;        // its messages
};
__device__ static __forceinline__ void lds_fence() { asm volatile("" ::: "memory"); }
__device__ static void gen_begin(GenCtx &g, const DevState &st, const mt_gen_cfg &cfg, int gdoc, int doc,
                                 LDS_AS uint8_t *gen_lds, int64_t tstride, int64_t pstride) {
    const int W = cfg.writers;
    g.last_ref = (LDS_AS int32_t *)gen_lds;
    g.short_id = g.last_ref + (W + 1);
    rng_init(g.rng, cfg.seed, st.gen_ids ? st.gen_ids[doc] : gdoc);
    // seed text (drawn exactly like the oracle / reference harness)
    uint16_t *arena = st.text + (size_t)doc * 2 * st.T;
    for (int i = 0; i < cfg.seed_len; i++) {
        (void)rng_next(g.rng);
        const uint16_t ch = (uint16_t)(97 + rng_uniform(g.rng, 26));
        if (lane() == 0) arena[i] = ch;
    }
    if (lane() == 0) init_doc_hdr(st, doc, cfg.seed_len);
    oslot_reset(st, doc);
    for (int j = lane(); j <= W; j += MT_WAVE) {
        g.last_ref[j] = 0;
        g.short_id[j] = 0;
    }
    gsync();
    g.next_short = 1;
    g.tu = g.pu = 0;
    // regions at fixed strides per message (mt_generate: tstride = ops * text_max + 1, ...)
    if (st.gen_off) {
        g.ob = st.gen_off[doc];
        g.n = (int)(st.gen_off[doc + 1] - g.ob);
    } else {
        g.ob = (int64_t)doc * cfg.ops;
        g.n = cfg.ops;
    }
    g.tb = g.ob * cfg.text_max + doc;
    g.pb = g.ob * (1 + 2 * (int64_t)cfg.max_keys_per_op) + doc;
    (void)tstride;
    (void)pstride;
}
// Writer, reference sequence number and minSeq of message t.
__device__ static void gen_pick(GenCtx &g, const mt_gen_cfg &cfg, int t, int &r, int &c, int &msn) {
    const int W = cfg.writers;
    const int k = 1 + (int)rng_uniform(g.rng, (uint32_t)W);
    int lo = max(g.last_ref[k], t - 1 - cfg.lag);
    if (lo < 0) lo = 0;
    r = lo + (int)rng_uniform(g.rng, (uint32_t)(t - 1 - lo + 1));
    lds_fence();
    if (lane() == 0) g.last_ref[k] = r;
    lds_fence();
    int m = 0x7fffffff;
    for (int j = 1 + lane(); j <= W; j += MT_WAVE) m = min(m, g.last_ref[j]);
    msn = -wave_max(-m);
    c = g.short_id[k];
    if (!c) {
        c = g.next_short++;
        lds_fence();
        if (lane() == 0) g.short_id[k] = c;
        lds_fence();
    }
}
// The op of message t given the writer's view length (drawn like the oracle's generator).
__device__ static void gen_op(GenCtx &g, const mt_gen_cfg &cfg, int t, int r, int c, int msn, int len,
                              OpIn &in, mt_op_rec *ops_out, uint16_t *text_out, uint32_t *props_out,
                              int64_t doc) {
    const uint32_t u = rng_next(g.rng);
    mt_op_rec &op = in.op;
    op.seq = t;
    op.ref_seq = r;
    op.min_seq = msn;
    op.client = (uint16_t)c;
    op.flags = 0;
    op.props = MT_NO_PROPS;
    op.payload = 0;
    in.pay_ok = true;
    in.nl = false;
    u64 plo = 0, phi = 0;
    if (len == 0 || (uint64_t)u < cfg.p_insert) {
        op.kind = MT_OP_INSERT;
        op.pos1 = (int)rng_uniform(g.rng, (uint32_t)(len + 1));
        const int tl = 1 + (int)rng_uniform(g.rng, (uint32_t)cfg.text_max);
        op.pos2 = tl;
        op.payload = (uint32_t)g.tu;   // local to the document's region (rebased by k_gen_compact)
        uint16_t ch = 0;
        for (int j = 0; j < tl; j++) {
            const uint32_t v = rng_next(g.rng);
            ch = (uint16_t)'\n';
            if ((uint64_t)v >= cfg.p_newline) ch = (uint16_t)(97 + rng_uniform(g.rng, 26));
            if (lane() == 0) text_out[g.tb + g.tu + j] = ch;
            if (j < 4)
                plo |= (u64)ch << (16 * j);
            else if (j < 8)
                phi |= (u64)ch << (16 * (j - 4));
        }
        in.nl = ch == '\n';
        in.pay_ok = tl <= 8;
        g.tu += tl;
        if (cfg.p_insert_props > 0 && (uint64_t)rng_next(g.rng) < cfg.p_insert_props) {
            op.props = (uint32_t)g.pu;
            g.pu += gen_props(g.rng, cfg, props_out + g.pb + g.pu);
        }
    } else {
        const int p1 = (int)rng_uniform(g.rng, (uint32_t)len);
        int m = 1;
        while (m < 64 && (uint64_t)rng_next(g.rng) < cfg.p_len_continue) m++;
        op.pos1 = p1;
        op.pos2 = min(p1 + m, len);
        if ((uint64_t)u < cfg.p_insert_remove) {
            op.kind = MT_OP_REMOVE;
        } else {
            op.kind = MT_OP_ANNOTATE;
            op.props = (uint32_t)g.pu;
            g.pu += gen_props(g.rng, cfg, props_out + g.pb + g.pu);
        }
    }
    in.pay_lo = plo;
    in.pay_hi = phi;
    if (lane() == 0) ops_out[g.ob + (t - 1)] = op;
    gsync();
}
// The document's text / property words used so far (k_gen_compact packs the regions).
__device__ static void gen_end(const GenCtx &g, int64_t *used_out, int doc) {
    if (lane() == 0) {
        used_out[2 * doc] = g.tu;
        used_out[2 * doc + 1] = g.pu;
    }
}

// Generates and applies cfg.ops messages per document; the view length each writer draws
// positions from is read off the live replica.
template <class T>
__global__ void __launch_bounds__(MT_WAVE) k_generate(DevState st, mt_gen_cfg cfg, uint32_t doc_base,
                                                      mt_op_rec *ops_out, uint16_t *text_out,
                                                      uint32_t *props_out, int64_t tstride,
                                                      int64_t pstride, int32_t *fail_out,
                                                      int32_t *dbg_len, int64_t *used_out, TierCaps caps) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS_AS uint8_t *smem = (LDS_AS uint8_t *)smem_raw;
    const int doc = blockIdx.x;
    if (doc >= st.n_docs) return;
    if (!T::kLds && !st.retry[doc]) return;
    const LdsLayout L = lds_layout(T::kLds, caps.S, caps.B, caps.H, 2 * (cfg.writers + 1));
    GenCtx g;
    gen_begin(g, st, cfg, (int)(doc_base + doc), doc, smem + L.offGen, tstride, pstride);
    DocT<T> d;
    if (!load_doc(d, st, doc, smem, L, caps.S, caps.B, caps.H)) {
        if (lane() == 0) st.retry[doc] = 1;
        return;
    }
    // op records carry offsets local to the document's region of the arenas
    const GLB_AS uint16_t *gt = (const GLB_AS uint16_t *)(text_out + g.tb);
    const GLB_AS uint32_t *gp = (const GLB_AS uint32_t *)(props_out + g.pb);
    for (int t = 1; t <= g.n && d.status == 0; t++) {
        int r, c, msn;
        gen_pick(g, cfg, t, r, c, msn);
        d.ocs = oslot_of(d, c);
        int vsum = 0;
        for (int base = 0; base < d.n; base += MT_WAVE) {
            const int i = base + lane();
            v4i a;
            u64 o;
            load_ao(d, i, i < d.n, a, o);
            vsum += i < d.n ? view_len(a, o, r, c, d.ocs) : 0;
        }
        const int len = wave_sum(vsum);
        if (dbg_len && lane() == 0) {
            int32_t *q = dbg_len + (g.ob + (t - 1)) * 4;
            q[0] = len;
            q[1] = d.n;
            q[2] = r;
            q[3] = c;
        }
        OpIn in;
        gen_op(g, cfg, t, r, c, msn, len, in, ops_out, text_out, props_out, doc);
        apply_op(d, in, gt, gp);
    }
    gen_end(g, used_out, doc);
    if (T::kLds && d.status == MT_DOC_RETRY) {
        if (lane() == 0) st.retry[doc] = 1;
        return;
    }
    if (lane() == 0) {
        if (d.status) fail_out[doc] = d.status;
        if (!T::kLds) st.retry[doc] = 0;
    }
    store_doc(d, st, doc);
}

// ---------------------------------------------------------------- paged kernels
// high-water marks -> stats[8..11] (mt_last_paged_peaks)
template <class T>
__device__ __forceinline__ void pg_peaks(const DevState &st, PagedDoc<T> &pd, int pk_ut, int pk_heap) {
    const int np = nbr(pd.up, 1);
    int ns = 0;
    for (int q = lane(); q < np; q += MT_WAVE) ns += pm_nseg(pd, pd.up.dir[q]);
    ns = wave_sum(ns);
    if (lane() == 0) {
        atomicMax(st.stats + 8, (uint32_t)np);
        atomicMax(st.stats + 9, (uint32_t)pk_ut);
        atomicMax(st.stats + 10, (uint32_t)pk_heap);
        atomicMax(st.stats + 11, (uint32_t)ns);
    }
}
// Replay of the documents flagged by the LDS tier (retry[doc]) in the paged layout: a
// document seen for the first time is converted from its flat state (initial contents, or
// what the LDS tier spilled) and stays paged until the next reset.
// waves per SIMD the paged kernel is compiled for (VGPR budget 512 / n); 0 = compiler choice
#ifndef MT_PAGED_WAVES
#define MT_PAGED_WAVES 3
#endif
// The kHM tier (page metadata in HBM) is held to 7-10 documents per CU by its LDS footprint,
// so at most 2-3 waves per SIMD run it anyway: compiled for 2 it keeps every value in its 256
// VGPRs, where the 168 of 3 waves spill 120 of them to scratch (tools/regs.sh P_HM)
// The last tiers at run-time capacities (full masks and table entries, kMayGrow: the hand-over
// and growth launches) take 18-27 KB of LDS per document at their usual capacities, 8 or
// fewer per CU, too: the same 2 waves (P_FULL spills 83 VGPRs at 3, P_BIG 177, none at 2)
#ifndef MT_HM_WAVES
#define MT_HM_WAVES 2
#endif
#ifndef MT_FULL_WAVES
#define MT_FULL_WAVES 2
#endif
// The packed tiers (12-byte table entries) exist for tables that dominate a document's LDS:
// C4's 39.7 KB runs 4 documents per CU, one wave per SIMD -- compiled for 3 it spilled 64
// VGPRs (tools/regs.sh P_C4)
#ifndef MT_PACKED_WAVES
#define MT_PACKED_WAVES 2
#endif
template <class T> constexpr int paged_waves() {
    return T::kHM ? MT_HM_WAVES
                  : (T::kMayGrow ? MT_FULL_WAVES : (T::kPacked ? MT_PACKED_WAVES : MT_PAGED_WAVES));
}
#if MT_PAGED_WAVES > 0
#define MT_PAGED_WPE __attribute__((amdgpu_waves_per_eu(paged_waves<T>())))
#else
#define MT_PAGED_WPE
#endif
// A tight launch (pc.tight) hands a document to the next launch -- retry[doc] = 2 from
// message resume[doc] -- when it does not fit its LDS capacities at load, or before a message
// that could outgrow them (pg_room); stats[12] counts those hand-overs.
// A last tier with PagedCaps.grow hands a document to the growth step the same way (retry[doc]
// = 3, stats[13] counts them).
template <class T>
__device__ __forceinline__ void pg_handover(const DevState &st, int doc, int64_t k, const PagedCaps &pc) {
    if (lane() == 0) {
        st.retry[doc] = pc.tight ? 2 : 3;
        st.resume[doc] = k;
        atomicAdd(st.stats + (pc.tight ? 12 : 13), 1u);
    }
}
// One launch of a sliced paged replay (mt_options.paged_slices): documents in [skip_lo,
// skip_hi) sit this launch out, the others replay at most `ops` messages (0: all) and keep
// their stage with resume[doc] at the next one; stats[0] counts documents in [cnt_lo, cnt_hi).
struct PagedSlice {
    int64_t ops;
    int skip_lo, skip_hi, cnt_lo, cnt_hi;
};

template <class T>
__global__ void __launch_bounds__(MT_WAVE) MT_PAGED_WPE k_replay_paged(DevState st, const mt_op_rec *ops,
                                                          const int64_t *off, const uint16_t *tin,
                                                          const uint32_t *pin, int use_resume, PagedCaps pc_arg,
                                                          PagedSlice sl) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS_AS uint8_t *smem = (LDS_AS uint8_t *)smem_raw;
    const PagedCaps pc = eff_caps<T>(pc_arg);
    const int di = blockIdx.x;   // dispatch position (slices count positions: hardware rounds)
    if (di >= st.n_docs) return;
    if (di >= sl.skip_lo && di < sl.skip_hi) return;
    const int doc = doc_at(st, di);
    if (st.retry[doc] != pc.stage) return;
    if (lane() == 0 && di >= sl.cnt_lo && di < sl.cnt_hi) atomicAdd(st.stats, 1u);
    const PagedLayout L = paged_layout(pc.PP, pc.PH, pc.UT, 0, (int)sizeof(typename T::O_v), T::kPacked, T::kHM);
    const int64_t k0 = use_resume ? st.resume[doc] : off[doc];
    const int64_t kend = off[doc + 1];
    if (k0 >= kend) {   // no message left for this document in the batch (no load / store)
        if (lane() == 0) st.retry[doc] = 0;
        return;
    }
    const int64_t k1 = sl.ops > 0 ? min(kend, k0 + sl.ops) : kend;   // this launch's last message + 1
    PagedDoc<T> pd;
    pg_setup(pd, st, doc, smem, L, pc);
    DocT<T> &w = pd.w;
    if (w.status) {
        if (lane() == 0) st.retry[doc] = 0;
        return;
    }
    if (st.hdr[doc].pad[HDR_PAGED]) {
        if (!pg_load(pd, st)) {
            if (pc.tight || pc.grow == 1) {
                pg_handover<T>(st, doc, k0, pc);
            } else if (lane() == 0) {   // cannot happen: the last tier has the document's capacities
                st.hdr[doc].status = MT_DOC_CAPACITY;
                st.retry[doc] = 0;
            }
            return;
        }
    } else if (!pg_convert(pd, flat_src(st, doc))) {
        // stays flat (the pages written so far are unreferenced): the next tier converts it
        // again (the growth step: at larger page / heap / table capacities), or only the
        // status changes
        // pages 7, heap 3, table 8, uid map 9 (pg_renumber): capacities the growth step raises
        const int cc = w.cap_cause;
        if ((pc.tight || (pc.grow == 1 && (cc == 7 || cc == 3 || cc == 8)) || (pc.grow && cc == 9)) &&
            w.status == MT_DOC_CAPACITY) {
            if (!pc.tight && cc == 9 && lane() == 0) st.hdr[doc].pad[HDR_DIAG] = 9;   // (for the growth step)
            pg_handover<T>(st, doc, k0, pc);
        } else if (lane() == 0) {
            st.hdr[doc].status = w.status == MT_DOC_RETRY ? MT_DOC_CAPACITY : w.status;
            st.retry[doc] = 0;
        }
        return;
    }
    const GLB_AS v4i *o4 = (const GLB_AS v4i *)ops;
    const GLB_AS uint16_t *gt = (const GLB_AS uint16_t *)tin;
    const GLB_AS uint32_t *gp = (const GLB_AS uint32_t *)pin;
    int pk_ut = 0, pk_heap = 0;
    int64_t spill_at = -1;
    for (int64_t kb = k0; kb < k1 && w.status == 0 && spill_at < 0; kb += MT_WAVE) {
        const int64_t k = kb + lane();
        v4i r0 = v4i{0, 0, 0, 0}, r1 = v4i{0, 0, 0, 0};
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
        int pok = 0;
        if (k < k1) {
            r0 = o4[2 * k];
            r1 = o4[2 * k + 1];
            const int kind = (r1.w >> 16) & 0xFF, flags = ((uint32_t)r1.w >> 24) & 0xFF;
            const int len = r1.x;
            // (the payload units are not prefetched with the records here: six more VGPRs live
            // through the op loop cost more in spills than op_insert's own read of them --
            // A/B on the C3 shard: 851 -> 843 ms, 18 -> 5 spilled VGPRs)
#ifdef MT_PAYPF
            if (kind == MT_OP_INSERT && !(flags & MT_F_MARKER) && len > 0) {
                const GLB_AS uint16_t *src = gt + (uint32_t)r1.y;
                if (len <= 8) {
                    pok = 1;
                    uint32_t u[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) u[j] = j < len ? src[j] : 0u;
                    w0 = u[0] | (u[1] << 16);
                    w1 = u[2] | (u[3] << 16);
                    w2 = u[4] | (u[5] << 16);
                    w3 = u[6] | (u[7] << 16);
                }
            }
#endif
        }
        const int cnt = (int)min((int64_t)MT_WAVE, k1 - kb);
        for (int j = 0; j < cnt && w.status == 0; j++) {
            OpIn in;
            in.op.seq = __builtin_amdgcn_readlane(r0.x, j);
            in.op.ref_seq = __builtin_amdgcn_readlane(r0.y, j);
            in.op.min_seq = __builtin_amdgcn_readlane(r0.z, j);
            in.op.pos1 = __builtin_amdgcn_readlane(r0.w, j);
            in.op.pos2 = __builtin_amdgcn_readlane(r1.x, j);
            in.op.payload = (uint32_t)__builtin_amdgcn_readlane(r1.y, j);
            in.op.props = (uint32_t)__builtin_amdgcn_readlane(r1.z, j);
            const uint32_t cw = (uint32_t)__builtin_amdgcn_readlane(r1.w, j);
            in.op.client = (uint16_t)(cw & 0xFFFF);
            in.op.kind = (uint8_t)((cw >> 16) & 0xFF);
            in.op.flags = (uint8_t)(cw >> 24);
            in.pay_lo = (u64)(uint32_t)__builtin_amdgcn_readlane((int)w0, j) |
                        ((u64)(uint32_t)__builtin_amdgcn_readlane((int)w1, j) << 32);
            in.pay_hi = (u64)(uint32_t)__builtin_amdgcn_readlane((int)w2, j) |
                        ((u64)(uint32_t)__builtin_amdgcn_readlane((int)w3, j) << 32);
            in.pay_ok = __builtin_amdgcn_readlane(pok, j) != 0;
            in.nl = false;   // op_insert derives it from the payload's last unit
            in.pay_lane = false;
            in.pay_v = 0;
#ifndef MT_NO_PAYMSG
            {   // a short insert's payload: one load per message, used by op_insert after the page
                // lookup (its latency hides behind the views and the window switch); A/B on the
                // 12.5k-document C3 shard: 844 -> 840 ms (profiles/r4/ab_paymsg.log)
                const int len = in.op.pos2;
                if (in.op.kind == MT_OP_INSERT && !(in.op.flags & MT_F_MARKER) && len > 0 && len <= 8) {
                    in.pay_ok = true;
                    in.pay_lane = true;
                    if (lane() < len) in.pay_v = gt[in.op.payload + lane()];
                }
            }
#endif
            if ((pc.tight || pc.grow) && !((pc.grow == 2 || pg_room(pd, in.op)) && pg_arena_room(pd, in.op, pc))) {
                spill_at = kb + j;
                break;
            }
            if (w.status) break;   // (an arena compaction failed)
            pg_apply_op(pd, in, gt, gp);
            pk_ut = max(pk_ut, pd.ut_n);
            pk_heap = max(pk_heap, w.heap_n);
        }
    }
    // a window capacity is a paged-layout capacity: there is no further tier
    if (w.status == MT_DOC_RETRY) w.status = MT_DOC_CAPACITY;
    pg_store(pd, st);
    pg_peaks(st, pd, pk_ut, pk_heap);
    if (spill_at >= 0 && w.status == 0)
        pg_handover<T>(st, doc, spill_at, pc);
    else if (k1 < kend && w.status == 0) {   // slice done: the next launch of this stage resumes
        if (lane() == 0) st.resume[doc] = k1;
    } else if (lane() == 0)
        st.retry[doc] = 0;
#ifdef MT_PROF
    if (st.prof) {
        atomicAdd(&st.prof[lane()], w.prof[lane()]);
        atomicAdd(&st.prof[64 + lane()], w.prof[64 + lane()]);
    }
#endif
}

// Generator for documents that outgrew the LDS tier: regenerated from the start in the
// paged layout (the draws are identical, so the op stream is the same).
// A tight launch hands a document that could outgrow its LDS capacities to the next launch,
// which regenerates it from the start (the draws are identical).
template <class T>
__global__ void __launch_bounds__(MT_WAVE) k_generate_paged(DevState st, mt_gen_cfg cfg, uint32_t doc_base,
                                                            mt_op_rec *ops_out, uint16_t *text_out,
                                                            uint32_t *props_out, int64_t tstride,
                                                            int64_t pstride, int32_t *fail_out,
                                                            int32_t *dbg_len, int64_t *used_out, PagedCaps pc) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS_AS uint8_t *smem = (LDS_AS uint8_t *)smem_raw;
    const int doc = blockIdx.x;
    if (doc >= st.n_docs) return;
    if (st.retry[doc] != pc.stage) return;
    const PagedLayout L = paged_layout(pc.PP, pc.PH, pc.UT, 2 * (cfg.writers + 1), (int)sizeof(typename T::O_v));
    GenCtx g;
    gen_begin(g, st, cfg, (int)(doc_base + doc), doc, smem + L.offGen, tstride, pstride);
    PagedDoc<T> pd;
    pg_setup(pd, st, doc, smem, L, pc);
    DocT<T> &w = pd.w;
    if (w.status || !pg_convert(pd, flat_src(st, doc))) {
        if (lane() == 0) {
            if (pc.tight && w.status == MT_DOC_CAPACITY) {
                st.retry[doc] = 2;
                atomicAdd(st.stats + 12, 1u);
            } else {
                fail_out[doc] = w.status == MT_DOC_RETRY ? MT_DOC_CAPACITY : w.status;
                st.retry[doc] = 0;
            }
        }
        return;
    }
    const GLB_AS uint16_t *gt = (const GLB_AS uint16_t *)(text_out + g.tb);
    const GLB_AS uint32_t *gp = (const GLB_AS uint32_t *)(props_out + g.pb);
    int pk_ut = 0, pk_heap = 0;
    for (int t = 1; t <= g.n && w.status == 0; t++) {
        int r, c, msn;
        gen_pick(g, cfg, t, r, c, msn);
        w.ocs = oslot_of(w, c);
        const int len = pg_views(pd, r, c);
        if (dbg_len && lane() == 0) {
            int32_t *q = dbg_len + (g.ob + (t - 1)) * 4;
            q[0] = len;
            q[1] = -1;
            q[2] = r;
            q[3] = c;
        }
        OpIn in;
        gen_op(g, cfg, t, r, c, msn, len, in, ops_out, text_out, props_out, doc);
        if (pc.tight && !pg_room(pd, in.op)) {
            if (lane() == 0) {
                st.retry[doc] = 2;
                atomicAdd(st.stats + 12, 1u);
            }
            return;
        }
        pg_apply_op(pd, in, gt, gp);
        pk_ut = max(pk_ut, pd.ut_n);
        pk_heap = max(pk_heap, w.heap_n);
    }
    gen_end(g, used_out, doc);
    if (w.status == MT_DOC_RETRY) w.status = MT_DOC_CAPACITY;
    if (lane() == 0) {
        if (w.status) fail_out[doc] = w.status;
        st.retry[doc] = 0;
    }
    pg_store(pd, st);
    pg_peaks(st, pd, pk_ut, pk_heap);
}

// A summary header staged by k_load_header (LoadScratch) becomes a paged document at the
// handle's full paged capacities (pg_convert from the staging buffers); the body appends
// then replay like any paged document's messages.
template <class T>
__global__ void __launch_bounds__(MT_WAVE) k_load_convert(DevState st, LoadScratch sc, PagedCaps pc, int lo) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    LDS_AS uint8_t *smem = (LDS_AS uint8_t *)smem_raw;
    const int r = blockIdx.x, doc = lo + r;   // summary r of the set -> document lo + r
    if (doc >= st.n_docs || sc.off[2 * r] < 0 || st.hdr[doc].status) return;
    const PagedLayout L = paged_layout(pc.PP, pc.PH, pc.UT, 0, (int)sizeof(typename T::O_v));
    PagedDoc<T> pd;
    pg_setup(pd, st, doc, smem, L, pc);
    DocT<T> &w = pd.w;
    FlatSrc src;
    src.A = (GLB_AS const v4i *)(sc.A + sc.off[2 * r]);
    src.O = (GLB_AS const u64 *)(sc.O + sc.off[2 * r]);
    src.Bv = (GLB_AS const v4u *)(sc.B + sc.off[2 * r]);
    src.cnt = (GLB_AS const uint8_t *)(sc.cnt + MT_LV * sc.off[2 * r + 1]);
    src.flg = (GLB_AS const int8_t *)(sc.flg + sc.off[2 * r + 1]);
    src.heap = nullptr;   // a fresh collaboration: heap_n == 0
    src.B = (size_t)w.hp->n_blk[0];
    src.os = src.ob = nullptr;   // canonical ordinals (pg_convert re-derives them)
    if (w.status == 0 && pg_convert(pd, src)) {
        pg_store(pd, st);
    } else if (lane() == 0) {
        st.hdr[doc].status = w.status == MT_DOC_RETRY || w.status == 0 ? MT_DOC_CAPACITY : w.status;
        st.hdr[doc].pad[HDR_DIAG] = w.cap_cause;
    }
}

