// mt_replay.hip -- HIP kernels and the C-ABI boundary (include/mt_replay.h) of the MI355X
// merge-tree replay backend.  Build: see fluidframework_amd/build.py (hipcc --offload-arch=gfx950).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mt_replay.h"
#include "mt_engine.h"

// ============================================================================ kernels
// Initial document contents (Client.insertSegmentLocal before collaboration: seq 0,
// client LocalClientId -1; MT/client.ts:202-215) and collaboration start
// (MT/mergeTree.ts:1287-1304): one leaf block under the root.
__global__ void __launch_bounds__(MT_WAVE) k_init(DevState st, const int64_t *seed_off,
                                                  const uint16_t *seed) {
    const int doc = blockIdx.x;
    if (doc >= st.n_docs) return;
    const int64_t s0 = seed_off ? seed_off[doc] : 0, s1 = seed_off ? seed_off[doc + 1] : 0;
    const int len = (int)(s1 - s0);
    uint16_t *text = st.text + (size_t)doc * 2 * st.T;
    for (int j = lane(); j < len && j < st.T; j += MT_WAVE) text[j] = seed[s0 + j];
    if (lane() == 0) {
        DocHdr h;
        memset(&h, 0, sizeof(h));
        h.depth = 1;
        h.n_blk[0] = 1;
        h.text_top = len;
        h.props_top = 1;
        h.next_uid = 1;
        h.delta_hash = MT_FNV_OFF;
        h.status = len > st.T ? MT_DOC_CAPACITY : 0;
        const size_t S = st.S;
        if (len > 0) {
            h.n_seg = 1;
            st.segA[doc * S] = make_int4(len, 0, MT_RSEQ_NONE, pack_cli(-1, 0));
            st.segO[doc * S] = 0ull;
            st.segB[doc * S] = make_uint4(0u, 0u, 0u, 0u);
        }
        st.cnt[(size_t)doc * MT_LV * st.B] = len > 0 ? 1 : 0;
        st.flg[(size_t)doc * st.B] = MT_SCOUR_UNDEF;
        st.hdr[doc] = h;
    }
}

// Client.applyMsg for every record of this document (one wavefront per document).
__global__ void __launch_bounds__(MT_WAVE) k_replay(DevState st, const mt_op_rec *ops,
                                                    const int64_t *off, const uint16_t *tin,
                                                    const uint32_t *pin) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int doc = blockIdx.x;
    if (doc >= st.n_docs) return;
    Doc d;
    load_doc(d, st, doc, smem);
    const int64_t k0 = off[doc], k1 = off[doc + 1];
    for (int64_t k = k0; k < k1 && d.status == 0; k++) {
        const mt_op_rec op = ops[k];
        apply_op(d, op, tin, pin);
    }
    store_doc(d);
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
__device__ static uint32_t gen_props(Rng &r, const mt_gen_cfg &cfg, uint32_t *out) {
    const uint32_t nk = 1 + rng_uniform(r, (uint32_t)cfg.max_keys_per_op);
    uint32_t count = 0;
    for (uint32_t j = 0; j < nk; j++) {
        const uint32_t key = rng_uniform(r, (uint32_t)cfg.n_keys);
        const bool is_null = (uint64_t)rng_next(r) < cfg.p_null;
        const uint32_t val = rng_uniform(r, (uint32_t)cfg.n_values);
        bool dup = false;
        for (uint32_t q = 0; q < count; q++)
            if (out[1 + 2 * q] == key) dup = true;   // lane 0 wrote these
        if (dup) continue;
        if (lane() == 0) {
            out[1 + 2 * count] = key;
            out[2 + 2 * count] = is_null ? MT_VAL_NULL : (val | (val == 0 ? MT_VAL_FALSY_BIT : 0u));
        }
        __syncthreads();
        count++;
    }
    if (lane() == 0) out[0] = count;
    __syncthreads();
    return 1 + 2 * count;
}

// Generates and applies cfg.ops messages per document (DESIGN.md "Synthetic op streams");
// the view length each writer draws positions from is read off the live replica.
__global__ void __launch_bounds__(MT_WAVE) k_generate(DevState st, mt_gen_cfg cfg, uint32_t doc_base,
                                                      mt_op_rec *ops_out, uint16_t *text_out,
                                                      uint32_t *props_out, int64_t tstride,
                                                      int64_t pstride, int32_t *fail_out,
                                                      int32_t *dbg_len) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int doc = blockIdx.x;
    if (doc >= st.n_docs) return;
    const int W = cfg.writers;
    int32_t *last_ref = (int32_t *)(smem + (MT_LV + 3) * st.B + 64 * 4);
    int32_t *short_id = last_ref + (W + 1);
    Rng rng;
    rng_init(rng, cfg.seed, (int)(doc_base + doc));
    // seed text (drawn exactly like the oracle / reference harness)
    uint16_t *arena = st.text + (size_t)doc * 2 * st.T;
    for (int i = 0; i < cfg.seed_len; i++) {
        (void)rng_next(rng);
        const uint16_t ch = (uint16_t)(97 + rng_uniform(rng, 26));
        if (lane() == 0) arena[i] = ch;
    }
    if (lane() == 0) {
        DocHdr h;
        memset(&h, 0, sizeof(h));
        h.depth = 1;
        h.n_blk[0] = 1;
        h.text_top = cfg.seed_len;
        h.props_top = 1;
        h.next_uid = 1;
        h.delta_hash = MT_FNV_OFF;
        const size_t S = st.S;
        if (cfg.seed_len > 0) {
            h.n_seg = 1;
            st.segA[doc * S] = make_int4(cfg.seed_len, 0, MT_RSEQ_NONE, pack_cli(-1, 0));
            st.segO[doc * S] = 0ull;
            st.segB[doc * S] = make_uint4(0u, 0u, 0u, 0u);
        }
        st.cnt[(size_t)doc * MT_LV * st.B] = cfg.seed_len > 0 ? 1 : 0;
        st.flg[(size_t)doc * st.B] = MT_SCOUR_UNDEF;
        st.hdr[doc] = h;
    }
    for (int j = lane(); j <= W; j += MT_WAVE) {
        last_ref[j] = 0;
        short_id[j] = 0;
    }
    __syncthreads();
    Doc d;
    load_doc(d, st, doc, smem);
    int next_short = 1;
    int64_t tu = 0, pu = 0;
    const int64_t tb = (int64_t)doc * tstride, pb = (int64_t)doc * pstride;
    for (int t = 1; t <= cfg.ops; t++) {
        const int k = 1 + (int)rng_uniform(rng, (uint32_t)W);
        int lo = max(last_ref[k], t - 1 - cfg.lag);
        if (lo < 0) lo = 0;
        const int r = lo + (int)rng_uniform(rng, (uint32_t)(t - 1 - lo + 1));
        __syncthreads();
        if (lane() == 0) last_ref[k] = r;
        __syncthreads();
        int msn = 0x7fffffff;
        for (int j = 1; j <= W; j++) msn = min(msn, last_ref[j]);
        int c = short_id[k];
        if (!c) {
            c = next_short++;
            __syncthreads();
            if (lane() == 0) short_id[k] = c;
            __syncthreads();
        }
        int vsum = 0;
        for (int base = 0; base < d.n; base += MT_WAVE) {
            const int i = base + lane();
            if (i < d.n) {
                const int4 a = d.A[i];
                vsum += view_len(a, d.O[i], r, c);
            }
        }
        const int len = wave_sum(vsum);
        if (dbg_len && lane() == 0) {
            int32_t *q = dbg_len + ((int64_t)doc * cfg.ops + (t - 1)) * 4;
            q[0] = len;
            q[1] = d.n;
            q[2] = r;
            q[3] = c;
        }
        const uint32_t u = rng_next(rng);
        mt_op_rec op;
        op.seq = t;
        op.ref_seq = r;
        op.min_seq = msn;
        op.client = (uint16_t)c;
        op.flags = 0;
        op.props = MT_NO_PROPS;
        op.payload = 0;
        if (len == 0 || (uint64_t)u < cfg.p_insert) {
            op.kind = MT_OP_INSERT;
            op.pos1 = (int)rng_uniform(rng, (uint32_t)(len + 1));
            const int tl = 1 + (int)rng_uniform(rng, (uint32_t)cfg.text_max);
            op.pos2 = tl;
            op.payload = (uint32_t)(tb + tu);
            for (int j = 0; j < tl; j++) {
                const uint32_t v = rng_next(rng);
                uint16_t ch = (uint16_t)'\n';
                if ((uint64_t)v >= cfg.p_newline) ch = (uint16_t)(97 + rng_uniform(rng, 26));
                if (lane() == 0) text_out[tb + tu + j] = ch;
            }
            tu += tl;
            if (cfg.p_insert_props > 0 && (uint64_t)rng_next(rng) < cfg.p_insert_props) {
                op.props = (uint32_t)(pb + pu);
                pu += gen_props(rng, cfg, props_out + pb + pu);
            }
        } else {
            const int p1 = (int)rng_uniform(rng, (uint32_t)len);
            int m = 1;
            while (m < 64 && (uint64_t)rng_next(rng) < cfg.p_len_continue) m++;
            op.pos1 = p1;
            op.pos2 = min(p1 + m, len);
            if ((uint64_t)u < cfg.p_insert_remove) {
                op.kind = MT_OP_REMOVE;
            } else {
                op.kind = MT_OP_ANNOTATE;
                op.props = (uint32_t)(pb + pu);
                pu += gen_props(rng, cfg, props_out + pb + pu);
            }
        }
        if (lane() == 0) ops_out[(int64_t)doc * cfg.ops + (t - 1)] = op;
        __syncthreads();
        apply_op(d, op, text_out, props_out);
        if (d.status) {
            if (lane() == 0) fail_out[doc] = d.status;
            break;
        }
    }
    store_doc(d);
}

// ---------------------------------------------------------------- checksums
__device__ static bool same_ordered(Doc &d, uint32_t ha, uint32_t hb) {
    if (ha == 0 || hb == 0) return ha == hb;
    if (ha == hb) return true;
    const uint32_t *a = prec(d, d.props_half, ha), *b = prec(d, d.props_half, hb);
    if (a[0] != b[0]) return false;
    for (uint32_t i = 0; i < 2 * a[0]; i++)
        if (a[1 + i] != b[1 + i]) return false;
    return true;
}
__device__ static u64 fold_run(Doc &d, u64 h, uint32_t ph, int len) {
    h = fnv_u32(h, (uint32_t)len);
    h = fnv_u32(h, ph ? 1u : 0u);
    if (ph) {
        const uint32_t *p = prec(d, d.props_half, ph);
        h = fnv_u32(h, p[0]);
        for (uint32_t i = 0; i < 2 * p[0]; i++) h = fnv_u32(h, p[1 + i]);
    }
    return h;
}
// mt_checksum per document (definitions: DESIGN.md "Checksums", oracle/mt_oracle.c).
__global__ void __launch_bounds__(MT_WAVE) k_checksum(DevState st, mt_checksum *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int doc = blockIdx.x;
    if (doc >= st.n_docs) return;
    Doc d;
    load_doc(d, st, doc, smem);
    int len = 0, ntext = 0;
    for (int base = 0; base < d.n; base += MT_WAVE) {
        const int i = base + lane();
        int l = 0, t = 0;
        if (i < d.n) {
            const int4 a = d.A[i];
            l = obs_len(a);
            t = (d.Bv[i].z & MT_MARKER_BIT) ? 0 : l;
        }
        len += wave_sum(l);
        ntext += wave_sum(t);
    }
    if (lane() == 0) {
        const uint16_t *tb = text_base(d, d.text_half);
        u64 th = fnv_u32(MT_FNV_OFF, (uint32_t)ntext), hk = MT_FNV_OFF, ph = MT_FNV_OFF;
        int g = 0, run_len = 0;
        bool have = false;
        uint32_t run_p = 0;
        for (int i = 0; i < d.n; i++) {
            const int4 a = d.A[i];
            const uint4 b = d.Bv[i];
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
            if (have && same_ordered(d, run_p, b.y)) {
                run_len += a.x;
            } else {
                if (have) ph = fold_run(d, ph, run_p, run_len);
                run_p = b.y;
                run_len = a.x;
                have = true;
            }
        }
        if (g & 63) th = fnv_u64(th, hk);
        if (have) ph = fold_run(d, ph, run_p, run_len);
        mt_checksum cs;
        cs.length = (uint32_t)len;
        cs.n_segments = (uint32_t)d.n;
        cs.text_hash = th;
        cs.props_hash = ph;
        cs.delta_hash = d.dhash;
        out[doc] = cs;
    }
}

// ============================================================================ host side
struct mt_handle {
    int device = 0;
    uint32_t n_docs = 0;
    DevState st{};
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.f;
    bool timed = false;      // ev0/ev1 bracket a launch not yet read by mt_sync
    std::string err;
    mt_checksum *d_sums = nullptr;
    int64_t *d_seed_off = nullptr;   // initial contents kept on device for mt_reset
    uint16_t *d_seed = nullptr;
};
struct mt_batch {
    int device = 0;
    uint32_t n_docs = 0;
    uint64_t n_ops = 0, text_len = 0, props_len = 0;
    int64_t *off = nullptr;
    mt_op_rec *ops = nullptr;
    uint16_t *text = nullptr;
    uint32_t *props = nullptr;
};

#define HIPCHK(h, x)                                                               \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            if (h) (h)->err = std::string(#x) + ": " + hipGetErrorString(e_);      \
            return MT_E_HIP;                                                       \
        }                                                                          \
    } while (0)

static size_t lds_bytes(const DevState &st, int extra_ints) {
    return (size_t)(MT_LV + 3) * st.B + 64 * 4 + (size_t)extra_ints * 4;
}

extern "C" {

mt_handle *mt_create(uint32_t n_docs, const mt_options *opt) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return nullptr;
    mt_options o{};
    if (opt) o = *opt;
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
    alloc((void **)&st.text, N * 2 * (size_t)st.T * sizeof(uint16_t));
    alloc((void **)&st.props, N * 2 * (size_t)st.P * MT_PREC * sizeof(uint32_t));
    if (st.DL) alloc((void **)&st.dlog, N * (size_t)st.DL * sizeof(int32_t));
    alloc((void **)&h->d_sums, N * sizeof(mt_checksum));
    if (!ok || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) {
        mt_destroy(h);
        return nullptr;
    }
    if (mt_load_initial_text(h, nullptr, nullptr) != 0) {
        mt_destroy(h);
        return nullptr;
    }
    return h;
}

void mt_destroy(mt_handle *h) {
    if (!h) return;
    hipSetDevice(h->device);
    DevState &st = h->st;
    void *ps[] = {st.hdr, st.segA, st.segO, st.segB, st.cnt, st.flg, st.heap, st.text, st.props, st.dlog, h->d_sums,
                  h->d_seed_off, h->d_seed};
    for (void *p : ps)
        if (p) hipFree(p);
    if (h->ev0) hipEventDestroy(h->ev0);
    if (h->ev1) hipEventDestroy(h->ev1);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
}

const char *mt_last_error(const mt_handle *h) { return h ? h->err.c_str() : "null handle"; }
uint32_t mt_num_docs(const mt_handle *h) { return h ? h->n_docs : 0; }

int mt_load_initial_text(mt_handle *h, const int64_t *seed_off, const uint16_t *seed_text) {
    if (!h) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->d_seed_off) hipFree(h->d_seed_off);
    if (h->d_seed) hipFree(h->d_seed);
    h->d_seed_off = nullptr;
    h->d_seed = nullptr;
    if (seed_off) {
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
    HIPCHK(h, hipSetDevice(h->device));
    if (h->st.DL) HIPCHK(h, hipMemsetAsync(h->st.dlog, 0, (size_t)h->n_docs * h->st.DL * 4, h->stream));
    hipLaunchKernelGGL(k_init, dim3(h->n_docs), dim3(MT_WAVE), 0, h->stream, h->st, h->d_seed_off, h->d_seed);
    HIPCHK(h, hipGetLastError());
    return 0;
}

mt_batch *mt_batch_upload(mt_handle *h, const int64_t *doc_op_off, const mt_op_rec *ops,
                          uint64_t n_ops, const uint16_t *text, uint64_t text_len,
                          const uint32_t *props, uint64_t props_len) {
    if (!h || !doc_op_off) return nullptr;
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
    }
    if (!ok) {
        h->err = "mt_batch_upload: device allocation/copy failed";
        mt_batch_free(b);
        return nullptr;
    }
    return b;
}

int mt_batch_apply_async(mt_handle *h, const mt_batch *b) {
    if (!h || !b || b->n_docs != h->n_docs) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipEventRecord(h->ev0, h->stream));
    hipLaunchKernelGGL(k_replay, dim3(h->n_docs), dim3(MT_WAVE), lds_bytes(h->st, 0), h->stream, h->st,
                       b->ops, b->off, b->text, b->props);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipEventRecord(h->ev1, h->stream));
    h->timed = true;
    return 0;
}

uint64_t mt_batch_num_ops(const mt_batch *b) { return b ? b->n_ops : 0; }

void mt_batch_free(mt_batch *b) {
    if (!b) return;
    hipSetDevice(b->device);
    if (b->off) hipFree(b->off);
    if (b->ops) hipFree(b->ops);
    if (b->text) hipFree(b->text);
    if (b->props) hipFree(b->props);
    delete b;
}

int mt_sync(mt_handle *h) {
    if (!h) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->timed) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, h->ev0, h->ev1) == hipSuccess) h->last_ms = ms;
        (void)hipGetLastError();   // never leave a sticky error for the next launch check
        h->timed = false;
    }
    return 0;
}

float mt_last_kernel_ms(const mt_handle *h) { return h ? h->last_ms : 0.f; }

int mt_apply_ops(mt_handle *h, const int64_t *doc_op_off, const mt_op_rec *ops, uint64_t n_ops,
                 const uint16_t *text, uint64_t text_len, const uint32_t *props,
                 uint64_t props_len) {
    mt_batch *b = mt_batch_upload(h, doc_op_off, ops, n_ops, text, text_len, props, props_len);
    if (!b) return MT_E_NOMEM;
    int rc = mt_batch_apply_async(h, b);
    if (rc == 0) rc = mt_sync(h);
    mt_batch_free(b);
    return rc;
}

mt_batch *mt_generate(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base,
                      int32_t *view_len_trace) {
    if (!h || !cfg || cfg->writers < 1 || cfg->ops < 0) return nullptr;
    if (hipSetDevice(h->device) != hipSuccess) return nullptr;
    auto *b = new mt_batch();
    b->device = h->device;
    b->n_docs = h->n_docs;
    const int64_t N = h->n_docs, ops = cfg->ops;
    const int64_t tstride = ops * cfg->text_max + 1;
    const int64_t pstride = ops * (1 + 2 * (int64_t)cfg->max_keys_per_op) + 1;
    b->n_ops = N * ops;
    b->text_len = N * tstride;
    b->props_len = N * pstride;
    int32_t *d_fail = nullptr, *d_trace = nullptr;
    if (view_len_trace && hipMalloc(&d_trace, std::max<int64_t>(N * ops, 1) * 16) != hipSuccess) {
        delete b;
        return nullptr;
    }
    bool ok = hipMalloc(&b->off, (N + 1) * sizeof(int64_t)) == hipSuccess &&
              hipMalloc(&b->ops, std::max<int64_t>(b->n_ops, 1) * sizeof(mt_op_rec)) == hipSuccess &&
              hipMalloc(&b->text, b->text_len * 2) == hipSuccess &&
              hipMalloc(&b->props, b->props_len * 4) == hipSuccess &&
              hipMalloc(&d_fail, N * 4) == hipSuccess;
    if (ok) {
        std::vector<int64_t> off(N + 1);
        for (int64_t i = 0; i <= N; i++) off[i] = i * ops;
        ok = hipMemcpy(b->off, off.data(), (N + 1) * 8, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemset(d_fail, 0, N * 4) == hipSuccess;
    }
    if (ok) {
        const size_t lds = lds_bytes(h->st, 2 * (cfg->writers + 1));
        hipLaunchKernelGGL(k_generate, dim3(h->n_docs), dim3(MT_WAVE), lds, h->stream, h->st, *cfg,
                           doc_index_base, b->ops, b->text, b->props, tstride, pstride, d_fail,
                           d_trace);
        ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(h->stream) == hipSuccess;
    }
    if (ok) {
        std::vector<int32_t> f(N);
        ok = hipMemcpy(f.data(), d_fail, N * 4, hipMemcpyDeviceToHost) == hipSuccess;
        for (int64_t i = 0; ok && i < N; i++)
            if (f[i]) {
                h->err = "mt_generate: document " + std::to_string(i) + " failed with status " + std::to_string(f[i]);
                ok = false;
            }
    }
    if (ok && d_trace)
        ok = hipMemcpy(view_len_trace, d_trace, N * ops * 16, hipMemcpyDeviceToHost) == hipSuccess;
    if (d_trace) hipFree(d_trace);
    if (d_fail) hipFree(d_fail);
    if (!ok) {
        if (h->err.empty()) h->err = "mt_generate failed";
        mt_batch_free(b);
        return nullptr;
    }
    return b;
}

int mt_generated_seeds(mt_handle *h, const mt_gen_cfg *cfg, uint32_t doc_index_base,
                       int64_t *seed_off, uint16_t *seed_text) {
    if (!h || !cfg) return MT_E_INVALID;
    int64_t pos = 0;
    for (uint32_t doc = 0; doc < h->n_docs; doc++) {
        seed_off[doc] = pos;
        Rng r;
        rng_init(r, cfg->seed, (int)(doc_index_base + doc));
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
};
static int fetch_doc(mt_handle *h, uint32_t doc, HostDoc &hd, bool with_text, bool with_props) {
    if (!h || doc >= h->n_docs) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const DevState &st = h->st;
    HIPCHK(h, hipMemcpy(&hd.hdr, st.hdr + doc, sizeof(DocHdr), hipMemcpyDeviceToHost));
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
    if (with_text) {
        hd.text.resize(st.T);
        HIPCHK(h, hipMemcpy(hd.text.data(), st.text + ((size_t)doc * 2 + hd.hdr.text_half) * st.T, st.T * 2,
                            hipMemcpyDeviceToHost));
    }
    if (with_props) {
        const size_t words = (size_t)st.P * MT_PREC;
        hd.props.resize(words);
        HIPCHK(h, hipMemcpy(hd.props.data(), st.props + ((size_t)doc * 2 + hd.hdr.props_half) * words, words * 4,
                            hipMemcpyDeviceToHost));
    }
    return 0;
}

int mt_get_status(mt_handle *h, int32_t *out_status) {
    if (!h || !out_status) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
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
        r[0] = a.x;
        r[1] = a.y;
        r[2] = (int)(short)(a.w & 0xFFFF);
        r[3] = a.z;
        r[4] = a.z == MT_RSEQ_NONE ? MT_RSEQ_NONE : (int)(short)((uint32_t)a.w >> 16);
        r[5] = __builtin_popcountll(hd.O[i]);
        r[6] = (b.z & MT_MARKER_BIT) ? (int32_t)b.x : -1;
        r[7] = b.y ? 1 : 0;
    }
    if (n_rows) *n_rows = (uint32_t)n;
    const int nb0 = hd.hdr.n_blk[0];
    for (int b = 0; b < nb0 && leaves && (uint32_t)b < cap_leaves; b++) leaves[b] = hd.cnt[b];
    if (n_leaves) *n_leaves = (uint32_t)nb0;
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

int mt_get_delta_log(mt_handle *h, uint32_t doc, int32_t *out, uint32_t cap, uint32_t *n) {
    if (!h || doc >= h->n_docs) return MT_E_INVALID;
    if (!h->st.DL) {
        if (n) *n = 0;
        return 0;
    }
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    DocHdr hdr;
    HIPCHK(h, hipMemcpy(&hdr, h->st.hdr + doc, sizeof(DocHdr), hipMemcpyDeviceToHost));
    const uint32_t cnt = std::min<uint32_t>((uint32_t)hdr.dlog_n, cap);
    if (out && cnt) HIPCHK(h, hipMemcpy(out, h->st.dlog + (size_t)doc * h->st.DL, cnt * 4, hipMemcpyDeviceToHost));
    if (n) *n = (uint32_t)hdr.dlog_n;
    return 0;
}

int mt_checksums_device(mt_handle *h, void *device_out) {
    if (!h || !device_out) return MT_E_INVALID;
    HIPCHK(h, hipSetDevice(h->device));
    hipLaunchKernelGGL(k_checksum, dim3(h->n_docs), dim3(MT_WAVE), lds_bytes(h->st, 0), h->stream, h->st,
                       (mt_checksum *)device_out);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return 0;
}

int mt_checksums(mt_handle *h, mt_checksum *out) {
    if (!h || !out) return MT_E_INVALID;
    int rc = mt_checksums_device(h, h->d_sums);
    if (rc) return rc;
    HIPCHK(h, hipMemcpy(out, h->d_sums, h->n_docs * sizeof(mt_checksum), hipMemcpyDeviceToHost));
    return 0;
}

}  // extern "C"
