// fetch_probe.hip -- calibrates the PMC FETCH_SIZE counter on the replay kernel's own read
// patterns (DESIGN.md §4 "Roofline accounting"; MI355X_MICROARCH.md: FETCH_SIZE reports 1/2
// of a wide coalesced 16 B/lane stream on gfx950).  Each dispatch reads a known set of bytes
// from a buffer far larger than the caches, once:
//   stream  -- 16 B per lane, coalesced, every line once (the guide's 1/2 case)
//   pages   -- k_replay_paged's window fetch: per access a random page, lanes 0..21 read the
//              slot's 16 B A word, 8 B O word and 16 B B word (22 live slots of 64)
//   probe16 -- the uid -> page map probe: one random 2-byte read per access
//   text8   -- a text gather: 8 consecutive UTF-16 units (16 B) at a random position
// Build (container): hipcc --offload-arch=gfx950 -O3 -o profiles/tools/fetch_probe profiles/tools/fetch_probe.hip
// Run (GPU box):     rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d <dir> -- profiles/tools/fetch_probe
// It prints, per dispatch, the bytes the lanes request and the bytes of the distinct 64-byte and
// 128-byte lines they touch; profiles/tools/fetch_probe.py puts them next to FETCH_SIZE.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CHK(x)                                                                             \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                          \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__global__ void __launch_bounds__(256) k_stream(const uint4 *a, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x1234u) sink[0] = acc;
}

// one wave per 64 threads; `per_wave` accesses each; page p of n_pages: A at a + p*64 (uint4),
// O at o + p*64 (u64), B at b + p*64 (uint4) -- the paged layout's slot arrays
__global__ void __launch_bounds__(64) k_pages(const uint4 *a, const uint64_t *o, const uint4 *b, uint32_t n_pages,
                                              int per_wave, uint32_t *sink) {
    const int l = threadIdx.x;
    uint32_t acc = 0;
    for (int k = 0; k < per_wave; k++) {
        // a bijection of the access id onto the pages: every page once
        const uint32_t p = ((blockIdx.x * (uint32_t)per_wave + k) * 0x9E3779B1u) & (n_pages - 1);
        if (l < 22) {
            const uint4 va = a[(size_t)p * 64 + l];
            const uint64_t vo = o[(size_t)p * 64 + l];
            const uint4 vb = b[(size_t)p * 64 + l];
            acc ^= va.x ^ va.w ^ (uint32_t)vo ^ vb.y ^ vb.z;
        }
    }
    if (acc == 0x1234u) sink[0] = acc;
}

__global__ void __launch_bounds__(64) k_probe16(const uint16_t *m, size_t n, int per_wave, uint32_t *sink) {
    uint32_t acc = 0;
    for (int k = 0; k < per_wave; k++) {
        const size_t i = ((size_t)((blockIdx.x * (uint32_t)per_wave + k) * 0x9E3779B1u) << 11) & (n - 1);
        if (threadIdx.x == 0) acc ^= m[i];
    }
    if (acc == 0x1234u) sink[0] = acc;
}

__global__ void __launch_bounds__(64) k_text8(const uint16_t *t, size_t n, int per_wave, uint32_t *sink) {
    uint32_t acc = 0;
    for (int k = 0; k < per_wave; k++) {
        const size_t i = ((((size_t)((blockIdx.x * (uint32_t)per_wave + k) * 0x9E3779B1u) << 11) +
                          (mix(blockIdx.x * 64u + k) & 2047u)) & (n - 1)) % (n - 8);
        if (threadIdx.x < 8) acc ^= t[i + threadIdx.x];
    }
    if (acc == 0x1234u) sink[0] = acc;
}

int main() {
    const size_t n_pages = 1u << 20;              // 1 Mi pages: 64 MiB A + 32 MiB O + 64 MiB B per 64 Ki pages
    const size_t slots = n_pages * 64;
    const size_t text_units = (size_t)1 << 31;    // 4 GiB of UTF-16 units
    const int waves = 16384, per_wave = 64;
    uint4 *a = nullptr, *b = nullptr;
    uint64_t *o = nullptr;
    uint16_t *t = nullptr;
    uint32_t *sink = nullptr;
    CHK(hipMalloc(&a, slots * sizeof(uint4)));
    CHK(hipMalloc(&b, slots * sizeof(uint4)));
    CHK(hipMalloc(&o, slots * sizeof(uint64_t)));
    CHK(hipMalloc(&t, text_units * 2));
    CHK(hipMalloc(&sink, 4));
    CHK(hipMemset(a, 1, slots * sizeof(uint4)));
    CHK(hipMemset(b, 2, slots * sizeof(uint4)));
    CHK(hipMemset(o, 3, slots * sizeof(uint64_t)));
    CHK(hipMemset(t, 4, text_units * 2));
    // evict: the stream pass below reads 1 GiB first, after the 6 GiB of memsets
    const size_t stream_n = ((size_t)1 << 30) / sizeof(uint4);
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4 *)t, stream_n, sink);
    CHK(hipDeviceSynchronize());
    printf("{\"kernel\": \"k_stream\", \"requested\": %zu, \"lines64\": %zu, \"lines128\": %zu}\n", stream_n * 16,
           stream_n * 16, stream_n * 16);
    hipLaunchKernelGGL(k_pages, dim3(waves), dim3(64), 0, 0, a, o, b, (uint32_t)n_pages, per_wave, sink);
    CHK(hipDeviceSynchronize());
    {   // 22 slots: A 352 B (6 x 64 B lines if page-aligned: 352 / 64 -> 5.5 -> 6; 3 x 128 B), O 176 B
        // (3 x 64, 2 x 128), B 352 B (6 x 64, 3 x 128); pages are 1 KiB / 512 B aligned
        const size_t acc = (size_t)waves * per_wave;
        printf("{\"kernel\": \"k_pages\", \"requested\": %zu, \"lines64\": %zu, \"lines128\": %zu}\n", acc * 22 * 40,
               acc * (6 + 3 + 6) * 64, acc * (3 + 2 + 3) * 128);
    }
    hipLaunchKernelGGL(k_probe16, dim3(waves), dim3(64), 0, 0, t, text_units, per_wave, sink);
    CHK(hipDeviceSynchronize());
    {
        const size_t acc = (size_t)waves * per_wave;
        printf("{\"kernel\": \"k_probe16\", \"requested\": %zu, \"lines64\": %zu, \"lines128\": %zu}\n", acc * 2,
               acc * 64, acc * 128);
    }
    hipLaunchKernelGGL(k_text8, dim3(waves), dim3(64), 0, 0, t, text_units, per_wave, sink);
    CHK(hipDeviceSynchronize());
    {   // 16 B at a random 2-byte offset: 1.25 x 64 B lines on average (crosses a 64 B line with
        // probability 14/32... computed exactly: offsets 0..31 units in a line, crossing when > 24)
        const size_t acc = (size_t)waves * per_wave;
        printf("{\"kernel\": \"k_text8\", \"requested\": %zu, \"lines64\": %zu, \"lines128\": %zu}\n", acc * 16,
               acc * 64 * 39 / 32, acc * 128 * 71 / 64);
    }
    hipFree(a);
    hipFree(b);
    hipFree(o);
    hipFree(t);
    hipFree(sink);
    return 0;
}
