// HBM streaming roof of one MI355X (profiles/hbm_roof.md): what a pure stream of 16-B-per-lane accesses
// sustains, so the BatchNorm / pool / streaming-conv passes can be judged against the device's own ceiling
// instead of a copy kernel of the framework.
//
// Patterns (bytes per element-slot: r = read, w = written):
//   read   : r 1, w 0  (sum folded into one store per thread)
//   write  : r 0, w 1
//   copy   : r 1, w 1
//   r2w1   : r 2, w 1  (the BN-backward apply pass: g, x in, dx out)
//   r1w1x  : r 1, w 1 plus a second read stream of the same size (= r2w1 with a multiply) -- alias of r2w1
// Swept: loads in flight per lane U (4 / 8 / 16, all issued before any use), blocks (256 threads) per launch,
// plain vs non-temporal (NT) loads + stores. Buffers 4 GiB per stream (16x the 256 MiB MALL), 10 timed reps after
// 2 warm-ups, best and median reported as TB/s of HBM bytes (reads + writes).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/hbm_roof.hip -o /tmp/hbm_roof && /tmp/hbm_roof [GiB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, const u32x4& v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// PAT 0 read, 1 write, 2 copy, 3 r2w1. n = 16-B chunks per stream. Chunk index of (iteration it, slot u):
// it * grid * 256 * U + blockIdx * 256 * U + u * 256 + tid -- every slot is one coalesced 1-KiB wave access.
template <int PAT, int U, bool NT>
__global__ __launch_bounds__(256) void stream_kernel(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                     u32x4* __restrict__ o, size_t n, uint32_t* sink) {
    const size_t per_iter = (size_t)gridDim.x * 256 * U;
    u32x4 acc = {0u, 0u, 0u, 0u};
    const u32x4 k = {threadIdx.x, 1u, 2u, 3u};
    for (size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x; base < n; base += per_iter) {
        u32x4 va[U], vb[U];
        if (PAT != 1) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t i = std::min(base + (size_t)u * 256, n - 1);
                va[u] = ld<NT>(a + i);
                if (PAT == 3) vb[u] = ld<NT>(b + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + (size_t)u * 256;
            if (i >= n) break;
            if (PAT == 0) acc ^= va[u];
            else if (PAT == 1) st<NT>(o + i, k);
            else if (PAT == 2) st<NT>(o + i, va[u]);
            else st<NT>(o + i, va[u] + vb[u]);
        }
    }
    if (PAT == 0 && (acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9e3779b9u) sink[0] = 1;  // keeps the loads live
}

template <int PAT, int U, bool NT>
double run(const u32x4* a, const u32x4* b, u32x4* o, size_t n, uint32_t* sink, int grid, double* med) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> t;
    for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((stream_kernel<PAT, U, NT>), dim3(grid), dim3(256), 0, 0, a, b, o, n, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    std::sort(t.begin(), t.end());
    const double bytes = (double)n * 16.0 * (PAT == 0 ? 1 : PAT == 1 ? 1 : PAT == 2 ? 2 : 3);
    *med = bytes / (t[t.size() / 2] * 1e-3) / 1e12;
    return bytes / (t[0] * 1e-3) / 1e12;
}

template <int PAT>
void sweep(const char* name, const u32x4* a, const u32x4* b, u32x4* o, size_t n, uint32_t* sink, int cus) {
    double best = 0.0;
    for (int bpc : {2, 4, 8, 16, 32}) {
        const int grid = bpc * cus;
        double m[6], v[6];
        v[0] = run<PAT, 4, false>(a, b, o, n, sink, grid, &m[0]);
        v[1] = run<PAT, 8, false>(a, b, o, n, sink, grid, &m[1]);
        v[2] = run<PAT, 16, false>(a, b, o, n, sink, grid, &m[2]);
        v[3] = run<PAT, 4, true>(a, b, o, n, sink, grid, &m[3]);
        v[4] = run<PAT, 8, true>(a, b, o, n, sink, grid, &m[4]);
        v[5] = run<PAT, 16, true>(a, b, o, n, sink, grid, &m[5]);
        printf("| %s | %d | %.2f / %.2f | %.2f / %.2f | %.2f / %.2f | %.2f / %.2f | %.2f / %.2f | %.2f / %.2f |\n", name,
               bpc, v[0], m[0], v[1], m[1], v[2], m[2], v[3], m[3], v[4], m[4], v[5], m[5]);
        for (double x : v) best = std::max(best, x);
    }
    printf("| **%s best** | | **%.2f** TB/s | | | | | |\n", name, best);
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 4.0;
    const size_t n = (size_t)(gib * (1ull << 30)) / 16;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    u32x4 *a, *b, *o;
    uint32_t* sink;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMalloc(&o, n * 16));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(a, 0x3c, n * 16));
    CK(hipMemset(b, 0x3c, n * 16));
    CK(hipMemset(o, 0, n * 16));
    if (argc > 2 && argv[2][0] == 'c') {  // counter calibration: one launch per pattern, known bytes
        double m;
        printf("calibration launches (GiB per stream %.2f): read, write, copy, r2w1 (plain), then NT\n", gib);
        run<0, 8, false>(a, b, o, n, sink, 4 * cus, &m);
        run<1, 8, false>(a, b, o, n, sink, 4 * cus, &m);
        run<2, 8, false>(a, b, o, n, sink, 4 * cus, &m);
        run<3, 8, false>(a, b, o, n, sink, 4 * cus, &m);
        run<0, 8, true>(a, b, o, n, sink, 4 * cus, &m);
        run<1, 8, true>(a, b, o, n, sink, 4 * cus, &m);
        run<2, 8, true>(a, b, o, n, sink, 4 * cus, &m);
        run<3, 8, true>(a, b, o, n, sink, 4 * cus, &m);
        return 0;
    }
    printf("%d CUs, %.1f GiB per stream; TB/s best / median of 10 reps (reads + writes)\n\n", cus, gib);
    printf("| pattern | blocks/CU | U4 | U8 | U16 | U4 NT | U8 NT | U16 NT |\n|---|---:|---:|---:|---:|---:|---:|---:|\n");
    sweep<0>("read", a, b, o, n, sink, cus);
    sweep<1>("write", a, b, o, n, sink, cus);
    sweep<2>("copy", a, b, o, n, sink, cus);
    sweep<3>("r2w1", a, b, o, n, sink, cus);
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(o));
    CK(hipFree(sink));
    return 0;
}
