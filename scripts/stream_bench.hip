// Streaming-pass microbenchmark for the BatchNorm apply kernels' access pattern (bn.hip):
// out = a*k1 + b*k2 + k0 over bf16 [R][C] rows (two 16-B streams in, one out), swept over the
// row -> block mapping, rows in flight per thread, grid size and store policy.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/stream_bench.hip -o /tmp/stream_bench
//   ./stream_bench [R C]         (default: the 256 @ 56x56 x 1024 shape, 822 M elements)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
    uint32_t a = __float_as_uint(lo), b = __float_as_uint(hi);
    a += 0x7fffu + ((a >> 16) & 1u);
    b += 0x7fffu + ((b >> 16) & 1u);
    return (a >> 16) | (b & 0xffff0000u);
}
__device__ __forceinline__ float bfw(const u32x4& w, int i) { return (i & 1) ? hi_bf(w[i >> 1]) : lo_bf(w[i >> 1]); }

// MAP 0: grid-stride, the U rows of a thread are gridDim*rpb rows apart (bn.hip today)
// MAP 1: block-contiguous, a block's iteration covers U*rpb consecutive rows
template <int U, int MAP, bool NT>
__global__ __launch_bounds__(256) void apply_kernel(const uint16_t* __restrict__ a, const uint16_t* __restrict__ b,
                                                    uint16_t* __restrict__ o, const float* __restrict__ kk, long R,
                                                    int C) {
    const int cpr = C / 8, rpb = 256 / cpr, tid = threadIdx.x;
    if (tid >= rpb * cpr) return;
    const int c0 = (tid % cpr) * 8;
    float k1[8], k2[8], k0[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        k1[i] = kk[c0 + i];
        k2[i] = kk[C + c0 + i];
        k0[i] = kk[2 * C + c0 + i];
    }
    const long rsub = tid / cpr;
    const long gstep = MAP == 0 ? (long)gridDim.x * rpb : (long)rpb;
    const long istep = MAP == 0 ? (long)U * gridDim.x * rpb : (long)U * gridDim.x * rpb;
    const long base0 = MAP == 0 ? (long)blockIdx.x * rpb : (long)blockIdx.x * U * rpb;
    for (long r0 = base0 + rsub; r0 < R; r0 += istep) {
        u32x4 va[U], vb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t off = (size_t)min(r0 + u * gstep, R - 1) * C + c0;
            va[u] = *reinterpret_cast<const u32x4*>(a + off);
            vb[u] = *reinterpret_cast<const u32x4*>(b + off);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long r = r0 + u * gstep;
            if (r >= R) break;
            u32x4 w;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float x0 = fmaf(k1[2 * i], bfw(va[u], 2 * i), fmaf(k2[2 * i], bfw(vb[u], 2 * i), k0[2 * i]));
                const float x1 =
                    fmaf(k1[2 * i + 1], bfw(va[u], 2 * i + 1), fmaf(k2[2 * i + 1], bfw(vb[u], 2 * i + 1), k0[2 * i + 1]));
                w[i] = pack_bf2(x0, x1);
            }
            u32x4* dst = reinterpret_cast<u32x4*>(o + (size_t)r * C + c0);
            if (NT) __builtin_nontemporal_store(w, dst);
            else *dst = w;
        }
    }
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

template <int U, int MAP, bool NT>
void run(const char* name, const uint16_t* a, const uint16_t* b, uint16_t* o, const float* kk, long R, int C,
         int grid) {
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((apply_kernel<U, MAP, NT>), dim3(grid), dim3(256), 0, 0, a, b, o, kk, R, C);
    CK(hipGetLastError());
    const int reps = 10;
    CK(hipEventRecord(s));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((apply_kernel<U, MAP, NT>), dim3(grid), dim3(256), 0, 0, a, b, o, kk, R, C);
    CK(hipEventRecord(e));
    CK(hipEventSynchronize(e));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, s, e));
    const double us = ms * 1e3 / reps, bytes = 3.0 * R * C * 2;
    printf("%-28s grid %6d  %8.1f us  %5.2f TB/s\n", name, grid, us, bytes / us / 1e6);
    fflush(stdout);
    CK(hipEventDestroy(s));
    CK(hipEventDestroy(e));
}

int main(int argc, char** argv) {
    const long R = argc > 2 ? atol(argv[1]) : 1024L * 56 * 56;
    const int C = argc > 2 ? atoi(argv[2]) : 256;
    if (C % 8 || 256 % (C / 8)) {
        fprintf(stderr, "C must be a multiple of 8 with C/8 dividing 256\n");
        return 1;
    }
    const size_t n = (size_t)R * C;
    uint16_t *a, *b, *o;
    float* kk;
    CK(hipMalloc(&a, n * 2));
    CK(hipMalloc(&b, n * 2));
    CK(hipMalloc(&o, n * 2));
    CK(hipMalloc(&kk, 3 * C * sizeof(float)));
    CK(hipMemset(a, 0x3f, n * 2));
    CK(hipMemset(b, 0x3f, n * 2));
    CK(hipMemset(kk, 0, 3 * C * sizeof(float)));
    printf("R %ld C %d (%.1f MB per stream)\n", R, C, n * 2 / 1e6);
    const int rpb = 256 / (C / 8);
    auto full = [&](int u) { return (int)((R + (long)u * rpb - 1) / ((long)u * rpb)); };
    for (int g : {1024, 2048, 4096}) {
        run<4, 0, false>("U4 grid-stride", a, b, o, kk, R, C, g);
        run<4, 1, false>("U4 block-contig", a, b, o, kk, R, C, g);
        run<4, 0, true>("U4 grid-stride nt", a, b, o, kk, R, C, g);
        run<4, 1, true>("U4 block-contig nt", a, b, o, kk, R, C, g);
        run<2, 1, false>("U2 block-contig", a, b, o, kk, R, C, g);
        run<8, 1, false>("U8 block-contig", a, b, o, kk, R, C, g);
    }
    run<1, 1, false>("U1 one row/thread (no loop)", a, b, o, kk, R, C, full(1));
    run<2, 1, false>("U2 no loop", a, b, o, kk, R, C, full(2));
    run<4, 1, false>("U4 no loop", a, b, o, kk, R, C, full(4));
    run<1, 1, true>("U1 no loop nt", a, b, o, kk, R, C, full(1));
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(o));
    CK(hipFree(kk));
    return 0;
}
