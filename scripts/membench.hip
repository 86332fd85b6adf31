// Read-bandwidth probe for the streaming 1x1 conv's operand pattern (conv_stream.hip), gfx950.
// Each wave walks 16-pixel groups of a [M][K] bf16 matrix (row = K * 2 bytes) with a prefetch D groups deep and
// folds every loaded dword into a checksum (so nothing is dead code). Patterns:
//   0 contiguous: instruction i of a group loads 1 KB contiguous (lane l: bytes i*1024 + l*16) -- the BN passes' form
//   1 mfma: lane (fr = l & 15, fq = l >> 4) loads row fr, bytes fq*16 + i*64 -- 16 rows x 64 B per instruction (the
//     16x16x32 B-fragment layout the streaming kernel loads straight into registers)
//   2 mfma32: as 1, but each lane takes 32 contiguous bytes (two 16-B loads, bytes fq*32 + j*16 + (i/2)*128)
// Build: hipcc --offload-arch=gfx950 -O3 -o membench scripts/membench.hip ; run: ./membench [M] [K]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int K, int D, int PAT>
__global__ __launch_bounds__(256, 2) void probe(const char* __restrict__ x, long M, unsigned* out) {
    constexpr int NI = K * 2 / 64;  // 16-B loads per lane per group (16 rows x K*2 bytes / 64 lanes / 16 B)
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long ngroups = M / 16;
    const long w0 = (long)blockIdx.x * 4 + wid, ws = (long)gridDim.x * 4;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(x), (short)0, 0x7FFFFFFF, 0x00020000);
    auto off = [&](int i) -> unsigned {
        const int fr = lane & 15, fq = lane >> 4;
        if (PAT == 0) return i * 1024 + lane * 16;
        if (PAT == 1) return fr * K * 2 + fq * 16 + i * 64;
        return fr * K * 2 + fq * 32 + (i & 1) * 16 + (i >> 1) * 128;
    };
    u32x4 pf[D][NI];
    unsigned acc = 0;
    auto fetch = [&](int d, long g) {
        const char* base = x + (g < ngroups ? g : 0) * 16 * K * 2;
        const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0,
                                                                            g < ngroups ? 0x7FFFFFFF : 0, 0x00020000);
#pragma unroll
        for (int i = 0; i < NI; ++i) pf[d][i] = __builtin_amdgcn_raw_buffer_load_b128(rg, off(i), 0, 0);
    };
    (void)r;
#pragma unroll
    for (int d = 0; d < D; ++d) fetch(d, w0 + d * ws);
    for (long g0 = w0; g0 < ngroups; g0 += D * ws) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            u32x4 v[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i) v[i] = pf[d][i];
            fetch(d, g0 + d * ws + D * ws);
#pragma unroll
            for (int i = 0; i < NI; ++i) acc += v[i][0] ^ v[i][1] ^ v[i][2] ^ v[i][3];
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int K, int D, int PAT>
float run(const char* x, long M, unsigned* out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((probe<K, D, PAT>), dim3(blocks), dim3(256), 0, 0, x, M, out);
    hipEventRecord(a);
    const int reps = 10;
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((probe<K, D, PAT>), dim3(blocks), dim3(256), 0, 0, x, M, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

template <int K>
void sweep(const char* x, long M, unsigned* out) {
    const double bytes = (double)M * K * 2;
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int bpc : {2, 4}) {
        const int blocks = cus * bpc;
        const char* names[3] = {"contiguous", "mfma16x64B", "mfma32B"};
        float t[3][2];
        t[0][0] = run<K, 2, 0>(x, M, out, blocks);
        t[1][0] = run<K, 2, 1>(x, M, out, blocks);
        t[2][0] = run<K, 2, 2>(x, M, out, blocks);
        t[0][1] = run<K, 4, 0>(x, M, out, blocks);
        t[1][1] = run<K, 4, 1>(x, M, out, blocks);
        t[2][1] = run<K, 4, 2>(x, M, out, blocks);
        for (int p = 0; p < 3; ++p)
            printf("K %4d  blocks/CU %d  %-11s  D=2 %7.1f us %5.2f TB/s   D=4 %7.1f us %5.2f TB/s\n", K, bpc, names[p],
                   t[p][0] * 1e3, bytes / (t[p][0] * 1e-3) / 1e12, t[p][1] * 1e3, bytes / (t[p][1] * 1e-3) / 1e12);
    }
}

int main(int argc, char** argv) {
    const long M = argc > 1 ? atol(argv[1]) : 3211264;
    const size_t maxbytes = (size_t)M * 320 * 2;
    char* x = nullptr;
    unsigned* out = nullptr;
    if (hipMalloc(&x, maxbytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(x, 1, maxbytes);
    sweep<64>(x, M, out);
    sweep<128>(x, M, out);
    sweep<256>(x, M, out);
    sweep<320>(x, M, out);
    hipFree(x);
    hipFree(out);
    return 0;
}
