// Ping-pong 256x256 implicit-GEMM conv kernel for gfx950 (MI355X): the long-K
// convs of ResNet (3x3 with C % 64 == 0, 1x1 with K >= 512) -- the reference's
// cuDNN conv fwd / dgrad (/root/reference/imagenet.py:312, fwd :123, bwd :128).
//
// Same gather-GEMM formulation, LDS row format (128-B rows, 16-B chunks XOR-
// swizzled by row & 7 on the DMA source) and staged epilogue as igemm_dma_kernel
// (conv_igemm_impl.h); what differs is the main-loop schedule, after the 256^2
// 8-phase GEMM template of cdna_hip_programming.md ("The 256^2 8-phase template"):
//
//  * 8 waves as 2 (pixel halves, wm) x 4 (64-channel quarters, wn); a wave owns
//    128 pixels x 64 channels = 8 x 4 MFMA fragments.
//  * A 64-deep K-tile is computed in 4 PHASES, one output quadrant each
//    (64 pixels x 32 channels, 16 MFMAs): (qm, qn) = (0,0), (0,1), (1,1), (1,0).
//    Fragments are read from LDS once per K-tile and held in registers across the
//    phases that reuse them.
//  * Each K-tile buffer is 4 LOAD UNITS of 128 rows (16 KiB, 2 LDS-DMA pieces per
//    wave): Xq0 / Xq1 = pixel quarter q of both halves, Ws0 / Ws1 = channel
//    eighth s of every quarter, each read in exactly one phase (Xq0 + Ws0 in phase
//    0, Ws1 in 1, Xq1 in 2). A unit's slot is therefore free two phases after its
//    read, and every phase issues one unit 4 phases ahead: unit h = 4 j + type
//    (types Xq0, Ws0, Ws1, Xq1) is issued in phase h - 6 and retired by the counted
//    s_waitcnt vmcnt(8) of phase h - 2 (4 units = 8 pieces still in flight), one
//    phase before its read (two K-tile buffers, 128 KiB).
//  * Phase = [ds_read the phase's fragments] [issue one unit] [vmcnt(8)] barrier
//    [lgkmcnt(0), s_setprio 1, 16 MFMAs, s_setprio 0] barrier.
//  * STAG: waves 4-7 (the SIMD partners of waves 0-3) run one barrier = half a
//    phase behind, so on every SIMD one wave's MFMAs run beside its partner's LDS
//    reads and DMA issue (MI355X_MICROARCH.md "Two waves per SIMD", item 9).

#pragma once

#include "conv_igemm_impl.h"

namespace {

__device__ __forceinline__ void pp_wait_vm(int n) {
#define PPW(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (((N) >> 4) << 14) | (0x7 << 4) | (0xF << 8))
    switch (n) {
        case 8: PPW(8); break;
        case 6: PPW(6); break;
        case 4: PPW(4); break;
        case 2: PPW(2); break;
        default: PPW(0); break;
    }
#undef PPW
}

template <int NI, int NJ>
__device__ __forceinline__ void pp_mfma(f32x4 (&acc)[4][8], int i0, int j0, const bf16x8 (&fw)[NI][2],
                                        const bf16x8 (&fx)[NJ][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                acc[i0 + i][j0 + j] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[i][ks], fx[j][ks], acc[i0 + i][j0 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
}

template <int N>
__device__ __forceinline__ void pp_read(bf16x8 (&f)[N][2], const bf16_t* base, int fk0, int fk1) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        f[i][0] = *reinterpret_cast<const bf16x8*>(base + i * 16 * LDK + fk0);
        f[i][1] = *reinterpret_cast<const bf16x8*>(base + i * 16 * LDK + fk1);
    }
}

// one 128-row unit = 2 DMA pieces per wave
constexpr int PP_UB = 128 * 128;
constexpr int PP_BUF = 4 * PP_UB;  // [Xq0][Xq1][Ws0][Ws1]

template <bool STAG>
__global__ __launch_bounds__(512, 1) void igemm_pp_kernel(const IGemmArgs a) {
    constexpr int BM = 256, BN = 256;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wid & 3, wm = wid >> 2;
    const int nbn = (a.Nout + BN - 1) / BN;
    const int ntiles = ((a.M + BM - 1) / BM) * nbn;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    if (lid >= ntiles) return;  // whole block (host launches exactly ntiles)
    const int m0 = (lid / nbn) * BM, n0 = (lid % nbn) * BN;
    const int nk = (a.nth * a.ntw * a.C) / BK;  // C % 64 == 0 (host)
    const int ohw = a.OH * a.OW;
    const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
    const char* zero = reinterpret_cast<const char*>(g_igemm_zero);
    const char* Xb = reinterpret_cast<const char*>(a.X);
    const char* Wb = reinterpret_cast<const char*>(a.Wk);

    // this lane's DMA rows: unit q / s, piece i -> unit row ur = (2 wid + i) * 8 + lrow
    const char* xrow[2][2];
    int ih0[2][2], iw0[2][2];
    bool mok[2][2];
    const char* wrow[2][2];
    bool nok[2][2];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int ur = (2 * wid + i) * 8 + lrow;
            const int m = m0 + (ur >> 6) * 128 + q * 64 + (ur & 63);
            mok[q][i] = m < a.M;
            const int mm = mok[q][i] ? m : 0;
            const int img = mm / ohw, rem = mm - img * ohw;
            const int oh = rem / a.OW, ow = rem - oh * a.OW;
            xrow[q][i] = Xb + (size_t)img * a.H * a.W * a.C * 2;
            ih0[q][i] = oh * a.sA;
            iw0[q][i] = ow * a.sA;
            const int n = n0 + (ur >> 5) * 64 + q * 32 + (ur & 31);
            nok[q][i] = n < a.Nout;
            wrow[q][i] = Wb + (size_t)(nok[q][i] ? n : 0) * a.ldb * 2;
        }
    // unit TYPE (0 Xq0, 1 Ws0, 2 Ws1, 3 Xq1; a compile-time constant at every call) of K-tile j
    auto issue_unit = [&](int type, int j) {
        if (j >= nk) return;
        const int kk = j * BK;
        const int t = kk / a.C;
        const int c = kk - t * a.C + lchunk * 8;
        const int ti = t / a.ntw, tj = t - ti * a.ntw;
        char* base = smem + (j & 1) * PP_BUF;
        if (type == 0 || type == 3) {
            const int q = type == 0 ? 0 : 1;
            const int dh = a.dh0 + ti * a.dhs, dw = a.dw0 + tj * a.dws;
            char* dst = base + q * PP_UB + wid * 2048;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ih = ih0[q][i] + dh, iw = iw0[q][i] + dw;
                const bool ok = mok[q][i] && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
                const char* src = ok ? xrow[q][i] + (((size_t)ih * a.W + iw) * a.C + c) * 2 : zero;
                __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                                 (void __attribute__((address_space(3)))*)(dst + i * 1024), 16, 0, 0);
            }
        } else {
            const int s = type == 1 ? 0 : 1;
            const int wtap = (a.kh0 + ti * a.khs) * a.KW + (a.kw0 + tj * a.kws);
            char* dst = base + (2 + s) * PP_UB + wid * 2048;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const char* src = nok[s][i] ? wrow[s][i] + ((size_t)wtap * a.C + c) * 2 : zero;
                __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                                 (void __attribute__((address_space(3)))*)(dst + i * 1024), 16, 0, 0);
            }
        }
    };
    // pieces still allowed in flight after phase g's issue: units up to h = g + 2 must have landed
    const int hmax = 4 * nk - 1;
    auto allowed = [&](int g) { return 2 * max(0, min(4, min(g + 6, hmax) - (g + 2))); };

    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float* st = a.stats ? a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * ((a.flags & IG_BNBWD) ? 3 : 2) * a.Nout
                        : nullptr;

    // prologue: units h = 0..5 (K-tile 0 whole, K-tile 1's Xq0 + Ws0), phase -1's wait
    issue_unit(0, 0);
    issue_unit(1, 0);
    issue_unit(2, 0);
    issue_unit(3, 0);
    issue_unit(0, 1);
    issue_unit(1, 1);
    pp_wait_vm(allowed(-1));
    __builtin_amdgcn_s_barrier();
    if (STAG && wm == 1) __builtin_amdgcn_s_barrier();

    const int fr = lane & 15;
    const int fk0 = (((lane >> 4) + 0) ^ (fr & 7)) * 8, fk1 = (((lane >> 4) + 4) ^ (fr & 7)) * 8;
    bf16x8 fx0[4][2], fx1[4][2], fw0[2][2], fw1[2][2];
    for (int kt = 0; kt < nk; ++kt) {
        const char* B = smem + (kt & 1) * PP_BUF;
        const bf16_t* X0 = reinterpret_cast<const bf16_t*>(B) + (wm * 64 + fr) * LDK;
        const bf16_t* X1 = reinterpret_cast<const bf16_t*>(B + PP_UB) + (wm * 64 + fr) * LDK;
        const bf16_t* W0 = reinterpret_cast<const bf16_t*>(B + 2 * PP_UB) + (wn * 32 + fr) * LDK;
        const bf16_t* W1 = reinterpret_cast<const bf16_t*>(B + 3 * PP_UB) + (wn * 32 + fr) * LDK;
        const int g = 4 * kt;
        // phase 0: quadrant (0, 0); issue Ws1 of K-tile kt+1
        pp_read<4>(fx0, X0, fk0, fk1);
        pp_read<2>(fw0, W0, fk0, fk1);
        issue_unit(2, kt + 1);
        pp_wait_vm(allowed(g));
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_mfma<2, 4>(acc, 0, 0, fw0, fx0);
        __builtin_amdgcn_s_barrier();
        // phase 1: quadrant (0, 1); issue Xq1 of K-tile kt+1
        pp_read<2>(fw1, W1, fk0, fk1);
        issue_unit(3, kt + 1);
        pp_wait_vm(allowed(g + 1));
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_mfma<2, 4>(acc, 2, 0, fw1, fx0);
        __builtin_amdgcn_s_barrier();
        // phase 2: quadrant (1, 1); issue Xq0 of K-tile kt+2
        pp_read<4>(fx1, X1, fk0, fk1);
        issue_unit(0, kt + 2);
        pp_wait_vm(allowed(g + 2));
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_mfma<2, 4>(acc, 2, 4, fw1, fx1);
        __builtin_amdgcn_s_barrier();
        // phase 3: quadrant (1, 0) from held fragments; issue Ws0 of K-tile kt+2
        issue_unit(1, kt + 2);
        pp_wait_vm(allowed(g + 3));
        __builtin_amdgcn_s_barrier();
        pp_mfma<2, 4>(acc, 0, 4, fw0, fx1);
        __builtin_amdgcn_s_barrier();
    }
    if (STAG && wm == 0) __builtin_amdgcn_s_barrier();  // re-align the barrier counts
    pp_wait_vm(0);
    __syncthreads();
    epilogue_lds<BM, BN, 512, 4, 8>(a, acc, smem, m0, n0, wm * 128, wn * 64, lane, tid, st);
}

template <bool STAG>
int launch_pp(const IGemmArgs& a, hipStream_t st) {
    const int ntiles = ((a.M + 255) / 256) * ((a.Nout + 255) / 256);
    const size_t lds = std::max((size_t)2 * PP_BUF, epi_lds_bytes(256, 256, 512));
    hipLaunchKernelGGL((igemm_pp_kernel<STAG>), dim3(ntiles), dim3(512), lds, st, a);
    IMK_CHECK_LAUNCH();
    return 0;
}

}  // namespace
