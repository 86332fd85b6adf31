// Implicit-GEMM conv main loop v4 for gfx950 (MI355X): one 4-wave workgroup per CU, a 256 x 256
// block tile and a 128 x 128 output tile PER WAVE (cuDNN's conv fwd / dgrad in the reference,
// /root/reference/imagenet.py:312, forward :123, backward :128).
//
// Why (profiles/gemm_ceiling_b1024.md + round-4 kernel trace of hipBLASLt on the same GEMM sizes):
// the library reaches 800-1,250 TFLOP/s on the R50 1x1 conv GEMMs with MT256x256 / MT256x160
// macro tiles on 256 threads (one wave per SIMD, 128 x 128 / 128 x 80 per wave), where v3's
// 64 x 64 (128 x 128 tile) and 64 x 128 (256 x 256 tile, 8 waves) per-wave tiles read 2x / 1.5x
// the LDS bytes per MFMA FLOP and keep two waves per SIMD contending for one matrix pipe.
//
// Structure (same gather formulation, LDS-DMA addressing through buffer descriptors and staged
// epilogue as v3, conv_igemm_v3.h):
//  * NS-deep LDS ring of RB-byte rows (RB 64: one 32-deep k-step per stage), stage s + NS - 1
//    issued while stage s computes; a stage is waited for (counted vmcnt) and published (barrier)
//    in the MIDDLE of the previous stage's MFMAs, so the fragment reads of the next k-step and
//    the DMA issue of the stage after overlap the matrix pipe instead of stopping it.
//  * fragments double-buffered in registers: 8 + 8 ds_read_b128 per k-step per wave feed
//    64 v_mfma_f32_16x16x32_bf16 (256 accumulator VGPRs); sched_group_barrier interleaves the
//    reads / DMA issues with the second half of the MFMAs.
//  * one tile per workgroup (the staged epilogue reuses the ring's LDS).

#pragma once

#include "conv_igemm_v3.h"

namespace {

template <int N>
__device__ __forceinline__ void wait_vm_lit() {
    __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (((N) >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// BM x BN block tile, WN waves along the channels (4 / WN along the pixels), NS-deep ring of RB-byte rows
// MF: MFMA shape, 16 (v_mfma_f32_16x16x32_bf16) or 32 (v_mfma_f32_32x32x16_bf16)
template <int BM, int BN, int WN, int NS, int RB, int MF>
__global__ __launch_bounds__(256, 1) void igemm_v4_kernel(const IGemmArgs a) {
    constexpr int NW = 4;
    constexpr int WM = NW / WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / MF, FN = TN / MF;  // fragments per wave along pixels / channels
    static_assert(MF == 16 || MF == 32, "MFMA shape");
    constexpr int RPP = 1024 / RB, CPR = RB / 16;
    constexpr int QA = BM / (RPP * NW), QB = BN / (RPP * NW);
    static_assert(QA >= 1 && QB >= 1 && WM * WN == NW && NS >= 3, "tile / wave split");
    constexpr int LPS = QA + QB;      // vmcnt units per stage
    constexpr int KS = RB / 2;        // k (bf16) per stage
    constexpr int NKS = RB / 64;      // 32-deep k-steps per stage
    constexpr int SAB = BM * RB, SBB = BN * RB;
    constexpr int LDKE = RB / 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sX = smem;
    char* sW = smem + NS * SAB;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wid % WN, wm = wid / WN;
    const int nbn = (a.Nout + BN - 1) / BN;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    if (lid >= ((a.M + BM - 1) / BM) * nbn) return;
    const int m0 = (lid / nbn) * BM, n0 = (lid % nbn) * BN;
    const int ntaps = a.nth * a.ntw;
    const int cps = a.C / KS;  // stages per tap (C % KS == 0, host)
    const int nk = ntaps * cps;
    const int ohw = a.OH * a.OW;
    const int lrow = lane / CPR;
    const int lchunk = (lane % CPR) ^ lds_swz<RB>(lrow);
    const __amdgpu_buffer_rsrc_t rx = v3_rsrc(a.X, (uint32_t)((size_t)a.N * a.H * a.W * a.C * 2));
    const __amdgpu_buffer_rsrc_t rw = v3_rsrc(a.Wk, (uint32_t)((size_t)a.Nout * a.ldb * 2));

    // per X piece: 32-bit byte offset of (img, ih0, iw0, lchunk) -- wraps for a border pixel's
    // out-of-image first tap; only valid taps' offsets (in range once the tap is added) are used --
    // and the valid-tap bit mask
    uint32_t xbase[QA], xmask[QA];
#pragma unroll
    for (int q = 0; q < QA; ++q) {
        const int m = m0 + (wid * QA + q) * RPP + lrow;
        const bool mok = m < a.M;
        const int mm = mok ? m : 0;
        const int img = mm / ohw, rem = mm - img * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        const int ih0 = oh * a.sA + a.dh0, iw0 = ow * a.sA + a.dw0;
        xbase[q] = (uint32_t)((((int64_t)img * a.H + ih0) * a.W + iw0) * a.C * 2 + lchunk * 16);
        uint32_t mk = 0;
        for (int ti = 0; ti < a.nth; ++ti) {
            const int ih = ih0 + ti * a.dhs;
            for (int tj = 0; tj < a.ntw; ++tj) {
                const int iw = iw0 + tj * a.dws;
                if (mok && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W) mk |= 1u << (ti * a.ntw + tj);
            }
        }
        xmask[q] = mk;
    }
    uint32_t vw[QB];
#pragma unroll
    for (int q = 0; q < QB; ++q) {
        const int n = n0 + (wid * QB + q) * RPP + lrow;
        vw[q] = n < a.Nout ? (uint32_t)(n * a.ldb * 2 + lchunk * 16) : OOB_OFF;
    }

    // issue cursor: stage is = tap it (= (iti, itj)) x channel stage ics. Straight-line (selects, no
    // branches) so the MFMA sequence around it stays one basic block; past the last stage the ring
    // keeps being fed with zero-filled stages (out-of-range offsets: no tap bit, no weight row), so
    // every wait below is the same compile-time vmcnt
    int it = 0, iti = 0, itj = 0, ics = 0, is = 0;
    auto issue_next = [&]() {
        const int buf = is % NS;
        char* dX = sX + buf * SAB + (wid * QA) * 1024;
        char* dW = sW + buf * SBB + (wid * QB) * 1024;
        const bool live = is < nk;
        const uint32_t xtap = (uint32_t)((iti * a.dhs * a.W + itj * a.dws) * a.C * 2) + (uint32_t)(ics * RB);
        const uint32_t wtap =
            (uint32_t)(((a.kh0 + iti * a.khs) * a.KW + (a.kw0 + itj * a.kws)) * a.C * 2) + (uint32_t)(ics * RB);
#pragma unroll
        for (int q = 0; q < QA; ++q) v3_dma(rx, dX + q * 1024, live && ((xmask[q] >> it) & 1) ? xbase[q] + xtap : OOB_OFF, 0);
#pragma unroll
        for (int q = 0; q < QB; ++q) v3_dma(rw, dW + q * 1024, live ? vw[q] : OOB_OFF, wtap);
        ++is;
        const bool adv = ++ics == cps;
        ics = adv ? 0 : ics;
        it += adv ? 1 : 0;
        const bool wrap = adv && itj + 1 == a.ntw;
        itj = adv ? (wrap ? 0 : itj + 1) : itj;
        iti += wrap ? 1 : 0;
    };
#pragma unroll
    for (int p = 0; p < NS - 1; ++p) issue_next();

    using accT = typename std::conditional<MF == 16, f32x4, f32x16>::type;
    accT acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = accT{};
    float* st = a.stats ? a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * ((a.flags & IG_BNBWD) ? 3 : 2) * a.Nout
                        : nullptr;

    // fragment reads: MF 16 -- lane reads row (lane & 15), 16-B chunk (lane >> 4) (+4 for the second
    // 32-deep k-step of a 128-B row); MF 32 -- row (lane & 31), chunk (lane >> 5) + 2 s for the 16-deep
    // sub-step s (+4 likewise). KF fragments per 32-deep k-step per tile row block.
    constexpr int KF = MF == 16 ? 1 : 2;
    const int fr = MF == 16 ? (lane & 15) : (lane & 31);
    const int fc = MF == 16 ? (lane >> 4) : (lane >> 5);
    int fk[2][KF];
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
        for (int u = 0; u < KF; ++u) fk[k2][u] = ((fc + 2 * u + 4 * k2) ^ lds_swz<RB>(fr)) * 8;
    const int xrow0 = (wm * TM + fr) * RB, wrow0 = (wn * TN + fr) * RB;

    // wait for stage 0 (NS - 2 stages stay in flight), publish it
    wait_vm_lit<(NS - 2) * LPS>();
    __builtin_amdgcn_s_barrier();
    bf16x8 fx[2][FM][KF], fw[2][FN][KF];
    auto read_frags = [&](int g, bf16x8 (&px)[FM][KF], bf16x8 (&pw)[FN][KF]) {
        const int buf = (g / NKS) % NS, k2 = g % NKS;
        const bf16_t* bx = reinterpret_cast<const bf16_t*>(sX + buf * SAB + xrow0);
        const bf16_t* bw = reinterpret_cast<const bf16_t*>(sW + buf * SBB + wrow0);
#pragma unroll
        for (int u = 0; u < KF; ++u) {
            const int kk = fk[k2][u];
#pragma unroll
            for (int j = 0; j < FM; ++j) px[j][u] = *reinterpret_cast<const bf16x8*>(bx + j * MF * LDKE + kk);
#pragma unroll
            for (int i = 0; i < FN; ++i) pw[i][u] = *reinterpret_cast<const bf16x8*>(bw + i * MF * LDKE + kk);
        }
    };
    auto mma = [&](int i, int j, const bf16x8& w, const bf16x8& x) {
        if constexpr (MF == 16)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, x, acc[i][j], 0, 0, 0);
        else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w, x, acc[i][j], 0, 0, 0);
    };
    read_frags(0, fx[0], fw[0]);
    // one 32-deep k-step g from register set (cx, cw); the next k-step's fragments go to (nx, nw), read
    // while this k-step's MFMAs run; the stage they come from is published at the top of the k-step.
    constexpr int NMF = FN * FM * KF;  // MFMAs per k-step
    auto kstep = [&](int g, const bf16x8 (&cx)[FM][KF], const bf16x8 (&cw)[FN][KF], bf16x8 (&nx)[FM][KF],
                     bf16x8 (&nw)[FN][KF]) {
        if ((g + 1) % NKS == 0) {
            // stage g / NKS + 1 landed for this wave, then for every wave; the stage NS - 2 beyond it goes
            // into the buffer of stage g / NKS - 1, whose fragments every wave consumed before this barrier
            wait_vm_lit<(NS - 3) * LPS>();
            __builtin_amdgcn_s_barrier();
            issue_next();
        }
        read_frags(g + 1, nx, nw);
#pragma unroll
        for (int u = 0; u < KF; ++u)
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) mma(i, j, cw[i][u], cx[j][u]);
        // interleave: per group, one DMA piece (while any), two fragment reads, NMF / NRD * 2 MFMAs
        constexpr int NRD = (FM + FN) * KF;      // fragment reads per k-step
        constexpr int NG = NRD / 2;              // groups
        constexpr int PER = NMF / NG;            // MFMAs per group
        constexpr int NDMA = (NKS == 1) ? LPS : (LPS + NKS - 1) / NKS;
#pragma unroll
        for (int p = 0; p < NG; ++p) {
            __builtin_amdgcn_sched_group_barrier(0x8, PER / 2, 0);
            if (p < NDMA) __builtin_amdgcn_sched_group_barrier(0x10, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x8, PER - PER / 2, 0);
        }
    };
    const int nsteps = nk * NKS;
    int g = 0;
    for (; g + 2 <= nsteps; g += 2) {
        kstep(g, fx[0], fw[0], fx[1], fw[1]);
        kstep(g + 1, fx[1], fw[1], fx[0], fw[0]);
    }
    if (g < nsteps) kstep(g, fx[0], fw[0], fx[1], fw[1]);
    wait_vm_lit<0>();
    __syncthreads();  // every DMA retired and every wave done reading: the ring is free
    if constexpr (MF == 16) {
        epilogue_lds<BM, BN, NW * 64, FN, FM>(a, acc, smem, m0, n0, wm * TM, wn * TN, lane, tid, st);
    } else {
        // 32x32 accumulator: lane holds pixel (lane & 31) of its tile and, for register r, channel
        // 8 (r >> 2) + 4 (lane >> 5) + (r & 3): four groups of 4 consecutive channels
        auto put = [&](char* sm, int P) {
#pragma unroll
            for (int j = 0; j < FM; ++j)
#pragma unroll
                for (int i = 0; i < FN; ++i)
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const int row = wm * TM + j * 32 + (lane & 31);
                        const int col = wn * TN + i * 32 + 8 * b + 4 * (lane >> 5);
                        const f32x16& v = acc[i][j];
                        *reinterpret_cast<u32x2*>(sm + row * P + col * 2) =
                            u32x2{pack_bf2(v[4 * b], v[4 * b + 1]), pack_bf2(v[4 * b + 2], v[4 * b + 3])};
                    }
        };
        epilogue_lds_put<BM, BN, NW * 64>(a, put, smem, m0, n0, tid, st);
    }
}

template <int BM, int BN, int WN, int NS, int RB, int MF>
int launch_v4(const IGemmArgs& a, hipStream_t st) {
    const int ntiles = ((a.M + BM - 1) / BM) * ((a.Nout + BN - 1) / BN);
    const size_t lds = std::max((size_t)NS * (BM + BN) * RB, epi_lds_bytes(BM, BN, 256));
    hipLaunchKernelGGL((igemm_v4_kernel<BM, BN, WN, NS, RB, MF>), dim3(ntiles), dim3(256), lds, st, a);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

// v4 shapes: v3's (C % 64 == 0, one tap per stage, staged epilogue)
inline bool v4_ok(const IGemmArgs& a) { return v3_ok(a); }

}  // namespace
