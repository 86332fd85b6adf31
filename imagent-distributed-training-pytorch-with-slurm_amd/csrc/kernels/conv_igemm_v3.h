// Implicit-GEMM conv main loop v3 for gfx950 (MI355X): the long-K convs with C % 64 == 0
// (every 3x3 and the K >= 256 1x1 convs of ResNet; cuDNN's conv fwd / dgrad in the reference,
// /root/reference/imagenet.py:312, forward :123, backward :128).
//
// Same gather-GEMM formulation, LDS ring (128-B rows, XOR-swizzled 16-B chunks, LDS-DMA fills)
// and staged epilogue as igemm_dma_kernel (conv_igemm_impl.h). What changed is the cost of a
// stage, measured by the main-loop decomposition of round 3 (scripts/dbg_mainloop.sh: the
// 128x128 ring on 256@14 3x3 took 335 us, of which the loop skeleton alone -- barriers,
// per-stage gather bookkeeping, epilogue -- was 102 us, the DMA path 165 us and the MFMA
// path 118 us, nearly additive):
//
//  * DMA addressing through BUFFER descriptors (buffer_load_dwordx4 ... lds): one 32-bit
//    per-lane offset per 8-row piece, recomputed only when the filter TAP changes (3 VALU),
//    the within-tap channel advance in the wave-uniform soffset (SALU), and out-of-image
//    taps / rows beyond M or Nout as an out-of-range offset that the buffer unit returns as
//    zeros (no zero line, no per-stage 64-bit address arithmetic, no per-stage division:
//    the tap index is tracked incrementally).
//  * Fragment reads software-pipelined: a stage's MFMAs run in half-k-step groups
//    (FN/2 x FM MFMAs) and each group's LDS reads are issued one group ahead, so the MFMA
//    chain no longer stops on s_waitcnt lgkmcnt(0) after every 8 MFMAs
//    (sched_group_barrier pins the DS-read / MFMA interleave).
//
// Out-of-range semantics relied on (raw buffer, stride 0): a lane whose offset is
// >= num_records reads zeros. Offsets of invalid lanes are OOB_OFF = 2^31 and tensors
// are < 2^31 bytes (host check), so the lane is out of range whether or not the
// hardware adds soffset into the check.

#pragma once

#include "conv_igemm_impl.h"

namespace {

constexpr uint32_t OOB_OFF = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t v3_rsrc(const void* p, uint32_t bytes) {
    // built from kernel arguments only (wave-uniform, cdna_hip_programming.md T20)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void v3_dma(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// RB: LDS row bytes per stage (128: BK 64; 64: BK 32). NS: ring depth.
// EB: operand element bytes. 2: bf16 (v_mfma_f32_16x16x32_bf16, two k-steps per 128-B stage); 1: fp8
// (IG_FP8, conv_igemm_fp8.hip): the same rows hold 128 k, ONE block-scaled v_mfma_scale_f32_16x16x128_f8f6f4
// per fragment pair and stage -- twice the bf16 MFMA cycles for four times the k, so the same LDS bytes and
// MFMA time per stage over half the stages. Each lane feeds 32 consecutive k of its row (logical chunks
// 2g, 2g + 1, g = lane >> 4) for BOTH operands; the per-tensor power-of-two scales ride in the
// instruction's E8M0 operands. FB: format of the gathered operand (0 e4m3, 1 e5m2 = dgrad's gradient).
// EB 4: fp32 operands (the fp32 training path's 3 x bf16 split, f32.hip): 128-B rows of 32 fp32 k, each lane
// reads its 8 k (32 B, chunks 2g, 2g + 1 as fp8) and splits them into bf16 hi + lo in registers; x w =
// hi hi + hi lo + lo hi on three v_mfma_f32_16x16x32_bf16 (fp32 accumulate, ~2^-16 relative per product);
// direct fp32 epilogue (+ bias, + accumulate).
// TI: K order of a multi-tap conv. false (default): filter tap outer, channel slice inner (consecutive stages read
// consecutive 128-B chunks of the same pixel rows). true (A/B, explicit tiles 27 / 28): channel slice outer, tap
// inner -- the 9 taps of a 3x3 re-read nearly the same rows of one 128-B channel column in 9 consecutive stages,
// a smaller L2 working set per tile; measured SLOWER in the R50 step (v3 128x128 14.6 -> 17.3 ms/step, 256x256
// 6.9 -> 8.0, round 5): the tap order's row locality is worth more than the smaller window.
template <int BM, int BN, int WN, int NS, int NW, int RB, int EB = 2, int FB = 0, bool TI = false>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void igemm_v3_kernel(const IGemmArgs a) {
    constexpr int WM = NW / WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    constexpr int RPP = 1024 / RB, CPR = RB / 16;
    constexpr int QA = BM / (RPP * NW), QB = BN / (RPP * NW);
    static_assert(QA >= 1 && QB >= 1 && WM * WN == NW && FN % 2 == 0, "tile / wave split");
    static_assert(EB == 2 || RB == 128, "fp8 / fp32: 128-B rows (one MFMA k-step per stage)");
    constexpr int LPS = QA + QB;
    constexpr int KS = RB / EB;       // k per stage
    constexpr int NKS = RB / 64;      // MFMA k-steps (32) per stage
    constexpr int SAB = BM * RB, SBB = BN * RB;
    constexpr int FH = FN / 2;        // channel fragments per half group
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
    const int cps = a.C / KS;          // stages per tap (C % 64 == 0, host)
    const int nk1 = ntaps * cps;       // stages of the first K segment
    const int nk = nk1 + (a.X2 ? a.C2 / KS : 0);  // + the second (X2: one tap, C2 % 64 == 0, host)
    const int ohw = a.OH * a.OW;
    const int lrow = lane / CPR;
    const int lchunk = (lane % CPR) ^ lds_swz<RB>(lrow);
    // descriptors based at the tile's first image (X) / first pixel row (X2): a tile's rows span a few images at
    // most, so the 32-bit buffer offsets hold for any tensor size (batch 2048 puts 3.3 GB in one layer-1 tensor)
    const int img0 = m0 / ohw;
    const size_t xo0 = (size_t)img0 * a.H * a.W * a.C * EB, xall = (size_t)a.N * a.H * a.W * a.C * EB;
    const __amdgpu_buffer_rsrc_t rx =
        v3_rsrc(reinterpret_cast<const char*>(a.X) + xo0, (uint32_t)min(xall - xo0, (size_t)0x7FFFFFFF));
    const __amdgpu_buffer_rsrc_t rw = v3_rsrc(a.Wk, (uint32_t)((size_t)a.Nout * a.ldb * EB));
    const size_t x2o0 = (size_t)m0 * a.C2 * 2;
    const __amdgpu_buffer_rsrc_t rx2 =
        v3_rsrc(a.X2 ? reinterpret_cast<const char*>(a.X2) + x2o0 : reinterpret_cast<const char*>(a.X),
                a.X2 ? (uint32_t)min((size_t)a.M * a.C2 * 2 - x2o0, (size_t)0x7FFFFFFF) : 0u);

    // per X piece: byte offset of (img, ih0, iw0, lchunk) -- may be "negative" (a border pixel's
    // first tap), only valid taps' offsets are ever used -- and the valid-tap bit mask
    int64_t xbase[QA];
    uint32_t xmask[QA];
#pragma unroll
    for (int q = 0; q < QA; ++q) {
        const int m = m0 + (wid * QA + q) * RPP + lrow;
        const bool mok = m < a.M;
        const int mm = mok ? m : 0;
        const int img = mm / ohw, rem = mm - img * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        const int ih0 = oh * a.sA + a.dh0, iw0 = ow * a.sA + a.dw0;
        xbase[q] = (((int64_t)(img - img0) * a.H + ih0) * a.W + iw0) * a.C * EB + lchunk * 16;
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
    uint32_t xbase2[QA];  // second K segment: pixel row m of X2 (pitch C2), out-of-range rows read zeros
#pragma unroll
    for (int q = 0; q < QA; ++q) {
        const int m = m0 + (wid * QA + q) * RPP + lrow;
        xbase2[q] = m < a.M ? (uint32_t)((size_t)(m - m0) * a.C2 * 2 + lchunk * 16) : OOB_OFF;
    }
    uint32_t vw[QB];
#pragma unroll
    for (int q = 0; q < QB; ++q) {
        const int n = n0 + (wid * QB + q) * RPP + lrow;
        vw[q] = n < a.Nout ? (uint32_t)(n * a.ldb * EB + lchunk * 16) : OOB_OFF;
    }

    // issue cursor: tap (ti, tj) = t, channel stage cs within the tap
    int it = 0, iti = 0, itj = 0, ics = 0, is = 0;
    uint32_t vx[QA];
    int xtap = 0, wtap = 0;  // uniform: byte offset of the tap in X, weight column of the tap
    auto set_tap = [&]() {
        const int dh = iti * a.dhs, dw = itj * a.dws;
        xtap = (dh * a.W + dw) * a.C * EB;
        wtap = ((a.kh0 + iti * a.khs) * a.KW + (a.kw0 + itj * a.kws)) * a.C * EB;
#pragma unroll
        for (int q = 0; q < QA; ++q)
            vx[q] = (xmask[q] >> it) & 1 ? (uint32_t)(xbase[q] + xtap) : OOB_OFF;
    };
    auto issue_next = [&]() {
        if (is >= nk) return;
        const int buf = is % NS;
        char* dX = sX + buf * SAB + (wid * QA) * 1024;
        char* dW = sW + buf * SBB + (wid * QB) * 1024;
        if (is >= nk1) {  // second K segment (one tap): X2 rows, weight columns C + (is - nk1) * KS
            const uint32_t so = (uint32_t)((is - nk1) * RB);
#pragma unroll
            for (int q = 0; q < QA; ++q) v3_dma(rx2, dX + q * 1024, xbase2[q], so);
#pragma unroll
            for (int q = 0; q < QB; ++q) v3_dma(rw, dW + q * 1024, vw[q], (uint32_t)(a.C * 2) + so);
            ++is;
            return;
        }
        const uint32_t cso = (uint32_t)(ics * RB);
#pragma unroll
        for (int q = 0; q < QA; ++q) v3_dma(rx, dX + q * 1024, vx[q], cso);
#pragma unroll
        for (int q = 0; q < QB; ++q) v3_dma(rw, dW + q * 1024, vw[q], (uint32_t)wtap + cso);
        ++is;
        if (TI && ntaps > 1) {  // next tap; after the last one, the next channel slice from tap 0
            if (++it == ntaps) {
                it = iti = itj = 0;
                ++ics;
            } else if (++itj == a.ntw) {
                itj = 0;
                ++iti;
            }
            if (ics < cps) set_tap();
        } else if (++ics == cps) {
            ics = 0;
            ++it;
            if (++itj == a.ntw) {
                itj = 0;
                ++iti;
            }
            if (it < ntaps) set_tap();
        }
    };
    set_tap();
#pragma unroll
    for (int p = 0; p < NS - 1; ++p) issue_next();
    // the fused BN backward's x / mask-bit chunks (128x128 bf16 tiles: the short-K dgrads): issued after the
    // prologue stages, landing under the main loop (the first stage wait covers them)
    constexpr bool PFE = EB == 2 && BM == 128 && BN == 128 && NW == 4;
    EpiPF<BM, BN, NW * 64> pf;
    if constexpr (PFE) epi_prefetch<BM, BN, NW * 64>(a, pf, m0, n0, tid);

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float* st = a.stats ? a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * ((a.flags & IG_BNBWD) ? 3 : 2) * a.Nout
                        : nullptr;

    const int fr = lane & 15;
    constexpr int LDKE = RB / 2;
    int fk[2];
    fk[0] = (((lane >> 4) + 0) ^ lds_swz<RB>(fr)) * 8;
    fk[1] = (((lane >> 4) + 4) ^ lds_swz<RB>(fr)) * 8;
    // fp8: the lane's 32 bytes are logical chunks 2g, 2g + 1 of its row (byte offsets); E8M0 scales
    const int f8c0 = ((2 * (lane >> 4)) ^ lds_swz<RB>(fr)) * 16, f8c1 = ((2 * (lane >> 4) + 1) ^ lds_swz<RB>(fr)) * 16;
    const int sx8 = EB == 1 ? 127 + a.xexp[0] : 127, sw8 = EB == 1 ? 127 + a.wexp[0] : 127;
    for (int s = 0; s < nk; ++s) {
        if (is - 1 - s >= NS - 2)
            __builtin_amdgcn_s_waitcnt((((NS - 2) * LPS) & 0xF) | ((((NS - 2) * LPS) >> 4) << 14) | (0x7 << 4) |
                                       (0xF << 8));
        else
            __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
        __builtin_amdgcn_s_barrier();
        issue_next();
        const int buf = s % NS;
        if constexpr (EB == 1) {
            // one 128-deep k-step: pixel fragments + channel half 0 first, half 1 read under half 0's MFMAs
            const char* cx = sX + buf * SAB + (wm * TM + fr) * RB;
            const char* cw = sW + buf * SBB + (wn * TN + fr) * RB;
            auto rd8 = [&](const char* p) {
                const u32x4 lo = *reinterpret_cast<const u32x4*>(p + f8c0);
                const u32x4 hi = *reinterpret_cast<const u32x4*>(p + f8c1);
                return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
            };
            i32x8 gx[FM], gw[FN];
#pragma unroll
            for (int j = 0; j < FM; ++j) gx[j] = rd8(cx + j * 16 * RB);
#pragma unroll
            for (int i = 0; i < FH; ++i) gw[i] = rd8(cw + i * 16 * RB);
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * (FM + FH), 0);
#pragma unroll
            for (int i = FH; i < FN; ++i) gw[i] = rd8(cw + i * 16 * RB);
            __builtin_amdgcn_sched_group_barrier(0x100, 2 * FH, 0);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(gw[i], gx[j], acc[i][j], 0, FB, 0, sw8,
                                                                                  0, sx8);
            __builtin_amdgcn_sched_group_barrier(0x8, FN * FM, 0);
            __builtin_amdgcn_s_setprio(0);
            continue;
        }
        if constexpr (EB == 4) {
            // one 32-deep k-step: 8 fp32 k per lane -> bf16 hi / lo fragments
            const char* cx = sX + buf * SAB + (wm * TM + fr) * RB;
            const char* cw = sW + buf * SBB + (wn * TN + fr) * RB;
            auto rds = [&](const char* p, bf16x8& hi, bf16x8& lo) {
                const f32x4 v0 = *reinterpret_cast<const f32x4*>(p + f8c0);
                const f32x4 v1 = *reinterpret_cast<const f32x4*>(p + f8c1);
                const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
                u32x4 h, l;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    h[k] = pack_bf2(v[2 * k], v[2 * k + 1]);
                    l[k] = pack_bf2(v[2 * k] - lo_bf(h[k]), v[2 * k + 1] - hi_bf(h[k]));
                }
                hi = __builtin_bit_cast(bf16x8, h);
                lo = __builtin_bit_cast(bf16x8, l);
            };
            bf16x8 xh[FM], xl[FM], wh[FN], wl[FN];
#pragma unroll
            for (int j = 0; j < FM; ++j) rds(cx + j * 16 * RB, xh[j], xl[j]);
#pragma unroll
            for (int i = 0; i < FN; ++i) rds(cw + i * 16 * RB, wh[i], wl[i]);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[i], xh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[i], xl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[i], xh[j], acc[i][j], 0, 0, 0);
                }
            __builtin_amdgcn_s_setprio(0);
            continue;
        }
        const bf16_t* bx = reinterpret_cast<const bf16_t*>(sX + buf * SAB + (wm * TM + fr) * RB);
        const bf16_t* bw = reinterpret_cast<const bf16_t*>(sW + buf * SBB + (wn * TN + fr) * RB);
        // groups g = (ks, h): h = 0 reads the k-step's pixel fragments + channel half 0, h = 1
        // channel half 1; each group's reads are issued before the previous group's MFMAs
        bf16x8 fx[2][FM], fw[2][FH];
#pragma unroll
        for (int j = 0; j < FM; ++j) fx[0][j] = *reinterpret_cast<const bf16x8*>(bx + j * 16 * LDKE + fk[0]);
#pragma unroll
        for (int i = 0; i < FH; ++i) fw[0][i] = *reinterpret_cast<const bf16x8*>(bw + i * 16 * LDKE + fk[0]);
        __builtin_amdgcn_sched_group_barrier(0x100, FM + FH, 0);  // group 0's reads first
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int g = 0; g < 2 * NKS; ++g) {
            const int ks = g >> 1, h = g & 1;
            const int xs = ks & 1, ws = g & 1;  // register sets of this group
            if (g + 1 < 2 * NKS) {  // prefetch group g + 1
                const int ks1 = (g + 1) >> 1, h1 = (g + 1) & 1;
                if (h1 == 0) {
#pragma unroll
                    for (int j = 0; j < FM; ++j)
                        fx[ks1 & 1][j] = *reinterpret_cast<const bf16x8*>(bx + j * 16 * LDKE + fk[ks1]);
                }
#pragma unroll
                for (int i = 0; i < FH; ++i)
                    fw[ws ^ 1][i] =
                        *reinterpret_cast<const bf16x8*>(bw + (h1 * FH + i) * 16 * LDKE + fk[ks1]);
                if (h1 == 0)
                    __builtin_amdgcn_sched_group_barrier(0x100, FM + FH, 0);  // DS reads
                else
                    __builtin_amdgcn_sched_group_barrier(0x100, FH, 0);
            }
#pragma unroll
            for (int i = 0; i < FH; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j)
                    acc[h * FH + i][j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[ws][i], fx[xs][j], acc[h * FH + i][j], 0, 0, 0);
            __builtin_amdgcn_sched_group_barrier(0x8, FH * FM, 0);  // MFMAs
        }
        __builtin_amdgcn_s_setprio(0);
    }
    if constexpr (EB == 4) {  // fp32 out: lane holds channels nb + i*16 + 4g + r of pixel mb + j*16 + fr
        const int g = lane >> 4;
        const bool accum = a.flags & IG_ACCUM;
        if (a.flags & IG_BNBWD) {
            // dgrad into a ReLU'd BatchNorm (fp32, bnx = its input x, bnsave = (mean, rstd)): the stored value is
            // g' = g * (bn(x) > 0) -- bn(x) computed as the apply kernel computes it -- and the 2-row slab slot
            // receives sum(g'), sum(g' xhat) (the fp32 backward fold's layout, f32.hip bn_fold_bwd_f32_kernel)
            const float* X = reinterpret_cast<const float*>(a.bnx);
            float* Y = reinterpret_cast<float*>(a.Y);
            float* sb = a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * 2 * a.Nout;
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int n = n0 + wn * TN + i * 16 + 4 * g;
                const bool nok = n < a.Nout;  // Nout % 4 == 0 (host)
                float mu[4], rs[4], sc[4], sh[4], s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    mu[r] = nok ? a.bnsave[n + r] : 0.f;
                    rs[r] = nok ? a.bnsave[a.Nout + n + r] : 0.f;
                    sc[r] = nok ? rs[r] * a.bngamma[n + r] : 0.f;
                    sh[r] = nok ? a.bnbeta[n + r] : 0.f;
                }
#pragma unroll
                for (int j = 0; j < FM; ++j) {
                    const int m = m0 + wm * TM + j * 16 + fr;
                    if (m >= a.M || !nok) continue;
                    const int img = m / ohw, rem = m - img * ohw;
                    const int oh = rem / a.OW, ow = rem - oh * a.OW;
                    const size_t e =
                        (((size_t)img * a.YH + oh * a.sY + a.oy) * a.YW + ow * a.sY + a.ox) * a.ldy + n;
                    const f32x4 xv = *reinterpret_cast<const f32x4*>(X + e);
                    f32x4 v = acc[i][j];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float o = (xv[r] - mu[r]) * sc[r] + sh[r];
                        if (!(o > 0.f)) v[r] = 0.f;
                        s1[r] += v[r];
                        s2[r] += v[r] * ((xv[r] - mu[r]) * rs[r]);
                    }
                    *reinterpret_cast<f32x4*>(Y + e) = v;
                }
                stat_pair_atomic(s1, s2, sb, sb + a.Nout, n, a.Nout, lane);  // every lane (DPP)
            }
            return;
        }
        if (!accum) {  // (+ bias) (+ the BatchNorm statistics as shifted sums into the slab, DPP-reduced)
            epilogue_tile<FN, FM>(a, acc, n0 + wn * TN + 4 * g, m0 + wm * TM + fr, lane, st);
            return;
        }
        float* Y = reinterpret_cast<float*>(a.Y);
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int m = m0 + wm * TM + j * 16 + fr;
            if (m >= a.M) continue;
            const int img = m / ohw, rem = m - img * ohw;
            const int oh = rem / a.OW, ow = rem - oh * a.OW;
            float* yp = Y + (((size_t)img * a.YH + oh * a.sY + a.oy) * a.YW + ow * a.sY + a.ox) * a.ldy;
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int n = n0 + wn * TN + i * 16 + 4 * g;
                if (n >= a.Nout) continue;  // Nout % 4 == 0 (host)
                f32x4 v = acc[i][j];
                if (a.bias) v += *reinterpret_cast<const f32x4*>(a.bias + n);
                f32x4* p = reinterpret_cast<f32x4*>(yp + n);
                if (accum) v += *p;
                *p = v;
            }
        }
        return;
    }
    __syncthreads();  // every DMA retired (last wait) and every wave done reading: the ring is free
    epilogue_lds<BM, BN, NW * 64, FN, FM>(a, acc, smem, m0, n0, wm * TM, wn * TN, lane, tid, st,
                                          PFE ? &pf : nullptr);
}

template <int BM, int BN, int WN, int NS, int NW, int RB, int EB = 2, int FB = 0, bool TI = false>
int launch_v3(const IGemmArgs& a, hipStream_t st) {
    const int ntiles = ((a.M + BM - 1) / BM) * ((a.Nout + BN - 1) / BN);
    const size_t lds = EB == 4 ? (size_t)NS * (BM + BN) * RB
                               : std::max((size_t)NS * (BM + BN) * RB, epi_lds_bytes(BM, BN, NW * 64));
    hipLaunchKernelGGL((igemm_v3_kernel<BM, BN, WN, NS, NW, RB, EB, FB, TI>), dim3(ntiles), dim3(NW * 64), lds, st, a);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

// shapes v3 covers: C % 64 == 0 (one tap per stage), taps <= 32, operands < 2^31 bytes, and the staged
// bf16 epilogue (no bias; ReLU only with the eval forward's folded BatchNorm, IG_AFFINE, without statistics)
inline bool v3_ok(const IGemmArgs& a) {
    if (a.C % 64 || a.nth * a.ntw > 32 || a.nth < 1 || a.ntw < 1) return false;
    if (a.flags & (IG_OUT_F32 | IG_STEM | IG_FP8)) return false;
    const bool eval_bn = a.flags & IG_AFFINE;
    if ((a.flags & IG_RELU) && !eval_bn) return false;
    if (eval_bn && (a.stats || (a.flags & IG_BNBWD))) return false;
    const bool bnb_bias = (a.flags & IG_BNBWD) && a.X2;  // the second segment's bias (bn_gram.hip)
    if ((a.bias && !eval_bn && !bnb_bias) || a.xbn || a.Nout % 8 || a.ldy % 8) return false;
    if (a.X2 && (a.C2 % 64 || a.C2 <= 0 || a.nth != 1 || a.ntw != 1 || a.sA != 1 || a.H != a.OH || a.W != a.OW ||
                 a.ldb < a.C + a.C2))
        return false;
    // (X / X2 descriptors are tile-based: any size; one image must stay below 2^31 bytes, the weights too)
    const size_t ib = (size_t)a.H * a.W * a.C * 2 * 4, wb = (size_t)a.Nout * a.ldb * 2;
    return ib < (1ull << 31) && wb < (1ull << 31);
}

// fp32 (3 x bf16 split, EB = 4) shapes v3 covers: C % 32 == 0 (one tap per 32-deep stage), fp32 out with
// optional bias / accumulate, Nout and ldy % 4 == 0 (16-B stores)
inline bool v3_ok32(const IGemmArgs& a) {
    if (a.C % 32 || a.nth * a.ntw > 32 || a.nth < 1 || a.ntw < 1) return false;
    if ((a.flags & ~(IG_ACCUM | IG_OUT_F32 | IG_BNBWD)) || !(a.flags & IG_OUT_F32)) return false;
    if ((a.stats && (a.flags & IG_ACCUM)) || a.xbn || a.X2 || a.Nout % 4 || a.ldy % 4) return false;
    if ((a.flags & IG_BNBWD) && (!a.stats || !a.bnx || !a.bnsave || !a.bngamma || !a.bnbeta || a.bias ||
                                 (a.flags & IG_ACCUM)))
        return false;
    const size_t xb = (size_t)a.N * a.H * a.W * a.C * 4, wb = (size_t)a.Nout * a.ldb * 4;
    return xb < (1ull << 31) && wb < (1ull << 31);
}

// fp8 shapes v3 covers (EB = 1): C % 128 == 0 (one tap per 128-deep stage), the staged bf16 epilogue
// (statistics, fused BN backward, accumulate), no second K segment, scales present
inline bool v3_ok8(const IGemmArgs& a) {
    if (!(a.flags & IG_FP8) || a.C % 128 || a.nth * a.ntw > 32 || a.nth < 1 || a.ntw < 1) return false;
    if (a.flags & (IG_OUT_F32 | IG_STEM | IG_RELU | IG_AFFINE | IG_EPI_DIRECT)) return false;
    if (a.bias || a.xbn || a.X2 || !a.xexp || !a.wexp || a.Nout % 8 || a.ldy % 8) return false;
    const size_t xb = (size_t)a.N * a.H * a.W * a.C, wb = (size_t)a.Nout * a.ldb;
    return xb < (1ull << 31) && wb < (1ull << 31);
}

}  // namespace
