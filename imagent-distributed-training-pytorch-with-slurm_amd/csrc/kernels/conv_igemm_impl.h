// MFMA implicit-GEMM convolution, NHWC bf16, for gfx950 (MI355X).
//
// Replaces cuDNN's conv fwd / dgrad kernels that the reference reaches via
// torchvision resnet18 (/root/reference/imagenet.py:312, forward :123,
// backward :128).
//
// ONE "gather GEMM" formulation serves the forward conv, the stride-1 dgrad,
// each parity class of a strided dgrad (sub-pixel decomposition, no wasted
// MACs), the 7x7 stem and the FC layer (a 1x1 conv on a 1x1 image):
//
//   out[pix(m)][n] = sum_{t < ntaps, c < C} X[gather(m, t)][c] * Wk[n][wtap(t)*C + c]
//
//   m      = (img, oh, ow) over the "row grid" OH x OW
//   gather = (img, oh*sA + dh(t), ow*sA + dw(t))   (zero outside the image)
//   pix    = (img, oh*sY + oy, ow*sY + ox)         (output pixel)
//   taps   = a rectangle: t = (i, j), dh = dh0 + i*dhs, dw = dw0 + j*dws,
//            weight tap = (kh0 + i*khs) * KW + (kw0 + j*kws)
//
//  * fwd:          sA = stride, dh0 = -pad, dhs = 1, taps = all KHxKW, Wk = W[Co][KH][KW][Ci]
//  * dgrad (s=1):  X = dY, dh0 = pad, dhs = -1, Wk = W^T[Ci][KH][KW][Co]
//  * dgrad (s>1):  one launch per output parity (ph, pw); only the taps with
//                  kh == (ph + pad) mod s contribute, output pixel s*oh + ph.
//  * stem:         C == 4, the KW taps x 4 channels of a kernel row are one
//                  contiguous NHWC segment -> K = KH x 32 (28 real + 4 zero).
//
// Two main-loop structures share one epilogue:
//
//  igemm_dma_kernel (every conv except the stem): operands go global -> LDS
//    by LDS-DMA (global_load_lds_dwordx4, one 1-KiB piece = 8 tile rows per
//    wave instruction, per-lane gather addresses, out-of-image taps read a
//    zero line) into an NS-deep ring of 128-B-row tiles. Stage s+NS-1 is in
//    flight while stage s computes; a counted s_waitcnt vmcnt + raw s_barrier
//    retire one stage per iteration (cdna_hip_programming.md §5 "Pipelining
//    across barriers"). No VGPRs, no ds_write for staging.
//  igemm_rs_kernel (stem): register staging with 8-byte half-predicated loads.
//
// Both are PERSISTENT when tiles have few K-stages: a block walks its tiles
// and their K-stages as ONE flattened stage sequence, so the next tile's loads
// overlap this tile's epilogue (memory-bound 1x1 convs).
// LDS tiles: 128-B rows (BK = 64 bf16) with 16-B chunks XOR-swizzled by
// (row & 7) -> conflict-free ds_read_b128 fragment reads (swizzle applied on
// the DMA SOURCE address, the LDS image stays lane-linear).
// MFMA v_mfma_f32_16x16x32_bf16 with the WEIGHTS as the A operand and the
// pixels as the B operand: each lane's accumulator holds 4 consecutive output
// CHANNELS of one pixel -> 8-byte NHWC stores with no LDS pass; BN statistics
// (sum, sum of squares) reduce over the 16 lanes of a row group and go to a
// 32-slot fp32 slab. Tiles are XCD-remapped so concurrently running channel
// tiles of one pixel panel share an XCD's L2.

#pragma once

#include <algorithm>
#include <cstdlib>

#include "common.h"

struct IGemmArgs {
    const bf16_t* X;   // gathered operand, NHWC [N][H][W][C]
    const bf16_t* Wk;  // [Nout][ldb] bf16
    void* Y;           // output NHWC, channel stride ldy
    const float* bias; // [Nout] or null
    float* stats;      // [STAT_SLOTS][2][Nout] (sum, sumsq) slab or null, fp32 atomics
    int N, H, W, C;
    int OH, OW, M;     // row grid, M = N*OH*OW
    int Nout, ldb;
    int sA;
    int nth, ntw, dh0, dhs, dw0, dws, kh0, khs, kw0, kws, KW;
    int YH, YW, sY, oy, ox, ldy;
    int flags;         // IG_* bits
    // IG_BNBWD: the BatchNorm this gradient flows into (all NHWC at the output
    // pixels, channel stride ldy == Nout)
    const bf16_t* bnx;     // BN input x
    // ReLU mask of the BN(+add)+ReLU output as bits (bn.hip bn_fwd ym: byte e/8 of element e, bit
    // e%8 = output > 0; 1/16 of the bytes of re-reading the bf16 output), or null: mask from x
    const uint8_t* bnym;
    const float* bnsave;   // [2][Nout] mean, rstd
    const float* bngamma;  // used with the from-x mask
    const float* bnbeta;
    const bf16_t* bnx2;    // second BN branch input (downsample), or null
    const float* bnsave2;
    // IG_FP8: X and Wk hold e4m3 values x*2^-ex, w*2^-ew; the per-tensor
    // exponents live on the device (delayed scaling, no host sync) and enter
    // the MFMA as E8M0 scales 127 + e
    const int* xexp;
    const int* wexp;
    // forward statistics are SHIFTED sums: sum(v - shift[n]), sum((v - shift[n])^2)
    // with shift = the BN's previous batch mean (null: 0). With shift ~ mean the
    // variance E[(v-s)^2] - E[v-s]^2 has no catastrophic cancellation even when
    // |mean| >> std (imk_bn_stats_finalize turns the slab into mean / variance).
    const float* shift;
    // conv_stream only: the gathered operand is relu(X * xbn[c] + xbn[C + c]) per input channel c --
    // the producing BatchNorm's apply + ReLU done on the consumer's operand load (ops/block.py),
    // so the BN output is never written
    const float* xbn;
    // v3 only: a second K segment -- after the C channels of X, C2 more from X2 (same pixels, row pitch C2;
    // 1x1 stride-1 gathers), the weights' columns [C, C + C2). With IG_BNBWD, `bias` [Nout] is added to
    // the sums before the mask (bn_gram.hip: the bottleneck's bn3 backward folded into conv3's dgrad)
    const bf16_t* X2;
    int C2;
    // IG_Q8OUT (streaming 1x1 only): also the e4m3 copy of the stored bf16 output for fp8 consumers, quantised
    // with 2^-y8exp[0] (delayed scaling, fp8.hip), |y| max into y8amax[blockIdx & 31] (as bn_fwd's y8)
    void* Y8;
    const int* y8exp;
    float* y8amax;
};

#define IG_OUT_F32 1   // fp32 output (else bf16)
#define IG_RELU 2      // ReLU on the output
#define IG_STEM 4      // stem row-segment gather
#define IG_ACCUM 8     // out += result (bf16 out only): fused gradient accumulation
#define IG_REGSTAGE 16 // force the register-staged main loop (A/B testing)
#define IG_BNBWD 32    // epilogue = ReLU mask + BatchNorm-backward reductions (slab [32][3][Nout])
#define IG_EPI_LDS 64  // LDS-staged coalesced epilogue (default for IG_BNBWD)
#define IG_EPI_DIRECT 128  // direct register epilogue even for IG_BNBWD (A/B testing)
#define IG_FP8 256     // fp8 operands on the block-scaled MFMA (conv_igemm_fp8.hip)
#define IG_BF8X 512    // with IG_FP8: the gathered operand X is e5m2 (gradients), Wk e4m3
#define IG_AFFINE 1024 // inference BN folded into the epilogue: out = acc * bias[n] + bias[Nout + n]
#define IG_NOSTREAM 2048  // never the streaming short-K 1x1 kernel (conv_stream.hip; A/B testing)
#define IG_ACCUM_SUB2 4096  // with IG_ACCUM: the old output is valid only at even (y, x) output pixels
                           // (a stride-2 1x1 dgrad wrote only that parity class, no memset); elsewhere 0
#define IG_RES 8192   // (streaming 1x1 only) out = act(affine(acc) + bnx[e]): a residual read from bnx, not from Y
#define IG_Q8OUT 32768  // (streaming 1x1 only) also the e4m3 copy of the output (Y8 / y8exp / y8amax)
#define IG_MASKOUT 16384  // (streaming 1x1 only, with IG_RELU) also write the ReLU mask of the stored output as bits
                          // into bnym (byte e / 8, bit e % 8; bn.hip bn_fwd's `ym` format)
#define STAT_SLOTS 32  // stats slab: [STAT_SLOTS][2][Nout]

static __device__ __attribute__((aligned(64))) uint32_t g_igemm_zero[16];  // zero line for masked DMA lanes (per TU)

namespace {

constexpr int BK = 64;   // K elements per stage = one 128-B LDS row
constexpr int LDK = BK;

__device__ __forceinline__ void waitcnt_vm(int n) {
    // s_waitcnt vmcnt(n) only (expcnt/lgkmcnt left at their maxima); n is a
    // small compile-time-like value chosen by an unrolled switch at the call site
#define WV(N) __builtin_amdgcn_s_waitcnt(((N) & 0xF) | (((N) >> 4) << 14) | (0x7 << 4) | (0xF << 8))
    switch (n) {
        case 0: WV(0); break;
        case 4: WV(4); break;
        case 6: WV(6); break;
        case 8: WV(8); break;
        case 12: WV(12); break;
        case 16: WV(16); break;
        default: WV(0); break;
    }
#undef WV
}

// ------------------------------------------------------------------ epilogue
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// Per-channel partial sums of a fragment -> the stats slab.
// Every tile adds into the same few Nout-long rows: contention, not bytes,
// bounds this (MI355X_MICROARCH.md "Global float atomics": one hot row is
// ~14x slower). Adds are spread over STAT_SLOTS copies by block id
// (neighbouring blocks sit on different XCDs); a fold kernel sums the slots.
// The 8 partial sums (4 channels x {A, B}) of a lane are reduced over the 16
// lanes of its DPP row by a transpose-reduce: xor-1 and xor-2 exchanges each
// halve the values a lane carries (4 + 2 DPP adds), then row rotations by 4
// and 8 finish the 4-lane groups (2 x 2 adds): 10 v_add_f32_dpp per fragment
// instead of 32 ds_bpermute + 32 adds. nb4 = first channel of the lane's
// 4-channel group; dB may be null.
__device__ __forceinline__ void stat_pair_atomic(const float (&sa)[4], const float (&sb)[4], float* dA, float* dB,
                                                 int nb4, int Nout, int lane) {
    const int l = lane & 15;
    const bool b0 = l & 1, b1 = (l >> 1) & 1;
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        v[2 * r] = sa[r];
        v[2 * r + 1] = sb[r];
    }
    float w[4], u[2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float keep = b0 ? v[4 + j] : v[j], send = b0 ? v[j] : v[4 + j];
        w[j] = keep + dpp_f32<0xB1>(send);  // quad_perm [1,0,3,2]
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const float keep = b1 ? w[2 + t] : w[t], send = b1 ? w[t] : w[2 + t];
        u[t] = keep + dpp_f32<0x4E>(send);  // quad_perm [2,3,0,1]
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        u[t] += dpp_f32<0x124>(u[t]);  // row_ror:4
        u[t] += dpp_f32<0x128>(u[t]);  // row_ror:8
    }
    // lane l < 4 holds channel r = 2*b0 + b1: u[0] = A, u[1] = B
    const int n = nb4 + 2 * b0 + b1;
    if (l < 4 && n < Nout) {
        atomicAdd(dA + n, u[0]);
        if (dB) atomicAdd(dB + n, u[1]);
    }
}

__device__ __forceinline__ void ld4bf(const bf16_t* p, float (&v)[4]) {
    const u32x2 w = *reinterpret_cast<const u32x2*>(p);
    v[0] = lo_bf(w[0]); v[1] = hi_bf(w[0]); v[2] = lo_bf(w[1]); v[3] = hi_bf(w[1]);
}

// IG_ACCUM: is the old output at output-grid pixel (oh, ow) valid (see IG_ACCUM_SUB2)?
__device__ __forceinline__ bool old_valid(const IGemmArgs& a, int oh, int ow) {
    if (!(a.flags & IG_ACCUM_SUB2)) return true;
    return (((oh * a.sY + a.oy) | (ow * a.sY + a.ox)) & 1) == 0;
}

// lane holds channels n = nb + i*16 + (lane>>4)*4 + r (r<4) of pixel m = mb + j*16 + (lane&15)
// Channel-fragment outer, pixel inner (as epilogue_bnb): the forward statistics
// of one fragment column (4 channels: shift, sum, sum of squares) are all that
// is live, and they go to the slab before the next column.
template <int FN, int FM>
__device__ __forceinline__ void epilogue_tile(const IGemmArgs& a, const f32x4 (&acc)[FN][FM], int nb, int mb,
                                              int lane, float* st) {
    const bool out_f32 = a.flags & IG_OUT_F32, relu = a.flags & IG_RELU, accum = a.flags & IG_ACCUM;
    const int ohw = a.OH * a.OW;
    long pixo[FM];
    bool oldok[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) {
        const int m = mb + j * 16;
        const int img = m / ohw, rem = m - img * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        pixo[j] = m < a.M ? (((long)img * a.YH + oh * a.sY + a.oy) * a.YW + ow * a.sY + a.ox) * a.ldy : -1;
        oldok[j] = accum && old_valid(a, oh, ow);
    }
    // shift of fragment column i, software-prefetched one column ahead
    const bool want_shift = st && a.shift;
    auto ld_shift = [&](int n, float (&o)[4]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (want_shift && n + r < a.Nout) ? a.shift[n + r] : 0.f;
    };
    float shn[4];
    ld_shift(nb, shn);
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const int n = nb + i * 16;
        const bool nok = n < a.Nout;
        const bool full = n + 3 < a.Nout && (a.ldy % 4) == 0;
        float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
        const float shv[4] = {shn[0], shn[1], shn[2], shn[3]};
        if (i + 1 < FN) ld_shift(n + 16, shn);
        if (nok) {
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                if (pixo[j] < 0) continue;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[i][j][r];
                    if (a.flags & IG_AFFINE) {  // folded inference BN: bias = [scale | shift]
                        if (n + r < a.Nout) v[r] = fmaf(v[r], a.bias[n + r], a.bias[a.Nout + n + r]);
                    } else if (a.bias) {
                        v[r] += (n + r < a.Nout) ? a.bias[n + r] : 0.f;
                    }
                }
                if (out_f32) {
                    float* y = reinterpret_cast<float*>(a.Y) + pixo[j] + n;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (relu) v[r] = fmaxf(v[r], 0.f);
                    if (full) {
                        *reinterpret_cast<f32x4*>(y) = f32x4{v[0], v[1], v[2], v[3]};
                    } else {
                        for (int r = 0; r < 4; ++r)
                            if (n + r < a.Nout) y[r] = v[r];
                    }
                } else {
                    bf16_t* y = reinterpret_cast<bf16_t*>(a.Y) + pixo[j] + n;
                    if (oldok[j]) {
                        if (full) {
                            const u32x2 o = *reinterpret_cast<const u32x2*>(y);
                            v[0] += lo_bf(o[0]); v[1] += hi_bf(o[0]); v[2] += lo_bf(o[1]); v[3] += hi_bf(o[1]);
                        } else {
                            for (int r = 0; r < 4; ++r)
                                if (n + r < a.Nout) v[r] += bf2f(y[r]);
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (relu) v[r] = fmaxf(v[r], 0.f);
                    const uint32_t lo = pack_bf2(v[0], v[1]), hi = pack_bf2(v[2], v[3]);
                    if (full) {
                        *reinterpret_cast<u32x2*>(y) = u32x2{lo, hi};
                    } else {
                        const bf16_t h[4] = {(bf16_t)(lo & 0xffff), (bf16_t)(lo >> 16), (bf16_t)(hi & 0xffff),
                                             (bf16_t)(hi >> 16)};
                        for (int r = 0; r < 4; ++r)
                            if (n + r < a.Nout) y[r] = h[r];
                    }
                    // statistics of the values BN will actually read (bf16-rounded)
                    v[0] = lo_bf(lo); v[1] = hi_bf(lo); v[2] = lo_bf(hi); v[3] = hi_bf(hi);
                }
                if (st) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float d = v[r] - shv[r];
                        s1[r] += d;
                        s2[r] += d * d;
                    }
                }
            }
        }
        if (st) stat_pair_atomic(s1, s2, st, st + a.Nout, n, a.Nout, lane);  // every lane (DPP)
    }
}

// IG_BNBWD epilogue (dgrad whose output is the upstream gradient g of a
// BatchNorm(+add)+ReLU), bf16 output with ldy == Nout, Nout % 8 == 0: the
// stored value is the ReLU-masked g (mask from the saved output's bit mask, or
// recomputed from the BN input x as fma(x, sc, sh) > 0) and the slab
// receives sum(g*xhat), sum(g) [, sum(g*xhat2)] (bn.hip row order), so the
// separate reduce pass over (g, x, y) disappears.
// Channel-fragment outer, pixel inner: every global read a fragment needs (x,
// y | x2, the old output when accumulating, BN parameters) is issued for all
// FM pixels before any is used -- one memory latency per fragment instead of
// FM -- and only 12 partial sums are live.
template <int FN, int FM>
__device__ __forceinline__ void epilogue_bnb(const IGemmArgs& a, const f32x4 (&acc)[FN][FM], int nb, int mb,
                                             int lane, float* st) {
    const bool accum = a.flags & IG_ACCUM;
    const bool has_y = a.bnym != nullptr, has_x2 = a.bnx2 != nullptr;
    const int ohw = a.OH * a.OW;
    long pixo[FM];
    bool oldok[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) {
        const int m = mb + j * 16;
        const int img = m / ohw, rem = m - img * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        pixo[j] = m < a.M ? (((long)img * a.YH + oh * a.sY + a.oy) * a.YW + ow * a.sY + a.ox) * a.ldy : -1;
        oldok[j] = accum && old_valid(a, oh, ow);
    }
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const int n = nb + i * 16;
        if (n >= a.Nout) continue;  // Nout % 8 == 0: a 4-channel group is all in or all out
        f32x4 mean = *reinterpret_cast<const f32x4*>(a.bnsave + n);
        f32x4 rstd = *reinterpret_cast<const f32x4*>(a.bnsave + a.Nout + n);
        f32x4 gam = {0.f, 0.f, 0.f, 0.f}, bet = {0.f, 0.f, 0.f, 0.f}, m2 = gam, r2 = gam;
        if (!has_y) {
            gam = *reinterpret_cast<const f32x4*>(a.bngamma + n);
            bet = *reinterpret_cast<const f32x4*>(a.bnbeta + n);
        }
        if (has_x2) {
            m2 = *reinterpret_cast<const f32x4*>(a.bnsave2 + n);
            r2 = *reinterpret_cast<const f32x4*>(a.bnsave2 + a.Nout + n);
        }
        u32x2 xw[FM], x2w[FM], ow[FM];
        uint32_t yw[FM];
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            xw[j] = x2w[j] = ow[j] = u32x2{0u, 0u};
            yw[j] = 0u;
            if (pixo[j] < 0) continue;
            const size_t e = (size_t)pixo[j] + n;
            xw[j] = *reinterpret_cast<const u32x2*>(a.bnx + e);
            if (has_y) yw[j] = (uint32_t)a.bnym[e >> 3] >> (e & 4);  // this lane's 4 channels
            if (has_x2) x2w[j] = *reinterpret_cast<const u32x2*>(a.bnx2 + e);
            if (oldok[j]) ow[j] = *reinterpret_cast<const u32x2*>(reinterpret_cast<const bf16_t*>(a.Y) + e);
        }
        float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f}, s3[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            if (pixo[j] < 0) continue;
            const float xv[4] = {lo_bf(xw[j][0]), hi_bf(xw[j][0]), lo_bf(xw[j][1]), hi_bf(xw[j][1])};
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r];
            if (accum) {
                v[0] += lo_bf(ow[j][0]); v[1] += hi_bf(ow[j][0]); v[2] += lo_bf(ow[j][1]); v[3] += hi_bf(ow[j][1]);
            }
            if (has_y) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (!((yw[j] >> r) & 1u)) v[r] = 0.f;
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float sc = gam[r] * rstd[r], sh = bet[r] - mean[r] * sc;
                    if (!(fmaf(xv[r], sc, sh) > 0.f)) v[r] = 0.f;
                }
            }
            const uint32_t lo = pack_bf2(v[0], v[1]), hi = pack_bf2(v[2], v[3]);
            *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(a.Y) + (size_t)pixo[j] + n) = u32x2{lo, hi};
            v[0] = lo_bf(lo); v[1] = hi_bf(lo); v[2] = lo_bf(hi); v[3] = hi_bf(hi);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                s1[r] += v[r];
                s2[r] += v[r] * ((xv[r] - mean[r]) * rstd[r]);
            }
            if (has_x2) {
                const float x2v[4] = {lo_bf(x2w[j][0]), hi_bf(x2w[j][0]), lo_bf(x2w[j][1]), hi_bf(x2w[j][1])};
#pragma unroll
                for (int r = 0; r < 4; ++r) s3[r] += v[r] * ((x2v[r] - m2[r]) * r2[r]);
            }
        }
        stat_pair_atomic(s2, s1, st, st + a.Nout, n, a.Nout, lane);
        if (has_x2) stat_pair_atomic(s3, s3, st + 2 * a.Nout, nullptr, n, a.Nout, lane);
    }
}

template <int FN, int FM, int EPI>
__device__ __forceinline__ void epilogue(const IGemmArgs& a, const f32x4 (&acc)[FN][FM], int nb, int mb, int lane,
                                         float* st) {
    if (EPI == 1)
        epilogue_bnb<FN, FM>(a, acc, nb, mb, lane, st);
    else
        epilogue_tile<FN, FM>(a, acc, nb, mb, lane, st);
}

// ---------------------------------------------------- LDS-staged epilogue
// (EPI 2; bf16 output, no bias / ReLU / fp32; one tile per block so the
// whole stage ring is free once the main loop has drained.)
// The block's BM x BN accumulator tile is rounded to bf16 into LDS (row pitch
// BN*2 + 16 B), then re-read as 16-B row chunks: consecutive lanes cover
// consecutive channels of one output pixel, so every global access of the
// epilogue -- the store, the IG_ACCUM read-back, and the IG_BNBWD reads of
// x, y / x2 -- is a coalesced row segment of BN*2 bytes instead of sixteen
// 32-B pieces per wave instruction. Statistics (forward: sum, sumsq; BNBWD:
// sum(g*xhat), sum(g) [, sum(g*xhat2)]) are per thread over its 8 channels,
// folded across the threads sharing a channel chunk in LDS, then one atomic
// per channel and quantity into the block's slab slot.
// (IG_ACCUM adds the old value to the bf16-rounded new one: one extra
// rounding of the new term versus the direct epilogue.)
// The fragment pass (1) is the caller's functor put(smem, P) (it writes this thread's accumulators as
// bf16 at [pixel row][channel] with row pitch P bytes), so any MFMA shape can feed it.
// IG_BNBWD on a dense output grid: the BatchNorm input x (and the mask bits) of this thread's epilogue chunks,
// loaded into registers at kernel START (epi_prefetch), so their HBM latency hides under the main loop instead
// of stalling the epilogue after it (v3; the short-K dgrads are epilogue-bound: 1024@14 -> 256 dgrad 251 us,
// with the fused BN backward 443 us before this)
// Staged-epilogue LDS swizzle (epilogue_lds_put): byte b of tile row r sits at b ^ ((r & 15) << 3) -- the row's
// 8-B slots XORed with the row's low 4 bits; shared with the streaming kernel's per-wave epilogue (conv_stream.hip).
__host__ __device__ constexpr int epi_swz(int row, int byte) { return byte ^ ((row & 15) << 3); }

// the 16-B chunk cc of a swizzled row r: chunk cc ^ ((r >> 1) & 7), its two 8-B halves swapped when r is odd
__device__ __forceinline__ u32x4 epi_read(const char* base, int row, int pitch, int cc) {
    const u32x4 t = *reinterpret_cast<const u32x4*>(base + row * pitch + ((cc * 16) ^ ((row & 14) << 3)));
    return (row & 1) ? u32x4{t[2], t[3], t[0], t[1]} : t;
}

// per-(quantity, channel-in-chunk) block stride of the statistics fold image [nq][8][RG][CPR] (floats): padded so
// the cc-fastest reads of two (or four) consecutive blocks fall in distinct banks
__host__ __device__ constexpr int epi_red_stride(int BN, int NT) {
    return (NT / (BN / 8)) * (BN / 8) + ((BN / 8) < 32 ? (BN / 8) : 0);
}

// staged-epilogue chunks per thread whose global reads (x, mask bits, accumulate operand) are issued together: 4.
// (Round 6 A/B with 8 for the 256-row tiles -- 2 round trips instead of 4, 241 VGPRs, no spills: dgrad + BN backward
// within +-2 % isolated, in-step 17,497 / 17,515 vs 17,511 / 17,484 img/s: not kept.) -DEPI_QB=n overrides (A/B builds)
#ifndef EPI_QB
#define EPI_QB 0
#endif

template <int BM, int BN, int NT>
struct EpiPF {
    static constexpr int CPR = BN / 8, RG = NT / CPR, NQ = BM / RG;
    u32x4 xo[NQ];
    uint32_t yo[NQ];
    bool on;
};

__device__ __forceinline__ bool epi_dense(const IGemmArgs& a) {
    return a.YH == a.OH && a.YW == a.OW && a.sY == 1 && a.oy == 0 && a.ox == 0 && !(a.flags & IG_ACCUM_SUB2);
}

template <int BM, int BN, int NT>
__device__ __forceinline__ void epi_prefetch(const IGemmArgs& a, EpiPF<BM, BN, NT>& pf, int m0, int n0, int tid) {
    using PF = EpiPF<BM, BN, NT>;
    pf.on = (a.flags & IG_BNBWD) && epi_dense(a);
    if (!pf.on) return;
    const int cc = tid % PF::CPR, rg = tid / PF::CPR;
    const int n = n0 + cc * 8;
    const bool nok = n < a.Nout;
#pragma unroll
    for (int q = 0; q < PF::NQ; ++q) {
        const int m = m0 + rg + PF::RG * q;
        const bool ok = nok && m < a.M;
        const long e = (long)(ok ? m : 0) * a.ldy + (nok ? n : 0);
        pf.xo[q] = (ok && a.bnx) ? *reinterpret_cast<const u32x4*>(a.bnx + e) : u32x4{0u, 0u, 0u, 0u};
        pf.yo[q] = (ok && a.bnym) ? a.bnym[e >> 3] : 0u;
    }
}

template <int BM, int BN, int NT, class Put>
__device__ __forceinline__ void epilogue_lds_put(const IGemmArgs& a, Put put, char* smem, int m0, int n0, int tid,
                                                 float* st, const EpiPF<BM, BN, NT>* pf = nullptr) {
    // LDS image of the bf16 tile: row pitch P = BN * 2 bytes (a multiple of the 256-B bank row for BN >= 128) with
    // the 8-B slots XOR-swizzled by the row: slot s of row r at s ^ (r & 15) (epi_swz). The fragment writes
    // (ds_write_b64, 16 lanes = 16 consecutive rows, one column) then cover 16 distinct slots of a 128-B bank window
    // and the row-chunk reads (ds_read_b128: a 16-B chunk cc of row r sits at chunk cc ^ ((r >> 1) & 7), halves
    // swapped when r is odd) hit 16 distinct 16-B slots per lane group: conflict-free both ways (the padded
    // BN * 2 + 16 pitch it replaces had 2-way conflicts on both)
    constexpr int P = BN * 2;       // LDS row pitch, bytes
    constexpr int CPR = BN / 8;     // 16-B chunks per row
    constexpr int RG = NT / CPR;    // rows processed concurrently (row groups)
    constexpr int NQ = BM / RG;     // chunks per thread
    static_assert(NT % CPR == 0 && BM % RG == 0, "epilogue split");
    const bool accum = a.flags & IG_ACCUM, bnb = a.flags & IG_BNBWD;
    const bool has_y = bnb && a.bnym, has_x2 = bnb && a.bnx2;
    // this thread's fixed channel chunk (step 2); the forward-statistics shift is
    // loaded now so its latency hides behind step (1)
    const int cc = tid % CPR, rg = tid / CPR;
    const int n = n0 + cc * 8;
    const bool nok = n < a.Nout;  // Nout % 8 == 0 on this path
    float mean[8], rstd[8], sc[8], sh[8], m2[8], r2[8];
    // plain epilogue: the eval forward's folded BatchNorm (IG_AFFINE: a.bias = [scale | shift] -> sc / sh),
    // applied to the bf16-rounded conv output as the training BatchNorm is, then the accumulate, then ReLU
    const bool affine = !bnb && (a.flags & IG_AFFINE), relu = !bnb && (a.flags & IG_RELU);
    if (!bnb) {  // forward statistics: mean[] holds the shift (previous batch mean, or 0)
        const bool ld = st && a.shift && nok;
        const f32x4 lo = ld ? *reinterpret_cast<const f32x4*>(a.shift + n) : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 hi = ld ? *reinterpret_cast<const f32x4*>(a.shift + n + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            mean[c] = lo[c];
            mean[4 + c] = hi[c];
        }
        const bool la = affine && nok;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f32x4 s4 = la ? *reinterpret_cast<const f32x4*>(a.bias + n + 4 * h) : f32x4{1.f, 1.f, 1.f, 1.f};
            const f32x4 t4 =
                la ? *reinterpret_cast<const f32x4*>(a.bias + a.Nout + n + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                sc[4 * h + c] = s4[c];
                sh[4 * h + c] = t4[c];
            }
        }
    }
    // (1) fragments -> LDS
    put(smem, P);
    __syncthreads();
    // (2) row chunks: thread -> fixed channel chunk cc, rows rg + RG*q
    float bb[8];  // IG_BNBWD: per-channel bias added before the mask (second K segment, bn_gram.hip)
#pragma unroll
    for (int c = 0; c < 8; ++c) bb[c] = 0.f;
    if (bnb && nok && a.bias) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f32x4 b4 = *reinterpret_cast<const f32x4*>(a.bias + n + 4 * h);
#pragma unroll
            for (int c = 0; c < 4; ++c) bb[4 * h + c] = b4[c];
        }
    }
    if (bnb && nok) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f32x4 mu = *reinterpret_cast<const f32x4*>(a.bnsave + n + 4 * h);
            const f32x4 rs = *reinterpret_cast<const f32x4*>(a.bnsave + a.Nout + n + 4 * h);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                mean[4 * h + r] = mu[r];
                rstd[4 * h + r] = rs[r];
            }
            if (!has_y) {
                const f32x4 g = *reinterpret_cast<const f32x4*>(a.bngamma + n + 4 * h);
                const f32x4 b = *reinterpret_cast<const f32x4*>(a.bnbeta + n + 4 * h);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    sc[4 * h + r] = g[r] * rs[r];
                    sh[4 * h + r] = b[r] - mu[r] * sc[4 * h + r];
                }
            }
            if (has_x2) {
                const f32x4 mu2 = *reinterpret_cast<const f32x4*>(a.bnsave2 + n + 4 * h);
                const f32x4 rs2 = *reinterpret_cast<const f32x4*>(a.bnsave2 + a.Nout + n + 4 * h);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    m2[4 * h + r] = mu2[r];
                    r2[4 * h + r] = rs2[r];
                }
            }
        }
    }
    float s1[8], s2[8], s3[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) s1[c] = s2[c] = s3[c] = 0.f;
    const int ohw = a.OH * a.OW;
    // dense output (every stride-1 conv and dgrad: the output grid IS the row grid): element offset m * ldy + n,
    // without the two runtime divisions per row chunk of the general (strided-dgrad phase / padded) map
    const bool dense = epi_dense(a);
    const bool pfon = pf && pf->on;  // x / mask bits already in registers (epi_prefetch)
    constexpr int QB = EPI_QB > 0 ? EPI_QB : 4;  // chunks whose global reads are issued together
#pragma unroll
    for (int q0 = 0; q0 < NQ; q0 += QB) {
        long e[QB];
        u32x4 xo[QB], x2o[QB], oo[QB];
        uint32_t yo[QB];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
            const int row = rg + RG * (q0 + u);
            const int m = m0 + row;
            e[u] = -1;
            if (q0 + u < NQ && m < a.M && nok) {
                bool ov = true;
                if (dense) {
                    e[u] = (long)m * a.ldy + n;
                } else {
                    const int img = m / ohw, rem = m - img * ohw;
                    const int oh = rem / a.OW, ow = rem - oh * a.OW;
                    e[u] = (((long)img * a.YH + oh * a.sY + a.oy) * a.YW + ow * a.sY + a.ox) * a.ldy + n;
                    ov = old_valid(a, oh, ow);
                }
                if (accum) {
                    oo[u] = ov ? *reinterpret_cast<const u32x4*>(reinterpret_cast<const bf16_t*>(a.Y) + e[u])
                               : u32x4{0u, 0u, 0u, 0u};
                }
                if (bnb) {
                    if (pfon) {
                        xo[u] = pf->xo[q0 + u];
                        yo[u] = pf->yo[q0 + u];
                    } else {
                        // (bnx null: the bits give the mask, sum(g xhat) is formed elsewhere -- bn_gram.hip)
                        xo[u] = a.bnx ? *reinterpret_cast<const u32x4*>(a.bnx + e[u]) : u32x4{0u, 0u, 0u, 0u};
                        if (has_y) yo[u] = a.bnym[e[u] >> 3];
                    }
                    if (has_x2) x2o[u] = *reinterpret_cast<const u32x4*>(a.bnx2 + e[u]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < QB; ++u) {
            if (e[u] < 0) continue;
            const int row = rg + RG * (q0 + u);
            const u32x4 t = epi_read(smem, row, P, cc);
            float v[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[2 * k] = lo_bf(t[k]) + bb[2 * k];
                v[2 * k + 1] = hi_bf(t[k]) + bb[2 * k + 1];
                if (affine) {
                    v[2 * k] = fmaf(v[2 * k], sc[2 * k], sh[2 * k]);
                    v[2 * k + 1] = fmaf(v[2 * k + 1], sc[2 * k + 1], sh[2 * k + 1]);
                }
                if (accum) {
                    v[2 * k] += lo_bf(oo[u][k]);
                    v[2 * k + 1] += hi_bf(oo[u][k]);
                }
                if (relu) {
                    v[2 * k] = fmaxf(v[2 * k], 0.f);
                    v[2 * k + 1] = fmaxf(v[2 * k + 1], 0.f);
                }
            }
            float xv[8];
            if (bnb) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    xv[2 * k] = lo_bf(xo[u][k]);
                    xv[2 * k + 1] = hi_bf(xo[u][k]);
                }
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const bool keep = has_y ? ((yo[u] >> c) & 1u) : (fmaf(xv[c], sc[c], sh[c]) > 0.f);
                    if (!keep) v[c] = 0.f;
                }
            }
            u32x4 o;
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = pack_bf2(v[2 * k], v[2 * k + 1]);
            *reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(a.Y) + e[u]) = o;
            if (st) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {  // statistics of the stored (bf16) values
                    v[2 * k] = lo_bf(o[k]);
                    v[2 * k + 1] = hi_bf(o[k]);
                }
                if (bnb) {
#pragma unroll
                    for (int c = 0; c < 8; ++c) {
                        s1[c] += v[c] * ((xv[c] - mean[c]) * rstd[c]);
                        s2[c] += v[c];
                    }
                    if (has_x2) {
#pragma unroll
                        for (int c = 0; c < 8; ++c) {
                            const float x2 = c & 1 ? hi_bf(x2o[u][c >> 1]) : lo_bf(x2o[u][c >> 1]);
                            s3[c] += v[c] * ((x2 - m2[c]) * r2[c]);
                        }
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < 8; ++c) {
                        const float d = v[c] - mean[c];
                        s1[c] += d;
                        s2[c] += d * d;
                    }
                }
            }
        }
    }
    if (!st) return;
    // (3) fold the RG row groups per channel in LDS, one atomic per channel and quantity. Image [nq][8][RG][CPR]
    // (+ pad per (q, c) block): the writes (fixed q, c; 32 lanes = consecutive (rg, cc)) and the reads (cc fastest)
    // are conflict-free ([nq][RG][BN] had 8-way conflicts on the writes)
    const int nq = has_x2 ? 3 : 2;
    constexpr int RS = epi_red_stride(BN, NT);
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();  // everyone is done reading the tile
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        red[(0 * 8 + c) * RS + rg * CPR + cc] = s1[c];
        red[(1 * 8 + c) * RS + rg * CPR + cc] = s2[c];
        if (has_x2) red[(2 * 8 + c) * RS + rg * CPR + cc] = s3[c];
    }
    __syncthreads();
    for (int idx = tid; idx < nq * BN; idx += NT) {
        const int qi = idx / BN, r = idx - qi * BN;
        const int c8 = r / CPR, k = r - c8 * CPR, ch = k * 8 + c8;
        if (n0 + ch >= a.Nout) continue;
        float sum = 0.f;
#pragma unroll 8
        for (int g = 0; g < RG; ++g) sum += red[(qi * 8 + c8) * RS + g * CPR + k];
        atomicAdd(st + qi * a.Nout + n0 + ch, sum);
    }
}

// 16x16x32 fragments (lane: 4 channels of one pixel, 8 B) -> the staged epilogue
template <int BM, int BN, int NT, int FN, int FM>
__device__ __forceinline__ void epilogue_lds(const IGemmArgs& a, const f32x4 (&acc)[FN][FM], char* smem, int m0,
                                             int n0, int wrow0, int wcol0, int lane, int tid, float* st,
                                             const EpiPF<BM, BN, NT>* pf = nullptr) {
    auto put = [&](char* sm, int P) {
#pragma unroll
        for (int j = 0; j < FM; ++j)
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int row = wrow0 + j * 16 + (lane & 15), col = wcol0 + i * 16 + (lane >> 4) * 4;
                const f32x4 v = acc[i][j];
                *reinterpret_cast<u32x2*>(sm + row * P + epi_swz(row, col * 2)) =
                    u32x2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
            }
    };
    epilogue_lds_put<BM, BN, NT>(a, put, smem, m0, n0, tid, st, pf);
}

// LDS row swizzle of the stage ring: the 16-B chunk a lane's fragment read or DMA
// write lands in is the logical chunk XOR swz(row).
//  * 128-B rows (BK = 64): swz = row & 7 -- the 8 rows of a ds_read_b128 lane group
//    cover all 8 chunk columns of the 256-B bank row;
//  * 64-B rows (BK = 32): a 256-B bank row holds 4 rows (bank group = 16 (row & 3) +
//    4 chunk), and a ds_read_b128 lane group {0-3,12-15,20-27} (and the three others,
//    MI355X_MICROARCH.md LDS table) takes row blocks {0,3} at logical chunk g and {1,2}
//    at g ^ 1: swz = h[(row >> 2) & 3] with h = {0, 2, 3, 1} gives all 16 bank groups
//    distinct physical chunks in every lane group -> conflict-free.
template <int RB>
__device__ __forceinline__ int lds_swz(int row) {
    if (RB == 128) return row & 7;
    return (120 >> (2 * ((row >> 2) & 3))) & 3;
}

// MFMA over one stage held in LDS (rows of RB bytes = RB / 64 k-steps of 32,
// chunk-swizzled); fk[ks] = element offset of the lane's 16-B chunk in k-step ks
template <int FN, int FM, int RB = 128>
__device__ __forceinline__ void mfma_stage(f32x4 (&acc)[FN][FM], const bf16_t* bx, const bf16_t* bw, int fk0,
                                           int fk1) {
    constexpr int LDKE = RB / 2;  // row pitch in elements
#pragma unroll
    for (int ks = 0; ks < RB / 64; ++ks) {
        bf16x8 fw[FN], fx[FM];
#pragma unroll
        for (int i = 0; i < FN; ++i)
            fw[i] = *reinterpret_cast<const bf16x8*>(bw + i * 16 * LDKE + (ks ? fk1 : fk0));
#pragma unroll
        for (int j = 0; j < FM; ++j)
            fx[j] = *reinterpret_cast<const bf16x8*>(bx + j * 16 * LDKE + (ks ? fk1 : fk0));
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[i], fx[j], acc[i][j], 0, 0, 0);
    }
}

// MFMA over one 128-deep fp8 stage (rows of 128 B, chunk-swizzled): one
// block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 per fragment pair at twice
// the bf16 MFMA rate. Each lane feeds 32 consecutive k of its row (logical
// chunks 2g, 2g+1, g = lane>>4) for BOTH operands -- the same lane->k map on
// A and B, so the hardware's k order inside the instruction cancels out. The
// per-tensor power-of-two scales ride in the instruction's E8M0 operands:
// dequantisation is free.
template <int FN, int FM, int FB>  // FB: format of the gathered operand, 0 e4m3 / 1 e5m2
__device__ __forceinline__ void mfma_stage_fp8(f32x4 (&acc)[FN][FM], const char* bx, const char* bw, int c0, int c1,
                                               int sw8, int sx8) {
    i32x8 fw[FN], fx[FM];
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const u32x4 lo = *reinterpret_cast<const u32x4*>(bw + i * 16 * 128 + c0);
        const u32x4 hi = *reinterpret_cast<const u32x4*>(bw + i * 16 * 128 + c1);
        fw[i] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int j = 0; j < FM; ++j) {
        const u32x4 lo = *reinterpret_cast<const u32x4*>(bx + j * 16 * 128 + c0);
        const u32x4 hi = *reinterpret_cast<const u32x4*>(bx + j * 16 * 128 + c1);
        fx[j] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    }
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fw[i], fx[j], acc[i][j], 0, FB, 0, sw8, 0, sx8);
}

// ======================================================= LDS-DMA ring kernel
// NW waves per block (4: two blocks per CU; 8: one big-tile block per CU,
// two waves per SIMD, fewer L2->LDS bytes per MFMA FLOP).
// EB = operand element bytes: 2 (bf16, 64-deep stages) or 1 (fp8 e4m3, 128-deep
// stages, IG_FP8): the DMA moves 16-B chunks either way, the gather differs
// only in elements per chunk.
// s_setprio(1) around each stage's MFMAs (256@14 3x3 fwd 366 -> 357 us, 512@7 3x3 337 -> 320 us,
// bench +0.9 %; static priority for the second half of the waves, MI355X_MICROARCH.md "Two waves
// per SIMD" item 4, measured neutral and removed)
// RB: LDS row bytes = K bytes per stage (128: BK 64 bf16; 64: BK 32 bf16, twice the stages in
// the same LDS -> more stages in flight for the 256x256 tile, whose 64-KiB BK-64 stages allow
// only a 2-deep ring in 160 KiB).
template <int BM, int BN, int WN, int NS, int MODE, int NW, int EPI, int EB = 2, int FB = 0,
          int RB = 128>  // MODE 0: one tap/stage
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void igemm_dma_kernel(const IGemmArgs a) {
    constexpr int WM = NW / WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    constexpr int RPP = 1024 / RB;             // rows per DMA piece (64 lanes x 16 B)
    constexpr int CPR = RB / 16;               // 16-B chunks per row
    constexpr int QA = BM / (RPP * NW), QB = BN / (RPP * NW);  // DMA pieces per wave per stage
    static_assert(QA >= 1 && QB >= 1 && WM * WN == NW, "tile / wave split");
    static_assert(RB == 128 || (RB == 64 && EB == 2), "64-B rows: bf16 only");
    constexpr int LPS = QA + QB;               // vmcnt units per stage
    constexpr int KS = RB / EB;                // k elements per stage (one LDS row)
    constexpr int CE = 16 / EB;                // elements per 16-B chunk
    constexpr int SAB = BM * RB, SBB = BN * RB;  // bytes per stage buffer
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sX = smem;                 // [NS][BM][RB]
    char* sW = smem + NS * SAB;      // [NS][BN][RB]

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wid % WN, wm = wid / WN;
    const int nbn = (a.Nout + BN - 1) / BN;
    const int nbm = (a.M + BM - 1) / BM;
    const int ntiles = nbm * nbn;
    const int G = gridDim.x;
    const int lid = xcd_remap(blockIdx.x, G);
    if (lid >= ntiles) return;
    const int my_tiles = (ntiles - lid + G - 1) / G;
    const int K = a.nth * a.ntw * a.C;
    const int nk = max(1, (K + KS - 1) / KS);
    const int nstages = my_tiles * nk;
    const int ohw = a.OH * a.OW;
    // this lane's DMA slot: row lane / CPR of each RPP-row piece, physical chunk
    // lane % CPR -> logical chunk (lane % CPR) ^ swz(row) (pieces start at multiples of RPP)
    const int lrow = lane / CPR;
    const int lchunk = (lane % CPR) ^ lds_swz<RB>(lrow);
    const char* zero = reinterpret_cast<const char*>(g_igemm_zero);
    const char* Xb = reinterpret_cast<const char*>(a.X);
    const char* Wb = reinterpret_cast<const char*>(a.Wk);

    // gather state of the tile being LOADED (rows wid*QA*8 + q*8 + lrow)
    const char* xrow[QA];
    int ih0[QA], iw0[QA];
    bool mok[QA];
    const char* wrow[QB];
    bool nok[QB];
    auto setup_rows = [&](int tile) {
        const int m0 = (tile / nbn) * BM, n0 = (tile % nbn) * BN;
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int m = m0 + (wid * QA + q) * RPP + lrow;
            mok[q] = m < a.M;
            const int mm = mok[q] ? m : 0;
            const int img = mm / ohw, rem = mm - img * ohw;
            const int oh = rem / a.OW, ow = rem - oh * a.OW;
            xrow[q] = Xb + (size_t)img * a.H * a.W * a.C * EB;
            ih0[q] = oh * a.sA;
            iw0[q] = ow * a.sA;
        }
#pragma unroll
        for (int q = 0; q < QB; ++q) {
            const int n = n0 + (wid * QB + q) * RPP + lrow;
            nok[q] = n < a.Nout;
            wrow[q] = Wb + (size_t)(nok[q] ? n : 0) * a.ldb * EB;
        }
    };
    auto issue = [&](int kt, int buf) {
        int t, c;
        const int k = kt * KS + lchunk * CE;
        if (MODE == 0) {
            t = (kt * KS) / a.C;
            c = kt * KS - t * a.C + lchunk * CE;
        } else {
            t = k / a.C;
            c = k - t * a.C;
        }
        const bool kok = k < K;
        const int ti = kok ? t / a.ntw : 0, tj = kok ? t - ti * a.ntw : 0;
        const int dh = a.dh0 + ti * a.dhs, dw = a.dw0 + tj * a.dws;
        const int wtap = (a.kh0 + ti * a.khs) * a.KW + (a.kw0 + tj * a.kws);
        char* dX = sX + buf * SAB + (wid * QA) * 1024;
        char* dW = sW + buf * SBB + (wid * QB) * 1024;
#pragma unroll
        for (int q = 0; q < QA; ++q) {
            const int ih = ih0[q] + dh, iw = iw0[q] + dw;
            const bool ok = kok && mok[q] && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
            const char* src = ok ? xrow[q] + (((size_t)ih * a.W + iw) * a.C + c) * EB : zero;
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                             (void __attribute__((address_space(3)))*)(dX + q * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < QB; ++q) {
            const char* src = (kok && nok[q]) ? wrow[q] + ((size_t)wtap * a.C + c) * EB : zero;
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                             (void __attribute__((address_space(3)))*)(dW + q * 1024), 16, 0, 0);
        }
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float* st = a.stats ? a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * ((a.flags & IG_BNBWD) ? 3 : 2) * a.Nout
                        : nullptr;

    // issue cursor (stage index + its tile / kt)
    int is = 0, itj = 0, ikt = 0;
    auto issue_next = [&]() {
        if (is < nstages) {
            if (ikt == 0) setup_rows(lid + itj * G);
            issue(ikt, is % NS);
            ++is;
            if (++ikt == nk) {
                ikt = 0;
                ++itj;
            }
        }
    };
#pragma unroll
    for (int p = 0; p < NS - 1; ++p) issue_next();

    const int fr = lane & 15;
    // fragment rows are 16-row aligned + fr, so swz(row) == swz(fr)
    const int fk0 = (((lane >> 4) + 0) ^ lds_swz<RB>(fr)) * 8, fk1 = (((lane >> 4) + 4) ^ lds_swz<RB>(fr)) * 8;
    // fp8: the lane's 32 bytes are logical chunks 2g, 2g+1 of its row (byte offsets)
    const int f8c0 = ((2 * (lane >> 4)) ^ (fr & 7)) * 16, f8c1 = ((2 * (lane >> 4) + 1) ^ (fr & 7)) * 16;
    const int sx8 = EB == 1 ? 127 + a.xexp[0] : 127, sw8 = EB == 1 ? 127 + a.wexp[0] : 127;
    int tj = 0, kt = 0;
    for (int s = 0; s < nstages; ++s) {
        // stage s landed for this wave when at most (stages issued after s) x LPS remain
        // (steady state: NS-2 stages beyond s are in flight; near the end fewer -> drain)
        if (is - 1 - s >= NS - 2)
            __builtin_amdgcn_s_waitcnt((((NS - 2) * LPS) & 0xF) | ((((NS - 2) * LPS) >> 4) << 14) | (0x7 << 4) |
                                       (0xF << 8));
        else
            __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
        __builtin_amdgcn_s_barrier();  // ... and for every wave; buffer (s-1)%NS is free
        issue_next();
        const int buf = s % NS;
        if (EB == 1)
            mfma_stage_fp8<FN, FM, FB>(acc, sX + buf * SAB + (wm * TM + fr) * 128, sW + buf * SBB + (wn * TN + fr) * 128,
                                   f8c0, f8c1, sw8, sx8);
        else {
            __builtin_amdgcn_s_setprio(1);
            mfma_stage<FN, FM, RB>(acc, reinterpret_cast<const bf16_t*>(sX + buf * SAB + (wm * TM + fr) * RB),
                                   reinterpret_cast<const bf16_t*>(sW + buf * SBB + (wn * TN + fr) * RB), fk0, fk1);
            __builtin_amdgcn_s_setprio(0);
        }
        if (++kt == nk) {
            const int tile = lid + tj * G;
            const int m0 = (tile / nbn) * BM, n0 = (tile % nbn) * BN;
            if (EPI == 2) break;  // one tile per block (host): staged epilogue after the loop
            epilogue<FN, FM, EPI>(a, acc, n0 + wn * TN + (lane >> 4) * 4, m0 + wm * TM + fr, lane, st);
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            kt = 0;
            ++tj;
        }
    }
    if (EPI == 2) {  // every stage has landed and (barrier) every wave is done reading the ring
        __syncthreads();
        const int m0 = (lid / nbn) * BM, n0 = (lid % nbn) * BN;
        epilogue_lds<BM, BN, NW * 64, FN, FM>(a, acc, smem, m0, n0, wm * TM, wn * TN, lane, tid, st);
    }
}

// ================================================= register-staged kernel
template <int BM, int BN, int WN, int MODE, int EPI>  // MODE 0: C%64==0, 1: C%8==0, 2: stem row segments
__global__ __launch_bounds__(256, 2) void igemm_rs_kernel(const IGemmArgs a) {
    constexpr int WM = 4 / WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int FM = TM / 16, FN = TN / 16;
    constexpr int A_CH = BM / 32, B_CH = BN / 32;  // 16-B chunks per thread per stage
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* sX = reinterpret_cast<bf16_t*>(smem);  // [2][BM][LDK]
    bf16_t* sW = sX + 2 * BM * LDK;                // [2][BN][LDK]

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wn = wid % WN, wm = wid / WN;
    const int nbn = (a.Nout + BN - 1) / BN;
    const int nbm = (a.M + BM - 1) / BM;
    const int ntiles = nbm * nbn;
    const int G = gridDim.x;
    const int lid = xcd_remap(blockIdx.x, G);
    if (lid >= ntiles) return;
    const int my_tiles = (ntiles - lid + G - 1) / G;
    const int K = MODE == 2 ? a.nth * 32 : a.nth * a.ntw * a.C;
    const int nk = max(1, (K + BK - 1) / BK);
    const int nstages = my_tiles * nk;
    const int col8 = tid & 7;
    const int ohw = a.OH * a.OW;

    const bf16_t* xrow[A_CH];
    int ih0[A_CH], iw0[A_CH];
    bool mok[A_CH];
    const bf16_t* wrow[B_CH];
    bool nok[B_CH];
    auto setup_rows = [&](int tile) {
        const int m0 = (tile / nbn) * BM, n0 = (tile % nbn) * BN;
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
            const int m = m0 + (tid >> 3) + 32 * i;
            mok[i] = m < a.M;
            const int mm = mok[i] ? m : 0;
            const int img = mm / ohw, rem = mm - img * ohw;
            const int oh = rem / a.OW, ow = rem - oh * a.OW;
            xrow[i] = a.X + (size_t)img * a.H * a.W * a.C;
            ih0[i] = oh * a.sA;
            iw0[i] = ow * a.sA;
        }
#pragma unroll
        for (int j = 0; j < B_CH; ++j) {
            const int n = n0 + (tid >> 3) + 32 * j;
            nok[j] = n < a.Nout;
            wrow[j] = a.Wk + (size_t)(nok[j] ? n : 0) * a.ldb;
        }
    };

    u32x4 rx[A_CH], rw[B_CH];
    auto load_stage = [&](int kt) {
        if (MODE == 2) {
            const int kh = kt * 2 + (col8 >> 2);
            const int seg = (col8 & 3) * 8, kw0 = seg >> 2;
            const bool kok = kh < a.nth;
#pragma unroll
            for (int i = 0; i < A_CH; ++i) {
                const int ih = ih0[i] + a.dh0 + kh, iw = iw0[i] + a.dw0 + kw0;
                const bool rok = kok && mok[i] && (unsigned)ih < (unsigned)a.H;
                const bool lo_ok = rok && kw0 < a.ntw && (unsigned)iw < (unsigned)a.W;
                const bool hi_ok = rok && kw0 + 1 < a.ntw && (unsigned)(iw + 1) < (unsigned)a.W;
                const long off = ((long)ih * a.W + iw) * 4;
                u32x2 lo = {0, 0}, hi = {0, 0};
                if (lo_ok) lo = *reinterpret_cast<const u32x2*>(xrow[i] + off);
                if (hi_ok) hi = *reinterpret_cast<const u32x2*>(xrow[i] + off + 4);
                rx[i] = u32x4{lo[0], lo[1], hi[0], hi[1]};
            }
#pragma unroll
            for (int j = 0; j < B_CH; ++j) {
                u32x4 v = {0, 0, 0, 0};
                if (kok && nok[j]) v = *reinterpret_cast<const u32x4*>(wrow[j] + kh * 32 + seg);
                rw[j] = v;
            }
            return;
        }
        const int k = kt * BK + col8 * 8;
        int t, c;
        if (MODE == 0) {
            t = (kt * BK) / a.C;
            c = kt * BK - t * a.C + col8 * 8;
        } else {
            t = k / a.C;
            c = k - t * a.C;
        }
        const bool kok = k < K;
        const int ti = kok ? t / a.ntw : 0, tj = kok ? t - ti * a.ntw : 0;
        const int dh = a.dh0 + ti * a.dhs, dw = a.dw0 + tj * a.dws;
        const int wtap = (a.kh0 + ti * a.khs) * a.KW + (a.kw0 + tj * a.kws);
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
            const int ih = ih0[i] + dh, iw = iw0[i] + dw;
            const bool ok = kok && mok[i] && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
            u32x4 v = {0, 0, 0, 0};
            if (ok) v = *reinterpret_cast<const u32x4*>(xrow[i] + ((size_t)ih * a.W + iw) * a.C + c);
            rx[i] = v;
        }
#pragma unroll
        for (int j = 0; j < B_CH; ++j) {
            u32x4 v = {0, 0, 0, 0};
            if (kok && nok[j]) v = *reinterpret_cast<const u32x4*>(wrow[j] + wtap * a.C + c);
            rw[j] = v;
        }
    };
    auto store_stage = [&](int buf) {
        bf16_t* dx = sX + buf * BM * LDK;
        bf16_t* dw = sW + buf * BN * LDK;
#pragma unroll
        for (int i = 0; i < A_CH; ++i)
            *reinterpret_cast<u32x4*>(dx + ((tid >> 3) + 32 * i) * LDK + ((col8 ^ ((tid >> 3) & 7)) * 8)) = rx[i];
#pragma unroll
        for (int j = 0; j < B_CH; ++j)
            *reinterpret_cast<u32x4*>(dw + ((tid >> 3) + 32 * j) * LDK + ((col8 ^ ((tid >> 3) & 7)) * 8)) = rw[j];
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float* st = a.stats ? a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * ((a.flags & IG_BNBWD) ? 3 : 2) * a.Nout
                        : nullptr;

    setup_rows(lid);
    load_stage(0);
    store_stage(0);
    __syncthreads();
    const int fr = lane & 15;
    const int fk0 = (((lane >> 4) + 0) ^ (fr & 7)) * 8, fk1 = (((lane >> 4) + 4) ^ (fr & 7)) * 8;
    int tj = 0, kt = 0;
    for (int s = 0; s < nstages; ++s) {
        const int buf = s & 1;
        const bool has_next = s + 1 < nstages;
        if (has_next) {
            if (kt + 1 == nk) {
                setup_rows(lid + (tj + 1) * G);
                load_stage(0);
            } else {
                load_stage(kt + 1);
            }
        }
        mfma_stage<FN, FM>(acc, sX + buf * BM * LDK + (wm * TM + fr) * LDK,
                           sW + buf * BN * LDK + (wn * TN + fr) * LDK, fk0, fk1);
        if (kt + 1 == nk) {
            const int tile = lid + tj * G;
            const int m0 = (tile / nbn) * BM, n0 = (tile % nbn) * BN;
            if (EPI == 2) break;  // one tile per block (host): staged epilogue after the loop
            epilogue<FN, FM, EPI>(a, acc, n0 + wn * TN + (lane >> 4) * 4, m0 + wm * TM + fr, lane, st);
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            kt = 0;
            ++tj;
        } else {
            ++kt;
        }
        if (has_next) store_stage(buf ^ 1);
        __syncthreads();
    }
    if (EPI == 2) {
        __syncthreads();
        const int m0 = (lid / nbn) * BM, n0 = (lid % nbn) * BN;
        epilogue_lds<BM, BN, 256, FN, FM>(a, acc, smem, m0, n0, wm * TM, wn * TN, lane, tid, st);
    }
}

template <typename KernelT>
int resident_blocks(KernelT kern, size_t lds, int threads = 256) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    return per_cu * cus;
}

// LDS bytes the staged epilogue needs: the bf16 tile, then the statistics fold
inline size_t epi_lds_bytes(int BM, int BN, int NT) {
    const size_t tile = (size_t)BM * BN * 2;
    const size_t red = (size_t)3 * 8 * epi_red_stride(BN, NT) * sizeof(float);
    return std::max(tile, red);
}

// persistent only where it pays: tiles with few K-stages (memory-bound 1x1
// convs) overlap the next tile's loads with this tile's epilogue; long-K tiles
// keep one tile per block (the hardware refills CUs without a tail)
inline int grid_size(int ntiles, int nk, int resident) {
    return (nk > 4 || ntiles < resident) ? ntiles : resident;
}

template <int BM, int BN, int WN, int NS, int MD, int NW = 4, int EPI = 0, int EB = 2, int FB = 0,
          int RB = 128>
int launch_dma(const IGemmArgs& a, hipStream_t st) {
    const int ntiles = ((a.M + BM - 1) / BM) * ((a.Nout + BN - 1) / BN);
    size_t lds = (size_t)NS * (BM + BN) * RB;
    if (EPI == 2) lds = std::max(lds, epi_lds_bytes(BM, BN, NW * 64));
    static int resident = 0;
    if (resident == 0)
        resident = resident_blocks(igemm_dma_kernel<BM, BN, WN, NS, MD, NW, EPI, EB, FB, RB>, lds, NW * 64);
    const int nk = (a.nth * a.ntw * a.C * EB + RB - 1) / RB;
    hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, WN, NS, MD, NW, EPI, EB, FB, RB>),
                       dim3(EPI == 2 ? ntiles : grid_size(ntiles, nk, resident)), dim3(NW * 64), lds, st, a);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

template <int BM, int BN, int WN, int MD, int EPI = 0>
int launch_rs(const IGemmArgs& a, hipStream_t st) {
    const int ntiles = ((a.M + BM - 1) / BM) * ((a.Nout + BN - 1) / BN);
    size_t lds = (size_t)2 * (BM + BN) * LDK * sizeof(bf16_t);
    if (EPI == 2) lds = std::max(lds, epi_lds_bytes(BM, BN, 256));
    static int resident = 0;
    if (resident == 0) resident = resident_blocks(igemm_rs_kernel<BM, BN, WN, MD, EPI>, lds);
    const int K = MD == 2 ? a.nth * 32 : a.nth * a.ntw * a.C;
    hipLaunchKernelGGL((igemm_rs_kernel<BM, BN, WN, MD, EPI>),
                       dim3(EPI == 2 ? ntiles : grid_size(ntiles, (K + BK - 1) / BK, resident)),
                       dim3(256), lds, st, a);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

}  // namespace

// fp8 paths live in their own translation unit (conv_igemm_fp8.hip) so the
// two halves of the kernel set compile in parallel
int conv_igemm_fp8(const IGemmArgs& a, int tile, hipStream_t st);
// short-K (C in {64, 128}) 1x1 convolutions as an HBM stream (conv_stream.hip);
// returns 1 when the shape / flags are not covered
int conv_stream(const IGemmArgs& a, hipStream_t st, int bn = 0);
int conv_stem(const IGemmArgs& a, hipStream_t st, int tile);
// 64 -> 64 3x3 stride-1 convs (fwd and dgrad) with weights and an input halo patch resident in
// LDS (conv_halo.hip); returns 1 when the shape / flags are not covered
int conv_halo(const IGemmArgs& a, hipStream_t st);
