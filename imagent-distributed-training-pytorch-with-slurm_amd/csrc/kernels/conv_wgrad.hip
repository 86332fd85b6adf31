// MFMA implicit-GEMM weight gradient, NHWC bf16 in, fp32 out, for gfx950.
//
// Replaces cuDNN's conv wgrad that the reference runs inside
// loss.backward() (/root/reference/imagenet.py:128), and fuses the DDP
// bucket copy-in (K20): the fp32 result is accumulated straight into the
// parameter's slot of the flat gradient arena that the RCCL all-reduce reads.
//
//   dW[co][tap*Ci + ci] += sum_m dY[m][co] * X[gather(m, tap)][ci]
//   m = (img, oh, ow) over the conv's output grid, gather = forward gather.
//
// The reduction runs over the pixel index m (up to 12.8 M rows), which is the
// OUTER (row) index of both NHWC operands. Tiles are staged row-major in LDS
// ([m][channel]) with 16-B register-staged writes and consumed with gfx950's
// transposing LDS read ds_read_b64_tr_b16 (cdna_hip_programming.md T10), so
// no operand ever has to be transposed in memory. The k (= m) order inside an
// MFMA fragment is permuted identically for both operands so that each
// 32-lane half reads 8 CONSECUTIVE rows: with a 288-B row pitch (256 + 32)
// those rows fall in disjoint 8-bank windows -> conflict-free reads.
//
// Split-K over m fills the chip (tiles x splits ~ 2-4 blocks per CU); partial
// tiles are added with no-return fp32 atomics in 64-B row segments (the
// chip-wide atomic rate, ~1.3 TB/s, is far above what these tiles need).
// Index math for the gather uses host-computed magic-number division.

#include <cstdlib>

#include "common.h"

struct WgradArgs {
    const bf16_t* dY;  // [M][Co]  (NHWC of the conv output)
    const bf16_t* X;   // NHWC [N][H][W][Ci]
    float* dW;         // [Co][KH*KW*Ci] fp32, accumulated (+=)
    int N, H, W, Ci, Co;
    int OH, OW, M;
    int KH, KW, stride, pad;
    int m_per_split;   // multiple of BR
    uint32_t mg_ohw, sh_ohw, mg_ow, sh_ow;  // magic division by OH*OW and OW
    int stem;          // bit 0: C == 4 row-segment gather, dW is [Co][KH][32]
    // the X operand is relu(X * xbn[c] + xbn[Ci + c]) (BatchNorm apply + ReLU of the conv's input,
    // never materialised: ops/block.py); out-of-image taps stay 0
    const float* xbn;
};

namespace {


__device__ __forceinline__ uint32_t fdiv(uint32_t n, uint32_t mg, uint32_t sh) {
    return (uint32_t)(((uint64_t)__umulhi(n, mg) + n) >> sh);
}

// NW waves per block: 4 (two blocks per CU) or 8 (one 256x256 block per CU:
// half the operand bytes per MFMA FLOP of a 128x128 tile)
// BR: pixels (reduction rows) per stage -- 64, or 32 (half the LDS: three
// 4-wave blocks per CU instead of two, more waves to hide the load latency)
// XB: the X operand gets the BatchNorm apply + ReLU of a.xbn while it is staged
template <int BCO, int BKC, int WCO, bool STEM, int NW = 4, int BR = 64, bool XB = false>
__global__ __launch_bounds__(NW * 64, NW == 4 ? (BR == 32 ? 3 : 2) : 1) void wgrad_kernel(const WgradArgs a) {
    constexpr int NT = NW * 64;
    constexpr int WKC = NW / WCO;
    constexpr int TCO = BCO / WCO, TKC = BKC / WKC;
    constexpr int FN = TCO / 16, FM = TKC / 16;
    constexpr int PCO = BCO * 2 + 32, PKC = BKC * 2 + 32;   // LDS row pitch, bytes
    constexpr int CPR_D = BCO / 8, CPR_X = BKC / 8;         // 16-B chunks per row
    constexpr int D_CH = BR * CPR_D / NT, X_CH = BR * CPR_X / NT;
    static_assert(D_CH >= 1 && X_CH >= 1 && NT % CPR_D == 0 && NT % CPR_X == 0, "staging split");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sD = smem;                      // [2][BR][PCO]
    char* sX = smem + 2 * BR * PCO;       // [2][BR][PKC]

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wco = wid % WCO, wkc = wid / WCO;
    const int K = STEM ? a.KH * 32 : a.KH * a.KW * a.Ci;
    const int nco = (a.Co + BCO - 1) / BCO, nkc = (K + BKC - 1) / BKC;
    const int ntiles = nco * nkc;
    const int bid = blockIdx.x;
    const int tile = bid % ntiles, split = bid / ntiles;  // splits of one tile on one XCD group
    const int tco = tile % nco, tkc = tile / nco;
    const int co0 = tco * BCO, kc0 = tkc * BKC;
    const int mbeg = split * a.m_per_split;
    const int mend = min(a.M, mbeg + a.m_per_split);
    if (mbeg >= mend) return;
    const int nst = (mend - mbeg + BR - 1) / BR;

    // fixed per-thread column chunk info
    // dY chunks: id = tid + 256*i -> row id / CPR_D, col id % CPR_D (col fixed iff 256 % CPR_D == 0)
    const int dcol = tid % CPR_D;
    const int dco = co0 + dcol * 8;
    const bool dco_ok = dco < a.Co;
    const int xcol = tid % CPR_X;
    const int xk = kc0 + xcol * 8;
    const bool xk_ok = xk < K;
    int xci, xdh, xdw, xkw0 = 0;
    if (STEM) {  // column = kh*32 + kw*4 + c
        const int kh = xk / 32, seg = xk - kh * 32;
        xkw0 = seg >> 2;
        xci = 0;
        xdh = kh - a.pad;
        xdw = xkw0 - a.pad;
    } else {
        const int xtap = xk_ok ? xk / a.Ci : 0;
        xci = xk - xtap * a.Ci;
        const int xkh = xtap / a.KW, xkw = xtap - xkh * a.KW;
        xdh = xkh - a.pad;
        xdw = xkw - a.pad;
    }

    // XB: this thread's 8 X channels are fixed (xci): their BN scale / shift stay in registers
    float bsc[8], bsh[8];
    if (XB) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int c = xk_ok ? xci + k : 0;
            bsc[k] = a.xbn[c];
            bsh[k] = a.xbn[a.Ci + c];
        }
    }
    bool xok[XB ? X_CH : 1];  // XB: the row exists (padding rows stay 0, not relu(shift))
    u32x4 rd[D_CH], rx[X_CH];
    auto load = [&](int st) {
        const int mb = mbeg + st * BR;
#pragma unroll
        for (int i = 0; i < D_CH; ++i) {
            const int row = (tid + NT * i) / CPR_D;
            const int m = mb + row;
            u32x4 v = {0, 0, 0, 0};
            if (m < mend && dco_ok) v = *reinterpret_cast<const u32x4*>(a.dY + (size_t)m * a.Co + dco);
            rd[i] = v;
        }
#pragma unroll
        for (int i = 0; i < X_CH; ++i) {
            const int row = (tid + NT * i) / CPR_X;
            const int m = mb + row;
            u32x4 v = {0, 0, 0, 0};
            if (XB) xok[i] = false;
            if (m < mend && xk_ok) {
                const uint32_t img = fdiv((uint32_t)m, a.mg_ohw, a.sh_ohw);
                const uint32_t rem = (uint32_t)m - img * (uint32_t)(a.OH * a.OW);
                const uint32_t oh = fdiv(rem, a.mg_ow, a.sh_ow);
                const uint32_t ow = rem - oh * (uint32_t)a.OW;
                const int ih = (int)oh * a.stride + xdh, iw = (int)ow * a.stride + xdw;
                if (STEM) {
                    if ((unsigned)ih < (unsigned)a.H) {
                        const bf16_t* p = a.X + (((long)img * a.H + ih) * a.W + iw) * 4;
                        u32x2 lo = {0, 0}, hi = {0, 0};
                        if (xkw0 < a.KW && (unsigned)iw < (unsigned)a.W) lo = *reinterpret_cast<const u32x2*>(p);
                        if (xkw0 + 1 < a.KW && (unsigned)(iw + 1) < (unsigned)a.W)
                            hi = *reinterpret_cast<const u32x2*>(p + 4);
                        v = u32x4{lo[0], lo[1], hi[0], hi[1]};
                    }
                } else if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W) {
                    v = *reinterpret_cast<const u32x4*>(a.X + (((size_t)img * a.H + ih) * a.W + iw) * a.Ci + xci);
                    if (XB) xok[i] = true;
                }
            }
            rx[i] = v;
        }
    };
    auto store = [&](int buf) {
        char* d = sD + buf * BR * PCO;
        char* x = sX + buf * BR * PKC;
#pragma unroll
        for (int i = 0; i < D_CH; ++i) {
            const int id = tid + NT * i;
            *reinterpret_cast<u32x4*>(d + (id / CPR_D) * PCO + (id % CPR_D) * 16) = rd[i];
        }
#pragma unroll
        for (int i = 0; i < X_CH; ++i) {
            const int id = tid + NT * i;
            u32x4 v = rx[i];
            if (XB) {  // y = relu(x * scale + shift), rounded to bf16 as the BN pass would have stored it
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    v[k] = xok[i] ? pack_bf2(fmaxf(fmaf(lo_bf(rx[i][k]), bsc[2 * k], bsh[2 * k]), 0.f),
                                             fmaxf(fmaf(hi_bf(rx[i][k]), bsc[2 * k + 1], bsh[2 * k + 1]), 0.f))
                                  : 0u;
            }
            *reinterpret_cast<u32x4*>(x + (id / CPR_X) * PKC + (id % CPR_X) * 16) = v;
        }
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // tr-read lane addressing: 16-lane group g, lane 4q+p -> row q, cols 4p..4p+3.
    // Fragment element e (0..7) of group g holds pixel row
    //   e<4: 4g + e          e>=4: 16 + 4g + (e-4)     (same for both operands)
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int row_a = 4 * g + q;          // first read
    const int row_b = 16 + 4 * g + q;     // second read

    load(0);
    store(0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) load(st + 1);
        const char* d = sD + buf * BR * PCO;
        const char* x = sX + buf * BR * PKC;
#pragma unroll
        for (int ks = 0; ks < BR / 32; ++ks) {
            bf16x8 fd[FN], fx[FM];
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int col = wco * TCO + i * 16 + 4 * p;
                const char* base = d + (ks * 32) * PCO + col * 2;
                s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_PTR(s16x4))(base + row_a * PCO));
                s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_PTR(s16x4))(base + row_b * PCO));
                fd[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int col = wkc * TKC + j * 16 + 4 * p;
                const char* base = x + (ks * 32) * PKC + col * 2;
                s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_PTR(s16x4))(base + row_a * PKC));
                s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_PTR(s16x4))(base + row_b * PKC));
                fx[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[i], fx[j], acc[i][j], 0, 0, 0);
        }
        if (st + 1 < nst) store(buf ^ 1);
        __syncthreads();
    }

    // acc[i][j][r]: co = co0 + wco*TCO + i*16 + (lane>>4)*4 + r ; k = kc0 + wkc*TKC + j*16 + (lane&15)
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = co0 + wco * TCO + i * 16 + (lane >> 4) * 4 + r;
            if (co >= a.Co) continue;
            float* dst = a.dW + (size_t)co * K;
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int k = kc0 + wkc * TKC + j * 16 + (lane & 15);
                if (k < K) atomicAdd(dst + k, acc[i][j][r]);
            }
        }
}

}  // namespace

#include "conv_wgrad_v3.h"
#include "conv_wgrad_stem.h"
#include "conv_wgrad_halo.h"

namespace {

template <int BCO, int BKC, int WCO, bool STEM, int NW = 4, int BR = 64, bool XB = false>
int launch1(WgradArgs a, int splits, hipStream_t st) {
    const int K = STEM ? a.KH * 32 : a.KH * a.KW * a.Ci;
    const int ntiles = ((a.Co + BCO - 1) / BCO) * ((K + BKC - 1) / BKC);
    if (splits <= 0) {
        // ~3 blocks per CU over 256 CUs (4-wave blocks, 2 resident per CU) or
        // ~2 (8-wave blocks, 1 resident), at least 4 stages per block
        // measured (conv_bench, R50 at 1024 img): the stem and the <= 128-channel 3x3 convs
        // (few tiles, latency-bound staging) gain from 4-5 blocks per CU (stem 1108 -> 944 us,
        // 64@56 3x3 630 -> 577, 128@28 3x3 502 -> 461); 1x1 convs lose (more split-K atomics)
        int target = NW == 4 ? 768 : 512;
        if (NW == 4 && STEM) target = 1280;
        else if (NW == 4 && a.KH * a.KW > 1 && a.Ci <= 128) target = 1024;
        const int want = (target + ntiles - 1) / ntiles;
        const int maxs = (a.M + 4 * BR - 1) / (4 * BR);
        splits = max(1, min(want, maxs));
    }
    int mps = (a.M + splits - 1) / splits;
    mps = (mps + BR - 1) / BR * BR;
    splits = (a.M + mps - 1) / mps;
    a.m_per_split = mps;
    const size_t lds = (size_t)2 * BR * ((BCO * 2 + 32) + (BKC * 2 + 32));
    hipLaunchKernelGGL((wgrad_kernel<BCO, BKC, WCO, STEM, NW, BR, XB>), dim3(ntiles * splits), dim3(NW * 64), lds,
                       st, a);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

// Stage depth by shape (measured, 1x MI355X, R50 @ 512 img): 32-row stages win
// on 1x1 convs, the stem and 64-channel tiles (-8..-20 %), 64-row stages on
// the 3x3 convs with 128x128 tiles (-15..-25 % vs 32).
template <int BCO, int BKC, int WCO, bool STEM>
int launch(WgradArgs a, int splits, hipStream_t st) {
    const bool br32 = STEM || BCO == 64 || a.KH * a.KW == 1;
    if constexpr (!STEM) {
        if (a.xbn)  // BN apply + ReLU of X on the staging path (padding taps stay 0)
            return br32 ? launch1<BCO, BKC, WCO, STEM, 4, 32, true>(a, splits, st)
                        : launch1<BCO, BKC, WCO, STEM, 4, 64, true>(a, splits, st);
    }
    return br32 ? launch1<BCO, BKC, WCO, STEM, 4, 32>(a, splits, st)
                : launch1<BCO, BKC, WCO, STEM, 4, 64>(a, splits, st);
}

}  // namespace

IMK_EXPORT int imk_conv_wgrad(const WgradArgs* args, int splits, void* stream) {
    const WgradArgs& a = *args;
    if (a.M <= 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if ((a.stem & 1) && a.xbn) return -110;
    if (a.stem & 1) {
        if (a.Ci != 4 || a.KW > 8 || a.Co % 8) return -102;
        // the 224-px 7x7 stem: the band kernel (conv_wgrad_stem.h; in-step 16,856 / 16,883 vs 16,738 / 16,756 img/s
        // with the register-staged stem loop below, same box)
        if (stem_wgrad_band_ok(a)) return launch_stem_wgrad_band(a, st);
        return launch<64, 128, 1, true>(a, splits, st);
    }
    if (a.Ci % 8 || a.Co % 8) return -100;
    // LDS-DMA main loop (conv_wgrad_v3.h) for the 1x1 convs it covers (conv_bench at 1024 img: 1x1
    // wgrads -790 us per step in total, e.g. 512 -> 256 @28 457 -> 325 us; on 3x3 the register-staged
    // kernel stays ahead, 128 @28 452 vs 497). IMAGENT_WGRAD_V3 = 0 off, 1: 1x1 with 64-row stages x 2, 2: 64 x 3,
    // 3: 32 x 4, 4: 128 x 2, 5: 64 x 2 for every shape it covers, 6 (default): 1x1 and the 3x3 shapes the halo kernel
    // below does not take (stride 2, 7x7 maps) instead of the register-staged loop. Isolated, the register-staged loop
    // is 4-15 % ahead on those 3x3 shapes (round 5, below); in-step on the side stream the LDS-DMA loop wins: 4096 img
    // 17,276 / 17,257 -> 17,354 / 17,330 img/s, 256 img 13,535 -> 13,567 (round 6, scripts/runs/wgv3_ab.sh, every
    // production shape's numerics in tests/test_conv_shapes_gpu.py)
    static const int v3 = [] {
        const char* e = getenv("IMAGENT_WGRAD_V3");
        return e ? atoi(e) : 6;
    }();
    static const int halo_mode = [] {  // IMAGENT_WGRAD_HALO, see the halo-kernel branch below
        const char* e = getenv("IMAGENT_WGRAD_HALO");
        return e ? atoi(e) : 2;
    }();
    // 6 also takes the 256 x 256 tile (16 waves, one block per CU, its own split count) when the step is large:
    // at least IMAGENT_WGRAD_WIDE_MIN_IMAGES images per GPU (default 2048); 7 (A/B): wherever it covers the shape.
    // In-step, one box each (scripts/runs/wgv7_ab.sh, wide_ab.sh): everywhere at 4096 img 17,419 / 17,392 ->
    // 17,672 / 17,702 img/s and 17,533 -> 17,786 / 17,782; at 256 img 13,510 -> 13,171, by a per-shape row bound
    // (>= 200,704 pixels: layers 1-2 at 256 img) 13,435 / 13,448 -> 13,386 / 13,390 -- the 128-KB blocks keep the
    // small main-stream kernels of a small step from co-residing (round 5's note above imk_conv_wgrad_variant), so
    // the bound is on the step size; at 2048 img round 5 measured the tile neutral in-step
    static const long wide_min = [] {
        const char* e = getenv("IMAGENT_WGRAD_WIDE_MIN_IMAGES");
        return e ? atol(e) : 2048L;
    }();
    const bool v3_rest = (v3 == 6 || v3 == 7) && !(halo_mode && wgrad_halo_ok(a, halo_mode >= 2, true));
    if (v3 && wgrad_v3_ok(a) && (v3 == 5 || v3_rest || (a.KH == 1 && a.KW == 1))) {
        if ((v3 == 7 || (v3 == 6 && (long)a.N >= wide_min)) && wgrad_v3w_ok<4, 4>(a))
            return launch_wgrad_v3<64, 2, 4, 4>(a, 0, st);
        switch (v3) {
            case 2: return launch_wgrad_v3<64, 3>(a, splits, st);
            case 3: return launch_wgrad_v3<32, 4>(a, splits, st);
            case 4: return launch_wgrad_v3<128, 2>(a, splits, st);
            default: return launch_wgrad_v3<64, 2>(a, splits, st);
        }
    }
    // 3x3 stride-1 with 64-channel slices: the halo-tiled kernel (conv_wgrad_halo.h); IMAGENT_WGRAD_HALO=0 off,
    // 1 only 64 -> 64, 2 (default) every shape it covers
    const int halo = halo_mode;  // (read once above)
    if (halo && wgrad_halo_ok(a, halo >= 2, true)) return launch_wgrad_halo(a, st);
    if (a.Co <= 64) return launch<64, 128, 1, false>(a, splits, st);
    // (an LDS-DMA ring variant with a 2*(row&7)-swizzled 256-B-row image measured
    // 2 % slower than this register-staged loop on every R50 shape: not kept)
    // (launch<256, 256, 2, false, 8> -- one 8-wave block per CU -- measured 23 %
    // slower in total: this register-staged loop needs two blocks per CU)
    // (round 5, 2048 img, 3x3 stride 2 / 7x7: the LDS-DMA loop waits on its fills -- SQ_WAIT_ANY 44 % of wave
    // cycles vs 22 % here, scripts/pmc_wgrad.sh; deeper rings cost blocks per CU and run slower still, 32-row
    // stages x 2 at four blocks per CU come within 4 % on 512 @7 and stay 5-15 % behind on the stride-2 shapes)
    return launch<128, 128, 2, false>(a, splits, st);
}

// explicit kernel choice (tests, A/B): -1 the register-staged kernel, -2 the stem's register-staged kernel, 1..4
// the v3 variants of IMAGENT_WGRAD_V3 and 6 its 256 x 256 tile (-106 when the shape is not one v3 covers), 9 the
// halo-tiled 64 -> 64 3x3 kernel, 0 the default dispatch (the band kernel for the 224-px stem)
IMK_EXPORT int imk_conv_wgrad_variant(const WgradArgs* args, int splits, int variant, void* stream) {
    const WgradArgs& a = *args;
    if (variant == 0) return imk_conv_wgrad(args, splits, stream);
    if (a.M <= 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (variant == -2) {  // the stem's register-staged kernel (A/B against the band kernel)
        if (!(a.stem & 1) || a.Ci != 4 || a.KW > 8 || a.Co % 8) return -106;
        return launch<64, 128, 1, true>(a, splits, st);
    }
    if (variant < 0) {
        if (a.stem || a.xbn || a.Ci % 8 || a.Co % 8) return -106;
        return a.Co <= 64 ? launch<64, 128, 1, false>(a, splits, st) : launch<128, 128, 2, false>(a, splits, st);
    }
    if (variant == 9) return wgrad_halo_ok(a) ? launch_wgrad_halo(a, st) : -106;
    if (!wgrad_v3_ok(a)) return -106;
    switch (variant) {
        case 1: return launch_wgrad_v3<64, 2>(a, splits, st);
        case 2: return launch_wgrad_v3<64, 3>(a, splits, st);
        case 3: return launch_wgrad_v3<32, 4>(a, splits, st);
        case 4: return launch_wgrad_v3<128, 2>(a, splits, st);
        // 256 x 256 tile on 16 waves, one block per CU (64-row stages x 2): isolated 1x1 wgrads at 2048 img 12-26 %
        // faster on the strided / 28x28 / 1024 -> 512 shapes, 2-4 % on the rest (32-row x 4 stages and the 8-wave
        // 128 x 256 / 256 x 128 tiles measured slower than the 128 x 128 tile); in-step neutral as the 1x1 default
        // (16,527 / 16,572 vs 16,522 / 16,542 img/s: its 128-KB blocks do not co-reside with the main stream's), so
        // not dispatched (scripts/wgrad_ab.py --set 1x1, README round 5)
        case 6: return wgrad_v3w_ok<4, 4>(a) ? launch_wgrad_v3<64, 2, 4, 4>(a, splits, st) : -106;
        default: return -106;
    }
}

// G += h2^T h2 for an [M][p] bf16 h2 (the Gram-form bottleneck's Gram matrix, ops/bn_gram.py), p = 64 / 128, G fp32
// [p][p] accumulated: the v3 weight-gradient loop with ONE staged operand (SYM 1), for p = 64 on h2 viewed as
// [M / 2][128] pixel pairs whose Gram matrix's two diagonal quadrants sum to G (SYM 2). -106: not a shape this covers
IMK_EXPORT int imk_gram_sym(const void* h2, float* G, long M, int p, int splits, void* stream) {
    if ((p != 64 && p != 128) || M <= 0 || (p == 64 && M % 2)) return -106;
    WgradArgs a{};
    a.dY = a.X = static_cast<const bf16_t*>(h2);
    a.dW = G;
    const long rows = p == 64 ? M / 2 : M;
    if (rows > 0x7FFFFFFF) return -106;
    a.N = (int)rows;
    a.H = a.W = a.OH = a.OW = 1;
    a.M = (int)rows;
    a.Ci = a.Co = 128;
    a.KH = a.KW = a.stride = 1;
    a.pad = 0;
    hipStream_t st = (hipStream_t)stream;
    return p == 64 ? launch_wgrad_v3<64, 2, 2, 2, 2>(a, splits, st) : launch_wgrad_v3<64, 2, 2, 2, 1>(a, splits, st);
}

// the stem's weight gradient with its BatchNorm's backward apply fused in (conv_wgrad_stem.h BNX): dY = g, the ReLU-
// masked maxpool-backward gradient; bnx = the BN input; coef [3][64] = (A, B, c) of imk_bn_bwd_coef. -106: not the
// band kernel's shape
IMK_EXPORT int imk_stem_wgrad_bnx(const WgradArgs* args, const void* bnx, const float* coef, void* stream) {
    const WgradArgs& a = *args;
    if (!stem_wgrad_band_ok(a) || !bnx || !coef || a.OH % 2) return -106;
    return launch_stem_wgrad_band_bnx(a, (hipStream_t)stream, static_cast<const bf16_t*>(bnx), coef);
}

IMK_EXPORT int imk_wgrad_args_size() { return (int)sizeof(WgradArgs); }
