// Weight gradient of the 7x7 / stride-2 stem (4 padded input channels -> 64) as a band kernel, gfx950 -- cuDNN's
// first-layer wgrad inside loss.backward() in the reference (/root/reference/imagenet.py:128, models.resnet50 :312).
//
//   dW[co][kh][t * 4 + c] += sum_p dY[p][co] X[img][2 oy + kh - 3][2 ox + t - 3][c]     (t = 0..7, tap 7 unused)
//
// The register-staged wgrad_kernel gathered two 8-B pieces per tap row per pixel (each input pixel feeds ~12
// output pixels) and ran at 266 TFLOP/s, 1.8 ms per call at 2048 img (profiles/r50_b2048_r5_conv_shapes.md). Here a
// persistent block stages a band -- R output rows of dY (R x 112 pixels x 64 channels) and the 2R + 5 input rows
// they read (as the forward's stem_band_kernel: 232-pixel rows with zero padding columns) -- in LDS ONCE, and
// every MFMA operand is a transposing LDS read (ds_read_b64_tr_b16, cdna_hip_programming.md T10) whose per-lane
// row address is the pixel's own: for dY the pixel's 128-B channel row, for X the pixel's window start in the
// staged input row (a kernel row's taps are contiguous there, 8 B each). Reduction = pixels (MFMA k = 32 pixels
// of the band), so no operand is ever transposed in memory.
//  * wave w owns kernel rows 2w, 2w + 1 (wave 3: row 6): 4 channel fragments x 2 rows x 2 tap halves = 16
//    accumulators, summed over all of its bands in registers, one fp32 atomic per element at the end;
//  * the next band is loaded into registers while the current one computes, then stored over it; R = 4 output rows
//    per band (80 KB: two blocks fill the CU's LDS) -- 1,054 us at 2048 img against 1,171 with R = 2 (the loop waits
//    on the next band's loads; more bytes in flight per block is what moves it);
//  * dY rows are XOR-swizzled by 16-B chunk so the 4 pixel rows x 2 lane groups of a 32-lane half hit distinct
//    banks (rows 0/2/8/10 and 1/3/9/11 of a k-step take different chunk pairs).
// The padded input channel (3) is zero, so its gradient is; tap 7's column is never added (stem_grad_fold reads
// taps 0..6, channels 0..2 only).

#pragma once

#include "common.h"

namespace {

constexpr int SWG_W = 224, SWG_OW = 112;
constexpr int SWG_SP = (SWG_W + 8) * 8;  // staged input row pitch, bytes (column c at byte (c + 4) * 8)

__device__ __forceinline__ int swg_swz(int row) { return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1; }

// BNX: the stem BatchNorm's backward apply fused into the staging -- a.dY is the ReLU-masked upstream gradient g
// (maxpool backward), bnx the BN input x, coef [3][64] = (A, B, c): the staged dY is bf16(A g + B x + c), what the
// apply pass would have stored, so the apply pass (read g and x, write dx) disappears
template <int R, bool BNX = false>
__global__ __launch_bounds__(256, 2) void stem_wgrad_band_kernel(const WgradArgs a, int nbands,
                                                                 const bf16_t* __restrict__ bnx,
                                                                 const float* __restrict__ coef) {
    constexpr int KH = 7;
    constexpr int PR = 2 * R + KH - 2;       // staged input rows per band
    constexpr int XB = PR * SWG_SP;          // X bytes in LDS
    constexpr int NPX = R * SWG_OW;          // pixels per band
    constexpr int NKS = NPX / 32;            // MFMA k-steps per band
    constexpr int XCH = PR * (SWG_W / 2);    // 16-B chunks of the band's input rows (224 px x 8 B = 112 chunks)
    constexpr int DCH = NPX * 8;             // 16-B chunks of the band's dY (128-B pixel rows)
    constexpr int XPT = (XCH + 255) / 256, DPT = (DCH + 255) / 256;
    static_assert(NPX % 32 == 0, "whole k-steps per band");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sX = smem;
    char* sD = smem + XB;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bpi = a.OH / R;  // bands per image (host: OH % R == 0)

    for (int e = tid; e < XB / 16; e += 256) reinterpret_cast<u32x4*>(smem)[e] = u32x4{0u, 0u, 0u, 0u};

    u32x4 sx[XPT], sd[DPT], sb[BNX ? DPT : 1];
    // BNX: this thread's 16-B chunks are always channel chunk tid & 7 (256 threads, 8 chunks per pixel row)
    float ka[BNX ? 8 : 1], kb[BNX ? 8 : 1], kc[BNX ? 8 : 1];
    if constexpr (BNX) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int ch = (tid & 7) * 8 + j;
            ka[j] = coef[ch];
            kb[j] = coef[64 + ch];
            kc[j] = coef[128 + ch];
        }
    }
    auto load_band = [&](int band) {  // global -> registers
        const int img = band / bpi, oy0 = (band - img * bpi) * R;
        const int iy0 = 2 * oy0 - 3;
#pragma unroll
        for (int t = 0; t < XPT; ++t) {
            const int e = tid + 256 * t;
            const int r = e / (SWG_W / 2), c16 = e - r * (SWG_W / 2), iy = iy0 + r;
            const bool ok = e < XCH && (unsigned)iy < (unsigned)a.H;
            sx[t] = ok ? *reinterpret_cast<const u32x4*>(a.X + (((size_t)img * a.H + iy) * SWG_W) * 4 + c16 * 8)
                       : u32x4{0u, 0u, 0u, 0u};
        }
        const size_t d0 = ((size_t)img * a.OH + oy0) * SWG_OW * 64;
#pragma unroll
        for (int t = 0; t < DPT; ++t) {
            const int e = tid + 256 * t;
            sd[t] = e < DCH ? *reinterpret_cast<const u32x4*>(a.dY + d0 + (size_t)e * 8) : u32x4{0u, 0u, 0u, 0u};
            if constexpr (BNX)
                sb[t] = e < DCH ? *reinterpret_cast<const u32x4*>(bnx + d0 + (size_t)e * 8) : u32x4{0u, 0u, 0u, 0u};
        }
    };
    auto store_band = [&]() {  // registers -> LDS
#pragma unroll
        for (int t = 0; t < XPT; ++t) {
            const int e = tid + 256 * t;
            if (e < XCH) {
                const int r = e / (SWG_W / 2), c16 = e - r * (SWG_W / 2);
                *reinterpret_cast<u32x4*>(sX + r * SWG_SP + 32 + c16 * 16) = sx[t];
            }
        }
#pragma unroll
        for (int t = 0; t < DPT; ++t) {
            const int e = tid + 256 * t;
            if (e < DCH) {
                const int p = e >> 3, c = e & 7;
                u32x4 v = sd[t];
                if constexpr (BNX) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const float lo = fmaf(ka[2 * k], lo_bf(sd[t][k]), fmaf(kb[2 * k], lo_bf(sb[t][k]), kc[2 * k]));
                        const float hi =
                            fmaf(ka[2 * k + 1], hi_bf(sd[t][k]), fmaf(kb[2 * k + 1], hi_bf(sb[t][k]), kc[2 * k + 1]));
                        v[k] = pack_bf2(lo, hi);
                    }
                }
                *reinterpret_cast<u32x4*>(sD + p * 128 + ((c ^ swg_swz(p)) << 4)) = v;
            }
        }
    };

    f32x4 acc[4][2][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int h = 0; h < 2; ++h) acc[i][k][h] = f32x4{0.f, 0.f, 0.f, 0.f};

    // transposed-read lanes: group g = lane >> 4 supplies k-step pixels 8g + q (lo) and 8g + 4 + q (hi), columns
    // 4p .. 4p + 3 (q = (lane >> 2) & 3, p = lane & 3)
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int ks0 = min(2 * wid, KH - 1), ks1 = min(2 * wid + 1, KH - 1);  // (wave 3: row 6 twice, second unused)
    const bool two = 2 * wid + 1 < KH;

    int band = blockIdx.x;
    if (band < nbands) load_band(band);
    __syncthreads();  // the zero fill
    if (band < nbands) store_band();
    __syncthreads();
    for (; band < nbands; band += gridDim.x) {
        const int nxt = band + gridDim.x;
        if (nxt < nbands) load_band(nxt);  // in flight under this band's MFMAs
#pragma unroll 1
        for (int s = 0; s < NKS; ++s) {
            bf16x8 fd[4], fx[2][2];
            const int px0 = s * 32 + 8 * g + q, px1 = px0 + 4;
            // dY^T fragments: channel block i (16 channels), pixel rows px0 / px1
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int c = 2 * i + (p >> 1);
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_PTR(s16x4))(sD + px0 * 128 + ((c ^ swg_swz(px0)) << 4) + 8 * (p & 1)));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (LDS_PTR(s16x4))(sD + px1 * 128 + ((c ^ swg_swz(px1)) << 4) + 8 * (p & 1)));
                fd[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
            // X fragments: kernel row ks, taps 4h + p (4 channels each) of the pixel's window
            const int ry0 = px0 >= SWG_OW ? px0 / SWG_OW : 0, ox0 = px0 - ry0 * SWG_OW;
            const int ry1 = px1 >= SWG_OW ? px1 / SWG_OW : 0, ox1 = px1 - ry1 * SWG_OW;
            const char* b0 = sX + 2 * ry0 * SWG_SP + (2 * ox0 + 1 + p) * 8;
            const char* b1 = sX + 2 * ry1 * SWG_SP + (2 * ox1 + 1 + p) * 8;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int ks = k ? ks1 : ks0;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(b0 + ks * SWG_SP + h * 32));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(b1 + ks * SWG_SP + h * 32));
                    fx[k][h] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int k = 0; k < 2; ++k)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        acc[i][k][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[i], fx[k][h], acc[i][k][h], 0, 0, 0);
        }
        __syncthreads();  // every wave done reading this band
        if (nxt < nbands) store_band();
        __syncthreads();
    }
    // acc[i][k][h][r]: co = 16 i + 4 (lane >> 4) + r, column = 16 h + (lane & 15) of kernel row 2 wid + k
    const int col = lane & 15;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (k == 1 && !two) break;
        const int ks = 2 * wid + k;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h == 1 && col >= 12) continue;  // tap 7: no weight
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    atomicAdd(a.dW + ((size_t)(16 * i + 4 * (lane >> 4) + r) * KH + ks) * 32 + 16 * h + col,
                              acc[i][k][h][r]);
        }
    }
}

// the band stem wgrad's shapes: 4-channel 224-wide input, 7x7 / stride 2 / pad 3, 64 channels, dW [64][7][32]
bool stem_wgrad_band_ok(const WgradArgs& a) {
    return (a.stem & 1) && !a.xbn && a.Ci == 4 && a.Co == 64 && a.KH == 7 && a.KW == 7 && a.stride == 2 &&
           a.pad == 3 && a.W == SWG_W && a.OW == SWG_OW && a.OH % 4 == 0 && a.OH == (a.H + 1) / 2 && a.M > 0;
}

template <int R, bool BNX>
int launch_stem_wgrad_band_r(const WgradArgs& a, hipStream_t st, const bf16_t* bnx, const float* coef) {
    const size_t lds = (size_t)(2 * R + 5) * SWG_SP + (size_t)R * SWG_OW * 128;
    static int resident = 0;
    if (resident == 0) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, stem_wgrad_band_kernel<R, BNX>, 256, lds) != hipSuccess ||
            per_cu < 1)
            per_cu = 1;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
        resident = per_cu * cus;
    }
    const int nbands = a.N * (a.OH / R);
    hipLaunchKernelGGL((stem_wgrad_band_kernel<R, BNX>), dim3(std::min(nbands, resident)), dim3(256), lds, st, a, nbands,
                       bnx, coef);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

// R = 4 output rows per band: 80 KB of LDS, two blocks fill the CU; the fused-apply form prefetches g AND x in
// registers, which leaves room for R = 2 only
int launch_stem_wgrad_band(const WgradArgs& a, hipStream_t st) {
    return launch_stem_wgrad_band_r<4, false>(a, st, nullptr, nullptr);
}
int launch_stem_wgrad_band_bnx(const WgradArgs& a, hipStream_t st, const bf16_t* bnx, const float* coef) {
    return launch_stem_wgrad_band_r<2, true>(a, st, bnx, coef);
}

}  // namespace
