// Halo-tiled weight gradient of the 3x3 stride-1 convs with Ci, Co % 64 == 0 (ResNet-50 64@56, 128@28,
// 256@14, 512@7; cuDNN's conv wgrad inside loss.backward() in the reference, /root/reference/imagenet.py:128):
//   dW[co][t][ci] += sum_p dY[p][co] * X[p + shift(t)][ci],   t = 3 ti + tj.
//
// The generic wgrad kernels tile K = 9 x Ci into 128-wide k tiles, so every input pixel is gathered
// from L2 into LDS once per k tile it feeds, and the register-staged main loop measured 404 (64@56) to
// 640 (512@7) TFLOP/s (profiles/r50_b1024_conv_shapes_v14.txt). Here, as in the forward halo kernel
// (conv_halo.hip), a band of R output rows of one image (R x W pixels, padded to NKS x 32 with zero
// dY rows) is staged ONCE per (64-channel co slice, 64-channel ci slice) of the block:
//   * dY band  [NKS*32 px][64 co] and the X patch [(R + 2) rows][PW px][64 ci] (band + 1-pixel halo,
//     out-of-image pixels as zeros) land in LDS by LDS-DMA through buffer descriptors (out-of-range
//     offsets read zeros), double-buffered: band n + 1 streams in while band n computes;
//   * all 9 taps read the same patch as shifted windows;
//   * wave w owns input channels 16w .. 16w + 15 for all 64 output channels and all 9 taps
//     (36 accumulators of 16x16), so one k-step (32 pixels) is 4 dY fragments + 9 X fragments for
//     36 MFMAs (v_mfma_f32_16x16x32_bf16, k = pixels);
//   * fragments by ds_read_b64_tr_b16 (pixel rows -> k): a 32-lane half reads 8 consecutive pixel
//     rows; rows are 128 B with 32-B segment s of row q stored at s ^ ((q >> 1) & 3), conflict-free
//     for any 8 consecutive rows -- and because the patch pitch PW is a multiple of 8, shifting a
//     window by a tap ROW keeps every row's swizzle, so the 3 tap rows share one address and an
//     immediate offset (3 addresses per k-step and read instead of 9);
//   * a persistent block = (co slice, ci slice, contiguous range of bands); the slices of one band
//     range are consecutive block ids (one XCD: the band's dY / X rows are fetched from HBM once and
//     re-read from that L2); the 144 accumulators per lane leave with one fp32 atomic each into the
//     gradient arena at the end.
// Shapes (host): Ci, Co % 64 == 0, KH = KW = 3, stride 1, pad 1, no operand BN, (W, R) in
// {(56, 4), (28, 4), (14, 14), (7, 7)} with H % R == 0. Measured at R50 / batch 1024 (conv_bench): 64@56
// 585 -> 275 us, 128@28 462 -> 306, 256@14 402 -> 271 (870 TFLOP/s); 512@7 390 vs 364 for the
// register-staged kernel (2 k-steps per band, 23 % zero padding): not the default there.
//
// (A stride-2 form that staged the four phase planes of the input measured slower than the register-staged
// kernel on every R50 stride-2 shape -- 128@56 s2 501 vs 456 us, 256@28 620 vs 440, 512@14 461 vs 402 -- and
// was removed in round 5; profiles/r50_b1024_round4_kernel_ab.md.)

#pragma once

#include <algorithm>

#include "common.h"

namespace {

constexpr uint32_t WH_OOB = 0x80000000u;

__device__ __forceinline__ int wh_swz(int q) { return (q >> 1) & 3; }

// physical 16-B chunk slot of logical chunk c (0..7) of row q (and its inverse: the map is an involution)
__device__ __forceinline__ int wh_slot(int c, int q) { return (((c >> 1) ^ wh_swz(q)) << 1) | (c & 1); }

template <int W, int R, int NKS, int PW>
__global__ __launch_bounds__(256, 1) void wgrad_halo_kernel(const WgradArgs a, int nbands, int nranges) {
    constexpr int BP = R * W;           // band pixels (NKS x 32 rows staged: the rest are zero dY rows)
    constexpr int PR = R + 2;           // patch rows
    constexpr int DYB = NKS * 32 * 128; // dY image bytes
    constexpr int PB = PR * PW * 128;   // patch image bytes
    constexpr int BUF = DYB + PB;
    constexpr int NDY = DYB / 1024, NP = NDY + PB / 1024;
    constexpr int PPW = (NP + 3) / 4;   // DMA pieces per wave per band
    static_assert(PW % 8 == 0 && W + 2 <= PW && BP <= NKS * 32 && NKS * 32 - BP < 32 &&
                      (PR * PW) % 8 == 0 && NP - 3 * PPW >= 0,
                  "band geometry");
    static_assert(2 * BUF <= 160 * 1024, "two band buffers in LDS");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nci = a.Ci / 64, npairs = (a.Co / 64) * nci;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int range = lid / npairs, pair = lid - range * npairs;
    const int co0 = (pair / nci) * 64, ci0 = (pair - (pair / nci) * nci) * 64;
    const int b0 = (int)((long)nbands * range / nranges), b1 = (int)((long)nbands * (range + 1) / nranges);
    if (b0 >= b1) return;  // whole block
    const int bpi = a.OH / R;
    const uint32_t ldy = (uint32_t)a.Co * 2, ldx = (uint32_t)a.Ci * 2;  // pixel pitches, bytes
    // descriptors based at the band's image (issue_band): 32-bit offsets for any batch size
    const size_t dall = (size_t)a.M * a.Co, xall = (size_t)a.N * a.H * a.W * a.Ci;

    // ---- DMA of band `band` into buffer `buf`: piece k of this wave = LDS rows 8k' .. 8k' + 7,
    // lane -> (row (lane >> 3), slot lane & 7), source chunk = slot's logical chunk
    const int drow = lane >> 3, dslot = lane & 7;
    auto issue_band = [&](int band, int buf) {
        const int img = band / bpi, y0 = (band - img * bpi) * R;
        const uint32_t pix0 = (uint32_t)(y0 * W);  // band's first (output) pixel within its image
        const size_t dimg = (size_t)img * a.OH * W * a.Co + co0, ximg = (size_t)img * a.H * a.W * a.Ci + ci0;
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<bf16_t*>(a.dY + dimg), (short)0, (int)min((dall - dimg) * 2, (size_t)0x7FFFFFFF), 0x00020000);
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<bf16_t*>(a.X + ximg), (short)0, (int)min((xall - ximg) * 2, (size_t)0x7FFFFFFF), 0x00020000);
#pragma unroll
        for (int k = 0; k < PPW; ++k) {
            const int piece = wid * PPW + k;
            if (piece >= NP) break;  // wave-uniform
            char* lds = smem + buf * BUF + piece * 1024;
            if (piece < NDY) {
                const int row = piece * 8 + drow;
                const uint32_t off = row < BP ? (pix0 + (uint32_t)row) * ldy + (uint32_t)(wh_slot(dslot, row) * 16)
                                              : WH_OOB;  // padded k rows: zeros
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (__attribute__((address_space(3))) void*)lds, 16, off, 0,
                                                         0, 0);
            } else {
                const int q = (piece - NDY) * 8 + drow;  // patch row index
                const int pr = q / PW, pc = q - pr * PW;
                const int iy = y0 - 1 + pr, ix = pc - 1;
                uint32_t off = WH_OOB;
                if ((unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                    off = ((uint32_t)iy * a.W + (uint32_t)ix) * ldx + (uint32_t)(wh_slot(dslot, q) * 16);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)lds, 16, off, 0,
                                                         0, 0);
            }
        }
    };

    // ---- fragment addresses (band-invariant, relative to the buffer base): lane 4q + p of its 16-lane
    // group reads row q of a 4-row block, columns 4p .. 4p + 3 of a 16-channel (32-B) segment; the
    // 32-lane half h reads rows 8 (2 r + h) + 4 g + q of k-step ks in read r (g = group within the half)
    const int h = lane >> 5, g = (lane >> 4) & 1, q4 = (lane >> 2) & 3, p4 = lane & 3;
    uint32_t adA[NKS][2][4], adB[NKS][2][3];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int P = ks * 32 + (2 * r + h) * 8 + 4 * g + q4;  // band pixel (row of the dY image)
#pragma unroll
            for (int i = 0; i < 4; ++i) adA[ks][r][i] = (uint32_t)(P * 128 + ((i ^ wh_swz(P)) << 5) + 8 * p4);
            const int Pp = P < BP ? P : 0;  // a padded k row (zero dY) reads any patch row: 0 x finite
            const int Q0 = (Pp / W) * PW + (Pp % W);  // patch row of tap (0, 0)
#pragma unroll
            for (int tj = 0; tj < 3; ++tj) {
                const int q = Q0 + tj;
                adB[ks][r][tj] = (uint32_t)(DYB + q * 128 + ((wid ^ wh_swz(q)) << 5) + 8 * p4);
            }
        }

    f32x4 acc[4][9];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

    issue_band(b0, 0);
    if (b0 + 1 < b1) issue_band(b0 + 1, 1);
    for (int band = b0; band < b1; ++band) {
        const int buf = (band - b0) & 1;
        // this band's pieces have landed (the next band's may still be in flight), in every wave
        constexpr int PPW0 = NP - 3 * PPW;  // wave 3's pieces per band (the others issue PPW)
        if (band + 1 < b1) {
            if (wid == 3)
                __builtin_amdgcn_s_waitcnt((PPW0 & 0xF) | ((PPW0 >> 4) << 14) | (0x7 << 4) | (0xF << 8));
            else
                __builtin_amdgcn_s_waitcnt((PPW & 0xF) | ((PPW >> 4) << 14) | (0x7 << 4) | (0xF << 8));
        } else
            __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
        __builtin_amdgcn_s_barrier();
        const char* base = smem + buf * BUF;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            bf16x8 fa[4], fb[9];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(base + adA[ks][0][i]));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(base + adA[ks][1][i]));
                fa[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
#pragma unroll
            for (int ti = 0; ti < 3; ++ti)
#pragma unroll
                for (int tj = 0; tj < 3; ++tj) {
                    const int toff = ti * PW * 128;  // tap row: the window shifted by ti patch rows
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (LDS_PTR(s16x4))(base + adB[ks][0][tj] + toff));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                        (LDS_PTR(s16x4))(base + adB[ks][1][tj] + toff));
                    fb[ti * 3 + tj] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
                }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int t = 0; t < 9; ++t)
                    acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[t], acc[i][t], 0, 0, 0);
        }
        // every wave is done reading this buffer before band + 2 overwrites it
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only (vmcnt 63, expcnt 7)
        __builtin_amdgcn_s_barrier();
        if (band + 2 < b1) issue_band(band + 2, buf);
    }

    // acc[i][t][r]: co = co0 + 16 i + 4 (lane >> 4) + r, k = t Ci + ci0 + 16 wid + (lane & 15)
    const int K = 9 * a.Ci;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float* dst = a.dW + (size_t)(co0 + 16 * i + 4 * (lane >> 4) + r) * K + ci0 + 16 * wid + (lane & 15);
#pragma unroll
            for (int t = 0; t < 9; ++t) atomicAdd(dst + t * a.Ci, acc[i][t][r]);
        }
}

// the shapes this kernel covers (host); wide = false: only 64 -> 64 (IMAGENT_WGRAD_HALO=1, A/B); dflt: the
// shapes the default dispatch gives it
inline bool wgrad_halo_ok(const WgradArgs& a, bool wide = true, bool dflt = false) {
    if (a.stem || a.xbn) return false;
    if (a.Ci % 64 || a.Co % 64 || a.KH != 3 || a.KW != 3 || a.pad != 1) return false;
    if (a.stride != 1) return false;
    if (!wide && (a.Ci != 64 || a.Co != 64)) return false;
    if (a.OW != a.W || a.OH != a.H) return false;
    // (W 7 is covered -- variant 9, tests -- but not taken by default: 2 k-steps per band with 23 % padding measured
    // 390 vs 364 us for the register-staged kernel at R50 512@7, batch 1024)
    const bool geo = (a.W == 56 && a.H % 4 == 0) || (a.W == 28 && a.H % 4 == 0) || (a.W == 14 && a.H % 14 == 0) ||
                     (a.W == 7 && a.H % 7 == 0 && !dflt);
    return geo && (size_t)a.H * a.W * a.Ci * 2 < (1ull << 31) && (size_t)a.OH * a.OW * a.Co * 2 < (1ull << 31);
}

template <int W, int R, int NKS, int PW>
int launch_wgrad_halo1(const WgradArgs& a, hipStream_t st) {
    const int nbands = a.N * (a.OH / R);
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
    }
    const int npairs = (a.Co / 64) * (a.Ci / 64);
    // ~one block per CU (LDS-bound residency), at least one band per range
    const int nranges = std::max(1, std::min(nbands, (cus + npairs - 1) / npairs));
    const size_t lds = 2 * ((size_t)NKS * 32 * 128 + (size_t)(R + 2) * PW * 128);
    hipLaunchKernelGGL((wgrad_halo_kernel<W, R, NKS, PW>), dim3(nranges * npairs), dim3(256), lds, st, a, nbands,
                       nranges);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

inline int launch_wgrad_halo(const WgradArgs& a, hipStream_t st) {
    switch (a.W) {
        case 56: return launch_wgrad_halo1<56, 4, 7, 64>(a, st);
        case 28: return launch_wgrad_halo1<28, 4, 4, 32>(a, st);
        case 14: return launch_wgrad_halo1<14, 14, 7, 16>(a, st);
        case 7: return launch_wgrad_halo1<7, 7, 2, 16>(a, st);
        default: return -106;
    }
}

}  // namespace
