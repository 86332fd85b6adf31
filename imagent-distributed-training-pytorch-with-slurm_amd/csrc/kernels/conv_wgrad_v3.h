// Weight-gradient main loop v3 for gfx950 (MI355X): dW[co][tap*Ci + ci] += sum_m dY[m][co] X[g(m,tap)][ci]
// for Ci % 128 == 0 and Co % 128 == 0 (every R50 3x3 but 64 -> 64, the K >= 128 1x1 convs) -- cuDNN's
// conv wgrad inside loss.backward() in the reference (/root/reference/imagenet.py:128).
//
// Why a second kernel: the register-staged wgrad_kernel (conv_wgrad.hip) measured 21.5 % MFMA busy
// on 128@28 3x3 with 6.4 VALU instructions per MFMA (scripts/pmc_conv.sh): every operand chunk goes
// global -> VGPR -> LDS with a 64-bit address and, for X, two magic-number divisions per row and
// stage. Here both operands are LDS-DMA fills through BUFFER descriptors (as igemm_v3_kernel):
//  * dY rows are contiguous in m: the lane offset is fixed, the stage advance is one add, rows past
//    M fall outside the descriptor's range (zeros);
//  * a k-tile is ONE filter tap x 128 input channels (Ci % 128 == 0), so every X row of a stage
//    has the same tap shift: one gather (img, ih, iw) per row and stage, out-of-image taps as an
//    out-of-range offset (zeros) -- no zero line, no per-chunk address math;
//  * LDS image: plain 256-B rows, chunk ch of row r at slot ch ^ (((r&3)<<2) | ((r>>2)&3))
//    (cdna_hip_programming.md T10 image (b)); the DMA lane -> (row, chunk) map applies the XOR on
//    the source side, so a 1-KB DMA instruction fills 4 whole rows;
//  * fragments by the transposing LDS read ds_read_b64_tr_b16 (rows = pixels = MFMA k); a 32-lane
//    half reads two 4-row blocks 8 rows apart (conflict-free on image (b)); the pixel order inside a
//    fragment is permuted identically for both operands (the sum over m does not care);
//  * NS-deep ring, counted vmcnt + one s_barrier per stage, split-K over m with fp32 atomics into
//    the gradient arena (as wgrad_kernel), XCD-aware block order: the tiles of one m-range share
//    an XCD (and its L2).

#pragma once

#include "common.h"

namespace {

constexpr uint32_t WG3_OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wg3_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void wg3_dma(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ int wg3_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// BR: pixel rows per stage (multiple of 32); NS: ring depth. WCO x WKC waves of 64 x 64 over a (64 WCO) x (64 WKC)
// tile: 2 x 2 (128 x 128, two blocks per CU) or wider tiles of one block per CU (256 x 256: 16 waves), which fetch
// half the operand bytes per MFMA FLOP -- the L2 -> LDS path, not the MFMA, bounds the 128 x 128 tile. A tile
// wider than 128 channels is staged as 128-channel sub-images of the same 256-B-row layout (sub-image h: channels
// 128 h .. 128 h + 127 of every row of the stage), so the DMA pieces and the transposed reads are unchanged.
// SYM (the Gram matrix G = h2^T h2 of a Gram-form bottleneck, bn_gram.hip, X == dY): 1 -- one operand staged once and
// read as both fragments; 2 -- a 64-channel h2 viewed as [M / 2][128] rows of pixel PAIRS, whose 128 x 128 Gram
// matrix holds G in its two diagonal quadrants (even pixels + odd pixels): only the two diagonal waves compute, both
// adding into the same 64 x 64 output (row pitch 64)
template <int BR, int NS, int WCO = 2, int WKC = 2, int SYM = 0>
__global__ __launch_bounds__(WCO * WKC * 64, WCO * WKC == 4 ? 2 : 1) void wgrad_v3_kernel(const WgradArgs a) {
    static_assert(SYM == 0 || (WCO == 2 && WKC == 2), "symmetric forms: the 128 x 128 tile");
    constexpr int NW = WCO * WKC;
    constexpr int TCO = 64 * WCO, TK = 64 * WKC;
    constexpr int NSD = (TCO + 127) / 128, NSX = (TK + 127) / 128;  // 128-channel sub-images per operand
    constexpr int SI = BR * 256;          // bytes of one sub-image per stage
    constexpr int SBD = NSD * SI, SBX = NSX * SI;
    constexpr int PD = NSD * (BR / 4) / NW, PX = NSX * (BR / 4) / NW;  // 1-KB pieces per wave per stage
    static_assert(PD >= 1 && PX >= 1 && PD * NW == NSD * (BR / 4) && PX * NW == NSX * (BR / 4), "piece split");
    constexpr int LPS = SYM ? PD : PD + PX;  // DMA instructions per wave per stage
    constexpr int NKS = BR / 32;          // MFMA k-steps per stage
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sD = smem;
    char* sX = SYM ? smem : smem + NS * SBD;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wco = wid % WCO, wkc = wid / WCO;
    const int K = a.KH * a.KW * a.Ci;
    const int nco = (a.Co + TCO - 1) / TCO, nkc = (K + TK - 1) / TK;  // (Co / K = 64: one half-used tile, wgrad_v3_ok)
    const int ntiles = nco * nkc;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int tile = lid % ntiles, split = lid / ntiles;
    const int co0 = (tile % nco) * TCO, kc0 = (tile / nco) * TK;
    const int mbeg = split * a.m_per_split;
    if (mbeg >= a.M) return;
    const int mend = min(a.M, mbeg + a.m_per_split);
    const int nst = (mend - mbeg + BR - 1) / BR;
    const int tap = kc0 / a.Ci, ci0 = kc0 - tap * a.Ci;
    const int dh = tap / a.KW - a.pad, dw = tap % a.KW - a.pad;

    // descriptors: the column offset (co0 / ci0) in the base, so a row's offset is row * ld * 2 +
    // chunk * 16 and anything at or past row M (dY) is out of range. Both are based at the split's first row
    // (dY) / first image (X, or first row when dense), so the 32-bit offsets hold for any tensor size
    const int ohw = a.OH * a.OW;
    const bool dense = a.KH == 1 && a.KW == 1 && a.stride == 1 && a.pad == 0 && a.OH == a.H && a.OW == a.W;
    const size_t dro = (size_t)mbeg * a.Co;
    const __amdgpu_buffer_rsrc_t rd =
        wg3_rsrc(a.dY + dro + co0, (uint32_t)min(((size_t)a.M * a.Co - dro - co0) * 2, (size_t)0x7FFFFFFF));
    const int img0 = mbeg / ohw;
    const size_t xro = dense ? (size_t)mbeg * a.Ci : (size_t)img0 * a.H * a.W * a.Ci;
    const __amdgpu_buffer_rsrc_t rx = wg3_rsrc(
        a.X + xro + ci0, (uint32_t)min(((size_t)a.N * a.H * a.W * a.Ci - xro - ci0) * 2, (size_t)0x7FFFFFFF));

    // this lane's DMA slots: piece j of an operand = sub-image j / (BR / 4), rows 4 (j % (BR / 4)) .. + 3; the lane
    // takes row + prow and source chunk (lane & 15) ^ swz(row) of the sub-image's 128 channels
    const int prow = lane >> 4;
    uint32_t voffd[PD], rowx[PX], colx[PX];
#pragma unroll
    for (int q = 0; q < PD; ++q) {
        const int j = wid * PD + q, h = j / (BR / 4);
        const int r = (j % (BR / 4)) * 4 + prow;
        voffd[q] = (uint32_t)(r * a.Co * 2 + h * 256 + (((lane & 15) ^ wg3_swz(r)) << 4));
    }
#pragma unroll
    for (int q = 0; q < PX; ++q) {
        const int j = wid * PX + q, h = j / (BR / 4);
        const int r = (j % (BR / 4)) * 4 + prow;
        rowx[q] = (uint32_t)r;
        colx[q] = (uint32_t)(h * 256 + (((lane & 15) ^ wg3_swz(r)) << 4));
    }
    const uint32_t dstep = (uint32_t)(BR * a.Co * 2);

    int is = 0;
    auto issue = [&]() {
        if (is >= nst) return;
        const int buf = is % NS;
        char* dD = sD + buf * SBD + wid * PD * 1024;
        char* dX = sX + buf * SBX + wid * PX * 1024;
        const int mb = mbeg + is * BR;
#pragma unroll
        for (int q = 0; q < PD; ++q) wg3_dma(rd, dD + q * 1024, voffd[q] + (uint32_t)is * dstep);
#pragma unroll
        for (int q = 0; q < (SYM ? 0 : PX); ++q) {
            const int m = mb + (int)rowx[q];
            uint32_t off = WG3_OOB;
            if (dense) {
                if (m < mend) off = (uint32_t)(m - mbeg) * (uint32_t)(a.Ci * 2) + colx[q];
            } else if (m < mend) {
                const uint32_t img = fdiv((uint32_t)m, a.mg_ohw, a.sh_ohw);
                const uint32_t rem = (uint32_t)m - img * (uint32_t)ohw;
                const uint32_t oh = fdiv(rem, a.mg_ow, a.sh_ow);
                const uint32_t ow = rem - oh * (uint32_t)a.OW;
                const int ih = (int)oh * a.stride + dh, iw = (int)ow * a.stride + dw;
                if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
                    off = (((img - (uint32_t)img0) * (uint32_t)a.H + (uint32_t)ih) * (uint32_t)a.W + (uint32_t)iw) *
                              (uint32_t)(a.Ci * 2) + colx[q];
            }
            wg3_dma(rx, dX + q * 1024, off);
        }
        ++is;
    };
#pragma unroll
    for (int p = 0; p < NS - 1; ++p) issue();

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // transposed-read addressing: group g = lane >> 4 reads rows R1 + q and R1 + 16 + q
    // (R1 = (g & 1) * 8 + (g >> 1) * 4: a 32-lane half's two blocks 8 rows apart), columns
    // c0 + 4p .. +3 of chunk (c0 / 8 + (p >> 1)) ^ swz(row), byte 8 * (p & 1); the wave's 64 columns are half
    // (wco & 1) of sub-image wco >> 1
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int r1 = (g & 1) * 8 + (g >> 1) * 4 + q4, r2 = r1 + 16;
    int offa[4][2], offb[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int ca = (wco & 1) * 8 + 2 * i + (p4 >> 1), cb = (wkc & 1) * 8 + 2 * i + (p4 >> 1);
        const int sa = (wco >> 1) * SI, sb = (wkc >> 1) * SI;
        offa[i][0] = sa + r1 * 256 + ((ca ^ wg3_swz(r1)) << 4) + 8 * (p4 & 1);
        offa[i][1] = sa + r2 * 256 + ((ca ^ wg3_swz(r2)) << 4) + 8 * (p4 & 1);
        offb[i][0] = sb + r1 * 256 + ((cb ^ wg3_swz(r1)) << 4) + 8 * (p4 & 1);
        offb[i][1] = sb + r2 * 256 + ((cb ^ wg3_swz(r2)) << 4) + 8 * (p4 & 1);
    }

    for (int s = 0; s < nst; ++s) {
        if (is - 1 - s >= NS - 2)
            __builtin_amdgcn_s_waitcnt((((NS - 2) * LPS) & 0xF) | ((((NS - 2) * LPS) >> 4) << 14) | (0x7 << 4) |
                                       (0xF << 8));
        else
            __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
        __builtin_amdgcn_s_barrier();
        issue();
        const int buf = s % NS;
        const char* bD = sD + buf * SBD;
        const char* bX = sX + buf * SBX;
        if (kc0 + wkc * 64 >= K || co0 + wco * 64 >= a.Co) continue;  // (wave-uniform) past K / Co: never computed
        if (SYM == 2 && wco != wkc) continue;                           // off-diagonal quadrant of the pair Gram
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            bf16x8 fd[4], fx[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(bD + ks * 8192 + offa[i][0]));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(bD + ks * 8192 + offa[i][1]));
                fd[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(bX + ks * 8192 + offb[j][0]));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(bX + ks * 8192 + offb[j][1]));
                fx[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[i], fx[j], acc[i][j], 0, 0, 0);
        }
    }

    // acc[i][j][r]: co = co0 + wco*64 + i*16 + (lane>>4)*4 + r ; k = kc0 + wkc*64 + j*16 + (lane&15)
    if (kc0 + wkc * 64 >= K || co0 + wco * 64 >= a.Co) return;
    if constexpr (SYM == 2) {
        if (wco != wkc) return;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float* dst = a.dW + (size_t)(i * 16 + (lane >> 4) * 4 + r) * 64 + (lane & 15);
#pragma unroll
                for (int j = 0; j < 4; ++j) atomicAdd(dst + j * 16, acc[i][j][r]);
            }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float* dst = a.dW + (size_t)(co0 + wco * 64 + i * 16 + (lane >> 4) * 4 + r) * K + kc0 + wkc * 64 + (lane & 15);
#pragma unroll
            for (int j = 0; j < 4; ++j) atomicAdd(dst + j * 16, acc[i][j][r]);
        }
}

// shapes this kernel covers (host): one tap per 128-wide k tile, whole 128-channel co tiles,
// byte offsets of both operands below 2^31
// Ci = 64 1x1 (ResNet-50 layer1's conv3 / downsample wgrads, the Gram-form bn3's T = g^T h2 on the critical path):
// one k tile whose 256-B X rows span two pixels -- the second pixel's 64 channels land in columns 64..127, which
// the waves owning them skip (no MFMA, no store); the last row's overhang reads zeros past the descriptor's range
bool wgrad_v3_ok(const WgradArgs& a) {
    if (a.stem || a.xbn) return false;
    if (a.Co % 128 && !(a.Co == 64 && a.KH == 1 && a.KW == 1)) return false;  // (Co = 64: the same, on dY's rows)
    if (a.Ci % 128 && !(a.Ci == 64 && a.KH == 1 && a.KW == 1)) return false;
    // (descriptors based per split: one split's rows / images must stay below 2^31 bytes -- the launcher's
    // splits keep a split to a few thousand rows; one image bound here)
    if ((size_t)a.H * a.W * a.Ci * 2 * 8 >= (1u << 31) || (size_t)a.OH * a.OW * a.Co * 2 * 8 >= (1u << 31)) return false;
    return true;
}

// the wide tiles cover whole tiles only (one filter tap per k tile: Ci % TK == 0)
template <int WCO, int WKC>
bool wgrad_v3w_ok(const WgradArgs& a) {
    return wgrad_v3_ok(a) && a.Co % (64 * WCO) == 0 && a.Ci % (64 * WKC) == 0;
}

template <int BR, int NS, int WCO = 2, int WKC = 2, int SYM = 0>
int launch_wgrad_v3(WgradArgs a, int splits, hipStream_t st) {
    constexpr int TCO = 64 * WCO, TK = 64 * WKC;
    const int K = a.KH * a.KW * a.Ci;
    const int ntiles = ((a.Co + TCO - 1) / TCO) * ((K + TK - 1) / TK);
    if (splits <= 0) {
        // one wave of blocks over 256 CUs (two per CU for the 4-wave tile): the 1x1 wgrads are split-K streams whose
        // second, partial wave of blocks cost more than the extra atomics of deeper splits save (same-box bench:
        // 512 blocks 15,314 / 15,357 img/s, 768 15,291, 1024 15,287 / 15,303, 1536 15,282)
        // (16-wave tile: IMAGENT_WGRAD_WIDE_TARGET blocks, A/B -- fewer than one per CU leaves CUs to the main
        // stream's small kernels, which otherwise wait for a slot behind the one-block-per-CU side-stream grid; measured
        // at 4096 img: 256 17,899 / 17,805, 192 17,805 / 17,790, 128 17,749 / 17,755 img/s -- one per CU stays)
        static const int wide_target = [] {
            const char* e = getenv("IMAGENT_WGRAD_WIDE_TARGET");
            return e && atoi(e) > 0 ? atoi(e) : 256;
        }();
        const int target = WCO * WKC == 4 ? 512 : wide_target;
        const int want = (target + ntiles - 1) / ntiles;
        const int maxs = (a.M + 4 * BR - 1) / (4 * BR);
        splits = max(1, min(want, maxs));
    }
    int mps = (a.M + splits - 1) / splits;
    mps = (mps + BR - 1) / BR * BR;  // whole stages: a split's last stage never reads the next split's rows
    // a split's dY rows / X images addressed by 32-bit offsets from its own base (kernel): keep each below 2^31
    const size_t ohw = (size_t)a.OH * a.OW, img = (size_t)a.H * a.W * a.Ci * 2;
    while (mps > BR && ((size_t)mps * a.Co * 2 >= (1u << 31) || ((size_t)mps / ohw + 2) * img >= (1u << 31)))
        mps = (mps / 2 + BR - 1) / BR * BR;
    splits = (a.M + mps - 1) / mps;
    a.m_per_split = mps;
    const size_t lds = (size_t)NS * ((TCO + 127) / 128 + (SYM ? 0 : (TK + 127) / 128)) * BR * 256;
    hipLaunchKernelGGL((wgrad_v3_kernel<BR, NS, WCO, WKC, SYM>), dim3(ntiles * splits), dim3(WCO * WKC * 64), lds, st, a);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

}  // namespace
