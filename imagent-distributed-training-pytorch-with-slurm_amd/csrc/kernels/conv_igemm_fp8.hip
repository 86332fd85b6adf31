// fp8 (OCP e4m3 / e5m2) implicit-GEMM convolutions on the block-scaled MFMA
// (v_mfma_scale_f32_16x16x128_f8f6f4; kernels in conv_igemm_impl.h, EB = 1):
//  * forward: X = e4m3 activations, Wk = e4m3 weights;
//  * dgrad (IG_BF8X): X = e5m2 upstream gradient, Wk = e4m3 transposed
//    weights, with the same fused epilogues as bf16 (IG_ACCUM residual
//    accumulation, IG_BNBWD BatchNorm-backward reductions).
// Per-tensor power-of-two scales (device ints xexp / wexp) ride in the MFMA's
// E8M0 scale operands.

//
// C % 128 == 0 (every ResNet conv but the 64-channel ones of the first stage) runs the v3 LDS-DMA main
// loop with 1-byte operands (conv_igemm_v3.h, EB = 1): 256x256 tiles for Nout >= 512 with enough tiles
// and K >= 512, 128x128 for Nout >= 128, 128x64 below; explicit tiles 17 / 18 / 19 force those.
// The rest (and explicit tiles 2 / 4 / 8) takes the round-1 ring (igemm_dma_kernel, EB = 1).

#include "conv_igemm_impl.h"
#include "conv_igemm_v3.h"

template <int FB>
static int launch_v3_fp8(const IGemmArgs& a, int tile, hipStream_t st) {
    const long t8 = (long)((a.M + 255) / 256) * ((a.Nout + 255) / 256);
    const int K = a.nth * a.ntw * a.C;
    if (tile == 0) tile = (a.Nout >= 512 && t8 >= 192 && K >= 512) ? 17 : (a.Nout >= 128 ? 18 : 19);
    switch (tile) {
        case 17: return launch_v3<256, 256, 2, 2, 8, 128, 1, FB>(a, st);
        case 18: return launch_v3<128, 128, 2, 2, 4, 128, 1, FB>(a, st);
        default: return launch_v3<128, 64, 1, 2, 4, 128, 1, FB>(a, st);
    }
}

int conv_igemm_fp8(const IGemmArgs& a, int tile, hipStream_t st) {
    const bool bf8x = a.flags & IG_BF8X;
    if (a.C % 16 != 0 || (a.flags & IG_OUT_F32) || a.bias || !a.xexp || !a.wexp) return -105;
    if (!bf8x && (a.flags & (IG_BNBWD | IG_ACCUM))) return -105;
    if ((tile == 0 || (tile >= 17 && tile <= 19)) && v3_ok8(a) && (tile != 19 || a.Nout % 64 == 0))
        return bf8x ? launch_v3_fp8<1>(a, tile, st) : launch_v3_fp8<0>(a, tile, st);
    if (tile >= 17 && tile <= 19) return -105;
    const int md8 = (a.C % 128) == 0 ? 0 : 1;
    const int K8 = a.nth * a.ntw * a.C;
    const bool lds_ok = a.Nout % 8 == 0 && a.ldy % 8 == 0 && !(a.flags & (IG_RELU | IG_EPI_DIRECT));
    const bool lds8 = lds_ok && ((a.flags & (IG_EPI_LDS | IG_BNBWD)) || (K8 + 127) / 128 > 4);
    if ((a.flags & IG_BNBWD) && !lds8) return -104;
    if (tile == 0) {
        tile = a.Nout <= 64 ? 4 : 2;
        if (a.Nout >= 256 && (long)((a.M + 255) / 256) * ((a.Nout + 255) / 256) >= 192) tile = 8;
    }
#define IG_F8(BM_, BN_, WN_, NS_, NW_, FB_)                                                              \
    (lds8 ? (md8 == 0 ? launch_dma<BM_, BN_, WN_, NS_, 0, NW_, 2, 1, FB_>(a, st)                         \
                      : launch_dma<BM_, BN_, WN_, NS_, 1, NW_, 2, 1, FB_>(a, st))                        \
          : (md8 == 0 ? launch_dma<BM_, BN_, WN_, NS_, 0, NW_, 0, 1, FB_>(a, st)                         \
                      : launch_dma<BM_, BN_, WN_, NS_, 1, NW_, 0, 1, FB_>(a, st)))
    switch (tile) {
        case 2: return bf8x ? IG_F8(128, 128, 2, 2, 4, 1) : IG_F8(128, 128, 2, 2, 4, 0);
        case 4: return bf8x ? IG_F8(128, 64, 1, 3, 4, 1) : IG_F8(128, 64, 1, 3, 4, 0);
        case 8: return bf8x ? IG_F8(256, 256, 2, 2, 8, 1) : IG_F8(256, 256, 2, 2, 8, 0);
        default: return -101;
    }
#undef IG_F8
}
