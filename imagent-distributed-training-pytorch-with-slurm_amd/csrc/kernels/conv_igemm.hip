// MFMA implicit-GEMM convolution for gfx950 (MI355X): the bf16 dispatcher.
// Kernels, layout and design notes: conv_igemm_impl.h; fp8: conv_igemm_fp8.hip.

#include "conv_igemm_impl.h"
#include "conv_igemm_v3.h"

// Tile selection (auto, tile 0):
//  * 64 -> 64 3x3 stride 1: the halo-tiled kernel (conv_halo.hip);
//  * 1x1 with C in {64, 128, 256, 512}: the streaming kernel (conv_stream.hip);
//  * C % 64 == 0 with the staged epilogue (every long-K conv, every fused BN-backward dgrad):
//    the v3 main loop (conv_igemm_v3.h), 256x256 tiles for Nout >= 256 (enough tiles), else 128x128
//    (round-3 A/B at R50 / 1024 img, profiles/r50_b1024_conv_v3.md);
//  * the rest (C % 64 != 0, direct epilogues, Nout <= 64): the LDS-DMA ring / register-staged
//    kernels of conv_igemm_impl.h.
// Explicit tiles (A/B, tests): 1-9 ring / register-staged variants, 17 / 18 v3 256x256 / 128x128.
// Measured and removed in round 3 (profiles/r50_b1024_v3_tile_study.md): v3 at 256x128, 128x256, 3-deep,
// and BK-32 4-deep rings, and a ping-pong 256x256 schedule with v3 addressing -- all within 2 % of v3.
// Measured slower and removed in round 3: the phased 256x256 kernel (profiles/
// r50_conv_phased_kernel.md), the ping-pong 256x256 kernel after the 8-phase template (-3.2 %),
// static wave priority for the second half of the waves (neutral).

// Smallest K (= taps x C) that takes the 256x256 v3 tile (one block per CU); below it the 128x128 tile (two blocks
// per CU) overlaps one block's epilogue with the other's main loop, which is what the epilogue-heavy short-K
// BN-backward dgrads need (A/B at batch 1024: 12,782 img/s with every conv on the big tile, 12,872 at 512)
constexpr int V3_BIG_MIN_K = 512;
// Narrowest output that takes the 256x256 v3 tile: 256 channels (one tile spans the whole output, so every pixel
// row is fetched once; in-step A/B at 2048 img: 16,597 / 16,586 vs 16,469 / 16,488 img/s with 512; isolated
// 256 -> 1024 @14 dgrad 327 vs 365 us, 512 -> 256 @28 fwd 842 vs 895 us)
constexpr int V3_BIG_MIN_N = 256;

// Wave-quantisation tail of the one-tile-per-block 256x256 kernels (one block per CU): with T tiles on S CUs the
// last of ceil(T / S) rounds runs T mod S tiles on an otherwise idle chip (R50 at 1024 img: 784 tiles on 256 CUs =
// 3 rounds + 16 tiles for every N = 256 conv at 14x14). When that remainder is at most 30 % of S, a FORWARD conv
// (no fused BN-backward / accumulating epilogue: in backward the weight-gradient side stream already fills the
// idle CUs of the last round) is split at an IMAGE boundary: the first I1 images fill exactly the whole rounds
// with 256x256 tiles, the remaining images run as 128x128 tiles (4x as many blocks, one quarter of the work each)
// right after. Every pixel-indexed operand advances by whole images; the statistics slabs accumulate across both
// launches.
constexpr float TAIL_FRAC = 0.3f;
static int device_cus() {
    static const int n = [] {
        int dev = 0, cus = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
        return cus;
    }();
    return n;
}

// images of the main part, or 0 when the conv is not split
static int tail_split_images(const IGemmArgs& a) {
    // (re-measured at 2048 img, end of round 5: in-step 16,538 / 16,531 / 16,538 with the split vs 16,491 / 16,487 /
    // 16,495 img/s without, alternating on one box -- kept)
    if (a.N < 2 || (a.flags & (IG_BNBWD | IG_ACCUM))) return 0;
    const long ohw = (long)a.OH * a.OW;
    const long nbn = (a.Nout + 255) / 256;
    const long tiles = ((a.M + 255) / 256) * nbn;
    const long S = device_cus();
    const long full = tiles / S, rem = tiles - full * S;
    if (full < 1 || rem == 0 || rem > TAIL_FRAC * S) return 0;
    const long mt = full * S / nbn;           // M tiles the whole rounds hold
    const long i1 = mt * 256 / ohw;           // whole images inside them
    return (i1 >= 1 && i1 < a.N) ? (int)i1 : 0;
}

static void advance_images(IGemmArgs& t, const IGemmArgs& a, int i1) {
    const long xs = (long)a.H * a.W * a.C, ys = (long)a.YH * a.YW * a.ldy;
    t.N = a.N - i1;
    t.M = t.N * a.OH * a.OW;
    t.X = a.X + i1 * xs;
    t.Y = static_cast<bf16_t*>(a.Y) + i1 * ys;  // staged epilogue: bf16 output only
    if (a.bnx) t.bnx = a.bnx + i1 * ys;
    if (a.bnym) t.bnym = a.bnym + i1 * ys / 8;
    if (a.bnx2) t.bnx2 = a.bnx2 + i1 * ys;
}

extern "C" int g_imk_conv_launches = 0;
IMK_EXPORT int imk_conv_launches() { return g_imk_conv_launches; }

IMK_EXPORT int imk_conv_igemm(const IGemmArgs* args, int tile, void* stream) {
    const IGemmArgs& a = *args;
    hipStream_t st = (hipStream_t)stream;
    if (a.M <= 0 || a.Nout <= 0) return 0;
    if ((a.flags & IG_ACCUM) && (a.flags & IG_OUT_F32)) return -103;
    if ((a.flags & IG_BNBWD) && ((a.flags & (IG_OUT_F32 | IG_RELU)) || a.Nout % 8 || a.ldy != a.Nout ||
                                 // no x (bn_gram.hip: sum(g xhat) comes from g^T h2): mask bits, staged epilogue
                                 (!a.bnx && (!a.bnym || (a.flags & IG_EPI_DIRECT))) ||
                                 !a.bnsave || !a.stats || (!a.bnym && (!a.bngamma || !a.bnbeta)) ||
                                 (a.bnx2 && !a.bnsave2)))
        return -104;
    if (a.flags & IG_STEM) {  // C == 4 row-segment gather, K = KH x 32
        if (a.C != 4 || a.ntw > 8 || a.dhs != 1 || a.dws != 1) return -102;
        if (tile == 0 || tile == 23) {  // band stem (tile 0) / streaming row-segment stem (23), conv_stream.hip
            const int r = conv_stem(a, st, tile);
            if (r != 1) return r;
        }
        return launch_rs<128, 64, 1, 2>(a, st);
    }
    if (a.xbn) {  // the operand BN + ReLU: the halo kernel (64 -> 64 3x3) or the streaming 1x1, nothing else
        if (a.flags & (IG_FP8 | IG_OUT_F32 | IG_RELU | IG_AFFINE | IG_STEM | IG_BNBWD | IG_ACCUM)) return -120;
        if (a.nth == 3 && a.ntw == 3) {
            const int r = conv_halo(a, st);
            return r == 1 ? -120 : r;
        }
        return conv_stream(a, st);
    }
    if (a.X2) {  // two K segments (bn_gram.hip): the streaming kernel for 256 + 64 -> 64, else the v3 loop
        // (the streaming kernel where it takes the shape: 963 vs 1087 us per call in-step for the layer-1 form;
        // tile != 0 forces the v3 loop, tests / A/B)
        if (tile == 0) {
            const int r = conv_stream(a, st);
            if (r != 1) return r;
        }
        if (!v3_ok(a) || a.Nout % 64) return -106;
        const long t8 = (long)((a.M + 255) / 256) * ((a.Nout + 255) / 256);
        if (a.Nout >= V3_BIG_MIN_N && t8 >= 192) return launch_v3<256, 256, 2, 2, 8, 128>(a, st);
        if (a.Nout == 64) return launch_v3<128, 64, 1, 2, 4, 128>(a, st);
        return launch_v3<128, 128, 2, 2, 4, 128>(a, st);
    }
    if (a.flags & IG_FP8) return conv_igemm_fp8(a, tile, st);
    if (a.C % 8 != 0) return -100;  // 16-byte chunks must not straddle taps
    if (tile == 0 && a.C == 64 && a.Nout == 64 && a.nth == 3 && a.ntw == 3) {
        const int r = conv_halo(a, st);
        if (r != 1) return r;
    }
    const int md = (a.C % BK) == 0 ? 0 : 1;
    // short-K 1x1 convs (K = C = 64 / 128) are HBM streams: weights resident in
    // LDS, pixel fragments straight from HBM (conv_stream.hip); tiles 20/21/22
    // force its 256/128/64-channel slices (A/B testing)
    const int bn_hint = tile >= 20 && tile <= 22 ? 256 >> (tile - 20) : 0;
    if (tile >= 20 && tile <= 22) tile = 0;
    const bool autotile = tile == 0;
    if (autotile && a.nth == 1 && a.ntw == 1 && (a.C == 64 || a.C == 128 || a.C == 256 || a.C == 512)) {
        const int r = conv_stream(a, st, bn_hint);
        if (r != 1) return r;
    }
    if (a.flags & (IG_RES | IG_MASKOUT | IG_Q8OUT)) return -121;  // only the streaming kernel has that epilogue
    if (autotile) tile = (a.Nout <= 64) ? 4 : 2;
    // measured on MI355X (profiles/r50_conv_layers_*): the register-staged
    // pipeline wins for 64-wide output tiles and single-stage (K <= 64) tiles,
    // the LDS-DMA ring for everything with a real K loop
    const int K = a.nth * a.ntw * a.C;
    const bool regstage = (a.flags & IG_REGSTAGE) || (autotile && (a.Nout <= 64 || K <= BK));
    // 256x256 tiles (8 waves, one block per CU) halve the L2->LDS bytes per
    // MFMA FLOP -- the measured limiter of the 128x128 tile (~70 GB/s per CU
    // of gathered rows, profiles/r50_conv_tiles_*.md) -- but only pay when
    // the output is >= 256 channels wide and there are enough of them to
    // occupy the chip
    if (autotile && !regstage && a.Nout >= 256) {
        const long t8 = (long)((a.M + 255) / 256) * ((a.Nout + 255) / 256);
        if (t8 >= 192) tile = 8;
    }
    const bool bnb = a.flags & IG_BNBWD;
    // staged epilogue: bf16, no bias; the eval forward's folded BatchNorm (+ ReLU) too
    const bool eval_bn = (a.flags & IG_AFFINE) && !a.stats;
    const bool lds_ok = !(a.flags & IG_OUT_F32) && (!(a.flags & IG_RELU) || eval_bn) && (!a.bias || eval_bn) &&
                        a.Nout % 8 == 0 && a.ldy % 8 == 0;
    // staged epilogue: always with the fused BN backward; otherwise for long-K
    // tiles (non-persistent anyway, +5-10 % measured) -- short-K memory-bound
    // 1x1 convs keep the persistent grid and its epilogue/prefetch overlap
    const bool use_lds = lds_ok && !(a.flags & IG_EPI_DIRECT) &&
                         (bnb || (a.flags & IG_EPI_LDS) || (K + BK - 1) / BK > 4);
    if (tile == 17 || tile == 18 || tile == 19 || tile == 27 || tile == 28 || (tile >= 29 && tile <= 32)) {
        // v3 main loop (conv_igemm_v3.h); 19: 256x128; 27 / 28: tap-inner; 29-32: deeper rings (round 6 A/B: the
        // 2-deep ring waits vmcnt(0) at every stage, so one stage of MFMA time must cover the fill latency):
        // 29 256x256 BK 32 x 4 (3 fills in flight, 128 KB), 30 256x256 BK 32 x 3, 31 128x128 BK 32 x 4 (64 KB,
        // two blocks / CU), 32 128x128 BK 64 x 3 (96 KB, one block / CU)
        if (!use_lds || !v3_ok(a)) return -105;
        switch (tile) {
            case 17: return launch_v3<256, 256, 2, 2, 8, 128>(a, st);
            case 19: return launch_v3<256, 128, 2, 2, 8, 128>(a, st);
            case 18: return launch_v3<128, 128, 2, 2, 4, 128>(a, st);
            case 27: return launch_v3<256, 256, 2, 2, 8, 128, 2, 0, true>(a, st);
            case 29: return launch_v3<256, 256, 2, 4, 8, 64>(a, st);
            case 30: return launch_v3<256, 256, 2, 3, 8, 64>(a, st);
            case 31: return launch_v3<128, 128, 2, 4, 4, 64>(a, st);
            case 32: return launch_v3<128, 128, 2, 3, 4, 128>(a, st);
            default: return launch_v3<128, 128, 2, 2, 4, 128, 2, 0, true>(a, st);
        }
        // (a 16-wave 256x256 tile of 64 x 64 waves, round 5: no faster than these on any R50 shape, its staged BN-backward
        // epilogue 1.4-1.7x slower from spills at 128 VGPRs -- not kept)
    }
    if (autotile && use_lds && md == 0 && a.Nout >= 128 && v3_ok(a)) {
        const long t8 = (long)((a.M + 255) / 256) * ((a.Nout + 255) / 256);
        // forward-type convs (BN statistics or the eval BN affine in the epilogue, no fused BN backward): 32-deep
        // stages with 2-3 fills in flight instead of 64-deep x 2 (whose vmcnt(0) at every stage leaves one stage of
        // MFMA time to cover the fill latency). Round 6, isolated at 2048 img (scripts/runs/ring_ab.sh, tiles 30 / 31
        // vs 17 / 18): forwards 256@14 3x3 554 -> 502 us, 1024 -> 256 @14 346 -> 325, 512@7 3x3 521 -> 491, 256@28
        // 3x3 s2 642 -> 567, 128@28 3x3 721 -> 665, 512 -> 128 @28 570 -> 498; the dgrads (plain or with the fused
        // BN backward) gain nothing (-3 .. +2 %). In-step at 4096 img the isolated gain does NOT carry over:
        // 17,317 / 17,289 img/s with it vs 17,358 / 17,395 without, alternating on one box -- so it stays OFF by
        // default; IMAGENT_V3_DEEP=1 turns it on (A/B), tiles 29-32 remain as tested explicit variants
        static const bool deep = [] {
            const char* e = getenv("IMAGENT_V3_DEEP");
            return e && atoi(e) != 0;
        }();
        const bool fwd_ring = deep && !bnb && (a.stats || (a.flags & IG_AFFINE));
        // (the fused BN-backward dgrads on 128x128 tiles with their epilogue operands prefetched instead: within
        // +-5 % per shape, profiles/r50_b1024_round4_kernel_ab.md -- not taken; again at 2048 img in round 5, isolated
        // 2-7 % faster, in-step 16,584 / 16,576 vs 16,612 / 16,621 img/s)
        if (a.Nout >= V3_BIG_MIN_N && t8 >= 192 && K >= V3_BIG_MIN_K) {
            const int i1 = tail_split_images(a);
            if (i1 > 0) {  // whole rounds of 256x256 tiles, the remaining images as 128x128 tiles
                IGemmArgs m = a, t = a;
                m.N = i1;
                m.M = i1 * a.OH * a.OW;
                advance_images(t, a, i1);
                const int r = fwd_ring ? launch_v3<256, 256, 2, 3, 8, 64>(m, st) : launch_v3<256, 256, 2, 2, 8, 128>(m, st);
                if (r != 0) return r;
                return fwd_ring ? launch_v3<128, 128, 2, 4, 4, 64>(t, st) : launch_v3<128, 128, 2, 2, 4, 128>(t, st);
            }
            return fwd_ring ? launch_v3<256, 256, 2, 3, 8, 64>(a, st) : launch_v3<256, 256, 2, 2, 8, 128>(a, st);
        }
        // (256x128 tiles on 8 waves for the 128-channel outputs, tile 19, round 5: forward 3-6 % faster stand-alone,
        // dgrad 6 % and the fused BN-backward dgrads 7-21 % slower, in-step 16,822 / 16,842 vs 17,003 / 16,991 img/s
        // -- not taken, profiles/r50_b2048_r5_v3_256x128.md)
        return fwd_ring ? launch_v3<128, 128, 2, 4, 4, 64>(a, st) : launch_v3<128, 128, 2, 2, 4, 128>(a, st);
    }
    if (bnb || use_lds) {  // the tiles the auto choice makes, with a fused / staged epilogue
        if (regstage || (tile != 2 && tile != 8)) {
            if (tile != 2) tile = 4;
#define IG_RSB(BM_, BN_, WN_, E_) \
    (md == 0 ? launch_rs<BM_, BN_, WN_, 0, E_>(a, st) : launch_rs<BM_, BN_, WN_, 1, E_>(a, st))
            if (use_lds) return tile == 2 ? IG_RSB(128, 128, 2, 2) : IG_RSB(128, 64, 1, 2);
            return tile == 2 ? IG_RSB(128, 128, 2, 1) : IG_RSB(128, 64, 1, 1);
#undef IG_RSB
        }
#define IG_DB(BM_, BN_, WN_, NS_, NW_, E_)                                                  \
    (md == 0 ? launch_dma<BM_, BN_, WN_, NS_, 0, NW_, E_>(a, st)                       \
             : launch_dma<BM_, BN_, WN_, NS_, 1, NW_, E_>(a, st))
        if (use_lds && tile == 8 && autotile) {
            const int i1 = tail_split_images(a);
            if (i1 > 0) {
                IGemmArgs m = a, t = a;
                m.N = i1;
                m.M = i1 * a.OH * a.OW;
                advance_images(t, a, i1);
                const int r = md == 0 ? launch_dma<256, 256, 2, 2, 0, 8, 2>(m, st)
                                      : launch_dma<256, 256, 2, 2, 1, 8, 2>(m, st);
                if (r != 0) return r;
                return md == 0 ? launch_dma<128, 128, 2, 2, 0, 4, 2>(t, st) : launch_dma<128, 128, 2, 2, 1, 4, 2>(t, st);
            }
        }
        if (use_lds) return tile == 8 ? IG_DB(256, 256, 2, 2, 8, 2) : IG_DB(128, 128, 2, 2, 4, 2);
        return tile == 8 ? IG_DB(256, 256, 2, 2, 8, 1) : IG_DB(128, 128, 2, 2, 4, 1);
#undef IG_DB
    }
    if (regstage) {
#define IG_RS(BM_, BN_, WN_) (md == 0 ? launch_rs<BM_, BN_, WN_, 0>(a, st) : launch_rs<BM_, BN_, WN_, 1>(a, st))
        switch (tile) {
            case 2: return IG_RS(128, 128, 2);
            case 4: return IG_RS(128, 64, 1);
            default: return -101;
        }
#undef IG_RS
    }
#define IG_D(BM_, BN_, WN_, NS_, NW_) \
    (md == 0 ? launch_dma<BM_, BN_, WN_, NS_, 0, NW_>(a, st) : launch_dma<BM_, BN_, WN_, NS_, 1, NW_>(a, st))
    switch (tile) {
        case 1: return IG_D(256, 64, 1, 2, 4);
        case 2: return IG_D(128, 128, 2, 2, 4);
        case 3: return IG_D(64, 128, 4, 3, 4);
        case 4: return IG_D(128, 64, 1, 3, 4);
        case 5: return IG_D(128, 128, 2, 3, 4);
        case 6: return IG_D(256, 128, 2, 3, 8);  // 144 KiB LDS, 8 waves of 64x64
        case 7: return IG_D(128, 256, 4, 3, 8);
        case 8: return IG_D(256, 256, 2, 2, 8);  // 128 KiB LDS, 8 waves of 64x128
        case 9: return IG_D(256, 128, 2, 2, 8);
        default: return -101;
    }
#undef IG_D
}

IMK_EXPORT int imk_igemm_args_size() { return (int)sizeof(IGemmArgs); }
