// MFMA implicit-GEMM convolution, NHWC bf16, for gfx950 (MI355X).
//
// Replaces cuDNN's conv fwd / dgrad kernels that the reference reaches via
// torchvision resnet18 (/root/reference/imagenet.py:312, forward :123,
// backward :128).
//
// ONE "gather GEMM" kernel serves the forward conv, the stride-1 dgrad, each
// parity class of a strided dgrad (sub-pixel decomposition, no wasted MACs),
// the 7x7 stem and the FC layer (a 1x1 conv on a 1x1 image):
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
//  * stem (MODE 2): C == 4, the KW taps x 4 channels of a kernel row are one
//                  contiguous NHWC segment -> K = KH x 32 (28 real + 4 zero).
//
// Structure: a PERSISTENT grid (occupancy x CUs blocks). Each block walks its
// output tiles and their K-stages as ONE flattened sequence of stages, so the
// register-staged global loads of stage s+1 (possibly the first stage of the
// NEXT tile) are in flight while stage s runs its MFMAs and, at a tile's last
// stage, its epilogue. This keeps HBM streaming for the memory-bound
// small-K layers (ResNet 1x1 convs have 1-4 K-stages per tile), where a
// one-tile-per-block grid serialised load -> compute -> store.
// 256 threads = 4 waves; block tile BM pixels x BN channels; BK = 64; LDS
// double buffer, 128-B rows with an XOR chunk swizzle (conflict-free reads). MFMA v_mfma_f32_16x16x32_bf16 with the
// WEIGHTS as the A operand and the pixels as the B operand, so each lane's
// accumulator holds 4 consecutive output CHANNELS of one pixel: 8-byte NHWC
// stores with no LDS pass, and BN statistics (sum, sum of squares) reduce over
// the 16 lanes of a row group, then go to a 32-slot slab with fp32 atomics.
// Tiles are XCD-remapped so concurrently running channel tiles of one pixel
// panel share an XCD's L2.

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
};

#define IG_OUT_F32 1   // fp32 output (else bf16)
#define IG_RELU 2      // ReLU on the output
#define IG_STEM 4      // stem row-segment gather (MODE 2)
#define IG_ACCUM 8     // out += result (bf16 out only): fused gradient accumulation
#define STAT_SLOTS 32  // stats slab: [STAT_SLOTS][2][Nout]

namespace {

constexpr int BK = 64;
constexpr int LDK = BK;  // 128-B rows, 16-B chunks XOR-swizzled by (row & 7): conflict-free ds_read_b128

template <int BM, int BN, int WN, int MODE>  // MODE 0: C%64==0, 1: C%8==0, 2: stem row segments
__global__ __launch_bounds__(256, 2) void igemm_kernel(const IGemmArgs a) {
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
    const int nk = max(1, (K + BK - 1) / BK);  // K == 0 (empty dgrad class): one zero stage
    const int nstages = my_tiles * nk;
    const int col8 = tid & 7;
    const int ohw = a.OH * a.OW;

    // gather-row state of the tile currently being LOADED
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
        if (MODE == 0) {  // C % 64 == 0: the whole K stage sits in one tap
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

    const bool out_f32 = a.flags & IG_OUT_F32, relu = a.flags & IG_RELU, accum = a.flags & IG_ACCUM;
    float* st = a.stats ? a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * 2 * a.Nout : nullptr;

    // ---------------- epilogue of one output tile ----------------
    // lane holds channels n = nb + i*16 + (lane>>4)*4 + r (r<4) of pixel m = mb + j*16 + (lane&15)
    auto epilogue = [&](int tile) {
        const int m0 = (tile / nbn) * BM, n0 = (tile % nbn) * BN;
        const int nb = n0 + wn * TN + (lane >> 4) * 4;
        const int mb = m0 + wm * TM + (lane & 15);
        float s1[FN][4], s2[FN][4];
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int m = mb + j * 16;
            if (m >= a.M) continue;
            const int img = m / ohw, rem = m - img * ohw;
            const int oh = rem / a.OW, ow = rem - oh * a.OW;
            const size_t pix = ((size_t)img * a.YH + oh * a.sY + a.oy) * a.YW + ow * a.sY + a.ox;
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int n = nb + i * 16;
                if (n >= a.Nout) continue;
                const bool full = n + 3 < a.Nout && (a.ldy % 4) == 0;
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[i][j][r];
                    if (a.bias) v[r] += (n + r < a.Nout) ? a.bias[n + r] : 0.f;
                }
                if (out_f32) {
                    float* y = reinterpret_cast<float*>(a.Y) + pix * a.ldy + n;
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
                    bf16_t* y = reinterpret_cast<bf16_t*>(a.Y) + pix * a.ldy + n;
                    if (accum) {
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
                        s1[i][r] += v[r];
                        s2[i][r] += v[r] * v[r];
                    }
                }
            }
        }
        if (st) {
            // Every tile adds into the same 2*Nout words: contention, not bytes,
            // bounds this (MI355X_MICROARCH.md "Global float atomics": one hot
            // row is ~14x slower). Adds are spread over STAT_SLOTS copies by
            // block id (neighbouring blocks sit on different XCDs) and issued as
            // one 16-lane instruction per 16 consecutive channels;
            // imk_bn_stats_finalize folds the slots.
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                float v1 = 0.f, v2 = 0.f;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float x1 = s1[i][r], x2 = s2[i][r];
#pragma unroll
                    for (int o = 1; o < 16; o <<= 1) {
                        x1 += __shfl_xor(x1, o, 64);
                        x2 += __shfl_xor(x2, o, 64);
                    }
                    if ((lane & 15) == r) {
                        v1 = x1;
                        v2 = x2;
                    }
                }
                const int n = nb + i * 16 + (lane & 15);
                if ((lane & 15) < 4 && n < a.Nout) {
                    atomicAdd(st + n, v1);
                    atomicAdd(st + a.Nout + n, v2);
                }
            }
        }
    };

    // ---------------- flattened (tile, K-stage) pipeline ----------------
    setup_rows(lid);
    load_stage(0);
    store_stage(0);
    __syncthreads();
    const int fr = lane & 15;
    // physical chunk of logical chunk (lane>>4) + 4*ks in a row with (row & 7) == (fr & 7)
    const int fk0 = (((lane >> 4) + 0) ^ (fr & 7)) * 8, fk1 = (((lane >> 4) + 4) ^ (fr & 7)) * 8;
    int tj = 0, kt = 0;  // tile ordinal / stage within tile of stage s
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
        const bf16_t* bx = sX + buf * BM * LDK + (wm * TM + fr) * LDK;
        const bf16_t* bw = sW + buf * BN * LDK + (wn * TN + fr) * LDK;
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
            bf16x8 fw[FN], fx[FM];
#pragma unroll
            for (int i = 0; i < FN; ++i)
                fw[i] = *reinterpret_cast<const bf16x8*>(bw + i * 16 * LDK + (ks ? fk1 : fk0));
#pragma unroll
            for (int j = 0; j < FM; ++j)
                fx[j] = *reinterpret_cast<const bf16x8*>(bx + j * 16 * LDK + (ks ? fk1 : fk0));
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[i], fx[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 == nk) {
            epilogue(lid + tj * G);
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
}

template <int BM, int BN, int WN, int MD>
int launch(const IGemmArgs& a, hipStream_t st) {
    const int nbm = (a.M + BM - 1) / BM, nbn = (a.Nout + BN - 1) / BN;
    const int ntiles = nbm * nbn;
    const size_t lds = (size_t)2 * (BM + BN) * LDK * sizeof(bf16_t);
    static int resident = 0;  // persistent grid = blocks resident per CU x CUs (queried once)
    if (resident == 0) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, igemm_kernel<BM, BN, WN, MD>, 256, lds) !=
            hipSuccess || per_cu < 1)
            per_cu = 1;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
        resident = per_cu * cus;
    }
    // persistent only where it pays: tiles with few K-stages (memory-bound 1x1
    // convs) overlap the next tile's loads with this tile's epilogue; long-K
    // tiles keep one tile per block (the hardware refills CUs without a tail)
    const int K = MD == 2 ? a.nth * 32 : a.nth * a.ntw * a.C;
    const int nk = (K + BK - 1) / BK;
    const int grid = (nk > 4 || ntiles < resident) ? ntiles : resident;
    hipLaunchKernelGGL((igemm_kernel<BM, BN, WN, MD>), dim3(grid), dim3(256), lds, st, a);
    IMK_CHECK_LAUNCH();
    return 0;
}

}  // namespace

// Tile selection: Nout <= 64 -> 128x64 (1x4 waves), else 128x128 (2x2 waves).
IMK_EXPORT int imk_conv_igemm(const IGemmArgs* args, int tile, void* stream) {
    const IGemmArgs& a = *args;
    hipStream_t st = (hipStream_t)stream;
    if (a.M <= 0 || a.Nout <= 0) return 0;
    if ((a.flags & IG_ACCUM) && (a.flags & IG_OUT_F32)) return -103;
    if (a.flags & IG_STEM) {  // C == 4 row-segment gather, K = KH x 32
        if (a.C != 4 || a.ntw > 8 || a.dhs != 1 || a.dws != 1) return -102;
        return launch<128, 64, 1, 2>(a, st);
    }
    if (a.C % 8 != 0) return -100;  // 16-byte chunks must not straddle taps
    const int md = (a.C % BK) == 0 ? 0 : 1;
    if (tile == 0) tile = (a.Nout <= 64) ? 4 : 2;
#define IG_L(BM_, BN_, WN_) (md == 0 ? launch<BM_, BN_, WN_, 0>(a, st) : launch<BM_, BN_, WN_, 1>(a, st))
    switch (tile) {
        case 1: return IG_L(256, 64, 1);
        case 2: return IG_L(128, 128, 2);
        case 3: return IG_L(64, 128, 4);
        case 4: return IG_L(128, 64, 1);
        default: return -101;
    }
#undef IG_L
}

IMK_EXPORT int imk_igemm_args_size() { return (int)sizeof(IGemmArgs); }
