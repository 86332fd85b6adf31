// fp32 training path for gfx950 (MI355X): the reference's own precision.
//
// The reference trains ResNet-18 at 448x448 in fp32 with no AMP (/root/reference/imagenet.py:281
// Resize(448), :312 resnet18, :442 batch 128). These kernels run that configuration on
// this framework's own code at fp32 accuracy (tests: <= 1e-4 relative against PyTorch fp32):
//
//  * igemm_f32_kernel: the same gather-GEMM formulation as the bf16 convs (IGemmArgs: forward,
//    stride-1 dgrad, each parity class of a strided dgrad, the 4-channel stem, the FC layer) on
//    the exact-f32 MFMA v_mfma_f32_16x16x4_f32 (one f32 operand per lane, fp32 accumulate; 1/16 of
//    the bf16 MFMA rate, MI355X_MICROARCH.md "Matrix cores"). The operand k order inside a 16-deep
//    LDS chunk is permuted identically for both operands (lane group g feeds k = 4g + s at sub-step
//    s), so every lane reads its 4 k-values with one ds_read_b128 from the same 128-B-row,
//    row-XOR-swizzled LDS image the bf16 kernels use. Register-staged double buffer, 128x128 tile,
//    2 blocks per CU: the MFMA pipe, not the operand path, is the limit at this rate.
//  * wgrad_f32_kernel: dW[co][k] += sum_m dY[m][co] X_gather[m][k], split over m with fp32
//    atomics into dW; both operands staged as [m][col] rows (pitch 144 floats: the two row
//    groups of a ds_read_b32 half-wave land 16 banks apart) and read transposed.
//  * BatchNorm (training statistics as per-block partial slabs folded in a fixed order ->
//    deterministic; apply with residual add + ReLU; backward reduce + apply), maxpool with
//    argmax, global average pool, FC bias column sums, input normalisation to fp32.

#include "conv_igemm_impl.h"
#include "conv_igemm_v3.h"

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ conv fwd / dgrad
constexpr int F_BM = 128, F_BN = 128, F_BK = 32;  // BK in floats: one 128-B LDS row

template <int MODE>  // 0: C % 32 == 0 (one tap per stage), 1: per-chunk tap (C % 4 == 0)
__global__ __launch_bounds__(256, 2) void igemm_f32_kernel(const IGemmArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* sX = reinterpret_cast<float*>(smem);          // [2][BM][32]
    float* sW = sX + 2 * F_BM * F_BK;                    // [2][BN][32]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wn = wid & 1, wm = wid >> 1;               // 2 x 2 waves, 64 x 64 each
    const int nbn = (a.Nout + F_BN - 1) / F_BN;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    if (lid >= ((a.M + F_BM - 1) / F_BM) * nbn) return;
    const int m0 = (lid / nbn) * F_BM, n0 = (lid % nbn) * F_BN;
    const int K = a.nth * a.ntw * a.C;
    const int nk = (K + F_BK - 1) / F_BK;
    const int ohw = a.OH * a.OW;
    const int col8 = tid & 7;  // this thread's 16-B chunk (4 k) of a staged row
    const float* X = reinterpret_cast<const float*>(a.X);
    const float* Wk = reinterpret_cast<const float*>(a.Wk);

    const float* xrow[4];
    int ih0[4], iw0[4];
    bool mok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + (tid >> 3) + 32 * i;
        mok[i] = m < a.M;
        const int mm = mok[i] ? m : 0;
        const int img = mm / ohw, rem = mm - img * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        xrow[i] = X + (size_t)img * a.H * a.W * a.C;
        ih0[i] = oh * a.sA;
        iw0[i] = ow * a.sA;
    }
    const float* wrow[4];
    bool nok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = n0 + (tid >> 3) + 32 * j;
        nok[j] = n < a.Nout;
        wrow[j] = Wk + (size_t)(nok[j] ? n : 0) * a.ldb;
    }
    f32x4v rx[4], rw[4];
    auto load = [&](int kt) {
        const int k = kt * F_BK + col8 * 4;
        int t, c;
        if (MODE == 0) {
            t = (kt * F_BK) / a.C;
            c = kt * F_BK - t * a.C + col8 * 4;
        } else {
            t = k / a.C;
            c = k - t * a.C;
        }
        const bool kok = k < K;
        const int ti = kok ? t / a.ntw : 0, tj = kok ? t - ti * a.ntw : 0;
        const int dh = a.dh0 + ti * a.dhs, dw = a.dw0 + tj * a.dws;
        const int wtap = (a.kh0 + ti * a.khs) * a.KW + (a.kw0 + tj * a.kws);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ih = ih0[i] + dh, iw = iw0[i] + dw;
            const bool ok = kok && mok[i] && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
            rx[i] = ok ? *reinterpret_cast<const f32x4v*>(xrow[i] + ((size_t)ih * a.W + iw) * a.C + c)
                       : f32x4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            rw[j] = (kok && nok[j]) ? *reinterpret_cast<const f32x4v*>(wrow[j] + (size_t)wtap * a.C + c)
                                    : f32x4v{0.f, 0.f, 0.f, 0.f};
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = (tid >> 3) + 32 * i;
            *reinterpret_cast<f32x4v*>(sX + (buf * F_BM + r) * F_BK + ((col8 ^ (r & 7)) * 4)) = rx[i];
            *reinterpret_cast<f32x4v*>(sW + (buf * F_BN + r) * F_BK + ((col8 ^ (r & 7)) * 4)) = rw[i];
        }
    };
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    load(0);
    store(0);
    __syncthreads();
    const int fr = lane & 15, g = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load(kt + 1);
        const float* bx = sX + (buf * F_BM + wm * 64 + fr) * F_BK;
        const float* bw = sW + (buf * F_BN + wn * 64 + fr) * F_BK;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int off = ((ks * 4 + g) ^ (fr & 7)) * 4;  // fragment rows are 16-aligned + fr
            f32x4v fw[4], fx[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) fw[i] = *reinterpret_cast<const f32x4v*>(bw + i * 16 * F_BK + off);
#pragma unroll
            for (int j = 0; j < 4; ++j) fx[j] = *reinterpret_cast<const f32x4v*>(bx + j * 16 * F_BK + off);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fw[i][s], fx[j][s], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) {  // buf ^ 1 was last read in iteration kt - 1, before its closing barrier
            store(buf ^ 1);
            __syncthreads();
        }
    }
    // epilogue: lane holds channels nb + i*16 + 4g + r of pixel mb + j*16 + fr
    const bool accum = a.flags & IG_ACCUM;
    const float* bias = a.bias;
    float* Y = reinterpret_cast<float*>(a.Y);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + j * 16 + fr;
        if (m >= a.M) continue;
        const int img = m / ohw, rem = m - img * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        float* yp = Y + (((size_t)img * a.YH + oh * a.sY + a.oy) * a.YW + ow * a.sY + a.ox) * a.ldy;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int n = n0 + wn * 64 + i * 16 + 4 * g;
            f32x4 v = acc[i][j];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (bias && n + r < a.Nout) v[r] += bias[n + r];
            if (n + 3 < a.Nout && (a.ldy & 3) == 0) {
                f32x4* p = reinterpret_cast<f32x4*>(yp + n);
                if (accum) v += *p;
                *p = v;
            } else {
                for (int r = 0; r < 4; ++r)
                    if (n + r < a.Nout) yp[n + r] = accum ? yp[n + r] + v[r] : v[r];
            }
        }
    }
}

// ------------------------------------------------------------------ conv fwd / dgrad, 3 x bf16 split
// The same gather-GEMM with each fp32 operand split into bf16 hi + lo (x = hi + lo, |x - hi - lo| <= 2^-18 |x|)
// and x*w computed as hi*hi + hi*lo + lo*hi on v_mfma_f32_16x16x32_bf16 (fp32 accumulate): the dropped lo*lo
// term and the rounding of lo leave ~2^-16 relative per product, three bf16 MFMAs cost 3/16 of the f32 MFMA
// cycles of the exact kernel above. Tile, loads and epilogue as igemm_f32_kernel; LDS per stage: hi / lo planes
// of both operands as 64-B rows (32 k), 16-B chunk c of row r at slot c ^ ((r >> 2) & 3) (conflict-free
// ds_read_b128 fragment reads: 16 rows of one chunk land on 16 distinct slots).
template <int MODE>
__global__ __launch_bounds__(256, 2) void igemm_f32s_kernel(const IGemmArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int PLANE = F_BM * F_BK * 2;  // one [128][32] bf16 plane
    constexpr int SBUF = 4 * PLANE;         // Xh, Xl, Wh, Wl
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wn = wid & 1, wm = wid >> 1;  // 2 x 2 waves, 64 x 64 each
    const int nbn = (a.Nout + F_BN - 1) / F_BN;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    if (lid >= ((a.M + F_BM - 1) / F_BM) * nbn) return;
    const int m0 = (lid / nbn) * F_BM, n0 = (lid % nbn) * F_BN;
    const int K = a.nth * a.ntw * a.C;
    const int nk = (K + F_BK - 1) / F_BK;
    const int ohw = a.OH * a.OW;
    const int col8 = tid & 7;  // this thread's 16-B fp32 chunk (4 k) of a staged row
    const float* X = reinterpret_cast<const float*>(a.X);
    const float* Wk = reinterpret_cast<const float*>(a.Wk);

    const float* xrow[4];
    int ih0[4], iw0[4];
    bool mok[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + (tid >> 3) + 32 * i;
        mok[i] = m < a.M;
        const int mm = mok[i] ? m : 0;
        const int img = mm / ohw, rem = mm - img * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        xrow[i] = X + (size_t)img * a.H * a.W * a.C;
        ih0[i] = oh * a.sA;
        iw0[i] = ow * a.sA;
    }
    const float* wrow[4];
    bool nok[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = n0 + (tid >> 3) + 32 * j;
        nok[j] = n < a.Nout;
        wrow[j] = Wk + (size_t)(nok[j] ? n : 0) * a.ldb;
    }
    f32x4v rx[4], rw[4];
    auto load = [&](int kt) {
        const int k = kt * F_BK + col8 * 4;
        int t, c;
        if (MODE == 0) {
            t = (kt * F_BK) / a.C;
            c = kt * F_BK - t * a.C + col8 * 4;
        } else {
            t = k / a.C;
            c = k - t * a.C;
        }
        const bool kok = k < K;
        const int ti = kok ? t / a.ntw : 0, tj = kok ? t - ti * a.ntw : 0;
        const int dh = a.dh0 + ti * a.dhs, dw = a.dw0 + tj * a.dws;
        const int wtap = (a.kh0 + ti * a.khs) * a.KW + (a.kw0 + tj * a.kws);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ih = ih0[i] + dh, iw = iw0[i] + dw;
            const bool ok = kok && mok[i] && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
            rx[i] = ok ? *reinterpret_cast<const f32x4v*>(xrow[i] + ((size_t)ih * a.W + iw) * a.C + c)
                       : f32x4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            rw[j] = (kok && nok[j]) ? *reinterpret_cast<const f32x4v*>(wrow[j] + (size_t)wtap * a.C + c)
                                    : f32x4v{0.f, 0.f, 0.f, 0.f};
    };
    // 4 fp32 -> 4 bf16 hi (8 B) + 4 bf16 lo (8 B) at row r, k = 4 col8 .. + 3
    auto put = [&](char* hi_plane, char* lo_plane, int r, const f32x4v& v) {
        const uint32_t h0 = pack_bf2(v[0], v[1]), h1 = pack_bf2(v[2], v[3]);
        const uint32_t l0 = pack_bf2(v[0] - lo_bf(h0), v[1] - hi_bf(h0));
        const uint32_t l1 = pack_bf2(v[2] - lo_bf(h1), v[3] - hi_bf(h1));
        const int off = r * 64 + (((col8 >> 1) ^ ((r >> 2) & 3)) << 4) + ((col8 & 1) << 3);
        *reinterpret_cast<u32x2*>(hi_plane + off) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(lo_plane + off) = u32x2{l0, l1};
    };
    auto store = [&](int buf) {
        char* b = smem + buf * SBUF;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = (tid >> 3) + 32 * i;
            put(b, b + PLANE, r, rx[i]);
            put(b + 2 * PLANE, b + 3 * PLANE, r, rw[i]);
        }
    };
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    load(0);
    store(0);
    __syncthreads();
    const int fr = lane & 15;
    const int foff = fr * 64 + ((((lane >> 4) ^ ((fr >> 2) & 3))) << 4);  // row fr of a 16-row block, chunk lane>>4
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load(kt + 1);
        const char* b = smem + buf * SBUF;
        bf16x8 xh[4], xl[4], whi[4], wlo[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ro = (wn * 64 + i * 16) * 64 + foff;
            whi[i] = *reinterpret_cast<const bf16x8*>(b + 2 * PLANE + ro);
            wlo[i] = *reinterpret_cast<const bf16x8*>(b + 3 * PLANE + ro);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ro = (wm * 64 + j * 16) * 64 + foff;
            xh[j] = *reinterpret_cast<const bf16x8*>(b + ro);
            xl[j] = *reinterpret_cast<const bf16x8*>(b + PLANE + ro);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlo[i], xh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi[i], xl[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(whi[i], xh[j], acc[i][j], 0, 0, 0);
            }
        if (kt + 1 < nk) {  // buf ^ 1 was last read in iteration kt - 1, before its closing barrier
            store(buf ^ 1);
            __syncthreads();
        }
    }
    // epilogue: lane holds channels nb + i*16 + 4g + r of pixel mb + j*16 + fr (as igemm_f32_kernel)
    const int g = lane >> 4;
    const bool accum = a.flags & IG_ACCUM;
    const float* bias = a.bias;
    float* Y = reinterpret_cast<float*>(a.Y);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + j * 16 + fr;
        if (m >= a.M) continue;
        const int img = m / ohw, rem = m - img * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        float* yp = Y + (((size_t)img * a.YH + oh * a.sY + a.oy) * a.YW + ow * a.sY + a.ox) * a.ldy;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int n = n0 + wn * 64 + i * 16 + 4 * g;
            f32x4 v = acc[i][j];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (bias && n + r < a.Nout) v[r] += bias[n + r];
            if (n + 3 < a.Nout && (a.ldy & 3) == 0) {
                f32x4* p = reinterpret_cast<f32x4*>(yp + n);
                if (accum) v += *p;
                *p = v;
            } else {
                for (int r = 0; r < 4; ++r)
                    if (n + r < a.Nout) yp[n + r] = accum ? yp[n + r] + v[r] : v[r];
            }
        }
    }
}

// ------------------------------------------------------------------------ wgrad
struct WgradF32Args {
    const float* dY;  // [M][Co] (output grid NHWC)
    const float* X;   // [N][H][W][C]
    float* dW;        // [Co][KH][KW][C] (+=)
    int N, H, W, C, Co, OH, OW, M, KH, KW, stride, pad, m_per_split;
};

constexpr int WG_M = 32;      // pixels per stage
constexpr int WG_P = 144;     // LDS row pitch (floats)

// The im2col gather of one 16-B chunk per (thread, u) of the wgrad X operand: its k column (tap kh, kw and
// channel c) never changes and its pixel row moves by exactly WG_M per stage, so the tap is decoded once and
// the pixel (img, oh, ow) is a cursor stepped by WG_M (no integer divisions in the main loop).
struct WgGather {
    int kh, kw, c, m, img, oh, ow;
    __device__ void init(const WgradF32Args& a, int k, int m0, int Kt) {
        const int kk = k < Kt ? k : 0;
        const int t = kk / a.C;
        c = kk - t * a.C;
        kh = k < Kt ? t / a.KW : -(1 << 20);  // a column past Kt never hits the image
        kw = t - (t / a.KW) * a.KW;
        m = m0;
        const int ohw = a.OH * a.OW;
        img = m0 / ohw;
        const int rem = m0 - img * ohw;
        oh = rem / a.OW;
        ow = rem - oh * a.OW;
    }
    __device__ f32x4v load(const WgradF32Args& a, int mend) const {
        const int ih = oh * a.stride - a.pad + kh, iw = ow * a.stride - a.pad + kw;
        if (m < mend && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
            return *reinterpret_cast<const f32x4v*>(a.X + (((size_t)img * a.H + ih) * a.W + iw) * a.C + c);
        return f32x4v{0.f, 0.f, 0.f, 0.f};
    }
    __device__ void step(const WgradF32Args& a) {
        m += WG_M;
        ow += WG_M;
        while (ow >= a.OW) {
            ow -= a.OW;
            if (++oh == a.OH) {
                oh = 0;
                ++img;
            }
        }
    }
};

template <int BCO, int BK>
__global__ __launch_bounds__(256, 2) void wgrad_f32_kernel(const WgradF32Args a) {
    constexpr int WCO = BCO == 128 ? 2 : 1, WK = 4 / WCO;  // 4 waves
    constexpr int TCO = BCO / WCO, TK = BK / WK;           // wave tile
    constexpr int FI = TCO / 16, FJ = TK / 16;
    constexpr int CA = WG_M * BCO / 4 / 256, CB = WG_M * BK / 4 / 256;  // 16-B chunks per thread per stage
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* sA = reinterpret_cast<float*>(smem);   // [2][WG_M][WG_P] dY
    float* sB = sA + 2 * WG_M * WG_P;             // [2][WG_M][WG_P] X gather
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wc = wid % WCO, wk = wid / WCO;
    const int Kt = a.KH * a.KW * a.C;
    const int nco = (a.Co + BCO - 1) / BCO, nkt = (Kt + BK - 1) / BK;
    const int tile = blockIdx.x % (nco * nkt), split = blockIdx.x / (nco * nkt);
    const int co0 = (tile % nco) * BCO, k0 = (tile / nco) * BK;
    const int mbeg = split * a.m_per_split, mend = min(a.M, mbeg + a.m_per_split);
    if (mbeg >= mend) return;
    WgGather gb[CB];
#pragma unroll
    for (int u = 0; u < CB; ++u) {
        const int q = tid + 256 * u;
        gb[u].init(a, k0 + (q % (BK / 4)) * 4, mbeg + q / (BK / 4), Kt);
    }
    // chunk assignment: A chunk q -> (row = q / (BCO/4), col4 = q % (BCO/4)); same for B with BK
    f32x4v ra[CA], rb[CB];
    auto load = [&](int mb) {
#pragma unroll
        for (int u = 0; u < CA; ++u) {
            const int q = tid + 256 * u;
            const int r = q / (BCO / 4), cc = (q % (BCO / 4)) * 4;
            const int m = mb + r, co = co0 + cc;
            ra[u] = (m < mend && co < a.Co) ? *reinterpret_cast<const f32x4v*>(a.dY + (size_t)m * a.Co + co)
                                            : f32x4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            rb[u] = gb[u].load(a, mend);
            gb[u].step(a);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int u = 0; u < CA; ++u) {
            const int q = tid + 256 * u;
            *reinterpret_cast<f32x4v*>(sA + (buf * WG_M + q / (BCO / 4)) * WG_P + (q % (BCO / 4)) * 4) = ra[u];
        }
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            const int q = tid + 256 * u;
            *reinterpret_cast<f32x4v*>(sB + (buf * WG_M + q / (BK / 4)) * WG_P + (q % (BK / 4)) * 4) = rb[u];
        }
    };
    f32x4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nst = (mend - mbeg + WG_M - 1) / WG_M;
    load(mbeg);
    store(0);
    __syncthreads();
    const int fr = lane & 15, g = lane >> 4;
    for (int s = 0; s < nst; ++s) {
        const int buf = s & 1;
        if (s + 1 < nst) load(mbeg + (s + 1) * WG_M);
        const float* ba = sA + buf * WG_M * WG_P + wc * TCO + fr;
        const float* bb = sB + buf * WG_M * WG_P + wk * TK + fr;
#pragma unroll
        for (int t = 0; t < WG_M / 4; ++t) {  // instruction t: lane group g feeds pixel 4t + g
            float fa[FI], fb[FJ];
#pragma unroll
            for (int i = 0; i < FI; ++i) fa[i] = ba[(4 * t + g) * WG_P + i * 16];
#pragma unroll
            for (int j = 0; j < FJ; ++j) fb[j] = bb[(4 * t + g) * WG_P + j * 16];
#pragma unroll
            for (int i = 0; i < FI; ++i)
#pragma unroll
                for (int j = 0; j < FJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        if (s + 1 < nst) {  // buf ^ 1 was last read in stage s - 1, before its closing barrier
            store(buf ^ 1);
            __syncthreads();
        }
    }
    // lane: rows (co) co0 + wc*TCO + i*16 + 4g + r, column (k) k0 + wk*TK + j*16 + fr
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            const int k = k0 + wk * TK + j * 16 + fr;
            if (k >= Kt) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + wc * TCO + i * 16 + 4 * g + r;
                if (co < a.Co) atomicAdd(a.dW + (size_t)co * Kt + k, acc[i][j][r]);
            }
        }
}

// The weight gradient with the 3 x bf16 split (as igemm_f32s_kernel): a 32-pixel stage is one
// v_mfma_f32_16x16x32_bf16 k-step; both operands staged as hi / lo bf16 planes of [32 px][256 B] rows
// (chunk ch of row r at slot ch ^ (((r & 3) << 2) | ((r >> 2) & 3)), cdna_hip_programming.md T10 image (b);
// a 64-column tile uses half of each row) and read as MFMA fragments by ds_read_b64_tr_b16 (pixels -> k),
// the pixel order inside a fragment permuted identically for both operands (the sum over m does not care).
__device__ __forceinline__ int wgs_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }

template <int BCO, int BK>
__global__ __launch_bounds__(256, 2) void wgrad_f32s_kernel(const WgradF32Args a) {
    constexpr int WCO = BCO == 128 ? 2 : 1, WK = 4 / WCO;  // 4 waves
    constexpr int TCO = BCO / WCO, TK = BK / WK;           // wave tile
    constexpr int FI = TCO / 16, FJ = TK / 16;
    constexpr int CA = WG_M * BCO / 4 / 256, CB = WG_M * BK / 4 / 256;  // fp32 16-B chunks per thread per stage
    constexpr int PL = WG_M * 256;                                      // one bf16 plane, bytes
    extern __shared__ __attribute__((aligned(16))) char smem[];          // [2][Ah, Al, Bh, Bl]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wc = wid % WCO, wk = wid / WCO;
    const int Kt = a.KH * a.KW * a.C;
    const int nco = (a.Co + BCO - 1) / BCO, nkt = (Kt + BK - 1) / BK;
    const int tile = blockIdx.x % (nco * nkt), split = blockIdx.x / (nco * nkt);
    const int co0 = (tile % nco) * BCO, k0 = (tile / nco) * BK;
    const int mbeg = split * a.m_per_split, mend = min(a.M, mbeg + a.m_per_split);
    if (mbeg >= mend) return;
    WgGather gb[CB];
#pragma unroll
    for (int u = 0; u < CB; ++u) {
        const int q = tid + 256 * u;
        gb[u].init(a, k0 + (q % (BK / 4)) * 4, mbeg + q / (BK / 4), Kt);
    }
    f32x4v ra[CA], rb[CB];
    auto load = [&](int mb) {
#pragma unroll
        for (int u = 0; u < CA; ++u) {
            const int q = tid + 256 * u;
            const int r = q / (BCO / 4), cc = (q % (BCO / 4)) * 4;
            const int m = mb + r, co = co0 + cc;
            ra[u] = (m < mend && co < a.Co) ? *reinterpret_cast<const f32x4v*>(a.dY + (size_t)m * a.Co + co)
                                            : f32x4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            rb[u] = gb[u].load(a, mend);
            gb[u].step(a);
        }
    };
    // 4 fp32 at (row r, column col .. col + 3) -> 8 B of the hi plane + 8 B of the lo plane
    auto put = [&](char* hp, char* lp, int r, int col, const f32x4v& v) {
        const uint32_t h0 = pack_bf2(v[0], v[1]), h1 = pack_bf2(v[2], v[3]);
        const uint32_t l0 = pack_bf2(v[0] - lo_bf(h0), v[1] - hi_bf(h0));
        const uint32_t l1 = pack_bf2(v[2] - lo_bf(h1), v[3] - hi_bf(h1));
        const int off = r * 256 + (((col >> 3) ^ wgs_swz(r)) << 4) + ((col & 4) << 1);
        *reinterpret_cast<u32x2*>(hp + off) = u32x2{h0, h1};
        *reinterpret_cast<u32x2*>(lp + off) = u32x2{l0, l1};
    };
    auto store = [&](int buf) {
        char* b = smem + buf * 4 * PL;
#pragma unroll
        for (int u = 0; u < CA; ++u) {
            const int q = tid + 256 * u;
            put(b, b + PL, q / (BCO / 4), (q % (BCO / 4)) * 4, ra[u]);
        }
#pragma unroll
        for (int u = 0; u < CB; ++u) {
            const int q = tid + 256 * u;
            put(b + 2 * PL, b + 3 * PL, q / (BK / 4), (q % (BK / 4)) * 4, rb[u]);
        }
    };
    f32x4 acc[FI][FJ];
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // transposed-read addressing (as wgrad_v3_kernel): group g reads rows r1 + q and r1 + 16 + q
    const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
    const int r1 = (g & 1) * 8 + (g >> 1) * 4 + q4, r2 = r1 + 16;
    int offa[FI][2], offb[FJ][2];
#pragma unroll
    for (int i = 0; i < FI; ++i) {
        const int ca = (wc * TCO) / 8 + 2 * i + (p4 >> 1);
        offa[i][0] = r1 * 256 + ((ca ^ wgs_swz(r1)) << 4) + 8 * (p4 & 1);
        offa[i][1] = r2 * 256 + ((ca ^ wgs_swz(r2)) << 4) + 8 * (p4 & 1);
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
        const int cb = (wk * TK) / 8 + 2 * j + (p4 >> 1);
        offb[j][0] = r1 * 256 + ((cb ^ wgs_swz(r1)) << 4) + 8 * (p4 & 1);
        offb[j][1] = r2 * 256 + ((cb ^ wgs_swz(r2)) << 4) + 8 * (p4 & 1);
    }
    auto frag = [&](const char* plane, const int (&o)[2]) {
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(plane + o[0]));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(s16x4))(plane + o[1]));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    const int nst = (mend - mbeg + WG_M - 1) / WG_M;
    load(mbeg);
    store(0);
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
        const int buf = s & 1;
        if (s + 1 < nst) load(mbeg + (s + 1) * WG_M);
        const char* b = smem + buf * 4 * PL;
        bf16x8 ah[FI], al[FI], bh[FJ], bl[FJ];
#pragma unroll
        for (int i = 0; i < FI; ++i) {
            ah[i] = frag(b, offa[i]);
            al[i] = frag(b + PL, offa[i]);
        }
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            bh[j] = frag(b + 2 * PL, offb[j]);
            bl[j] = frag(b + 3 * PL, offb[j]);
        }
#pragma unroll
        for (int i = 0; i < FI; ++i)
#pragma unroll
            for (int j = 0; j < FJ; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
            }
        if (s + 1 < nst) {  // buf ^ 1 was last read in stage s - 1, before its closing barrier
            store(buf ^ 1);
            __syncthreads();
        }
    }
    // lane: rows (co) co0 + wc*TCO + i*16 + 4g + r, column (k) k0 + wk*TK + j*16 + (lane & 15)
    const int fr = lane & 15;
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) {
            const int k = k0 + wk * TK + j * 16 + fr;
            if (k >= Kt) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = co0 + wc * TCO + i * 16 + 4 * g + r;
                if (co < a.Co) atomicAdd(a.dW + (size_t)co * Kt + k, acc[i][j][r]);
            }
        }
}

// ------------------------------------------------------------------ BatchNorm
// Partial sums per block over rows [r0, r1): slab[blk][q][C], q = 0: sum(v - s), 1: sum((v - s)^2)
// (forward; s = shift[c]) or q = 0: sum(g'), 1: sum(g' * xhat) (backward; g' = g masked by y > 0).
// Thread layout: C/4 threads per row (f32x4), 256 / (C/4) rows per pass.
constexpr int BN_MAXB = 1024;

template <bool BWD>
__global__ __launch_bounds__(256) void bn_partial_f32_kernel(const float* __restrict__ x,
                                                             const float* __restrict__ g,
                                                             const float* __restrict__ y,
                                                             const float* __restrict__ stat,  // shift | mean,rstd
                                                             float* __restrict__ slab, long R, int C) {
    // channel slice blockIdx.y of CW = min(C, 1024) channels (4 per thread): C = 2048 (the ResNet-50/101/152
    // bottleneck outputs) takes two slices
    const int CW = C < 1024 ? C : 1024;
    const int cpr = CW / 4, rpb = 256 / cpr, tid = threadIdx.x;
    const int ch = tid % cpr, c0 = (int)blockIdx.y * CW + ch * 4;
    const bool active = tid < rpb * cpr;
    f32x4v s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s1, sh = s1, rs = s1;
    if (active) {
        sh = *reinterpret_cast<const f32x4v*>(stat + c0);
        if (BWD) rs = *reinterpret_cast<const f32x4v*>(stat + C + c0);
    }
    const long rows_per_blk = (R + gridDim.x - 1) / gridDim.x;
    const long r0 = (long)blockIdx.x * rows_per_blk, r1 = min(R, r0 + rows_per_blk);
    if (active)
        for (long r = r0 + tid / cpr; r < r1; r += rpb) {
            const size_t off = (size_t)r * C + c0;
            const f32x4v xv = *reinterpret_cast<const f32x4v*>(x + off);
            if (!BWD) {
                const f32x4v d = xv - sh;
                s1 += d;
                s2 += d * d;
            } else {
                f32x4v gv = *reinterpret_cast<const f32x4v*>(g + off);
                if (y) {
                    const f32x4v yv = *reinterpret_cast<const f32x4v*>(y + off);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (!(yv[q] > 0.f)) gv[q] = 0.f;
                }
                s1 += gv;
                s2 += gv * ((xv - sh) * rs);
            }
        }
    __shared__ float red[2][256 * 4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        red[0][tid * 4 + q] = s1[q];
        red[1][tid * 4 + q] = s2[q];
    }
    __syncthreads();
    for (int c = tid; c < CW; c += 256) {  // fixed-order fold over the rows of this block
        const int cc = c / 4, q = c % 4;
        float a1 = 0.f, a2 = 0.f;
        for (int rr = 0; rr < rpb; ++rr) {
            a1 += red[0][(rr * cpr + cc) * 4 + q];
            a2 += red[1][(rr * cpr + cc) * 4 + q];
        }
        const int cg = (int)blockIdx.y * CW + c;
        slab[((size_t)blockIdx.x * 2 + 0) * C + cg] = a1;
        slab[((size_t)blockIdx.x * 2 + 1) * C + cg] = a2;
    }
}

// fold of the per-block partials: 16 channels per 256-thread block (64-B coalesced slab rows), 16 fixed slab
// partitions per channel summed in double, then the 16 partition sums in order -> deterministic (one block
// per 64 channels with 4 partitions ran the 1024-row fold as 256 dependent loads: 70 us; FOLD_CH blocks now)
constexpr int FOLD_CH = 16;
__device__ __forceinline__ void fold_slab(const float* __restrict__ slab, int nb, int C, double& a1, double& a2,
                                          bool& active, int& c) {
    __shared__ double red[2][16][FOLD_CH];
    const int cl = threadIdx.x % FOLD_CH, part = threadIdx.x / FOLD_CH;
    c = blockIdx.x * FOLD_CH + cl;
    active = c < C;
    double s1 = 0.0, s2 = 0.0;
    if (active)
#pragma unroll 8
        for (int b = part; b < nb; b += 16) {  // loads batched, adds in order
            s1 += slab[((size_t)b * 2) * C + c];
            s2 += slab[((size_t)b * 2 + 1) * C + c];
        }
    red[0][part][cl] = s1;
    red[1][part][cl] = s2;
    __syncthreads();
    a1 = 0.0;
    a2 = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        a1 += red[0][q][cl];
        a2 += red[1][q][cl];
    }
    active = active && part == 0;
}

// forward fold: save[0..C) = mean, save[C..2C) = rstd; running stats (momentum, unbiased var)
__global__ __launch_bounds__(256) void bn_fold_fwd_f32_kernel(const float* __restrict__ slab, int nb,
                                                              const float* __restrict__ shift,
                                                              float* __restrict__ save, float* __restrict__ rmean,
                                                              float* __restrict__ rvar, long R, int C, float eps,
                                                              float momentum) {
    double a1, a2;
    bool active;
    int c;
    fold_slab(slab, nb, C, a1, a2, active, c);
    if (!active) return;
    const double md = a1 / (double)R;
    const double var = fmax(a2 / (double)R - md * md, 0.0);
    const float mean = (float)(md + shift[c]);
    save[c] = mean;
    save[C + c] = (float)(1.0 / sqrt(var + (double)eps));
    if (rmean) {
        rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
        rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(var * (double)R / (double)max(1L, R - 1));
    }
}

// backward fold: red[0..C) = sum(g'), red[C..2C) = sum(g' xhat); dbeta / dgamma accumulate
__global__ __launch_bounds__(256) void bn_fold_bwd_f32_kernel(const float* __restrict__ slab, int nb,
                                                              float* __restrict__ red, float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta, int C) {
    double a1, a2;
    bool active;
    int c;
    fold_slab(slab, nb, C, a1, a2, active, c);
    if (!active) return;
    red[c] = (float)a1;
    red[C + c] = (float)a2;
    if (dbeta) dbeta[c] += (float)a1;
    if (dgamma) dgamma[c] += (float)a2;
}

// y = (x - mean) rstd gamma + beta (+ res) (ReLU). FIXED: the grid stride (gridDim * 1024 elements) is a
// multiple of C, so a thread's 4 channels never change and their coefficients are loaded once
template <bool FIXED>
__global__ __launch_bounds__(256) void bn_apply_f32_kernel(const float* __restrict__ x, const float* __restrict__ save,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ res, float* __restrict__ y,
                                                           long n4, int C, int relu) {
    const long t0 = (long)blockIdx.x * 256 + threadIdx.x;
    float mean[4], sc[4], sh[4];
    auto coef = [&](int c0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = c0 + q;
            mean[q] = save[c];
            sc[q] = save[C + c] * gamma[c];
            sh[q] = beta[c];
        }
    };
    if (FIXED) coef((int)((t0 * 4) % C));
    for (long t = t0; t < n4; t += (long)gridDim.x * 256) {
        if (!FIXED) coef((int)((t * 4) % C));
        const f32x4v xv = reinterpret_cast<const f32x4v*>(x)[t];
        f32x4v o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = (xv[q] - mean[q]) * sc[q] + sh[q];
        if (res) o += reinterpret_cast<const f32x4v*>(res)[t];
        if (relu)
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = fmaxf(o[q], 0.f);
        reinterpret_cast<f32x4v*>(y)[t] = o;
    }
}

// dx = gamma rstd (g' - sum(g')/R - xhat sum(g' xhat)/R); dres = g' (when requested)
template <bool FIXED>  // as bn_apply_f32_kernel
__global__ __launch_bounds__(256) void bn_bwd_apply_f32_kernel(const float* __restrict__ g,
                                                               const float* __restrict__ y,
                                                               const float* __restrict__ x,
                                                               const float* __restrict__ save,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ red, float* __restrict__ dx,
                                                               float* __restrict__ dres, long n4, int C, float inv) {
    const long t0 = (long)blockIdx.x * 256 + threadIdx.x;
    // dx = gamma rstd (g' - sum(g')/R - (x - mean) rstd sum(g' xhat)/R)
    float mean[4], k1[4], r0[4], r1[4];
    auto coef = [&](int c0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int c = c0 + q;
            const float rstd = save[C + c];
            mean[q] = save[c];
            k1[q] = gamma[c] * rstd;
            r0[q] = red[c] * inv;
            r1[q] = rstd * (red[C + c] * inv);
        }
    };
    if (FIXED) coef((int)((t0 * 4) % C));
    for (long t = t0; t < n4; t += (long)gridDim.x * 256) {
        if (!FIXED) coef((int)((t * 4) % C));
        f32x4v gv = reinterpret_cast<const f32x4v*>(g)[t];
        if (y) {
            const f32x4v yv = reinterpret_cast<const f32x4v*>(y)[t];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (!(yv[q] > 0.f)) gv[q] = 0.f;
        }
        if (dres) reinterpret_cast<f32x4v*>(dres)[t] = gv;
        const f32x4v xv = reinterpret_cast<const f32x4v*>(x)[t];
        f32x4v o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = k1[q] * (gv[q] - r0[q] - (xv[q] - mean[q]) * r1[q]);
        reinterpret_cast<f32x4v*>(dx)[t] = o;
    }
}

// ------------------------------------------------------------------ pooling, FC bias, input
// maxpool k x k / s / p (k <= 3), NHWC, one thread per output pixel x 4 channels (16-B accesses);
// idx = argmax window slot per channel
__global__ __launch_bounds__(256) void maxpool_f32_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                          int OH, int OW, int k, int s, int p) {
    const int C4 = C / 4;
    const long total = (long)N * OH * OW * C4;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
        const int c = (int)(t % C4) * 4;
        const long pix = t / C4;
        const int ow = pix % OW, oh = (pix / OW) % OH, n = pix / ((long)OW * OH);
        f32x4v best = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        int bi[4] = {0, 0, 0, 0};
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < k; ++j) {
                const int ih = oh * s - p + i, iw = ow * s - p + j;
                if ((unsigned)ih >= (unsigned)H || (unsigned)iw >= (unsigned)W) continue;
                const f32x4v v = *reinterpret_cast<const f32x4v*>(x + (((size_t)n * H + ih) * W + iw) * C + c);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (v[q] > best[q] || (v[q] != v[q] && best[q] == best[q])) {
                        best[q] = v[q];
                        bi[q] = i * k + j;
                    }
            }
        *reinterpret_cast<f32x4v*>(y + pix * C + c) = best;
        *reinterpret_cast<uint32_t*>(idx + pix * C + c) =
            (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
    }
}

// gather form: dx[n][ih][iw][c] = sum of dy over the windows whose argmax is (ih, iw)
__global__ __launch_bounds__(256) void maxpool_bwd_f32_kernel(const float* __restrict__ dy,
                                                              const uint8_t* __restrict__ idx,
                                                              float* __restrict__ dx, int N, int H, int W, int C,
                                                              int OH, int OW, int k, int s, int p) {
    const int C4 = C / 4;
    const long total = (long)N * H * W * C4;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
        const int c = (int)(t % C4) * 4;
        const long pix = t / C4;
        const int iw = pix % W, ih = (pix / W) % H, n = pix / ((long)W * H);
        f32x4v acc = {0.f, 0.f, 0.f, 0.f};
        // windows (oh, ow) with oh*s - p <= ih <= oh*s - p + k - 1
        const int oh_lo = max(0, (ih + p - k + s) / s), oh_hi = min(OH - 1, (ih + p) / s);
        const int ow_lo = max(0, (iw + p - k + s) / s), ow_hi = min(OW - 1, (iw + p) / s);
        for (int oh = oh_lo; oh <= oh_hi; ++oh)
            for (int ow = ow_lo; ow <= ow_hi; ++ow) {
                const int i = ih - (oh * s - p), j = iw - (ow * s - p);
                if (i < 0 || i >= k || j < 0 || j >= k) continue;
                const size_t o = (((size_t)n * OH + oh) * OW + ow) * C + c;
                const uint32_t id4 = *reinterpret_cast<const uint32_t*>(idx + o);
                const f32x4v g = *reinterpret_cast<const f32x4v*>(dy + o);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (((id4 >> (8 * q)) & 0xff) == (uint32_t)(i * k + j)) acc[q] += g[q];
            }
        *reinterpret_cast<f32x4v*>(dx + pix * C + c) = acc;
    }
}

__global__ __launch_bounds__(256) void avgpool_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int N,
                                                          int HW, int C) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= N * C) return;
    const int n = t / C, c = t % C;
    float acc = 0.f;
    for (int i = 0; i < HW; ++i) acc += x[((size_t)n * HW + i) * C + c];
    y[t] = acc / (float)HW;
}

__global__ __launch_bounds__(256) void avgpool_bwd_f32_kernel(const float* __restrict__ dy, float* __restrict__ dx,
                                                              int N, int HW, int C) {
    const long total = (long)N * HW * C;
    const float inv = 1.f / (float)HW;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
        const int c = t % C;
        const int n = t / ((long)HW * C);
        dx[t] = dy[(size_t)n * C + c] * inv;
    }
}

// out[c] += sum_r x[r][c]  (FC bias gradient), fixed order
__global__ __launch_bounds__(256) void colsum_f32_kernel(const float* __restrict__ x, float* __restrict__ out, int R,
                                                         int C) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    float acc = 0.f;
    for (int r = 0; r < R; ++r) acc += x[(size_t)r * C + c];
    out[c] += acc;
}

// uint8 HWC (crop / flip) -> fp32 NHWC with Cp channels (3 real, the rest 0)
__global__ __launch_bounds__(256) void normalize_f32_kernel(const uint8_t* __restrict__ in, float* __restrict__ out,
                                                            const int* __restrict__ crop,
                                                            const uint8_t* __restrict__ flip, int B, int Hs, int Ws,
                                                            int H, int W, int Cp, float m0, float m1, float m2,
                                                            float is0, float is1, float is2) {
    const long total = (long)B * H * W;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
        const int w = t % W;
        const long r = t / W;
        const int h = r % H;
        const int b = r / H;
        const int oy = crop ? crop[2 * b] : 0, ox = crop ? crop[2 * b + 1] : 0;
        const int sw = (flip && flip[b]) ? (W - 1 - w) : w;
        const uint8_t* px = in + (((size_t)b * Hs + (h + oy)) * Ws + (sw + ox)) * 3;
        float* o = out + (size_t)t * Cp;
        o[0] = ((float)px[0] * (1.f / 255.f) - m0) * is0;
        o[1] = ((float)px[1] * (1.f / 255.f) - m1) * is1;
        o[2] = ((float)px[2] * (1.f / 255.f) - m2) * is2;
        for (int c = 3; c < Cp; ++c) o[c] = 0.f;
    }
}

int sgrid(long work) {
    long b = (work + 255) / 256;
    return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

int bn_blocks(long R, int C) {
    const int rpb = 256 / ((C < 1024 ? C : 1024) / 4);  // rows per block of one channel slice (bn_partial_f32)
    long b = (R + 4L * rpb - 1) / (4L * rpb);  // >= 4 rows per thread
    return (int)(b < BN_MAXB ? (b > 0 ? b : 1) : BN_MAXB);
}

}  // namespace

// ------------------------------------------------------------------ C ABI
// fp32 conv arithmetic: 0 exact f32 MFMA (igemm_f32_kernel, wgrad_f32_kernel), 1 the 3 x bf16 split
// (igemm_f32s_kernel, wgrad_f32s_kernel)
static int g_f32_split = [] {
    const char* e = getenv("IMAGENT_F32_SPLIT");
    return e ? atoi(e) : 0;
}();
IMK_EXPORT int imk_set_f32_split(int on) {
    g_f32_split = on ? 1 : 0;
    return 0;
}

// a.stats (a [STAT_SLOTS][2][Nout] slab, zeroed; shifted by a.shift): the BatchNorm statistics of the output,
// accumulated by the v3 split kernel's epilogue -> returns 0; any other kernel leaves the slab alone and returns
// 2 (the caller runs the statistics pass)
IMK_EXPORT int imk_conv_f32(const IGemmArgs* args, void* stream) {
    const IGemmArgs& a = *args;
    if (a.M <= 0 || a.Nout <= 0) return 0;
    if (a.C % 4 || (a.flags & ~(IG_ACCUM | IG_OUT_F32 | IG_BNBWD))) return -100;
    const int ntiles = ((a.M + F_BM - 1) / F_BM) * ((a.Nout + F_BN - 1) / F_BN);
    const size_t lds = 2 * (F_BM + F_BN) * F_BK * sizeof(float);  // (= the split kernel's 2 x 4 bf16 planes)
    // split arithmetic, C % 32 == 0: the v3 LDS-DMA ring with fp32 rows (conv_igemm_v3.h, EB = 4); the register-
    // staged kernel below for the rest
    if (g_f32_split && v3_ok32(a)) {
        const int r = a.Nout <= 64 ? launch_v3<128, 64, 1, 2, 4, 128, 4>(a, (hipStream_t)stream)
                                   : launch_v3<128, 128, 2, 2, 4, 128, 4>(a, (hipStream_t)stream);
        return r;
    }
    IGemmArgs b = a;
    b.stats = nullptr;  // the kernels below have no statistics / BN-backward epilogue
    b.flags &= ~IG_BNBWD;
    const int nost = a.stats ? 2 : 0;
    if (g_f32_split) {
        if (a.C % F_BK == 0)
            hipLaunchKernelGGL(igemm_f32s_kernel<0>, dim3(ntiles), dim3(256), lds, (hipStream_t)stream, b);
        else
            hipLaunchKernelGGL(igemm_f32s_kernel<1>, dim3(ntiles), dim3(256), lds, (hipStream_t)stream, b);
    } else if (a.C % F_BK == 0)
        hipLaunchKernelGGL(igemm_f32_kernel<0>, dim3(ntiles), dim3(256), lds, (hipStream_t)stream, b);
    else
        hipLaunchKernelGGL(igemm_f32_kernel<1>, dim3(ntiles), dim3(256), lds, (hipStream_t)stream, b);
    IMK_CHECK_LAUNCH();
    return nost;
}

// BatchNorm backward whose masked gradient g' and reductions came from the producing dgrad's epilogue (imk_conv_f32
// with IG_BNBWD: slab [STAT_SLOTS][2][C] = sum(g'), sum(g' xhat)): fold (dgamma / dbeta +=) + apply pass
IMK_EXPORT int imk_bn_bwd_slab_f32(const float* g, const float* x, const float* save, const float* gamma,
                                   const float* slab, float* red, float* dgamma, float* dbeta, float* dx, long R, int C,
                                   void* stream) {
    if (C % 4 || R <= 0) return -100;
    hipLaunchKernelGGL(bn_fold_bwd_f32_kernel, dim3((C + FOLD_CH - 1) / FOLD_CH), dim3(256), 0, (hipStream_t)stream,
                       slab, STAT_SLOTS, red, dgamma, dbeta, C);
    IMK_CHECK_LAUNCH();
    const long n4 = R * C / 4;
    const int grid = sgrid(n4);
    if ((long)grid * 1024 % C == 0)
        hipLaunchKernelGGL(bn_bwd_apply_f32_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, g, nullptr, x,
                           save, gamma, red, dx, nullptr, n4, C, 1.f / (float)R);
    else
        hipLaunchKernelGGL(bn_bwd_apply_f32_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, g, nullptr,
                           x, save, gamma, red, dx, nullptr, n4, C, 1.f / (float)R);
    IMK_CHECK_LAUNCH();
    return 0;
}

// training statistics from a conv epilogue's [STAT_SLOTS][2][C] slab of sums shifted by `shift` (imk_conv_f32
// with a.stats): save <- (mean, rstd), running stats updated (as imk_bn_stats_f32, one launch, no pass over x)
IMK_EXPORT int imk_bn_fold_slab_f32(const float* slab, const float* shift, float* save, float* rmean, float* rvar,
                                    long R, int C, float eps, float momentum, void* stream) {
    if (C <= 0 || R <= 0) return -100;
    hipLaunchKernelGGL(bn_fold_fwd_f32_kernel, dim3((C + FOLD_CH - 1) / FOLD_CH), dim3(256), 0, (hipStream_t)stream,
                       slab, STAT_SLOTS, shift, save, rmean, rvar, R, C, eps, momentum);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_wgrad_f32(const float* dy, const float* x, float* dw, int N, int H, int W, int C, int Co, int OH,
                             int OW, int KH, int KW, int stride, int pad, void* stream) {
    if (C % 4 || Co % 4) return -100;
    WgradF32Args a{dy, x, dw, N, H, W, C, Co, OH, OW, N * OH * OW, KH, KW, stride, pad, 0};
    const int Kt = KH * KW * C;
    const bool small = Co <= 64;
    const int BCO = small ? 64 : 128, BK = 128;
    const int tiles = ((Co + BCO - 1) / BCO) * ((Kt + BK - 1) / BK);
    // enough blocks for 2 per CU, at least 8 pixel stages per split
    int splits = (512 + tiles - 1) / tiles;
    const int max_splits = (a.M + 8 * WG_M - 1) / (8 * WG_M);
    splits = std::max(1, std::min(splits, max_splits));
    a.m_per_split = ((a.M + splits - 1) / splits + WG_M - 1) / WG_M * WG_M;
    splits = (a.M + a.m_per_split - 1) / a.m_per_split;
    if (g_f32_split) {  // 3 x bf16 split: hi / lo planes of [32 px][256 B], two buffers
        const size_t lds = 2 * 4 * WG_M * 256;
        if (small)
            hipLaunchKernelGGL((wgrad_f32s_kernel<64, 128>), dim3(tiles * splits), dim3(256), lds, (hipStream_t)stream, a);
        else
            hipLaunchKernelGGL((wgrad_f32s_kernel<128, 128>), dim3(tiles * splits), dim3(256), lds, (hipStream_t)stream,
                               a);
        IMK_CHECK_LAUNCH();
        return 0;
    }
    const size_t lds = 2 * 2 * WG_M * WG_P * sizeof(float);
    if (small)
        hipLaunchKernelGGL((wgrad_f32_kernel<64, 128>), dim3(tiles * splits), dim3(256), lds, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL((wgrad_f32_kernel<128, 128>), dim3(tiles * splits), dim3(256), lds, (hipStream_t)stream,
                           a);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_bn_slab_floats_f32(int C) { return BN_MAXB * 2 * C; }

// statistics-pass channel slices (bn_partial_f32_kernel): C <= 1024 with C / 4 dividing 256, or a
// multiple of 1024 (several 1024-channel slices)
static bool bn_f32_shape_ok(int C) {
    if (C % 4 || C <= 0) return false;
    return C <= 1024 ? 256 % (C / 4) == 0 : C % 1024 == 0;
}
static int bn_f32_slices(int C) { return C <= 1024 ? 1 : C / 1024; }

// training forward statistics: save <- (mean, rstd); running stats updated when rmean != null.
// shift: per-channel values near the mean (the previous batch mean) for the shifted sums.
IMK_EXPORT int imk_bn_stats_f32(const float* x, const float* shift, float* slab, float* save, float* rmean,
                                float* rvar, long R, int C, float eps, float momentum, void* stream) {
    if (!bn_f32_shape_ok(C)) return -100;
    const int nb = bn_blocks(R, C);
    // two passes: the mean (sums shifted by the caller's estimate), then the variance as the sum of
    // squares about that mean -- no E[x^2] - E[x]^2 cancellation (PyTorch uses Welford)
    for (int pass = 0; pass < 2; ++pass) {
        const float* sh = pass == 0 ? shift : save;
        hipLaunchKernelGGL((bn_partial_f32_kernel<false>), dim3(nb, bn_f32_slices(C)), dim3(256), 0, (hipStream_t)stream, x, nullptr,
                           nullptr, sh, slab, R, C);
        IMK_CHECK_LAUNCH();
        hipLaunchKernelGGL(bn_fold_fwd_f32_kernel, dim3((C + FOLD_CH - 1) / FOLD_CH), dim3(256), 0, (hipStream_t)stream, slab, nb,
                           sh, save, pass ? rmean : nullptr, rvar, R, C, eps, momentum);
        IMK_CHECK_LAUNCH();
    }
    return 0;
}

IMK_EXPORT int imk_bn_apply_f32(const float* x, const float* save, const float* gamma, const float* beta,
                                const float* res, float* y, long R, int C, int relu, void* stream) {
    if (C % 4) return -100;
    const long n4 = R * C / 4;
    const int grid = sgrid(n4);
    if ((long)grid * 1024 % C == 0)
        hipLaunchKernelGGL(bn_apply_f32_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, save, gamma,
                           beta, res, y, n4, C, relu);
    else
        hipLaunchKernelGGL(bn_apply_f32_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, save, gamma,
                           beta, res, y, n4, C, relu);
    IMK_CHECK_LAUNCH();
    return 0;
}

// backward: g' = g * (y > 0) (y null: no ReLU); red <- (sum g', sum g' xhat); dgamma/dbeta +=;
// dx = BN backward of g'; dres <- g' (nullable)
IMK_EXPORT int imk_bn_bwd_f32(const float* g, const float* y, const float* x, const float* save, const float* gamma,
                              float* slab, float* red, float* dgamma, float* dbeta, float* dx, float* dres, long R,
                              int C, void* stream) {
    if (!bn_f32_shape_ok(C)) return -100;
    const int nb = bn_blocks(R, C);
    hipLaunchKernelGGL((bn_partial_f32_kernel<true>), dim3(nb, bn_f32_slices(C)), dim3(256), 0, (hipStream_t)stream, x, g, y, save,
                       slab, R, C);
    IMK_CHECK_LAUNCH();
    hipLaunchKernelGGL(bn_fold_bwd_f32_kernel, dim3((C + FOLD_CH - 1) / FOLD_CH), dim3(256), 0, (hipStream_t)stream, slab, nb, red,
                       dgamma, dbeta, C);
    IMK_CHECK_LAUNCH();
    const long n4 = R * C / 4;
    const int grid = sgrid(n4);
    if ((long)grid * 1024 % C == 0)
        hipLaunchKernelGGL(bn_bwd_apply_f32_kernel<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, g, y, x, save,
                           gamma, red, dx, dres, n4, C, 1.f / (float)R);
    else
        hipLaunchKernelGGL(bn_bwd_apply_f32_kernel<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, g, y, x,
                           save, gamma, red, dx, dres, n4, C, 1.f / (float)R);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_maxpool_f32(const float* x, float* y, void* idx, int N, int H, int W, int C, int OH, int OW, int k,
                               int s, int p, void* stream) {
    if (k > 3 || C % 4) return -100;
    hipLaunchKernelGGL(maxpool_f32_kernel, dim3(sgrid((long)N * OH * OW * C / 4)), dim3(256), 0, (hipStream_t)stream, x,
                       y, (uint8_t*)idx, N, H, W, C, OH, OW, k, s, p);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_maxpool_bwd_f32(const float* dy, const void* idx, float* dx, int N, int H, int W, int C, int OH,
                                   int OW, int k, int s, int p, void* stream) {
    if (C % 4) return -100;
    hipLaunchKernelGGL(maxpool_bwd_f32_kernel, dim3(sgrid((long)N * H * W * C / 4)), dim3(256), 0, (hipStream_t)stream,
                       dy, (const uint8_t*)idx, dx, N, H, W, C, OH, OW, k, s, p);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_avgpool_f32(const float* x, float* y, int N, int HW, int C, void* stream) {
    hipLaunchKernelGGL(avgpool_f32_kernel, dim3((N * C + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, y, N, HW,
                       C);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_avgpool_bwd_f32(const float* dy, float* dx, int N, int HW, int C, void* stream) {
    hipLaunchKernelGGL(avgpool_bwd_f32_kernel, dim3(sgrid((long)N * HW * C)), dim3(256), 0, (hipStream_t)stream, dy,
                       dx, N, HW, C);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_colsum_f32(const float* x, float* out, int R, int C, void* stream) {
    hipLaunchKernelGGL(colsum_f32_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, out, R, C);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_normalize_u8_f32(const void* in, float* out, const int* crop, const void* flip, int B, int Hs,
                                    int Ws, int H, int W, int Cp, const float* mean, const float* std, void* stream) {
    hipLaunchKernelGGL(normalize_f32_kernel, dim3(sgrid((long)B * H * W)), dim3(256), 0, (hipStream_t)stream,
                       (const uint8_t*)in, out, crop, (const uint8_t*)flip, B, Hs, Ws, H, W, Cp, mean[0], mean[1],
                       mean[2], 1.f / std[0], 1.f / std[1], 1.f / std[2]);
    IMK_CHECK_LAUNCH();
    return 0;
}

// softmax-xent backward with an fp32 gradient (the bf16 path's imk_xent_bwd rounds dz to bf16)
namespace {
__global__ __launch_bounds__(256) void xent_bwd_f32_kernel(const float* __restrict__ logits,
                                                           const int64_t* __restrict__ labels,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ gout, float* __restrict__ dz,
                                                           int B, int NC, float smoothing) {
    const int row = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= NC) return;
    const float scale = gout[0] / (float)B;
    const float p = expf(logits[(size_t)row * NC + i] - lse[row]);
    const float t = (i == labels[row] ? 1.f - smoothing : 0.f) + smoothing / (float)NC;
    dz[(size_t)row * NC + i] = (p - t) * scale;
}
}  // namespace

IMK_EXPORT int imk_xent_bwd_f32(const float* logits, const int64_t* labels, const float* lse, const float* gout,
                                float* dz, int B, int NC, float smoothing, void* stream) {
    hipLaunchKernelGGL(xent_bwd_f32_kernel, dim3((NC + 255) / 256, B), dim3(256), 0, (hipStream_t)stream, logits,
                       labels, lse, gout, dz, B, NC, smoothing);
    IMK_CHECK_LAUNCH();
    return 0;
}
