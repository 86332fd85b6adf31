// Pooling, softmax cross-entropy + top-k, fused SGD, input normalisation and
// weight re-layout kernels for gfx950 (MI355X). NHWC bf16 activations.
//
// Reference counterparts:
//   K10/K11 max_pool2d_with_indices (+bwd)      -> maxpool_fwd / maxpool_bwd
//   K12     adaptive_avg_pool2d (+bwd)          -> avgpool_fwd / avgpool_bwd
//   K14-K16 log_softmax + nll_loss (+bwd), topk/eq/sum (accuracy(),
//           /root/reference/imagenet.py:63-79, :124, :134) -> xent_fwd / xent_bwd
//   K18     foreach SGD (imagenet.py:131, :325)  -> sgd_flat (one pass over
//           the flat param/grad/momentum arenas, also refreshes the bf16 shadow)
//   K21     ToTensor + Normalize (imagenet.py:280-283, CPU in the reference)
//           -> normalize_u8 (uint8 HWC -> bf16 NHWC, optional crop / flip)
//   K13     fc bias gradient -> colsum_bf16
//   -       bf16 weight shadows: [Co][T][Ci] -> [Ci][T][Co] for dgrad (batched)

#include <cstdlib>
#include <vector>

#include <hip/hip_ext.h>

#include "common.h"

namespace {

// ------------------------------------------------------------------ maxpool
// argmax stored per element as the in-window index (uint8), so the backward
// is a gather over the <= ceil(k/s)^2 windows that contain an input pixel.
// Flat grid-stride over (pixel, 8-channel chunk) with 32-bit unsigned index
// math. Every window's loads are issued before any is used, from clamped
// (always valid) addresses with the validity kept as a mask: the
// branch-per-window form waits one L2 round trip per window (the stem's pool
// backward measured 594 us, 4x its bytes; profiles/r50_b512_v5_kernel_stats.md).
// Optional BatchNorm(+ReLU) prologue for the stem (BNF): the pool reads the
// BN INPUT x and pools bf16(relu(x*sc + sh)) -- the BN output (4x the pool's
// output bytes) is never written or re-read. Per-channel constants from the
// finalized conv-epilogue statistics exactly as bn_fwd_kernel uses them (bn.hip).
struct PoolBnf {
    const float* sums;  // [2][C] mean, biased variance (imk_bn_stats_finalize)
    const float* gamma;
    const float* beta;
    float* save;        // [2][C] mean, rstd (for the backward)
    float inv_cnt, eps;
    bf16_t* xsel;       // optional: the BN input at each window's argmax, like y (the backward's BN sums)
};

template <int KMAX, bool BNF = false>  // KMAX > 0: k <= KMAX, windows unrolled; 0: generic k
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H,
                                                          int W, int C, int OH, int OW, int k, int s,
                                                          int p, PoolBnf bnf = {}) {
    const uint32_t cpr = C / 8;
    const uint32_t total = (uint32_t)N * OH * OW * cpr;
    float bsc[8], bsh[8];
    if constexpr (BNF) {  // fixed channel chunk per thread (256 % cpr == 0, host check)
        const uint32_t t0 = blockIdx.x * 256u + threadIdx.x;
        const int c0 = (int)(t0 % cpr) * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float mean = bnf.sums[c0 + i];  // finalized (mean, biased variance)
            const float rstd = rsqrtf(bnf.sums[C + c0 + i] + bnf.eps);
            bsc[i] = rstd * bnf.gamma[c0 + i];
            bsh[i] = bnf.beta[c0 + i] - mean * bsc[i];
            if (t0 < cpr) {
                bnf.save[c0 + i] = mean;
                bnf.save[C + c0 + i] = rstd;
            }
        }
    }
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < total; t += gridDim.x * 256u) {
        const uint32_t pix = t / cpr, ch = t - pix * cpr;
        const uint32_t row = pix / (uint32_t)OW, ow = pix - row * OW;
        const uint32_t n = row / (uint32_t)OH, oh = row - n * OH;
        const bf16_t* xn = x + (size_t)n * H * W * C + ch * 8;
        float best[8];
        int bi[8];
        uint32_t bx[8];  // BNF: the raw bf16 input at the argmax
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            best[i] = -INFINITY;
            bi[i] = 0;
            bx[i] = 0;
        }
        auto take = [&](const u32x4& w, bool ok, int win) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float a = lo_bf(w[i]), b = hi_bf(w[i]);
                if constexpr (BNF) {  // the bf16 value the unfused BN+ReLU would have stored
                    a = bf2f(f2bf(fmaxf(fmaf(a, bsc[2 * i], bsh[2 * i]), 0.f)));
                    b = bf2f(f2bf(fmaxf(fmaf(b, bsc[2 * i + 1], bsh[2 * i + 1]), 0.f)));
                }
                // strict > keeps the first maximum (torch semantics); NaN propagates
                if (ok && (a > best[2 * i] || (a != a && best[2 * i] == best[2 * i]))) {
                    best[2 * i] = a;
                    bi[2 * i] = win;
                    bx[2 * i] = w[i] & 0xffffu;
                }
                if (ok && (b > best[2 * i + 1] || (b != b && best[2 * i + 1] == best[2 * i + 1]))) {
                    best[2 * i + 1] = b;
                    bi[2 * i + 1] = win;
                    bx[2 * i + 1] = w[i] >> 16;
                }
            }
        };
        if constexpr (KMAX > 0) {
            constexpr int KK = KMAX > 0 ? KMAX * KMAX : 1;
            u32x4 v[KK];
            bool ok[KK];
#pragma unroll
            for (int dh = 0; dh < KMAX; ++dh)
#pragma unroll
                for (int dw = 0; dw < KMAX; ++dw) {
                    const int ih = (int)oh * s - p + dh, iw = (int)ow * s - p + dw;
                    ok[dh * KMAX + dw] = dh < k && dw < k && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
                    const int ihc = min(max(ih, 0), H - 1), iwc = min(max(iw, 0), W - 1);
                    v[dh * KMAX + dw] = *reinterpret_cast<const u32x4*>(xn + ((size_t)ihc * W + iwc) * C);
                }
#pragma unroll
            for (int dh = 0; dh < KMAX; ++dh)
#pragma unroll
                for (int dw = 0; dw < KMAX; ++dw) take(v[dh * KMAX + dw], ok[dh * KMAX + dw], dh * k + dw);
        } else {
            for (int dh = 0; dh < k; ++dh) {
                const int ih = (int)oh * s - p + dh;
                if ((unsigned)ih >= (unsigned)H) continue;
                for (int dw = 0; dw < k; ++dw) {
                    const int iw = (int)ow * s - p + dw;
                    if ((unsigned)iw >= (unsigned)W) continue;
                    take(*reinterpret_cast<const u32x4*>(xn + ((size_t)ih * W + iw) * C), true, dh * k + dw);
                }
            }
        }
        u32x4 o;
        uint32_t i0 = 0, i1 = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = pack_bf2(best[2 * i], best[2 * i + 1]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            i0 |= (uint32_t)bi[i] << (8 * i);
            i1 |= (uint32_t)bi[4 + i] << (8 * i);
        }
        const size_t off = (size_t)pix * C + ch * 8;
        *reinterpret_cast<u32x4*>(y + off) = o;
        if (idx) *reinterpret_cast<u32x2*>(idx + off) = u32x2{i0, i1};
        if constexpr (BNF) {
            if (bnf.xsel) {
                u32x4 xs;
#pragma unroll
                for (int i = 0; i < 4; ++i) xs[i] = bx[2 * i] | (bx[2 * i + 1] << 16);
                *reinterpret_cast<u32x4*>(bnf.xsel + off) = xs;
            }
        }
    }
}

// Optional BatchNorm-backward epilogue for the stem (BNR): the pool's input
// gradient g is the upstream gradient of BN+ReLU(x); the kernel stores it
// ReLU-masked (mask recomputed from x) and reduces sum(g*xhat), sum(g) per
// channel into slot (block & 31) of the BN's [32][3][C] backward slab -- the
// separate reduce pass over (g, x) disappears (bn.hip bn_bwd_reduce_kernel).
struct PoolBnr {
    const bf16_t* x;     // BN input, NHWC like dx
    const float* save;   // [2][C] mean, rstd
    const float* gamma;
    const float* beta;
    float* slab;         // [32][3][C]
    const bf16_t* xsel;  // quad kernel, BNR 2: the BN input at each window's argmax (maxpool_fwd_kernel BNF), like dy
};

// WMAX > 0: at most WMAX candidate windows per dimension (ceil(k/s) <= WMAX),
// unrolled; 0: generic
template <int WMAX, bool BNR = false>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx,
                                                          bf16_t* __restrict__ dx, int N, int H, int W,
                                                          int C, int OH, int OW, int k, int s, int p,
                                                          PoolBnr bnr = {}) {
    const uint32_t cpr = C / 8;
    const uint32_t total = (uint32_t)N * H * W * cpr;
    // BNR: the thread's channel chunk is fixed (256 % cpr == 0, host check)
    const int cfix = (int)((blockIdx.x * 256u + threadIdx.x) % cpr) * 8;
    float mean[8], rstd[8], sc[8], sh[8], sgx[8], sg[8];
    if constexpr (BNR) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            mean[i] = bnr.save[cfix + i];
            rstd[i] = bnr.save[C + cfix + i];
            sc[i] = rstd[i] * bnr.gamma[cfix + i];
            sh[i] = bnr.beta[cfix + i] - mean[i] * sc[i];
            sgx[i] = sg[i] = 0.f;
        }
    }
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < total; t += gridDim.x * 256u) {
        const uint32_t pix = t / cpr, ch = t - pix * cpr;
        const uint32_t row = pix / (uint32_t)W, iw = pix - row * W;
        const uint32_t n = row / (uint32_t)H, ih = row - n * H;
        const size_t nbase = (size_t)n * OH * OW * C + ch * 8;
        float acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
        auto add = [&](const u32x4& g, const u32x2& ii, bool ok, int want) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t w = i < 2 ? ii[0] : ii[1];
                const int sh = 16 * (i & 1);
                if (ok && (int)((w >> sh) & 0xff) == want) acc[2 * i] += lo_bf(g[i]);
                if (ok && (int)((w >> (sh + 8)) & 0xff) == want) acc[2 * i + 1] += hi_bf(g[i]);
            }
        };
        // windows containing (ih, iw): oh in [oh_hi - WMAX + 1, oh_hi], oh_hi = (ih + p) / s
        const int oh_hi = ((int)ih + p) / s, ow_hi = ((int)iw + p) / s;
        if constexpr (WMAX > 0) {
            constexpr int WW = WMAX > 0 ? WMAX * WMAX : 1;
            u32x4 g[WW];
            u32x2 ii[WW];
            bool ok[WW];
            int want[WW];
#pragma unroll
            for (int a = 0; a < WMAX; ++a)
#pragma unroll
                for (int b = 0; b < WMAX; ++b) {
                    const int oh = oh_hi - a, ow = ow_hi - b, q = a * WMAX + b;
                    const int dh = (int)ih - (oh * s - p), dw = (int)iw - (ow * s - p);
                    ok[q] = oh >= 0 && oh < OH && ow >= 0 && ow < OW && dh < k && dw < k;
                    want[q] = dh * k + dw;
                    const size_t off = nbase + ((size_t)min(max(oh, 0), OH - 1) * OW + min(max(ow, 0), OW - 1)) * C;
                    g[q] = *reinterpret_cast<const u32x4*>(dy + off);
                    ii[q] = *reinterpret_cast<const u32x2*>(idx + off);
                }
#pragma unroll
            for (int q = 0; q < WMAX * WMAX; ++q) add(g[q], ii[q], ok[q], want[q]);
        } else {
            const int oh_lo = max(0, ((int)ih + p - k + s) / s), ow_lo = max(0, ((int)iw + p - k + s) / s);
            for (int oh = oh_lo; oh <= min(OH - 1, oh_hi); ++oh) {
                const int dh = (int)ih - (oh * s - p);
                if (dh < 0 || dh >= k) continue;
                for (int ow = ow_lo; ow <= min(OW - 1, ow_hi); ++ow) {
                    const int dw = (int)iw - (ow * s - p);
                    if (dw < 0 || dw >= k) continue;
                    const size_t off = nbase + ((size_t)oh * OW + ow) * C;
                    add(*reinterpret_cast<const u32x4*>(dy + off), *reinterpret_cast<const u32x2*>(idx + off), true,
                        dh * k + dw);
                }
            }
        }
        if constexpr (BNR) {  // ReLU mask from x, statistics of the stored (bf16) gradient
            const u32x4 xw = *reinterpret_cast<const u32x4*>(bnr.x + (size_t)pix * C + ch * 8);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float xv = i & 1 ? hi_bf(xw[i >> 1]) : lo_bf(xw[i >> 1]);
                if (!(fmaf(xv, sc[i], sh[i]) > 0.f)) acc[i] = 0.f;
                const float gq = bf2f(f2bf(acc[i]));
                sg[i] += gq;
                sgx[i] += gq * ((xv - mean[i]) * rstd[i]);
            }
        }
        u32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = pack_bf2(acc[2 * i], acc[2 * i + 1]);
        *reinterpret_cast<u32x4*>(dx + (size_t)pix * C + ch * 8) = o;
    }
    if constexpr (BNR) {
        // lanes sharing a channel chunk: xor-fold over lane offsets cpr .. 32,
        // then LDS adds across the block's waves, one global atomic per
        // channel and quantity into the block's slab slot
        __shared__ float red[2][2048];
        const int lane = threadIdx.x & 63;
        for (int c = threadIdx.x; c < 2 * C; c += 256) red[c / C][c % C] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            for (int o2 = (int)cpr; o2 < 64; o2 <<= 1) {
                sg[i] += __shfl_xor(sg[i], o2, 64);
                sgx[i] += __shfl_xor(sgx[i], o2, 64);
            }
        __syncthreads();
        if (lane < (int)cpr) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                atomicAdd(&red[0][cfix + i], sgx[i]);
                atomicAdd(&red[1][cfix + i], sg[i]);
            }
        }
        __syncthreads();
        float* slot = bnr.slab + (size_t)(blockIdx.x & 31) * 3 * C;
        for (int c = threadIdx.x; c < 2 * C; c += 256) atomicAdd(slot + (c / C) * C + c % C, red[c / C][c % C]);
    }
}

// 3x3 / stride 2 / pad 1 max-pool backward with H = 2 OH, W = 2 OW (the ResNet
// stem pool), one thread per 2x2 input quad and 8-channel chunk: the quad
// (2i + a, 2j + b) is covered by exactly the windows (i + {0, 1}, j + {0, 1}),
// so each window's gradient and argmax are loaded once per quad instead of
// once per input pixel (4 + 4 loads per 4 pixels instead of 16 + 16). Input
// pixel (a, b) takes window (i + u, j + v) iff (u == 0 || a == 1) and
// (v == 0 || b == 1), at window offset (1 + a - 2u) * 3 + (1 + b - 2v).
// BNR 1: ReLU mask and BN sums from the BN input x at every input pixel (as
// maxpool_bwd_kernel); BNR 2: from the forward's per-window argmax input xsel
// instead -- a pixel only receives gradient as some window's argmax, so its
// mask and x are that window's (the same sums, term for term): x (4x the
// pooled bytes) is not read.
template <int BNR, bool NT = false>
__global__ __launch_bounds__(256) void maxpool_bwd_quad_kernel(const bf16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx,
                                                               bf16_t* __restrict__ dx, int N, int C, int OH,
                                                               int OW, PoolBnr bnr) {
    const uint32_t cpr = C / 8;
    const uint32_t total = (uint32_t)N * OH * OW * cpr;
    const int H = 2 * OH, W = 2 * OW;
    const int cfix = (int)((blockIdx.x * 256u + threadIdx.x) % cpr) * 8;
    float mean[8], rstd[8], sc[8], sh[8], sgx[8], sg[8];
    if constexpr (BNR) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            mean[i] = bnr.save[cfix + i];
            rstd[i] = bnr.save[C + cfix + i];
            sc[i] = rstd[i] * bnr.gamma[cfix + i];
            sh[i] = bnr.beta[cfix + i] - mean[i] * sc[i];
            sgx[i] = sg[i] = 0.f;
        }
    }
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < total; t += gridDim.x * 256u) {
        const uint32_t q = t / cpr, ch = t - q * cpr;
        const uint32_t qrow = q / (uint32_t)OW, j = q - qrow * OW;
        const uint32_t n = qrow / (uint32_t)OH, i = qrow - n * OH;
        u32x4 g[4];
        u32x2 ii[4];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const bool ok = (int)i + u < OH && (int)j + v < OW;
                const size_t off = (((size_t)n * OH + i + (ok ? u : 0)) * OW + j + (ok ? v : 0)) * C + ch * 8;
                g[u * 2 + v] = ok ? *reinterpret_cast<const u32x4*>(dy + off) : u32x4{0u, 0u, 0u, 0u};
                ii[u * 2 + v] = ok ? *reinterpret_cast<const u32x2*>(idx + off) : u32x2{0xffffffffu, 0xffffffffu};
            }
        u32x4 xs[4];
        if constexpr (BNR == 2) {  // each window's ReLU mask from its argmax input, applied to its gradient
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    const bool ok = (int)i + u < OH && (int)j + v < OW;
                    const size_t off = (((size_t)n * OH + i + (ok ? u : 0)) * OW + j + (ok ? v : 0)) * C + ch * 8;
                    xs[u * 2 + v] = *reinterpret_cast<const u32x4*>(bnr.xsel + off);
                    u32x4& gg = g[u * 2 + v];
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        uint32_t gw = gg[c];
                        if (!(fmaf(lo_bf(xs[u * 2 + v][c]), sc[2 * c], sh[2 * c]) > 0.f)) gw &= 0xffff0000u;
                        if (!(fmaf(hi_bf(xs[u * 2 + v][c]), sc[2 * c + 1], sh[2 * c + 1]) > 0.f)) gw &= 0x0000ffffu;
                        gg[c] = gw;
                    }
                }
        }
        u32x4 xw[4];
        if constexpr (BNR == 1) {
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    xw[a * 2 + b] = *reinterpret_cast<const u32x4*>(
                        bnr.x + (((size_t)n * H + 2 * i + a) * W + 2 * j + b) * C + ch * 8);
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                float acc[8], xv[8];  // xv (BNR 2): the pixel's x, from a window that took it
#pragma unroll
                for (int c = 0; c < 8; ++c) acc[c] = xv[c] = 0.f;
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int v = 0; v < 2; ++v) {
                        if ((u == 1 && a == 0) || (v == 1 && b == 0)) continue;
                        const int want = (1 + a - 2 * u) * 3 + (1 + b - 2 * v);
                        const u32x4 gg = g[u * 2 + v];
                        const u32x2 w2 = ii[u * 2 + v];
#pragma unroll
                        for (int c = 0; c < 4; ++c) {
                            const uint32_t w = c < 2 ? w2[0] : w2[1];
                            const int s8 = 16 * (c & 1);
                            if ((int)((w >> s8) & 0xff) == want) {
                                acc[2 * c] += lo_bf(gg[c]);
                                if constexpr (BNR == 2) xv[2 * c] = lo_bf(xs[u * 2 + v][c]);
                            }
                            if ((int)((w >> (s8 + 8)) & 0xff) == want) {
                                acc[2 * c + 1] += hi_bf(gg[c]);
                                if constexpr (BNR == 2) xv[2 * c + 1] = hi_bf(xs[u * 2 + v][c]);
                            }
                        }
                    }
                if constexpr (BNR == 2) {
#pragma unroll
                    for (int c = 0; c < 8; ++c) {
                        const float gq = bf2f(f2bf(acc[c]));
                        sg[c] += gq;
                        sgx[c] += gq * ((xv[c] - mean[c]) * rstd[c]);
                    }
                }
                if constexpr (BNR == 1) {
                    const u32x4 x4 = xw[a * 2 + b];
#pragma unroll
                    for (int c = 0; c < 8; ++c) {
                        const float xv = c & 1 ? hi_bf(x4[c >> 1]) : lo_bf(x4[c >> 1]);
                        if (!(fmaf(xv, sc[c], sh[c]) > 0.f)) acc[c] = 0.f;
                        const float gq = bf2f(f2bf(acc[c]));
                        sg[c] += gq;
                        sgx[c] += gq * ((xv - mean[c]) * rstd[c]);
                    }
                }
                u32x4 o;
#pragma unroll
                for (int c = 0; c < 4; ++c) o[c] = pack_bf2(acc[2 * c], acc[2 * c + 1]);
                u32x4* dst = reinterpret_cast<u32x4*>(dx + (((size_t)n * H + 2 * i + a) * W + 2 * j + b) * C + ch * 8);
                if (NT) __builtin_nontemporal_store(o, dst);
                else *dst = o;
            }
    }
    if constexpr (BNR) {  // as maxpool_bwd_kernel: lane xor-fold, LDS adds, one atomic per channel
        __shared__ float red[2][2048];
        const int lane = threadIdx.x & 63;
        for (int c = threadIdx.x; c < 2 * C; c += 256) red[c / C][c % C] = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c)
            for (int o2 = (int)cpr; o2 < 64; o2 <<= 1) {
                sg[c] += __shfl_xor(sg[c], o2, 64);
                sgx[c] += __shfl_xor(sgx[c], o2, 64);
            }
        __syncthreads();
        if (lane < (int)cpr) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                atomicAdd(&red[0][cfix + c], sgx[c]);
                atomicAdd(&red[1][cfix + c], sg[c]);
            }
        }
        __syncthreads();
        float* slot = bnr.slab + (size_t)(blockIdx.x & 31) * 3 * C;
        for (int c = threadIdx.x; c < 2 * C; c += 256) atomicAdd(slot + (c / C) * C + c % C, red[c / C][c % C]);
    }
}

// the quad backward's output (4x the bytes it reads) with non-temporal stores: scripts/pool_bench.py at 4096 img,
// one box, twice each: 2,583 / 2,583 us plain vs 2,539 / 2,536 us NT (scripts/runs/pool_ab.sh). IMAGENT_POOL_NT=0: off
static bool pool_nt() {
    static const bool v = [] {
        const char* e = getenv("IMAGENT_POOL_NT");
        return e && *e ? atoi(e) != 0 : true;
    }();
    return v;
}

// the stem pool's quad-gather backward covers 3x3 / stride 2 / pad 1 on even inputs
bool pool_quad_ok(int H, int W, int OH, int OW, int k, int s, int p) {
    return k == 3 && s == 2 && p == 1 && H == 2 * OH && W == 2 * OW;
}

// ------------------------------------------------------------------ avgpool
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ y, int N, int HW, int C) {
    const int cpr = C / 8;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= N * cpr) return;
    const int n = t / cpr, ch = t % cpr;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16_t* p = x + (size_t)n * HW * C + ch * 8;
    for (int i = 0; i < HW; ++i) {
        const u32x4 w = *reinterpret_cast<const u32x4*>(p + (size_t)i * C);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc[2 * j] += lo_bf(w[j]);
            acc[2 * j + 1] += hi_bf(w[j]);
        }
    }
    const float inv = 1.f / (float)HW;
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = pack_bf2(acc[2 * j] * inv, acc[2 * j + 1] * inv);
    *reinterpret_cast<u32x4*>(y + (size_t)n * C + ch * 8) = o;
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          bf16_t* __restrict__ dx, int N, int HW, int C) {
    const int cpr = C / 8;
    const long total = (long)N * HW * cpr;
    const float inv = 1.f / (float)HW;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
        const int ch = t % cpr;
        const long pix = t / cpr;
        const int n = pix / HW;
        const u32x4 g = *reinterpret_cast<const u32x4*>(dy + (size_t)n * C + ch * 8);
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = pack_bf2(lo_bf(g[j]) * inv, hi_bf(g[j]) * inv);
        *reinterpret_cast<u32x4*>(dx + pix * C + ch * 8) = o;
    }
}

// ------------------------------------------------------- softmax xent + top-k
// one wave per row. metrics[0] += loss, [1] += top1 hits, [2] += top5 hits, [3] += rows
__global__ __launch_bounds__(256) void xent_fwd_kernel(const float* __restrict__ logits,
                                                       const int64_t* __restrict__ labels,
                                                       float* __restrict__ lse_out,
                                                       float* __restrict__ loss_mean,
                                                       float* __restrict__ metrics, int B, int NC,
                                                       float smoothing) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= B) return;
    const float* z = logits + (size_t)row * NC;
    const int64_t lab = labels[row];
    float mx = -INFINITY;
    for (int i = lane; i < NC; i += 64) mx = fmaxf(mx, z[i]);
    mx = wave_max(mx);
    float se = 0.f, sz = 0.f;
    for (int i = lane; i < NC; i += 64) {
        se += expf(z[i] - mx);  // precise exp/log: B x NC elements, the fp32 path's loss
        sz += z[i];
    }
    se = wave_sum(se);
    sz = wave_sum(sz);
    const float lse = mx + logf(se);
    const float zl = (lab >= 0 && lab < NC) ? z[lab] : 0.f;
    // rank of the label: #classes with a strictly larger logit
    int gt = 0;
    for (int i = lane; i < NC; i += 64) gt += z[i] > zl;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) gt += __shfl_xor(gt, o, 64);
    if (lane == 0) {
        const float nll = lse - zl;
        const float loss = (1.f - smoothing) * nll + smoothing * (lse - sz / (float)NC);
        lse_out[row] = lse;
        atomicAdd(loss_mean, loss / (float)B);
        if (metrics) {
            atomicAdd(metrics + 0, loss);
            atomicAdd(metrics + 1, gt < 1 ? 1.f : 0.f);
            atomicAdd(metrics + 2, gt < 5 ? 1.f : 0.f);
            atomicAdd(metrics + 3, 1.f);
        }
    }
}

// dlogits = g/B * (softmax - (1-eps)*onehot - eps/NC), bf16 out (feeds the fc dgrad/wgrad)
__global__ __launch_bounds__(256) void xent_bwd_kernel(const float* __restrict__ logits,
                                                       const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ gout,
                                                       bf16_t* __restrict__ dz, int B, int NC,
                                                       float smoothing) {
    const int row = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= NC) return;
    const float scale = gout[0] / (float)B;
    const float p = __expf(logits[(size_t)row * NC + i] - lse[row]);
    const float t = (i == labels[row] ? 1.f - smoothing : 0.f) + smoothing / (float)NC;
    dz[(size_t)row * NC + i] = f2bf((p - t) * scale);
}

// out[c] += sum_r x[r][c]. Block = 64 columns x 4 row lanes, blockIdx.y = a
// slice of rows: every thread sums a few rows (one column per thread, 128-B
// coalesced row segments per wave), the 4 row lanes fold in LDS and one
// atomic per column per block adds into out (the fc bias gradient in the
// arena). The one-thread-per-column form waited 512 dependent loads (119 us).
__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ x,
                                                     float* __restrict__ out, int R, int C) {
    __shared__ float red[4][64];
    const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    const int rows = (R + gridDim.y - 1) / gridDim.y;
    const int r0 = blockIdx.y * rows, r1 = min(R, r0 + rows);
    float s = 0.f;
    if (c < C)
        for (int r = r0 + rl; r < r1; r += 4) s += bf2f(x[(size_t)r * C + c]);
    red[rl][cl] = s;
    __syncthreads();
    if (rl == 0 && c < C) atomicAdd(out + c, (red[0][cl] + red[1][cl]) + (red[2][cl] + red[3][cl]));
}

// ------------------------------------------------------------------ SGD
// torch.optim.SGD math ([torch] optim/sgd.py:343-380), on the flat arenas:
//   g' = g*gs + wd*p ; buf = first ? g' : mu*buf + (1-damp)*g' ;
//   d = nesterov ? g' + mu*buf : buf ; p -= lr*d ; shadow = bf16(p)
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ buf, bf16_t* __restrict__ shadow,
                                                  long n, float lr, float mu, float damp, float wd,
                                                  int nesterov, int first, float gs) {
    const long n4 = n / 4;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4 + (n % 4 ? 1 : 0);
         i += (long)gridDim.x * 256) {
        if (i < n4) {
            f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
            const f32x4 gv = reinterpret_cast<const f32x4*>(g)[i];
            f32x4 bv = first ? f32x4{0, 0, 0, 0} : reinterpret_cast<f32x4*>(buf)[i];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float gg = gv[j] * gs + wd * pv[j];
                float b = mu != 0.f ? (first ? gg : mu * bv[j] + (1.f - damp) * gg) : gg;
                bv[j] = b;
                const float d = nesterov ? gg + mu * b : b;
                pv[j] -= lr * d;
            }
            reinterpret_cast<f32x4*>(p)[i] = pv;
            if (mu != 0.f) reinterpret_cast<f32x4*>(buf)[i] = bv;
            if (shadow)
                reinterpret_cast<u32x2*>(shadow)[i] = u32x2{pack_bf2(pv[0], pv[1]), pack_bf2(pv[2], pv[3])};
        } else {
            for (long e = n4 * 4; e < n; ++e) {
                float gg = g[e] * gs + wd * p[e];
                float b = mu != 0.f ? (first ? gg : mu * buf[e] + (1.f - damp) * gg) : gg;
                if (mu != 0.f) buf[e] = b;
                const float d = nesterov ? gg + mu * b : b;
                p[e] -= lr * d;
                if (shadow) shadow[e] = f2bf(p[e]);
            }
        }
    }
}

__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ p,
                                                        bf16_t* __restrict__ o, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) o[i] = f2bf(p[i]);
}

__global__ __launch_bounds__(256) void uncast_bf16_kernel(const bf16_t* __restrict__ i_,
                                                          float* __restrict__ o, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) o[i] = bf2f(i_[i]);
}

// --------------------------------------------------------- normalize (uint8)
// in: uint8 [B][Hs][Ws][3] (decoded HWC images), out: bf16 [B][H][W][Cp]
// out = (x/255 - mean)/std per channel, padded channels 0; per-sample crop
// offset (oy, ox) and horizontal flip.
__global__ __launch_bounds__(256) void normalize_kernel(const uint8_t* __restrict__ in,
                                                        bf16_t* __restrict__ out,
                                                        const int* __restrict__ crop,
                                                        const uint8_t* __restrict__ flip, int B, int Hs,
                                                        int Ws, int H, int W, int Cp, float m0, float m1,
                                                        float m2, float is0, float is1, float is2) {
    const long total = (long)B * H * W;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
        const int w = t % W;
        const long r = t / W;
        const int h = r % H;
        const int b = r / H;
        const int oy = crop ? crop[2 * b] : 0, ox = crop ? crop[2 * b + 1] : 0;
        const int sw = (flip && flip[b]) ? (W - 1 - w) : w;
        const uint8_t* px = in + (((size_t)b * Hs + (h + oy)) * Ws + (sw + ox)) * 3;
        const float c0 = ((float)px[0] * (1.f / 255.f) - m0) * is0;
        const float c1 = ((float)px[1] * (1.f / 255.f) - m1) * is1;
        const float c2 = ((float)px[2] * (1.f / 255.f) - m2) * is2;
        bf16_t* o = out + (size_t)t * Cp;
        if (Cp == 8) {
            *reinterpret_cast<u32x4*>(o) = u32x4{pack_bf2(c0, c1), pack_bf2(c2, 0.f), 0u, 0u};
        } else if (Cp == 4) {
            *reinterpret_cast<u32x2*>(o) = u32x2{pack_bf2(c0, c1), pack_bf2(c2, 0.f)};
        } else {
            o[0] = f2bf(c0);
            o[1] = f2bf(c1);
            o[2] = f2bf(c2);
            for (int c = 3; c < Cp; ++c) o[c] = 0;
        }
    }
}

// 4 consecutive output pixels of a row per thread (W % 4 == 0, Cp 4 / 8): one 32-bit division per 4 pixels instead
// of three 64-bit ones per pixel, and 16-B stores (2 per thread at Cp 4) instead of one 8-B store per pixel. The
// per-pixel kernel above moved 2.9 TB/s at 4096 img (775 us for 2.26 GB, profiles/r50_b4096_r6_stream_tables.md)
template <int CP>
__global__ __launch_bounds__(256) void normalize4_kernel(const uint8_t* __restrict__ in, bf16_t* __restrict__ out,
                                                         const int* __restrict__ crop,
                                                         const uint8_t* __restrict__ flip, int B, int Hs, int Ws,
                                                         int H, int W, float m0, float m1, float m2, float is0,
                                                         float is1, float is2) {
    const uint32_t qpr = (uint32_t)W / 4, total = (uint32_t)B * (uint32_t)H * qpr;
    for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < total; t += gridDim.x * 256u) {
        const uint32_t row = t / qpr, q = t - row * qpr;
        const uint32_t b = row / (uint32_t)H, h = row - b * (uint32_t)H;
        const int oy = crop ? crop[2 * b] : 0, ox = crop ? crop[2 * b + 1] : 0;
        const bool fl = flip && flip[b];
        const uint8_t* src = in + (((size_t)b * Hs + (h + oy)) * Ws + ox) * 3;
        uint32_t px[4][3];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int w = 4 * (int)q + k, sw = fl ? (W - 1 - w) : w;
#pragma unroll
            for (int c = 0; c < 3; ++c) px[k][c] = src[sw * 3 + c];
        }
        u32x2 o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float c0 = ((float)px[k][0] * (1.f / 255.f) - m0) * is0;
            const float c1 = ((float)px[k][1] * (1.f / 255.f) - m1) * is1;
            const float c2 = ((float)px[k][2] * (1.f / 255.f) - m2) * is2;
            o[k] = u32x2{pack_bf2(c0, c1), pack_bf2(c2, 0.f)};
        }
        u32x4* dst = reinterpret_cast<u32x4*>(out + ((size_t)row * W + 4 * q) * CP);
        if (CP == 4) {
            dst[0] = u32x4{o[0][0], o[0][1], o[1][0], o[1][1]};
            dst[1] = u32x4{o[2][0], o[2][1], o[3][0], o[3][1]};
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) dst[k] = u32x4{o[k][0], o[k][1], 0u, 0u};
        }
    }
}

// --------------------------------------------------------- resize + normalize (uint8)
// The record store at a smaller size than the model input (data/records.py, --record-resize): in uint8
// [B][Hs][Ws][3] -> out bf16 [B][H][W][Cp] with a bilinear resample (half-pixel centres, edge clamp:
// torch's interpolate(bilinear, align_corners=False) and PIL's upscaling filter) fused into the normalize,
// optional horizontal flip. One thread per output pixel; its 4 source pixels are 12 bytes of 2 rows, served
// by L2 (each source pixel is read by ~(H/Hs)^2 neighbouring threads).
__global__ __launch_bounds__(256) void resize_normalize_kernel(const uint8_t* __restrict__ in,
                                                               bf16_t* __restrict__ out,
                                                               const uint8_t* __restrict__ flip, int B, int Hs,
                                                               int Ws, int H, int W, int Cp, float m0, float m1,
                                                               float m2, float is0, float is1, float is2) {
    const long total = (long)B * H * W;
    const float sy = (float)Hs / (float)H, sx = (float)Ws / (float)W;
    for (long t = (long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long)gridDim.x * 256) {
        const int w = t % W;
        const long r = t / W;
        const int h = r % H;
        const int b = r / H;
        const int ww = (flip && flip[b]) ? (W - 1 - w) : w;
        const float fy = fmaxf((h + 0.5f) * sy - 0.5f, 0.f), fx = fmaxf((ww + 0.5f) * sx - 0.5f, 0.f);
        const int y0 = min((int)fy, Hs - 1), x0 = min((int)fx, Ws - 1);
        const int y1 = min(y0 + 1, Hs - 1), x1 = min(x0 + 1, Ws - 1);
        const float ly = fy - (float)y0, lx = fx - (float)x0;
        const uint8_t* row0 = in + ((size_t)b * Hs + y0) * Ws * 3;
        const uint8_t* row1 = in + ((size_t)b * Hs + y1) * Ws * 3;
        float c[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float top = (float)row0[x0 * 3 + k] * (1.f - lx) + (float)row0[x1 * 3 + k] * lx;
            const float bot = (float)row1[x0 * 3 + k] * (1.f - lx) + (float)row1[x1 * 3 + k] * lx;
            c[k] = top * (1.f - ly) + bot * ly;
        }
        const float c0 = (c[0] * (1.f / 255.f) - m0) * is0;
        const float c1 = (c[1] * (1.f / 255.f) - m1) * is1;
        const float c2 = (c[2] * (1.f / 255.f) - m2) * is2;
        bf16_t* o = out + (size_t)t * Cp;
        if (Cp == 8) {
            *reinterpret_cast<u32x4*>(o) = u32x4{pack_bf2(c0, c1), pack_bf2(c2, 0.f), 0u, 0u};
        } else if (Cp == 4) {
            *reinterpret_cast<u32x2*>(o) = u32x2{pack_bf2(c0, c1), pack_bf2(c2, 0.f)};
        } else {
            o[0] = f2bf(c0);
            o[1] = f2bf(c1);
            o[2] = f2bf(c2);
            for (int cc = 3; cc < Cp; ++cc) o[cc] = 0;
        }
    }
}

// ------------------------------------------------- batched weight transposes
// dst[ci][t][co] = src[co][t][ci]  for every conv in the descriptor table.
struct TDesc {
    const bf16_t* src;
    bf16_t* dst;
    int Co, T, Ci;
    int tile0;  // first global tile index of this descriptor
};

__global__ __launch_bounds__(256) void transpose_batched_kernel(const TDesc* __restrict__ d, int nd) {
    __shared__ bf16_t tile[32][33];
    int lo = 0, hi = nd - 1;
    const int b = blockIdx.x;
    while (lo < hi) {  // last descriptor with tile0 <= b
        const int mid = (lo + hi + 1) >> 1;
        if (d[mid].tile0 <= b) lo = mid; else hi = mid - 1;
    }
    const TDesc a = d[lo];
    int rem = b - a.tile0;
    const int nci = (a.Ci + 31) / 32, nco = (a.Co + 31) / 32;
    const int tci = rem % nci;
    rem /= nci;
    const int tco = rem % nco;
    const int t = rem / nco;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int r = ty; r < 32; r += 8) {
        const int co = tco * 32 + r, ci = tci * 32 + tx;
        if (co < a.Co && ci < a.Ci) tile[r][tx] = a.src[((size_t)co * a.T + t) * a.Ci + ci];
    }
    __syncthreads();
    for (int r = ty; r < 32; r += 8) {
        const int ci = tci * 32 + r, co = tco * 32 + tx;
        if (co < a.Co && ci < a.Ci) a.dst[((size_t)ci * a.T + t) * a.Co + co] = tile[tx][r];
    }
}

int stream_grid(long work, int per_block = 256) {
    long b = (work + per_block - 1) / per_block;
    return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace

IMK_EXPORT int imk_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int OH,
                               int OW, int k, int s, int p, void* stream) {
    if (C % 8) return -100;
    const long total = (long)N * OH * OW * (C / 8);
    if (total >= (1L << 32) - 8192L * 256) return -101;  // 32-bit index math
    const dim3 g(stream_grid(total)), b(256);
    if (k <= 3)
        hipLaunchKernelGGL(maxpool_fwd_kernel<3>, g, b, 0, (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y,
                           (uint8_t*)idx, N, H, W, C, OH, OW, k, s, p);
    else
        hipLaunchKernelGGL(maxpool_fwd_kernel<0>, g, b, 0, (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y,
                           (uint8_t*)idx, N, H, W, C, OH, OW, k, s, p);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_maxpool_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W, int C,
                               int OH, int OW, int k, int s, int p, void* stream) {
    if (C % 8) return -100;
    const long total = (long)N * H * W * (C / 8);
    if (total >= (1L << 32) - 8192L * 256) return -101;  // 32-bit index math
    if (pool_quad_ok(H, W, OH, OW, k, s, p)) {
        hipLaunchKernelGGL((pool_nt() ? maxpool_bwd_quad_kernel<0, true> : maxpool_bwd_quad_kernel<0, false>), dim3(stream_grid(total / 4)), dim3(256), 0,
                           (hipStream_t)stream, (const bf16_t*)dy, (const uint8_t*)idx, (bf16_t*)dx, N, C, OH,
                           OW, PoolBnr{});
        IMK_CHECK_LAUNCH();
        return 0;
    }
    const dim3 g(stream_grid(total)), b(256);
    if ((k + s - 1) / s <= 2)
        hipLaunchKernelGGL(maxpool_bwd_kernel<2>, g, b, 0, (hipStream_t)stream, (const bf16_t*)dy,
                           (const uint8_t*)idx, (bf16_t*)dx, N, H, W, C, OH, OW, k, s, p);
    else
        hipLaunchKernelGGL(maxpool_bwd_kernel<0>, g, b, 0, (hipStream_t)stream, (const bf16_t*)dy,
                           (const uint8_t*)idx, (bf16_t*)dx, N, H, W, C, OH, OW, k, s, p);
    IMK_CHECK_LAUNCH();
    return 0;
}

// BN(+ReLU) forward fused into the maxpool that consumes it (the stem): y =
// maxpool(relu(bn(x))) with argmax indices; save <- (mean, rstd)
IMK_EXPORT int imk_maxpool_fwd_bn(const void* x, const float* sums, const float* gamma, const float* beta,
                                  float* save, void* y, void* idx, void* xsel, int N, int H, int W, int C, int OH,
                                  int OW, int k, int s, int p, float eps, void* stream) {
    if (C % 8 || 256 % (C / 8) || k > 3) return -100;
    const long total = (long)N * OH * OW * (C / 8);
    if (total >= (1L << 32) - 8192L * 256) return -101;  // 32-bit index math
    const dim3 g(stream_grid(total)), b(256);
    hipLaunchKernelGGL((maxpool_fwd_kernel<3, true>), g, b, 0, (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y,
                       (uint8_t*)idx, N, H, W, C, OH, OW, k, s, p,
                       PoolBnf{sums, gamma, beta, save, 1.f / (float)((long)N * H * W), eps, (bf16_t*)xsel});
    IMK_CHECK_LAUNCH();
    return 0;
}

// maxpool backward fused with the BN(+ReLU) backward reductions of the BN that
// feeds the pool (the stem): dx = ReLU-masked gradient, slab += (sum g*xhat, sum g). xsel (the forward's
// per-window argmax input, imk_maxpool_fwd_bn) replaces the read of x on the 2x2-quad path
IMK_EXPORT int imk_maxpool_bwd_bnr(const void* dy, const void* idx, void* dx, const void* x, const void* xsel,
                                   const float* save, const float* gamma, const float* beta, float* slab, int N,
                                   int H, int W, int C, int OH, int OW, int k, int s, int p, void* stream) {
    if (C % 8 || C > 2048 || 256 % (C / 8) || (k + s - 1) / s > 2) return -100;
    const long total = (long)N * H * W * (C / 8);
    if (total >= (1L << 32) - 8192L * 256) return -101;  // 32-bit index math
    if (pool_quad_ok(H, W, OH, OW, k, s, p)) {
        const PoolBnr bnr{(const bf16_t*)x, save, gamma, beta, slab, (const bf16_t*)xsel};
        if (xsel)
            hipLaunchKernelGGL((pool_nt() ? maxpool_bwd_quad_kernel<2, true> : maxpool_bwd_quad_kernel<2, false>), dim3(stream_grid(total / 4)), dim3(256), 0,
                               (hipStream_t)stream, (const bf16_t*)dy, (const uint8_t*)idx, (bf16_t*)dx, N, C, OH,
                               OW, bnr);
        else
            hipLaunchKernelGGL((pool_nt() ? maxpool_bwd_quad_kernel<1, true> : maxpool_bwd_quad_kernel<1, false>), dim3(stream_grid(total / 4)), dim3(256), 0,
                               (hipStream_t)stream, (const bf16_t*)dy, (const uint8_t*)idx, (bf16_t*)dx, N, C, OH,
                               OW, bnr);
        IMK_CHECK_LAUNCH();
        return 0;
    }
    if (!x) return -100;  // the per-pixel path needs x
    const dim3 g(stream_grid(total)), b(256);
    hipLaunchKernelGGL((maxpool_bwd_kernel<2, true>), g, b, 0, (hipStream_t)stream, (const bf16_t*)dy,
                       (const uint8_t*)idx, (bf16_t*)dx, N, H, W, C, OH, OW, k, s, p,
                       PoolBnr{(const bf16_t*)x, save, gamma, beta, slab});
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_avgpool_fwd(const void* x, void* y, int N, int HW, int C, void* stream) {
    if (C % 8) return -100;
    const int threads = N * (C / 8);
    hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((threads + 255) / 256), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)x, (bf16_t*)y, N, HW, C);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_avgpool_bwd(const void* dy, void* dx, int N, int HW, int C, void* stream) {
    if (C % 8) return -100;
    hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(stream_grid((long)N * HW * (C / 8))), dim3(256), 0,
                       (hipStream_t)stream, (const bf16_t*)dy, (bf16_t*)dx, N, HW, C);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_xent_fwd(const float* logits, const int64_t* labels, float* lse, float* loss_mean,
                            float* metrics, int B, int NC, float smoothing, void* stream) {
    // the mean loss is accumulated by the blocks: cleared here (no separate fill launch by the caller)
    if (hipMemsetAsync(loss_mean, 0, sizeof(float), (hipStream_t)stream) != hipSuccess) return -1;
    hipLaunchKernelGGL(xent_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, (hipStream_t)stream, logits,
                       labels, lse, loss_mean, metrics, B, NC, smoothing);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_xent_bwd(const float* logits, const int64_t* labels, const float* lse,
                            const float* gout, void* dz, int B, int NC, float smoothing, void* stream) {
    hipLaunchKernelGGL(xent_bwd_kernel, dim3((NC + 255) / 256, B), dim3(256), 0, (hipStream_t)stream,
                       logits, labels, lse, gout, (bf16_t*)dz, B, NC, smoothing);
    IMK_CHECK_LAUNCH();
    return 0;
}

// The stem's weight gradient from its row-segment layout gp [Co][KH][32] (channel-padded 4-channel pixels, kw * 4 +
// ci) into the master gradient, stored [Co][KH][KW][Ci] in the arena (+=, gradient accumulation), clearing gp for
// the next step's atomic accumulation in the same pass (one launch instead of a fill + a strided add).
__global__ __launch_bounds__(256) void stem_grad_fold_kernel(float* __restrict__ gp, float* __restrict__ grad, int Co,
                                                             int Ci, int KH, int KW) {
    const int n = Co * Ci * KH * KW;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
        const int ci = e % Ci, kw = (e / Ci) % KW, kh = (e / (Ci * KW)) % KH, co = e / (Ci * KW * KH);
        float* src = gp + ((size_t)co * KH + kh) * 32 + kw * 4 + ci;
        grad[e] += *src;
        *src = 0.f;
    }
}

IMK_EXPORT int imk_stem_grad_fold(float* gp, float* grad, int Co, int Ci, int KH, int KW, void* stream) {
    if (Co <= 0 || Ci <= 0 || Ci > 4 || KW * 4 > 32 || KH <= 0) return -100;
    const int n = Co * Ci * KH * KW;
    hipLaunchKernelGGL(stem_grad_fold_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, gp, grad,
                       Co, Ci, KH, KW);
    IMK_CHECK_LAUNCH();
    return 0;
}

// Zero a device buffer on a stream (the per-step gradient arena / workspace clears): one hipMemsetAsync (a runtime
// fill, not an ATen FillFunctor launch).
IMK_EXPORT int imk_memset0(void* p, long bytes, void* stream) {
    if (!p || bytes < 0) return -100;
    if (bytes && hipMemsetAsync(p, 0, (size_t)bytes, (hipStream_t)stream) != hipSuccess) return -1;
    return 0;
}

// The stem's bf16 weight shadow [Co][KH][KW][Ci] into its row-segment layout [Co][KH][32] (kw * 4 + ci; the padded
// channel and taps stay zero), after every optimizer step (one launch instead of an ATen strided copy).
__global__ __launch_bounds__(256) void stem_pad_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                       int Co, int KH, int KW, int Ci) {
    const int n = Co * KH * KW * Ci;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
        const int ci = e % Ci, kw = (e / Ci) % KW, r = e / (Ci * KW);  // r = co * KH + kh
        dst[(size_t)r * 32 + kw * 4 + ci] = src[e];
    }
}

IMK_EXPORT int imk_stem_pad(const void* src, void* dst, int Co, int KH, int KW, int Ci, void* stream) {
    if (Co <= 0 || KH <= 0 || Ci <= 0 || Ci > 4 || KW * 4 > 32) return -100;
    const int n = Co * KH * KW * Ci;
    hipLaunchKernelGGL(stem_pad_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)src,
                       (bf16_t*)dst, Co, KH, KW, Ci);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_colsum_bf16(const void* x, float* out, int R, int C, void* stream) {
    const int slices = R >= 64 ? min(32, R / 16) : 1;
    hipLaunchKernelGGL(colsum_kernel, dim3((C + 63) / 64, slices), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, out, R, C);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_sgd(float* p, const float* g, float* buf, void* shadow, long n, float lr, float mu,
                       float damp, float wd, int nesterov, int first, float gs, void* stream) {
    hipLaunchKernelGGL(sgd_kernel, dim3(stream_grid((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, p,
                       g, buf, (bf16_t*)shadow, n, lr, mu, damp, wd, nesterov, first, gs);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_cast_bf16(const float* p, void* o, long n, void* stream) {
    hipLaunchKernelGGL(cast_bf16_kernel, dim3(stream_grid(n)), dim3(256), 0, (hipStream_t)stream, p,
                       (bf16_t*)o, n);
    IMK_CHECK_LAUNCH();
    return 0;
}

// bf16 -> fp32 (the bf16 gradient all-reduce writes the reduced buckets back into the fp32 arena)
IMK_EXPORT int imk_uncast_bf16(const void* i, float* o, long n, void* stream) {
    hipLaunchKernelGGL(uncast_bf16_kernel, dim3(stream_grid(n)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)i, o, n);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_resize_normalize_u8(const void* in, void* out, const void* flip, int B, int Hs, int Ws, int H,
                                       int W, int Cp, const float* mean, const float* std, void* stream) {
    if (Hs < 1 || Ws < 1 || H < 1 || W < 1 || Cp < 3) return -1;
    hipLaunchKernelGGL(resize_normalize_kernel, dim3(stream_grid((long)B * H * W)), dim3(256), 0,
                       (hipStream_t)stream, (const uint8_t*)in, (bf16_t*)out, (const uint8_t*)flip, B, Hs, Ws, H,
                       W, Cp, mean[0], mean[1], mean[2], 1.f / std[0], 1.f / std[1], 1.f / std[2]);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_normalize_u8(const void* in, void* out, const int* crop, const void* flip, int B,
                                int Hs, int Ws, int H, int W, int Cp, const float* mean,
                                const float* std, void* stream) {
    if (W % 4 == 0 && (Cp == 4 || Cp == 8) && (long)B * H * (W / 4) < (1L << 31)) {
        const dim3 g(stream_grid((long)B * H * (W / 4))), bl(256);
        if (Cp == 4)
            hipLaunchKernelGGL(normalize4_kernel<4>, g, bl, 0, (hipStream_t)stream, (const uint8_t*)in, (bf16_t*)out,
                               crop, (const uint8_t*)flip, B, Hs, Ws, H, W, mean[0], mean[1], mean[2], 1.f / std[0],
                               1.f / std[1], 1.f / std[2]);
        else
            hipLaunchKernelGGL(normalize4_kernel<8>, g, bl, 0, (hipStream_t)stream, (const uint8_t*)in, (bf16_t*)out,
                               crop, (const uint8_t*)flip, B, Hs, Ws, H, W, mean[0], mean[1], mean[2], 1.f / std[0],
                               1.f / std[1], 1.f / std[2]);
        IMK_CHECK_LAUNCH();
        return 0;
    }
    hipLaunchKernelGGL(normalize_kernel, dim3(stream_grid((long)B * H * W)), dim3(256), 0,
                       (hipStream_t)stream, (const uint8_t*)in, (bf16_t*)out, crop,
                       (const uint8_t*)flip, B, Hs, Ws, H, W, Cp, mean[0], mean[1], mean[2],
                       1.f / std[0], 1.f / std[1], 1.f / std[2]);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_transpose_batched(const void* descs, int nd, int total_tiles, void* stream) {
    if (nd <= 0) return 0;
    hipLaunchKernelGGL(transpose_batched_kernel, dim3(total_tiles), dim3(256), 0, (hipStream_t)stream,
                       (const TDesc*)descs, nd);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_tdesc_size() { return (int)sizeof(TDesc); }

// A stream restricted to `quarters` / 4 of the CUs (ops/streams.py IMAGENT_SIDE_CUMASK: the weight-gradient side
// stream confined so that it cannot flood every CU while the main stream's critical-path kernels wait for slots).
// CU i is enabled when (i / 8) % 4 < quarters: a quarter-pattern that is uniform over the 8 XCDs whether the mask bits
// enumerate CUs XCD-major (i / 32 = XCD) or round-robin over XCDs (i % 8 = XCD). A CU-masked stream also gets a
// hardware queue of its own. Kept for the process lifetime (never destroyed).
IMK_EXPORT int imk_stream_create_cumask(int quarters, void** out) {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    if (quarters < 1 || quarters > 4 || ncu <= 0) return -2;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int i = 0; i < ncu; ++i)
        if ((i / 8) % 4 < quarters) mask[i / 32] |= 1u << (i % 32);
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) return -3;
    *out = (void*)s;
    return 0;
}
