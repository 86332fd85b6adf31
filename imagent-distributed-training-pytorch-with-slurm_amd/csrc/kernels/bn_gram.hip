// BatchNorm backward of a bottleneck's last BatchNorm (bn3) without its apply pass, gfx950.
//
// The reference trains torchvision's Bottleneck (imagenet.py:312; backward :128):
//     x3 = conv3(h2)  (1x1, p -> 4p channels),  y = relu(bn3(x3) + identity)
// Its BatchNorm backward is, per output channel o (bn_bwd_apply_kernel, bn.hip),
//     dx3 = A_o g + B_o x3 + c_o,   A = gamma rstd,  B = -gamma rstd^2 mean(g xhat),
//                                   c = -gamma rstd mean(g) - B mean
// for the ReLU-masked upstream gradient g (its reductions come from the producing dgrad's epilogue).
// dx3 is 4p channels wide -- the widest activation of the block -- and the apply pass that writes
// it (read g, x3; write dx3) was the largest BatchNorm cost of the step. Both consumers of dx3 are
// linear in it, and x3 = h2 W3^T, so the x3 term folds into p x p matrices:
//   dgrad:  dh2 = dx3 W3 = g (diag(A) W3) + h2 (W3^T diag(B) W3) + c W3
//           -> ONE GEMM over K = [g | h2] (4p + p instead of 4p: +25 % MACs) with the weights
//              Wcat[i] = [A_o W3[o][i] | Q[j][i]], Q = W3^T diag(B) W3, and the bias c W3;
//   wgrad:  dW3 = dx3^T h2 = diag(A) (g^T h2) + diag(B) W3 (h2^T h2) + c (1^T h2)
//           -> the weight-gradient GEMM of g, the p x p Gram matrix G = h2^T h2 (+25 %), the
//              column sums of h2, and an elementwise fix-up (bn_gram_wgrad_fixup_kernel).
// (x3 enters as h2 W3^T in full precision instead of its bf16-rounded copy: a 2^-9 relative
// difference inside the B term.) ops/block.py drives it; tests/test_model_gpu.py holds it to the
// fp32 PyTorch model.

#include <algorithm>

#include "common.h"

namespace {

constexpr int BWD_SLOTS_G = 32;  // the BN-backward reduction slab slots (bn.hip BWD_SLOTS, STAT_SLOTS)

// coef [3][C] = (A, B, c) from the dgrad epilogue's slab [S][3][C] (sum g xhat, sum g, -);
// dgamma / dbeta accumulate as in the apply pass (slot order as stats_finalize_kernel)
__global__ void bn_bwd_coef_kernel(const float* __restrict__ slab, const float* __restrict__ save,
                                   const float* __restrict__ gamma, float* __restrict__ dgamma,
                                   float* __restrict__ dbeta, float* __restrict__ coef, int S, int C,
                                   float inv_cnt) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float sgx = 0.f, sg = 0.f;
    for (int s = 0; s < S; ++s) {
        sgx += slab[(size_t)s * 3 * C + c];
        sg += slab[(size_t)s * 3 * C + C + c];
    }
    if (dgamma) dgamma[c] += sgx;
    if (dbeta) dbeta[c] += sg;
    const float mean = save[c], rstd = save[C + c], gr = gamma[c] * rstd;
    const float k0 = -gr * inv_cnt * sg, kx = -gr * inv_cnt * sgx * rstd;
    coef[c] = gr;
    coef[C + c] = kx;
    coef[2 * C + c] = k0 - kx * mean;
}

// dgrad weights: wt [p][ldw] bf16 = W3^T (row i: input channel i of conv3, columns o < C4),
// Q [p][p] fp32 -> wcat [p][C4 + p] bf16 = [A_o wt[i][o] | Q[i][j]], bias [p] = sum_o c_o wt[i][o]
__global__ __launch_bounds__(256) void bn_gram_dgrad_weights_kernel(const bf16_t* __restrict__ wt, int ldw,
                                                                    const float* __restrict__ coef,
                                                                    const float* __restrict__ Q,
                                                                    bf16_t* __restrict__ wcat,
                                                                    float* __restrict__ bias, int p, int C4) {
    const int i = blockIdx.x;
    const int ld = C4 + p;
    float part = 0.f;
    for (int o = threadIdx.x; o < C4; o += 256) {
        const float w = bf2f(wt[(size_t)i * ldw + o]);
        wcat[(size_t)i * ld + o] = f2bf(w * coef[o]);
        part += w * coef[2 * C4 + o];
    }
    for (int j = threadIdx.x; j < p; j += 256) wcat[(size_t)i * ld + C4 + j] = f2bf(Q[(size_t)i * p + j]);
    __shared__ float red[256];
    red[threadIdx.x] = part;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) bias[i] = red[0];
}

// The small fp32 GEMMs of the Gram form, C[M][N] = sum_k A(m, k) B(k, n), on the VALU (fp32 products: P feeds
// bn3's variance, which must not lose what the centring keeps). 64 x 64 output tile per block, 4 x 4 per thread,
// K staged through LDS in chunks of 16 ([k][m] / [k][n] images read as float4), split over gridDim.z blocks of 64 k
// each (~256 blocks at R50: the unsplit 16-64-block grids waited out one global round trip per chunk, 65 us per
// p = 256 Q in the step) that ADD into the zeroed output (fp32 atomics; the per-step zeroed Gram workspace).
// M, N % 64 == 0, K % 64 == 0.
//  MODE 0: P = W3 Gc, the centred Gram matrix Gc = G - s s^T / rows formed on the operand load
//          (A(o, j) = W3[o][j], bf16 [C4][p]; B(j, i) = G[j][i] - s[j] s[i] / rows; M = C4, N = K = p);
//  MODE 1: Q = W3^T diag(B) W3 for the folded dgrad weights (A(i, o) = wt[i][o] B_o, B(o, j) = wt[j][o],
//          wt = W3^T [p][ldw] bf16, B = coef[C4 ..]; M = N = p, K = C4).
// (torch.mm ran these as 16-workgroup hipBLASLt kernels plus bf16 -> fp32 weight casts: 160 us per P call in
// the step, profiles/r50_b1024_v21_stream_tables.md)
template <int MODE>
__global__ __launch_bounds__(256) void bn_gram_gemm_kernel(const bf16_t* __restrict__ w, int ldw,
                                                           const float* __restrict__ G, const float* __restrict__ s,
                                                           const float* __restrict__ coef, float* __restrict__ out,
                                                           int M, int N, int K, float inv_rows) {
    __shared__ __attribute__((aligned(16))) float sa[16][68], sb[16][68];
    const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    const int kb = blockIdx.z * 64;
    for (int k0 = kb; k0 < kb + 64; k0 += 16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // A: 64 rows x 16 k, k fastest in memory
            const int e = tid + 256 * q, r = e >> 4, kk = e & 15;
            float v = bf2f(w[(size_t)(m0 + r) * ldw + k0 + kk]);
            if (MODE == 1) v *= coef[K + k0 + kk];
            sa[kk][r] = v;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q;
            if (MODE == 0) {  // B: 16 k x 64 n, n fastest in memory
                const int kk = e >> 6, c = e & 63;
                const int j = k0 + kk, i = n0 + c;
                sb[kk][c] = G[(size_t)j * N + i] - s[j] * s[i] * inv_rows;
            } else {  // B(o, j) = wt[j][o]: k fastest in memory
                const int c = e >> 4, kk = e & 15;
                sb[kk][c] = bf2f(w[(size_t)(n0 + c) * ldw + k0 + kk]);
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            const f32x4 a4 = *reinterpret_cast<const f32x4*>(&sa[kk][ty * 4]);
            const f32x4 b4 = *reinterpret_cast<const f32x4*>(&sb[kk][tx * 4]);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a4[i], b4[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) atomicAdd(out + (size_t)(m0 + ty * 4 + i) * N + n0 + tx * 4 + j, acc[i][j]);
}

// dW3 [C4][p] += A_o T[o][i] + B_o P[o][i] + (c_o + B_o mean_o) s[i]   (T = g^T h2, P = W3 Gc with the centred
// Gram matrix, s = colsum h2). From dW3 = dx3^T h2 = A T + B W3 G + c s^T and W3 G = P + mean s^T: the centred form
// adds no two large, nearly equal terms when |mean| >> std (c_o + B_o mean_o = -A_o mean(g) is small)
__global__ __launch_bounds__(64) void bn_gram_wgrad_fixup_kernel(float* __restrict__ dw,
                                                                  const float* __restrict__ T,
                                                                  const float* __restrict__ P,
                                                                  const float* __restrict__ coef,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ s, int C4, int p) {
    // one wave per (row o, 256 columns): the row's three coefficients are wave-uniform scalar loads, 4 columns per
    // lane; p is a multiple of 4 (the host checks), so every row starts 16-B aligned
    const int o = blockIdx.y;
    const int i = (blockIdx.x * 64 + threadIdx.x) * 4;
    if (i >= p) return;
    const float a = coef[o], b = coef[C4 + o], k0 = fmaf(b, mean[o], coef[2 * C4 + o]);
    const long e = (long)o * p + i;
    const float4 t = *reinterpret_cast<const float4*>(T + e), q = *reinterpret_cast<const float4*>(P + e);
    const float4 sv = *reinterpret_cast<const float4*>(s + i);
    float4 d = *reinterpret_cast<const float4*>(dw + e);
    d.x += fmaf(a, t.x, fmaf(b, q.x, k0 * sv.x));
    d.y += fmaf(a, t.y, fmaf(b, q.y, k0 * sv.y));
    d.z += fmaf(a, t.z, fmaf(b, q.z, k0 * sv.z));
    d.w += fmaf(a, t.w, fmaf(b, q.w, k0 * sv.w));
    *reinterpret_cast<float4*>(dw + e) = d;
}

// As bn_bwd_coef_kernel, with sum(g xhat) NOT from the slab but from T = g^T h2 (the weight gradient's GEMM):
// x3 = h2 W3^T, so sum_m g[m][o] (x3[m][o] - mean_o) = sum_i W3[o][i] (T[o][i] - sg_o mu_i), mu = colsum(h2) / rows,
// centred per element (the uncentred rstd (W3 . T - mean sg) differences two large, nearly equal sums when
// |mean| >> std). The producing dgrad then never reads x3 (BNBwdFuse without x). One wave per channel.
__global__ __launch_bounds__(256) void bn_bwd_coef_T_kernel(const float* __restrict__ slab, const float* __restrict__ T,
                                                            const bf16_t* __restrict__ w, const float* __restrict__ hs,
                                                            const float* __restrict__ save,
                                                            const float* __restrict__ gamma, float* __restrict__ dgamma,
                                                            float* __restrict__ dbeta, float* __restrict__ coef, int S,
                                                            int C, int p, float inv_cnt) {
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (o >= C) return;  // wave-uniform
    float sg = 0.f;
    for (int s = lane; s < S; s += 64) sg += slab[(size_t)s * 3 * C + C + o];
    sg = wave_sum(sg);
    const float sgm = sg * inv_cnt;
    float dot = 0.f;
    for (int i = lane; i < p; i += 64)
        dot += bf2f(w[(size_t)o * p + i]) * fmaf(-sgm, hs[i], T[(size_t)o * p + i]);
    dot = wave_sum(dot);
    if (lane) return;
    const float mean = save[o], rstd = save[C + o], gr = gamma[o] * rstd;
    const float sgx = rstd * dot;
    if (dgamma) dgamma[o] += sgx;
    if (dbeta) dbeta[o] += sg;
    const float k0 = -gr * inv_cnt * sg, kx = -gr * inv_cnt * sgx * rstd;
    coef[o] = gr;
    coef[C + o] = kx;
    coef[2 * C + o] = k0 - kx * mean;
}

// bn3's training statistics WITHOUT conv3's output (x3 = h2 W3^T, never written): per output channel o,
//   mean = W3[o] . colsum(h2) / M,   var = W3[o] . P[o] / M  with P = W3 Gc, Gc = G - s s^T / M (G = h2^T h2),
// i.e. var = W3[o]^T Cov(h2) W3[o]: the covariance is formed BEFORE the contraction with W3, so a channel whose
// |mean| >> std (W3[o] aligned with the mean of h2) does not lose its variance to E[x3^2] - mean^2 cancellation
// (tests/test_bn_numerics_gpu.py, |mean| / std >= 30 against fp64). Biased, as the training BatchNorm normalises.
// -> stats [2][C] (mean, var; the running-statistics update reads it), save [2][C] (mean, rstd; the backward),
// aff [2][C] (gamma rstd, beta - mean gamma rstd; conv3's epilogue applies it). One wave per channel.
__global__ __launch_bounds__(256) void bn_gram_fwd_stats_kernel(const bf16_t* __restrict__ w, const float* __restrict__ s,
                                                                const float* __restrict__ P, const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, float* __restrict__ stats,
                                                                float* __restrict__ save, float* __restrict__ aff,
                                                                const float* __restrict__ add_shift, int C, int p,
                                                                float inv_m, float eps) {
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (o >= C) return;  // wave-uniform
    float m1 = 0.f, m2 = 0.f;
    for (int i = lane; i < p; i += 64) {
        const float wi = bf2f(w[(size_t)o * p + i]);
        m1 += wi * s[i];
        m2 += wi * P[(size_t)o * p + i];
    }
    m1 = wave_sum(m1) * inv_m;
    m2 = wave_sum(m2) * inv_m;
    if (lane) return;
    const float var = fmaxf(m2, 0.f), rstd = rsqrtf(var + eps), sc = gamma[o] * rstd;
    stats[o] = m1;
    stats[C + o] = var;
    save[o] = m1;
    save[C + o] = rstd;
    aff[o] = sc;
    aff[C + o] = beta[o] - m1 * sc + (add_shift ? add_shift[o] : 0.f);
}

}  // namespace

// add_shift (may be null): added to the epilogue shift (a downsample block's shortcut-BN shift, folded into bn3's)
IMK_EXPORT int imk_bn_gram_fwd_stats(const void* w, const float* s, const float* P, const float* gamma,
                                     const float* beta, float* stats, float* save, float* aff, const float* add_shift,
                                     long M, int C, int p, float eps, void* stream) {
    if (M <= 0 || C <= 0 || p <= 0) return -100;
    hipLaunchKernelGGL(bn_gram_fwd_stats_kernel, dim3((C + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)w, s, P, gamma, beta, stats, save, aff, add_shift, C, p, 1.f / (float)M, eps);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_bn_bwd_coef_T(const float* scratch, const float* T, const void* w, const float* hs,
                                 const float* save, const float* gamma, float* dgamma_acc, float* dbeta_acc,
                                 float* coef, long R, int C, int p, void* stream) {
    if (R <= 0 || C <= 0 || p <= 0) return -100;
    hipLaunchKernelGGL(bn_bwd_coef_T_kernel, dim3((C + 3) / 4), dim3(256), 0, (hipStream_t)stream, scratch, T,
                       (const bf16_t*)w, hs, save, gamma, dgamma_acc, dbeta_acc, coef, BWD_SLOTS_G, C, p,
                       1.f / (float)R);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_bn_bwd_coef(const float* scratch, const float* save, const float* gamma, float* dgamma_acc,
                               float* dbeta_acc, float* coef, long R, int C, void* stream) {
    if (R <= 0 || C <= 0) return -100;
    hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, scratch, save,
                       gamma, dgamma_acc, dbeta_acc, coef, BWD_SLOTS_G, C, 1.f / (float)R);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_bn_gram_dgrad_weights(const void* wt, int ldw, const float* coef, const float* Q, void* wcat,
                                         float* bias, int p, int C4, void* stream) {
    if (p <= 0 || C4 <= 0 || ldw < C4) return -100;
    hipLaunchKernelGGL(bn_gram_dgrad_weights_kernel, dim3(p), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)wt, ldw, coef, Q, (bf16_t*)wcat, bias, p, C4);
    IMK_CHECK_LAUNCH();
    return 0;
}

// Q += W3^T diag(B) W3 [p][p] (wt = W3^T [p][ldw] bf16; Q zeroed by the caller)
IMK_EXPORT int imk_bn_gram_q(const void* wt, int ldw, const float* coef, float* Q, int p, int C4, void* stream) {
    if (p <= 0 || p % 64 || C4 <= 0 || C4 % 64 || ldw < C4) return -100;
    hipLaunchKernelGGL(bn_gram_gemm_kernel<1>, dim3(p / 64, p / 64, C4 / 64), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)wt, ldw, nullptr, nullptr, coef, Q, p, p, C4, 0.f);
    IMK_CHECK_LAUNCH();
    return 0;
}

// P += W3 (G - s s^T / rows) [C4][p] (W3 [C4][p] bf16, G [p][p], s [p]; P zeroed by the caller)
IMK_EXPORT int imk_bn_gram_p(const void* w, const float* G, const float* s, float* P, long rows, int C4, int p,
                             void* stream) {
    if (rows <= 0 || p <= 0 || p % 64 || C4 <= 0 || C4 % 64) return -100;
    hipLaunchKernelGGL(bn_gram_gemm_kernel<0>, dim3(p / 64, C4 / 64, p / 64), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)w, p, G, s, nullptr, P, C4, p, p, 1.f / (float)rows);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_bn_gram_wgrad_fixup(float* dw, const float* T, const float* P, const float* coef,
                                       const float* mean, const float* s, int C4, int p, void* stream) {
    if (p <= 0 || C4 <= 0 || C4 > 65535 || p % 4) return -100;
    hipLaunchKernelGGL(bn_gram_wgrad_fixup_kernel, dim3((p + 255) / 256, C4), dim3(64), 0, (hipStream_t)stream, dw, T, P, coef,
                       mean, s, C4, p);
    IMK_CHECK_LAUNCH();
    return 0;
}
