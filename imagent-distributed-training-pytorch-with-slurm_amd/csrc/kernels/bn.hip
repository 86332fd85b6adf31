// BatchNorm (training + eval) fused with residual add and ReLU, NHWC bf16.
//
// Replaces cuDNN/ATen native_batch_norm (+_backward), relu_ / threshold_
// backward and the residual add of torchvision's BasicBlock/Bottleneck
// (reference model at /root/reference/imagenet.py:312).
//
// Statistics: the per-channel shifted (sum, sum of squares) of the BN input
// come from the producing conv's epilogue (conv_igemm.hip, 32-slot fp32 slab,
// shift = the previous batch mean) and imk_bn_stats_finalize turns them into
// (mean, variance), so the forward is ONE streaming pass: read x (+ residual),
// write y.
// Semantics follow nn.BatchNorm2d: biased variance to normalise, unbiased
// variance into running_var, momentum 0.1, eps 1e-5, num_batches_tracked++.
//
// Backward is two streaming passes (reduce -> apply). The ReLU mask:
//  * plain BN+ReLU (mode 0): recomputed from x as fma(x, sc, sh) > 0 - the
//    output y is never re-read (2 of the 6-8 bytes per element saved per pass);
//  * BN + residual (+ReLU) (modes 1/2): taken from the saved output y > 0.
// dgamma/dbeta are accumulated straight into the parameters' slots of the flat
// gradient arena.
//
// Layout: rows r = (n, h, w), C channels contiguous; each thread owns one
// 16-B chunk (8 channels) of a row -> per-thread channel constants live in
// registers, loads/stores are 16 B per lane (cdna_hip_programming.md G13).

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "common.h"

namespace {

constexpr int U = 4;  // rows per thread per loop iteration (loads batched ahead of the math)
constexpr int BWD_SLOTS = 32;  // backward reduction slab slots

// optional e5m2 copies of the backward outputs (dx, dx2) for the fp8 dgrad
// (conv_igemm_fp8.hip, IG_BF8X), quantised with 2^-exp and amax-tracked in
// 32-slot rows (folded by imk_fp8_update_exp): delayed scaling as forward
struct G8Out {
    uint32_t* q[2];
    const int* exp[2];
    float* amax[2];
};

constexpr float E5M2_MAX = 57344.f;

__device__ __forceinline__ uint32_t pack4_bf8(float a, float b, float c, float d) {
    a = fminf(fmaxf(a, -E5M2_MAX), E5M2_MAX);
    b = fminf(fmaxf(b, -E5M2_MAX), E5M2_MAX);
    c = fminf(fmaxf(c, -E5M2_MAX), E5M2_MAX);
    d = fminf(fmaxf(d, -E5M2_MAX), E5M2_MAX);
    int w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    w = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
    return (uint32_t)w;
}


struct Vec8 {
    float v[8];
};

__device__ __forceinline__ Vec8 ld8(const bf16_t* p) {
    const u32x4 w = *reinterpret_cast<const u32x4*>(p);
    Vec8 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        r.v[2 * i] = lo_bf(w[i]);
        r.v[2 * i + 1] = hi_bf(w[i]);
    }
    return r;
}
__device__ __forceinline__ void ld8f(const float* p, float (&o)[8]) {
    const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        o[i] = a[i];
        o[4 + i] = b[i];
    }
}

__device__ __forceinline__ void st8(bf16_t* p, const Vec8& x) {
    u32x4 w;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack_bf2(x.v[2 * i], x.v[2 * i + 1]);
    *reinterpret_cast<u32x4*>(p) = w;
}

// packed 16-B row chunk: load, element i as f32, store (NT: non-temporal -- the streamed output
// is read back by the next kernel only after far more than the L2 / MALL has passed through)
__device__ __forceinline__ u32x4 ldw(const bf16_t* p) { return *reinterpret_cast<const u32x4*>(p); }
// non-temporal load of a streamed operand (read once; scripts/hbm_roof.hip: r2w1 6.32 vs 5.92 TB/s plain)
template <bool NTL>
__device__ __forceinline__ u32x4 ldwn(const bf16_t* p) {
    if (NTL) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return *reinterpret_cast<const u32x4*>(p);
}
__device__ __forceinline__ float bfw(const u32x4& w, int i) { return (i & 1) ? hi_bf(w[i >> 1]) : lo_bf(w[i >> 1]); }
template <bool NT>
__device__ __forceinline__ void stw(bf16_t* p, const u32x4& w) {
    if (NT) __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
    else *reinterpret_cast<u32x4*>(p) = w;
}

// store the bf16 row chunk; with q: also its e5m2 copy, track |.| max in m
template <bool NT, bool Q8>
__device__ __forceinline__ void stq(bf16_t* p, const float (&o)[8], uint32_t* q, size_t off, float s, float& m) {
    u32x4 w;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack_bf2(o[2 * i], o[2 * i + 1]);
    stw<NT>(p, w);
    if (Q8 && q) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = bfw(w, i);
#pragma unroll
        for (int i = 0; i < 8; ++i) m = fmaxf(m, fabsf(v[i]));
        reinterpret_cast<u32x2*>(q)[off / 8] =
            u32x2{pack4_bf8(v[0] * s, v[1] * s, v[2] * s, v[3] * s), pack4_bf8(v[4] * s, v[5] * s, v[6] * s, v[7] * s)};
    }
}


// ---------------------------------------------------------------- slab fold inside the consumer
// The fold of a producer's [S][Q][C] statistics slab (formerly its own launch before every BN pass: stats_finalize_mv
// forward, stats_finalize backward) done by the consumer pass itself: the first ceil(n / 256) blocks each fold 256 of
// the n quantities, store them, and publish with an agent-scope release + counter (cdna_hip_programming.md
// Guideline 16 R1: sc1 stores, vmcnt(0) per wave, barrier, relaxed agent fetch_add); every block
// workgroup waits for the counter (one lane's relaxed polls, one acquire fence, a barrier) before using them. The folding blocks are the lowest block ids, dispatched first, and never wait on a later
// block: no deadlock whatever the residency. The counter (zero at launch: zeroed with the slabs once per step) lives
// in the BN's backward scratch (imk_bn_bwd_scratch_floats' last row).
constexpr int FOLD_S = 32;  // slab slots the in-pass fold supports (STAT_SLOTS = BWD_SLOTS = 32; host-checked)
static_assert(BWD_SLOTS == FOLD_S, "backward slab slots");
struct SlabFold {
    const float* slab;   // [S][n] (backward) or [S][2][C] shifted sums (forward); null: no fold, `out` is ready
    const float* shift;  // forward: the shift the sums were taken around (the previous batch mean) or null
    float* out;          // backward: [n] sums; forward: [2][C] (mean, biased variance)
    uint32_t* cnt;       // publish counter, zero at launch (zeroed with the slabs once per step)
    int S;
    float inv_cnt;       // forward only
};

__device__ __forceinline__ void fold_publish(const SlabFold& f, int n, bool fwd, int C) {
    const int nfold = (n + 255) / 256;
    if ((int)blockIdx.x < nfold) {
        const int i = blockIdx.x * 256 + threadIdx.x;
        if (i < n) {
            // all FOLD_S slot loads issued before the adds (one L2 round trip, not S dependent ones: the rest of the
            // grid waits on this), summed in the separate launches' order
            if (fwd) {  // channel i: mean = shift + E[d], var = E[d^2] - E[d]^2 (fixed order, as stats_finalize_mv)
                float va[FOLD_S], vb[FOLD_S];
#pragma unroll
                for (int k = 0; k < FOLD_S; ++k) {
                    va[k] = f.slab[(size_t)k * 2 * C + i];
                    vb[k] = f.slab[(size_t)k * 2 * C + C + i];
                }
                float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < FOLD_S; ++k) {
                    a[k & 3] += va[k];
                    b[k & 3] += vb[k];
                }
                const float m1 = ((a[0] + a[1]) + (a[2] + a[3])) * f.inv_cnt;
                const float m2 = ((b[0] + b[1]) + (b[2] + b[3])) * f.inv_cnt;
                __hip_atomic_store(f.out + i, (f.shift ? f.shift[i] : 0.f) + m1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);  // write-through (sc1): no release fence needed
                __hip_atomic_store(f.out + C + i, fmaxf(m2 - m1 * m1, 0.f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {  // quantity i: plain sum over the slots (as stats_finalize_kernel)
                float v[FOLD_S];
#pragma unroll
                for (int k = 0; k < FOLD_S; ++k) v[k] = f.slab[(size_t)k * n + i];
                float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < FOLD_S; ++k) a[k & 3] += v[k];
                __hip_atomic_store(f.out + i, (a[0] + a[1]) + (a[2] + a[3]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(f.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// per workgroup (every thread of the block must call it): ONE lane polls the counter (relaxed, long sleeps: the
// grid's pollers share one word), the barrier releases the block; the payload was stored sc1 and is read sc1 (no
// L1 invalidate: Guideline 16, R1 with sc1 consumer loads)
__device__ __forceinline__ void fold_wait(const SlabFold& f, int n) {
    const uint32_t nfold = (uint32_t)((n + 255) / 256);
    if (threadIdx.x == 0)
        while (__hip_atomic_load(f.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nfold)
            __builtin_amdgcn_s_sleep(32);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler ordering only: every later load of the
    __syncthreads();                                         //  folded values is an sc1 load, fld())
}

// a folded value: sc1 (agent-scope relaxed) load when it was published inside this launch, else a plain load
__device__ __forceinline__ float fld(const float* p, bool sc) {
#ifdef IMAGENT_BN_APPLY_SERIAL
    return sc ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
#else
    // always the sc1 load: an L2-coherent read is as valid for a value written before the launch, and a runtime
    // choice between two loads made every per-channel constant a branch with its own load and wait
    (void)sc;
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

// ---------------------------------------------------------------- forward
// y = relu?( (x-mean)*rstd*g + b  [+ res | + (x2-mean2)*rstd2*g2 + b2] )
// NT: non-temporal output stores; Q8: also the e4m3 copy y8 (fp8 path; the plain kernel carries none
// of its code: 94 -> fewer VGPRs)
template <int MODE, bool RELU, bool NT, bool Q8>  // MODE 0: none, 1: identity residual, 2: second BN branch
__global__ __launch_bounds__(256) void bn_fwd_kernel(
    const bf16_t* __restrict__ x, const float* sums, const float* __restrict__ gamma,
    const float* __restrict__ beta, const bf16_t* __restrict__ x2, const float* __restrict__ sums2,
    const float* __restrict__ gamma2, const float* __restrict__ beta2, bf16_t* __restrict__ y,
    float* __restrict__ save, float* __restrict__ save2, long R, int C, float inv_cnt, float eps,
    int eval, uint32_t* __restrict__ y8, const int* __restrict__ exp8, float* __restrict__ amax8,
    uint8_t* __restrict__ ym, float* __restrict__ colsum, SlabFold fold) {
    if (fold.slab) fold_publish(fold, C, true, C);  // (mode 0; `sums` is fold.out: read after fold_wait)
    const int cpr = C / 8;                // chunks per row
    const int rpb = 256 / cpr;            // rows per block-iteration (C <= 2048)
    const int tid = threadIdx.x;
    // fp8 copy of the output for the next conv (delayed-scaled e4m3, fp8.hip)
    const float q8 = Q8 ? ldexpf(1.f, -exp8[0]) : 0.f;
    float m8 = 0.f;
    // colsum (mode 0): column sums of the stored (bf16) output -- the Gram-form bn3 backward's 1^T h2
    // (bn_gram.hip) -- per thread over its rows, folded over the block's row groups, one atomic per
    // channel per block (host: C / 8 divides 256, every lane active)
    float cs[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) cs[i] = 0.f;
    if (fold.slab) fold_wait(fold, C);
    if (tid >= rpb * cpr) return;  // (host: with y8, every lane is active -- C/8 divides 256)
    const int ch = tid % cpr, c0 = ch * 8;
    float sc[8], sh[8], sc2[8], sh2[8];
    // per-channel constants by 16-B loads (c0 % 8 == 0, 32-B aligned arrays)
    auto consts = [&](const float* su, const float* g, const float* b, float* sv, float (&k)[8], float (&o)[8]) {
        float s0[8], s1[8], gg[8], bb[8];
        if (fold.slab && su == sums) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                s0[i] = fld(su + c0 + i, true);
                s1[i] = fld(su + C + c0 + i, true);
            }
        } else {
            ld8f(su + c0, s0);
            ld8f(su + C + c0, s1);
        }
        ld8f(g + c0, gg);
        ld8f(b + c0, bb);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            // training: the finalized batch (mean, biased variance); eval: the running ones
            const float mean = s0[i], rstd = rsqrtf(s1[i] + eps);
            k[i] = rstd * gg[i];
            o[i] = bb[i] - mean * k[i];
            if (sv && blockIdx.x == 0 && tid < cpr) {
                sv[c0 + i] = mean;
                sv[C + c0 + i] = rstd;
            }
        }
    };
    consts(sums, gamma, beta, save, sc, sh);
    if (MODE == 2) consts(sums2, gamma2, beta2, save2, sc2, sh2);
    // U rows per thread per iteration, all loads issued before any math: 4x
    // the bytes in flight of a one-row loop (HBM needs ~72 KiB per CU). The rows stay packed
    // bf16 words until their math (unpacked early they doubled the VGPRs: 4 waves/SIMD -> 6+)
    // block-contiguous rows: a block's iteration covers U*rpb consecutive rows (scripts/stream_bench.hip:
    // +1-2 % over U rows gridDim*rpb apart)
    const long step = rpb;
    for (long r0 = (long)blockIdx.x * U * rpb + tid / cpr; r0 < R; r0 += (long)gridDim.x * U * rpb) {
        u32x4 v[U], s[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // unconditional loads from a clamped row: a guarded load makes hipcc branch
            // around it and wait vmcnt(0) per row (2 loads in flight instead of 2U)
            const long r = min(r0 + u * step, R - 1);
            v[u] = ldw(x + (size_t)r * C + c0);
            if (MODE != 0) s[u] = ldw(x2 + (size_t)r * C + c0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long r = r0 + u * step;
            if (r >= R) break;
            float o8[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                float o = fmaf(bfw(v[u], i), sc[i], sh[i]);
                if (MODE == 1) o += bfw(s[u], i);
                if (MODE == 2) o += fmaf(bfw(s[u], i), sc2[i], sh2[i]);
                o8[i] = RELU ? fmaxf(o, 0.f) : o;
            }
            u32x4 pw;
#pragma unroll
            for (int i = 0; i < 4; ++i) pw[i] = pack_bf2(o8[2 * i], o8[2 * i + 1]);
            stw<NT>(y + (size_t)r * C + c0, pw);
            if (MODE == 0 && colsum) {
#pragma unroll
                for (int i = 0; i < 8; ++i) cs[i] += bfw(pw, i);
            }
            if (MODE != 0 && RELU && ym) {  // the ReLU mask as bits for the backward's dgrad epilogue
                uint32_t b = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) {  // stored bf16 > 0: nonzero, sign clear, not NaN
                    const uint32_t h = (pw[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
                    b |= (h != 0u && h <= 0x7F80u ? 1u : 0u) << i;
                }
                ym[((size_t)r * C + c0) >> 3] = (uint8_t)b;
            }
            if (Q8) {
                // quantise the bf16-rounded output the bf16 consumers see (unpacked
                // from the stored words: one shift / mask per value)
                float w[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) w[i] = bfw(pw, i);
#pragma unroll
                for (int i = 0; i < 8; ++i) m8 = fmaxf(m8, fabsf(w[i]));
                reinterpret_cast<u32x2*>(y8)[((size_t)r * C + c0) / 8] =
                    u32x2{pack4_fp8(w[0] * q8, w[1] * q8, w[2] * q8, w[3] * q8),
                          pack4_fp8(w[4] * q8, w[5] * q8, w[6] * q8, w[7] * q8)};
            }
        }
    }
    if (MODE == 0 && colsum) {
        __shared__ float red[256][9];  // [thread][channel of its chunk] (+1: bank spread)
#pragma unroll
        for (int i = 0; i < 8; ++i) red[tid][i] = cs[i];
        __syncthreads();
        for (int c = tid; c < C; c += 256) {
            const int cc = c / 8, i = c % 8;
            float t = 0.f;
            for (int g = 0; g < rpb; ++g) t += red[g * cpr + cc][i];
            atomicAdd(colsum + c, t);
        }
    }
    if (Q8) {  // every lane active (host check): block max, one atomic per block into a 32-slot amax row
        __shared__ float wm[4];
        m8 = wave_max(m8);
        if ((tid & 63) == 0) wm[tid >> 6] = m8;
        __syncthreads();
        if (tid == 0) atomic_max_pos(amax8 + (blockIdx.x & 31), fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3])));
    }
}

// ---------------------------------------------------------------- deterministic mode
// IMAGENT_DETERMINISTIC=1 (ops/conv.py set_deterministic): batch statistics without float atomics, so two
// passes over the same data give bit-identical BatchNorm statistics (and everything downstream of them).
// Forward: the conv runs without its epilogue statistics and this pass reads its output: per-thread sums
// over a fixed row sequence, a fixed-order fold of the block's rows in LDS, one plain store per channel
// into the block's own partial row, then det_fold_kernel adds the rows in block order into slot 0 of the
// BN's slab. Backward: bn_bwd_reduce_kernel with `partial` (the same fold). Same statistics as the
// epilogue path (shifted sums around work.save, imk_bn_stats_finalize), different summation order.
__global__ __launch_bounds__(256) void bn_stats_det_kernel(const bf16_t* __restrict__ y, const float* __restrict__ shift,
                                                           float* __restrict__ partial, long R, int C) {
    __shared__ float red[2048];  // [rpb][C]
    const int cpr = C / 8, rpb = 256 / cpr, tid = threadIdx.x;
    const bool active = tid < rpb * cpr;
    const int c0 = (tid % cpr) * 8, rsub = tid / cpr;
    float sh[8], s1[8], s2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        sh[i] = shift ? shift[c0 + i] : 0.f;
        s1[i] = s2[i] = 0.f;
    }
    if (active) {
        const long step = (long)gridDim.x * rpb;
        for (long r0 = (long)blockIdx.x * rpb + rsub; r0 < R; r0 += U * step) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = ldw(y + (size_t)min(r0 + u * step, R - 1) * C + c0);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (r0 + u * step >= R) break;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float d = bfw(v[u], i) - sh[i];
                    s1[i] += d;
                    s2[i] += d * d;
                }
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        __syncthreads();
        if (active) {
#pragma unroll
            for (int i = 0; i < 8; ++i) red[rsub * C + c0 + i] = q ? s2[i] : s1[i];
        }
        __syncthreads();
        for (int c = tid; c < C; c += 256) {
            float t = 0.f;
            for (int rr = 0; rr < rpb; ++rr) t += red[rr * C + c];
            partial[(size_t)blockIdx.x * 2 * C + q * C + c] = t;
        }
    }
}

// out[i] += sum over b = 0 .. nb - 1 (in that order) of partial[b * stride + i], i < n
// 16 columns per 256-thread block, 16 fixed row partitions per column (rows b = part, part + 16, ...) summed
// in order, then the 16 partition sums in order: deterministic, and 16 independent load streams per column
// instead of one serial walk over up to 1024 rows
constexpr int DET_COLS = 16;
__global__ __launch_bounds__(256) void det_fold_kernel(const float* __restrict__ partial, int nb, int stride, int n,
                                                       float* __restrict__ out) {
    __shared__ float red[16][DET_COLS];
    const int cl = threadIdx.x % DET_COLS, part = threadIdx.x / DET_COLS;
    const int i = blockIdx.x * DET_COLS + cl;
    float s = 0.f;
    if (i < n)
#pragma unroll 8
        for (int b = part; b < nb; b += 16) s += partial[(size_t)b * stride + i];  // loads batched, adds in order
    red[part][cl] = s;
    __syncthreads();
    if (part || i >= n) return;
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][cl];
    out[i] += t;
}

int g_det = 0;            // deterministic mode (imk_set_deterministic)
float* g_det_ws = nullptr;  // BN-backward partial rows (main stream only): <= 1024 blocks x 3 x 2048 channels
constexpr size_t DET_WS_FLOATS = (size_t)1024 * 3 * 2048;

// inference BatchNorm as the conv epilogue's per-channel [scale; shift] (IG_AFFINE), for every BN of the
// model in ONE launch over a descriptor table (models/native.py _forward_eval): out = [g rstd; b - mean g rstd]
struct AffDesc {
    const float* gamma;
    const float* beta;
    const float* rmean;
    const float* rvar;
    float* out;
    int C;
    float eps;
};

__global__ void bn_eval_affine_kernel(const AffDesc* __restrict__ d, int n) {
    const AffDesc a = d[blockIdx.x];
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
        const float sc = a.gamma[c] * rsqrtf(a.rvar[c] + a.eps);
        a.out[c] = sc;
        a.out[a.C + c] = a.beta[c] - a.rmean[c] * sc;
    }
}

// running stats update + num_batches_tracked: all layers of a step are updated
// by ONE launch over a descriptor table (imk_bn_running_update)
struct RunDesc {
    const float* sums;
    float* rmean;
    float* rvar;
    long long* nbt;
    int C;
    float inv_cnt, unbias, momentum;
};

__global__ void bn_running_kernel(const RunDesc* __restrict__ d, int n) {
    const RunDesc a = d[blockIdx.x];
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
        const float mean = a.sums[c], var = a.sums[a.C + c];  // finalized (mean, biased variance)
        a.rmean[c] = (1.f - a.momentum) * a.rmean[c] + a.momentum * mean;
        a.rvar[c] = (1.f - a.momentum) * a.rvar[c] + a.momentum * var * a.unbias;
    }
    if (threadIdx.x == 0 && a.nbt) a.nbt[0] += 1;
}

// Fold the conv epilogue's [S][2][C] SHIFTED statistics slab (sum d, sum d^2
// with d = v - shift[c]) into [2][C] = (mean, biased variance), fixed fold order:
//   mean = shift + E[d],  var = E[d^2] - E[d]^2   (no cancellation when shift ~ mean)
__global__ __launch_bounds__(64) void stats_finalize_mv_kernel(const float* __restrict__ slab,
                                                               const float* __restrict__ shift,
                                                               float* __restrict__ out, int S, int C,
                                                               float inv_cnt) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c >= C) return;
    float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int k = 0; k < S; ++k) {
        a[k & 3] += slab[(size_t)k * 2 * C + c];
        b[k & 3] += slab[(size_t)k * 2 * C + C + c];
    }
    const float m1 = ((a[0] + a[1]) + (a[2] + a[3])) * inv_cnt;
    const float m2 = ((b[0] + b[1]) + (b[2] + b[3])) * inv_cnt;
    out[c] = (shift ? shift[c] : 0.f) + m1;
    out[C + c] = fmaxf(m2 - m1 * m1, 0.f);
}

// stats_finalize_mv + the BatchNorm's per-channel affine: for a BN whose apply + ReLU runs on the
// consumer conv's operand load (ops/block.py, conv_stream XBN / wgrad XB) this replaces the forward
// pass: save = (mean, rstd) as bn_fwd_kernel writes it, ss = (gamma * rstd, beta - mean * gamma * rstd)
__global__ __launch_bounds__(64) void stats_finalize_affine_kernel(const float* __restrict__ slab,
                                                                   float* __restrict__ save, float* __restrict__ out,
                                                                   const float* __restrict__ gamma,
                                                                   const float* __restrict__ beta,
                                                                   float* __restrict__ ss, int S, int C,
                                                                   float inv_cnt, float eps, int use_shift) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    if (c >= C) return;
    float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int k = 0; k < S; ++k) {
        a[k & 3] += slab[(size_t)k * 2 * C + c];
        b[k & 3] += slab[(size_t)k * 2 * C + C + c];
    }
    const float m1 = ((a[0] + a[1]) + (a[2] + a[3])) * inv_cnt;
    const float m2 = ((b[0] + b[1]) + (b[2] + b[3])) * inv_cnt;
    const float mean = (use_shift ? save[c] : 0.f) + m1;  // shift = the previous batch mean (read first)
    const float var = fmaxf(m2 - m1 * m1, 0.f);
    out[c] = mean;
    out[C + c] = var;
    const float rstd = rsqrtf(var + eps), sc = gamma[c] * rstd;
    save[c] = mean;
    save[C + c] = rstd;
    ss[c] = sc;
    ss[C + c] = beta[c] - mean * sc;
}

// Fold a [S][n] slab into [n] sums (backward reductions).
__global__ __launch_bounds__(64) void stats_finalize_kernel(const float* __restrict__ slab,
                                                            float* __restrict__ out, int S, int n) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int k = 0; k < S; ++k) s[k & 3] += slab[(size_t)k * n + i];
    out[i] = (s[0] + s[1]) + (s[2] + s[3]);
}

// ---------------------------------------------------------------- backward
// MASK 0: no ReLU; 1: ReLU mask from the saved output y; 2: from x (mode 0 only:
// y = relu(fma(x, sc, sh)) with the forward's sc = rstd*gamma, sh = beta - mean*sc)
template <int MASK>
__device__ __forceinline__ void relu_mask(Vec8& g, const u32x4& yw, const Vec8& xv, const float* sc,
                                          const float* sh) {
    if (MASK == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (!(lo_bf(yw[i]) > 0.f)) g.v[2 * i] = 0.f;
            if (!(hi_bf(yw[i]) > 0.f)) g.v[2 * i + 1] = 0.f;
        }
    } else if (MASK == 2) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (!(fmaf(xv.v[i], sc[i], sh[i]) > 0.f)) g.v[i] = 0.f;
    }
}

// per-channel sums  Sg = sum g,  Sgx = sum g * xhat  (MODE 2 also Sgx2 over
// the downsample branch x2) into a zeroed fp32 scratch [3][C], one atomic per
// channel per block.
template <int MASK, int MODE>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const bf16_t* __restrict__ x,
    const float* __restrict__ save, const float* __restrict__ gamma, const float* __restrict__ beta,
    const bf16_t* __restrict__ x2, const float* __restrict__ save2, float* __restrict__ scratch, long R,
    int C, float* __restrict__ partial) {
    __shared__ float red[2048];  // [rpb][C], rpb*C == 2048
    const int cpr = C / 8, rpb = 256 / cpr, tid = threadIdx.x;
    const bool active = tid < rpb * cpr;
    const int ch = tid % cpr, c0 = ch * 8, rsub = tid / cpr;
    float mean[8], rstd[8], m2[8], r2[8], sc[8], sh[8];
    float acc[3][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        mean[i] = save[c0 + i];
        rstd[i] = save[C + c0 + i];
        if (MASK == 2) {
            sc[i] = rstd[i] * gamma[c0 + i];
            sh[i] = beta[c0 + i] - mean[i] * sc[i];
        }
        if (MODE == 2) {
            m2[i] = save2[c0 + i];
            r2[i] = save2[C + c0 + i];
        }
        acc[0][i] = acc[1][i] = acc[2][i] = 0.f;
    }
    if (active) {
        const long step = (long)gridDim.x * rpb;
        for (long r0 = (long)blockIdx.x * rpb + rsub; r0 < R; r0 += U * step) {
            Vec8 g[U], xv[U], x2v[U];
            u32x4 yv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                // clamped row, unconditional loads (see bn_fwd_kernel); rows past R add 0
                const size_t off = (size_t)min(r0 + u * step, R - 1) * C + c0;
                g[u] = ld8(dy + off);
                xv[u] = ld8(x + off);
                if (MODE == 2) x2v[u] = ld8(x2 + off);
                if (MASK == 1) yv[u] = *reinterpret_cast<const u32x4*>(y + off);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const long r = r0 + u * step;
                relu_mask<MASK>(g[u], yv[u], xv[u], sc, sh);
                if (r >= R) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) g[u].v[i] = 0.f;
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    acc[0][i] += g[u].v[i] * (xv[u].v[i] - mean[i]) * rstd[i];
                    acc[1][i] += g[u].v[i];
                    if (MODE == 2) acc[2][i] += g[u].v[i] * (x2v[u].v[i] - m2[i]) * r2[i];
                }
            }
        }
    }
    const int nq = MODE == 2 ? 3 : 2;
#pragma unroll
    for (int qi = 0; qi < 3; ++qi) {
        if (qi >= nq) break;
        __syncthreads();
        if (active) {
#pragma unroll
            for (int i = 0; i < 8; ++i) red[rsub * C + c0 + i] = acc[qi][i];
        }
        __syncthreads();
        // one add per channel per block into slot (block & 31) of the [32][3][C]
        // slab: 1024 blocks adding into the same 3*C words serialise at the
        // memory-side atomic unit (the conv-epilogue statistics lesson)
        // (deterministic mode: a plain store into this block's own row of `partial`, folded in block order)
        float* slot = scratch + (size_t)(blockIdx.x & (BWD_SLOTS - 1)) * 3 * C;
        for (int c = tid; c < C; c += 256) {
            float s = 0.f;
            for (int rr = 0; rr < rpb; ++rr) s += red[rr * C + c];
            if (partial)
                partial[(size_t)blockIdx.x * 3 * C + qi * C + c] = s;
            else
                atomicAdd(slot + qi * C + c, s);
        }
    }
}

// dx = gamma*rstd*(g - Sg/R - xhat*Sgx/R) = k1 g + kx x + k0 per channel; MODE 1 also writes the
// residual gradient g, MODE 2 the downsample-branch input gradient. Block 0 also adds the sums into
// the arena slots of dgamma/dbeta (+= : gradient accumulation). Rows stay packed bf16 words until
// their math and the per-channel constants are three FMAs' worth (108 -> fewer VGPRs, more waves).
template <int MASK, int MODE, bool NT, bool Q8, bool NTL = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y, const bf16_t* __restrict__ x,
    const float* __restrict__ save, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* scratch, bf16_t* __restrict__ dx, bf16_t* __restrict__ dres,
    const bf16_t* __restrict__ x2, const float* __restrict__ save2, const float* __restrict__ gamma2,
    bf16_t* __restrict__ dx2, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ dgamma2, float* __restrict__ dbeta2, long R, int C, float inv_cnt, G8Out g8, int sgxo,
    SlabFold fold) {
    if (fold.slab) {  // (`scratch` is fold.out)
        fold_publish(fold, 3 * C, false, C);
        fold_wait(fold, 3 * C);
    }
    constexpr int UB = MODE == 2 ? 2 : U;  // three streams in, two out: half the rows in flight
    const int cpr = C / 8, rpb = 256 / cpr, tid = threadIdx.x;
    const float qs0 = Q8 && g8.q[0] ? ldexpf(1.f, -g8.exp[0][0]) : 0.f;
    const float qs1 = Q8 && g8.q[1] ? ldexpf(1.f, -g8.exp[1][0]) : 0.f;
    float m0 = 0.f, m1 = 0.f;
#ifdef IMAGENT_BN_DG_BLOCK0
    if (blockIdx.x == 0) {
        for (int c = tid; c < C; c += 256) {
            const bool sc = fold.slab != nullptr;
            if (dgamma) dgamma[c] += fld(scratch + sgxo + c, sc);
            if (dbeta) dbeta[c] += fld(scratch + C + c, sc);
            if (MODE == 2) {
                if (dgamma2) dgamma2[c] += fld(scratch + 2 * C + c, sc);
                if (dbeta2) dbeta2[c] += fld(scratch + C + c, sc);
            }
        }
    }
#else
    // dgamma / dbeta accumulation spread over the first ceil(C / 256) blocks, one channel per thread, every operand
    // loaded before the first store (formerly block 0 alone walked C / 256 iterations whose read-modify-writes the
    // possible aliasing of dgamma / dbeta / scratch serialised into the pass's tail). scripts/runs/dg_ab.sh, one box:
    // 256 img 12,922 / 12,941 vs 12,921 / 12,954 img/s (block 0 alone, -DIMAGENT_BN_DG_BLOCK0), 4096 img 17,312 vs
    // 17,197 -- neutral at small batch, kept (no serial section left in the pass)
    for (int c = blockIdx.x * 256 + tid; c < C; c += gridDim.x * 256) {
        const bool sc = fold.slab != nullptr;
        const float sgx = fld(scratch + sgxo + c, sc), sg = fld(scratch + C + c, sc);
        const float sgx2 = MODE == 2 ? fld(scratch + 2 * C + c, sc) : 0.f;
        const float og = dgamma ? dgamma[c] : 0.f, ob = dbeta ? dbeta[c] : 0.f;
        const float og2 = MODE == 2 && dgamma2 ? dgamma2[c] : 0.f, ob2 = MODE == 2 && dbeta2 ? dbeta2[c] : 0.f;
        if (dgamma) dgamma[c] = og + sgx;
        if (dbeta) dbeta[c] = ob + sg;
        if (MODE == 2) {
            if (dgamma2) dgamma2[c] = og2 + sgx2;
            if (dbeta2) dbeta2[c] = ob2 + sg;
        }
    }
#endif
    if (tid >= rpb * cpr) return;
    const int ch = tid % cpr, c0 = ch * 8;
    float k1[8], kx[8], k0[8], q1[8], qx[8], q0[8], sc[8], sh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int c = c0 + i;
        const float mean = save[c], rstd = save[C + c];
        const float gr = gamma[c] * rstd;
        if (MASK == 2) {
            sc[i] = gr;
            sh[i] = beta[c] - mean * gr;
        }
        const bool sc = fold.slab != nullptr;
        k1[i] = gr;
        kx[i] = -gr * inv_cnt * fld(scratch + sgxo + c, sc) * rstd;
        k0[i] = -gr * inv_cnt * fld(scratch + C + c, sc) - kx[i] * mean;
        if (MODE == 2) {
            const float m2 = save2[c], rs2 = save2[C + c];
            const float g2 = gamma2[c] * rs2;
            q1[i] = g2;
            qx[i] = -g2 * inv_cnt * fld(scratch + 2 * C + c, sc) * rs2;
            q0[i] = -g2 * inv_cnt * fld(scratch + C + c, sc) - qx[i] * m2;
        }
    }
    const long step = rpb;  // block-contiguous rows (see bn_fwd_kernel)
    for (long r0 = (long)blockIdx.x * UB * rpb + tid / cpr; r0 < R; r0 += (long)gridDim.x * UB * rpb) {
        u32x4 g[UB], xv[UB], x2v[UB], yv[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            // clamped row, unconditional loads (see bn_fwd_kernel); rows past R are not stored
            const size_t off = (size_t)min(r0 + u * step, R - 1) * C + c0;
            g[u] = ldwn<NTL>(dy + off);
            xv[u] = ldwn<NTL>(x + off);
            if (MODE == 2) x2v[u] = ldwn<NTL>(x2 + off);
            if (MASK == 1) yv[u] = ldwn<NTL>(y + off);
        }
#ifndef IMAGENT_BN_APPLY_SERIAL
        // every row's loads stay issued before any math: left alone, the compiler sank the loads of rows 1..U-1 below
        // the previous row's `r >= R` exit, so a wave had ONE row (g, x) in flight -- load, wait, math, store, next
        // row (the forward pass kept its U rows). An empty asm that takes every loaded chunk as a register operand pins
        // the loads above it (one wait for all of them); the rows past R compute on clamped loads and are not stored.
        // scripts/runs/apply_ab.sh, one box: per-step apply passes at 256 img 3,511 -> 3,038 us, bench.py 256 img
        // 12,992 -> 13,369 / 13,370 img/s, 4096 img 17,183 / 17,221 -> 17,227 / 17,273 (2048-img passes isolated +1.7 %)
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            asm volatile("" ::"v"(g[u]), "v"(xv[u]));
            if (MODE == 2) asm volatile("" ::"v"(x2v[u]));
            if (MASK == 1) asm volatile("" ::"v"(yv[u]));
        }
#endif
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            const long r = r0 + u * step;
#ifdef IMAGENT_BN_APPLY_SERIAL
            if (r >= R) break;
#else
            if (r >= R) continue;
#endif
            const size_t off = (size_t)r * C + c0;
            float gv[8], o[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                gv[i] = bfw(g[u], i);
                if (MASK == 1 && !(bfw(yv[u], i) > 0.f)) gv[i] = 0.f;
                if (MASK == 2 && !(fmaf(bfw(xv[u], i), sc[i], sh[i]) > 0.f)) gv[i] = 0.f;
                o[i] = fmaf(k1[i], gv[i], fmaf(kx[i], bfw(xv[u], i), k0[i]));
            }
            stq<NT, Q8>(dx + off, o, g8.q[0], off, qs0, m0);
            if (MODE == 1) {
                u32x4 w;
#pragma unroll
                for (int i = 0; i < 4; ++i) w[i] = pack_bf2(gv[2 * i], gv[2 * i + 1]);
                stw<NT>(dres + off, w);
            }
            if (MODE == 2) {
#pragma unroll
                for (int i = 0; i < 8; ++i) o[i] = fmaf(q1[i], gv[i], fmaf(qx[i], bfw(x2v[u], i), q0[i]));
                stq<NT, Q8>(dx2 + off, o, g8.q[1], off, qs1, m1);
            }
        }
    }
    if (Q8) {  // every lane active (host check): block max -> slot (blockIdx & 31)
        __shared__ float wm[2][4];
        m0 = wave_max(m0);
        m1 = wave_max(m1);
        if ((tid & 63) == 0) {
            wm[0][tid >> 6] = m0;
            wm[1][tid >> 6] = m1;
        }
        __syncthreads();
        if (tid < 2 && g8.q[tid])
            atomic_max_pos(g8.amax[tid] + (blockIdx.x & 31),
                           fmaxf(fmaxf(wm[tid][0], wm[tid][1]), fmaxf(wm[tid][2], wm[tid][3])));
    }
}

// non-temporal stores of the streamed outputs: scripts/bn_bench.py at batch 1024, per step fwd 9328 -> 9077 us,
// bwd apply 12310 -> 12053 us (round 3; in-step within noise at round-4 HEAD, kept)
constexpr bool bn_nt() { return true; }

// Streaming passes size their grid by grid_for (<= 2048 blocks = 8 per CU); a variant whose registers allow
// fewer resident blocks per CU (bn_fwd mode 1: 94 VGPRs, 5 waves / SIMD) then runs its grid-stride loop in
// 1.6 "rounds", the last one on 60 % of the slots. resident_grid caps the grid at what fits at once
// (round 3: +0.2 % img/s, within noise; kept because the capped grid never does worse).
int resident_grid(const void* kernel, int grid) {
    static std::mutex mu;
    static std::unordered_map<const void*, int> cap;
    static int ncu = 0;
    std::lock_guard<std::mutex> lk(mu);
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = -1;
    }
    if (ncu < 0) return grid;
    auto it = cap.find(kernel);
    if (it == cap.end()) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu <= 0)
            per_cu = 1 << 20;  // unknown: no cap
        it = cap.emplace(kernel, per_cu * ncu).first;
    }
    return grid < it->second ? grid : it->second;
}

// backward apply pass: blocks per CU of its grid and non-temporal operand loads. The streaming roof of the r2w1
// pattern (g, x in; dx out) is highest at LOW occupancy with NT accesses (scripts/hbm_roof.hip, profiles/
// hbm_roof.md: 6.32 TB/s at 2 blocks / CU vs 5.7-5.8 at 8). Round 6, same box, bench.py at 2048 img: 8 blocks / CU
// plain loads 17,351 / 17,363 img/s, 2 + NT 17,458 / 17,478, 4 + NT 17,541 (scripts/bn_bench.py: bwd apply per
// step 25.15 -> 23.75 ms). IMAGENT_BN_APPLY_BPC / IMAGENT_BN_NTLOAD override.
static int env_int(const char* k, int d) {
    const char* v = getenv(k);
    return v && *v ? atoi(v) : d;
}
static int apply_bpc() {
    static const int v = env_int("IMAGENT_BN_APPLY_BPC", 4);
    return v;
}
// Non-temporal loads at every size by default: with the loads batched, plain loads below 256 MB per tensor won
// isolated at 256 img (scripts/bn_bench.py, operands still cached from the previous call: apply passes 3,036 ->
// 2,915 us per step) but lost in-step (bench.py 256 img 13,492 / 13,510 NT vs 13,453 / 13,427 img/s,
// scripts/runs/ntmin_ab.sh). IMAGENT_BN_NTLOAD_MIN_MB: smallest tensor (MB) that takes NT loads (A/B).
static bool apply_ntload(long R, int C) {
    static const bool v = env_int("IMAGENT_BN_NTLOAD", 1) != 0;
    static const long min_bytes = (long)env_int("IMAGENT_BN_NTLOAD_MIN_MB", 0) << 20;
    return v && R * (long)C * 2 >= min_bytes;
}
static int n_cus() {
    static const int n = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
        return cus;
    }();
    return n;
}

int grid_for(long R, int C) {
    const int rpb = 256 / (C / 8);
    long blocks = (R + U * rpb - 1) / (U * rpb);
    // 8 resident blocks per CU (2048 threads) for streaming, then grid-stride
    return (int)(blocks < 2048 ? blocks : 2048);
}

}  // namespace

// mode: 0 plain, 1 + identity residual (x2), 2 + second BN branch (x2, sums2, gamma2, beta2)
// y8 (optional): e4m3 copy of y quantised with 2^-exp8[0]; amax8 ([32] slots,
// folded by imk_fp8_update_exp) receives max |y|; ym (optional, modes 1 / 2 with ReLU): the mask
// y > 0 as bits, byte e/8 of element e (IGemmArgs.bnym)
IMK_EXPORT int imk_bn_fwd(const void* x, const float* sums, const float* gamma, const float* beta,
                          const void* x2, const float* sums2, const float* gamma2, const float* beta2,
                          void* y, float* save, float* save2, long R, int C, int mode, int relu,
                          float eps, int eval, void* y8, const int* exp8, float* amax8, void* ym,
                          float* colsum, const float* fslab, const float* fshift, void* fcnt, int fS,
                          void* stream) {
    if (C % 8 || C > 2048) return -100;
    if (y8 && (256 % (C / 8) || !exp8 || !amax8)) return -102;
    if (colsum && (mode != 0 || 256 % (C / 8))) return -103;
    // fslab: fold the conv epilogue's [fS][2][C] shifted-sum slab into `sums` inside this pass (mode 0, training)
    if (fslab && (mode != 0 || eval || !fcnt || fS != FOLD_S)) return -104;
    const SlabFold fold{fslab, fshift, const_cast<float*>(sums), static_cast<uint32_t*>(fcnt), fS, 1.f / (float)R};
    const float inv_cnt = 1.f / (float)R;
    const int grid = std::max(grid_for(R, C), fslab ? (C + 255) / 256 : 1);
    hipStream_t st = (hipStream_t)stream;
    const bool nt = bn_nt(), q8 = y8 != nullptr;
#define LK(M, RL, NT, Q8)                                                                               \
    hipLaunchKernelGGL((bn_fwd_kernel<M, RL, NT, Q8>),                                                  \
                       dim3(resident_grid((const void*)bn_fwd_kernel<M, RL, NT, Q8>, grid)), dim3(256), 0, st, (const bf16_t*)x, sums, \
                       gamma, beta, (const bf16_t*)x2, sums2, gamma2, beta2, (bf16_t*)y, save, save2, R, C,   \
                       inv_cnt, eps, eval, (uint32_t*)y8, exp8, amax8, (uint8_t*)ym, colsum, fold)
#define L(M, RL)                                              \
    do {                                                      \
        if (q8) { if (nt) LK(M, RL, true, true); else LK(M, RL, false, true); }   \
        else { if (nt) LK(M, RL, true, false); else LK(M, RL, false, false); } \
    } while (0)
    if (mode == 0) { if (relu) L(0, true); else L(0, false); }
    else if (mode == 1) { if (relu) L(1, true); else L(1, false); }
    else { if (relu) L(2, true); else L(2, false); }
#undef LK
#undef L
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_bn_running_update(const void* descs, int n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(bn_running_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream,
                       (const RunDesc*)descs, n);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_bn_rundesc_size() { return (int)sizeof(RunDesc); }

IMK_EXPORT int imk_bn_eval_affine(const void* descs, int n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(bn_eval_affine_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, (const AffDesc*)descs, n);
    IMK_CHECK_LAUNCH();
    return 0;
}
IMK_EXPORT int imk_bn_affdesc_size() { return (int)sizeof(AffDesc); }

// Apply-only backward for a gradient g that the producing dgrad already
// ReLU-masked, with its reductions already in the [BWD_SLOTS][3][C] slab of
// `scratch` (conv epilogue IG_BNBWD): fold + dx (mode 0/1; for mode 1 the
// caller uses g itself as the residual-branch gradient) or dx, dx2 (mode 2).
IMK_EXPORT int imk_bn_bwd_apply(const void* g, const void* x, const float* save, const float* gamma,
                                const void* x2, const float* save2, const float* gamma2, float* scratch,
                                void* dx, void* dx2, float* dgamma_acc, float* dbeta_acc, float* dgamma2_acc,
                                float* dbeta2_acc, long R, int C, int mode, const void* g8desc, int sgx_row,
                                int fold_in, void* stream) {
    // sgx_row (mode 0 / 1): the slab row holding sum(g xhat) -- 2 when `scratch` is a Gram-form bn3's slab whose
    // third row the producing dgrad filled with the downsample BN's sum(g xhat_d) (ops/block.py)
    if (C % 8 || C > 2048 || sgx_row < 0 || sgx_row > 2 || (mode == 2 && sgx_row)) return -100;
    // g8desc (host pointer, may be null): {q0, q1, exp0, exp1, amax0, amax1} device pointers of the
    // e5m2 copies of dx / dx2 (fp8 dgrad)
    G8Out g8{};
    if (g8desc) {
        const void* const* d = static_cast<const void* const*>(g8desc);
        g8.q[0] = (uint32_t*)d[0];
        g8.q[1] = (uint32_t*)d[1];
        g8.exp[0] = (const int*)d[2];
        g8.exp[1] = (const int*)d[3];
        g8.amax[0] = (float*)d[4];
        g8.amax[1] = (float*)d[5];
        if ((g8.q[0] || g8.q[1]) && 256 % (C / 8)) return -102;
    }
    hipStream_t st = (hipStream_t)stream;
    float* folded = scratch + (size_t)BWD_SLOTS * 3 * C;
    // fold_in: the apply pass folds the slab itself (SlabFold; its counter in the scratch's last row), else one
    // launch of its own
    SlabFold fold{};
    static const bool fold_ok = env_int("IMAGENT_BN_FOLD_IN", 1) != 0;  // 0: the separate fold launch (A/B)
    fold_in = fold_in && fold_ok;
    if (fold_in) {
        fold = SlabFold{scratch, nullptr, folded, reinterpret_cast<uint32_t*>(folded + 3 * C), BWD_SLOTS, 0.f};
    } else {
        hipLaunchKernelGGL(stats_finalize_kernel, dim3((3 * C + 63) / 64), dim3(64), 0, st, scratch, folded,
                           BWD_SLOTS, 3 * C);
        IMK_CHECK_LAUNCH();
    }
    const int grid = std::max(std::min(grid_for(R, C), apply_bpc() * n_cus()), fold_in ? (3 * C + 255) / 256 : 1);
    const float inv_cnt = 1.f / (float)R;
    const bool nt = bn_nt(), q8 = g8.q[0] || g8.q[1], ntl = apply_ntload(R, C);
#define LK(M, NT, Q8, NTL)                                                                           \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<0, M, NT, Q8, NTL>),                                          \
                       dim3(resident_grid((const void*)bn_bwd_apply_kernel<0, M, NT, Q8, NTL>, grid)), dim3(256), 0, st, (const bf16_t*)g, \
                       nullptr, (const bf16_t*)x, save, gamma, nullptr, folded, (bf16_t*)dx, nullptr,       \
                       (const bf16_t*)x2, save2, gamma2, (bf16_t*)dx2, dgamma_acc, dbeta_acc,               \
                       dgamma2_acc, dbeta2_acc, R, C, inv_cnt, g8, sgx_row * C, fold)
#define LA(M)                                                                  \
    do {                                                                       \
        if (q8) { if (nt) LK(M, true, true, false); else LK(M, false, true, false); }        \
        else if (ntl) LK(M, true, false, true);                                \
        else { if (nt) LK(M, true, false, false); else LK(M, false, false, false); }         \
    } while (0)
    if (mode == 2) LA(2); else LA(0);
#undef LK
#undef LA
    IMK_CHECK_LAUNCH();
    return 0;
}

// [BWD_SLOTS][3][C] slab, folded [3][C], one more row: word 0 the backward fold's counter, word 1 the forward's
IMK_EXPORT int imk_bn_bwd_scratch_floats(int C) { return (BWD_SLOTS * 3 + 4) * C; }

// forward statistics: shifted-sum slab [S][2][C] -> out [2][C] = (mean, biased variance)
// deterministic mode on / off; on: allocates the partial-row workspace once (no allocation inside a capture)
IMK_EXPORT int imk_set_deterministic(int on) {
    if (on && !g_det_ws && hipMalloc(&g_det_ws, DET_WS_FLOATS * sizeof(float)) != hipSuccess) return -1;
    g_det = on ? 1 : 0;
    return 0;
}

// forward BatchNorm statistics of y [R][C] (bf16) as shifted sums around `shift` (or raw sums) added to
// slot 0 of the [S][2][C] slab, in a fixed summation order (deterministic mode). `partial`: the caller's
// stream-ordered workspace of imk_bn_stats_det_floats(R, C) floats (the downsample conv's statistics run on
// the side stream beside the main chain's, so no shared scratch here)
IMK_EXPORT long imk_bn_stats_det_floats(long R, int C) { return (long)std::min(grid_for(R, C), 2048) * 2 * C; }

IMK_EXPORT int imk_bn_stats_det(const void* y, const float* shift, float* slab, float* partial, long R, int C,
                                void* stream) {
    if (C % 8 || C > 2048 || R <= 0 || !partial) return -100;
    hipStream_t st = (hipStream_t)stream;
    const int grid = std::min(grid_for(R, C), 2048);
    hipLaunchKernelGGL(bn_stats_det_kernel, dim3(grid), dim3(256), 0, st, (const bf16_t*)y, shift, partial, R, C);
    IMK_CHECK_LAUNCH();
    hipLaunchKernelGGL(det_fold_kernel, dim3((2 * C + DET_COLS - 1) / DET_COLS), dim3(256), 0, st, partial, grid, 2 * C, 2 * C,
                       slab);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_bn_stats_finalize(const float* slab, const float* shift, float* out, int S, int C, long R,
                                     void* stream) {
    if (R <= 0) return -100;
    hipLaunchKernelGGL(stats_finalize_mv_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream,
                       slab, shift, out, S, C, 1.f / (float)R);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_bn_finalize_affine(const float* slab, float* save, float* out, const float* gamma,
                                      const float* beta, float* ss, int S, int C, long R, float eps, int use_shift,
                                      void* stream) {
    if (R <= 0) return -100;
    hipLaunchKernelGGL(stats_finalize_affine_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, slab,
                       save, out, gamma, beta, ss, S, C, 1.f / (float)R, eps, use_shift);
    IMK_CHECK_LAUNCH();
    return 0;
}

// scratch: fp32 [BWD_SLOTS][3][C] slab followed by the folded [3][C], all
// zero-initialised by the caller.
// mode 0: plain, 1: also dres (= masked dy, identity residual), 2: also dx2 (downsample BN branch)
// relu: 0 none, 1 mask from y, 2 mask from x (mode 0 only; needs gamma/beta/save as in forward)
IMK_EXPORT int imk_bn_bwd(const void* dy, const void* y, const void* x, const float* save,
                          const float* gamma, const float* beta, const void* x2, const float* save2,
                          const float* gamma2, float* scratch, void* dx, void* dres, void* dx2,
                          float* dgamma_acc, float* dbeta_acc, float* dgamma2_acc,
                          float* dbeta2_acc, long R, int C, int mode, int relu, void* stream) {
    if (C % 8 || C > 2048) return -100;
    if (relu == 2 && mode != 0) return -101;
    hipStream_t st = (hipStream_t)stream;
    const int grid = grid_for(R, C);
    const int rgrid = grid < 1024 ? grid : 1024;
#define LR(MK, M)                                                                                  \
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<MK, M>), dim3(rgrid), dim3(256), 0, st,               \
                       (const bf16_t*)dy, (const bf16_t*)y, (const bf16_t*)x, save, gamma, beta,    \
                       (const bf16_t*)x2, save2, scratch, R, C, det)
    float* det = g_det ? g_det_ws : nullptr;
    if (mode == 2) { if (relu) LR(1, 2); else LR(0, 2); }
    else { if (relu == 2) LR(2, 0); else if (relu) LR(1, 0); else LR(0, 0); }
#undef LR
    IMK_CHECK_LAUNCH();
    if (det) {  // the blocks' rows in block order into slot 0
        const int n = (mode == 2 ? 3 : 2) * C;  // the quantities this mode reduces
        hipLaunchKernelGGL(det_fold_kernel, dim3((n + DET_COLS - 1) / DET_COLS), dim3(256), 0, st, det, rgrid, 3 * C, n, scratch);
        IMK_CHECK_LAUNCH();
    }
    float* folded = scratch + (size_t)BWD_SLOTS * 3 * C;
    hipLaunchKernelGGL(stats_finalize_kernel, dim3((3 * C + 63) / 64), dim3(64), 0, st, scratch, folded,
                       BWD_SLOTS, 3 * C);
    IMK_CHECK_LAUNCH();
    const float inv_cnt = 1.f / (float)R;
#define LA(MK, M)                                                                                  \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<MK, M, false, false>), dim3(grid), dim3(256), 0, st, (const bf16_t*)dy, \
                       (const bf16_t*)y, (const bf16_t*)x, save, gamma, beta, folded, (bf16_t*)dx,   \
                       (bf16_t*)dres, (const bf16_t*)x2, save2, gamma2, (bf16_t*)dx2, dgamma_acc,    \
                       dbeta_acc, dgamma2_acc, dbeta2_acc, R, C, inv_cnt, G8Out{}, 0, SlabFold{})
    if (mode == 0) { if (relu == 2) LA(2, 0); else if (relu) LA(1, 0); else LA(0, 0); }
    else if (mode == 1) { if (relu) LA(1, 1); else LA(0, 1); }
    else { if (relu) LA(1, 2); else LA(0, 2); }
#undef LA
    IMK_CHECK_LAUNCH();
    return 0;
}
