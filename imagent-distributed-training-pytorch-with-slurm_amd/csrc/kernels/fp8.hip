// fp8 (OCP e4m3) quantisation for the fp8 forward path, gfx950.
//
// SURVEY §7.2 step 6 / BASELINE config "ResNet-50 fp8 (CDNA4 fp8 MFMA conv)":
// the forward convolutions read e4m3 activations and weights through the
// block-scaled MFMA (conv_igemm.hip, IG_FP8). Scales are per tensor and powers
// of two, q = x * 2^-e, so they ride in the MFMA's E8M0 scale operands
// (127 + e) and dequantisation costs nothing.
//  * weights: exact per-step scaling -- one amax pass and one quantise pass
//    over a descriptor table of all conv weights (fp32 masters -> e4m3);
//  * activations: delayed scaling (as in FP8 training recipes): a tensor is
//    quantised with the exponent derived from the previous step's amax, the
//    current amax is recorded for the next step (imk_fp8_update_exp).
// Values beyond the e4m3 range saturate to +-448.

#include "common.h"

namespace {

constexpr int AMAX_SLOTS = 32;  // per-tensor amax slots (atomic max spread by block id)

// exponent e with amax * 2^-e <= 448 (>= 2^-margin headroom), clamped
__device__ __forceinline__ int exp_for(float amax, int margin) {
    if (!(amax > 0.f)) return 0;
    int e = (int)ceilf(log2f(amax / E4M3_MAX)) + margin;
    return max(-60, min(60, e));
}

// bf16 activations -> e4m3 with the stored exponent; |x| max -> amax
__global__ __launch_bounds__(256) void quant_act_kernel(const bf16_t* __restrict__ x, uint32_t* __restrict__ y,
                                                        long n8, const int* __restrict__ exp_in,
                                                        float* __restrict__ amax) {
    const float s = ldexpf(1.f, -exp_in[0]);
    float m = 0.f;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
        const u32x4 w = reinterpret_cast<const u32x4*>(x)[i];
        float v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[2 * k] = lo_bf(w[k]);
            v[2 * k + 1] = hi_bf(w[k]);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(v[k]));
        u32x2 o;
        o[0] = pack4_fp8(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
        o[1] = pack4_fp8(v[4] * s, v[5] * s, v[6] * s, v[7] * s);
        reinterpret_cast<u32x2*>(y)[i] = o;
    }
    __shared__ float wm[4];
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0 && amax)
        atomic_max_pos(amax + (blockIdx.x & (AMAX_SLOTS - 1)), fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3])));
}

// one wave per tensor: fold its AMAX_SLOTS slots, exponent for the next step, clear
__global__ void update_exp_kernel(float* __restrict__ amax, int* __restrict__ e, int n, int margin) {
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (t >= n) return;
    float* row = amax + (size_t)t * AMAX_SLOTS;
    float a = lane < AMAX_SLOTS ? row[lane] : 0.f;
    a = wave_max(a);
    if (lane < AMAX_SLOTS) row[lane] = 0.f;
    if (lane == 0 && a > 0.f) e[t] = exp_for(a, margin);  // no observation: keep the exponent
}

struct QDesc {
    const float* src;  // fp32 master weights (any contiguous layout)
    uint32_t* dst;     // e4m3 bytes, same layout
    long n4;           // elements / 4
    int* exp;          // per-tensor exponent (written)
    float* amax;       // per-tensor scratch (zeroed by the caller)
    uint8_t* dstT;     // optional e4m3 copy of a conv weight [Co][T][Ci] transposed to [Ci][T][Co] (dgrad)
    int T, Ci;
};

// pass 1: per-tensor amax (blockIdx.y = tensor)
__global__ __launch_bounds__(256) void weight_amax_kernel(const QDesc* __restrict__ d) {
    const QDesc q = d[blockIdx.y];
    float m = 0.f;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < q.n4; i += (long)gridDim.x * 256) {
        const f32x4 v = reinterpret_cast<const f32x4*>(q.src)[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) atomic_max_pos(q.amax, m);
}

// pass 2: exponent from this step's amax, quantise
__global__ __launch_bounds__(256) void weight_quant_kernel(const QDesc* __restrict__ d, int margin) {
    const QDesc q = d[blockIdx.y];
    const int e = exp_for(q.amax[0], margin);
    if (blockIdx.x == 0 && threadIdx.x == 0) q.exp[0] = e;
    const float s = ldexpf(1.f, -e);
    const long tc = (long)q.T * q.Ci;
    const long Co = q.dstT ? q.n4 * 4 / tc : 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < q.n4; i += (long)gridDim.x * 256) {
        const f32x4 v = reinterpret_cast<const f32x4*>(q.src)[i];
        const uint32_t w = pack4_fp8(v[0] * s, v[1] * s, v[2] * s, v[3] * s);
        q.dst[i] = w;
        if (q.dstT) {  // element e = 4i + j of [Co][T][Ci] -> [Ci][T][Co]
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const long e = 4 * i + j;
                const long co = e / tc, rem = e - co * tc;
                const long t = rem / q.Ci, ci = rem - t * q.Ci;
                q.dstT[(ci * q.T + t) * Co + co] = (uint8_t)(w >> (8 * j));
            }
        }
    }
}

}  // namespace

// x: bf16 [n] (n % 8 == 0, 16-B aligned) -> y: e4m3 [n]; exp_in: device int;
// amax (device float[32] slots, may be null) receives max |x|
IMK_EXPORT int imk_quant_fp8(const void* x, void* y, long n, const int* exp_in, float* amax, void* stream) {
    if (n % 8) return -100;
    const long n8 = n / 8;
    long blocks = (n8 + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) return 0;
    hipLaunchKernelGGL(quant_act_kernel, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                       (uint32_t*)y, n8, exp_in, amax);
    IMK_CHECK_LAUNCH();
    return 0;
}

// e[i] = exponent for max(amax[i][0..31]) (delayed scaling, next step); amax rows cleared
IMK_EXPORT int imk_fp8_update_exp(float* amax, int* e, int n, int margin, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(update_exp_kernel, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, amax, e, n,
                       margin);
    IMK_CHECK_LAUNCH();
    return 0;
}

// all weights of a step: descs = device array of n QDesc, amax scratch zeroed by the caller
IMK_EXPORT int imk_quant_fp8_weights(const void* descs, int n, long max_n4, int margin, void* stream) {
    if (n <= 0) return 0;
    long bx = (max_n4 + 255) / 256;
    if (bx > 64) bx = 64;
    if (bx < 1) bx = 1;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(weight_amax_kernel, dim3((int)bx, n), dim3(256), 0, st, (const QDesc*)descs);
    IMK_CHECK_LAUNCH();
    hipLaunchKernelGGL(weight_quant_kernel, dim3((int)bx, n), dim3(256), 0, st, (const QDesc*)descs, margin);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_qdesc_size() { return (int)sizeof(QDesc); }
