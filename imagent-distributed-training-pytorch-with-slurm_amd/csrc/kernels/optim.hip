// LARS (layer-wise adaptive rate scaling, You et al. 2017) over the flat
// parameter arena, for the large-batch configuration (BASELINE.json: global
// batch 8192). Two launches per step over a per-tensor descriptor table:
//   1. per-tensor ||w||^2 and ||g||^2 (block reduce, one atomic per block)
//   2. the update, blockIdx.y = tensor:
//        trust = eta * ||w|| / (||g|| + wd * ||w||)   (adapted tensors; 1 else)
//        d = g + wd * w ;  v = mu * v + lr * trust * d ;  w -= v
//      plus the bf16 compute shadow, like the fused SGD kernel (misc.hip).
// BatchNorm weights/biases and the fc bias are conventionally neither decayed
// nor adapted (`adapt` = 0 in their descriptors).

#include "common.h"

struct LarsDesc {
    float* p;
    const float* g;
    float* buf;
    bf16_t* shadow;  // may be null
    long n;
    int adapt;       // 1: LARS trust ratio + weight decay; 0: plain momentum SGD, no decay
    int pad;
};

namespace {

__global__ __launch_bounds__(256) void lars_norms_kernel(const LarsDesc* __restrict__ d, float* __restrict__ norms,
                                                         int T, float gs) {
    const LarsDesc q = d[blockIdx.y];
    float sw = 0.f, sg = 0.f;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < q.n; i += (long)gridDim.x * 256) {
        const float w = q.p[i], g = q.g[i] * gs;
        sw += w * w;
        sg += g * g;
    }
    __shared__ float red[2][4];
    sw = wave_sum(sw);
    sg = wave_sum(sg);
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = sw;
        red[1][threadIdx.x >> 6] = sg;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(norms + blockIdx.y, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
        atomicAdd(norms + T + blockIdx.y, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
    }
}

__global__ __launch_bounds__(256) void lars_update_kernel(const LarsDesc* __restrict__ d,
                                                          const float* __restrict__ norms, int T, float lr,
                                                          float mu, float wd, float eta, float gs, int first) {
    const LarsDesc q = d[blockIdx.y];
    float trust = 1.f, wdt = 0.f;
    if (q.adapt) {
        wdt = wd;
        const float wn = sqrtf(norms[blockIdx.y]), gn = sqrtf(norms[T + blockIdx.y]);
        if (wn > 0.f && gn > 0.f) trust = eta * wn / (gn + wd * wn);
    }
    const float step = lr * trust;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < q.n; i += (long)gridDim.x * 256) {
        const float w = q.p[i];
        const float dd = q.g[i] * gs + wdt * w;
        const float v = first ? step * dd : mu * q.buf[i] + step * dd;
        q.buf[i] = v;
        const float nw = w - v;
        q.p[i] = nw;
        if (q.shadow) q.shadow[i] = f2bf(nw);
    }
}

}  // namespace

// descs: device array of T LarsDesc; norms: device float[2*T] scratch (zeroed here)
IMK_EXPORT int imk_lars_step(const void* descs, int T, long max_n, float* norms, float lr, float mu, float wd,
                             float eta, float gs, int first, void* stream) {
    if (T <= 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(norms, 0, sizeof(float) * 2 * T, st) != hipSuccess) return -1;
    long bx = (max_n + 1023) / 1024;
    if (bx > 64) bx = 64;
    if (bx < 1) bx = 1;
    hipLaunchKernelGGL(lars_norms_kernel, dim3((int)bx, T), dim3(256), 0, st, (const LarsDesc*)descs, norms, T, gs);
    IMK_CHECK_LAUNCH();
    hipLaunchKernelGGL(lars_update_kernel, dim3((int)bx, T), dim3(256), 0, st, (const LarsDesc*)descs,
                       (const float*)norms, T, lr, mu, wd, eta, gs, first);
    IMK_CHECK_LAUNCH();
    return 0;
}

IMK_EXPORT int imk_lars_desc_size() { return (int)sizeof(LarsDesc); }
