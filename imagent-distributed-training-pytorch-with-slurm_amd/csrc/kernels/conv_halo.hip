// Halo-tiled 3x3 convolution for 64 -> 64 channels, stride 1, pad 1 (gfx950).
//
// The ResNet stage-1 3x3 convs (R50 64@56, R18 64@112; forward and their
// stride-1 dgrads) were the slowest GEMMs of the step on the generic implicit-
// GEMM tiles (~390 TFLOP/s, profiles/conv_shape_kernels.md): with K = 9 x 64
// and only 64 output channels, every 64-deep K-stage re-gathers the tile's
// pixel rows into LDS (9x per input pixel) and the LDS writes, not the MFMAs,
// set the pace. Here a persistent block keeps
//   * ALL 9 taps of the weights resident in LDS (9 x 64 x 128 B = 72 KiB,
//     loaded once per block), and
//   * one input PATCH per band of R output rows: (R + 2) x (W + 2) pixels x
//     64 channels (the band plus its 1-pixel halo), written to LDS once and
//     read by all 9 taps as shifted windows,
// so an input pixel crosses into LDS once instead of nine times. The next
// band's patch is prefetched into registers while the current band computes.
//
// LDS images: 128-B rows (one pixel's / one output channel's 64 bf16), 16-B
// chunk c stored at chunk c ^ (row & 7) -- the rows a ds_read_b128 lane group
// touches (8 consecutive pixels of one chunk + 8 of the next, or 16 channel
// rows) land on distinct bank slots. The patch pitch PW is a multiple of 8
// pixels so a 16-pixel MFMA group that wraps to the next output row keeps
// that property.
//
// Band = R x W = 224 output pixels = 14 groups of 16; wave w < 7 computes
// groups 2w, 2w+1 for all 64 channels (v_mfma_f32_16x16x32_bf16, acc[4][2]),
// wave 7 only loads. Epilogue: the accumulators go to an LDS staging tile as
// bf16; the band's 224 output pixels are contiguous in NHWC, so every thread
// then streams whole 16-B chunks (store, IG_ACCUM read-back, fused BN-backward
// reads of x / y / x2) with a fixed 8-channel slice, and keeps its statistics
// (forward: shifted sum / sum of squares; BN backward: sum g*xhat, sum g,
// sum g*x2hat) in registers across all its bands: one LDS fold and one atomic
// per channel per block at the end (the direct register epilogue measured
// 285 of 544 us at R50 64@56, batch 1024).

#include "conv_igemm_impl.h"

namespace {

constexpr int HALO_WB = 9 * 64 * 128;  // weight image bytes

// patch pitch (pixels): 16-pixel MFMA groups that wrap to the next output row
// (W % 16 != 0) need a pitch that is a multiple of 8 to keep the swizzle
// conflict-free across the wrap; otherwise W + 2 (less LDS)
constexpr int halo_pw(int W) { return (W % 16 == 0) ? W + 2 : ((W + 2 + 7) / 8) * 8; }
constexpr int HALO_SP = 136;  // staged-epilogue row pitch, bytes (34 dwords: conflict-free 8-B writes)
constexpr size_t halo_lds(int W, int R) {
    return (size_t)HALO_WB + (size_t)(R + 2) * halo_pw(W) * 128 + (size_t)R * W * HALO_SP;
}

__device__ __forceinline__ void unpack8(const u32x4 w, float (&v)[8]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[2 * k] = lo_bf(w[k]);
        v[2 * k + 1] = hi_bf(w[k]);
    }
}

template <int W, int R, int EPI>  // EPI 0: forward (+ shifted BN statistics), 1: fused BN backward, 2: + second BN branch
__global__ __launch_bounds__(512, 1) void halo3x3_kernel(const IGemmArgs a, int nbands) {
    constexpr int PW = halo_pw(W);
    constexpr int PCOLS = W + 2, PROWS = R + 2;
    constexpr int NCH = PROWS * PCOLS * 8;     // 16-B chunks per patch
    constexpr int PMAX = (NCH + 511) / 512;    // per thread
    constexpr int BP = R * W;                  // band pixels
    static_assert(BP == 224, "band = 14 groups of 16 pixels");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sW = smem;                                  // [9][64][128 B] weights
    char* sP = smem + HALO_WB;                        // [PROWS][PW][128 B] input patch
    char* sE = sP + PROWS * PW * 128;                 // [BP][HALO_SP] staged bf16 output

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int G = gridDim.x;
    const int lid = xcd_remap(blockIdx.x, G);
    const int b0 = (int)((long)nbands * lid / G), b1 = (int)((long)nbands * (lid + 1) / G);
    if (b0 >= b1) return;  // whole block
    const int bands_per_img = a.H / R;

    // ---- weights: all 9 taps, [t][n][128 B] swizzled
    for (int id = tid; id < 9 * 64 * 8; id += 512) {
        const int c = id & 7, n = (id >> 3) & 63, t = id >> 9;
        const int ti = t / 3, tj = t - ti * 3;
        const int wtap = (a.kh0 + ti * a.khs) * a.KW + (a.kw0 + tj * a.kws);
        const u32x4 v = *reinterpret_cast<const u32x4*>(a.Wk + (size_t)n * a.ldb + wtap * 64 + c * 8);
        *reinterpret_cast<u32x4*>(sW + (t * 64 + n) * 128 + ((c ^ (n & 7)) << 4)) = v;
    }

    // a.xbn (forward): the patch is relu(x * scale + shift) per channel -- the producing BatchNorm's
    // apply + ReLU done while staging (ops/block.py); out-of-image pixels stay 0. A thread's chunks all
    // hold channels (tid & 7) * 8 .. + 7, so its 16 constants live in registers
    const bool xbn = EPI == 0 && a.xbn != nullptr;
    float xsc[8], xsh[8];
    if (xbn) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            xsc[k] = a.xbn[(tid & 7) * 8 + k];
            xsh[k] = a.xbn[64 + (tid & 7) * 8 + k];
        }
    }
    u32x4 pr[PMAX];
    bool pv[PMAX];  // chunk inside the image (xbn: transformed at staging)
    auto load_patch = [&](int band) {  // branch-free: out-of-image chunks are out-of-range buffer offsets (zeros)
        const int img = band / bands_per_img, y0 = (band - img * bands_per_img) * R;
        const __amdgpu_buffer_rsrc_t rxi = buf_rsrc(a.X + (size_t)img * a.H * W * 64);
#pragma unroll
        for (int i = 0; i < PMAX; ++i) {
            const int id = tid + i * 512;
            const int c = id & 7, pix = id >> 3;
            const int prow = pix / PCOLS, pcol = pix - prow * PCOLS;
            const int iy = y0 - 1 + prow, ix = pcol - 1;
            pv[i] = id < NCH && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)W;
            pr[i] = buf_ld16(rxi, pv[i] ? (uint32_t)(((iy * W + ix) * 64 + c * 8) * 2) : BUF_OOB);
        }
    };
    auto store_patch = [&]() {
#pragma unroll
        for (int i = 0; i < PMAX; ++i) {
            const int id = tid + i * 512;
            if (id < NCH) {
                const int c = id & 7, pix = id >> 3;
                const int prow = pix / PCOLS, pcol = pix - prow * PCOLS;
                const int q = prow * PW + pcol;
                u32x4 v = pr[i];
                if (xbn && pv[i]) {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        v[k] = pack_bf2(fmaxf(fmaf(lo_bf(v[k]), xsc[2 * k], xsh[2 * k]), 0.f),
                                        fmaxf(fmaf(hi_bf(v[k]), xsc[2 * k + 1], xsh[2 * k + 1]), 0.f));
                }
                *reinterpret_cast<u32x4*>(sP + q * 128 + ((c ^ (q & 7)) << 4)) = v;
            }
        }
    };

    const int fr = lane & 15, kq = lane >> 4;
    const bool active = wid < 7;
    // patch pixel of this lane's output pixel in groups 2w, 2w+1 (tap offset 0)
    int q0[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int p = (2 * wid + j) * 16 + fr;
        const int r = p / W, x = p - r * W;
        q0[j] = (r + 1) * PW + (x + 1);
    }

    // ---- staged epilogue, per wave: the wave's own 32 pixels (groups 2w, 2w+1), lane = fixed
    // 8-channel chunk ec of pixels 32 w + ep0 + 8 k -- no block barrier between a wave's MFMAs
    // and its epilogue, so one wave's stores overlap the other waves' MFMAs
    const int ec = lane & 7, ep0 = 32 * wid + (lane >> 3);
    const bool want_st = a.stats != nullptr;
    const bool accum = a.flags & IG_ACCUM;
    const bool affine = a.flags & IG_AFFINE, relu = a.flags & IG_RELU;  // eval forward (EPI 0 only)
    const bool has_y = EPI >= 1 && a.bnym != nullptr;
    constexpr bool has_x2 = EPI == 2;
    float c0[8], c1[8], c2[8], c3[8];  // per-channel constants (see below)
    float s1[8], s2[8], s3[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int n = ec * 8 + k;
        s1[k] = s2[k] = s3[k] = 0.f;
        if (EPI == 0) {  // c0 = shift; c2 / c3 = the folded inference BatchNorm (IG_AFFINE: a.bias = [scale | shift])
            c0[k] = (want_st && a.shift) ? a.shift[n] : 0.f;
            c1[k] = 0.f;
            c2[k] = affine ? a.bias[n] : 1.f;
            c3[k] = affine ? a.bias[a.Nout + n] : 0.f;
        } else {  // c0 = mean, c1 = rstd, c2/c3 = mask affine (from x) or second branch mean / rstd
            c0[k] = a.bnsave[n];
            c1[k] = a.bnsave[a.Nout + n];
            if (has_x2) {
                c2[k] = a.bnsave2[n];
                c3[k] = a.bnsave2[a.Nout + n];
            } else if (!has_y) {
                const float sc = a.bngamma[n] * c1[k];
                c2[k] = sc;
                c3[k] = a.bnbeta[n] - c0[k] * sc;
            } else {
                c2[k] = c3[k] = 0.f;
            }
        }
    }

    load_patch(b0);
    for (int b = b0; b < b1; ++b) {
        __syncthreads();  // previous patch / staging reads done (and the weights are in)
        store_patch();
        __syncthreads();
        // the epilogue's global operands of THIS band go out before the next band's patch loads: vmcnt retires
        // in issue order, so the epilogue's wait for them leaves the patch prefetch in flight
        const int img = b / bands_per_img, y0 = (b - img * bands_per_img) * R;
        const size_t m0 = (size_t)(img * a.H + y0) * W;
        const __amdgpu_buffer_rsrc_t ry = buf_rsrc(reinterpret_cast<const bf16_t*>(a.Y) + m0 * 64);
        // (x and the mask bits of the BN-backward epilogue at W = 56; the rarer accumulated output, the second
        // branch's x (EPI 2) and the 112-wide band read in the epilogue itself: up front they spill at 256 VGPRs)
        constexpr bool PRE = EPI == 1 && W == 56;
        u32x4 xw[4];
        uint32_t yw[4];
        const __amdgpu_buffer_rsrc_t rx2 = buf_rsrc(a.bnx2 + m0 * 64, has_x2);
        const __amdgpu_buffer_rsrc_t rbx = buf_rsrc(a.bnx + m0 * 64, EPI >= 1);
        const __amdgpu_buffer_rsrc_t rym = buf_rsrc(a.bnym + m0 * 8, has_y);
        if (PRE && active) {
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
                const uint32_t off = (uint32_t)(((ep0 + 8 * k4) * 64 + ec * 8) * 2);
                xw[k4] = buf_ld16(rbx, off);
                yw[k4] = has_y ? __builtin_amdgcn_raw_buffer_load_b8(rym, off >> 4, 0, 0) : 0u;
            }
        }
        load_patch(b + 1 < b1 ? b + 1 : b);  // in flight while this band computes (the last band re-reads itself)
        if (active) {
            f32x4 acc[4][2];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int ti = t / 3, tj = t - ti * 3;
                const int dq = (a.dh0 + ti * a.dhs) * PW + (a.dw0 + tj * a.dws);
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const int c = kq + 4 * ks;
                    bf16x8 fw[4], fx[2];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        fw[i] = *reinterpret_cast<const bf16x8*>(sW + (t * 64 + i * 16 + fr) * 128 +
                                                                 ((c ^ (fr & 7)) << 4));
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int q = q0[j] + dq;
                        fx[j] = *reinterpret_cast<const bf16x8*>(sP + q * 128 + ((c ^ (q & 7)) << 4));
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[i], fx[j], acc[i][j], 0, 0, 0);
                }
            }
            __builtin_amdgcn_s_setprio(0);
            // lane holds channels kq*4 + i*16 + r of pixel (2w + j)*16 + fr -> bf16 into the wave's rows
            // of the staging tile (written and read back by this wave only: LDS order, no barrier)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int p = (2 * wid + j) * 16 + fr;
                    *reinterpret_cast<u32x2*>(sE + p * HALO_SP + (kq * 4 + i * 16) * 2) =
                        u32x2{pack_bf2(acc[i][j][0], acc[i][j][1]), pack_bf2(acc[i][j][2], acc[i][j][3])};
                }
        }
        if (!active) continue;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // coalesced epilogue: the band's output pixels are contiguous in NHWC
        constexpr int EU = PRE ? 4 : 1;  // register arrays need the unrolled loop; the late-load form stays rolled
#pragma unroll EU
        for (int k4 = 0; k4 < 4; ++k4) {
            const int p = ep0 + 8 * k4;
            const uint32_t off = (uint32_t)((p * 64 + ec * 8) * 2);
            float v[8];
            unpack8(*reinterpret_cast<const u32x4*>(sE + p * HALO_SP + ec * 16), v);
            if (EPI == 0 && affine) {
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = fmaf(v[q], c2[q], c3[q]);
            }
            if (accum) {
                float o[8];
                unpack8(buf_ld16(ry, off), o);
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] += o[q];
            }
            if (EPI >= 1) {
                u32x4 xk;
                uint32_t yk;
                if constexpr (PRE) {
                    xk = xw[k4];
                    yk = yw[k4];
                } else {
                    xk = buf_ld16(rbx, off);
                    yk = has_y ? __builtin_amdgcn_raw_buffer_load_b8(rym, off >> 4, 0, 0) : 0u;
                }
                float xv[8], mk[8];
                unpack8(xk, xv);
                if (has_y) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) mk[q] = (yk >> q) & 1u ? 1.f : 0.f;
                } else {
#pragma unroll
                    for (int q = 0; q < 8; ++q) mk[q] = fmaf(xv[q], c2[q], c3[q]);
                }
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (!(mk[q] > 0.f)) v[q] = 0.f;
                u32x4 out;
#pragma unroll
                for (int q = 0; q < 4; ++q) out[q] = pack_bf2(v[2 * q], v[2 * q + 1]);
                buf_st16(ry, off, out);
                unpack8(out, v);
                float x2v[8];
                if (has_x2) unpack8(buf_ld16(rx2, off), x2v);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    s1[q] += v[q] * ((xv[q] - c0[q]) * c1[q]);  // sum g * xhat
                    s2[q] += v[q];                            // sum g
                    if (has_x2) s3[q] += v[q] * ((x2v[q] - c2[q]) * c3[q]);
                }
            } else {
                if (relu) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
                }
                u32x4 out;
#pragma unroll
                for (int q = 0; q < 4; ++q) out[q] = pack_bf2(v[2 * q], v[2 * q + 1]);
                buf_st16(ry, off, out);
                if (want_st) {
                    unpack8(out, v);
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float d = v[q] - c0[q];
                        s1[q] += d;
                        s2[q] += d * d;
                    }
                }
            }
        }
    }
    if (!want_st) return;
    // ---- statistics: fold the 64 threads of each channel chunk in LDS, one atomic per
    // channel and quantity for the whole persistent block
    __syncthreads();
    float* red = reinterpret_cast<float*>(sP);  // [3][512][8] floats (48 KiB: patch + staging area)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        red[(0 * 512 + tid) * 8 + q] = s1[q];
        red[(1 * 512 + tid) * 8 + q] = s2[q];
        if (has_x2) red[(2 * 512 + tid) * 8 + q] = s3[q];
    }
    __syncthreads();
    const int nq = has_x2 ? 3 : 2;
    if (tid < 64 * nq) {
        const int qq = tid >> 6, n = tid & 63, c = n >> 3, k = n & 7;
        float sum = 0.f;
        for (int u = c; u < 512; u += 8) sum += red[(qq * 512 + u) * 8 + k];
        float* st = a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * (EPI >= 1 ? 3 : 2) * a.Nout;
        atomicAdd(st + qq * a.Nout + n, sum);
    }
}

int halo_cus() {
    static const int n = [] {
        int dev = 0, cus = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
        return cus;
    }();
    return n;
}

// blocks per CU: one persistent block per CU (2 measured within noise, round-4 switch sweep)
constexpr int HALO_BLOCKS_PER_CU = 1;

template <int W, int R, int EPI>
int launch_halo(const IGemmArgs& a, hipStream_t st) {
    const size_t lds = halo_lds(W, R);
    const int nbands = a.N * (a.H / R);
    const int G = std::min(nbands, halo_cus() * HALO_BLOCKS_PER_CU);
    hipLaunchKernelGGL((halo3x3_kernel<W, R, EPI>), dim3(G), dim3(512), lds, st, a, nbands);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

bool tap_in_halo(int d0, int ds) { return d0 >= -1 && d0 <= 1 && d0 + 2 * ds >= -1 && d0 + 2 * ds <= 1; }

}  // namespace

// Returns 1 when the shape / flags are not the halo kernel's (caller falls back).
int conv_halo(const IGemmArgs& a, hipStream_t st) {
    if (a.flags & (IG_OUT_F32 | IG_STEM | IG_REGSTAGE | IG_FP8 | IG_ACCUM_SUB2)) return 1;
    // the eval forward's folded BatchNorm (+ ReLU after the optional accumulate): plain epilogue only
    if ((a.flags & (IG_AFFINE | IG_RELU)) && ((a.flags & IG_BNBWD) || a.stats || a.xbn)) return 1;
    if ((a.flags & IG_RELU) && !(a.flags & IG_AFFINE)) return 1;
    if ((a.bias && !(a.flags & IG_AFFINE)) || a.C != 64 || a.Nout != 64 || a.ldb < 9 * 64 || a.ldy != 64) return 1;
    if (a.nth != 3 || a.ntw != 3 || a.KW != 3 || a.sA != 1 || a.sY != 1 || a.oy != 0 || a.ox != 0) return 1;
    if (a.OH != a.H || a.OW != a.W || a.YH != a.H || a.YW != a.W) return 1;
    if (!tap_in_halo(a.dh0, a.dhs) || !tap_in_halo(a.dw0, a.dws)) return 1;
    if (a.kh0 + 2 * a.khs < 0 || a.kh0 + 2 * a.khs > 2 || a.kh0 < 0 || a.kh0 > 2) return 1;
    if (a.kw0 + 2 * a.kws < 0 || a.kw0 + 2 * a.kws > 2 || a.kw0 < 0 || a.kw0 > 2) return 1;
    const bool bnb = a.flags & IG_BNBWD;
    if (bnb && a.bnx2 && !a.bnym) return 1;  // a second BN branch needs the output's mask bits (c2/c3 hold its constants)
    if (a.W == 56 && a.H % 4 == 0)
        return bnb ? (a.bnx2 ? launch_halo<56, 4, 2>(a, st) : launch_halo<56, 4, 1>(a, st)) : launch_halo<56, 4, 0>(a, st);
    if (a.W == 112 && a.H % 2 == 0)
        return bnb ? (a.bnx2 ? launch_halo<112, 2, 2>(a, st) : launch_halo<112, 2, 1>(a, st))
                   : launch_halo<112, 2, 0>(a, st);
    return 1;
}
