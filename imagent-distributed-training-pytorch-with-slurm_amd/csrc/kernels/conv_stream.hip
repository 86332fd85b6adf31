// Streaming 1x1 convolution for SHORT reductions (K = C in {64, 128, 256}), gfx950.
//
// ResNet bottlenecks spend their 56x56 / 28x28 stages in 1x1 convolutions with
// K = 64 or 128: the expansion conv3 (64 -> 256, 128 -> 512) forward, and the
// dgrad of conv1 (256 -> 64, 512 -> 128: dX[M][256] = dY[M][64] x W) with the
// BN-backward epilogue. These are pure HBM streams (output bytes = 4x input
// bytes) -- the generic tiled kernels (conv_igemm_impl.h) reload the weight
// tile per output tile, keep one 16-KB stage in flight per block and measured
// 2.1 TB/s on them (profiles/r50_b512_v5_*). Same jobs as cuDNN's conv fwd /
// dgrad for those shapes (reference model imagenet.py:312).
//
// Structure (one persistent block = 4 waves per (pixel range, channel slice)):
//  * the block's weight slice [BN][K] lives in LDS for the whole kernel
//    (16-B chunks XOR-swizzled by row -> conflict-free ds_read_b128 A
//    fragments);
//  * each wave walks 16-pixel groups; the pixel operand is the MFMA B
//    fragment, and in NHWC one lane's B fragment (8 consecutive channels of
//    one pixel) is ONE 16-B global load -- no LDS staging at all. D groups
//    are prefetched into registers ahead of use (bytes in flight per CU ~
//    8 waves x D x 2-4 KB);
//  * every global access of the group loop is a raw BUFFER load / store off a wave-uniform base (the group's
//    first row) with per-lane 32-bit offsets; rows past M and groups past the end are out-of-range offsets
//    (loads read zeros, stores are dropped), so the loop has no divergent memory branch. With the former
//    predicated pointer loads the compiler's waitcnt bookkeeping fell back to s_waitcnt vmcnt(0) around them
//    (277 of them in the fused-output kernel), draining the prefetch in every group's epilogue; now the
//    epilogue's own operands (BN-backward x / mask, residual) are issued before the next prefetch and waited
//    for with a counted vmcnt (round 5: <64,256> fused output 870 -> 742 us, <128,128> 508 -> 380 us in-step);
//  * the weight fragments go through a register ring read several MFMAs ahead (sched_group_barrier pins the
//    interleave; left alone the scheduler issued each ds_read right before its MFMA and waited for it);
//  * v_mfma_f32_16x16x32_bf16, weights = A (rows = output channels);
//  * epilogue per group: the 16 x BN bf16 tile goes through a wave-private LDS
//    buffer and comes back as 16-B row chunks, so every global store / read of
//    the epilogue is a coalesced row segment, and each lane always holds the
//    SAME 8 channels -> BatchNorm statistics (forward: sum, sumsq; IG_BNBWD:
//    sum(g*xhat), sum(g) [, sum(g*xhat2)]) accumulate in 16-24 registers over
//    the whole kernel and leave with one lane fold + one atomic per channel
//    and quantity per wave.
// Semantics are those of igemm's plain / IG_ACCUM / IG_BNBWD epilogues.

#include <cstdlib>

#include "conv_igemm_impl.h"

namespace {

// MODE 0: plain epilogue (+ optional IG_ACCUM); IG_BNBWD with the ReLU mask
// from the saved output y (1), recomputed from x (2), y + second BN branch x2 (3); 4: the plain epilogue with
// a training block's fused output (IG_RES residual (+ scale), IG_MASKOUT mask bits, IG_Q8OUT e4m3 copy) -- a
// mode of its own so that the registers of those paths never weigh on the plain kernels (eval, forward convs)
// STEM: the 7x7/2 stem as a row-segment gather (C = 4 padded channels, a
// kernel row = 8 taps x 4 channels = 32 K elements, K = KH x 32): one MFMA
// k-step per kernel row, the lane's B fragment = 2 taps x 4 channels = two
// 8-B loads (each predicated on the image border).
// XBN: the pixel operand is relu(x * scale[c] + shift[c]) (a.xbn [2][C]), applied to each B fragment
// in registers right before its MFMAs (8 channels per lane per k-step: 2 KS x 8 constants per lane)
// K2: a second K segment of K2 channels from X2 (same pixels, row pitch K2; the weights' columns [K, K + K2)),
// with IG_BNBWD the Gram-form conv3 dgrad over [g | h2] (bn_gram.hip): `bias` [Nout] is added to the sums
// before the ReLU mask (as the v3 loop's two-segment form)
template <bool STEM, int KT>
constexpr int stream_rp() {  // LDS weight row pitch in 16-B chunks: 16-chunk swizzle groups stay inside the row
    return STEM ? 32 : (KT / 8 <= 16 ? KT / 8 : (KT / 8 + 15) / 16 * 16);
}

template <int K, int BN, int D, int MODE, bool STEM = false, bool XBN = false, int K2 = 0>
__global__ __launch_bounds__(256, 2) void conv_stream_kernel(const IGemmArgs a) {
    constexpr int KS1 = K / 32;       // k-steps from X
    constexpr int KS = (K + K2) / 32; // MFMA k-steps per group
    constexpr int FN = BN / 16;       // channel fragments
    constexpr int CPR = (K + K2) / 8; // 16-B chunks per weight row
    constexpr int RP = stream_rp<STEM, K + K2>();   // LDS weight row pitch, chunks
    constexpr int RB = RP * 16;                     // ... bytes
    constexpr int SWM = (RP < 16 ? RP : 16) - 1;    // chunk swizzle mask: conflict-free A reads
    constexpr int EP = BN * 2;        // epilogue LDS row pitch (bytes), rows swizzled as the staged epilogue (epi_swz)
    constexpr int CH = BN / 8;        // 16-B output chunks per pixel
    constexpr int PPR = 64 / CH;      // pixels per epilogue read instruction
    constexpr int NR = 16 / PPR;      // epilogue reads per 16-pixel group
    constexpr bool bnb = MODE >= 1 && MODE <= 3, has_y = MODE == 1 || MODE == 3, has_x2 = MODE == 3;
    constexpr bool FO = MODE == 4;
    // chunks whose global reads are batched; with the BN-backward epilogue all
    // of a group's reads (x, y | x2, old) are issued before its MFMAs
    constexpr int QB = bnb ? NR : (NR < 4 ? NR : 4);
    static_assert(!bnb || NR <= 4, "BN-backward epilogue: slices of <= 128 channels");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    char* sW = smem;
    char* sE = smem + BN * RB + wid * 16 * EP;

    const int nsl = a.Nout / BN;
    const int G = gridDim.x;  // multiple of nsl (host)
    const int lid = xcd_remap(blockIdx.x, G);
    const int slice = lid % nsl, pb = lid / nsl, npb = G / nsl;
    const int n0 = slice * BN;
    const bool accum = a.flags & IG_ACCUM;

    // weight slice -> LDS: chunk c of row r at slot c ^ (r & SWM)
    for (int idx = tid; idx < BN * CPR; idx += 256) {
        const int r = idx / CPR, c = idx % CPR;
        const u32x4 v = *reinterpret_cast<const u32x4*>(a.Wk + (size_t)(n0 + r) * a.ldb + c * 8);
        *reinterpret_cast<u32x4*>(sW + r * RB + ((c ^ (r & SWM)) * 16)) = v;
    }

    // fixed epilogue channel chunk of this lane + the BN constants it needs
    const int cc = lane % CH;
    const int n = n0 + cc * 8;
    float mean[8], rstd[8], sc[8], sh[8], m2[8], r2[8];
    if (bnb) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const f32x4 mu = *reinterpret_cast<const f32x4*>(a.bnsave + n + 4 * h);
            const f32x4 rs = *reinterpret_cast<const f32x4*>(a.bnsave + a.Nout + n + 4 * h);
            f32x4 g = {0.f, 0.f, 0.f, 0.f}, b = g, mu2 = g, rs2 = g;
            if (!has_y) {
                g = *reinterpret_cast<const f32x4*>(a.bngamma + n + 4 * h);
                b = *reinterpret_cast<const f32x4*>(a.bnbeta + n + 4 * h);
            }
            if (has_x2) {
                mu2 = *reinterpret_cast<const f32x4*>(a.bnsave2 + n + 4 * h);
                rs2 = *reinterpret_cast<const f32x4*>(a.bnsave2 + a.Nout + n + 4 * h);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                mean[4 * h + r] = mu[r];
                rstd[4 * h + r] = rs[r];
                sc[4 * h + r] = g[r] * rs[r];
                sh[4 * h + r] = b[r] - mu[r] * sc[4 * h + r];
                m2[4 * h + r] = mu2[r];
                r2[4 * h + r] = rs2[r];
            }
        }
    }
    // plain epilogue: forward statistics (mean[] holds the shift: previous batch mean, or 0) and the eval
    // forward's folded BatchNorm (IG_AFFINE: a.bias = [scale | shift] -> sc / sh) + ReLU after the accumulate
    const bool affine = !bnb && (a.flags & IG_AFFINE), relu = !bnb && (a.flags & IG_RELU);
    // IG_RES: the residual comes from bnx (training: a Gram-form block's bn3 + shortcut + ReLU in conv3's epilogue,
    // ops/block.py), IG_MASKOUT: the ReLU mask of the stored output as bits (the next block's dgrad epilogue)
    // (bnsave2 non-null with IG_RES: a per-channel scale on the residual, a downsample block's shortcut BN whose
    // shift the caller folded into bias[Nout..])
    const bool resid = FO && (a.flags & IG_RES), maskout = FO && relu && (a.flags & IG_MASKOUT);
    const bool resaff = resid && a.bnsave2;
    // IG_Q8OUT: the e4m3 copy of the stored output (delayed-scaled, amax-tracked) for an fp8 consumer
    const bool q8out = FO && (a.flags & IG_Q8OUT);
    const float q8s = q8out ? ldexpf(1.f, -a.y8exp[0]) : 0.f;
    float m8 = 0.f;
    float rsc[8];
    if (!bnb) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            mean[c] = (a.stats && a.shift) ? a.shift[n + c] : 0.f;
            sc[c] = affine ? a.bias[n + c] : 1.f;
            sh[c] = affine ? a.bias[a.Nout + n + c] : 0.f;
            rsc[c] = resaff ? a.bnsave2[n + c] : 1.f;
        }
    }
    float s1[8], s2[8], s3[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) s1[c] = s2[c] = s3[c] = 0.f;
    float gbias[K2 > 0 ? 8 : 1];
    if constexpr (K2 > 0) {
#pragma unroll
        for (int c = 0; c < 8; ++c) gbias[c] = a.bias[n + c];
    }

    const int ohw = a.OH * a.OW;
    const bool dense = a.sA == 1 && a.H == a.OH && a.W == a.OW;  // input row == output pixel
    const int ngroups = (a.M + 15) / 16;
    const int wstride = npb * 4;
    const int w0 = pb * 4 + wid;
    const int fr = lane & 15, fq = lane >> 4;

    u32x4 pf[D][KS];
    auto fetch = [&](int d, int g) {
        const int m = g * 16 + fr;
        const bool ok = g < ngroups && m < a.M;
        if constexpr (STEM) {
            int img = 0, oh = 0, ow = 0;
            if (ok) {
                img = m / ohw;
                const int rem = m - img * ohw;
                oh = rem / a.OW;
                ow = rem - oh * a.OW;
            }
            const int kw0 = 2 * fq;
            const int iw = ow * a.sA + a.dw0 + kw0;
            const bool lo_w = ok && kw0 < a.ntw && (unsigned)iw < (unsigned)a.W;
            const bool hi_w = ok && kw0 + 1 < a.ntw && (unsigned)(iw + 1) < (unsigned)a.W;
            const bf16_t* base = a.X + (size_t)img * a.H * a.W * 4;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const int ih = oh * a.sA + a.dh0 + ks;
                const bool rok = ks < a.nth && (unsigned)ih < (unsigned)a.H;
                const bf16_t* q = base + ((long)ih * a.W + iw) * 4;
                u32x2 lo = {0u, 0u}, hi = {0u, 0u};
                if (rok && lo_w) lo = *reinterpret_cast<const u32x2*>(q);
                if (rok && hi_w) hi = *reinterpret_cast<const u32x2*>(q + 4);
                pf[d][ks] = u32x4{lo[0], lo[1], hi[0], hi[1]};
            }
            return;
        }
        // branch-free: buffer loads off a wave-uniform base (the group's first input row); rows past M and groups
        // past the end read zeros through an out-of-range offset (no divergent load, so the compiler's vmcnt
        // bookkeeping stays exact and the prefetch stays in flight, see the header)
        const bool gok = g < ngroups;
        const int m0 = gok ? g * 16 : 0;
        size_t row0 = m0;
        if (!dense) {
            const int img = m0 / ohw, rem = m0 - img * ohw;
            const int oh = rem / a.OW, ow = rem - oh * a.OW;
            row0 = ((size_t)img * a.H + oh * a.sA) * a.W + ow * a.sA;
        }
        uint32_t off = BUF_OOB;
        if (ok) {
            size_t row = (size_t)m;
            if (!dense) {
                const int img = m / ohw, rem = m - img * ohw;
                const int oh = rem / a.OW, ow = rem - oh * a.OW;
                row = ((size_t)img * a.H + oh * a.sA) * a.W + ow * a.sA;
            }
            off = (uint32_t)((row - row0) * a.C * 2) + fq * 16;
        }
        const __amdgpu_buffer_rsrc_t rx = buf_rsrc(a.X + row0 * a.C, true);
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) pf[d][ks] = buf_ld16(rx, off + ks * 64);
        if constexpr (K2 > 0) {  // (dense rows only: host check)
            const __amdgpu_buffer_rsrc_t rx2 = buf_rsrc(a.X2 + (size_t)m0 * K2, true);
            const uint32_t off2 = ok ? (uint32_t)(fr * K2 * 2 + fq * 16) : BUF_OOB;
#pragma unroll
            for (int ks = KS1; ks < KS; ++ks) pf[d][ks] = buf_ld16(rx2, off2 + (ks - KS1) * 64);
        }
    };
    // epilogue operand addressing of group g
    struct EpiBase {
        __amdgpu_buffer_rsrc_t ry, ro, rbx, rx2o, rym, ry8;
    };
    auto epi_base = [&](int g) {
        const size_t eb0 = (size_t)(g < ngroups ? g * 16 : 0) * a.ldy;
        const bf16_t* ybase = reinterpret_cast<const bf16_t*>(a.Y) + eb0;
        EpiBase e;
        e.ry = buf_rsrc(ybase, true);
        e.ro = buf_rsrc(accum ? ybase : a.bnx + eb0, accum || resid);
        e.rbx = buf_rsrc(a.bnx + eb0, bnb && a.bnx);  // bnx null (mask bits given): x is never read (zeros)
        e.rx2o = buf_rsrc(a.bnx2 + eb0, has_x2);
        e.rym = buf_rsrc(a.bnym + eb0 / 8, has_y || maskout);
        e.ry8 = buf_rsrc(reinterpret_cast<const uint8_t*>(a.Y8) + eb0, q8out);
        return e;
    };
    auto epi_off = [&](int g, int u, bool& ev, uint32_t& o2) {  // row u * PPR + lane / CH of group g, channels n..
        const int pr = u * PPR + lane / CH;
        ev = g < ngroups && g * 16 + pr < a.M;
        o2 = ev ? (uint32_t)(pr * a.ldy + n) * 2 : BUF_OOB;  // bytes from the group's base
    };
    auto oo_off = [&](int g, int u, uint32_t o2) {
        if (accum && (a.flags & IG_ACCUM_SUB2)) {  // dense output grid: only even (oh, ow) accumulate
            const int rem = (g * 16 + u * PPR + lane / CH) % ohw, oh = rem / a.OW;
            if (((oh | (rem - oh * a.OW)) & 1) != 0) return BUF_OOB;
        }
        return o2;
    };
    // EPF: the epilogue's global operands (residual / BN-backward x, mask bits, second-branch x) are prefetched D
    // groups ahead, as the pixel operand is: issued at the start of their own group they left one memory latency
    // exposed per group (<256, 64> fused output at 14x14: 3.5 us per group and wave for 32 MFMAs). Kept where
    // the registers allow (no spill at 256 VGPRs)
    constexpr bool early = bnb || FO;
    constexpr int EPR = FO ? 4 : bnb ? 4 + (has_y ? 1 : 0) + (has_x2 ? 4 : 0) : 0;  // VGPRs per row chunk
    constexpr bool EPF = early && !STEM && !XBN && D * NR * EPR <= (K >= 256 && BN >= 128 ? 16 : 32);
    u32x4 eoo[EPF ? D : 1][NR], exo[EPF ? D : 1][NR], ex2o[EPF ? D : 1][NR];
    uint32_t eyo[EPF ? D : 1][NR];
    auto issue_early = [&](int d, int g) {
        const EpiBase e = epi_base(g);
#pragma unroll
        for (int u = 0; u < NR; ++u) {
            bool ev;
            uint32_t o2;
            epi_off(g, u, ev, o2);
            eoo[d][u] = buf_ld16(e.ro, oo_off(g, u, o2));
            if (bnb) {
                exo[d][u] = buf_ld16(e.rbx, o2);
                if (has_y) eyo[d][u] = __builtin_amdgcn_raw_buffer_load_b8(e.rym, ev ? o2 >> 4 : BUF_OOB, 0, 0);
                if (has_x2) ex2o[d][u] = buf_ld16(e.rx2o, o2);
            }
        }
    };
#pragma unroll
    for (int d = 0; d < D; ++d) fetch(d, w0 + d * wstride);
    if constexpr (EPF) {
#pragma unroll
        for (int d = 0; d < D; ++d) issue_early(d, w0 + d * wstride);
    }
    __syncthreads();  // weight slice visible

    int aoff[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) aoff[ks] = fr * RB + (((ks * 4 + fq) ^ (fr & SWM)) * 16);
    float xsc[XBN ? KS : 1][8], xsh[XBN ? KS : 1][8];  // this lane's channels ks * 32 + fq * 8 + e
    if constexpr (XBN) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f32x4 sc4 = *reinterpret_cast<const f32x4*>(a.xbn + ks * 32 + fq * 8 + 4 * h);
                const f32x4 sh4 = *reinterpret_cast<const f32x4*>(a.xbn + a.C + ks * 32 + fq * 8 + 4 * h);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    xsc[ks][4 * h + r] = sc4[r];
                    xsh[ks][4 * h + r] = sh4[r];
                }
            }
    }

    for (int g0 = w0; g0 < ngroups; g0 += D * wstride) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int g = g0 + d * wstride;  // past the end: every access out of range (no divergent exit)
            bf16x8 fb[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                if constexpr (XBN) {  // BN apply + ReLU on the operand (rows past M are never stored)
                    u32x4 w = pf[d][ks];
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        w[k] = pack_bf2(fmaxf(fmaf(lo_bf(w[k]), xsc[ks][2 * k], xsh[ks][2 * k]), 0.f),
                                        fmaxf(fmaf(hi_bf(w[k]), xsc[ks][2 * k + 1], xsh[ks][2 * k + 1]), 0.f));
                    fb[ks] = __builtin_bit_cast(bf16x8, w);
                } else {
                    fb[ks] = __builtin_bit_cast(bf16x8, pf[d][ks]);
                }
            }
            // the group's epilogue operands: wave-uniform bases at the group's pixel row, per-lane byte offsets
            // (rows past M: out of range, loads read zeros and stores are dropped). Every load of the loop body is
            // unconditional, so the waits stay counted and the prefetch stays in flight
            const EpiBase eb = epi_base(g);
            bool ev[NR];
            uint32_t o2[NR];
            u32x4 oo[NR], xo[NR], x2o[NR];
            uint32_t yo[NR];
#pragma unroll
            for (int u = 0; u < NR; ++u) epi_off(g, u, ev[u], o2[u]);
            auto issue = [&](int u) {  // late / at-group-start form of the epilogue operand loads
                if (early || accum) oo[u] = buf_ld16(eb.ro, oo_off(g, u, o2[u]));
                if (bnb) {
                    xo[u] = buf_ld16(eb.rbx, o2[u]);
                    if (has_y) yo[u] = __builtin_amdgcn_raw_buffer_load_b8(eb.rym, ev[u] ? o2[u] >> 4 : BUF_OOB, 0, 0);
                    if (has_x2) x2o[u] = buf_ld16(eb.rx2o, o2[u]);
                }
            };
            if constexpr (EPF) {  // issued D groups ago (below): take them over
#pragma unroll
                for (int u = 0; u < NR; ++u) {
                    oo[u] = eoo[d][u];
                    if (bnb) {
                        xo[u] = exo[d][u];
                        if (has_y) yo[u] = eyo[d][u];
                        if (has_x2) x2o[u] = ex2o[d][u];
                    }
                }
            } else if constexpr (early) {
                // the BN-backward (x / mask) and residual reads go out before the MFMAs and BEFORE the next
                // prefetch: waiting for them leaves the prefetch in flight
#pragma unroll
                for (int u = 0; u < NR; ++u) issue(u);
            }
            fetch(d, g + D * wstride);
            f32x4 acc[FN];
#pragma unroll
            for (int i = 0; i < FN; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
            // weight fragments through a ring of RR registers, read RR - 1 MFMAs ahead of use, MFMA t = (k-step
            // t / FN, channel fragment t % FN) (the group barriers pin the interleave: left to itself the scheduler
            // issued each ds_read right before its MFMA and waited for it, a full LDS latency per MFMA)
            constexpr int NT = KS * FN, RR = NT < 8 ? NT : FN >= 16 && (FO || XBN) ? 3 : (FN >= 16 || MODE == 3 ? 4 : 8);
            bf16x8 fa[RR];
#pragma unroll
            for (int t = 0; t < RR - 1; ++t)
                fa[t] = *reinterpret_cast<const bf16x8*>(sW + (t % FN) * 16 * RB + aoff[t / FN]);
            __builtin_amdgcn_sched_group_barrier(0x100, RR - 1, 0);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                if (t + RR - 1 < NT) {
                    const int u = t + RR - 1;
                    fa[u % RR] = *reinterpret_cast<const bf16x8*>(sW + (u % FN) * 16 * RB + aoff[u / FN]);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
                acc[t % FN] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t % RR], fb[t / FN], acc[t % FN], 0, 0, 0);
                __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
            }
            // (1) fragments -> wave-private LDS rows (pixel fr, 4 channels per lane).
            // DS instructions of one wave execute in order: the re-reads below see
            // these writes, and the previous group's reads are complete (their
            // results were consumed) before these writes land.
#pragma unroll
            for (int i = 0; i < FN; ++i)
                *reinterpret_cast<u32x2*>(sE + fr * EP + epi_swz(fr, (i * 16 + fq * 4) * 2)) =
                    u32x2{pack_bf2(acc[i][0], acc[i][1]), pack_bf2(acc[i][2], acc[i][3])};
            __builtin_amdgcn_wave_barrier();
            // (2) coalesced row chunks: pixel q*PPR + lane/CH, channels n .. n+7
#pragma unroll
            for (int q0 = 0; q0 < NR; q0 += QB) {
                if constexpr (!early) {
#pragma unroll
                    for (int u = 0; u < QB; ++u) issue(q0 + u);
                }
#pragma unroll
                for (int u = 0; u < QB; ++u) {
                    const int q = q0 + u;
                    const int p = q * PPR + lane / CH;
                    const u32x4 t = epi_read(sE, p, EP, cc);
                    const float vf = ev[q] ? 1.f : 0.f;  // rows past M: stores dropped, statistics masked
                    float v[8];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        v[2 * k] = lo_bf(t[k]);
                        v[2 * k + 1] = hi_bf(t[k]);
                        if (affine) {
                            v[2 * k] = fmaf(v[2 * k], sc[2 * k], sh[2 * k]);
                            v[2 * k + 1] = fmaf(v[2 * k + 1], sc[2 * k + 1], sh[2 * k + 1]);
                        }
                        if (resaff) {
                            v[2 * k] = fmaf(lo_bf(oo[q][k]), rsc[2 * k], v[2 * k]);
                            v[2 * k + 1] = fmaf(hi_bf(oo[q][k]), rsc[2 * k + 1], v[2 * k + 1]);
                        } else if (accum || resid) {
                            v[2 * k] += lo_bf(oo[q][k]);
                            v[2 * k + 1] += hi_bf(oo[q][k]);
                        }
                        if (relu) {
                            v[2 * k] = fmaxf(v[2 * k], 0.f);
                            v[2 * k + 1] = fmaxf(v[2 * k + 1], 0.f);
                        }
                    }
                    if constexpr (K2 > 0) {
#pragma unroll
                        for (int c = 0; c < 8; ++c) v[c] += gbias[c];
                    }
                    float xv[8];
                    if (bnb) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            xv[2 * k] = lo_bf(xo[q][k]);
                            xv[2 * k + 1] = hi_bf(xo[q][k]);
                        }
#pragma unroll
                        for (int c = 0; c < 8; ++c) {
                            const bool keep = has_y ? ((yo[q] >> c) & 1u) : (fmaf(xv[c], sc[c], sh[c]) > 0.f);
                            if (!keep) v[c] = 0.f;
                        }
                    }
                    u32x4 o;
#pragma unroll
                    for (int k = 0; k < 4; ++k) o[k] = pack_bf2(v[2 * k], v[2 * k + 1]);
                    __builtin_amdgcn_raw_buffer_store_b128(o, eb.ry, o2[q], 0, 0);
                    if (q8out) {  // quantise the bf16-rounded values the bf16 consumers see
                        float w[8];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            w[2 * k] = lo_bf(o[k]);
                            w[2 * k + 1] = hi_bf(o[k]);
                        }
#pragma unroll
                        for (int i = 0; i < 8; ++i) m8 = fmaxf(m8, fabsf(w[i]) * vf);
                        __builtin_amdgcn_raw_buffer_store_b64(
                            u32x2{pack4_fp8(w[0] * q8s, w[1] * q8s, w[2] * q8s, w[3] * q8s),
                                  pack4_fp8(w[4] * q8s, w[5] * q8s, w[6] * q8s, w[7] * q8s)},
                            eb.ry8, ev[q] ? o2[q] / 2 : BUF_OOB, 0, 0);
                    }
                    if (maskout) {  // stored bf16 > 0: nonzero, sign clear, not NaN (as bn_fwd's ym)
                        uint32_t b = 0;
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const uint32_t h = (o[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
                            b |= (h != 0u && h <= 0x7F80u ? 1u : 0u) << i;
                        }
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b, eb.rym, ev[q] ? o2[q] / 16 : BUF_OOB, 0, 0);
                    }
                    if (a.stats) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {  // statistics of the stored (bf16) values
                            v[2 * k] = lo_bf(o[k]) * vf;
                            v[2 * k + 1] = hi_bf(o[k]) * vf;
                        }
                        if (bnb) {
#pragma unroll
                            for (int c = 0; c < 8; ++c) {
                                s1[c] += v[c] * ((xv[c] - mean[c]) * rstd[c]);
                                s2[c] += v[c];
                            }
                            if (has_x2) {
#pragma unroll
                                for (int c = 0; c < 8; ++c) {
                                    const float x2 = c & 1 ? hi_bf(x2o[q][c >> 1]) : lo_bf(x2o[q][c >> 1]);
                                    s3[c] += v[c] * ((x2 - m2[c]) * r2[c]);
                                }
                            }
                        } else {
#pragma unroll
                            for (int c = 0; c < 8; ++c) {
                                const float d = (v[c] - mean[c]) * vf;
                                s1[c] += d;
                                s2[c] += d * d;
                            }
                        }
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            if constexpr (EPF) issue_early(d, g + D * wstride);
        }
    }
    if (q8out) {  // one atomic per wave into the 32-slot amax row
        m8 = wave_max(m8);
        if (lane == 0) atomic_max_pos(a.y8amax + (blockIdx.x & 31), m8);
    }
    if (!a.stats) return;
    // fold the lanes that share a channel chunk, one atomic per channel and quantity
#pragma unroll
    for (int c = 0; c < 8; ++c) {
#pragma unroll
        for (int o = CH; o < 64; o <<= 1) {
            s1[c] += __shfl_xor(s1[c], o, 64);
            s2[c] += __shfl_xor(s2[c], o, 64);
            if (has_x2) s3[c] += __shfl_xor(s3[c], o, 64);
        }
    }
    if (lane >= CH) return;
    float* st = a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * (bnb ? 3 : 2) * a.Nout;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        atomicAdd(st + n + c, s1[c]);
        atomicAdd(st + a.Nout + n + c, s2[c]);
        if (has_x2) atomicAdd(st + 2 * a.Nout + n + c, s3[c]);
    }
}

template <int K, int BN, int D, int MODE, bool STEM = false, bool XBN = false, int K2 = 0>
int launch_stream1(const IGemmArgs& a, hipStream_t st) {
    constexpr int RP = stream_rp<STEM, K + K2>();
    const size_t lds = (size_t)BN * RP * 16 + 4 * 16 * (BN * 2);
    static int resident = 0;
    if (resident == 0) resident = resident_blocks(conv_stream_kernel<K, BN, D, MODE, STEM, XBN, K2>, lds);
    const int nsl = a.Nout / BN;
    const int ngroups = (a.M + 15) / 16;
    // enough pixel blocks to fill the chip, but >= D groups per wave
    const int npb = std::max(1, std::min(resident / nsl, (ngroups + 4 * D - 1) / (4 * D)));
    hipLaunchKernelGGL((conv_stream_kernel<K, BN, D, MODE, STEM, XBN, K2>), dim3(npb * nsl), dim3(256), lds, st, a);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

template <int K, int BN, int D>
int launch_plain(const IGemmArgs& a, hipStream_t st) {
    if (a.flags & (IG_RES | IG_MASKOUT | IG_Q8OUT)) return launch_stream1<K, BN, D, 4>(a, st);
    return launch_stream1<K, BN, D, 0>(a, st);
}

template <int K, int BN, int D>
int launch_stream(const IGemmArgs& a, hipStream_t st) {
    if (!(a.flags & IG_BNBWD)) return launch_plain<K, BN, D>(a, st);
    if constexpr (BN <= 128) {
        if (a.bnx2) return a.bnym ? launch_stream1<K, BN, D, 3>(a, st) : 1;
        return a.bnym ? launch_stream1<K, BN, D, 1>(a, st) : launch_stream1<K, BN, D, 2>(a, st);
    }
    return 1;
}

// The 7x7 / stride-2 stem (C = 4 padded channels -> 64) as a band kernel: a persistent block stages R output rows'
// worth of input rows (2R + 5 rows x the full padded width, 4 channels) in LDS ONCE and builds every B fragment
// from there -- a kernel row's 8 taps x 4 channels of one output pixel are 64 contiguous LDS bytes -- instead of
// gathering two 8-B pieces per tap row per pixel from L1/L2 (each input pixel fed ~12 output pixels: the
// streaming stem ran at 2.0 TB/s, 1.06 ms per call at 1024 img, profiles/r50_b1024_r5_standalone.md). Weights
// (64 x 7 x 32) live in registers (28 A fragments per lane). The next band's rows are loaded into registers
// while the current band computes, then written to the other LDS buffer. Epilogue as the streaming kernel's
// (wave-private swizzled LDS transpose -> coalesced 16-B stores, shifted forward statistics, or the eval
// forward's folded BatchNorm + ReLU).
// Layout: LDS input row pitch SP = 232 pixels x 8 B; input column c at byte (c + 4) * 8 (columns -4 .. -1 and
// W .. W + 3 stay zero: the padding taps and the zero-weight 8th tap read finite zeros).
template <int R>
__global__ __launch_bounds__(256, 2) void stem_band_kernel(const IGemmArgs a, int nbands) {
    constexpr int KH = 7, KS = 7, FN = 4;             // kernel rows (= MFMA k-steps), 64 / 16 channel fragments
    constexpr int PR = 2 * R + KH - 2;                  // staged input rows per band
    constexpr int SP = 232 * 8;                         // LDS row pitch, bytes
    constexpr int BUF = PR * SP;
    constexpr int EP = 64 * 2;                          // epilogue row pitch (64 channels)
    constexpr int W16 = 112;                            // 16-B chunks per input row (224 px x 8 B)
    constexpr int NCH = PR * W16;                       // chunks per band
    constexpr int CPT = (NCH + 255) / 256;              // chunks per thread
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* sE = smem + 2 * BUF + (threadIdx.x >> 6) * 16 * EP;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int bpi = (a.OH + R - 1) / R;  // bands per image

    // zero both buffers once (padding columns stay zero: the band loads write columns 0 .. W-1 only)
    for (int e = tid; e < 2 * BUF / 16; e += 256) reinterpret_cast<u32x4*>(smem)[e] = u32x4{0u, 0u, 0u, 0u};
    // weights: A fragment (kernel row ks, channel fragment i) = Wk[i * 16 + fr][ks * 32 + fq * 8 .. + 8]
    bf16x8 wa[KS][FN];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < FN; ++i)
            wa[ks][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(
                                                       a.Wk + (size_t)(i * 16 + fr) * a.ldb + ks * 32 + fq * 8));
    // epilogue constants of this lane's fixed channel chunk
    const int cc = lane & 7, n = cc * 8;
    const bool affine = a.flags & IG_AFFINE, relu = a.flags & IG_RELU;
    float mean[8], sc[8], sh[8], s1[8], s2[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        mean[c] = (a.stats && a.shift) ? a.shift[n + c] : 0.f;
        sc[c] = affine ? a.bias[n + c] : 1.f;
        sh[c] = affine ? a.bias[a.Nout + n + c] : 0.f;
        s1[c] = s2[c] = 0.f;
    }

    u32x4 stage[CPT];
    auto load_band = [&](int band) {  // global -> registers
        const int img = band / bpi, oy0 = (band - img * bpi) * R;
        const int iy0 = 2 * oy0 - 3;
#pragma unroll
        for (int t = 0; t < CPT; ++t) {
            const int e = tid + 256 * t;
            const int r = e / W16, c16 = e - r * W16, iy = iy0 + r;
            const bool ok = e < NCH && (unsigned)iy < (unsigned)a.H;
            stage[t] = ok ? *reinterpret_cast<const u32x4*>(a.X + (((size_t)img * a.H + iy) * a.W) * 4 + c16 * 8)
                          : u32x4{0u, 0u, 0u, 0u};
        }
    };
    auto store_band = [&](int buf) {  // registers -> LDS (column 0 at byte 32)
#pragma unroll
        for (int t = 0; t < CPT; ++t) {
            const int e = tid + 256 * t;
            if (e < NCH) {
                const int r = e / W16, c16 = e - r * W16;
                *reinterpret_cast<u32x4*>(smem + buf * BUF + r * SP + 32 + c16 * 16) = stage[t];
            }
        }
    };

    int band = blockIdx.x;
    if (band < nbands) load_band(band);
    __syncthreads();  // (the zero fill)
    if (band < nbands) store_band(0);
    __syncthreads();
    int buf = 0;
    for (; band < nbands; band += gridDim.x) {
        const int nxt = band + gridDim.x;
        if (nxt < nbands) load_band(nxt);  // in flight under this band's MFMAs
        const int img = band / bpi, oy0 = (band - img * bpi) * R;
        const char* sb = smem + buf * BUF;
        const int rows = min(R, a.OH - oy0);
        const int ngroups = rows * (a.OW / 16);
        for (int g = wid; g < ngroups; g += 4) {
            const int ry = g / (a.OW / 16), ox0 = (g - ry * (a.OW / 16)) * 16;
            const int ox = ox0 + fr;
            f32x4 acc[FN];
#pragma unroll
            for (int i = 0; i < FN; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                // taps 2fq, 2fq + 1 of kernel row ks: input row 2 (oy0 + ry) + ks - 3 = staged row 2 ry + ks,
                // columns 2 ox - 3 + 2 fq .. + 1 at byte (2 ox + 1 + 2 fq) * 8
                const char* pb = sb + (2 * ry + ks) * SP + (2 * ox + 1 + 2 * fq) * 8;
                const u32x2 lo = *reinterpret_cast<const u32x2*>(pb);
                const u32x2 hi = *reinterpret_cast<const u32x2*>(pb + 8);
                const bf16x8 fb = __builtin_bit_cast(bf16x8, u32x4{lo[0], lo[1], hi[0], hi[1]});
#pragma unroll
                for (int i = 0; i < FN; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[ks][i], fb, acc[i], 0, 0, 0);
            }
            // (1) fragments -> wave-private LDS rows (pixel fr, channels i * 16 + 4 fq .. + 3), swizzled
#pragma unroll
            for (int i = 0; i < FN; ++i)
                *reinterpret_cast<u32x2*>(sE + fr * EP + epi_swz(fr, (i * 16 + fq * 4) * 2)) =
                    u32x2{pack_bf2(acc[i][0], acc[i][1]), pack_bf2(acc[i][2], acc[i][3])};
            __builtin_amdgcn_wave_barrier();
            // (2) row chunks: pixel q * 8 + lane / 8, channels n .. n + 7
            const long m0 = ((long)img * a.OH + oy0 + ry) * a.OW + ox0;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int p = q * 8 + (lane >> 3);
                const u32x4 t = epi_read(sE, p, EP, cc);
                float v[8];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v[2 * k] = fmaf(lo_bf(t[k]), sc[2 * k], sh[2 * k]);
                    v[2 * k + 1] = fmaf(hi_bf(t[k]), sc[2 * k + 1], sh[2 * k + 1]);
                    if (relu) {
                        v[2 * k] = fmaxf(v[2 * k], 0.f);
                        v[2 * k + 1] = fmaxf(v[2 * k + 1], 0.f);
                    }
                }
                u32x4 o;
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] = pack_bf2(v[2 * k], v[2 * k + 1]);
                *reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(a.Y) + (m0 + p) * a.ldy + n) = o;
                if (a.stats) {
#pragma unroll
                    for (int c = 0; c < 8; ++c) {  // statistics of the stored (bf16) values
                        const float d = (c & 1 ? hi_bf(o[c >> 1]) : lo_bf(o[c >> 1])) - mean[c];
                        s1[c] += d;
                        s2[c] += d * d;
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        // buffer buf ^ 1 was last read in the previous band, which every wave finished before the barrier below in
        // that iteration; the barrier orders these stores before the next band's reads
        if (nxt < nbands) store_band(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    if (!a.stats) return;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
#pragma unroll
        for (int o = 8; o < 64; o <<= 1) {
            s1[c] += __shfl_xor(s1[c], o, 64);
            s2[c] += __shfl_xor(s2[c], o, 64);
        }
    }
    if (lane >= 8) return;
    float* st = a.stats + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * 2 * a.Nout;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        atomicAdd(st + n + c, s1[c]);
        atomicAdd(st + a.Nout + n + c, s2[c]);
    }
}

// the band stem's shapes: 4-channel 224-wide input, 7x7 / stride 2 / pad 3, 64 channels, 16 | OW, dense bf16 output
bool stem_band_ok(const IGemmArgs& a) {
    if (a.flags & (IG_OUT_F32 | IG_FP8 | IG_ACCUM | IG_BNBWD | IG_NOSTREAM | IG_RES | IG_MASKOUT | IG_Q8OUT)) return false;
    if ((a.flags & IG_RELU) && !(a.flags & IG_AFFINE)) return false;
    if ((a.bias && !(a.flags & IG_AFFINE)) || a.xbn || a.X2) return false;
    return a.C == 4 && a.W == 224 && a.nth == 7 && a.ntw == 7 && a.sA == 2 && a.dh0 == -3 && a.dw0 == -3 &&
           a.dhs == 1 && a.dws == 1 && a.Nout == 64 && a.ldb == 7 * 32 && a.ldy == 64 && a.OW % 16 == 0 &&
           2 * (a.OW - 1) - 3 + 8 <= a.W + 3 && a.sY == 1 && a.YH == a.OH && a.YW == a.OW && a.oy == 0 && a.ox == 0;
}

int launch_stem_band(const IGemmArgs& a, hipStream_t st) {
    // R = 4 output rows per band (2048 img: 1,205 us; R = 2 1,391, R = 6 1,344 and R = 8 2,258 spill -- the 28 weight
    // fragments held in registers leave no room for a taller band's prefetch)
    constexpr int R = 4;
    const size_t lds = 2 * (size_t)(2 * R + 5) * 232 * 8 + 4 * 16 * 64 * 2;
    static int resident = 0;
    if (resident == 0) resident = resident_blocks(stem_band_kernel<R>, lds);
    const int nbands = a.N * ((a.OH + R - 1) / R);
    hipLaunchKernelGGL((stem_band_kernel<R>), dim3(std::min(nbands, resident)), dim3(256), lds, st, a, nbands);
    CONV_COUNTED();
    IMK_CHECK_LAUNCH();
    return 0;
}

}  // namespace

// the 7x7 stem forward: the band kernel (tile 0) or the streaming row-segment kernel (tile 23, A/B); 1: not covered
int conv_stem(const IGemmArgs& a, hipStream_t st, int tile) {
    if (tile == 0 && stem_band_ok(a)) return launch_stem_band(a, st);
    return conv_stream(a, st, 0);
}

// Returns 1 if the shape is not one this kernel covers (caller falls back).
// bn: channel-slice width (0 auto: the widest that divides Nout; 64/128/256 forced)
int conv_stream(const IGemmArgs& a, hipStream_t st, int bn) {
    const int bn_hint = bn;  // explicit slice width (tiles 20-22), before the defaults below
    // the eval forward's folded BatchNorm (+ ReLU): plain epilogue, no statistics
    const bool eval_bn = a.flags & IG_AFFINE;
    if ((a.flags & IG_RELU) && !eval_bn) return 1;
    if (eval_bn && (a.stats || a.xbn || (a.flags & IG_BNBWD))) return 1;
    if ((a.flags & (IG_RES | IG_MASKOUT | IG_Q8OUT)) &&
        (!eval_bn || (a.flags & (IG_ACCUM | IG_BNBWD | IG_STEM)) || ((a.flags & IG_RES) && !a.bnx) ||
         ((a.flags & IG_MASKOUT) && (!a.bnym || !(a.flags & IG_RELU))) ||
         ((a.flags & IG_Q8OUT) && (!a.Y8 || !a.y8exp || !a.y8amax))))
        return -121;
    const bool has_bias = a.bias && !eval_bn;
    if (a.X2) {
        // the Gram-form conv3 dgrad of a 64-channel bottleneck (bn_gram.hip): K = [g (256) | h2 (64)] into 64
        // channels with bn2's BN-backward epilogue, weights [64][320] resident in LDS (the 128 x 64 v3 tile
        // re-stages them per tile and ran these HBM streams at ~2.7 TB/s)
        if (!(a.flags & IG_BNBWD) || (a.flags & (IG_ACCUM | IG_FP8 | IG_OUT_F32 | IG_AFFINE | IG_NOSTREAM | IG_RES |
                                                  IG_MASKOUT | IG_Q8OUT)) ||
            a.C != 256 || a.C2 != 64 || a.Nout != 64 || a.ldb != 320 || a.ldy != 64 || !a.bias || a.bnx2 ||
            a.nth != 1 || a.ntw != 1 || a.sA != 1 || a.H != a.OH || a.W != a.OW || a.sY != 1 || a.YH != a.OH ||
            a.YW != a.OW || a.dh0 != 0 || a.dw0 != 0 || a.kh0 != 0 || a.kw0 != 0 || a.oy != 0 || a.ox != 0)
            return 1;
        return a.bnym ? launch_stream1<256, 64, 2, 1, false, false, 64>(a, st)
                      : launch_stream1<256, 64, 2, 2, false, false, 64>(a, st);
    }
    if (a.flags & IG_STEM) {  // 7x7 stem, C = 4, K = 7 x 32
        if (a.flags & (IG_OUT_F32 | IG_FP8 | IG_ACCUM | IG_BNBWD | IG_NOSTREAM)) return 1;
        if (has_bias || a.C != 4 || a.nth != 7 || a.ntw > 8 || a.ldb != 7 * 32 || a.Nout % 64 || a.ldy != a.Nout ||
            a.sY != 1 || a.YH != a.OH || a.YW != a.OW)
            return 1;
        return launch_stream1<7 * 32, 64, 2, 0, true>(a, st);
    }
    if (a.flags & (IG_OUT_F32 | IG_FP8 | IG_REGSTAGE | IG_NOSTREAM)) return 1;
    if (a.xbn) {  // BN apply + ReLU on the operand load: K = 64 / 128 plain-epilogue 1x1 convs only
        if ((a.flags & (IG_BNBWD | IG_ACCUM)) || a.bias || a.nth != 1 || a.ntw != 1 || a.sA != 1 ||
            a.H != a.OH || a.W != a.OW || a.sY != 1 || a.YH != a.OH || a.YW != a.OW || a.ldy != a.Nout ||
            a.ldb < a.C || a.dh0 != 0 || a.dw0 != 0)
            return -120;
        if (a.C == 64 && a.Nout % 256 == 0) return launch_stream1<64, 256, 2, 0, false, true>(a, st);
        if (a.C == 64 && a.Nout % 128 == 0) return launch_stream1<64, 128, 3, 0, false, true>(a, st);
        if (a.C == 128 && a.Nout % 128 == 0) return launch_stream1<128, 128, 2, 0, false, true>(a, st);
        return -120;
    }
    if (has_bias || a.nth != 1 || a.ntw != 1 || a.dh0 != 0 || a.dw0 != 0 || a.kh0 != 0 || a.kw0 != 0) return 1;
    if (a.sY != 1 || a.oy != 0 || a.ox != 0 || a.YH != a.OH || a.YW != a.OW || a.ldy != a.Nout) return 1;
    if (a.Nout % 64 != 0 || a.ldb < a.C) return 1;
    if ((long)(a.OH - 1) * a.sA >= a.H || (long)(a.OW - 1) * a.sA >= a.W) return 1;
    // K = 256 into > 128 channels (bottleneck conv3 / downsample forwards): 64-channel
    // weight slices resident in LDS, the slices of one pixel range on one XCD (the pixels
    // are fetched from HBM once and re-read from that XCD's L2).
    // Only K = 256: at K = 512 the v3 tiles win (conv_bench at 1024 img: 512 -> 2048 @7 fwd 210 -> 179 us,
    // 512 -> 1024 /2 @28 443 -> 375, 2048 -> 512 dgrad 209 -> 152; K = 256 stays here: 256 -> 1024 @14
    // fwd 264 vs 370).
    // 128-channel slices where Nout allows (half the slices re-reading each pixel group, twice the MFMAs per
    // loaded fragment: 256 -> 1024 @14 fwd 277 -> 246 us at 1024 img, round 5); tile 22 forces 64
    if (!(a.flags & IG_BNBWD) && a.C == 256 && a.Nout > 128) {
        if (bn != 64 && a.Nout % 128 == 0) return launch_plain<256, 128, 2>(a, st);
        if (bn != 0 && bn != 64) return 1;
        return launch_plain<256, 64, 2>(a, st);
    }
    int maxbn = (a.C == 64 && !(a.flags & IG_BNBWD)) ? 256 : 128;
    if (a.flags & IG_BNBWD) {
        // BN-backward epilogue: every K = 64 / 128 / 256 dgrad, with or without the second BN branch, 128-channel
        // slices. Same-box bench A/B at R50 / 1024 with the ReLU mask as bits (round 3): 73.9 ms/step vs 75.2 with
        // K = 128 on the tiled kernels and 75.0 with the second branch there too; 64-channel slices neutral
        maxbn = 128;
    }
    if (bn == 0) bn = maxbn;
    while (bn > 64 && (bn > maxbn || a.Nout % bn)) bn >>= 1;
    if (a.C == 64) {
        // 256-channel slices: the fused-output / operand-BN variants prefetch 2 groups (3 spill at 256 VGPRs)
        if (bn == 256)
            return (a.flags & (IG_RES | IG_MASKOUT | IG_Q8OUT)) ? launch_stream1<64, 256, 2, 4>(a, st)
                                                                : launch_stream1<64, 256, 3, 0>(a, st);
        if (bn == 128) return launch_stream<64, 128, 3>(a, st);
        return launch_stream<64, 64, 3>(a, st);
    }
    if (a.C == 128) {
        if (bn == 128) return launch_stream<128, 128, 2>(a, st);
        return launch_stream<128, 64, 2>(a, st);
    }
    // K = 256 BN-backward dgrads into wide outputs (bottleneck conv1 dgrads 256 -> 512 @28, 256 -> 1024 @14): 64-channel
    // weight slices resident in LDS (as the K = 256 forwards) instead of the one-tile-per-block v3 loop, whose
    // 4-stage main loop leaves these epilogue-heavy GEMMs latency-bound (-20 % per call, round 4)
    if (a.C == 256 && (a.flags & IG_BNBWD) && a.Nout > 128) {
        // 128-channel slices (half the slices re-reading each pixel group): in-step A/B at 2048 img 16,622 / 16,663
        // vs 16,530 / 16,522 img/s with 64 (1024 -> 256 @14 dgrad + BN backward 705 -> 488 us, 512 -> 256 @28
        // 1460 -> 1033; at 1024 img round 5 they had measured even); tile 22 forces 64. The second-BN-branch form
        // stays on 64 (at 128 it spills 96 B: in-step 16,604 / 16,651 vs 16,662 / 16,653)
        if (bn_hint != 64 && a.Nout % 128 == 0 && !a.bnx2)
            return a.bnym ? launch_stream1<256, 128, 2, 1>(a, st) : launch_stream1<256, 128, 2, 2>(a, st);
        if (a.bnx2) return a.bnym ? launch_stream1<256, 64, 2, 3>(a, st) : 1;
        return a.bnym ? launch_stream1<256, 64, 2, 1>(a, st) : launch_stream1<256, 64, 2, 2>(a, st);
    }
    // K = 256 into <= 128 channels (bottleneck conv1 256 -> 64 / 128): 64-channel
    // slices, plain epilogue
    if (a.C == 256 && a.Nout <= 128) {
        if (!(a.flags & IG_BNBWD)) return launch_plain<256, 64, 2>(a, st);
        if (!a.bnx2) return a.bnym ? launch_stream1<256, 64, 2, 1>(a, st) : launch_stream1<256, 64, 2, 2>(a, st);
    }
    return 1;
}
