// Shared helpers for the gfx950 (CDNA4, MI355X) kernels.
// Wave = 64 lanes; MFMA 16x16x32 bf16 fragments; bf16 stored as raw u16.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

typedef uint16_t bf16_t;  // storage type (raw bits)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

#define WAVE 64
#define LDS_PTR(T) __attribute__((address_space(3))) T*

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

// Round-to-nearest-even via the hardware convert (v_cvt_pk_bf16_f32 on gfx950;
// NaN stays NaN - MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ bf16_t f2bf(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
    return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ float lo_bf(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks that the dispatcher deals to the same XCD
// (b % 8 equal) get a contiguous range of logical tile ids, so neighbouring
// tiles that share operand panels hit the same 4 MiB L2.
// raw buffer access: num_records 2^31 - 1 (or 0 for an operand a launch does not use: loads read zeros, stores
// are dropped); per-lane offsets >= BUF_OOB are out of range. Branch-free predication for the streaming loops:
// a predicated pointer load puts the load under a divergent branch, and the compiler's waitcnt bookkeeping then
// falls back to s_waitcnt vmcnt(0) around it, draining every prefetch in flight (conv_stream.hip, conv_halo.hip)
constexpr uint32_t BUF_OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, bool on = true) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, on ? 0x7FFFFFFF : 0, 0x00020000);
}
__device__ __forceinline__ u32x4 buf_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ void buf_st16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    if (nwg <= 8) return orig;
    const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (orig >> 3);
}

#define IMK_EXPORT extern "C" __attribute__((visibility("default")))

// host-side count of conv kernel launches (conv_igemm.hip): lets the per-call conv log
// (ops/conv.py IMAGENT_CONV_LOG) map each call to its kernel dispatches in a rocprof trace
// (scripts/conv_roofline.py)
extern "C" int g_imk_conv_launches;
#define CONV_COUNTED() (++g_imk_conv_launches)

#define IMK_CHECK_LAUNCH()                         \
    do {                                           \
        hipError_t e_ = hipGetLastError();         \
        if (e_ != hipSuccess) return (int)e_;      \
    } while (0)

// ---- fp8 (OCP e4m3, gfx950 v_cvt_pk_fp8_f32), saturating to +-448
constexpr float E4M3_MAX = 448.f;

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
    a = fminf(fmaxf(a, -E4M3_MAX), E4M3_MAX);
    b = fminf(fmaxf(b, -E4M3_MAX), E4M3_MAX);
    c = fminf(fmaxf(c, -E4M3_MAX), E4M3_MAX);
    d = fminf(fmaxf(d, -E4M3_MAX), E4M3_MAX);
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
    return (uint32_t)w;
}

__device__ __forceinline__ void atomic_max_pos(float* p, float v) {
    // v >= 0: IEEE order of non-negative floats == order of their bit patterns
    atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v));
}
