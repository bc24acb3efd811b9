// Shared device helpers for the trustworthy_dl gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in csrc/:
//  * bf16 tensors are passed as raw uint16 storage; conversion f32->bf16 uses the native
//    v_cvt_pk_bf16_f32 (via the clang __bf16 cast), which keeps NaNs NaN.
//  * wave size is 64 (hard-coded, never warpSize tricks from 32-lane code).
//  * every entry point is `extern "C" int tdl_*(..., hipStream_t)` returning hipError_t of
//    the launch, so the Python side can launch on any (graph-capturing) stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define TDL_API extern "C" __attribute__((visibility("default")))

typedef uint16_t bf16_t;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
}
// Unpack / pack 8 bf16 held in a 16-byte uint4.
__device__ __forceinline__ void unpack8(const uint4 u, float* f) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
// Two floats -> two bf16 in ONE v_cvt_pk_bf16_f32 (a vector conversion; two scalar __bf16 casts
// compiled to two single-source conversions plus a shift and an SDWA or: 4 VALU instead of 1 — a
// third of gemm_pd's epilogue instructions).  Bit-identical to f2bf on each element.
typedef float tdl_f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 tdl_bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {
    const tdl_bf16x2_t r = __builtin_convertvector((tdl_f32x2_t){a, b}, tdl_bf16x2_t);
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
    return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}
__device__ __forceinline__ void unpack4(const uint2 u, float* f) {
    f[0] = __uint_as_float(u.x << 16);
    f[1] = __uint_as_float(u.x & 0xffff0000u);
    f[2] = __uint_as_float(u.y << 16);
    f[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ uint2 pack4(const float* f) {
    return make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
}

// ---------------------------------------------------------------- wave / block reductions
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
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats.  All threads get it.
__device__ __forceinline__ float block_sum(float v, float* red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float r = 0.f;
    for (int i = 0; i < nw; ++i) r += red[i];
    return r;
}
__device__ __forceinline__ float block_max(float v, float* red) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float r = -INFINITY;
    for (int i = 0; i < nw; ++i) r = fmaxf(r, red[i]);
    return r;
}

// ---------------------------------------------------------------- Philox4x32-10 counter RNG
struct Philox {
    __device__ static inline uint4 round(uint4 c, uint2 k) {
        const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
        uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
        uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
        return make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    }
    __device__ static inline uint4 gen(uint64_t seed, uint64_t counter) {
        uint4 c = make_uint4((uint32_t)counter, (uint32_t)(counter >> 32), 0u, 0u);
        uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            c = round(c, k);
            k.x += 0x9E3779B9u;
            k.y += 0xBB67AE85u;
        }
        return c;
    }
};
__device__ __forceinline__ float u32_to_unit(uint32_t x) {  // (0, 1]
    return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------- GELU (tanh approximation)
// gelu(u) = 0.5 u (1 + tanh(a)) = u * sigmoid(2a),  a = k0 (u + k1 u^3).
// Written as u / (1 + 2^(u (c0 + c1 u^2))) with the log2(e) factor folded into c0/c1: one v_exp, one
// v_rcp (1 ulp, far below bf16 resolution) and a few FMAs per element.  The IEEE division of the
// tanh form cost ~10 VALU per element and left both kernels ALU-bound (fwd 24, bwd 31 VALU / element).
#define TDL_GELU_C0 (-2.0f * 0.7978845608028654f * 1.4426950408889634f)
#define TDL_GELU_C1 (-2.0f * 0.7978845608028654f * 0.044715f * 1.4426950408889634f)
__device__ __forceinline__ float gelu_sigmoid2a(float u) {  // sigmoid(2a)
    const float e = __builtin_amdgcn_exp2f(u * fmaf(TDL_GELU_C1, u * u, TDL_GELU_C0));
    return __builtin_amdgcn_rcpf(1.0f + e);
}
__device__ __forceinline__ float gelu_tanh(float u) { return u * gelu_sigmoid2a(u); }
__device__ __forceinline__ float gelu_tanh_grad(float u) {
    // d/du [u s(u)] = s + u s (1 - s) 2 k0 (1 + 3 k1 u^2)
    const float s = gelu_sigmoid2a(u);
    const float da = 2.0f * 0.7978845608028654f * fmaf(3.0f * 0.044715f, u * u, 1.0f);
    return fmaf(u * s * (1.0f - s), da, s);
}

#define TDL_LAUNCH_CHECK() return (int)hipGetLastError()
