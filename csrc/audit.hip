// Backward-audit primitives for the commit-then-reveal gradient check (security/grad_audit.py,
// parallel/commitments.py).  Reference: the gradient check there is a host z-score
// (/root/reference/attack_detector.py:109-141) that a sign flip passes; r4's replacement sampled
// 1/16 of the gradient under sign patterns derived from public values, which an adaptive adversary
// can evade by perturbing only the unsampled coordinates or the null space of the public signs.
//
//  * word hash   — exact, order-independent 64-bit hash of a range of 32-bit words:
//                  H = sum_j mix(w_j ^ mix(j ^ seed))  (mod 2^64, integer atomics: any launch order
//                  gives the same bits), optionally copying the range into a snapshot in the same
//                  pass.  Commits the running gradient after every micro-batch and the applied one.
//  * keyed sketch — K = 4 full-coverage random-sign projections sum_j s_k(key, j) (a_j - b_j) with
//                  the signs derived from a PRIVATE per-step key revealed only after the
//                  commitments were sent; two-pass, fixed-order reduction (deterministic).
// The mixing function is the same 32-bit integer mix as the CPU reference in grad_audit.py, so CPU
// and GPU give identical hashes and signs (constants < 2^31: the CPU path multiplies in int64).
#include "common.h"

namespace {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x6c8e9cf5u;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

constexpr int HB = 256;

// acc += sum over j in [lo, hi) of mix(x[j] ^ mix(j ^ seed)); dst (nullable): dst[j] = x[j]
__global__ __launch_bounds__(HB) void word_hash_kernel(const uint32_t* __restrict__ x, uint32_t* __restrict__ dst,
                                                      long long lo, long long hi, uint32_t seed,
                                                      unsigned long long* __restrict__ acc) {
    __shared__ unsigned long long red[HB / 64];
    unsigned long long s = 0;
    const long long stride = (long long)gridDim.x * HB;
    for (long long j = lo + (long long)blockIdx.x * HB + threadIdx.x; j < hi; j += stride) {
        const uint32_t w = x[j];
        if (dst != nullptr) dst[j] = w;
        s += mix32(w ^ mix32((uint32_t)j ^ seed));
    }
    s = wave_sum_u64(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
#pragma unroll
        for (int i = 0; i < HB / 64; ++i) t += red[i];
        atomicAdd(acc, t);   // integer add: exact and order-independent
    }
}

// part[block][k] = sum over this block's j of s_k(key, j) * (a[j] - b[j])   (b nullable)
__global__ __launch_bounds__(HB) void keyed_sketch_partial_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                                 long long lo, long long hi, uint32_t k0, uint32_t k1,
                                                                 float* __restrict__ part) {
    __shared__ float red[HB / 64][4];
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    const long long stride = (long long)gridDim.x * HB;
    for (long long j = lo + (long long)blockIdx.x * HB + threadIdx.x; j < hi; j += stride) {
        const float v = b != nullptr ? a[j] - b[j] : a[j];
        const uint32_t h = mix32(mix32((uint32_t)j ^ k0) ^ k1);
#pragma unroll
        for (int k = 0; k < 4; ++k) s[k] += (h >> (28 + k)) & 1u ? -v : v;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = wave_sum(s[k]);
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) red[threadIdx.x >> 6][k] = s[k];
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < HB / 64; ++i) t += red[i][threadIdx.x];
        part[blockIdx.x * 4 + threadIdx.x] = t;
    }
}

// out[k] (+)= sum over blocks of part[.][k], in block order (one wave per k)
__global__ __launch_bounds__(256) void keyed_sketch_final_kernel(const float* __restrict__ part, int nb, float* __restrict__ out,
                                                                int accumulate) {
    const int k = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float t = 0.f;
    for (int i = lane; i < nb; i += 64) t += part[i * 4 + k];
    t = wave_sum(t);
    if (lane == 0) out[k] = accumulate ? out[k] + t : t;
}

int grid_for(long long n, int cap) {
    const long long b = (n + HB * 8 - 1) / (HB * 8);   // ~8 elements per thread
    return (int)(b < 1 ? 1 : b > cap ? cap : b);
}

}  // namespace

// acc (device uint64, caller-zeroed) += word hash of x[lo:hi) (32-bit words); dst (nullable) gets a copy
TDL_API int tdl_word_hash(const void* x, void* dst, long long lo, long long hi, unsigned int seed,
                          unsigned long long* acc, hipStream_t s) {
    if (hi <= lo) return 0;
    word_hash_kernel<<<grid_for(hi - lo, 2048), HB, 0, s>>>((const uint32_t*)x, (uint32_t*)dst, lo, hi, seed, acc);
    TDL_LAUNCH_CHECK();
}

// number of partial rows the keyed sketch uses (workspace: 4 floats each)
TDL_API long long tdl_keyed_sketch_ws_floats(long long n) { return 4LL * grid_for(n, 1024); }

// out[0..3] (+)= keyed sketch of (a - b)[lo:hi) (b nullable) under key (k0, k1); ws >= ws_floats
TDL_API int tdl_keyed_sketch(const float* a, const float* b, long long lo, long long hi, unsigned int k0,
                             unsigned int k1, float* ws, float* out, int accumulate, hipStream_t s) {
    if (hi <= lo) {
        if (!accumulate) hipMemsetAsync(out, 0, 4 * sizeof(float), s);
        TDL_LAUNCH_CHECK();
    }
    const int nb = grid_for(hi - lo, 1024);
    keyed_sketch_partial_kernel<<<nb, HB, 0, s>>>(a, b, lo, hi, k0, k1, ws);
    keyed_sketch_final_kernel<<<1, 256, 0, s>>>(ws, nb, out, accumulate);
    TDL_LAUNCH_CHECK();
}
