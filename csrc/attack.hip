// Deterministic fault / attack injection on stage tensors.
// The reference only names an `AdversarialAttacker` (experiment_runner.py:23, 91-97, 187-188)
// and never ships it; this is the device side of ours: in-place perturbation of gradients,
// parameters or activations of a target stage, driven by a counter-based Philox RNG so a
// (seed, offset) pair reproduces the exact same attack on any GPU / stream / graph replay.
//
// modes: 0 scale (x *= a)            1 gaussian noise (x += a * N(0,1))
//        2 sign flip (x = -a * x)    3 zero (x = 0)
//        4 relative noise (x *= 1 + a * N(0,1))   5 uniform shift (x += a)
#include "common.h"

template <typename T>
__device__ __forceinline__ float ld(const T* p, int64_t i);
template <> __device__ __forceinline__ float ld<float>(const float* p, int64_t i) { return p[i]; }
template <> __device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
__device__ __forceinline__ void st(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st(bf16_t* p, int64_t i, float v) { p[i] = f2bf(v); }

template <typename T>
__global__ __launch_bounds__(256) void inject_kernel(T* __restrict__ x, int64_t n, int mode, float a, uint64_t seed,
                                                     uint64_t offset) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
    for (int64_t base = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 4; base < n; base += stride) {
        float z[4] = {0.f, 0.f, 0.f, 0.f};
        if (mode == 1 || mode == 4) {
            const uint4 r = Philox::gen(seed, offset + (uint64_t)(base >> 2));
            // Box-Muller on two pairs
            const float u1 = u32_to_unit(r.x), u2 = u32_to_unit(r.y), u3 = u32_to_unit(r.z), u4 = u32_to_unit(r.w);
            const float r1 = sqrtf(-2.f * __logf(u1)), r2 = sqrtf(-2.f * __logf(u3));
            float s1, c1, s2, c2;
            __sincosf(6.283185307f * u2, &s1, &c1);
            __sincosf(6.283185307f * u4, &s2, &c2);
            z[0] = r1 * c1; z[1] = r1 * s1; z[2] = r2 * c2; z[3] = r2 * s2;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t i = base + k;
            if (i >= n) break;
            float v = ld<T>(x, i);
            switch (mode) {
                case 0: v *= a; break;
                case 1: v += a * z[k]; break;
                case 2: v = -a * v; break;
                case 3: v = 0.f; break;
                case 4: v *= 1.f + a * z[k]; break;
                default: v += a; break;
            }
            st(x, i, v);
        }
    }
}

TDL_API int tdl_attack_inject(void* x, int dtype, int64_t n, int mode, float intensity, uint64_t seed, uint64_t offset,
                              hipStream_t s) {
    const int64_t work = (n / 4 + 255) / 256;
    const int grid = (int)(work < 4096 ? (work > 0 ? work : 1) : 4096);
    if (dtype == 1) inject_kernel<bf16_t><<<grid, 256, 0, s>>>((bf16_t*)x, n, mode, intensity, seed, offset);
    else inject_kernel<float><<<grid, 256, 0, s>>>((float*)x, n, mode, intensity, seed, offset);
    TDL_LAUNCH_CHECK();
}
