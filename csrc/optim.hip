// Fused AdamW over a stage's FLAT parameter space (replaces the
// never-populated per-node optimizers of distributed_trainer.py:441-446).
//
// Every stage keeps its parameters in four contiguous fp32 buffers (master, exp_avg,
// exp_avg_sq, main_grad) and the model-visible bf16 weights in one contiguous buffer, so
// the whole optimizer step is ONE bandwidth-bound launch (float4 / 16-byte lanes) that also
// zeroes the gradient.  `ctrl` is a 2-float device control block written by the
// verification path: ctrl[0] = gradient scale (clipping), ctrl[1] != 0 => the stage's
// gradient was flagged by the verifier: the update is skipped (quarantined) on device, with
// no host round trip, and the gradient is still cleared.
#include "common.h"

__global__ __launch_bounds__(256) void adamw_flat_kernel(float* __restrict__ master, float* __restrict__ m,
                                                         float* __restrict__ v, float* __restrict__ grad,
                                                         bf16_t* __restrict__ out, int64_t n, float lr, float b1,
                                                         float b2, float eps, float wd, float bc1, float bc2,
                                                         const float* __restrict__ ctrl, int zero_grad) {
    const float gscale = ctrl ? ctrl[0] : 1.0f;
    const bool skip = ctrl ? (ctrl[1] != 0.0f) : false;
    const float step_size = lr / bc1;
    const float inv_sqrt_bc2 = rsqrtf(bc2);
    const int64_t n4 = n / 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // two float4 groups per lane per trip, all eight 16-B loads issued before any math (the single-
    // group loop kept one load set in flight per lane: ~4.6 TB/s over the 34 B / parameter stream)
    auto update = [&](float4 g, float4 p, float4 mm, float4 vv, int64_t i) {
        float pa[4] = {p.x, p.y, p.z, p.w}, ga[4] = {g.x, g.y, g.z, g.w};
        float ma[4] = {mm.x, mm.y, mm.z, mm.w}, va[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float gg = ga[k] * gscale;
            ma[k] = b1 * ma[k] + (1.f - b1) * gg;
            va[k] = b2 * va[k] + (1.f - b2) * gg * gg;
            pa[k] = pa[k] * (1.f - lr * wd);
            pa[k] -= step_size * ma[k] / (sqrtf(va[k]) * inv_sqrt_bc2 + eps);
        }
        ((float4*)master)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
        ((float4*)m)[i] = make_float4(ma[0], ma[1], ma[2], ma[3]);
        ((float4*)v)[i] = make_float4(va[0], va[1], va[2], va[3]);
        if (out) ((uint2*)out)[i] = make_uint2(pack2(pa[0], pa[1]), pack2(pa[2], pa[3]));
    };
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (; i + stride < n4; i += 2 * stride) {
        const int64_t j = i + stride;
        const float4 g0 = ((const float4*)grad)[i], g1 = ((const float4*)grad)[j];
        if (!skip) {
            const float4 p0 = ((const float4*)master)[i], p1 = ((const float4*)master)[j];
            const float4 m0 = ((const float4*)m)[i], m1 = ((const float4*)m)[j];
            const float4 v0 = ((const float4*)v)[i], v1 = ((const float4*)v)[j];
            update(g0, p0, m0, v0, i);
            update(g1, p1, m1, v1, j);
        }
        if (zero_grad) {
            ((float4*)grad)[i] = z4;
            ((float4*)grad)[j] = z4;
        }
    }
    for (; i < n4; i += stride) {
        const float4 g = ((const float4*)grad)[i];
        if (!skip) update(g, ((const float4*)master)[i], ((const float4*)m)[i], ((const float4*)v)[i], i);
        if (zero_grad) ((float4*)grad)[i] = z4;
    }
    // tail (n % 4)
    for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        if (!skip) {
            const float gg = grad[i] * gscale;
            m[i] = b1 * m[i] + (1.f - b1) * gg;
            v[i] = b2 * v[i] + (1.f - b2) * gg * gg;
            float p = master[i] * (1.f - lr * wd);
            p -= step_size * m[i] / (sqrtf(v[i]) * inv_sqrt_bc2 + eps);
            master[i] = p;
            if (out) out[i] = f2bf(p);
        }
        if (zero_grad) grad[i] = 0.f;
    }
}

TDL_API int tdl_adamw_flat(float* master, float* m, float* v, float* grad, void* out_bf16, int64_t n, float lr, float b1,
                           float b2, float eps, float wd, float bc1, float bc2, const float* ctrl, int zero_grad,
                           hipStream_t s) {
    const int64_t work = (n / 4 + 255) / 256;
    const int grid = (int)(work < 2048 ? (work > 0 ? work : 1) : 2048);
    adamw_flat_kernel<<<grid, 256, 0, s>>>(master, m, v, grad, (bf16_t*)out_bf16, n, lr, b1, b2, eps, wd, bc1, bc2, ctrl,
                                           zero_grad);
    TDL_LAUNCH_CHECK();
}

__global__ void fill_f32_kernel(float* __restrict__ p, int64_t n, float val) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = val;
}

TDL_API int tdl_fill_f32(float* p, int64_t n, float val, hipStream_t s) {
    const int64_t work = (n + 255) / 256;
    fill_f32_kernel<<<(int)(work < 4096 ? (work > 0 ? work : 1) : 4096), 256, 0, s>>>(p, n, val);
    TDL_LAUNCH_CHECK();
}

// dst = src (nbytes) when *flag > 0, else nothing: one launch whose workgroups read the device flag
// and leave at once when it is zero (the auditor's verified optimizer state replaces a stage's
// tampered one without a host read of the verdict; parallel/audit.py _heal_from_mirror).
__global__ __launch_bounds__(256) void copy_if_kernel(const float* __restrict__ flag, const uint4* __restrict__ src,
                                                      uint4* __restrict__ dst, int64_t n16,
                                                      const unsigned char* __restrict__ src_tail,
                                                      unsigned char* __restrict__ dst_tail, int tail) {
    if (!(flag[0] > 0.f)) return;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && threadIdx.x < tail) dst_tail[threadIdx.x] = src_tail[threadIdx.x];
}

TDL_API int tdl_copy_if(const float* flag, const void* src, void* dst, int64_t nbytes, hipStream_t s) {
    if (((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return (int)hipErrorInvalidValue;
    const int64_t n16 = nbytes / 16;
    const int tail = (int)(nbytes - n16 * 16);
    const int64_t work = (n16 + 255) / 256;
    const int grid = (int)(work < 2048 ? (work > 0 ? work : 1) : 2048);
    copy_if_kernel<<<grid, 256, 0, s>>>(flag, (const uint4*)src, (uint4*)dst, n16,
                                        (const unsigned char*)src + n16 * 16, (unsigned char*)dst + n16 * 16, tail);
    TDL_LAUNCH_CHECK();
}

// acc[i] += sum_s part[s * n + i]  — the reduction of a split-K weight-gradient GEMM whose S partial
// products were written (fp32) by one batched GEMM; one streaming pass, float4-vectorised.
__global__ __launch_bounds__(256) void splitk_reduce_add_kernel(float* __restrict__ acc, const float* __restrict__ part,
                                                                int S, int64_t n4) {
    const float4* p4 = (const float4*)part;
    float4* a4 = (float4*)acc;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        float4 a = a4[i];
        for (int s = 0; s < S; ++s) {
            const float4 v = p4[(int64_t)s * n4 + i];
            a.x += v.x;
            a.y += v.y;
            a.z += v.z;
            a.w += v.w;
        }
        a4[i] = a;
    }
}

TDL_API int tdl_splitk_reduce_add(float* acc, const float* part, int S, int64_t n, hipStream_t s) {
    if (n % 4 != 0 || ((uintptr_t)acc & 15) || ((uintptr_t)part & 15)) return (int)hipErrorInvalidValue;
    const int64_t n4 = n / 4;
    int64_t g = (n4 + 255) / 256;
    if (g > 4096) g = 4096;
    splitk_reduce_add_kernel<<<(int)(g > 0 ? g : 1), 256, 0, s>>>(acc, part, S, n4);
    TDL_LAUNCH_CHECK();
}
