// NHWC bf16 max-pooling (ResNet stem 3x3 / stride 2 / pad 1, VGG 2x2 / stride 2) with the window
// argmax kept as one byte per output element, so the backward is a deterministic gather (no atomics,
// no second pass over the input).  Replaces torch's max_pool2d_with_indices kernels on the native
// conv path (ops/conv.py), SURVEY 2.8 K13 (conv stages of the ImageNet ResNets / VGG).
//
// Each thread owns 8 consecutive channels of one pixel (16-byte loads / stores; C % 8 == 0).
// Ties keep the first window position in row-major order, NaN wins (torch semantics).
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C, int P,
                                                          int Q, int R, int S, int stride, int pad) {
    const int C8 = C / 8;
    const int64_t total = (int64_t)N * P * Q * C8;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int c8 = (int)(t % C8);
        int64_t pix = t / C8;
        const int q = (int)(pix % Q);
        pix /= Q;
        const int p = (int)(pix % P);
        const int n = (int)(pix / P);
        float m[8];
        uint8_t a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) m[k] = -INFINITY, a[k] = 0;
        for (int r = 0; r < R; ++r) {
            const int h = p * stride - pad + r;
            if (h < 0 || h >= H) continue;
            for (int s = 0; s < S; ++s) {
                const int w = q * stride - pad + s;
                if (w < 0 || w >= W) continue;
                float v[8];
                unpack8(*(const uint4*)(x + (((size_t)n * H + h) * W + w) * C + 8 * c8), v);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    if (v[k] > m[k] || (v[k] != v[k] && m[k] == m[k])) {
                        m[k] = v[k];
                        a[k] = (uint8_t)(r * S + s);
                    }
                }
            }
        }
        const size_t o = (((size_t)n * P + p) * Q + q) * C + 8 * c8;
        *(uint4*)(y + o) = pack8(m);
        uint2 packed;
        packed.x = a[0] | (a[1] << 8) | (a[2] << 16) | ((uint32_t)a[3] << 24);
        packed.y = a[4] | (a[5] << 8) | (a[6] << 16) | ((uint32_t)a[7] << 24);
        *(uint2*)(arg + o) = packed;
    }
}

// dx[n, h, w, c] = sum over the output windows (p, q) containing (h, w) whose argmax is (h, w)
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                          bf16_t* __restrict__ dx, int N, int H, int W, int C, int P,
                                                          int Q, int R, int S, int stride, int pad) {
    const int C8 = C / 8;
    const int64_t total = (int64_t)N * H * W * C8;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int c8 = (int)(t % C8);
        int64_t pix = t / C8;
        const int w = (int)(pix % W);
        pix /= W;
        const int h = (int)(pix % H);
        const int n = (int)(pix / H);
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        // outputs p with p * stride - pad <= h <= p * stride - pad + R - 1
        const int p_lo = max(0, (h + pad - R + stride) / stride), p_hi = min(P - 1, (h + pad) / stride);
        const int q_lo = max(0, (w + pad - S + stride) / stride), q_hi = min(Q - 1, (w + pad) / stride);
        for (int p = p_lo; p <= p_hi; ++p) {
            const int r = h + pad - p * stride;
            if (r < 0 || r >= R) continue;
            for (int q = q_lo; q <= q_hi; ++q) {
                const int s = w + pad - q * stride;
                if (s < 0 || s >= S) continue;
                const uint8_t want = (uint8_t)(r * S + s);
                const size_t o = (((size_t)n * P + p) * Q + q) * C + 8 * c8;
                const uint2 ap = *(const uint2*)(arg + o);
                float g[8];
                unpack8(*(const uint4*)(dy + o), g);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint8_t ak = (uint8_t)(((k < 4 ? ap.x : ap.y) >> (8 * (k & 3))) & 0xff);
                    if (ak == want) acc[k] += g[k];
                }
            }
        }
        *(uint4*)(dx + (((size_t)n * H + h) * W + w) * C + 8 * c8) = pack8(acc);
    }
}

// Global average pool (the ResNet / VGG classifier head): out[n][c] = mean over H*W of x[n][h][w][c].
__global__ __launch_bounds__(256) void gap_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N, int HW,
                                                      int C) {
    const int C8 = C / 8;
    const int64_t total = (int64_t)N * C8;
    const float inv = 1.f / (float)HW;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int c8 = (int)(t % C8), n = (int)(t / C8);
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const bf16_t* p = x + (size_t)n * HW * C + 8 * c8;
        for (int i = 0; i < HW; ++i) {
            float v[8];
            unpack8(*(const uint4*)(p + (size_t)i * C), v);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += v[k];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] *= inv;
        *(uint4*)(y + (size_t)n * C + 8 * c8) = pack8(acc);
    }
}

__global__ __launch_bounds__(256) void gap_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int N, int HW,
                                                      int C) {
    const int C8 = C / 8;
    const int64_t total = (int64_t)N * HW * C8;
    const float inv = 1.f / (float)HW;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int c8 = (int)(t % C8);
        const int n = (int)(t / ((int64_t)C8 * HW));
        float g[8];
        unpack8(*(const uint4*)(dy + (size_t)n * C + 8 * c8), g);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] *= inv;
        *(uint4*)(dx + (size_t)t * 8) = pack8(g);
    }
}

int grid_for(int64_t work) {
    const int64_t g = (work + 255) / 256;
    return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

}  // namespace

TDL_API int tdl_maxpool_fwd(const void* x, void* y, uint8_t* arg, int N, int H, int W, int C, int P, int Q, int R, int S,
                            int stride, int pad, hipStream_t s) {
    if (C % 8 || R * S > 255 || R <= 0 || S <= 0 || stride <= 0) return (int)hipErrorInvalidValue;
    maxpool_fwd_kernel<<<grid_for((int64_t)N * P * Q * (C / 8)), 256, 0, s>>>((const bf16_t*)x, (bf16_t*)y, arg, N, H, W,
                                                                              C, P, Q, R, S, stride, pad);
    TDL_LAUNCH_CHECK();
}

TDL_API int tdl_maxpool_bwd(const void* dy, const uint8_t* arg, void* dx, int N, int H, int W, int C, int P, int Q, int R,
                            int S, int stride, int pad, hipStream_t s) {
    if (C % 8 || R * S > 255 || R <= 0 || S <= 0 || stride <= 0) return (int)hipErrorInvalidValue;
    maxpool_bwd_kernel<<<grid_for((int64_t)N * H * W * (C / 8)), 256, 0, s>>>((const bf16_t*)dy, arg, (bf16_t*)dx, N, H,
                                                                              W, C, P, Q, R, S, stride, pad);
    TDL_LAUNCH_CHECK();
}

TDL_API int tdl_global_avgpool_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t s) {
    if (C % 8 || HW <= 0) return (int)hipErrorInvalidValue;
    gap_fwd_kernel<<<grid_for((int64_t)N * (C / 8)), 256, 0, s>>>((const bf16_t*)x, (bf16_t*)y, N, HW, C);
    TDL_LAUNCH_CHECK();
}

TDL_API int tdl_global_avgpool_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t s) {
    if (C % 8 || HW <= 0) return (int)hipErrorInvalidValue;
    gap_bwd_kernel<<<grid_for((int64_t)N * HW * (C / 8)), 256, 0, s>>>((const bf16_t*)dy, (bf16_t*)dx, N, HW, C);
    TDL_LAUNCH_CHECK();
}
