// BatchNorm (+ residual add) (+ ReLU) for NHWC bf16 activations — the pointwise half of the
// conv blocks whose GEMM half is csrc/conv.hip.  Training-mode batch statistics come from the
// conv epilogue (per-channel sum / sum of squares), so the forward is ONE streaming pass:
//     out = act(gamma * (x - mean) * rstd + beta (+ res))
// and block 0 also writes mean/rstd (saved for backward) and updates the running statistics.
// Backward is two passes: a per-channel reduction of g = dout * act'(out) and g * xhat (written
// straight into fp32 accumulators, also feeding dgamma / dbeta), then the elementwise
//     dx = gamma * rstd * (g - sum(g)/M - xhat * sum(g xhat)/M),   dres = g.
#include "common.h"

namespace {

// ---------------------------------------------------------------- forward
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ stats,
                                                         const float* __restrict__ run_mean, const float* __restrict__ run_var,
                                                         const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                                         const bf16_t* __restrict__ res, bf16_t* __restrict__ out,
                                                         float* __restrict__ save_mean, float* __restrict__ save_rstd,
                                                         float* __restrict__ upd_mean, float* __restrict__ upd_var,
                                                         int64_t M, int C, float eps, float momentum, int relu) {
    const int CV = C >> 3;
    const bool train = stats != nullptr;
    const float invM = 1.f / (float)M;
    if (blockIdx.x == 0) {
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            float mean, var;
            if (train) {
                mean = stats[c] * invM;
                var = fmaxf(stats[C + c] * invM - mean * mean, 0.f);
            } else {
                mean = run_mean[c];
                var = run_var[c];
            }
            if (save_mean) {
                save_mean[c] = mean;
                save_rstd[c] = rsqrtf(var + eps);
            }
            if (train && upd_mean) {
                const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
                upd_mean[c] = (1.f - momentum) * upd_mean[c] + momentum * mean;
                upd_var[c] = (1.f - momentum) * upd_var[c] + momentum * unbiased;
            }
        }
    }
    const int64_t nvec = M * CV;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
        const int c0 = (int)(v % CV) * 8;
        float xv[8], g[8], b[8], rv[8];
        unpack8(((const uint4*)x)[v], xv);
        unpack8(*(const uint4*)(gamma + c0), g);
        unpack8(*(const uint4*)(beta + c0), b);
        if (res) unpack8(((const uint4*)res)[v], rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int c = c0 + e;
            float mean, var;
            if (train) {
                mean = stats[c] * invM;
                var = fmaxf(stats[C + c] * invM - mean * mean, 0.f);
            } else {
                mean = run_mean[c];
                var = run_var[c];
            }
            float y = (xv[e] - mean) * rsqrtf(var + eps) * g[e] + b[e];
            if (res) y += rv[e];
            xv[e] = relu ? fmaxf(y, 0.f) : y;
        }
        ((uint4*)out)[v] = pack8(xv);
    }
}

// ---------------------------------------------------------------- backward pass 1: reductions
// block = 256 threads = RPB rows x VPB channel-vectors; grid (row chunks, channel-vector groups)
__global__ __launch_bounds__(256) void bn_act_bwd_reduce_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ out,
                                                                const bf16_t* __restrict__ x, const float* __restrict__ mean,
                                                                const float* __restrict__ rstd, float* __restrict__ sums,
                                                                int64_t M, int C, int rows_per_block, int relu) {
    __shared__ float red[2][256][8];
    const int CV = C >> 3;
    const int VPB = CV < 256 ? CV : 256;
    const int RPB = 256 / VPB;
    const int t = threadIdx.x;
    const int cvl = t % VPB, r0 = t / VPB;
    const int cv = blockIdx.y * VPB + cvl;
    float sg[8] = {}, sgx[8] = {};
    if (r0 < RPB && cv < CV) {
        const int c0 = cv * 8;
        float mu[8], rs[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            mu[e] = mean[c0 + e];
            rs[e] = rstd[c0 + e];
        }
        const int64_t rbeg = (int64_t)blockIdx.x * rows_per_block;
        const int64_t rend = rbeg + rows_per_block < M ? rbeg + rows_per_block : M;
        for (int64_t r = rbeg + r0; r < rend; r += RPB) {
            const int64_t v = r * CV + cv;
            float dv[8], xv[8];
            unpack8(((const uint4*)dout)[v], dv);
            unpack8(((const uint4*)x)[v], xv);
            if (relu) {
                float ov[8];
                unpack8(((const uint4*)out)[v], ov);
#pragma unroll
                for (int e = 0; e < 8; ++e) dv[e] = ov[e] > 0.f ? dv[e] : 0.f;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                sg[e] += dv[e];
                sgx[e] += dv[e] * (xv[e] - mu[e]) * rs[e];
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        red[0][t][e] = sg[e];
        red[1][t][e] = sgx[e];
    }
    __syncthreads();
    if (r0 == 0 && cv < CV) {
        for (int k = 1; k < RPB; ++k) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                sg[e] += red[0][k * VPB + cvl][e];
                sgx[e] += red[1][k * VPB + cvl][e];
            }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            atomicAdd(sums + cv * 8 + e, sg[e]);
            atomicAdd(sums + C + cv * 8 + e, sgx[e]);
        }
    }
}

// ---------------------------------------------------------------- backward pass 2: elementwise
__global__ __launch_bounds__(256) void bn_act_bwd_dx_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ out,
                                                            const bf16_t* __restrict__ x, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, const bf16_t* __restrict__ gamma,
                                                            const float* __restrict__ sums, bf16_t* __restrict__ dx,
                                                            bf16_t* __restrict__ dres, float* __restrict__ dgamma,
                                                            float* __restrict__ dbeta, int64_t M, int C, int relu) {
    const int CV = C >> 3;
    const float invM = 1.f / (float)M;
    if (blockIdx.x == 0 && dgamma) {
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            dgamma[c] += sums[C + c];
            dbeta[c] += sums[c];
        }
    }
    const int64_t nvec = M * CV;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
        const int c0 = (int)(v % CV) * 8;
        float dv[8], xv[8], g[8];
        unpack8(((const uint4*)dout)[v], dv);
        unpack8(((const uint4*)x)[v], xv);
        unpack8(*(const uint4*)(gamma + c0), g);
        if (relu) {
            float ov[8];
            unpack8(((const uint4*)out)[v], ov);
#pragma unroll
            for (int e = 0; e < 8; ++e) dv[e] = ov[e] > 0.f ? dv[e] : 0.f;
        }
        if (dres) ((uint4*)dres)[v] = pack8(dv);
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int c = c0 + e;
            const float rs = rstd[c];
            const float xh = (xv[e] - mean[c]) * rs;
            o[e] = g[e] * rs * (dv[e] - sums[c] * invM - xh * sums[C + c] * invM);
        }
        ((uint4*)dx)[v] = pack8(o);
    }
}

int grid_for(int64_t nvec) {
    int64_t g = (nvec + 255) / 256;
    if (g > 4096) g = 4096;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

// stats: [2C] (sum, sumsq) in training mode, or null to normalise with run_mean/run_var (eval).
// save_mean/save_rstd: [C] or null.  upd_mean/upd_var: running buffers to update (train) or null.
TDL_API int tdl_bn_act_fwd(const void* x, const float* stats, const float* run_mean, const float* run_var,
                           const void* gamma, const void* beta, const void* res, void* out, float* save_mean,
                           float* save_rstd, float* upd_mean, float* upd_var, int64_t M, int C, float eps,
                           float momentum, int relu, hipStream_t s) {
    if (C % 8 != 0) return (int)hipErrorInvalidValue;
    bn_act_fwd_kernel<<<grid_for(M * (C / 8)), 256, 0, s>>>(
        (const bf16_t*)x, stats, run_mean, run_var, (const bf16_t*)gamma, (const bf16_t*)beta, (const bf16_t*)res,
        (bf16_t*)out, save_mean, save_rstd, upd_mean, upd_var, M, C, eps, momentum, relu);
    TDL_LAUNCH_CHECK();
}

// sums: scratch [2C] (zeroed here).  dgamma/dbeta: fp32 accumulators (+=) or null.
TDL_API int tdl_bn_act_bwd(const void* dout, const void* out, const void* x, const float* mean, const float* rstd,
                           const void* gamma, float* sums, void* dx, void* dres, float* dgamma, float* dbeta, int64_t M,
                           int C, int relu, hipStream_t s) {
    if (C % 8 != 0) return (int)hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(sums, 0, sizeof(float) * 2 * C, s);
    if (e != hipSuccess) return (int)e;
    const int CV = C / 8;
    const int VPB = CV < 256 ? CV : 256;
    const int RPB = 256 / VPB;
    const int gy = (CV + VPB - 1) / VPB;
    // ~4 waves of row work per CU across the grid, each block >= 8 row passes
    int64_t rows_per_block = (M * gy + 1023) / 1024;
    if (rows_per_block < 8 * RPB) rows_per_block = 8 * RPB;
    rows_per_block = (rows_per_block + RPB - 1) / RPB * RPB;
    const dim3 grid((unsigned)((M + rows_per_block - 1) / rows_per_block), gy);
    bn_act_bwd_reduce_kernel<<<grid, 256, 0, s>>>((const bf16_t*)dout, (const bf16_t*)out, (const bf16_t*)x, mean, rstd,
                                                  sums, M, C, (int)rows_per_block, relu);
    bn_act_bwd_dx_kernel<<<grid_for(M * CV), 256, 0, s>>>((const bf16_t*)dout, (const bf16_t*)out, (const bf16_t*)x, mean,
                                                          rstd, (const bf16_t*)gamma, sums, (bf16_t*)dx, (bf16_t*)dres,
                                                          dgamma, dbeta, M, C, relu);
    TDL_LAUNCH_CHECK();
}
