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

// Backward sums: one [2C] row (sum dv | sum dv * xhat) per BN, zeroed by the forward, completed in a
// fixed order by the last workgroup of a reduction (bn_partial_fold_kernel here, or the data-gradient
// convolution's statistics finalize, conv.hip), which also adds them into dbeta / dgamma: the dx
// pass reads the row directly (the former replicated rows needed a separate fold launch per BN).
// Backward reduction: each row-chunk workgroup STORES its per-channel partial sums into its own
// row of a [NB_MAX][2C] block (no atomics: the former per-block fp32 atomics into the replicas were
// ~25 us per million on MI355X and dominated the pass for C >= 512, scripts/bench_bn.py), then
// bn_partial_fold_kernel sums the rows in FOLD_G row groups (FOLD_G x 2C atomics in total).
constexpr int NB_MAX = 1024;
constexpr int FOLD_G = 16;

// ---------------------------------------------------------------- forward
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ stats,
                                                         const float* __restrict__ run_mean, const float* __restrict__ run_var,
                                                         const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                                         const bf16_t* __restrict__ res, bf16_t* __restrict__ out,
                                                         float* __restrict__ save_mean, float* __restrict__ save_rstd,
                                                         float* __restrict__ upd_mean, float* __restrict__ upd_var,
                                                         float* __restrict__ zero_buf, int64_t zero_n,
                                                         int64_t M, int C, float eps, float momentum, int relu) {
    const int CV = C >> 3;
    const bool train = stats != nullptr;
    // zero the backward's replicated reduction buffer here (saves a memset launch per BN layer)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < zero_n; i += (int64_t)gridDim.x * blockDim.x)
        zero_buf[i] = 0.f;
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
    if ((blockDim.x % CV) == 0) {
        // every thread of the grid-stride loop keeps the same 8 channels: fold BN into one
        // per-channel scale/shift computed once (the per-element rsqrt made this pass ALU-bound)
        const int64_t v0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        const int c0 = (int)(v0 % CV) * 8;
        // first activation (and residual) vector in flight before the per-channel fold below: most
        // threads handle one or two vectors, so the fold's own loads would otherwise serialise
        // with them (one more HBM round trip per thread)
        uint4 xq = make_uint4(0, 0, 0, 0), rq = make_uint4(0, 0, 0, 0);
        if (v0 < nvec) {
            xq = ((const uint4*)x)[v0];
            if (res) rq = ((const uint4*)res)[v0];
        }
        float sc[8], sh[8];
        {
            float g[8], b[8];
            unpack8(*(const uint4*)(gamma + c0), g);
            unpack8(*(const uint4*)(beta + c0), b);
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
                sc[e] = rsqrtf(var + eps) * g[e];
                sh[e] = b[e] - mean * sc[e];
            }
        }
        for (int64_t v = v0; v < nvec; v += stride) {
            // next vector's loads issued before this one's math and store (software pipelining)
            uint4 xn = make_uint4(0, 0, 0, 0), rn = make_uint4(0, 0, 0, 0);
            if (v + stride < nvec) {
                xn = ((const uint4*)x)[v + stride];
                if (res) rn = ((const uint4*)res)[v + stride];
            }
            float xv[8];
            unpack8(xq, xv);
            if (res) {
                float rv[8];
                unpack8(rq, rv);
#pragma unroll
                for (int e = 0; e < 8; ++e) xv[e] = fmaf(xv[e], sc[e], sh[e]) + rv[e];
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) xv[e] = fmaf(xv[e], sc[e], sh[e]);
            }
            if (relu) {
#pragma unroll
                for (int e = 0; e < 8; ++e) xv[e] = fmaxf(xv[e], 0.f);
            }
            ((uint4*)out)[v] = pack8(xv);
            xq = xn;
            rq = rn;
        }
        return;
    }
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
// ReLU mask: from the stored output (out), or — for a BN whose output was never materialised (its
// apply + ReLU folded into the next convolution's operand load) — recomputed from x with the same
// per-channel scale / shift the convolution used (pro = [scale | shift]).
__global__ __launch_bounds__(256) void bn_act_bwd_reduce_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ out,
                                                                const bf16_t* __restrict__ x, const float* __restrict__ mean,
                                                                const float* __restrict__ rstd, float* __restrict__ part,
                                                                int64_t M, int C, int rows_per_block, int relu,
                                                                const float* __restrict__ pro,
                                                                unsigned* __restrict__ fold_cnt) {
    __shared__ float red[2][256][8];
    // the fold (next launch on the stream) counts its arrivals here: zero the counters
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < (2 * C + 255) / 256) fold_cnt[threadIdx.x] = 0u;
    const int CV = C >> 3;
    const int VPB = CV < 256 ? CV : 256;
    const int RPB = 256 / VPB;
    const int t = threadIdx.x;
    const int cvl = t % VPB, r0 = t / VPB;
    const int cv = blockIdx.y * VPB + cvl;
    float sg[8] = {}, sgx[8] = {};
    if (r0 < RPB && cv < CV) {
        const int c0 = cv * 8;
        float mu[8], rs[8], psc[8], psh[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            mu[e] = mean[c0 + e];
            rs[e] = rstd[c0 + e];
            psc[e] = pro ? pro[c0 + e] : 0.f;
            psh[e] = pro ? pro[C + c0 + e] : 0.f;
        }
        const int64_t rbeg = (int64_t)blockIdx.x * rows_per_block;
        const int64_t rend = rbeg + rows_per_block < M ? rbeg + rows_per_block : M;
        // 4 rows per iteration: 12 independent 16-byte loads in flight per thread (the loop is
        // a pure HBM stream; one row at a time left it latency-bound at ~half the bandwidth)
        constexpr int U = 4;
        for (int64_t r = rbeg + r0; r < rend; r += U * RPB) {
            uint4 dq[U], xq[U], oq[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t rr = r + (int64_t)u * RPB;
                const bool ok = rr < rend;
                const int64_t v = (ok ? rr : r) * CV + cv;
                dq[u] = ok ? ((const uint4*)dout)[v] : make_uint4(0, 0, 0, 0);
                xq[u] = ((const uint4*)x)[v];
                oq[u] = (relu && out) ? ((const uint4*)out)[v] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float dv[8], xv[8];
                unpack8(dq[u], dv);
                unpack8(xq[u], xv);
                if (relu && out) {
                    float ov[8];
                    unpack8(oq[u], ov);
#pragma unroll
                    for (int e = 0; e < 8; ++e) dv[e] = ov[e] > 0.f ? dv[e] : 0.f;
                } else if (relu) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) dv[e] = fmaf(xv[e], psc[e], psh[e]) > 0.f ? dv[e] : 0.f;
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    sg[e] += dv[e];
                    sgx[e] += dv[e] * (xv[e] - mu[e]) * rs[e];
                }
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
        float* row = part + (size_t)blockIdx.x * 2 * C;
        *(float4*)(row + cv * 8) = make_float4(sg[0], sg[1], sg[2], sg[3]);
        *(float4*)(row + cv * 8 + 4) = make_float4(sg[4], sg[5], sg[6], sg[7]);
        *(float4*)(row + C + cv * 8) = make_float4(sgx[0], sgx[1], sgx[2], sgx[3]);
        *(float4*)(row + C + cv * 8 + 4) = make_float4(sgx[4], sgx[5], sgx[6], sgx[7]);
    }
}

// Sum of the nb partial rows -> replica 0 (zeroed by the forward), in a FIXED order (the recompute
// audit evaluates a stage twice and compares; see conv.hip stats_finalize_kernel): grid (2C / 256,
// FOLD_G), each thread one column over the rows r = y (mod FOLD_G) of its group (coalesced across
// the wave, 4 loads in flight), the group total stored in row y (read by this group only); the LAST
// group of the column block to arrive (agent-scope counter; hand-off by drained sc1 stores + barrier + one relaxed add, sc1 loads on the reading side: conv.hip stats_arrive) adds the FOLD_G
// totals in group order.  cnt: zeroed by bn_act_bwd_reduce_kernel.
__global__ __launch_bounds__(256) void bn_partial_fold_kernel(float* __restrict__ sums, float* __restrict__ partials,
                                                              int nb, int C, unsigned* __restrict__ cnt,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta) {
    __shared__ int is_last;
    const int col = blockIdx.x * blockDim.x + threadIdx.x;
    float* part = partials + col;
    if (col < 2 * C) {
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int r = blockIdx.y;
        for (; r + 3 * FOLD_G < nb; r += 4 * FOLD_G) {
            a0 += part[(size_t)r * 2 * C];
            a1 += part[(size_t)(r + FOLD_G) * 2 * C];
            a2 += part[(size_t)(r + 2 * FOLD_G) * 2 * C];
            a3 += part[(size_t)(r + 3 * FOLD_G) * 2 * C];
        }
        for (; r < nb; r += FOLD_G) a0 += part[(size_t)r * 2 * C];
        // row y < FOLD_G <= NB_MAX; agent-scope (sc1, write-through) store: see stats_finalize_kernel
        __hip_atomic_store(part + (size_t)blockIdx.y * 2 * C, (a0 + a1) + (a2 + a3), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    // every storing wave drains its stores (workgroup-scope release: s_waitcnt), then one lane counts in
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's sc1 stores have landed
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = prev == FOLD_G - 1;
    }
    __syncthreads();
    if (!is_last || col >= 2 * C) return;
    float a = 0.f;
#pragma unroll
    for (int g = 0; g < FOLD_G; ++g)
        a += __hip_atomic_load(part + (size_t)g * 2 * C, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float tot = sums[col] + a;
    sums[col] = tot;
    if (dgamma != nullptr) {
        if (col < C) dbeta[col] += tot;
        else dgamma[col - C] += tot;
    }
}

// ---------------------------------------------------------------- backward pass 2: elementwise
__global__ __launch_bounds__(256) void bn_act_bwd_dx_kernel(const bf16_t* __restrict__ dout, const bf16_t* __restrict__ out,
                                                            const bf16_t* __restrict__ x, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, const bf16_t* __restrict__ gamma,
                                                            const float* __restrict__ sums, bf16_t* __restrict__ dx,
                                                            bf16_t* __restrict__ dres, int64_t M, int C, int relu,
                                                            const float* __restrict__ pro) {
    const int CV = C >> 3;
    const float invM = 1.f / (float)M;
    const int64_t nvec = M * CV;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * blockDim.x) {
        const int c0 = (int)(v % CV) * 8;
        float dv[8], xv[8], g[8];
        unpack8(((const uint4*)dout)[v], dv);
        unpack8(((const uint4*)x)[v], xv);
        unpack8(*(const uint4*)(gamma + c0), g);
        if (relu && out) {
            float ov[8];
            unpack8(((const uint4*)out)[v], ov);
#pragma unroll
            for (int e = 0; e < 8; ++e) dv[e] = ov[e] > 0.f ? dv[e] : 0.f;
        } else if (relu) {
#pragma unroll
            for (int e = 0; e < 8; ++e) dv[e] = fmaf(xv[e], pro[c0 + e], pro[C + c0 + e]) > 0.f ? dv[e] : 0.f;
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

// Training statistics of a BN whose apply + ReLU is folded into the next convolution: mean / rstd
// (saved for backward), running-statistics update, the per-channel fold pro = [gamma * rstd |
// beta - mean * gamma * rstd] (fp32), and the zeroed backward reduction buffer — no pass over the
// activations at all.
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ stats, const bf16_t* __restrict__ gamma,
                                                          const bf16_t* __restrict__ beta, float* __restrict__ save_mean,
                                                          float* __restrict__ save_rstd, float* __restrict__ upd_mean,
                                                          float* __restrict__ upd_var, float* __restrict__ pro,
                                                          float* __restrict__ zero_buf, int64_t zero_n, int64_t M, int C,
                                                          float eps, float momentum) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < zero_n; i += (int64_t)gridDim.x * blockDim.x)
        zero_buf[i] = 0.f;
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float invM = 1.f / (float)M;
    const float mean = stats[c] * invM;
    const float var = fmaxf(stats[C + c] * invM - mean * mean, 0.f);
    const float rs = rsqrtf(var + eps);
    save_mean[c] = mean;
    save_rstd[c] = rs;
    if (upd_mean) {
        const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
        upd_mean[c] = (1.f - momentum) * upd_mean[c] + momentum * mean;
        upd_var[c] = (1.f - momentum) * upd_var[c] + momentum * unbiased;
    }
    const float sc = rs * bf2f(gamma[c]);
    pro[c] = sc;
    pro[C + c] = bf2f(beta[c]) - mean * sc;
}

int grid_for(int64_t nvec) {
    int64_t g = (nvec + 255) / 256;
    if (g > 4096) g = 4096;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

// Floats of the backward-sums row for C channels (allocated with the forward, kept to the backward).
TDL_API int64_t tdl_bn_bwd_ws_floats(int C) { return (int64_t)2 * C; }
// Floats of the backward's per-block partial rows (scratch of ONE backward call, not kept).
// + the fold's arrival counters (one per 256-column block)
TDL_API int64_t tdl_bn_bwd_part_floats(int C) { return (int64_t)NB_MAX * 2 * C + (2 * C + 255) / 256; }

// stats: [2C] (sum, sumsq) in training mode, or null to normalise with run_mean/run_var (eval).
// save_mean/save_rstd: [C] or null.  upd_mean/upd_var: running buffers to update (train) or null.
// bwd_ws: tdl_bn_bwd_ws_floats(C) floats zeroed here for the later backward (or null).
TDL_API int tdl_bn_act_fwd(const void* x, const float* stats, const float* run_mean, const float* run_var,
                           const void* gamma, const void* beta, const void* res, void* out, float* save_mean,
                           float* save_rstd, float* upd_mean, float* upd_var, float* bwd_ws, int64_t M, int C,
                           float eps, float momentum, int relu, hipStream_t s) {
    if (C % 8 != 0) return (int)hipErrorInvalidValue;
    bn_act_fwd_kernel<<<grid_for(M * (C / 8)), 256, 0, s>>>(
        (const bf16_t*)x, stats, run_mean, run_var, (const bf16_t*)gamma, (const bf16_t*)beta, (const bf16_t*)res,
        (bf16_t*)out, save_mean, save_rstd, upd_mean, upd_var, bwd_ws, bwd_ws ? (int64_t)2 * C : 0, M, C, eps,
        momentum, relu);
    TDL_LAUNCH_CHECK();
}

// stats [2C] (sum, sumsq) -> save_mean / save_rstd [C], running stats (or null), pro [2C], and
// bwd_ws (tdl_bn_bwd_ws_floats(C)) zeroed for the backward.
TDL_API int tdl_bn_finalize(const float* stats, const void* gamma, const void* beta, float* save_mean, float* save_rstd,
                            float* upd_mean, float* upd_var, float* pro, float* bwd_ws, int64_t M, int C, float eps,
                            float momentum, hipStream_t s) {
    if (C % 8 != 0 || stats == nullptr || pro == nullptr || bwd_ws == nullptr) return (int)hipErrorInvalidValue;
    const int64_t zn = (int64_t)2 * C;
    int g = (int)((zn + 255) / 256);
    const int gc = (C + 255) / 256;
    if (g < gc) g = gc;
    bn_finalize_kernel<<<g, 256, 0, s>>>(stats, (const bf16_t*)gamma, (const bf16_t*)beta, save_mean, save_rstd,
                                         upd_mean, upd_var, pro, bwd_ws, zn, M, C, eps, momentum);
    TDL_LAUNCH_CHECK();
}

static int bn_act_bwd_impl(const void* dout, const void* out, const void* x, const float* mean, const float* rstd,
                           const void* gamma, float* sums, float* part, void* dx, void* dres, float* dgamma, float* dbeta,
                           int64_t M, int C, int relu, const float* pro, hipStream_t s) {
    if (C % 8 != 0 || (relu && out == nullptr && pro == nullptr) || part == nullptr) return (int)hipErrorInvalidValue;
    const int CV = C / 8;
    const int VPB = CV < 256 ? CV : 256;
    const int RPB = 256 / VPB;
    const int gy = (CV + VPB - 1) / VPB;
    // ~1024 workgroups in total (4 per CU, each thread >= one 4-row unrolled iteration: 12 loads
    // in flight), at most NB_MAX row chunks (the partial rows of the workspace)
    int64_t rows_per_block = (M * gy + 1023) / 1024;
    if (rows_per_block < 4 * RPB) rows_per_block = 4 * RPB;
    if (rows_per_block < (M + NB_MAX - 1) / NB_MAX) rows_per_block = (M + NB_MAX - 1) / NB_MAX;
    rows_per_block = (rows_per_block + RPB - 1) / RPB * RPB;
    const int nb = (int)((M + rows_per_block - 1) / rows_per_block);
    const dim3 grid((unsigned)nb, gy);
    bn_act_bwd_reduce_kernel<<<grid, 256, 0, s>>>((const bf16_t*)dout, (const bf16_t*)out, (const bf16_t*)x, mean, rstd,
                                                  part, M, C, (int)rows_per_block, relu, pro,
                                                  (unsigned*)(part + (size_t)NB_MAX * 2 * C));
    bn_partial_fold_kernel<<<dim3((2 * C + 255) / 256, FOLD_G), 256, 0, s>>>(
        sums, part, nb, C, (unsigned*)(part + (size_t)NB_MAX * 2 * C), dgamma, dbeta);
    bn_act_bwd_dx_kernel<<<grid_for(M * CV), 256, 0, s>>>(
        (const bf16_t*)dout, (const bf16_t*)out, (const bf16_t*)x, mean, rstd, (const bf16_t*)gamma,
        sums, (bf16_t*)dx, (bf16_t*)dres, M, C, relu, pro);
    TDL_LAUNCH_CHECK();
}

// sums: the forward's bwd_ws (zeroed there); part: tdl_bn_bwd_part_floats(C) floats of scratch.
// dgamma/dbeta: fp32 accumulators (+=) or null.
TDL_API int tdl_bn_act_bwd(const void* dout, const void* out, const void* x, const float* mean, const float* rstd,
                           const void* gamma, float* sums, float* part, void* dx, void* dres, float* dgamma, float* dbeta,
                           int64_t M, int C, int relu, hipStream_t s) {
    return bn_act_bwd_impl(dout, out, x, mean, rstd, gamma, sums, part, dx, dres, dgamma, dbeta, M, C, relu, nullptr, s);
}

// Backward of a folded BN (+ ReLU) whose two per-channel sums were already reduced (and added into
// dbeta / dgamma) by the producing data-gradient convolution (tdl_conv_dgrad_bnsums): the
// elementwise pass only.
TDL_API int tdl_bn_act_bwd_pro_summed(const void* dout, const void* x, const float* mean, const float* rstd,
                                      const void* gamma, const float* pro, const float* sums, void* dx, int64_t M, int C,
                                      hipStream_t s) {
    if (C % 8 != 0 || pro == nullptr) return (int)hipErrorInvalidValue;
    bn_act_bwd_dx_kernel<<<grid_for(M * (C / 8)), 256, 0, s>>>(
        (const bf16_t*)dout, nullptr, (const bf16_t*)x, mean, rstd, (const bf16_t*)gamma, sums,
        (bf16_t*)dx, nullptr, M, C, 1, pro);
    TDL_LAUNCH_CHECK();
}

// Backward of a folded BN (+ ReLU): no stored output, the mask is recomputed from x with pro.
TDL_API int tdl_bn_act_bwd_pro(const void* dout, const void* x, const float* mean, const float* rstd, const void* gamma,
                               const float* pro, float* sums, float* part, void* dx, float* dgamma, float* dbeta, int64_t M,
                               int C, int relu, hipStream_t s) {
    return bn_act_bwd_impl(dout, nullptr, x, mean, rstd, gamma, sums, part, dx, nullptr, dgamma, dbeta, M, C, relu, pro, s);
}
