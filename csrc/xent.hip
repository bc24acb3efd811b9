// Softmax cross-entropy over LM-head logits (replaces the
// CrossEntropyLoss of distributed_trainer.py:435-439, applied to real logits).
//
// Logits are bf16 [M, ld] with ld >= V (vocab padded to a multiple of 64 so every row is
// 16-byte aligned); columns >= V are padding and are masked out.  One 256-thread block per
// row, online (max, sum-exp) per thread, a single block merge.  The backward recomputes
// softmax from the saved log-sum-exp and writes dlogits in place (the logits buffer is dead
// after the loss), scaled by a DEVICE scalar (grad_output / n_valid) so no host sync is needed.
#include "common.h"
#include <cstdlib>

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
    const float mn = fmaxf(m, m2);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mn));
    m = mn;
}

__global__ __launch_bounds__(256) void xent_fwd_kernel(const bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss, float* __restrict__ lse_out, int V, int ld,
                                                       int ignore_index) {
    __shared__ float red_m[4], red_s[4];
    const int row = blockIdx.x;
    const bf16_t* lr = logits + (size_t)row * ld;
    float m = -INFINITY, s = 0.f;
    const int nvec = V / 8;
    for (int i = threadIdx.x; i < nvec; i += 256) {
        float v[8];
        unpack8(((const uint4*)lr)[i], v);
        float vm = v[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) vm = fmaxf(vm, v[k]);
        float vs = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) vs += __expf(v[k] - vm);
        online_merge(m, s, vm, vs);
    }
    for (int j = nvec * 8 + threadIdx.x; j < V; j += 256) online_merge(m, s, bf2f(lr[j]), 1.f);
    // wave merge
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
        online_merge(m, s, m2, s2);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red_m[wid] = m;
        red_s[wid] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float M0 = red_m[0], S0 = red_s[0];
        for (int w = 1; w < 4; ++w) online_merge(M0, S0, red_m[w], red_s[w]);
        const float lse = M0 + __logf(S0);
        lse_out[row] = lse;
        const int64_t lab = labels[row];
        loss[row] = (lab == ignore_index || lab < 0 || lab >= V) ? 0.f : lse - bf2f(lr[lab]);
    }
}

TDL_API int tdl_xent_fwd(const void* logits, const int64_t* labels, float* loss, float* lse, int M, int V, int ld,
                         hipStream_t s) {
    xent_fwd_kernel<<<M, 256, 0, s>>>((const bf16_t*)logits, labels, loss, lse, V, ld, -100);
    TDL_LAUNCH_CHECK();
}

// dlogits[r, j] = (softmax_j - [j == label]) * scale  for j < V, 0 for padding columns.
__global__ __launch_bounds__(256) void xent_bwd_kernel(const bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse_in, const float* __restrict__ scale_ptr,
                                                       bf16_t* __restrict__ dlogits, int V, int ld, int ignore_index) {
    const int row = blockIdx.x;
    const int64_t lab = labels[row];
    const bool ign = (lab == ignore_index || lab < 0 || lab >= V);
    const float lse = lse_in[row];
    const float sc = ign ? 0.f : scale_ptr[0];
    const bf16_t* lr = logits + (size_t)row * ld;
    bf16_t* dr = dlogits + (size_t)row * ld;
    const int nvec = ld / 8;
    for (int i = threadIdx.x; i < nvec; i += 256) {
        float v[8];
        unpack8(((const uint4*)lr)[i], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = i * 8 + k;
            float p = j < V ? __expf(v[k] - lse) : 0.f;
            if (j == lab) p -= 1.f;
            v[k] = p * sc;
        }
        ((uint4*)dr)[i] = pack8(v);
    }
    for (int j = nvec * 8 + threadIdx.x; j < ld; j += 256) {
        float p = j < V ? __expf(bf2f(lr[j]) - lse) : 0.f;
        if (j == lab) p -= 1.f;
        dr[j] = f2bf(p * sc);
    }
}

TDL_API int tdl_xent_bwd(const void* logits, const int64_t* labels, const float* lse, const float* scale_ptr, void* dlogits,
                         int M, int V, int ld, float unused, hipStream_t s) {
    (void)unused;
    xent_bwd_kernel<<<M, 256, 0, s>>>((const bf16_t*)logits, labels, lse, scale_ptr, (bf16_t*)dlogits, V, ld, -100);
    TDL_LAUNCH_CHECK();
}

// Fused forward + backward over one logits row: pass 1 = online (max, sum-exp)
// and the label logit -> loss row, lse; pass 2 re-reads the row (just streamed, so mostly an L2 /
// MALL hit: a GPT-2 row is 100 KB) and overwrites it IN PLACE with
//   dlogits = (softmax - onehot) * scale     (scale = DEVICE scalar, e.g. 1 / n_valid),
// so the LM head's loss stage reads + writes the logits once instead of read / read / write with
// separate forward and backward kernels.
__global__ __launch_bounds__(256) void xent_fused_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                         float* __restrict__ loss, float* __restrict__ lse_out,
                                                         const float* __restrict__ scale_ptr, int V, int ld,
                                                         int ignore_index) {
    __shared__ float red_m[4], red_s[4], bcast[1];
    const int row = blockIdx.x;
    bf16_t* lr = logits + (size_t)row * ld;
    float m = -INFINITY, s = 0.f;
    const int nvec = V / 8;
    // four 16-B loads per lane in flight per trip (one at a time left each block latency-bound:
    // ~4.2 TB/s over the row's read / re-read / write)
    int i0 = threadIdx.x;
    for (; i0 + 3 * 256 < nvec; i0 += 4 * 256) {
        uint4 q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = ((const uint4*)lr)[i0 + u * 256];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float v[8];
            unpack8(q[u], v);
            float vm = v[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) vm = fmaxf(vm, v[k]);
            float vs = 0.f;
#pragma unroll
            for (int k = 0; k < 8; ++k) vs += __expf(v[k] - vm);
            online_merge(m, s, vm, vs);
        }
    }
    for (int i = i0; i < nvec; i += 256) {
        float v[8];
        unpack8(((const uint4*)lr)[i], v);
        float vm = v[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) vm = fmaxf(vm, v[k]);
        float vs = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) vs += __expf(v[k] - vm);
        online_merge(m, s, vm, vs);
    }
    for (int j = nvec * 8 + threadIdx.x; j < V; j += 256) online_merge(m, s, bf2f(lr[j]), 1.f);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
        online_merge(m, s, m2, s2);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red_m[wid] = m;
        red_s[wid] = s;
    }
    __syncthreads();
    const int64_t lab = labels[row];
    const bool ign = (lab == ignore_index || lab < 0 || lab >= V);
    if (threadIdx.x == 0) {
        float M0 = red_m[0], S0 = red_s[0];
        for (int w = 1; w < 4; ++w) online_merge(M0, S0, red_m[w], red_s[w]);
        const float lse = M0 + __logf(S0);
        lse_out[row] = lse;
        loss[row] = ign ? 0.f : lse - bf2f(lr[lab]);  // label logit read before any overwrite
        bcast[0] = lse;
    }
    __syncthreads();
    const float lse = bcast[0];
    const float sc = ign ? 0.f : scale_ptr[0];
    const int nv = ld / 8;
    auto dl8 = [&](const uint4& q, int i) -> uint4 {
        float v[8];
        unpack8(q, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = i * 8 + k;
            float p = j < V ? __expf(v[k] - lse) : 0.f;
            if (j == lab) p -= 1.f;
            v[k] = p * sc;
        }
        return pack8(v);
    };
    int i1 = threadIdx.x;
    for (; i1 + 3 * 256 < nv; i1 += 4 * 256) {
        uint4 q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = ((const uint4*)lr)[i1 + u * 256];
#pragma unroll
        for (int u = 0; u < 4; ++u) ((uint4*)lr)[i1 + u * 256] = dl8(q[u], i1 + u * 256);
    }
    for (int i = i1; i < nv; i += 256) {
        float v[8];
        unpack8(((const uint4*)lr)[i], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int j = i * 8 + k;
            float p = j < V ? __expf(v[k] - lse) : 0.f;
            if (j == lab) p -= 1.f;
            v[k] = p * sc;
        }
        ((uint4*)lr)[i] = pack8(v);
    }
    for (int j = nv * 8 + threadIdx.x; j < ld; j += 256) {
        float p = j < V ? __expf(bf2f(lr[j]) - lse) : 0.f;
        if (j == lab) p -= 1.f;
        lr[j] = f2bf(p * sc);
    }
}

// Opaque to the optimiser: the row stays live as packed bf16 (4 VGPRs per vector) and is unpacked
// again in each pass (two shifts per pair), instead of being kept as 8 unpacked floats per vector
// across passes (291 VGPRs, one wave per SIMD).
template <int NV>
__device__ __forceinline__ void keep_packed(uint4 (&q)[NV]) {
#pragma unroll
    for (int t = 0; t < NV; ++t) asm volatile("" : "+v"(q[t].x), "+v"(q[t].y), "+v"(q[t].z), "+v"(q[t].w));
}

// Register-resident variant: the block's 256 lanes hold the whole row (NV x 16 B per lane: a GPT-2
// row of 50304 bf16 is 25 vectors per lane), all loads are issued before any math, and the
// dlogits pass works from registers, so HBM sees exactly one read and one write of the logits.
// Measured slower than the two-pass kernel (see tdl_xent_fused); kept as the opt-in alternative.
template <int NV>
__global__ __launch_bounds__(256) void xent_fused_reg_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ labels,
                                                             float* __restrict__ loss, float* __restrict__ lse_out,
                                                             const float* __restrict__ scale_ptr, int V, int ld,
                                                             int ignore_index) {
    __shared__ float red_m[4], red_s[4], bcast[1];
    const int row = blockIdx.x;
    bf16_t* lr = logits + (size_t)row * ld;
    const int nvl = ld / 8;
    uint4 q[NV];
#pragma unroll
    for (int t = 0; t < NV; ++t) {
        const int i = threadIdx.x + t * 256;
        if (i < nvl) q[t] = ((const uint4*)lr)[i];
    }
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < NV; ++t) {
        const int i = threadIdx.x + t * 256;
        if (i < nvl) {
            float v[8];
            unpack8(q[t], v);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (i * 8 + k < V) m = fmaxf(m, v[k]);
        }
    }
    keep_packed<NV>(q);
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NV; ++t) {
        const int i = threadIdx.x + t * 256;
        if (i < nvl) {
            float v[8];
            unpack8(q[t], v);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (i * 8 + k < V) s += __expf(v[k] - m);
        }
    }
    keep_packed<NV>(q);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
        online_merge(m, s, m2, s2);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red_m[wid] = m;
        red_s[wid] = s;
    }
    __syncthreads();
    const int64_t lab = labels[row];
    const bool ign = (lab == ignore_index || lab < 0 || lab >= V);
    if (threadIdx.x == 0) {
        float M0 = red_m[0], S0 = red_s[0];
        for (int w = 1; w < 4; ++w) online_merge(M0, S0, red_m[w], red_s[w]);
        const float lse = M0 + __logf(S0);
        lse_out[row] = lse;
        loss[row] = ign ? 0.f : lse - bf2f(lr[lab]);  // row not yet overwritten: stores follow the barrier
        bcast[0] = lse;
    }
    __syncthreads();
    const float lse = bcast[0];
    const float sc = ign ? 0.f : scale_ptr[0];
#pragma unroll
    for (int t = 0; t < NV; ++t) {
        const int i = threadIdx.x + t * 256;
        if (i < nvl) {
            float v[8];
            unpack8(q[t], v);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int j = i * 8 + k;
                float p = j < V ? __expf(v[k] - lse) : 0.f;
                if (j == lab) p -= 1.f;
                v[k] = p * sc;
            }
            ((uint4*)lr)[i] = pack8(v);
        }
    }
}

TDL_API int tdl_xent_fused(void* logits, const int64_t* labels, float* loss, float* lse, const float* scale_ptr, int M,
                           int V, int ld, hipStream_t s) {
    if (M <= 0) return 0;
    // Two-pass by default: its re-read of the just-streamed row hits L2 / MALL, and measured faster
    // than the register-resident kernel (rocprof, 32k GPT-2 rows: 1.56 ms vs 1.70 ms; the latter's
    // 164 VGPRs leave two waves per SIMD that each load a whole row before any math, so loads and
    // stores of neighbouring rows barely overlap).  TDL_XENT_REG=1 selects it (A/B switch).
    static const bool two_pass = [] { const char* e = getenv("TDL_XENT_REG"); return !(e && e[0] == '1'); }();
    if (!two_pass && ld % 8 == 0 && ld <= 256 * 8 * 25 && ld > 256 * 8 * 16) {
        xent_fused_reg_kernel<25><<<M, 256, 0, s>>>((bf16_t*)logits, labels, loss, lse, scale_ptr, V, ld, -100);
    } else if (!two_pass && ld % 8 == 0 && ld <= 256 * 8 * 16) {
        xent_fused_reg_kernel<16><<<M, 256, 0, s>>>((bf16_t*)logits, labels, loss, lse, scale_ptr, V, ld, -100);
    } else {
        xent_fused_kernel<<<M, 256, 0, s>>>((bf16_t*)logits, labels, loss, lse, scale_ptr, V, ld, -100);
    }
    TDL_LAUNCH_CHECK();
}
