// LayerNorm, bias+GELU(tanh) and token/position embedding kernels (bf16 I/O, fp32 math).
//
// Replaces the torch LayerNorm / GELU / Embedding used by the GPT-2 blocks that the
// reference partitions (distributed_trainer.py:124-135).
// Parameter gradients are accumulated straight into fp32 "main_grad" buffers with one
// float atomic per column per workgroup (row-summed on chip first), so the per-micro-batch
// bf16 weight-grad tensor and its separate accumulate kernel never exist.
#include "common.h"
#include <cstdlib>

template <int VEC, int CH>
__device__ __forceinline__ void ln_vload(const bf16_t* p, float* v) {
    if constexpr (VEC == 8) unpack8(*(const uint4*)p, v);
    else unpack4(*(const uint2*)p, v);
}

// ============================================================== LayerNorm forward
// One wave per row; every lane owns CH chunks of VEC contiguous columns
// (N == 64 * VEC * CH), so the whole row lives in registers: two-pass mean/var, exact.
template <int VEC, int CH>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                     const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int M, float eps) {
    constexpr int N = 64 * VEC * CH;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const bf16_t* xr = x + (size_t)row * N;
    float v[CH][VEC];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int col = (c * 64 + lane) * VEC;
        if constexpr (VEC == 8) unpack8(*(const uint4*)(xr + col), v[c]);
        else unpack4(*(const uint2*)(xr + col), v[c]);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int i = 0; i < VEC; ++i) s += v[c][i];
    const float mean = wave_sum(s) * (1.0f / N);
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            const float d = v[c][i] - mean;
            q += d * d;
        }
    const float rstd = rsqrtf(wave_sum(q) * (1.0f / N) + eps);
    bf16_t* yr = y + (size_t)row * N;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int col = (c * 64 + lane) * VEC;
        float wf[VEC], bf[VEC], o[VEC];
        if constexpr (VEC == 8) {
            unpack8(*(const uint4*)(w + col), wf);
            unpack8(*(const uint4*)(b + col), bf);
        } else {
            unpack4(*(const uint2*)(w + col), wf);
            unpack4(*(const uint2*)(b + col), bf);
        }
#pragma unroll
        for (int i = 0; i < VEC; ++i) o[i] = (v[c][i] - mean) * rstd * wf[i] + bf[i];
        if constexpr (VEC == 8) *(uint4*)(yr + col) = pack8(o);
        else *(uint2*)(yr + col) = pack4(o);
    }
    if (lane == 0) {
        mean_out[row] = mean;
        rstd_out[row] = rstd;
    }
}

// Generic fallback: one 256-thread block per row, two passes over global memory.
__global__ __launch_bounds__(256) void ln_fwd_generic(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                      const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int M, int N, float eps) {
    __shared__ float red[16];
    const int row = blockIdx.x;
    const bf16_t* xr = x + (size_t)row * N;
    float s = 0.f;
    for (int i = threadIdx.x; i < N; i += blockDim.x) s += bf2f(xr[i]);
    const float mean = block_sum(s, red) / N;
    float q = 0.f;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const float d = bf2f(xr[i]) - mean;
        q += d * d;
    }
    const float rstd = rsqrtf(block_sum(q, red) / N + eps);
    for (int i = threadIdx.x; i < N; i += blockDim.x)
        y[(size_t)row * N + i] = f2bf((bf2f(xr[i]) - mean) * rstd * bf2f(w[i]) + bf2f(b[i]));
    if (threadIdx.x == 0) {
        mean_out[row] = mean;
        rstd_out[row] = rstd;
    }
}

TDL_API int tdl_layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                              int M, int N, float eps, hipStream_t s) {
    const dim3 blk(256), grd((M + 3) / 4);
    auto X = (const bf16_t*)x; auto W = (const bf16_t*)w; auto B = (const bf16_t*)b; auto Y = (bf16_t*)y;
    switch (N) {
        case 256:  ln_fwd_kernel<4, 1><<<grd, blk, 0, s>>>(X, W, B, Y, mean, rstd, M, eps); break;
        case 512:  ln_fwd_kernel<8, 1><<<grd, blk, 0, s>>>(X, W, B, Y, mean, rstd, M, eps); break;
        case 768:  ln_fwd_kernel<4, 3><<<grd, blk, 0, s>>>(X, W, B, Y, mean, rstd, M, eps); break;
        case 1024: ln_fwd_kernel<8, 2><<<grd, blk, 0, s>>>(X, W, B, Y, mean, rstd, M, eps); break;
        case 1280: ln_fwd_kernel<4, 5><<<grd, blk, 0, s>>>(X, W, B, Y, mean, rstd, M, eps); break;
        case 1536: ln_fwd_kernel<8, 3><<<grd, blk, 0, s>>>(X, W, B, Y, mean, rstd, M, eps); break;
        case 2048: ln_fwd_kernel<8, 4><<<grd, blk, 0, s>>>(X, W, B, Y, mean, rstd, M, eps); break;
        default: ln_fwd_generic<<<M, 256, 0, s>>>(X, W, B, Y, mean, rstd, M, N, eps); break;
    }
    TDL_LAUNCH_CHECK();
}

// ============================================================== residual add + bias + LayerNorm forward
// Pre-LN block junction: y1 = x + z + bz (the residual stream after a projection whose GEMM ran
// without bias), h = LN(y1), and optionally y1b = y1 + b2 (the next projection's bias pre-added,
// so that projection's GEMM can accumulate onto y1b in place: y = y1b + f @ W).  LN statistics
// are taken over the bf16-rounded y1 that is stored, i.e. exactly what LN backward re-reads.
template <int VEC, int CH>
__global__ __launch_bounds__(256) void add_bias_ln_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ z, const bf16_t* __restrict__ bz,
    const bf16_t* __restrict__ b2, const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
    bf16_t* __restrict__ y1, bf16_t* __restrict__ y1b, bf16_t* __restrict__ h, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int M, float eps) {
    constexpr int N = 64 * VEC * CH;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const size_t off = (size_t)row * N;
    float v[CH][VEC];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int col = (c * 64 + lane) * VEC;
        float zv[VEC], bv[VEC];
        ln_vload<VEC, CH>(x + off + col, v[c]);
        ln_vload<VEC, CH>(z + off + col, zv);
        ln_vload<VEC, CH>(bz + col, bv);
#pragma unroll
        for (int i = 0; i < VEC; ++i) v[c][i] = (v[c][i] + zv[i]) + bv[i];
        if constexpr (VEC == 8) {
            const uint4 q = pack8(v[c]);
            *(uint4*)(y1 + off + col) = q;
            unpack8(q, v[c]);
        } else {
            const uint2 q = pack4(v[c]);
            *(uint2*)(y1 + off + col) = q;
            unpack4(q, v[c]);
        }
        if (y1b) {
            float o[VEC];
            ln_vload<VEC, CH>(b2 + col, bv);
#pragma unroll
            for (int i = 0; i < VEC; ++i) o[i] = v[c][i] + bv[i];
            if constexpr (VEC == 8) *(uint4*)(y1b + off + col) = pack8(o);
            else *(uint2*)(y1b + off + col) = pack4(o);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int i = 0; i < VEC; ++i) s += v[c][i];
    const float mean = wave_sum(s) * (1.0f / N);
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            const float d = v[c][i] - mean;
            q += d * d;
        }
    const float rstd = rsqrtf(wave_sum(q) * (1.0f / N) + eps);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int col = (c * 64 + lane) * VEC;
        float wf[VEC], bf[VEC], o[VEC];
        ln_vload<VEC, CH>(w + col, wf);
        ln_vload<VEC, CH>(b + col, bf);
#pragma unroll
        for (int i = 0; i < VEC; ++i) o[i] = (v[c][i] - mean) * rstd * wf[i] + bf[i];
        if constexpr (VEC == 8) *(uint4*)(h + off + col) = pack8(o);
        else *(uint2*)(h + off + col) = pack4(o);
    }
    if (lane == 0) {
        mean_out[row] = mean;
        rstd_out[row] = rstd;
    }
}

TDL_API int tdl_add_bias_ln_fwd(const void* x, const void* z, const void* bz, const void* b2, const void* w,
                                const void* b, void* y1, void* y1b, void* h, float* mean, float* rstd, int M, int N,
                                float eps, hipStream_t s) {
    const dim3 blk(256), grd((M + 3) / 4);
    auto X = (const bf16_t*)x; auto Z = (const bf16_t*)z; auto BZ = (const bf16_t*)bz; auto B2 = (const bf16_t*)b2;
    auto W = (const bf16_t*)w; auto B = (const bf16_t*)b;
    auto Y1 = (bf16_t*)y1; auto Y1B = (bf16_t*)y1b; auto H = (bf16_t*)h;
    if (y1b && !b2) return (int)hipErrorInvalidValue;
#define TDL_ABLN(V, C) add_bias_ln_fwd_kernel<V, C><<<grd, blk, 0, s>>>(X, Z, BZ, B2, W, B, Y1, Y1B, H, mean, rstd, M, eps)
    switch (N) {
        case 256:  TDL_ABLN(4, 1); break;
        case 512:  TDL_ABLN(8, 1); break;
        case 768:  TDL_ABLN(4, 3); break;
        case 1024: TDL_ABLN(8, 2); break;
        case 1280: TDL_ABLN(4, 5); break;
        case 1536: TDL_ABLN(8, 3); break;
        case 2048: TDL_ABLN(8, 4); break;
        default: return (int)hipErrorInvalidValue;  // callers use the unfused path for other widths
    }
#undef TDL_ABLN
    TDL_LAUNCH_CHECK();
}

// ============================================================== LayerNorm backward
// 4 waves per block, each wave walks RPW rows; dgamma/dbeta are summed per lane over the
// wave's rows, then across the 4 waves through LDS, then one fp32 atomic per column.
//
// Residual fusion (pre-LN transformer block, y = x + f(LN(x))): with ``dres`` non-null the kernel
// writes dx = LN_bwd(dy) + dres, so the autograd "skip + branch" gradient add never runs.  With
// SUMS it also emits per-block column partials of dres and of dx (the bias gradients of the two
// projections that feed the residual stream), so those need no separate column-sum pass either.

template <int VEC, int CH, int RPW, bool RES, bool SUMS>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const bf16_t* __restrict__ dres,
                                                     bf16_t* __restrict__ dx, float* __restrict__ part, int M) {
    constexpr int N = 64 * VEC * CH;
    constexpr int NS = SUMS ? 4 : 2;  // column partial sets: dgamma, dbeta [, sum dres, sum dx]
    __shared__ float red[2][4][N];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    float dw[CH][VEC], db[CH][VEC], wf[CH][VEC];
    float sr[SUMS ? CH : 1][VEC], sx[SUMS ? CH : 1][VEC];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int col = (c * 64 + lane) * VEC;
        ln_vload<VEC, CH>(w + col, wf[c]);
#pragma unroll
        for (int i = 0; i < VEC; ++i) dw[c][i] = db[c][i] = 0.f;
        if constexpr (SUMS) {
#pragma unroll
            for (int i = 0; i < VEC; ++i) sr[c][i] = sx[c][i] = 0.f;
        }
    }
    const int row0 = (blockIdx.x * 4 + wid) * RPW;
    for (int r = 0; r < RPW; ++r) {
        const int row = row0 + r;
        if (row >= M) break;
        const float mu = mean_in[row], rs = rstd_in[row];
        float xv[CH][VEC], gv[CH][VEC];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int col = (c * 64 + lane) * VEC;
            if constexpr (VEC == 8) {
                unpack8(*(const uint4*)(x + (size_t)row * N + col), xv[c]);
                unpack8(*(const uint4*)(dy + (size_t)row * N + col), gv[c]);
            } else {
                unpack4(*(const uint2*)(x + (size_t)row * N + col), xv[c]);
                unpack4(*(const uint2*)(dy + (size_t)row * N + col), gv[c]);
            }
        }
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const float xh = (xv[c][i] - mu) * rs;
                xv[c][i] = xh;
                dw[c][i] += gv[c][i] * xh;
                db[c][i] += gv[c][i];
                const float g = gv[c][i] * wf[c][i];
                gv[c][i] = g;
                s1 += g;
                s2 += g * xh;
            }
        float rv[CH][VEC];
        if constexpr (RES) {
#pragma unroll
            for (int c = 0; c < CH; ++c) ln_vload<VEC, CH>(dres + (size_t)row * N + (c * 64 + lane) * VEC, rv[c]);
        }
        s1 = wave_sum(s1) * (1.0f / N);
        s2 = wave_sum(s2) * (1.0f / N);
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int col = (c * 64 + lane) * VEC;
            float o[VEC];
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                o[i] = rs * (gv[c][i] - s1 - xv[c][i] * s2);
                if constexpr (RES) o[i] += rv[c][i];
            }
            if constexpr (VEC == 8) {
                const uint4 q = pack8(o);
                *(uint4*)(dx + (size_t)row * N + col) = q;
                if constexpr (SUMS) unpack8(q, o);  // column sums of the bf16 values actually stored
            } else {
                const uint2 q = pack4(o);
                *(uint2*)(dx + (size_t)row * N + col) = q;
                if constexpr (SUMS) unpack4(q, o);
            }
            if constexpr (SUMS) {
#pragma unroll
                for (int i = 0; i < VEC; ++i) {
                    sr[c][i] += rv[c][i];
                    sx[c][i] += o[i];
                }
            }
        }
    }
    // per-block partial sums with plain stores (the column sum over blocks runs in colsum_f32_kernel):
    // hundreds of blocks atomically adding into the same N floats is the contended-atomic worst case
    float* prow = part + (size_t)blockIdx.x * NS * N;
#pragma unroll
    for (int pass = 0; pass < NS / 2; ++pass) {
        if (pass) __syncthreads();
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const int col = (c * 64 + lane) * VEC + i;
                if (pass == 0) {
                    red[0][wid][col] = dw[c][i];
                    red[1][wid][col] = db[c][i];
                } else if constexpr (SUMS) {
                    red[0][wid][col] = sr[c][i];
                    red[1][wid][col] = sx[c][i];
                }
            }
        __syncthreads();
        for (int col = threadIdx.x; col < N; col += 256) {
            prow[2 * pass * N + col] = red[0][0][col] + red[0][1][col] + red[0][2][col] + red[0][3][col];
            prow[(2 * pass + 1) * N + col] = red[1][0][col] + red[1][1][col] + red[1][2][col] + red[1][3][col];
        }
    }
}

// acc[c] += sum_g part[g * ld + c]; grid (ceil(N/256), ceil(G/CS)).  Each thread issues its CS
// loads at once (latency, not bandwidth, bounds this pass) and adds with <= ceil(G/CS) atomics per column.
constexpr int CS_ROWS = 16;
__global__ __launch_bounds__(256) void colsum_f32_kernel(const float* __restrict__ part, int G, int N, int ld,
                                                         float* __restrict__ acc) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= N) return;
    const int g0 = blockIdx.y * CS_ROWS;
    float v[CS_ROWS];
#pragma unroll
    for (int i = 0; i < CS_ROWS; ++i) v[i] = (g0 + i < G) ? part[(size_t)(g0 + i) * ld + col] : 0.f;
#pragma unroll
    for (int w = CS_ROWS / 2; w > 0; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; ++i) v[i] += v[i + w];
    if (gridDim.y == 1) acc[col] += v[0];
    else atomicAdd(acc + col, v[0]);
}

// Vectorised column sum of G partial rows: lane = 4 columns (16-B loads), a wave = 256 columns, the
// four waves of a block take consecutive row strips of `rw` rows each and merge through LDS, so each
// column gets ONE atomic per 4*rw rows.  The scalar kernels above load 4 B per lane and issue one
// atomic per 16 rows (rocprof: 17 us for the 16.7 MB of a 32k-row LayerNorm backward, ~1 TB/s).
struct AccPtrs4 { float* p[4]; };
__global__ __launch_bounds__(256) void colsum_f32_vec_kernel(const float* __restrict__ part, int G, int N, int ld,
                                                             int rw, AccPtrs4 accs) {
    __shared__ float4 red[3][64];
    float* acc = accs.p[blockIdx.z];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int col = (blockIdx.x * 64 + lane) * 4;
    const bool live = acc != nullptr && col < N;
    const float* src = part + (size_t)blockIdx.z * N;
    const int r0 = (blockIdx.y * 4 + wid) * rw;
    const int r1 = min(r0 + rw, G);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (live) {
        int r = r0;
        for (; r + 8 <= r1; r += 8) {
            float4 q[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) q[i] = *(const float4*)(src + (size_t)(r + i) * ld + col);
#pragma unroll
            for (int i = 0; i < 8; ++i) { a.x += q[i].x; a.y += q[i].y; a.z += q[i].z; a.w += q[i].w; }
        }
        for (; r < r1; ++r) {
            const float4 q = *(const float4*)(src + (size_t)r * ld + col);
            a.x += q.x; a.y += q.y; a.z += q.z; a.w += q.w;
        }
    }
    if (wid) red[wid - 1][lane] = a;
    __syncthreads();
    if (wid == 0 && acc != nullptr) {  // whole wave (uniform): the shuffles below need every lane
#pragma unroll
        for (int w = 0; w < 3; ++w) {
            const float4 q = red[w][lane];
            a.x += q.x; a.y += q.y; a.z += q.z; a.w += q.w;
        }
        if (gridDim.y == 1) {
            if (live) { acc[col] += a.x; acc[col + 1] += a.y; acc[col + 2] += a.z; acc[col + 3] += a.w; }
        } else {
            // coalesced atomics: instruction k covers the 64 consecutive columns base + 64k + lane
            // (held by lane 16k + lane/4, component lane%4), as in embed_bwd_wte_coalesced_kernel
            const int base = blockIdx.x * 256, e = lane & 3;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int src = k * 16 + (lane >> 2);
                const float v0 = __shfl(a.x, src, 64), v1 = __shfl(a.y, src, 64);
                const float v2 = __shfl(a.z, src, 64), v3 = __shfl(a.w, src, 64);
                const int c = base + k * 64 + lane;
                if (c < N) atomicAdd(acc + c, e == 0 ? v0 : e == 1 ? v1 : e == 2 ? v2 : v3);
            }
        }
    }
}

// rows per wave: the largest of 64/32/16/8 that still gives >= 512 blocks (a few per CU)
static inline void launch_colsum_vec(const float* part, int G, int N, int ld, AccPtrs4 a, int sets, hipStream_t s) {
    const int gx = (N / 4 + 63) / 64;
    int rw = 64;
    while (rw > 8 && (long)gx * ((G + 4 * rw - 1) / (4 * rw)) * sets < 512) rw >>= 1;
    const dim3 grd(gx, (G + 4 * rw - 1) / (4 * rw), sets);
    colsum_f32_vec_kernel<<<grd, 256, 0, s>>>(part, G, N, ld, rw, a);
}

static inline void launch_colsum_f32(const float* part, int G, int N, int ld, float* acc, hipStream_t s) {
    if (N % 4 == 0 && ld % 4 == 0) {
        launch_colsum_vec(part, G, N, ld, AccPtrs4{{acc, nullptr, nullptr, nullptr}}, 1, s);
        return;
    }
    const dim3 grd((N + 255) / 256, (G + CS_ROWS - 1) / CS_ROWS);
    colsum_f32_kernel<<<grd, 256, 0, s>>>(part, G, N, ld, acc);
}

// Several column-partial sets stored side by side in each partial row (set z at column offset z*N),
// reduced into their own accumulators by one launch (grid.z = number of sets).
struct AccPtrs { float* p[4]; };
__global__ __launch_bounds__(256) void colsum_f32_multi_kernel(const float* __restrict__ part, int G, int N, int ld,
                                                               AccPtrs accs) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    float* acc = accs.p[blockIdx.z];
    if (col >= N || acc == nullptr) return;
    const float* src = part + (size_t)blockIdx.z * N;
    const int g0 = blockIdx.y * CS_ROWS;
    float v[CS_ROWS];
#pragma unroll
    for (int i = 0; i < CS_ROWS; ++i) v[i] = (g0 + i < G) ? src[(size_t)(g0 + i) * ld + col] : 0.f;
#pragma unroll
    for (int w = CS_ROWS / 2; w > 0; w >>= 1)
#pragma unroll
        for (int i = 0; i < w; ++i) v[i] += v[i + w];
    if (gridDim.y == 1) acc[col] += v[0];
    else atomicAdd(acc + col, v[0]);
}

__global__ __launch_bounds__(256) void ln_bwd_generic(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ w, const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in, const bf16_t* __restrict__ dres,
                                                      bf16_t* __restrict__ dx, float* __restrict__ dw_acc,
                                                      float* __restrict__ db_acc, float* __restrict__ sres_acc,
                                                      float* __restrict__ sdx_acc, int M, int N) {
    __shared__ float red[16];
    const int row = blockIdx.x;
    const float mu = mean_in[row], rs = rstd_in[row];
    float s1 = 0.f, s2 = 0.f;
    for (int i = threadIdx.x; i < N; i += 256) {
        const float xh = (bf2f(x[(size_t)row * N + i]) - mu) * rs;
        const float g = bf2f(dy[(size_t)row * N + i]) * bf2f(w[i]);
        s1 += g;
        s2 += g * xh;
    }
    s1 = block_sum(s1, red) / N;
    s2 = block_sum(s2, red) / N;
    for (int i = threadIdx.x; i < N; i += 256) {
        const float xh = (bf2f(x[(size_t)row * N + i]) - mu) * rs;
        const float gy = bf2f(dy[(size_t)row * N + i]);
        const float r = dres ? bf2f(dres[(size_t)row * N + i]) : 0.f;
        const bf16_t o = f2bf(rs * (gy * bf2f(w[i]) - s1 - xh * s2) + r);
        dx[(size_t)row * N + i] = o;
        atomicAdd(dw_acc + i, gy * xh);
        atomicAdd(db_acc + i, gy);
        if (sres_acc) atomicAdd(sres_acc + i, r);
        if (sdx_acc) atomicAdd(sdx_acc + i, bf2f(o));
    }
}

template <int RPW, bool RES, bool SUMS>
static void launch_ln_bwd(const bf16_t* DY, const bf16_t* X, const bf16_t* W, const float* mean, const float* rstd,
                          const bf16_t* DR, bf16_t* DX, float* part, int M, int G, int N, bool& tiled, hipStream_t s) {
    const dim3 blk(256), grd(G);
    tiled = true;
    switch (N) {
        case 256:  ln_bwd_kernel<4, 1, RPW, RES, SUMS><<<grd, blk, 0, s>>>(DY, X, W, mean, rstd, DR, DX, part, M); break;
        case 512:  ln_bwd_kernel<8, 1, RPW, RES, SUMS><<<grd, blk, 0, s>>>(DY, X, W, mean, rstd, DR, DX, part, M); break;
        case 768:  ln_bwd_kernel<4, 3, RPW, RES, SUMS><<<grd, blk, 0, s>>>(DY, X, W, mean, rstd, DR, DX, part, M); break;
        case 1024: ln_bwd_kernel<8, 2, RPW, RES, SUMS><<<grd, blk, 0, s>>>(DY, X, W, mean, rstd, DR, DX, part, M); break;
        case 1280: ln_bwd_kernel<4, 5, RPW, RES, SUMS><<<grd, blk, 0, s>>>(DY, X, W, mean, rstd, DR, DX, part, M); break;
        case 1536: ln_bwd_kernel<8, 3, RPW, RES, SUMS><<<grd, blk, 0, s>>>(DY, X, W, mean, rstd, DR, DX, part, M); break;
        case 2048: ln_bwd_kernel<8, 4, RPW, RES, SUMS><<<grd, blk, 0, s>>>(DY, X, W, mean, rstd, DR, DX, part, M); break;
        default: tiled = false; break;
    }
}

// dx = LN_bwd(dy) [+ dres]; dgamma/dbeta [+ colsum(dres), colsum(dx)] accumulated into fp32 buffers.
// part: workspace of tdl_layernorm_bwd_ws_floats(M, N) floats (per-block column partials).
TDL_API int tdl_layernorm_bwd_res(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                                  const void* dres, void* dx, float* dw_acc, float* db_acc, float* sres_acc,
                                  float* sdx_acc, int M, int N, float* part, hipStream_t s) {
    auto DY = (const bf16_t*)dy; auto X = (const bf16_t*)x; auto W = (const bf16_t*)w; auto DX = (bf16_t*)dx;
    auto DR = (const bf16_t*)dres;
    const bool sums = sres_acc != nullptr || sdx_acc != nullptr;
    if (sums && !dres) return (int)hipErrorInvalidValue;
    // Rows per wave.  With the four partial sets (SUMS) the column partials at 8 rows / block are as large
    // as dx; 32 rows / block (rpw 8) writes a quarter of them and the column-sum pass shrinks to match,
    // at an unchanged kernel time.  With two sets the longer row loop costs more than it saves
    // (rocprof A/B, profiles/r1_ln_bwd_rpw_ab.json), so those keep 8 rows / block.  TDL_LN_RPW=2|8
    // forces one choice.
    static const int forced = [] { const char* e = getenv("TDL_LN_RPW"); return e ? atoi(e) : 0; }();
    const int rpw = forced == 2 || forced == 8 ? forced : (sums ? 8 : 2);
    const int G = (M + 4 * rpw - 1) / (4 * rpw);
    bool tiled;
    if (rpw == 8) {
        if (!dres) launch_ln_bwd<8, false, false>(DY, X, W, mean, rstd, DR, DX, part, M, G, N, tiled, s);
        else if (!sums) launch_ln_bwd<8, true, false>(DY, X, W, mean, rstd, DR, DX, part, M, G, N, tiled, s);
        else launch_ln_bwd<8, true, true>(DY, X, W, mean, rstd, DR, DX, part, M, G, N, tiled, s);
    } else {
        if (!dres) launch_ln_bwd<2, false, false>(DY, X, W, mean, rstd, DR, DX, part, M, G, N, tiled, s);
        else if (!sums) launch_ln_bwd<2, true, false>(DY, X, W, mean, rstd, DR, DX, part, M, G, N, tiled, s);
        else launch_ln_bwd<2, true, true>(DY, X, W, mean, rstd, DR, DX, part, M, G, N, tiled, s);
    }
    if (tiled) {
        const int ns = sums ? 4 : 2;
        if (N % 4 == 0) {
            launch_colsum_vec(part, G, N, ns * N,
                              AccPtrs4{{dw_acc, db_acc, sums ? sres_acc : nullptr, sums ? sdx_acc : nullptr}}, ns, s);
        } else {
            AccPtrs a{{dw_acc, db_acc, sums ? sres_acc : nullptr, sums ? sdx_acc : nullptr}};
            const dim3 grd((N + 255) / 256, (G + CS_ROWS - 1) / CS_ROWS, ns);
            colsum_f32_multi_kernel<<<grd, 256, 0, s>>>(part, G, N, ns * N, a);
        }
    } else {
        ln_bwd_generic<<<M, 256, 0, s>>>(DY, X, W, mean, rstd, DR, DX, dw_acc, db_acc, sres_acc, sdx_acc, M, N);
    }
    TDL_LAUNCH_CHECK();
}

TDL_API int tdl_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                              void* dx, float* dw_acc, float* db_acc, int M, int N, float* part, hipStream_t s) {
    return tdl_layernorm_bwd_res(dy, x, w, mean, rstd, nullptr, dx, dw_acc, db_acc, nullptr, nullptr, M, N, part, s);
}

// sized for the 4-set (residual + sums) variant
TDL_API int64_t tdl_layernorm_bwd_ws_floats(int M, int N) { return (int64_t)4 * N * ((M + 7) / 8); }

// ============================================================== bias + GELU(tanh)
// y = gelu(x + b); x,y [M,N] bf16 (may alias), N % 8 == 0.  Block tile: R rows x 2048 columns
// (256 threads x 8); every row's 16-B load is issued before any math, so each lane keeps R loads
// in flight (a grid-stride loop with one load per iteration left this kernel latency-bound at
// ~4.4 TB/s).  The bias is loaded once per lane.
template <int R>
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ b,
                                                            bf16_t* __restrict__ y, int M, int N) {
    const int col = (blockIdx.x * 256 + threadIdx.x) * 8;
    if (col >= N) return;
    const int row0 = blockIdx.y * R;
    float bb[8];
    unpack8(*(const uint4*)(b + col), bb);
    uint4 xq[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = min(row0 + r, M - 1);
        xq[r] = *(const uint4*)(x + (size_t)row * N + col);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        if (row >= M) break;
        float v[8];
        unpack8(xq[r], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = gelu_tanh(v[k] + bb[k]);
        *(uint4*)(y + (size_t)row * N + col) = pack8(v);
    }
}

TDL_API int tdl_bias_gelu_fwd(const void* x, const void* b, void* y, int M, int N, hipStream_t s) {
    if (N % 8) return (int)hipErrorInvalidValue;
    constexpr int R = 8;
    const dim3 grd((N / 8 + 255) / 256, (M + R - 1) / R);
    bias_gelu_fwd_kernel<R><<<grd, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)b, (bf16_t*)y, M, N);
    TDL_LAUNCH_CHECK();
}

// dx = dy * gelu'(x + b); db += colsum(dx).  b may be null (x already holds the biased pre-activation).  Block tile: R rows x 2048 columns (256 thr x 8).
template <int R>
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ b, bf16_t* __restrict__ dx,
                                                            float* __restrict__ part, int M, int N) {
    const int col = (blockIdx.x * 256 + threadIdx.x) * 8;
    if (col >= N) return;
    const int row0 = blockIdx.y * R;
    float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, acc[8];
    if (b) unpack8(*(const uint4*)(b + col), bb);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    // issue every row's loads before any math: R x 32 B in flight per lane hides HBM latency
    uint4 gq[R], xq[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = min(row0 + r, M - 1);
        gq[r] = *(const uint4*)(dy + (size_t)row * N + col);
        xq[r] = *(const uint4*)(x + (size_t)row * N + col);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int row = row0 + r;
        if (row >= M) break;
        float g[8], v[8];
        unpack8(gq[r], g);
        unpack8(xq[r], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float d = g[k] * gelu_tanh_grad(v[k] + bb[k]);
            v[k] = d;
            acc[k] += d;
        }
        *(uint4*)(dx + (size_t)row * N + col) = pack8(v);
    }
    if (part) {  // plain-stored per-row-block partial column sums
        float4* p = (float4*)(part + (size_t)blockIdx.y * N + col);
        p[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        p[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
}

TDL_API int tdl_bias_gelu_bwd(const void* dy, const void* x, const void* b, void* dx, float* db_acc, int M, int N,
                              float* part, hipStream_t s) {
    // part: (ceil(M/16) * N) floats when db_acc is set
    constexpr int R = 16;
    const dim3 grd((N / 8 + 255) / 256, (M + R - 1) / R);
    bias_gelu_bwd_kernel<R><<<grd, 256, 0, s>>>((const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)b, (bf16_t*)dx,
                                                db_acc ? part : nullptr, M, N);
    if (db_acc) launch_colsum_f32(part, (int)grd.y, N, N, db_acc, s);
    TDL_LAUNCH_CHECK();
}

// ============================================================== bias gradient: acc[N] += sum_rows dy[M,N] (bf16)
// Block = 4 waves; lane owns 8 consecutive columns of a 512-column tile; each wave sums a
// 16-row strip with all loads issued up front, the 4 waves merge through LDS, then ONE fp32
// atomic per column per block (replaces torch's .float() copy + reduce + add: 3 passes -> 1).
__global__ __launch_bounds__(256) void colsum_bf16_kernel(const bf16_t* __restrict__ dy, float* __restrict__ acc_out,
                                                          int M, int N) {
    constexpr int RW = 4;  // 16 rows per block: >= 512 blocks at M = 4096 even for N = 1024
    __shared__ float red[4][512];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int col = blockIdx.x * 512 + lane * 8;
    const int row0 = blockIdx.y * (4 * RW) + w * RW;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (col < N) {
        uint4 q[RW];
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int row = min(row0 + r, M - 1);
            q[r] = *(const uint4*)(dy + (size_t)row * N + col);
        }
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            if (row0 + r >= M) break;
            float v[8];
            unpack8(q[r], v);
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += v[k];
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) red[w][lane * 8 + k] = acc[k];
    __syncthreads();
    for (int c = threadIdx.x; c < 512; c += 256) {
        const int gc = blockIdx.x * 512 + c;
        if (gc < N) acc_out[(size_t)blockIdx.y * N + gc] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    }
}

// acc[n] += sum over g < G of part[g * ld + n] (fp32 partial rows from another kernel)
TDL_API int tdl_colsum_f32(const float* part, int G, int N, int ld, float* acc, hipStream_t s) {
    if (G <= 0 || N <= 0) return (int)hipErrorInvalidValue;
    launch_colsum_f32(part, G, N, ld, acc, s);
    TDL_LAUNCH_CHECK();
}

TDL_API int tdl_colsum_bf16(const void* dy, float* acc, int M, int N, float* part, hipStream_t s) {
    // part: (ceil(M/16) * N) floats of per-block partials, then one short column-sum pass
    if (N % 8) return (int)hipErrorInvalidValue;
    const dim3 grd((N + 511) / 512, (M + 15) / 16);
    colsum_bf16_kernel<<<grd, 256, 0, s>>>((const bf16_t*)dy, part, M, N);
    launch_colsum_f32(part, (int)grd.y, N, N, acc, s);
    TDL_LAUNCH_CHECK();
}

// ============================================================== embeddings
// out[b,t,:] = wte[ids[b,t],:] + wpe[t,:]   (one wave per token, H % 512 == 0 or H % 256 == 0)
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ wte,
                                                        const bf16_t* __restrict__ wpe, bf16_t* __restrict__ out,
                                                        int B, int T, int H) {
    const int tok = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tok >= B * T) return;
    const int lane = threadIdx.x & 63, t = tok % T;
    const int64_t id = ids[tok];
    for (int col = lane * 4; col < H; col += 256) {
        float a[4], p[4];
        unpack4(*(const uint2*)(wte + id * H + col), a);
        unpack4(*(const uint2*)(wpe + (size_t)t * H + col), p);
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] += p[k];
        *(uint2*)(out + (size_t)tok * H + col) = pack4(a);
    }
}

TDL_API int tdl_embedding_fwd(const int64_t* ids, const void* wte, const void* wpe, void* out, int B, int T, int H,
                              int unused, hipStream_t s) {
    (void)unused;
    embed_fwd_kernel<<<(B * T + 3) / 4, 256, 0, s>>>(ids, (const bf16_t*)wte, (const bf16_t*)wpe, (bf16_t*)out, B, T, H);
    TDL_LAUNCH_CHECK();
}

// wte_grad[ids[b,t],:] += dout[b,t,:] (fp32 atomics; repeated ids collide correctly)
__global__ __launch_bounds__(256) void embed_bwd_wte_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ dout,
                                                            float* __restrict__ wte_grad, int BT, int H) {
    const int tok = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tok >= BT) return;
    const int lane = threadIdx.x & 63;
    const int64_t id = ids[tok];
    for (int col = lane * 4; col < H; col += 256) {
        float g[4];
        unpack4(*(const uint2*)(dout + (size_t)tok * H + col), g);
#pragma unroll
        for (int k = 0; k < 4; ++k) atomicAdd(wte_grad + id * H + col + k, g[k]);
    }
}
// Same scatter with coalesced atomics (H % 256 == 0): the lane that loaded 4 columns is not the lane
// that adds them; after four shuffles, atomic instruction k of a wave covers the 64 consecutive fp32
// columns c0 + 64k .. +63 (256 B, two cache lines) instead of one column in every 16 B of a 1 KB span
// (eight lines), so L2 sees a quarter of the atomic transactions.
__global__ __launch_bounds__(256) void embed_bwd_wte_coalesced_kernel(const int64_t* __restrict__ ids,
                                                                      const bf16_t* __restrict__ dout,
                                                                      float* __restrict__ wte_grad, int BT, int H) {
    const int tok = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tok >= BT) return;  // uniform per wave: the shuffles below see all 64 lanes
    const int lane = threadIdx.x & 63;
    float* dst = wte_grad + ids[tok] * (int64_t)H;
    const int e = lane & 3;
    for (int c0 = 0; c0 < H; c0 += 256) {
        float g[4];
        unpack4(*(const uint2*)(dout + (size_t)tok * H + c0 + lane * 4), g);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int src = k * 16 + (lane >> 2);  // holder of column c0 + 64k + lane
            const float v0 = __shfl(g[0], src, 64), v1 = __shfl(g[1], src, 64);
            const float v2 = __shfl(g[2], src, 64), v3 = __shfl(g[3], src, 64);
            atomicAdd(dst + c0 + k * 64 + lane, e == 0 ? v0 : e == 1 ? v1 : e == 2 ? v2 : v3);
        }
    }
}
// wpe_grad[t,:] += sum_b dout[b,t,:]  (single writer per element, no atomics)
__global__ __launch_bounds__(256) void embed_bwd_wpe_kernel(const bf16_t* __restrict__ dout, float* __restrict__ wpe_grad,
                                                            int B, int T, int H) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= (size_t)T * H) return;
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += bf2f(dout[(size_t)b * T * H + i]);
    wpe_grad[i] += acc;
}

TDL_API int tdl_embedding_bwd(const int64_t* ids, const void* dout, float* wte_grad, float* wpe_grad, int B, int T, int H,
                              int unused, hipStream_t s) {
    (void)unused;
    if (wte_grad && H % 256 == 0)
        embed_bwd_wte_coalesced_kernel<<<(B * T + 3) / 4, 256, 0, s>>>(ids, (const bf16_t*)dout, wte_grad, B * T, H);
    else if (wte_grad)
        embed_bwd_wte_kernel<<<(B * T + 3) / 4, 256, 0, s>>>(ids, (const bf16_t*)dout, wte_grad, B * T, H);
    if (wpe_grad)
        embed_bwd_wpe_kernel<<<(int)(((size_t)T * H + 255) / 256), 256, 0, s>>>((const bf16_t*)dout, wpe_grad, B, T, H);
    TDL_LAUNCH_CHECK();
}

// ============================================================== dst_f32 += src (bf16 or f32)
__global__ __launch_bounds__(256) void add_into_f32_kernel(float* __restrict__ dst, const void* __restrict__ src,
                                                           int64_t n, int src_bf16) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] += src_bf16 ? bf2f(((const bf16_t*)src)[i]) : ((const float*)src)[i];
}

TDL_API int tdl_add_into_f32(float* dst, const void* src, int64_t n, int src_bf16, hipStream_t s) {
    const int64_t blocks = (n + 255) / 256;
    add_into_f32_kernel<<<(int)(blocks < 8192 ? blocks : 8192), 256, 0, s>>>(dst, src, n, src_bf16);
    TDL_LAUNCH_CHECK();
}

// ============================================================== y = x * (*scale), bf16, device scalar
// Scales by an fp32 DEVICE scalar (e.g. an autograd grad_output) without a host sync and without
// rounding the scalar to bf16 first: fp32 product, one rounding.  x, y 16-byte aligned, n % 8 == 0.
__global__ __launch_bounds__(256) void scale_bf16_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         const float* __restrict__ scale, int64_t n8) {
    const float sc = scale[0];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        float v[8];
        unpack8(((const uint4*)x)[i], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= sc;
        ((uint4*)y)[i] = pack8(v);
    }
}

TDL_API int tdl_scale_bf16(const void* x, void* y, const float* scale, int64_t n, hipStream_t s) {
    if (n % 8 != 0 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return (int)hipErrorInvalidValue;
    const int64_t n8 = n / 8, blocks = (n8 + 255) / 256;
    scale_bf16_kernel<<<(int)(blocks < 4096 ? blocks : 4096), 256, 0, s>>>((const bf16_t*)x, (bf16_t*)y, scale, n8);
    TDL_LAUNCH_CHECK();
}

// ============================================================== bf16 transpose: out[C,R] = in[R,C]^T
// Builds the [out, in] forward-GEMM copy of a block weight once per weight generation
// (ops/layers.py fwd_weight).  64x64 tile per 256-thread block: every lane moves 16 B per access
// on both sides (8 lanes cover one 128-B row segment), the turn happens in LDS.  A row of the LDS
// tile is 64 + 2 bf16 wide so the column reads of one wave spread over the banks.  R % 64 == 0 and
// C % 64 == 0 (checked by the entry point).
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                             int R, int C) {
    constexpr int LDW = 66;
    __shared__ unsigned short tile[64 * LDW];
    const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
    const unsigned short* src = reinterpret_cast<const unsigned short*>(in);
    unsigned short* dst = reinterpret_cast<unsigned short*>(out);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int v = threadIdx.x + h * 256;          // 512 vectors of 8 bf16
        const int r = v >> 3, cg = (v & 7) * 8;
        const uint4 q = *reinterpret_cast<const uint4*>(src + (size_t)(r0 + r) * C + c0 + cg);
        const unsigned short* e = reinterpret_cast<const unsigned short*>(&q);
#pragma unroll
        for (int k = 0; k < 8; ++k) tile[r * LDW + cg + k] = e[k];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int v = threadIdx.x + h * 256;
        const int c = v >> 3, rg = (v & 7) * 8;
        uint4 q;
        unsigned short* e = reinterpret_cast<unsigned short*>(&q);
#pragma unroll
        for (int k = 0; k < 8; ++k) e[k] = tile[(rg + k) * LDW + c];
        *reinterpret_cast<uint4*>(dst + (size_t)(c0 + c) * R + r0 + rg) = q;
    }
}

TDL_API int tdl_transpose_bf16(const void* in, void* out, int R, int C, hipStream_t s) {
    if (R % 64 || C % 64 || R <= 0 || C <= 0) return (int)hipErrorInvalidValue;
    transpose_bf16_kernel<<<dim3(C / 64, R / 64), 256, 0, s>>>((const bf16_t*)in, (bf16_t*)out, R, C);
    TDL_LAUNCH_CHECK();
}

// Batched form: every stale forward-layout copy of a stage in ONE launch per 64 weights
// (ops/layers.py prebuild_fwd_weights, called at the head of a stage's forward), instead of one
// launch per weight at its first use (97 launches of ~6.6 us, ~1.9 TB/s, per GPT-2-medium step).
// Workgroup t takes tile t of the concatenated tile lists (first[j] = first tile of job j).
constexpr int TBATCH_MAX = 64;
struct TransposeBatch {
    const bf16_t* in[TBATCH_MAX];
    bf16_t* out[TBATCH_MAX];
    int R[TBATCH_MAX], C[TBATCH_MAX];
    int first[TBATCH_MAX + 1];
    int n;
};

__global__ __launch_bounds__(256) void transpose_bf16_batch_kernel(const TransposeBatch b) {
    const int t = blockIdx.x;
    int j = 0;
    while (j + 1 < b.n && b.first[j + 1] <= t) ++j;   // uniform per workgroup
    const int C = b.C[j], R = b.R[j];
    const int lt = t - b.first[j], tc = C / 64;
    const int r0 = (lt / tc) * 64, c0 = (lt % tc) * 64;
    constexpr int LDW = 66;
    __shared__ unsigned short tile[64 * LDW];
    const unsigned short* src = reinterpret_cast<const unsigned short*>(b.in[j]);
    unsigned short* dst = reinterpret_cast<unsigned short*>(b.out[j]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int v = threadIdx.x + h * 256;
        const int r = v >> 3, cg = (v & 7) * 8;
        const uint4 q = *reinterpret_cast<const uint4*>(src + (size_t)(r0 + r) * C + c0 + cg);
        const unsigned short* e = reinterpret_cast<const unsigned short*>(&q);
#pragma unroll
        for (int k = 0; k < 8; ++k) tile[r * LDW + cg + k] = e[k];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int v = threadIdx.x + h * 256;
        const int c = v >> 3, rg = (v & 7) * 8;
        uint4 q;
        unsigned short* e = reinterpret_cast<unsigned short*>(&q);
#pragma unroll
        for (int k = 0; k < 8; ++k) e[k] = tile[(rg + k) * LDW + c];
        *reinterpret_cast<uint4*>(dst + (size_t)(c0 + c) * R + r0 + rg) = q;
    }
}

TDL_API int tdl_transpose_bf16_batch(TransposeBatch b, hipStream_t s) {
    if (b.n <= 0 || b.n > TBATCH_MAX || b.first[0] != 0) return (int)hipErrorInvalidValue;
    for (int j = 0; j < b.n; ++j) {
        if (b.R[j] % 64 || b.C[j] % 64 || b.R[j] <= 0 || b.C[j] <= 0 || !b.in[j] || !b.out[j]) return (int)hipErrorInvalidValue;
        if (b.first[j + 1] - b.first[j] != (b.R[j] / 64) * (b.C[j] / 64)) return (int)hipErrorInvalidValue;
    }
    transpose_bf16_batch_kernel<<<b.first[b.n], 256, 0, s>>>(b);
    TDL_LAUNCH_CHECK();
}
