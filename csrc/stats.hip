// Verification-path reduction kernels:
//   K1 tensor_stats      one-pass moments (Chan/Pebay merge to the 4th moment) + min/max/L1/L2/Linf
//   K2 histogram quantile approximate median / p25 / p75 from a 2048-bin histogram over [min,max]
//   K3 grad_stats        segmented (per-parameter) norm / dot-with-EMA-reference / ref-norm over a
//                        stage's FLAT fp32 gradient, EMA reference updated in the same pass
//   K4 zscore_detect     device ring-buffer baseline + z-score decision (attack_detector.py:292-342)
//   K5 trust_update      fused EMA/decay/FSM trust update over all nodes (trust_manager.py:92-181)
// They replace the reference's host path: `.cpu().numpy()` of whole activations plus
// numpy/scipy statistics (attack_detector.py:78,185-223) and per-tensor `.item()` syncs
// (distributed_trainer.py:242-256).  Everything stays on device; the caller reads back a
// few dozen floats asynchronously.
#include "common.h"

#define NSTAT 12
#define NHIST 2048
#define MAXPART 1024
#define REF_STRIDE 8   // K3: EMA-reference (cosine) chunks, one in REF_STRIDE

struct Moments {  // central-moment partial, fp64
    double n, mean, m2, m3, m4, mn, mx, abssum;
};

__device__ __forceinline__ void merge(Moments& a, const Moments& b) {
    if (b.n == 0.0) return;
    if (a.n == 0.0) { a = b; return; }
    const double na = a.n, nb = b.n, n = na + nb;
    const double delta = b.mean - a.mean, dn = delta / n, dn2 = dn * dn;
    const double t1 = delta * dn * na * nb;
    const double m4 = a.m4 + b.m4 + t1 * dn2 * (na * na - na * nb + nb * nb) + 6.0 * dn2 * (na * na * b.m2 + nb * nb * a.m2) +
                      4.0 * dn * (na * b.m3 - nb * a.m3);
    const double m3 = a.m3 + b.m3 + t1 * dn * (na - nb) + 3.0 * dn * (na * b.m2 - nb * a.m2);
    a.m2 = a.m2 + b.m2 + t1;
    a.m3 = m3;
    a.m4 = m4;
    a.mean = a.mean + nb * dn;
    a.n = n;
    a.mn = fmin(a.mn, b.mn);
    a.mx = fmax(a.mx, b.mx);
    a.abssum += b.abssum;
}

__device__ __forceinline__ Moments shfl_xor_m(const Moments& m, int o) {
    Moments r;
    r.n = __shfl_xor(m.n, o, 64); r.mean = __shfl_xor(m.mean, o, 64);
    r.m2 = __shfl_xor(m.m2, o, 64); r.m3 = __shfl_xor(m.m3, o, 64); r.m4 = __shfl_xor(m.m4, o, 64);
    r.mn = __shfl_xor(m.mn, o, 64); r.mx = __shfl_xor(m.mx, o, 64); r.abssum = __shfl_xor(m.abssum, o, 64);
    return r;
}

// Thread-local accumulator: shifted power sums in fp32 (shift = first value seen).
struct ThreadAcc {
    float c, s1, s2, s3, s4, mn, mx, abssum;
    int n;
    __device__ void init() { c = 0.f; s1 = s2 = s3 = s4 = 0.f; mn = INFINITY; mx = -INFINITY; abssum = 0.f; n = 0; }
    __device__ __forceinline__ void add(float x) {
        if (n == 0) c = x;
        const float d = x - c, d2 = d * d;
        s1 += d; s2 += d2; s3 += d2 * d; s4 += d2 * d2;
        mn = fminf(mn, x); mx = fmaxf(mx, x); abssum += fabsf(x);
        ++n;
    }
    __device__ Moments to_moments() const {
        Moments m;
        m.n = n; m.mn = mn; m.mx = mx; m.abssum = abssum;
        if (n == 0) { m.mean = m.m2 = m.m3 = m.m4 = 0.0; return m; }
        const double N = n, S1 = s1, S2 = s2, S3 = s3, S4 = s4, mu = S1 / N;
        m.mean = (double)c + mu;
        m.m2 = S2 - S1 * mu;
        m.m3 = S3 - 3.0 * mu * S2 + 2.0 * S1 * mu * mu;
        m.m4 = S4 - 4.0 * mu * S3 + 6.0 * mu * mu * S2 - 3.0 * S1 * mu * mu * mu;
        if (m.m2 < 0.0) m.m2 = 0.0;
        return m;
    }
};

// Block merge of per-thread moments -> thread 0 holds the block result. `sh` >= 16 Moments.
__device__ Moments block_merge(Moments m, Moments* sh) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        Moments other = shfl_xor_m(m, o);
        // fixed merge order keeps the reduction deterministic
        if ((threadIdx.x & o) == 0) merge(m, other); else { merge(other, m); m = other; }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) sh[wid] = m;
    __syncthreads();
    Moments r = sh[0];
    for (int w = 1; w < nw; ++w) merge(r, sh[w]);
    return r;
}

__device__ __forceinline__ float load_elem(const void* x, int dtype, int64_t i) {
    return dtype == 1 ? bf2f(((const bf16_t*)x)[i]) : ((const float*)x)[i];
}

// ------------------------------------------------------------------ K1 pass 1 (flat tensor)
__global__ __launch_bounds__(256) void moments_partial_kernel(const void* __restrict__ x, int dtype, int64_t n,
                                                              Moments* __restrict__ part, float* __restrict__ nonfinite) {
    __shared__ Moments sh[16];
    ThreadAcc acc;
    acc.init();
    int bad = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (dtype == 1) {
        const int64_t nv = n / 8;
        for (int64_t i = tid; i < nv; i += stride) {
            float v[8];
            unpack8(((const uint4*)x)[i], v);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (isfinite(v[k])) acc.add(v[k]); else ++bad;
            }
        }
        for (int64_t i = nv * 8 + tid; i < n; i += stride) {
            const float v = bf2f(((const bf16_t*)x)[i]);
            if (isfinite(v)) acc.add(v); else ++bad;
        }
    } else {
        const int64_t nv = n / 4;
        for (int64_t i = tid; i < nv; i += stride) {
            const float4 f = ((const float4*)x)[i];
            const float v[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (isfinite(v[k])) acc.add(v[k]); else ++bad;
            }
        }
        for (int64_t i = nv * 4 + tid; i < n; i += stride) {
            const float v = ((const float*)x)[i];
            if (isfinite(v)) acc.add(v); else ++bad;
        }
    }
    Moments r = block_merge(acc.to_moments(), sh);
    if (threadIdx.x == 0) part[blockIdx.x] = r;
    if (bad) atomicAdd(nonfinite, (float)bad);
}

// Finalize moments (1 block): merge `np` partials in order, write the stat vector slots that
// do not need quantiles, store [min,max] range for the histogram pass, zero the histogram.
__device__ void write_moment_stats(const Moments& r, float* out, float* range) {
    const double n = r.n > 0 ? r.n : 1.0;
    const double var = r.m2 / n;
    const double sd = sqrt(var);
    out[0] = (float)r.mean;
    out[1] = (float)sd;
    out[2] = (float)r.mn;
    out[3] = (float)r.mx;
    out[5] = var > 0 ? (float)((r.m3 / n) / (var * sd)) : 0.f;
    out[6] = var > 0 ? (float)((r.m4 / n) / (var * var) - 3.0) : -3.f;
    out[9] = (float)r.abssum;
    out[10] = (float)sqrt(r.m2 + r.n * r.mean * r.mean);
    out[11] = (float)fmax(fabs(r.mn), fabs(r.mx));
    range[0] = (float)r.mn;
    range[1] = (float)r.mx;
}

__global__ __launch_bounds__(256) void moments_final_kernel(const Moments* __restrict__ part, int np, float* __restrict__ out,
                                                            float* __restrict__ range, unsigned* __restrict__ hist) {
    __shared__ Moments sh[16];
    Moments m;
    m.n = 0.0; m.mean = m.m2 = m.m3 = m.m4 = 0.0; m.mn = INFINITY; m.mx = -INFINITY; m.abssum = 0.0;
    for (int i = threadIdx.x; i < np; i += blockDim.x) merge(m, part[i]);
    Moments r = block_merge(m, sh);
    if (threadIdx.x == 0) write_moment_stats(r, out, range);
    for (int i = threadIdx.x; i < NHIST; i += blockDim.x) hist[i] = 0u;
}

// ------------------------------------------------------------------ K2 histogram + quantiles
// Quantiles of very large tensors come from a uniform systematic sample of <= HIST_SAMPLE elements
// (rank error ~ 1/sqrt(sample) << one bin): whole-tensor histograms of near-zero-centred gradients
// pile every element onto a few bins and serialise on their LDS atomics.
#define HIST_SAMPLE (1 << 22)
__global__ __launch_bounds__(256) void hist_kernel(const void* __restrict__ x, int dtype, int64_t n,
                                                   const float* __restrict__ range, unsigned* __restrict__ hist) {
    __shared__ unsigned h[NHIST];
    for (int i = threadIdx.x; i < NHIST; i += blockDim.x) h[i] = 0u;
    __syncthreads();
    const float lo = range[0], hi = range[1];
    const float scale = hi > lo ? NHIST / (hi - lo) : 0.f;
    const int64_t step = n > HIST_SAMPLE ? n / HIST_SAMPLE : 1;
    const int64_t ns = n / step;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < ns; j += stride) {
        const int64_t i = j * step;
        const float v = load_elem(x, dtype, i);
        if (!isfinite(v)) continue;
        int b = (int)((v - lo) * scale);
        b = b < 0 ? 0 : (b >= NHIST ? NHIST - 1 : b);
        atomicAdd(&h[b], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NHIST; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}

__device__ float hist_quantile(const unsigned* hist, double total, double q, float lo, float hi) {
    if (total <= 0) return 0.f;
    if (!(hi > lo)) return lo;
    const double k = q * (total - 1.0);
    double cum = 0.0;
    const double w = (double)(hi - lo) / NHIST;
    for (int b = 0; b < NHIST; ++b) {
        const double c = hist[b];
        if (c > 0 && k < cum + c) {
            const double frac = (k - cum + 0.5) / c;
            return (float)(lo + (b + frac) * w);
        }
        cum += c;
    }
    return hi;
}

// Quantiles from the histogram, one block: every thread owns 8 consecutive bins, a block scan of
// the per-thread counts gives each thread its cumulative offset, and the thread whose bins hold
// rank k = q (total - 1) interpolates inside its bin (hist_quantile's convention).
__global__ __launch_bounds__(256) void quantile_kernel(const unsigned* __restrict__ hist, const float* __restrict__ range,
                                                       float* __restrict__ out) {
    constexpr int PER = NHIST / 256;
    __shared__ double scan[256];
    const int t = threadIdx.x;
    double c[PER], mine = 0.0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        c[k] = hist[t * PER + k];
        mine += c[k];
    }
    scan[t] = mine;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan (integers in doubles: exact)
        const double v = t >= o ? scan[t - o] : 0.0;
        __syncthreads();
        scan[t] += v;
        __syncthreads();
    }
    const double total = scan[255];
    const double before = scan[t] - mine;
    const float lo = range[0], hi = range[1];
    const double qs[3] = {0.5, 0.25, 0.75};
    const int slot[3] = {4, 7, 8};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        if (total <= 0) {
            if (t == 0) out[slot[q]] = 0.f;
            continue;
        }
        if (!(hi > lo)) {
            if (t == 0) out[slot[q]] = lo;
            continue;
        }
        const double kq = qs[q] * (total - 1.0);
        if (t == 255 && kq >= total) out[slot[q]] = hi;
        if (kq < before || kq >= before + mine) continue;
        const double w = (double)(hi - lo) / NHIST;
        double cum = before;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            if (c[k] > 0 && kq < cum + c[k]) {
                out[slot[q]] = (float)(lo + (t * PER + k + (kq - cum + 0.5) / c[k]) * w);
                break;
            }
            cum += c[k];
        }
    }
}

// Workspace layout (bytes): [Moments x MAXPART][range 2 f32 | nonfinite f32 | pad][hist NHIST u32]
TDL_API int64_t tdl_stats_workspace_bytes() {
    return (int64_t)sizeof(Moments) * MAXPART + 16 + 4 * NHIST;
}

static inline int stat_grid(int64_t n) {
    int64_t g = (n + 256 * 16 - 1) / (256 * 16);
    if (g < 1) g = 1;
    if (g > MAXPART) g = MAXPART;
    if (g > 512) g = 512;
    return (int)g;
}

// out[12] = TENSOR_STATS order; out[12] (if out_extra) = non-finite element count.
TDL_API int tdl_tensor_stats(const void* x, int dtype, int64_t n, float* out, void* ws, int with_quantiles, hipStream_t s) {
    Moments* part = (Moments*)ws;
    float* range = (float*)((char*)ws + sizeof(Moments) * MAXPART);
    float* nonfinite = range + 2;
    unsigned* hist = (unsigned*)(range + 4);
    const int g = stat_grid(n);
    hipMemsetAsync(nonfinite, 0, sizeof(float), s);
    moments_partial_kernel<<<g, 256, 0, s>>>(x, dtype, n, part, nonfinite);
    moments_final_kernel<<<1, 256, 0, s>>>(part, g, out, range, hist);
    if (with_quantiles) {
        hist_kernel<<<g, 256, 0, s>>>(x, dtype, n, range, hist);
        quantile_kernel<<<1, 256, 0, s>>>(hist, range, out);
    }
    hipMemcpyAsync(out + NSTAT, nonfinite, sizeof(float), hipMemcpyDeviceToDevice, s);
    TDL_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ K3 segmented gradient stats
// chunks: int64 [C][3] = (segment, start, end) with end - start <= CHUNK; ordered by segment.
// seg_first: int32 [S + 1] first chunk of every segment.
// Three stages, every one of them parallel and deterministic (fixed reduction orders):
//   partial  one block per chunk: moments + (sum g^2, sum g.ref, sum ref^2, #non-finite), EMA
//            reference update in place (ref_valid==0: ref <- g).  Launched over any chunk range,
//            so the engine can run it per layer on a side stream while the backward of earlier
//            layers is still going (pipeline.py, verification overlap);
//   segment  one wave per segment: merges its chunks -> norm, cosine, segment moments;
//   summary  one block: merges the S segment moments -> TENSOR_STATS, norm summary, histogram range.
// Workspace: [Moments x C][double x 5C][Moments x S][range 2f | nonfinite f | pad f][hist NHIST u32]
struct GradWs {
    Moments* part;
    double* part_seg;
    Moments* seg;
    float* range;
    float* nonfinite;
    unsigned* hist;
};

__host__ __device__ inline GradWs grad_ws(void* ws, int C, int S) {
    GradWs w;
    w.part = (Moments*)ws;
    w.part_seg = (double*)((char*)ws + sizeof(Moments) * (size_t)C);
    w.seg = (Moments*)(w.part_seg + 5 * (size_t)C);
    w.range = (float*)(w.seg + (size_t)S);
    w.nonfinite = w.range + 2;
    w.hist = (unsigned*)(w.range + 4);
    return w;
}

TDL_API int64_t tdl_grad_stats_ws_bytes(int C, int S) {
    return (int64_t)sizeof(Moments) * C + 40ll * C + (int64_t)sizeof(Moments) * S + 16 + 4 * NHIST;
}

// REDUCE = false: the gradient g is final in memory (grad_partial_kernel).
// REDUCE = true : the chunk's gradient is completed here first — g[i] += sum over the split-K slabs of
//   a weight-gradient GEMM (slabs: [nsplit][segment numel], element i - seg_off; same fold order as
//   tdl_splitk_reduce_add, so the stored gradient and every statistic are bit-identical to the
//   reduce-then-partial sequence) — and the statistics are taken from the registers, so the final
//   gradient is never re-read (grad_reduce_partial_kernel; ops/gemm.py matmul_f32_acc with a sink).
template <bool REDUCE>
__device__ __forceinline__ void grad_partial_body(float* __restrict__ g, float* __restrict__ ref,
                                                  const int64_t* __restrict__ chunks, int c, int ref_valid, float beta,
                                                  Moments* __restrict__ part, double* __restrict__ part_seg,
                                                  const float* __restrict__ slabs, int nsplit, int64_t seg_off,
                                                  int64_t seg_n) {
    __shared__ double red[12][4];
    const int64_t start = chunks[3 * c + 1], end = chunks[3 * c + 2];
    // the EMA reference (cosine feature) is kept on every REF_STRIDE-th chunk only: a 1/8 sample
    // of a stage's parameters estimates the cosine to well within its step-to-step noise at an
    // eighth of the reference traffic (read + write of an fp32 copy of the gradient)
    if (ref && (c % REF_STRIDE) != 0) ref = nullptr;
    // One shift for the whole chunk — the mean of the finite values among its first 64 elements
    // (completed from the slabs in REDUCE mode), computed identically by every wave and read
    // before any lane stores: every lane's shifted power sums are then about the same point and
    // the block combines them by plain addition — no per-level Chan/Pebay merge of fp64 moment
    // structs, which cost more than the 32 elements per lane themselves.
    float shift;
    {
        const int64_t i0 = start + (threadIdx.x & 63);
        float v0 = 0.f;
        if (i0 < end) {
            v0 = g[i0];
            if constexpr (REDUCE) {
                for (int s = 0; s < nsplit; ++s) v0 += slabs[(int64_t)s * seg_n + (i0 - seg_off)];
            }
        }
        const bool ok = i0 < end && isfinite(v0);
        const float num = wave_sum(ok ? v0 : 0.f), den = wave_sum(ok ? 1.f : 0.f);
        shift = den > 0.f ? num / den : 0.f;
    }
    if constexpr (REDUCE) __syncthreads();
    float s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f, mn = INFINITY, mx = -INFINITY, abssum = 0.f;
    int cnt = 0;
    float sq = 0.f, dot = 0.f, rsq = 0.f;
    int bad = 0;
    // per element: moments of the finite gradient values, the EMA reference update and the
    // gradient . reference dot product (returns the new reference value)
    auto proc = [&](float v, float r) -> float {
        if (isfinite(v)) {
            const float d = v - shift, d2 = d * d;
            s1 += d; s2 += d2; s3 += d2 * d; s4 += d2 * d2;
            mn = fminf(mn, v); mx = fmaxf(mx, v); abssum += fabsf(v);
            ++cnt;
            sq += v * v;
        } else {
            ++bad;
        }
        if (ref_valid) {
            dot += v * r;
            rsq += r * r;
            return beta * r + (1.f - beta) * (isfinite(v) ? v : 0.f);
        }
        return isfinite(v) ? v : 0.f;
    };
    auto load1 = [&](int64_t i) -> float {
        float v = g[i];
        if constexpr (REDUCE) {
            for (int s = 0; s < nsplit; ++s) v += slabs[(int64_t)s * seg_n + (i - seg_off)];
            g[i] = v;
        }
        return v;
    };
    auto load4 = [&](int64_t i) -> float4 {
        float4 v = *(const float4*)(g + i);
        if constexpr (REDUCE) {
            for (int s = 0; s < nsplit; ++s) {
                const float4 w = *(const float4*)(slabs + (int64_t)s * seg_n + (i - seg_off));
                v.x += w.x;
                v.y += w.y;
                v.z += w.z;
                v.w += w.w;
            }
            *(float4*)(g + i) = v;
        }
        return v;
    };
    // 16-byte vector body over the 4-aligned part of the chunk, scalar head / tail
    int64_t vbeg = (start + 3) & ~(int64_t)3;
    if (vbeg > end) vbeg = end;
    const int64_t vend = vbeg + ((end - vbeg) & ~(int64_t)3);
    for (int64_t i = start + threadIdx.x; i < vbeg; i += blockDim.x) {
        const float nr = proc(load1(i), ref ? ref[i] : 0.f);
        if (ref) ref[i] = nr;
    }
    // main body: 4 float4 per lane per trip, every load issued before any math (a layer's chunks
    // are ~1.5 blocks per CU, so latency is hidden by loads in flight, not by occupancy)
    int64_t i = vbeg + 4 * (int64_t)threadIdx.x;
    const int64_t step = 4 * (int64_t)blockDim.x;
    for (; i + 3 * step < vend; i += 4 * step) {
        float4 v[4], r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = load4(i + u * step);
        if (ref) {
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = *(const float4*)(ref + i + u * step);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float4 nr;
            nr.x = proc(v[u].x, r[u].x);
            nr.y = proc(v[u].y, r[u].y);
            nr.z = proc(v[u].z, r[u].z);
            nr.w = proc(v[u].w, r[u].w);
            if (ref) *(float4*)(ref + i + u * step) = nr;
        }
    }
    for (; i < vend; i += step) {
        const float4 v = load4(i);
        const float4 r = ref ? *(const float4*)(ref + i) : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 nr;
        nr.x = proc(v.x, r.x);
        nr.y = proc(v.y, r.y);
        nr.z = proc(v.z, r.z);
        nr.w = proc(v.w, r.w);
        if (ref) *(float4*)(ref + i) = nr;
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += blockDim.x) {
        const float nr = proc(load1(i), ref ? ref[i] : 0.f);
        if (ref) ref[i] = nr;
    }
    // wave sums in fp64 (fixed shuffle tree), then the 4 waves in a fixed order: deterministic
    double a[10] = {(double)cnt, (double)s1, (double)s2, (double)s3, (double)s4, (double)abssum,
                    (double)sq, (double)dot, (double)rsq, (double)bad};
    mn = wave_min(mn);
    mx = wave_max(mx);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        a[k] = wave_sum_d(a[k]);
        if (lane == 0) red[k][wid] = a[k];
    }
    if (lane == 0) {
        red[10][wid] = mn;
        red[11][wid] = mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t[10];
#pragma unroll
        for (int k = 0; k < 10; ++k) t[k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
        Moments r;
        r.n = t[0];
        r.mn = fmin(fmin(red[10][0], red[10][1]), fmin(red[10][2], red[10][3]));
        r.mx = fmax(fmax(red[11][0], red[11][1]), fmax(red[11][2], red[11][3]));
        r.abssum = t[5];
        if (t[0] == 0.0) {
            r.mean = r.m2 = r.m3 = r.m4 = 0.0;
        } else {
            const double N = t[0], S1 = t[1], S2 = t[2], S3 = t[3], S4 = t[4], mu = S1 / N;
            r.mean = (double)shift + mu;
            r.m2 = S2 - S1 * mu;
            r.m3 = S3 - 3.0 * mu * S2 + 2.0 * S1 * mu * mu;
            r.m4 = S4 - 4.0 * mu * S3 + 6.0 * mu * mu * S2 - 3.0 * S1 * mu * mu * mu;
            if (r.m2 < 0.0) r.m2 = 0.0;
        }
        part[c] = r;
        part_seg[5 * c] = t[6];
        part_seg[5 * c + 1] = t[7];
        part_seg[5 * c + 2] = t[8];
        part_seg[5 * c + 3] = t[9];
        part_seg[5 * c + 4] = ref ? t[6] : 0.0;   // |g|^2 over the reference-tracked chunks
    }
}

__global__ __launch_bounds__(256) void grad_partial_kernel(float* __restrict__ g, float* __restrict__ ref,
                                                           const int64_t* __restrict__ chunks, int c0, int ref_valid,
                                                           float beta, Moments* __restrict__ part,
                                                           double* __restrict__ part_seg) {
    grad_partial_body<false>(g, ref, chunks, c0 + blockIdx.x, ref_valid, beta, part, part_seg, nullptr, 0, 0, 0);
}

__global__ __launch_bounds__(256) void grad_reduce_partial_kernel(float* __restrict__ g, float* __restrict__ ref,
                                                                  const int64_t* __restrict__ chunks, int c0,
                                                                  int ref_valid, float beta, Moments* __restrict__ part,
                                                                  double* __restrict__ part_seg,
                                                                  const float* __restrict__ slabs, int nsplit,
                                                                  int64_t seg_off, int64_t seg_n) {
    grad_partial_body<true>(g, ref, chunks, c0 + blockIdx.x, ref_valid, beta, part, part_seg, slabs, nsplit, seg_off,
                            seg_n);
}

// One workgroup per segment: each lane merges a fixed strided set of the segment's chunks (Chan /
// Pebay, fixed order), then a fixed-order block merge — deterministic.  (One wave per segment left
// the 6k-chunk embedding segment to 64 lanes and put an ~85 us serial merge on the step's tail.)
__global__ __launch_bounds__(256) void grad_segment_kernel(const Moments* __restrict__ part,
                                                           const double* __restrict__ part_seg,
                                                           const int* __restrict__ seg_first, int S, int ref_valid,
                                                           float* __restrict__ out, Moments* __restrict__ seg,
                                                           float* __restrict__ nonfinite) {
    __shared__ Moments sh[16];
    __shared__ double red[5][4];
    const int sg = blockIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    Moments m;
    m.n = 0.0; m.mean = m.m2 = m.m3 = m.m4 = 0.0; m.mn = INFINITY; m.mx = -INFINITY; m.abssum = 0.0;
    double a[5] = {0.0, 0.0, 0.0, 0.0, 0.0};   // sq, dot, rsq, bad, sq over the reference-tracked chunks
    for (int c = seg_first[sg] + threadIdx.x; c < seg_first[sg + 1]; c += blockDim.x) {
        merge(m, part[c]);
#pragma unroll
        for (int k = 0; k < 5; ++k) a[k] += part_seg[5 * c + k];
    }
    m = block_merge(m, sh);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        a[k] = wave_sum_d(a[k]);
        if (lane == 0) red[k][wid] = a[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) t[k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
        const double sq = t[0], dot = t[1], rsq = t[2], bad = t[3], sqt = t[4];
        const double den = sqrt(sqt * rsq);
        out[18 + sg] = (float)sqrt(sq);
        // no tracked chunk in this segment (or no reference yet): no cosine (sentinel 2)
        out[18 + S + sg] = !ref_valid ? 1.f : (den > 0.0 ? (float)(dot / den) : 2.f);
        seg[sg] = m;
        if (bad > 0) atomicAdd(nonfinite, (float)bad);  // integer counts: exact in any order
    }
}

// out layout: [0..11] tensor stats, [12] num_gradients, [13] grad_norms_mean, [14] grad_norms_std,
// [15] grad_norms_max, [16] cosine_similarity, [17] nonfinite, [18 .. 18+S) norms, [18+S .. 18+2S) cos.
__global__ __launch_bounds__(256) void grad_summary_kernel(const Moments* __restrict__ seg, int S,
                                                           float* __restrict__ out, float* __restrict__ range,
                                                           unsigned* __restrict__ hist, const float* __restrict__ nonfinite) {
    __shared__ Moments sh[16];
    __shared__ float red[16];
    Moments m;
    m.n = 0.0; m.mean = m.m2 = m.m3 = m.m4 = 0.0; m.mn = INFINITY; m.mx = -INFINITY; m.abssum = 0.0;
    for (int i = threadIdx.x; i < S; i += blockDim.x) merge(m, seg[i]);
    Moments r = block_merge(m, sh);
    if (threadIdx.x == 0) write_moment_stats(r, out, range);
    for (int i = threadIdx.x; i < NHIST; i += blockDim.x) hist[i] = 0u;
    const float* norms = out + 18;
    const float* coss = out + 18 + S;
    float nsum = 0.f, nsq = 0.f, nmax = 0.f, csum = 0.f, cn = 0.f;
    for (int sgi = threadIdx.x; sgi < S; sgi += blockDim.x) {
        const float nrm = norms[sgi];
        nsum += nrm;
        nsq += nrm * nrm;
        nmax = fmaxf(nmax, nrm);
        if (coss[sgi] <= 1.5f) {
            csum += coss[sgi];
            cn += 1.f;
        }
    }
    nsum = block_sum(nsum, red);
    nsq = block_sum(nsq, red);
    csum = block_sum(csum, red);
    cn = block_sum(cn, red);
    nmax = block_max(nmax, red);
    if (threadIdx.x == 0) {
        const float mean = nsum / S;
        out[12] = (float)S;
        out[13] = mean;
        out[14] = sqrtf(fmaxf(nsq / S - mean * mean, 0.f));
        out[15] = nmax;
        out[16] = cn > 0.f ? csum / cn : 1.f;
        out[17] = nonfinite[0];
    }
}

// Partial pass over chunks [c0, c1) (any order of disjoint ranges; every chunk exactly once per step).
TDL_API int tdl_grad_stats_partial(const float* g, float* ref, const int64_t* table, int C, int S, int c0, int c1,
                                   float beta, void* ws, int ref_valid, hipStream_t s) {
    if (c0 < 0 || c1 > C || c0 > c1) return (int)hipErrorInvalidValue;
    if (c1 == c0) return 0;
    GradWs w = grad_ws(ws, C, S);
    grad_partial_kernel<<<c1 - c0, 256, 0, s>>>((float*)g, ref, table, c0, ref_valid, beta, w.part, w.part_seg);
    TDL_LAUNCH_CHECK();
}

// Split-K reduce of one segment's weight gradient fused with its partial pass: chunks [c0, c1) must
// be exactly the chunks of the segment starting at flat offset seg_off (seg_n elements), slabs =
// [nsplit][seg_n] fp32.  g[seg_off ..] += sum of the slabs, statistics from the summed values.
TDL_API int tdl_grad_stats_reduce_partial(float* g, const float* slabs, int nsplit, long long seg_off, long long seg_n,
                                          float* ref, const int64_t* table, int C, int S, int c0, int c1, float beta,
                                          void* ws, int ref_valid, hipStream_t s) {
    if (c0 < 0 || c1 > C || c0 >= c1 || nsplit < 1) return (int)hipErrorInvalidValue;
    if ((seg_off & 3) || (seg_n & 3) || ((uintptr_t)g & 15) || ((uintptr_t)slabs & 15)) return (int)hipErrorInvalidValue;
    GradWs w = grad_ws(ws, C, S);
    grad_reduce_partial_kernel<<<c1 - c0, 256, 0, s>>>(g, ref, table, c0, ref_valid, beta, w.part, w.part_seg, slabs,
                                                       nsplit, seg_off, seg_n);
    TDL_LAUNCH_CHECK();
}

// Segment + summary (+ histogram quantiles) after every chunk's partial has run.
TDL_API int tdl_grad_stats_final(const float* g, const int64_t* table, int C, float* out, int64_t n, int S, void* ws,
                                 int ref_valid, int with_quantiles, hipStream_t s) {
    GradWs w = grad_ws(ws, C, S);
    const int* seg_first = (const int*)(table + 3 * (size_t)C);
    hipMemsetAsync(w.nonfinite, 0, sizeof(float) * 2, s);
    grad_segment_kernel<<<S, 256, 0, s>>>(w.part, w.part_seg, seg_first, S, ref_valid, out, w.seg,
                                                    w.nonfinite);
    grad_summary_kernel<<<1, 256, 0, s>>>(w.seg, S, out, w.range, w.hist, w.nonfinite);
    if (with_quantiles) {
        const int hg = stat_grid(n);
        hist_kernel<<<hg, 256, 0, s>>>(g, 0, n, w.range, w.hist);
        quantile_kernel<<<1, 256, 0, s>>>(w.hist, w.range, out);
    }
    TDL_LAUNCH_CHECK();
}

TDL_API int tdl_grad_stats(const float* g, float* ref, const int64_t* table, int C, float* out, int64_t n, float beta,
                           int S, void* ws, int ref_valid, int with_quantiles, hipStream_t s) {
    int rc = tdl_grad_stats_partial(g, ref, table, C, S, 0, C, beta, ws, ref_valid, s);
    if (rc) return rc;
    return tdl_grad_stats_final(g, table, C, out, n, S, ws, ref_valid, with_quantiles, s);
}

// Bare clipping norm (verification off): sum over segments of w_s * ||g_s||^2, deterministic.
// One block per chunk writes its weighted partial; one block sums them in a fixed order.
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const float* __restrict__ g, const int64_t* __restrict__ chunks,
                                                            const float* __restrict__ seg_w, double* __restrict__ part) {
    __shared__ float red[16];
    const int c = blockIdx.x;
    const int64_t start = chunks[3 * c + 1], end = chunks[3 * c + 2];
    const int sgi = (int)chunks[3 * c];
    float sq = 0.f;
    int64_t vbeg = (start + 3) & ~(int64_t)3;
    if (vbeg > end) vbeg = end;
    const int64_t vend = vbeg + ((end - vbeg) & ~(int64_t)3);
    for (int64_t i = start + threadIdx.x; i < vbeg; i += blockDim.x) sq += g[i] * g[i];
    for (int64_t i = vbeg + 4 * (int64_t)threadIdx.x; i < vend; i += 4 * (int64_t)blockDim.x) {
        const float4 v = *(const float4*)(g + i);
        sq += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (int64_t i = vend + threadIdx.x; i < end; i += blockDim.x) sq += g[i] * g[i];
    sq = block_sum(sq, red);
    if (threadIdx.x == 0) part[c] = (double)sq * (double)seg_w[sgi];
}

__global__ __launch_bounds__(256) void sumsq_final_kernel(const double* __restrict__ part, int C, float* __restrict__ out) {
    __shared__ double sh[4];
    double v = 0.0;
    for (int i = threadIdx.x; i < C; i += blockDim.x) v += part[i];
    v = wave_sum_d(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) out[0] = (float)(sh[0] + sh[1] + sh[2] + sh[3]);
}

TDL_API int tdl_grad_sumsq(const float* g, const int64_t* table, int C, const float* seg_w, double* ws, float* out,
                           hipStream_t s) {
    if (C <= 0) return (int)hipErrorInvalidValue;
    sumsq_partial_kernel<<<C, 256, 0, s>>>(g, table, seg_w, ws);
    sumsq_final_kernel<<<1, 256, 0, s>>>(ws, C, out);
    TDL_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ K4 z-score detection
// ring: f32 [H][K] history; state: int32 [4] = (count, head, quarantine_run, seen)
// cur: f32 [K]; out: f32 [4 + K] = (flag, mean_z, confidence, n_valid, z_0..z_{K-1}; z = -1 if skipped)
// Exact order statistic of v[0..n) (n <= 128, one wave): value of rank `r` (0-based).
__device__ float wave_select(const float* v, int n, int r, int lane) {
    float found = 0.f;
    for (int i = lane; i < n; i += 64) {
        const float vi = v[i];
        int lt = 0, eq_before = 0;
        for (int j = 0; j < n; ++j) {
            const float vj = v[j];
            lt += vj < vi;
            eq_before += (vj == vi) && (j < i);
        }
        if (lt + eq_before == r) found = vi;
    }
    // exactly one lane holds rank r; others hold 0 -> take the sum
    return wave_sum(found);
}

// robust = 1: baseline over the `window` most recent entries, center = median, scale = 1.4826 * MAD
//             (robust to earlier attacked samples);
// robust = 2: as 1 about a robust linear trend of the window (the drift of real training), with the
//             scale floored at abs_floor + rel_floor * |center|;
// robust = 0: reference mean / population std over the whole history window.
// robust | 4: the decision statistic is the largest per-feature |z| (targeted feature sets) instead
//             of the mean over features (the reference's 17-feature rule).
__device__ __forceinline__ float wave_median(const float* v, int n, int lane) {
    return (n & 1) ? wave_select(v, n, n / 2, lane)
                   : 0.5f * (wave_select(v, n, n / 2 - 1, lane) + wave_select(v, n, n / 2, lane));
}

constexpr int ZS_EARLY_MIN = 8;
constexpr float ZS_EARLY_FACTOR = 3.f;

__global__ __launch_bounds__(256) void zscore_kernel(float* __restrict__ ring, int* __restrict__ state,
                                                     const float* __restrict__ cur, int K, int H, int warmup,
                                                     float z_decision, int window, int exclude_current,
                                                     int max_quarantine, int robust, float rel_floor,
                                                     float abs_floor, float* __restrict__ out) {
    __shared__ float zs[64];
    __shared__ float col[4][128];
    __shared__ int cnt_sh;
    const bool agg_max = (robust & 4) != 0;  // decision on the largest |z| instead of the mean
    // early gate (bit 8): during warm-up, once ZS_EARLY_MIN entries exist, a gross outlier (largest
    // |z| > ZS_EARLY_FACTOR x z_decision) is flagged and kept out of the baseline — otherwise an
    // attack that is already running while a baseline (re)builds (a stage re-planned after a
    // re-shard) is learnt as normal and masks its later injections
    const bool early_gate = (robust & 8) != 0;
    robust &= 3;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int count = state[0], head = state[1];
    if (!exclude_current) {  // reference order: append, then baseline over the window incl. current
        __syncthreads();
        for (int k = threadIdx.x; k < K; k += blockDim.x) ring[(size_t)head * K + k] = cur[k];
        __syncthreads();
        head = (head + 1) % H;
        count = count < H ? count + 1 : H;
    }
    const bool ready = count >= warmup;
    const bool early = !ready && early_gate && robust && count >= ZS_EARLY_MIN;
    const int wn = robust ? (count < window ? count : window) : count;
    for (int k = wid; k < K; k += 4) {
        float center, scale;
        if (robust) {
            float* v = col[wid];
            for (int j = lane; j < wn; j += 64) {
                const int idx = ((head - 1 - j) % H + H) % H;  // most recent first
                v[j] = ring[(size_t)idx * K + k];
            }
            __builtin_amdgcn_wave_barrier();
            float trend0 = 0.f;
            if (robust == 2 && wn >= 8) {
                // detrended baseline: a robust line through the medians of the recent and the older
                // half of the window (slope per step); residuals about it give centre and scale, and
                // the centre is the line's prediction for the current step.  A gradient statistic
                // that drifts smoothly as the model learns is then not an outlier; a jump is.
                const int h = wn / 2;
                const float mr = wave_median(v, h, lane);
                const float mo = wave_median(v + h, h, lane);
                const float slope = (mr - mo) / (float)h;
                const float tr = -1.f - 0.5f * (float)(h - 1);
                __builtin_amdgcn_wave_barrier();
                for (int j = lane; j < wn; j += 64) v[j] -= mr + slope * ((float)(-1 - j) - tr);
                __builtin_amdgcn_wave_barrier();
                trend0 = mr + slope * (0.f - tr);
            }
            const float med = wave_median(v, wn, lane);
            __builtin_amdgcn_wave_barrier();
            for (int j = lane; j < wn; j += 64) v[j] = fabsf(v[j] - med);
            __builtin_amdgcn_wave_barrier();
            const float mad = wave_median(v, wn, lane);
            __builtin_amdgcn_wave_barrier();
            center = trend0 + med;
            scale = 1.4826f * mad;
            if (robust == 2 && scale > 0.f) scale = fmaxf(scale, abs_floor + rel_floor * fabsf(center));
        } else {
            float s = 0.f;
            for (int h = lane; h < count; h += 64) s += ring[(size_t)h * K + k];
            const float mean = wave_sum(s) / (count > 0 ? count : 1);
            float q = 0.f;
            for (int h = lane; h < count; h += 64) {
                const float d = ring[(size_t)h * K + k] - mean;
                q += d * d;
            }
            center = mean;
            scale = sqrtf(wave_sum(q) / (count > 0 ? count : 1));
        }
        if (lane == 0) {
            float z = -1.f;
            if ((ready || early) && scale > 0.f) {
                const float c = cur[k];
                z = isfinite(c) ? fabsf((c - center) / scale) : 1e6f;
            }
            zs[k] = z;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float sum = 0.f, mx = 0.f;
        int nv = 0;
        for (int k = 0; k < K; ++k)
            if (zs[k] >= 0.f) { sum += zs[k]; mx = fmaxf(mx, zs[k]); ++nv; }
        const float mz = agg_max ? mx : (nv ? sum / nv : 0.f);
        const bool flag = ready ? mz > z_decision : (early && mz > ZS_EARLY_FACTOR * z_decision);
        out[0] = flag ? 1.f : 0.f;
        out[1] = mz;
        out[2] = fminf(1.f, mz / 5.f);
        out[3] = (float)nv;
        int appended = 0;
        if (exclude_current) {
            if (flag && state[2] < max_quarantine) {
                state[2] += 1;
            } else {
                state[2] = 0;
                appended = 1;
            }
        }
        cnt_sh = appended;
        state[3] += 1;
    }
    for (int k = threadIdx.x; k < K; k += blockDim.x) out[4 + k] = zs[k];
    __syncthreads();
    if (exclude_current && cnt_sh) {
        for (int k = threadIdx.x; k < K; k += blockDim.x) ring[(size_t)head * K + k] = cur[k];
        head = (head + 1) % H;
        count = count < H ? count + 1 : H;
    }
    if (threadIdx.x == 0) {
        state[0] = count;
        state[1] = head;
    }
}

TDL_API int tdl_zscore_detect(float* ring, int* state, const float* cur, int K, int H, int warmup, float z_decision,
                              int window, int exclude_current, int max_quarantine, int robust, float rel_floor,
                              float abs_floor, float* out, hipStream_t s) {
    if (K > 64 || ((robust & 3) && window > 128)) return (int)hipErrorInvalidValue;
    zscore_kernel<<<1, 256, 0, s>>>(ring, state, cur, K, H, warmup, z_decision, window, exclude_current,
                                    max_quarantine, robust, rel_floor, abs_floor, out);
    TDL_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ K5 trust update
// status codes: 0 TRUSTED, 1 SUSPICIOUS, 2 COMPROMISED, 3 RECOVERING, 4 OFFLINE
__global__ void trust_update_kernel(float* __restrict__ values, int* __restrict__ counts, int* __restrict__ status,
                                    const float* __restrict__ metrics, const float* __restrict__ w,
                                    const int* __restrict__ flags, const float* __restrict__ recovery, int N, float thr,
                                    float decay_rate, float dt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    int st = status[i];
    if (st == 4) return;  // OFFLINE: frozen until the runtime re-admits the node
    float old = values[i];
    if (flags && flags[i]) {  // detection => mark_compromised (trust_manager.py:183-196)
        st = 2;
        old = 0.1f;
    }
    const float* m = metrics + 6 * i;
    const float comp[6] = {1.f - fminf(1.f, m[0]), m[1], 1.f - fminf(1.f, m[2] / 10.f), fminf(1.f, m[3]),
                           1.f - fminf(1.f, m[4]), m[5]};
    float score = 0.f;
    for (int k = 0; k < 6; ++k) score += w[k] * comp[k];
    score = fminf(1.f, fmaxf(0.f, score));
    const float decay = expf(-decay_rate * dt);
    float fin = 0.9f * old * decay + 0.1f * score;
    if (st == 3 && recovery) fin += recovery[i];
    fin = fminf(1.f, fmaxf(0.f, fin));
    int ns;
    if (fin < 0.3f) ns = 2;
    else if (fin < thr) ns = 1;
    else if (st == 2 && fin > 0.8f) ns = 3;
    else if (st == 3 && fin > 0.9f) ns = 0;
    else ns = 0;  // fin >= thr
    values[i] = fin;
    status[i] = ns;
    counts[i] += 1;
}

TDL_API int tdl_trust_update(float* values, int* counts, int* status, const float* metrics, const float* weights,
                             const int* flags, const float* recovery, int N, float thr, float decay_rate, float dt,
                             hipStream_t s) {
    trust_update_kernel<<<(N + 63) / 64, 64, 0, s>>>(values, counts, status, metrics, weights, flags, recovery, N, thr,
                                                     decay_rate, dt);
    TDL_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ K6 stage-verifier step tail
// security/stage_verifier.py StageVerifier.finish_step, fused: everything the verifier does after
// the statistics and detector kernels — digest row, output-deviation and gradient-consistency trust
// metrics, the two EMA baselines, the sign-flip rule, quarantine control and the clipping sum of
// squares — in ONE launch.  The torch form (kept for CPU and as TDL_VERIFY_FUSED=0) issued ~110
// element-sized kernels per stage and step, ~0.55 ms of the GPT-2-small step's 1.2 ms verification
// overhead (bench --trace-phases: verify 1.06 vs 0.42 ms).  Host values (stage id, the four runtime
// metrics, the ground-truth bit) travel as kernel arguments, so no host-to-device copy either.
// Digest slots: security/stage_verifier.py (D_*).
struct VerifyFinishArgs {
    float* d;
    const float* loss;          // [1] or null
    int stage_id;
    int out_on;                 // output statistics observed this step (and output detection on)
    const float* out_res;       // output detector [flag, z, conf, ...]
    const float* out_stats;     // [13]: 0 mean, 1 std, 12 non-finite count
    float* out_mu;
    float* out_sd;
    float* out_n;
    float warmup, deadzone, beta;
    int grad_mode;              // 0: no gradient statistics, 1: bare (sum of squares only), 2: full
    const float* sumsq_bare;    // mode 1: [1]
    const float* g;             // mode 2: grad statistics [18 + 2 S]
    int S;
    const float* clip_w;        // [S]
    int gdet;                   // gradient detector ran this step
    const float* grad_res;      // its [flag, z, conf, ...]
    int targeted;               // sign-flip rule on (targeted feature set)
    float sign_flip_cos;
    float* norm_ema;            // [S]
    float* norm_n;
    float tol;
    int symmetric;
    float hm0, hm1, hm2, hm3;   // latency, utilization, error, uptime (host, one step lagged)
    int truth;
    int quarantine;
    float* ctrl;                // [2]: clip scale (not touched here), skip
};

enum {
    VD_LOSS = 0, VD_OUT_FLAG = 1, VD_OUT_Z = 2, VD_GRAD_FLAG = 3, VD_GRAD_Z = 4, VD_METRICS = 5, VD_GRAD_SUMSQ = 11,
    VD_OUT_MEAN = 12, VD_OUT_STD = 13, VD_GRAD_L2 = 14, VD_NONFINITE = 15, VD_GRAD_COS = 16, VD_ATTACK_TRUTH = 17,
    VD_PRESENT = 18, VD_STAGE = 19, VD_OUT_CONF = 20, VD_GRAD_CONF = 21,
    VD_DIGEST = 115  // security/stage_verifier.py DIGEST
};

__global__ __launch_bounds__(256) void verify_finish_kernel(VerifyFinishArgs a) {
    __shared__ float red[16];
    __shared__ float sh_keep_g, sh_b_g;
    const int t = threadIdx.x;
    float* d = a.d;
    for (int i = t; i < VD_DIGEST; i += 256) d[i] = 0.f;
    // gradient flag (needed by every thread for the EMA update): detector flag, sign-flip rule
    float gflag = 0.f;
    const bool full = a.grad_mode == 2;
    if (full && a.gdet) {
        gflag = a.grad_res[0];
        if (a.targeted) {
            const float warm = a.norm_n[0] >= a.warmup ? 1.f : 0.f;
            gflag = fmaxf(gflag, (a.g[16] < a.sign_flip_cos ? 1.f : 0.f) * warm);
        }
    }
    // per-parameter reductions over the pre-update EMA: clipping sum of squares, consistency
    float sq = 0.f, cs = 0.f, nv = 0.f;
    if (full) {
        for (int i = t; i < a.S; i += 256) {
            const float nrm = a.g[18 + i];
            const float ema = a.norm_ema[i];
            sq += nrm * nrm * a.clip_w[i];
            const float r = nrm / fmaxf(ema, 1e-30f);
            float sc = a.symmetric ? fminf(r, 1.f / fmaxf(r, 1e-30f)) : fminf(r, 1.f);
            sc = fminf(sc * a.tol, 1.f);
            const float valid = ema > 0.f ? 1.f : 0.f;
            cs += sc * valid;
            nv += valid;
        }
        sq = block_sum(sq, red);
        cs = block_sum(cs, red);
        nv = block_sum(nv, red);
    }
    __syncthreads();   // digest zeroed by every thread before thread 0 writes it
    if (t == 0) {
        d[VD_PRESENT] = 1.f;
        d[VD_STAGE] = (float)a.stage_id;
        if (a.loss) d[VD_LOSS] = a.loss[0];
        float nonfin = 0.f;
        if (a.out_on) {
            const float flag = a.out_res[0];
            d[VD_OUT_FLAG] = flag;
            d[VD_OUT_Z] = a.out_res[1];
            d[VD_OUT_CONF] = a.out_res[2];
            const float mu = a.out_stats[0], sd = a.out_stats[1];
            d[VD_OUT_MEAN] = mu;
            d[VD_OUT_STD] = sd;
            const float omu = a.out_mu[0], osd = a.out_sd[0], on = a.out_n[0];
            const float ready = on >= a.warmup ? 1.f : 0.f;
            float dev = fminf((fabsf(mu - omu) + fabsf(sd - osd)) / (2.f * fmaxf(osd, 1e-12f)), 1.f);
            dev = fmaxf(dev - a.deadzone, 0.f) / (1.f - a.deadzone);
            d[VD_METRICS + 0] = dev * ready;
            const float keep = 1.f - flag;
            const float first = on == 0.f ? 1.f : 0.f;
            const float b = a.beta * (1.f - first);
            a.out_mu[0] = keep * (b * omu + (1.f - b) * mu) + (1.f - keep) * omu;
            a.out_sd[0] = keep * (b * osd + (1.f - b) * sd) + (1.f - keep) * osd;
            a.out_n[0] = on + keep;
            nonfin += a.out_stats[12];
        }
        if (a.grad_mode == 1) {
            d[VD_GRAD_SUMSQ] = a.sumsq_bare[0];
            d[VD_METRICS + 1] = 1.f;
        } else if (full) {
            d[VD_GRAD_L2] = a.g[10];
            d[VD_GRAD_COS] = a.g[16];
            nonfin += a.g[17];
            if (a.gdet) {
                d[VD_GRAD_FLAG] = gflag;
                d[VD_GRAD_Z] = a.grad_res[1];
                d[VD_GRAD_CONF] = a.grad_res[2];
            }
            const float ready = a.norm_n[0] >= a.warmup ? 1.f : 0.f;
            const float cons = cs / fmaxf(nv, 1.f);
            d[VD_METRICS + 1] = ready * cons + (1.f - ready) * 1.f;
        } else {
            d[VD_METRICS + 1] = 1.f;
        }
        d[VD_NONFINITE] = nonfin;
        d[VD_METRICS + 2] = a.hm0;
        d[VD_METRICS + 3] = a.hm1;
        d[VD_METRICS + 4] = fminf(a.hm2 + (nonfin > 0.f ? 1.f : 0.f), 1.f);
        d[VD_METRICS + 5] = a.hm3;
        d[VD_ATTACK_TRUTH] = a.truth ? 1.f : 0.f;
        float skip = 0.f;
        if (a.quarantine && full && a.gdet) skip = fmaxf(gflag, nonfin > 0.f ? 1.f : 0.f);
        a.ctrl[1] = skip;
        if (full) d[VD_GRAD_SUMSQ] = sq * (1.f - skip);
        const float keep = 1.f - gflag;
        const float first = full ? (a.norm_n[0] == 0.f ? 1.f : 0.f) : 0.f;
        sh_keep_g = keep;
        sh_b_g = a.beta * (1.f - first);
    }
    __syncthreads();
    if (full) {
        const float keep = sh_keep_g, b = sh_b_g;
        for (int i = t; i < a.S; i += 256) {
            const float ema = a.norm_ema[i], nrm = a.g[18 + i];
            a.norm_ema[i] = keep * (b * ema + (1.f - b) * nrm) + (1.f - keep) * ema;
        }
        if (t == 0) a.norm_n[0] += keep;
    }
}

// targeted detector features (security/stage_verifier.py _out_features / _grad_features):
// out: [mean, log std, log |max|], grad: [log ||g||, log max per-parameter norm, log element std]
__global__ void verify_features_kernel(const float* __restrict__ o, const float* __restrict__ g, float* __restrict__ of,
                                       float* __restrict__ gf) {
    if (threadIdx.x != 0) return;
    if (o) {
        of[0] = o[0];
        of[1] = logf(fmaxf(o[1], 1e-30f));
        of[2] = logf(fmaxf(o[11], 1e-30f));
    }
    if (g) {
        gf[0] = logf(fmaxf(g[10], 1e-30f));
        gf[1] = logf(fmaxf(g[15], 1e-30f));
        gf[2] = logf(fmaxf(g[1], 1e-30f));
    }
}

TDL_API int tdl_verify_features(const float* o, const float* g, float* of, float* gf, hipStream_t s) {
    verify_features_kernel<<<1, 64, 0, s>>>(o, g, of, gf);
    TDL_LAUNCH_CHECK();
}

TDL_API int64_t tdl_verify_args_bytes() { return (int64_t)sizeof(VerifyFinishArgs); }

TDL_API int tdl_verify_finish(const VerifyFinishArgs* args, hipStream_t s) {
    verify_finish_kernel<<<1, 256, 0, s>>>(*args);
    TDL_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ K7 KL(softmax(b) || softmax(a)), batchmean
// a, b: f32 [R, C]; out f32 [1] (accumulated with atomics; caller zeroes).  One block per row.
__global__ __launch_bounds__(256) void kl_kernel(const float* __restrict__ a, const float* __restrict__ b, int R, int C,
                                                 float* __restrict__ out) {
    __shared__ float red[16];
    const int row = blockIdx.x;
    const float* ar = a + (size_t)row * C;
    const float* br = b + (size_t)row * C;
    float ma = -INFINITY, mb = -INFINITY;
    for (int j = threadIdx.x; j < C; j += 256) { ma = fmaxf(ma, ar[j]); mb = fmaxf(mb, br[j]); }
    ma = block_max(ma, red);
    mb = block_max(mb, red);
    float sa = 0.f, sb = 0.f;
    for (int j = threadIdx.x; j < C; j += 256) { sa += __expf(ar[j] - ma); sb += __expf(br[j] - mb); }
    sa = block_sum(sa, red);
    sb = block_sum(sb, red);
    const float lsa = ma + __logf(sa), lsb = mb + __logf(sb);
    float kl = 0.f;
    for (int j = threadIdx.x; j < C; j += 256) {
        const float lq = br[j] - lsb;  // log target prob
        kl += __expf(lq) * (lq - (ar[j] - lsa));
    }
    kl = block_sum(kl, red);
    if (threadIdx.x == 0) atomicAdd(out, kl / R);
}

TDL_API int tdl_kl_div_softmax(const float* a, const float* b, int R, int C, float* out, hipStream_t s) {
    hipMemsetAsync(out, 0, sizeof(float), s);
    kl_kernel<<<R, 256, 0, s>>>(a, b, R, C, out);
    TDL_LAUNCH_CHECK();
}

// ============================================================================ parameter integrity
// Deterministic checksum of a bf16 weight buffer: (sum, sum of squares, position-weighted sum) in
// fp64.  Element -> block assignment, per-thread order and both reduction trees are fixed, so bit-
// identical data gives a bit-identical checksum: the engine compares the checksum of a stage's
// compute weights taken right after its optimizer step with the one taken before the next update —
// any write outside the optimizer (parameter perturbation, memory corruption) shows up.
namespace {
constexpr int CK_BLOCKS = 2048;  // 8 blocks per CU

__global__ __launch_bounds__(256) void checksum_partial_kernel(const bf16_t* __restrict__ x, int64_t n,
                                                               int64_t per_block, double* __restrict__ part) {
    __shared__ double red[3][4];
    const int64_t beg = (int64_t)blockIdx.x * per_block;
    const int64_t end = beg + per_block < n ? beg + per_block : n;
    double s = 0.0, q = 0.0, w = 0.0;
    // position weight (i % 1021) + 1, carried incrementally: one 64-bit modulo per thread, then
    // +2048 elements per iteration = +6 (mod 1021) — a per-element int64 modulo was the cost
    int r = (int)((beg + threadIdx.x * 8) % 1021);
    auto acc8 = [&](const float (&f)[8]) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const double v = (double)f[e];
            const int re = r + e;
            s += v;
            q += v * v;
            w += v * (double)(re < 1021 ? re + 1 : re - 1020);
        }
        r += 2048 - 2 * 1021;
        if (r >= 1021) r -= 1021;
    };
    int64_t i = beg + threadIdx.x * 8;
    // four 16-B loads in flight per lane per trip (one at a time left the pass latency-bound); the
    // vectors are then summed in the same per-lane order as before: bit-identical results
    for (; i + 3 * 2048 + 8 <= end; i += 4 * 2048) {
        uint4 qv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) qv[u] = *(const uint4*)(x + i + u * 2048);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float f[8];
            unpack8(qv[u], f);
            acc8(f);
        }
    }
    for (; i < end; i += 256 * 8) {
        float f[8];
        if (i + 8 <= end) {
            unpack8(*(const uint4*)(x + i), f);
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = i + e < end ? bf2f(x[i + e]) : 0.f;
        }
        acc8(f);
    }
    s = wave_sum_d(s);
    q = wave_sum_d(q);
    w = wave_sum_d(w);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red[0][wid] = s;
        red[1][wid] = q;
        red[2][wid] = w;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const double* r = red[threadIdx.x];
        part[(int64_t)blockIdx.x * 3 + threadIdx.x] = ((r[0] + r[1]) + r[2]) + r[3];
    }
}

// Fixed-shape reduction of the per-block partials (256 threads, contiguous runs per thread, then
// wave / cross-wave sums in a fixed order): deterministic for a given nb.
__global__ __launch_bounds__(256) void checksum_final_kernel(const double* __restrict__ part, int nb,
                                                             double* __restrict__ out) {
    __shared__ double red[3][4];
    const int per = (nb + 255) / 256;
    double a[3] = {0.0, 0.0, 0.0};
    for (int b = threadIdx.x * per; b < (threadIdx.x + 1) * per && b < nb; ++b) {
#pragma unroll
        for (int k = 0; k < 3; ++k) a[k] += part[b * 3 + k];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        a[k] = wave_sum_d(a[k]);
        if (lane == 0) red[k][wid] = a[k];
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const double* r = red[threadIdx.x];
        out[threadIdx.x] = ((r[0] + r[1]) + r[2]) + r[3];
    }
}
}  // namespace

// out: 3 doubles; ws: 3 * 2048 doubles.  n bf16 elements, 16-byte aligned base.
TDL_API int tdl_checksum_bf16(const void* x, int64_t n, double* ws, double* out, hipStream_t s) {
    if (((uintptr_t)x & 15) != 0) return (int)hipErrorInvalidValue;
    int64_t per_block = (n + CK_BLOCKS - 1) / CK_BLOCKS;
    per_block = (per_block + 7) / 8 * 8;
    const int nb = (int)((n + per_block - 1) / per_block);
    checksum_partial_kernel<<<nb > 0 ? nb : 1, 256, 0, s>>>((const bf16_t*)x, n, per_block, ws);
    checksum_final_kernel<<<1, 256, 0, s>>>(ws, nb > 0 ? nb : 1, out);
    TDL_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ K6 cosine Gram matrix
// N x N cosine similarity of N flat vectors of length D (node output digests / replica sketches,
// attack_detector.py:143-162 + 365-379), N <= 16, read IN PLACE through a pointer table (no
// stacked copy).  Phase 1: every block takes a strided share of D and accumulates all N(N+1)/2
// pair dot products in fp64 registers-per-thread, block-reduced in a fixed order into its slot of
// `part`.  Phase 2: one block sums the slots per pair in block order and normalises.  Deterministic.
#define GRAM_MAXN 16
#define GRAM_PAIRS (GRAM_MAXN * (GRAM_MAXN + 1) / 2)
struct GramPtrs {
    const void* p[GRAM_MAXN];
};

__global__ __launch_bounds__(256) void gram_partial_kernel(GramPtrs ptrs, int N, int64_t D, int dtype,
                                                           double* __restrict__ part) {
    __shared__ double red[4];
    const int npairs = N * (N + 1) / 2;
    for (int pr = 0; pr < npairs; ++pr) {
        // pair index -> (i, j), i <= j
        int i = 0, rem = pr;
        while (rem >= N - i) { rem -= N - i; ++i; }
        const int j = i + rem;
        double acc = 0.0;
        for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < D; k += (int64_t)gridDim.x * blockDim.x) {
            const float a = dtype == 1 ? bf2f(((const bf16_t*)ptrs.p[i])[k]) : ((const float*)ptrs.p[i])[k];
            const float b = dtype == 1 ? bf2f(((const bf16_t*)ptrs.p[j])[k]) : ((const float*)ptrs.p[j])[k];
            acc += (double)a * (double)b;
        }
        acc = wave_sum_d(acc);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0) part[(size_t)blockIdx.x * GRAM_PAIRS + pr] = red[0] + red[1] + red[2] + red[3];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void gram_final_kernel(const double* __restrict__ part, int nblk, int N,
                                                         float* __restrict__ out) {
    __shared__ double dots[GRAM_PAIRS];
    const int npairs = N * (N + 1) / 2;
    for (int pr = threadIdx.x; pr < npairs; pr += blockDim.x) {
        double s = 0.0;
        for (int b = 0; b < nblk; ++b) s += part[(size_t)b * GRAM_PAIRS + pr];
        dots[pr] = s;
    }
    __syncthreads();
    for (int pr = threadIdx.x; pr < npairs; pr += blockDim.x) {
        int i = 0, rem = pr;
        while (rem >= N - i) { rem -= N - i; ++i; }
        const int j = i + rem;
        auto diag = [&](int a) { return a * N - a * (a - 1) / 2; };  // pair index of (a, a)
        const double den = sqrt(dots[diag(i)] * dots[diag(j)]);
        const float c = den > 0.0 ? (float)(dots[pr] / den) : 0.f;
        out[i * N + j] = c;
        out[j * N + i] = c;
    }
}

TDL_API int64_t tdl_gram_ws_bytes() { return (int64_t)sizeof(double) * 512 * GRAM_PAIRS; }

TDL_API int tdl_cosine_gram(const void* const* ptrs, int N, int64_t D, int dtype, float* out, void* ws, hipStream_t s) {
    if (N < 1 || N > GRAM_MAXN || D <= 0) return (int)hipErrorInvalidValue;
    GramPtrs gp{};
    for (int i = 0; i < N; ++i) gp.p[i] = ptrs[i];
    int64_t nb = (D + 256 * 8 - 1) / (256 * 8);
    const int nblk = (int)(nb < 1 ? 1 : (nb > 512 ? 512 : nb));
    gram_partial_kernel<<<nblk, 256, 0, s>>>(gp, N, D, dtype, (double*)ws);
    gram_final_kernel<<<1, 256, 0, s>>>((const double*)ws, nblk, N, out);
    TDL_LAUNCH_CHECK();
}
