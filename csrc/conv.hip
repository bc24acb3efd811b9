// Implicit-GEMM convolutions for the VGG / ResNet blocks, NHWC bf16, fp32 accumulate,
// gfx950 MFMA v_mfma_f32_32x32x16_bf16.  Replaces the MIOpen path the CNN stages used before.
//
// Layouts (torch channels_last == NHWC storage; weights [Cout][R][S][Cin] == KRSC, k = (r, s, c)
// with c fastest).  Cin % 8 == 0 so one 16-byte vector is 8 channels of one tap (the Python side
// pads the 3-channel stem input/weight to 8).
//
// conv_nt  — D[cout][m] = sum_k Wk[cout][k] * Act[m][k]   (both operands k-contiguous: "NT")
//   forward : Act[m=(n,p,q)][k=(r,s,c)] = X [n][p*st-pad+r][q*st-pad+s][c]          (0 outside)
//   dgrad   : Act[m=(n,h,w)][k=(r,s,k')] = dY[n][(h+pad-r)/st][(w+pad-s)/st][k']  (0 unless the
//             division is exact and in range) with Wk = W permuted to [Cin][R][S][Cout]
//   Workgroup tile BCO (cout: 64|128) x 128 (m), K step 64, 4 waves as 2 (cout) x 2 (m).  Both
//   operands are register-staged (global -> VGPR prefetch of tile t+1 while tile t computes, then
//   one LDS write + ONE barrier per K step), LDS rows of 128 B XOR-swizzled by (row>>1)&7 so the
//   ds_read_b128 fragment reads of a 32-lane half hit 16 distinct 16-byte slots.  The weight tile
//   is the MFMA A operand, so the accumulator has m on the lane and 4 consecutive output channels
//   per register group: the epilogue writes 8-byte NHWC vectors.  Optional fused epilogue: per
//   output-channel sum / sum-of-squares of the bf16-rounded outputs (BatchNorm batch statistics):
//   one partial row per workgroup (registers -> shuffles -> LDS), summed by a small finalize pass
//   (an earlier version issued per-wave same-address atomics: 4-8x slower forward, rocprof).
// conv_wgrad — dW[cout][k] = sum_m dY[m][cout] * Act[m][k]   (reduction over output pixels)
//   Both operands are m-major, so tiles are staged [32 m][cols] and read as MFMA fragments with
//   the gfx950 transposing LDS read ds_read_b64_tr_b16 (rows padded to 320 B: conflict-free).
//   Tile BCO x 128 (k), m step 32, split over m across grid.z; partial tiles are reduced into a
//   [Cout][R][S][Cin] fp32 image (lane-contiguous atomics when split > 1) and added to the
//   parameter's [Cout][Cin][R][S] gradient by one transpose pass (1x1: straight into it).
#include "common.h"

#include <math.h>
#include <mutex>
#include <unordered_map>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

namespace {

__device__ __forceinline__ bf16x8_t as_bf16x8(uint4 u) { return __builtin_bit_cast(bf16x8_t, u); }

__device__ __forceinline__ short4_t tr_read(const bf16_t* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(p));
}
__device__ __forceinline__ bf16x8_t tr_pair(const bf16_t* p_lo, const bf16_t* p_hi) {
    const short4_t a = tr_read(p_lo), b = tr_read(p_hi);
    const short8_t c = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, c);
}

// Bijective XCD-aware remap (cdna_hip_programming.md T1): consecutive logical tiles land on the
// same XCD (private L2), so the blocks that share an activation panel share its L2 lines.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

struct ConvDims {
    int N, Hin, Win, Cin;   // gathered tensor (X for fwd/wgrad, dY for dgrad), NHWC
    int P, Q, Cout;         // GEMM output: rows m = N*P*Q pixels, Cout channels (NHWC)
    int R, S, stride, pad;  // filter geometry of the FORWARD convolution
};

// Output-parity class of a strided data gradient: dX pixel (h, w) with h = h0 + cs i, w = w0 + cs j
// only receives the taps r = r0 + cs t (t < nr), s = s0 + cs u (u < ns), where r0 = (h0 + pad) mod cs
// (every other tap lands between dY pixels).  One launch per class runs a GEMM over exactly those
// taps instead of masking 3 of every 4 (stride 2) to zero inside the K loop.  The identity class
// (cs = 1, Ps = P, nr = R, ...) is the plain convolution.  row_off: first statistics partial row of
// the class (the classes of one call share one partial-row buffer and one finalize).
struct ConvCls {
    int Ps, Qs, h0, w0, r0, s0, nr, ns, cs, row_off;
};

constexpr int BM = 128;  // m (pixels) per workgroup
constexpr int FIN_CNT = 256;  // statistics-finalize arrival counters (column blocks of 64, 2 Cout <= 16384)
constexpr int BK = 64;   // k per step

// In-kernel statistics finalize.  The partial rows of a call are summed in a FIXED order (the
// recompute audit needs bit-identical statistics, see stats_finalize_kernel) by the workgroups that
// produce them, so no finalize launch sits between a convolution and its BatchNorm: rows are
// grouped by gs; the last workgroup (per column tile) to store a row of a group sums the group's
// rows into the group's first row, and the last group to finish adds the group totals in group
// order into stats (and acc_lo / acc_hi, see stats_finalize_kernel).  cnt: per-stream arrival
// counters, left at zero by the workgroups that consume them; tile t uses [t (ngroups + 1), ...).
// Training-mode BatchNorm finalize of the convolution's output (the BN folded into the next
// convolution, ops/conv.py): what bn.hip tdl_bn_finalize computes, done by the finishing workgroups
// (mean / rstd, running statistics, pro = [gamma * rstd | beta - mean * gamma * rstd], zeroed
// backward-sum row), so the next convolution follows without a finalize launch in between.
struct BnFin {
    const bf16_t *gamma, *beta;
    float *save_mean, *save_rstd, *upd_mean, *upd_var, *pro, *zero_sums;
    int64_t count;
    float eps, momentum;
};

struct FinArgs {
    unsigned* cnt;      // null: partial rows only (stats_finalize_kernel runs after)
    int gs, ngroups, rows, accumulate;
    float *stats, *acc_lo, *acc_hi;
    BnFin bn;           // bn.pro null: no BN finalize
};

// sum over q in [q0, q1) of p[q * step * ld], agent-scope loads, fixed order: 8 lanes of partial
// sums (q mod 8) added pairwise at the end
__device__ __forceinline__ float sum_rows(const float* p, int q0, int q1, int step, int ld) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int q = q0;
    for (; q + 8 <= q1; q += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            v[u] = __hip_atomic_load(p + (size_t)(q + u) * step * ld, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] += v[u];
    }
    for (int u = 0; q < q1; ++q, ++u)
        a[u] += __hip_atomic_load(p + (size_t)q * step * ld, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// Every thread of the workgroup calls this after its row's columns [c0, c0 + nc) of both halves
// (sum | sum of squares, row stride 2 Cout) were written with agent-scope stores.
__device__ __forceinline__ void stats_arrive(float* __restrict__ part, int Cout, int row, int c0, int nc, int tile,
                                             const FinArgs& f) {
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's row stores have landed
    __syncthreads();
    const int g = row / f.gs, r0 = g * f.gs, r1 = min(f.rows, r0 + f.gs);
    unsigned* gc = f.cnt + (size_t)tile * (f.ngroups + 1) + g;
    unsigned* cc = f.cnt + (size_t)tile * (f.ngroups + 1) + f.ngroups;
    // hand-off form (MI355X_MICROARCH.md, "Hand-offs measured with sc1 loads", row 1): every storing
    // wave drained its sc1 (agent-scope) stores, a workgroup barrier, ONE lane's agent-scope add;
    // the workgroup whose add came last reads the rows with sc1 loads after a barrier: no acquire
    // fence needed (and none of its ~1.7 us per workgroup)
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == (unsigned)(r1 - r0 - 1);
        if (last) __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    const int t = threadIdx.x;
    const int ch = c0 + (t < nc ? t : t - nc);
    const bool act = t < 2 * nc && ch < Cout;
    const size_t col = (size_t)(t < nc ? 0 : Cout) + ch;
    if (act)   // 8 independent loads in flight (a serial chain of agent-scope loads is latency-bound)
        __hip_atomic_store(part + (size_t)r0 * 2 * Cout + col, sum_rows(part + col, r0, r1, 1, 2 * Cout),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(cc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = prev == (unsigned)(f.ngroups - 1);
        if (last) __hip_atomic_store(cc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!last) return;
    __shared__ float tot[256];   // this tile's column totals (2 nc <= 256) for the BN finalize
    if (act) {
        const float a = sum_rows(part + col, 0, f.ngroups, f.gs, 2 * Cout);
        const float v = f.accumulate ? f.stats[col] + a : a;
        f.stats[col] = v;
        tot[t] = v;
        if (f.acc_lo != nullptr) {
            if (t < nc) f.acc_lo[ch] += v;
            else f.acc_hi[ch] += v;
        }
    }
    if (f.bn.pro == nullptr) return;
    __syncthreads();
    if (t >= nc || ch >= Cout) return;
    const BnFin& b = f.bn;
    const float invM = 1.f / (float)b.count;
    const float mean = tot[t] * invM;
    const float var = fmaxf(tot[nc + t] * invM - mean * mean, 0.f);
    const float rs = rsqrtf(var + b.eps);
    b.save_mean[ch] = mean;
    b.save_rstd[ch] = rs;
    if (b.upd_mean != nullptr) {
        const float unbiased = b.count > 1 ? var * (float)b.count / (float)(b.count - 1) : var;
        b.upd_mean[ch] = (1.f - b.momentum) * b.upd_mean[ch] + b.momentum * mean;
        b.upd_var[ch] = (1.f - b.momentum) * b.upd_var[ch] + b.momentum * unbiased;
    }
    const float sc = rs * bf2f(b.gamma[ch]);
    b.pro[ch] = sc;
    b.pro[Cout + ch] = bf2f(b.beta[ch]) - mean * sc;
    b.zero_sums[ch] = 0.f;
    b.zero_sums[Cout + ch] = 0.f;
}

// ============================================================================ conv_nt (fwd / dgrad)
// BatchNorm-apply + ReLU of the PREVIOUS layer folded into an activation operand load: the staged
// 8-channel vector of pre-BN values y becomes relu(y * scale[c] + shift[c]) (pro = [scale[C] |
// shift[C]], fp32, from tdl_bn_finalize), rounded to bf16 exactly as a materialised BN output would
// be.  Zero padding stays zero (only in-range taps are transformed).
__device__ __forceinline__ void pro_load(const float* __restrict__ pro, int C, int c, float* sc, float* sh) {
    const float4 a = *(const float4*)(pro + c), b = *(const float4*)(pro + c + 4);
    const float4 e = *(const float4*)(pro + C + c), f = *(const float4*)(pro + C + c + 4);
    sc[0] = a.x, sc[1] = a.y, sc[2] = a.z, sc[3] = a.w, sc[4] = b.x, sc[5] = b.y, sc[6] = b.z, sc[7] = b.w;
    sh[0] = e.x, sh[1] = e.y, sh[2] = e.z, sh[3] = e.w, sh[4] = f.x, sh[5] = f.y, sh[6] = f.z, sh[7] = f.w;
}
__device__ __forceinline__ uint4 pro_apply(uint4 v, const float* sc, const float* sh) {
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], sc[e], sh[e]), 0.f);
    return pack8(f);
}

// BNB (data gradient of a convolution whose input was relu(BN(y)) folded into its operand load): the
// epilogue also reduces the BN backward's two per-channel sums over the stored gradient g of the
// never-materialised BN output — sum(dv) and sum(dv * xhat) with dv = g where y * scale + shift > 0
// (the ReLU mask, recomputed from y = bx) and xhat = (y - mean) * rstd; bnp = [scale | shift | mean |
// rstd] fp32 [4 C] — into the STATS partial rows, so the BN backward needs no reduction pass.
template <int BCO, bool TRANSPOSED, bool STATS, bool PRO = false, bool BNB = false>
__global__ __launch_bounds__(256, 2) void conv_nt_kernel(const bf16_t* __restrict__ act, const bf16_t* __restrict__ wk,
                                                         bf16_t* __restrict__ out, float* __restrict__ part,
                                                         ConvDims d, ConvCls cl, const float* __restrict__ pro,
                                                         const bf16_t* __restrict__ bx = nullptr,
                                                         float* __restrict__ zero_stats = nullptr,
                                                         unsigned* __restrict__ fin_cnt = nullptr,
                                                         float* __restrict__ splitws = nullptr, int kps = 0,
                                                         FinArgs fin = FinArgs{}) {
    // the statistics finalize (next launch on the stream) accumulates into stats: zero it here
    // instead of a separate memset launch per convolution; likewise its arrival counters
    if (zero_stats != nullptr && blockIdx.x == 0)
        for (int i = threadIdx.x; i < 2 * d.Cout; i += blockDim.x) zero_stats[i] = 0.f;
    if (fin_cnt != nullptr && blockIdx.x == 0 && threadIdx.x < FIN_CNT) fin_cnt[threadIdx.x] = 0u;
    static_assert(!(PRO && TRANSPOSED), "the BN prologue applies to forward activations only");
    static_assert(!BNB || (TRANSPOSED && STATS), "BN-backward sums: data-gradient kernels with the STATS rows");
    constexpr int TCO = BCO / 64;   // 32-row cout tiles per wave (waves are 2 x 2)
    constexpr int AROWS = BCO / 32; // weight rows staged per thread (BCO rows x 8 chunks / 256 threads)
    __shared__ __attribute__((aligned(16))) bf16_t As[2][BCO * BK];
    __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BM * BK];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, lr = lane & 31;
    const int wco = w >> 1, wm = w & 1;
    const int PQs = cl.Ps * cl.Qs;
    const int M = d.N * PQs;                 // output pixels of this class
    const int Kw = d.R * d.S * d.Cin;        // weight row length
    const int K = cl.nr * cl.ns * d.Cin;     // reduction length of this class
    const int ntco = (d.Cout + BCO - 1) / BCO, ntm = (M + BM - 1) / BM;
    const int wg = xcd_remap(blockIdx.x, ntco * ntm);
    const int tco = wg % ntco, tm = wg / ntco;
    const int co0 = tco * BCO, m0 = tm * BM;

    // ---- per-thread staging geometry: rows srow + 32 i, 16-byte chunk sch of the 64-wide k step
    const int srow = tid >> 3, sch = tid & 7;
    int b_img[4], b_y[4], b_x[4];  // image offset, and spatial origin of each staged pixel row
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + srow + 32 * i;
        if (m < M) {
            const int n = m / PQs, pq = m - n * PQs, ip = pq / cl.Qs, jq = pq - ip * cl.Qs;
            const int p = cl.h0 + cl.cs * ip, q = cl.w0 + cl.cs * jq;
            b_img[i] = n;
            b_y[i] = TRANSPOSED ? p + d.pad : p * d.stride - d.pad;
            b_x[i] = TRANSPOSED ? q + d.pad : q * d.stride - d.pad;
        } else {
            b_img[i] = -1;
            b_y[i] = b_x[i] = 0;
        }
    }
    uint4 areg[AROWS], breg[4];
    // BN prologue state of the staged tile: the transform is applied when the tile is written to
    // LDS (after the current tile's MFMAs), not at load time, so the global loads stay in flight
    // behind the MFMAs; only in-range taps are transformed (padding stays zero)
    float psc[8], psh[8];
    uint32_t bok = 0;
    auto gload = [&](int k0) {
        const int kk = k0 + 8 * sch;
        const bool kin = kk < K;
        int c = 0, r = 0, s = 0;
        if (kin) {
            const int rs = kk / d.Cin;
            c = kk - rs * d.Cin;
            const int tr = rs / cl.ns;
            r = cl.r0 + cl.cs * tr;
            s = cl.s0 + cl.cs * (rs - tr * cl.ns);
        }
        const int kw = (r * d.S + s) * d.Cin + c;   // == kk for the identity class
#pragma unroll
        for (int i = 0; i < AROWS; ++i) {
            const int co = co0 + srow + 32 * i;
            areg[i] = (kin && co < d.Cout) ? *(const uint4*)(wk + (size_t)co * Kw + kw) : make_uint4(0, 0, 0, 0);
        }
        if (PRO && kin) pro_load(pro, d.Cin, c, psc, psh);
        bok = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (kin && b_img[i] >= 0) {
                int y, x;
                bool ok;
                if (TRANSPOSED) {
                    const int ty = b_y[i] - r, tx = b_x[i] - s;
                    y = ty / d.stride;
                    x = tx / d.stride;
                    ok = ty >= 0 && tx >= 0 && y * d.stride == ty && x * d.stride == tx && y < d.Hin && x < d.Win;
                } else {
                    y = b_y[i] + r;
                    x = b_x[i] + s;
                    ok = (unsigned)y < (unsigned)d.Hin && (unsigned)x < (unsigned)d.Win;
                }
                if (ok) {
                    v = *(const uint4*)(act + (((size_t)b_img[i] * d.Hin + y) * d.Win + x) * d.Cin + c);
                    bok |= 1u << i;
                }
            }
            breg[i] = v;
        }
    };
    // LDS image: 64 bf16 (8 x 16-byte chunks) per row, chunk XOR-swizzled by (row >> 1) & 7
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AROWS; ++i) {
            const int row = srow + 32 * i;
            *(uint4*)(As[buf] + row * BK + ((sch ^ ((row >> 1) & 7)) << 3)) = areg[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = srow + 32 * i;
            const uint4 v = (PRO && ((bok >> i) & 1u)) ? pro_apply(breg[i], psc, psh) : breg[i];
            *(uint4*)(Bs[buf] + row * BK + ((sch ^ ((row >> 1) & 7)) << 3)) = v;
        }
    };

    f32x16 acc[TCO][2];
#pragma unroll
    for (int i = 0; i < TCO; ++i) acc[i][0] = acc[i][1] = f32x16{};

    // split-K (splitws != null): workgroup (x, z) runs K steps [z kps, (z + 1) kps) and stores its
    // fp32 partial tile; conv_split_epi_kernel sums the slices in order and runs the epilogue
    const int nk = (K + BK - 1) / BK;
    const int kt0 = splitws != nullptr ? (int)blockIdx.y * kps : 0;
    const int kt1 = splitws != nullptr ? min(nk, kt0 + kps) : nk;
    gload(kt0 * BK);
    sstore(0);
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
        const int buf = (kt - kt0) & 1;
        const bool has_next = kt + 1 < kt1;
        if (has_next) gload((kt + 1) * BK);
        const bf16_t* A_ = As[buf];
        const bf16_t* B_ = Bs[buf];
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            const int ch = 2 * ks + h;
            bf16x8_t af[TCO], bfr[2];
#pragma unroll
            for (int i = 0; i < TCO; ++i) {
                const int row = wco * (BCO / 2) + 32 * i + lr;
                af[i] = as_bf16x8(*(const uint4*)(A_ + row * BK + ((ch ^ ((row >> 1) & 7)) << 3)));
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = wm * 64 + 32 * j + lr;
                bfr[j] = as_bf16x8(*(const uint4*)(B_ + row * BK + ((ch ^ ((row >> 1) & 7)) << 3)));
            }
#pragma unroll
            for (int i = 0; i < TCO; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = MFMA32(af[i], bfr[j], acc[i][j]);
        }
        if (has_next) sstore(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: lane owns pixel m, registers 4g..4g+3 are channels co + 8g + 4h + 0..3.
    // STATS: per-channel sum / sumsq of the stored (bf16-rounded) values, reduced over the wave's
    // two pixel tiles in registers, over its 32 lanes by shuffles and over the two pixel-waves in
    // LDS; each workgroup writes its own partial row part[tm][2 * Cout] (no atomics, no memset).
    if (splitws != nullptr) {
        float* slab = splitws + (size_t)blockIdx.y * M * d.Cout;
#pragma unroll
        for (int i = 0; i < TCO; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int co = co0 + wco * (BCO / 2) + 32 * i + 8 * g + 4 * h;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int m = m0 + wm * 64 + 32 * j + lr;
                    if (m < M && co < d.Cout)
                        *(float4*)(slab + (size_t)m * d.Cout + co) =
                            make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
                }
            }
        return;
    }
    float* red = reinterpret_cast<float*>(As[0]);  // [2 (wm)][BCO][2], free after the K loop
    int mfull[2];   // the lane's two output pixels as indices of the full [N][P][Q] image
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int m = m0 + wm * 64 + 32 * j + lr;
        const int n = m / PQs, pq = m - n * PQs, ip = pq / cl.Qs, jq = pq - ip * cl.Qs;
        mfull[j] = (n * d.P + cl.h0 + cl.cs * ip) * d.Q + cl.w0 + cl.cs * jq;
    }
#pragma unroll
    for (int i = 0; i < TCO; ++i) {
        const int cl = wco * (BCO / 2) + 32 * i;  // tile-local first channel of this MFMA tile
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int co = co0 + cl + 8 * g + 4 * h;
            float sv[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
            float bsc[4] = {}, bsh[4] = {}, bmu[4] = {}, brs[4] = {};
            if (BNB && co < d.Cout) {   // Cout % 8 == 0: the 4 channels are all in range
                const float4 a = *(const float4*)(pro + co), b = *(const float4*)(pro + d.Cout + co);
                const float4 c = *(const float4*)(pro + 2 * d.Cout + co), e = *(const float4*)(pro + 3 * d.Cout + co);
                bsc[0] = a.x, bsc[1] = a.y, bsc[2] = a.z, bsc[3] = a.w;
                bsh[0] = b.x, bsh[1] = b.y, bsh[2] = b.z, bsh[3] = b.w;
                bmu[0] = c.x, bmu[1] = c.y, bmu[2] = c.z, bmu[3] = c.w;
                brs[0] = e.x, brs[1] = e.y, brs[2] = e.z, brs[3] = e.w;
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int m = m0 + wm * 64 + 32 * j + lr, mf = mfull[j];
                const bool mok = m < M;
                float v[4] = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
                const uint2 pk = pack4(v);
                if (mok && co < d.Cout) *(uint2*)(out + (size_t)mf * d.Cout + co) = pk;
                if (STATS && mok) {
                    float r[4];
                    unpack4(pk, r);
                    if constexpr (BNB) {
                        float xv[4] = {0.f, 0.f, 0.f, 0.f};
                        if (co < d.Cout) unpack4(*(const uint2*)(bx + (size_t)mf * d.Cout + co), xv);
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float dv = fmaf(xv[e], bsc[e], bsh[e]) > 0.f ? r[e] : 0.f;
                            sv[e] += dv;
                            sq[e] += dv * (xv[e] - bmu[e]) * brs[e];
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            sv[e] += r[e];
                            sq[e] += r[e] * r[e];
                        }
                    }
                }
            }
            if (STATS) {
#pragma unroll
                for (int o = 1; o < 32; o <<= 1)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        sv[e] += __shfl_xor(sv[e], o, 64);
                        sq[e] += __shfl_xor(sq[e], o, 64);
                    }
                if (lr < 4) {
                    const float s_ = lr == 0 ? sv[0] : lr == 1 ? sv[1] : lr == 2 ? sv[2] : sv[3];
                    const float q_ = lr == 0 ? sq[0] : lr == 1 ? sq[1] : lr == 2 ? sq[2] : sq[3];
                    const int c = cl + 8 * g + 4 * h + lr;
                    red[(wm * BCO + c) * 2] = s_;
                    red[(wm * BCO + c) * 2 + 1] = q_;
                }
            }
        }
    }
    if (STATS) {
        __syncthreads();
        for (int c = tid; c < BCO; c += 256) {
            const int co = co0 + c;
            if (co < d.Cout) {
                float* rowp = part + (size_t)(cl.row_off + tm) * 2 * d.Cout;
                const float s_ = red[c * 2] + red[(BCO + c) * 2], q_ = red[c * 2 + 1] + red[(BCO + c) * 2 + 1];
                if (fin.cnt != nullptr) {   // read back by another workgroup: agent-scope (sc1) stores
                    __hip_atomic_store(rowp + co, s_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(rowp + d.Cout + co, q_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    rowp[co] = s_;
                    rowp[d.Cout + co] = q_;
                }
            }
        }
        if (fin.cnt != nullptr) stats_arrive(part, d.Cout, cl.row_off + tm, co0, BCO, tco, fin);
    }
}

// Epilogue of a split-K convolution: out = bf16(sum of the split slices, in slice order) and, with
// STATS, the per-channel partial rows of the 128-pixel tile exactly as conv_nt_kernel writes them
// (BNB: the BatchNorm-backward sums of the folded BN).  Workgroup = 128 pixels x 64 channels;
// thread = 4 channels x 8 pixels, 16 threads per 256-byte row segment.
template <bool STATS, bool BNB>
__global__ __launch_bounds__(256) void conv_split_epi_kernel(const float* __restrict__ ws, int split, int M, int Cout,
                                                             bf16_t* __restrict__ out, float* __restrict__ part,
                                                             const bf16_t* __restrict__ bx,
                                                             const float* __restrict__ bnp, FinArgs fin) {
    __shared__ float red[16][64][2];
    const int tm = blockIdx.x, cb = blockIdx.y * 64;
    const int cg = threadIdx.x & 15, rr = threadIdx.x >> 4;
    const int co = cb + 4 * cg;
    const bool cok = co < Cout;
    float sv[4] = {0.f, 0.f, 0.f, 0.f}, sq[4] = {0.f, 0.f, 0.f, 0.f};
    float bsc[4] = {}, bsh[4] = {}, bmu[4] = {}, brs[4] = {};
    if (BNB && cok) {
        const float4 a = *(const float4*)(bnp + co), b = *(const float4*)(bnp + Cout + co);
        const float4 c = *(const float4*)(bnp + 2 * Cout + co), e = *(const float4*)(bnp + 3 * Cout + co);
        bsc[0] = a.x, bsc[1] = a.y, bsc[2] = a.z, bsc[3] = a.w;
        bsh[0] = b.x, bsh[1] = b.y, bsh[2] = b.z, bsh[3] = b.w;
        bmu[0] = c.x, bmu[1] = c.y, bmu[2] = c.z, bmu[3] = c.w;
        brs[0] = e.x, brs[1] = e.y, brs[2] = e.z, brs[3] = e.w;
    }
#pragma unroll 2
    for (int i = 0; i < 8; ++i) {
        const int m = tm * BM + rr + 16 * i;
        if (m >= M || !cok) continue;
        float4 a = *(const float4*)(ws + (size_t)m * Cout + co);
        for (int z = 1; z < split; ++z) {
            const float4 b = *(const float4*)(ws + ((size_t)z * M + m) * Cout + co);
            a.x += b.x, a.y += b.y, a.z += b.z, a.w += b.w;
        }
        float v[4] = {a.x, a.y, a.z, a.w};
        const uint2 pk = pack4(v);
        *(uint2*)(out + (size_t)m * Cout + co) = pk;
        if (STATS) {
            float r[4];
            unpack4(pk, r);
            if constexpr (BNB) {
                float xv[4];
                unpack4(*(const uint2*)(bx + (size_t)m * Cout + co), xv);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float dv = fmaf(xv[e], bsc[e], bsh[e]) > 0.f ? r[e] : 0.f;
                    sv[e] += dv;
                    sq[e] += dv * (xv[e] - bmu[e]) * brs[e];
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    sv[e] += r[e];
                    sq[e] += r[e] * r[e];
                }
            }
        }
    }
    if (!STATS) return;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        red[rr][4 * cg + e][0] = sv[e];
        red[rr][4 * cg + e][1] = sq[e];
    }
    __syncthreads();
    if (threadIdx.x < 128) {
        const int c = threadIdx.x & 63, q = threadIdx.x >> 6;
        float t = 0.f;
        for (int k = 0; k < 16; ++k) t += red[k][c][q];
        if (cb + c < Cout)
            __hip_atomic_store(part + (size_t)tm * 2 * Cout + q * Cout + cb + c, t, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (fin.cnt != nullptr) stats_arrive(part, Cout, tm, cb, 64, blockIdx.y, fin);
}

// stats[c] += sum over the ntm partial rows of part[r][c], c < 2*Cout, in a FIXED order: the
// recompute audit (parallel/pipeline.py) compares a stage's outputs and gradients with a second
// evaluation, so BatchNorm statistics must not depend on the order fp32 atomics land in (a float-
// atomic version differed by up to one bf16 ulp per call, which the BN backward amplified to 4-10 %
// of the largest input gradient: scripts/audit_probe.py, profiles/r4_audit_probe_resnet50.txt).
// Workgroup (x, y) sums rows [y rpb, (y + 1) rpb) of its 64 columns and stores the total in the
// group's first row; the LAST workgroup of column block x to arrive (agent-scope counter, drained sc1 stores /
// sc1 loads, see stats_arrive) adds the gridDim.y group totals in group order.  fin_cnt: zeroed by the conv kernel.
// acc_lo / acc_hi (nullable): the completed column c is also added into acc_lo[c] (c < cols / 2) or
// acc_hi[c - cols / 2] (a folded BN's backward sums -> dbeta / dgamma).
__global__ __launch_bounds__(256) void stats_finalize_kernel(float* __restrict__ part, int rows, int cols,
                                                             int rows_per_block, float* __restrict__ stats,
                                                             unsigned* __restrict__ fin_cnt,
                                                             float* __restrict__ acc_lo = nullptr,
                                                             float* __restrict__ acc_hi = nullptr) {
    __shared__ float red[4][64];
    __shared__ int is_last;
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
    const int r0 = blockIdx.y * rows_per_block;
    const int r1 = min(rows, r0 + rows_per_block);
    float acc = 0.f;
    if (c < cols)
        for (int r = r0 + rg; r < r1; r += 4) acc += part[(size_t)r * cols + c];
    red[rg][threadIdx.x & 63] = acc;
    __syncthreads();
    // wave 0 (rg == 0) stores the group total as an agent-scope (sc1, write-through) store and
    // drains it before thread 0 of that same wave counts in; the last workgroup reads the totals
    // with sc1 loads (no L2 write-back / invalidate fences: a wbl2 per workgroup wrote back the
    // convolution's whole dirty output and cost ~1.4 % of a ResNet-50 step)
    if (rg == 0 && c < cols)
        __hip_atomic_store(part + (size_t)r0 * cols + c,
                           ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's sc1 stores have landed
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(fin_cnt + blockIdx.x, 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        is_last = prev == gridDim.y - 1;
    }
    __syncthreads();
    if (!is_last) return;
    float a = 0.f;
    if (c < cols)
        for (int g = rg; g < (int)gridDim.y; g += 4)
            a += __hip_atomic_load(part + (size_t)g * rows_per_block * cols + c, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    red[rg][threadIdx.x & 63] = a;
    __syncthreads();
    if (rg == 0 && c < cols) {
        const float v = stats[c] + (((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x]);
        stats[c] = v;
        if (acc_lo != nullptr) {
            const int half = cols >> 1;
            if (c < half) acc_lo[c] += v;
            else acc_hi[c - half] += v;
        }
    }
}

// ============================================================================ conv_wgrad
constexpr int WBM = 32;          // m rows per reduction step
constexpr int WLD_PAD = 32;      // row padding (elements): 320-byte rows -> conflict-free tr reads

template <int BCO, bool PRO = false>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                            float* __restrict__ dw, ConvDims d, int m_per_split,
                                                            int mode, const float* __restrict__ pro) {
    constexpr int TCO = BCO / 64;
    constexpr int LDY = BCO + WLD_PAD, LDX = 128 + WLD_PAD;
    constexpr int YCH = BCO / 8;        // 16-byte chunks per dY row
    constexpr int YROWS = 256 / YCH;    // rows covered by one pass of 256 threads
    __shared__ __attribute__((aligned(16))) bf16_t Ys[2][WBM * LDY];
    __shared__ __attribute__((aligned(16))) bf16_t Xs[2][WBM * LDX];

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, lr = lane & 31;
    const int wco = w >> 1, wk = w & 1;
    const int M = d.N * d.P * d.Q;
    const int K = d.R * d.S * d.Cin;
    const int ntco = (d.Cout + BCO - 1) / BCO, ntk = (K + 127) / 128;
    const int wg = xcd_remap(blockIdx.x, ntco * ntk);
    const int tco = wg % ntco, tk = wg / ntco;
    const int co0 = tco * BCO, k0 = tk * 128;
    const int mbeg = blockIdx.z * m_per_split;
    const int mend = min(M, mbeg + m_per_split);
    const int PQ = d.P * d.Q;

    // X staging: thread -> (row xr + 16 i, chunk xc); its k chunk (r, s, c) is fixed for the block
    const int xr = tid >> 4, xc = tid & 15;
    const int kk = k0 + 8 * xc;
    const bool kin = kk < K;
    int kc = 0, kr = 0, ks = 0;
    if (kin) {
        const int rs = kk / d.Cin;
        kc = kk - rs * d.Cin;
        kr = rs / d.S;
        ks = rs - kr * d.S;
    }
    float psc[8], psh[8];  // BN prologue of this thread's fixed 8 channels
    if (PRO && kin) pro_load(pro, d.Cin, kc, psc, psh);
    // dY staging: thread -> (row yr + YROWS i, chunk yc)
    const int yr = tid / YCH, yc = tid - yr * YCH;
    uint4 yreg[WBM / YROWS], xreg[2];
    uint32_t xok = 0;  // in-range X rows of the staged tile (BN prologue applied at LDS-write time)
    auto gload = [&](int mb) {
        xok = 0;
#pragma unroll
        for (int i = 0; i < WBM / YROWS; ++i) {
            const int m = mb + yr + YROWS * i;
            const int co = co0 + 8 * yc;
            yreg[i] = (m < mend && co < d.Cout) ? *(const uint4*)(dy + (size_t)m * d.Cout + co) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int m = mb + xr + 16 * i;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (kin && m < mend) {
                const int n = m / PQ, pq = m - n * PQ, p = pq / d.Q, q = pq - p * d.Q;
                const int y = p * d.stride - d.pad + kr, xx = q * d.stride - d.pad + ks;
                if ((unsigned)y < (unsigned)d.Hin && (unsigned)xx < (unsigned)d.Win) {
                    v = *(const uint4*)(x + (((size_t)n * d.Hin + y) * d.Win + xx) * d.Cin + kc);
                    xok |= 1u << i;
                }
            }
            xreg[i] = v;
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < WBM / YROWS; ++i) *(uint4*)(Ys[buf] + (yr + YROWS * i) * LDY + 8 * yc) = yreg[i];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint4 v = (PRO && ((xok >> i) & 1u)) ? pro_apply(xreg[i], psc, psh) : xreg[i];
            *(uint4*)(Xs[buf] + (xr + 16 * i) * LDX + 8 * xc) = v;
        }
    };

    f32x16 acc[TCO][2];
#pragma unroll
    for (int i = 0; i < TCO; ++i) acc[i][0] = acc[i][1] = f32x16{};
    // transposed-read geometry: 16-lane group (gg = lane>>4 & 1 selects 16 columns), lane 4q+p
    const int tq = (lane & 15) >> 2, tp = lane & 3, tcol = 16 * ((lane >> 4) & 1) + 4 * tp;

    if (mbeg < mend) {
        gload(mbeg);
        sstore(0);
    }
    __syncthreads();
    int buf = 0;
    for (int mb = mbeg; mb < mend; mb += WBM) {
        const bool has_next = mb + WBM < mend;
        if (has_next) gload(mb + WBM);
        const bf16_t* Y_ = Ys[buf];
        const bf16_t* X_ = Xs[buf];
#pragma unroll
        for (int st = 0; st < WBM / 16; ++st) {
            const int rb = 16 * st + 8 * h + tq;  // element j<4: row rb+j... (same map for A and B)
            bf16x8_t af[TCO], bfr[2];
#pragma unroll
            for (int i = 0; i < TCO; ++i) {
                const int cb = wco * (BCO / 2) + 32 * i + tcol;
                af[i] = tr_pair(Y_ + rb * LDY + cb, Y_ + (rb + 4) * LDY + cb);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int cb = wk * 64 + 32 * j + tcol;
                bfr[j] = tr_pair(X_ + rb * LDX + cb, X_ + (rb + 4) * LDX + cb);
            }
#pragma unroll
            for (int i = 0; i < TCO; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = MFMA32(af[i], bfr[j], acc[i][j]);
        }
        if (has_next) sstore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }

    // ---- epilogue: lane owns filter column k = (r, s, c); registers are output channels.
    // dw is [Cout][K] (K = R*S*Cin, c fastest) so consecutive lanes hit consecutive addresses.
    // mode 0: store, 1: +=, 2: fp32 atomic add (split reduction)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int k = k0 + wk * 64 + 32 * j + lr;
        if (k >= K) continue;
#pragma unroll
        for (int i = 0; i < TCO; ++i) {
            const int cb = co0 + wco * (BCO / 2) + 32 * i;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int co = cb + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                if (co >= d.Cout) continue;
                float* dst = dw + (size_t)co * K + k;
                if (mode == 2) atomicAdd(dst, acc[i][j][reg]);
                else if (mode == 1) *dst += acc[i][j][reg];
                else *dst = acc[i][j][reg];
            }
        }
    }
}

// dst[co][c][rs] += src[co][rs][c]   (KRSC fp32 workspace -> the parameter's [Cout][Cin][R][S] grad)
__global__ __launch_bounds__(256) void krsc_to_kcrs_add_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                               int Cout, int RS, int Cin) {
    const int64_t n = (int64_t)Cout * RS * Cin;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % Cin);
        const int64_t t = i / Cin;
        const int rs = (int)(t % RS);
        const int64_t co = t / RS;
        dst[(co * Cin + c) * RS + rs] += src[i];
    }
}

// TDL_BN_IN_CONV=0: the folded BN's finalize as its own launch after the convolution (A/B switch)
bool tdl_bn_in_conv_on() {
    static const bool v = [] {
        const char* e = getenv("TDL_BN_IN_CONV");
        return e == nullptr || atoi(e) != 0;
    }();
    return v;
}

// TDL_CONV_FIN_FUSED=0: statistics finalize as its own launch (stats_finalize_kernel; A/B switch)
bool conv_fin_fused_on() {
    static const bool v = [] {
        const char* e = getenv("TDL_CONV_FIN_FUSED");
        return e == nullptr || atoi(e) != 0;
    }();
    return v;
}

// Arrival counters of the in-kernel statistics finalize (FinArgs), one zeroed block per stream
// (calls on one stream are ordered; every counter is reset to zero by the workgroup that consumes it).
constexpr int CNT_MAX = 8192;
unsigned* stream_counters(hipStream_t s) {
    static std::mutex mu;
    static std::unordered_map<uint64_t, unsigned*> blocks;
    // the counters live on the STREAM's device (local mode runs stages on several GPUs from one
    // thread whose current device need not be the stream's: ADVICE r4)
    int dev = 0;
    if (hipStreamGetDevice(s, &dev) != hipSuccess) return nullptr;
    const uint64_t key = (uint64_t)(uintptr_t)s ^ ((uint64_t)dev << 56);
    std::lock_guard<std::mutex> lock(mu);
    auto it = blocks.find(key);
    if (it != blocks.end()) return it->second;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    unsigned* p = nullptr;
    bool ok = hipMalloc(&p, CNT_MAX * sizeof(unsigned)) == hipSuccess;
    if (ok && hipMemsetAsync(p, 0, CNT_MAX * sizeof(unsigned), s) != hipSuccess) {
        (void)hipFree(p);
        ok = false;
    }
    if (cur != dev) (void)hipSetDevice(cur);
    if (!ok) return nullptr;
    blocks[key] = p;
    return p;
}

// TDL_CONV_SPLIT=0: no split-K for convolutions whose grid leaves the chip short (A/B switch)
bool conv_split_on() {
    static const bool v = [] {
        const char* e = getenv("TDL_CONV_SPLIT");
        return e == nullptr || atoi(e) != 0;
    }();
    return v;
}

// TDL_CONV_PARITY=0: strided data gradients as one masked GEMM over all taps (A/B switch)
bool conv_parity_on() {
    static const bool v = [] {
        const char* e = getenv("TDL_CONV_PARITY");
        return e == nullptr || atoi(e) != 0;
    }();
    return v;
}

bool dims_ok(const ConvDims& d) {
    return d.Cin % 8 == 0 && d.Cout % 8 == 0 && d.N > 0 && d.P > 0 && d.Q > 0 && d.R > 0 && d.S > 0 && d.stride > 0 &&
           (long long)d.N * d.Hin * d.Win * d.Cin < (1ll << 31) && (long long)d.N * d.P * d.Q * d.Cout < (1ll << 31);
}

}  // namespace

// act: gathered NHWC tensor [N][Hin][Win][Cin]; wk: [Cout][R][S][Cin]; out: [N][P][Q][Cout].
// transposed = 1 -> data-gradient mapping (act = dY, wk = W permuted to [Cin][R][S][Cout]).
// stats: null, or fp32 [2 * Cout] = (per-channel sum, sum of squares) of out; then stats_ws must
// hold tdl_conv_stats_ws_floats(...) floats (one partial row per 128-pixel tile).
// partial rows: one per 128-pixel tile, + 3 for the tile rounding of the 4 parity classes of a
// stride-2 data gradient
static int64_t stats_rows(int M) { return (M + BM - 1) / BM + 3; }

TDL_API int64_t tdl_conv_stats_ws_floats(int M, int Cout) {
    return stats_rows(M) * 2 * Cout + FIN_CNT;   // + the finalize's arrival counters
}

// Split-K factor of a one-class convolution GEMM (M pixels x Cout channels, reduction K): the
// 14 x 14 / 7 x 7 layers of ResNet-50 at batch 64 launch 196 / 100 workgroups of 128 x 128 on 256
// CUs (2 fit per CU), so their long K loops (up to 72 steps) run on a fraction of the chip.  Split
// until ~512 workgroups, each keeping >= 8 K steps.
static int conv_split_of(int M, int Cout, int K) {
    if (!conv_split_on()) return 1;
    const int ntm = (M + BM - 1) / BM, ntco = Cout > 64 ? (Cout + 127) / 128 : (Cout + 63) / 64;
    const int nblk = ntm * ntco, nk = (K + BK - 1) / BK;
    if (nblk >= 256 || nk < 16) return 1;
    int split = min(4, (512 + nblk - 1) / nblk);
    while (split > 1 && nk / split < 8) --split;
    if (split <= 1) return 1;
    const int kps = (nk + split - 1) / split;
    return (nk + kps - 1) / kps;
}

// Whole workspace of one tdl_conv_nt* call: statistics partial rows + finalize counters, then the
// split-K slices (when conv_split_of splits; parity = 1 for a stride-2 data gradient: no split)
TDL_API int64_t tdl_conv_ws_floats(int M, int Cout, int K, int parity) {
    const int split = parity ? 1 : conv_split_of(M, Cout, K);
    return tdl_conv_stats_ws_floats(M, Cout) + (split > 1 ? (int64_t)split * M * Cout : 0);
}

static int conv_nt_impl(const void* act, const void* wk, void* out, float* stats, float* stats_ws, int N, int Hin,
                        int Win, int Cin, int P, int Q, int Cout, int R, int S, int stride, int pad, int transposed,
                        const float* pro, hipStream_t s, const void* bnb_x = nullptr, bool stats_accumulate = false,
                        float* acc_lo = nullptr, float* acc_hi = nullptr, const BnFin* bnfin = nullptr,
                        int* bn_done = nullptr) {
    if (bn_done != nullptr) *bn_done = 0;
    ConvDims d{N, Hin, Win, Cin, P, Q, Cout, R, S, stride, pad};
    const bool bnb = bnb_x != nullptr;
    if (!dims_ok(d) || (pro != nullptr && transposed && !bnb)) return (int)hipErrorInvalidValue;
    if (bnb && (!transposed || pro == nullptr || stats == nullptr || Cout % 8)) return (int)hipErrorInvalidValue;
    const int M = N * P * Q;
    const bool st = stats != nullptr;
    if (st && stats_ws == nullptr) return (int)hipErrorInvalidValue;
    const bool big = Cout > 64;
    auto A = (const bf16_t*)act;
    auto W = (const bf16_t*)wk;
    auto O = (bf16_t*)out;
    float* zs = (st && !stats_accumulate) ? stats : nullptr;
    unsigned* cnt = st ? (unsigned*)(stats_ws + (size_t)stats_rows(M) * 2 * Cout) : nullptr;
    if (st && (2 * Cout + 63) / 64 > FIN_CNT) return (int)hipErrorInvalidValue;
    // a stride-2 data gradient runs as its 4 output-parity classes (ConvCls), the rest as one class
    const int cs = (transposed && stride == 2 && conv_parity_on()) ? 2 : 1;
    const int Kall = R * S * Cin;
    const int split = (!(transposed && stride == 2) && stats_ws != nullptr) ? conv_split_of(M, Cout, Kall) : 1;
    // statistics finalized inside the producing kernels (FinArgs) when the counters fit
    FinArgs fin{};
    if (st && conv_fin_fused_on()) {
        int total = 0;
        for (int h0 = 0; h0 < cs; ++h0)
            for (int w0 = 0; w0 < cs; ++w0) {
                const int ps = (P - h0 + cs - 1) / cs, qs = (Q - w0 + cs - 1) / cs;
                if (ps > 0 && qs > 0) total += (N * ps * qs + BM - 1) / BM;
            }
        const int ntiles = split > 1 ? (Cout + 63) / 64 : (Cout + (big ? 127 : 63)) / (big ? 128 : 64);
        const int gs = max(4, (int)ceilf(sqrtf((float)total)));
        const int ngroups = (total + gs - 1) / gs;
        unsigned* sc = ntiles * (ngroups + 1) <= CNT_MAX ? stream_counters(s) : nullptr;
        if (sc != nullptr) {
            fin = FinArgs{sc, gs, ngroups, total, stats_accumulate ? 1 : 0, stats, acc_lo, acc_hi, BnFin{}};
            if (bnfin != nullptr && bnfin->pro != nullptr && tdl_bn_in_conv_on()) {
                fin.bn = *bnfin;
                if (bn_done != nullptr) *bn_done = 1;
            }
            zs = nullptr;   // the last workgroup stores the totals (=, or += when accumulating)
            cnt = nullptr;
        }
    }
    int rows = 0;
    for (int h0 = 0; h0 < cs; ++h0)
        for (int w0 = 0; w0 < cs; ++w0) {
            ConvCls cl{P, Q, 0, 0, 0, 0, R, S, 1, rows};
            if (cs > 1) {
                cl.Ps = (P - h0 + cs - 1) / cs;
                cl.Qs = (Q - w0 + cs - 1) / cs;
                cl.h0 = h0, cl.w0 = w0, cl.cs = cs;
                cl.r0 = (h0 + pad) % cs, cl.s0 = (w0 + pad) % cs;
                cl.nr = cl.r0 < R ? (R - cl.r0 + cs - 1) / cs : 0;
                cl.ns = cl.s0 < S ? (S - cl.s0 + cs - 1) / cs : 0;
            }
            if (cl.Ps <= 0 || cl.Qs <= 0) continue;
            const int ntm = (N * cl.Ps * cl.Qs + BM - 1) / BM;
            rows += ntm;
            const int nblk0 = ntm * ((Cout + (big ? 127 : 63)) / (big ? 128 : 64));
            // split-K (one-class GEMMs, workspace given): slices after the statistics area (never for a
            // stride-2 data gradient, parity classes or not: tdl_conv_ws_floats(parity = 1) sized the
            // caller's workspace without slices)
            const int nk = (Kall + BK - 1) / BK;
            const int kps = (nk + split - 1) / split;
            const FinArgs fin_nt = split > 1 ? FinArgs{} : fin;   // split: the epilogue kernel finalizes
            float* sws = split > 1 ? stats_ws + tdl_conv_stats_ws_floats(M, Cout) : nullptr;
            const dim3 nblk(nblk0, split);
            // a class with no taps (1x1 stride 2: three of four) runs an empty K loop and stores zeros
#define LAUNCH(BCO, TR, ST) conv_nt_kernel<BCO, TR, ST><<<nblk, 256, 0, s>>>(A, W, O, stats_ws, d, cl, nullptr, nullptr, \
                                                                             zs, cnt, sws, kps, fin_nt)
#define LAUNCHP(BCO, ST) conv_nt_kernel<BCO, false, ST, true><<<nblk, 256, 0, s>>>(A, W, O, stats_ws, d, cl, pro, nullptr, \
                                                                                  zs, cnt, sws, kps, fin_nt)
#define LAUNCHB(BCO) conv_nt_kernel<BCO, true, true, false, true><<<nblk, 256, 0, s>>>(A, W, O, stats_ws, d, cl, pro, \
                                                                                    (const bf16_t*)bnb_x, nullptr, cnt, sws, kps, \
                                                                                    fin_nt)
    if (bnb) {
        if (big) LAUNCHB(128);
        else LAUNCHB(64);
    } else if (pro != nullptr) {
        if (big) { if (st) LAUNCHP(128, true); else LAUNCHP(128, false); }
        else { if (st) LAUNCHP(64, true); else LAUNCHP(64, false); }
    } else if (big) {
        if (transposed) { if (st) LAUNCH(128, true, true); else LAUNCH(128, true, false); }
        else { if (st) LAUNCH(128, false, true); else LAUNCH(128, false, false); }
    } else {
        if (transposed) { if (st) LAUNCH(64, true, true); else LAUNCH(64, true, false); }
        else { if (st) LAUNCH(64, false, true); else LAUNCH(64, false, false); }
    }
#undef LAUNCH
#undef LAUNCHP
#undef LAUNCHB
            if (split > 1) {
                const dim3 ge(ntm, (Cout + 63) / 64);
                if (bnb)
                    conv_split_epi_kernel<true, true><<<ge, 256, 0, s>>>(sws, split, M, Cout, O, stats_ws,
                                                                         (const bf16_t*)bnb_x, pro, fin);
                else if (st)
                    conv_split_epi_kernel<true, false><<<ge, 256, 0, s>>>(sws, split, M, Cout, O, stats_ws, nullptr,
                                                                          nullptr, fin);
                else
                    conv_split_epi_kernel<false, false><<<ge, 256, 0, s>>>(sws, split, M, Cout, O, nullptr, nullptr,
                                                                           nullptr, FinArgs{});
            }
        }
    if (st && fin.cnt == nullptr) {
        const int rpb = 64;
        const dim3 g((2 * Cout + 63) / 64, (rows + rpb - 1) / rpb);
        stats_finalize_kernel<<<g, 256, 0, s>>>(stats_ws, rows, 2 * Cout, rpb, stats, cnt, acc_lo, acc_hi);
    }
    TDL_LAUNCH_CHECK();
}

// dw (fp32 [Cout][Cin][R][S], accumulated) += sum_m dY[m][co] * im2col(X)[m][k].  For R*S > 1 the
// kernel reduces into ws (fp32, Cout*R*S*Cin floats, [Cout][R][S][Cin]) and one pass adds it to dw.
static int conv_wgrad_impl(const void* dy, const void* x, float* dw, float* ws, int N, int Hin, int Win, int Cin, int P,
                           int Q, int Cout, int R, int S, int stride, int pad, int num_cu, const float* pro,
                           hipStream_t s) {
    ConvDims d{N, Hin, Win, Cin, P, Q, Cout, R, S, stride, pad};
    if (!dims_ok(d)) return (int)hipErrorInvalidValue;
    const int M = N * P * Q, K = R * S * Cin;
    const bool big = Cout > 64;
    const int bco = big ? 128 : 64;
    const int tiles = ((Cout + bco - 1) / bco) * ((K + 127) / 128);
    // split the pixel reduction until the grid holds ~2 workgroups per CU, each >= 16 steps
    const int target = 2 * (num_cu > 0 ? num_cu : 256);
    int split = (target + tiles - 1) / tiles;
    const int max_split = (M + 16 * WBM - 1) / (16 * WBM);
    if (split > max_split) split = max_split;
    if (split < 1) split = 1;
    int mps = (M + split - 1) / split;
    mps = (mps + WBM - 1) / WBM * WBM;
    split = (M + mps - 1) / mps;
    const bool direct = R * S == 1;  // KRSC == KCRS: reduce straight into the gradient
    if (!direct && ws == nullptr) return (int)hipErrorInvalidValue;
    float* target_buf = direct ? dw : ws;
    int mode = direct ? (split > 1 ? 2 : 1) : (split > 1 ? 2 : 0);
    if (!direct && split > 1) {
        hipError_t e = hipMemsetAsync(ws, 0, sizeof(float) * (size_t)Cout * K, s);
        if (e != hipSuccess) return (int)e;
    }
    const dim3 grid(tiles, 1, split);
    const bf16_t *Y = (const bf16_t*)dy, *X = (const bf16_t*)x;
    if (pro != nullptr) {
        if (big) conv_wgrad_kernel<128, true><<<grid, 256, 0, s>>>(Y, X, target_buf, d, mps, mode, pro);
        else conv_wgrad_kernel<64, true><<<grid, 256, 0, s>>>(Y, X, target_buf, d, mps, mode, pro);
    } else {
        if (big) conv_wgrad_kernel<128><<<grid, 256, 0, s>>>(Y, X, target_buf, d, mps, mode, nullptr);
        else conv_wgrad_kernel<64><<<grid, 256, 0, s>>>(Y, X, target_buf, d, mps, mode, nullptr);
    }
    if (!direct) {
        const int64_t n = (int64_t)Cout * K;
        int g = (int)((n + 255) / 256);
        if (g > 2048) g = 2048;
        krsc_to_kcrs_add_kernel<<<g, 256, 0, s>>>(ws, dw, Cout, R * S, Cin);
    }
    TDL_LAUNCH_CHECK();
}

TDL_API int tdl_conv_nt(const void* act, const void* wk, void* out, float* stats, float* stats_ws, int N, int Hin,
                        int Win, int Cin, int P, int Q, int Cout, int R, int S, int stride, int pad, int transposed,
                        hipStream_t s) {
    return conv_nt_impl(act, wk, out, stats, stats_ws, N, Hin, Win, Cin, P, Q, Cout, R, S, stride, pad, transposed,
                        nullptr, s);
}

// Forward convolution with batch statistics whose BatchNorm (folded into the NEXT convolution) is
// finalized by the same kernels (BnFin; pro = null for a plain convolution input).  *bn_done = 1
// when it was; 0 -> the caller runs tdl_bn_finalize (statistics finalized by a separate launch).
TDL_API int tdl_conv_fwd_bn(const void* act, const void* wk, void* out, float* stats, float* stats_ws, int N, int Hin,
                            int Win, int Cin, int P, int Q, int Cout, int R, int S, int stride, int pad,
                            const float* pro, const BnFin* bn, int* bn_done, hipStream_t s) {
    if (stats == nullptr || bn == nullptr || bn_done == nullptr) return (int)hipErrorInvalidValue;
    return conv_nt_impl(act, wk, out, stats, stats_ws, N, Hin, Win, Cin, P, Q, Cout, R, S, stride, pad, 0, pro, s,
                        nullptr, false, nullptr, nullptr, bn, bn_done);
}

// Forward convolution of relu(BN(y)) without materialising it: act = the previous layer's pre-BN
// output y, pro = [scale | shift] fp32 [2 Cin] from tdl_bn_finalize.
TDL_API int tdl_conv_nt_pro(const void* act, const void* wk, void* out, float* stats, float* stats_ws, int N, int Hin,
                            int Win, int Cin, int P, int Q, int Cout, int R, int S, int stride, int pad,
                            const float* pro, hipStream_t s) {
    if (pro == nullptr) return (int)hipErrorInvalidValue;
    return conv_nt_impl(act, wk, out, stats, stats_ws, N, Hin, Win, Cin, P, Q, Cout, R, S, stride, pad, 0, pro, s);
}

// Both kernel layouts of a conv weight w [Cout][C][R][S] (bf16, the nn.Conv2d parameter) in one pass:
// krsc [Cout][R][S][Cp] (forward) and crsk [Cp][R][S][Cout] (data gradient), input channels zero-
// padded to Cp (>= C).  Either output may be null.
__global__ __launch_bounds__(256) void conv_weight_layouts_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ krsc,
                                                                  bf16_t* __restrict__ crsk, int Cout, int C, int Cp,
                                                                  int RS) {
    const int64_t n = (int64_t)Cout * Cp * RS;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        // i enumerates the krsc image: co, rs, c (c fastest)
        const int c = (int)(i % Cp);
        const int64_t t = i / Cp;
        const int rs = (int)(t % RS);
        const int co = (int)(t / RS);
        const bf16_t v = c < C ? w[((int64_t)co * C + c) * RS + rs] : (bf16_t)0;
        if (krsc) krsc[i] = v;
        if (crsk) crsk[((int64_t)c * RS + rs) * Cout + co] = v;
    }
}

// Up to LAYOUT_MAX weights' layouts in ONE launch (kernel argument by value, no descriptor upload):
// a stage's convolution weights change every optimizer step, and one launch per weight put ~50
// dependent ~7 us launches at the head of each ResNet-50 forward.  Grid (blocks per weight, n).
constexpr int LAYOUT_MAX = 32;
struct LayoutBatch {
    const bf16_t* w[LAYOUT_MAX];
    bf16_t* krsc[LAYOUT_MAX];
    bf16_t* crsk[LAYOUT_MAX];
    int Cout[LAYOUT_MAX], C[LAYOUT_MAX], Cp[LAYOUT_MAX], RS[LAYOUT_MAX];
    int n;
};

__global__ __launch_bounds__(256) void conv_weight_layouts_batch_kernel(const LayoutBatch b) {
    const int j = blockIdx.y;
    const bf16_t* __restrict__ w = b.w[j];
    bf16_t* __restrict__ krsc = b.krsc[j];
    bf16_t* __restrict__ crsk = b.crsk[j];
    const int Cout = b.Cout[j], C = b.C[j], Cp = b.Cp[j], RS = b.RS[j];
    const int64_t n = (int64_t)Cout * Cp * RS;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % Cp);
        const int64_t t = i / Cp;
        const int rs = (int)(t % RS);
        const int co = (int)(t / RS);
        const bf16_t v = c < C ? w[((int64_t)co * C + c) * RS + rs] : (bf16_t)0;
        krsc[i] = v;
        crsk[((int64_t)c * RS + rs) * Cout + co] = v;
    }
}

// Python packs the LayoutBatch (ctypes structure passed by value).
TDL_API int tdl_conv_weight_layouts_batch(LayoutBatch b, hipStream_t s) {
    if (b.n <= 0 || b.n > LAYOUT_MAX) return (int)hipErrorInvalidValue;
    for (int j = 0; j < b.n; ++j)
        if (b.Cp[j] < b.C[j] || b.Cout[j] <= 0 || b.RS[j] <= 0 || !b.w[j] || !b.krsc[j] || !b.crsk[j])
            return (int)hipErrorInvalidValue;
    conv_weight_layouts_batch_kernel<<<dim3(64, b.n), 256, 0, s>>>(b);
    TDL_LAUNCH_CHECK();
}

TDL_API int tdl_conv_weight_layouts(const void* w, void* krsc, void* crsk, int Cout, int C, int Cp, int RS, hipStream_t s) {
    if (Cp < C || Cout <= 0 || RS <= 0) return (int)hipErrorInvalidValue;
    const int64_t n = (int64_t)Cout * Cp * RS;
    int64_t g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    conv_weight_layouts_kernel<<<(int)(g > 0 ? g : 1), 256, 0, s>>>((const bf16_t*)w, (bf16_t*)krsc, (bf16_t*)crsk, Cout, C,
                                                                   Cp, RS);
    TDL_LAUNCH_CHECK();
}

// Data gradient dbn of a convolution whose input relu(BN(y)) was folded into its operand load, with
// the BN backward's per-channel sums reduced in its epilogue (see BNB): sums (fp32 [2 C], the BN's
// backward row, zeroed by its forward) += (sum dv, sum dv * xhat), and the completed sums are added
// into dbeta / dgamma (fp32 [C] each, or both null); bnp = [scale | shift | mean | rstd] fp32 [4 C];
// y = the BN input (NHWC, same shape as dbn).  Pair with tdl_bn_act_bwd_pro_summed.
TDL_API int tdl_conv_dgrad_bnsums(const void* dy, const void* wd, void* dbn, float* ws, int N, int Hin, int Win, int Cin,
                                  int P, int Q, int Cout, int R, int S, int stride, int pad, const void* y,
                                  const float* bnp, float* sums, float* dgamma, float* dbeta, hipStream_t s) {
    if (y == nullptr || bnp == nullptr || sums == nullptr || ws == nullptr || (dgamma == nullptr) != (dbeta == nullptr))
        return (int)hipErrorInvalidValue;
    return conv_nt_impl(dy, wd, dbn, sums, ws, N, Hin, Win, Cin, P, Q, Cout, R, S, stride, pad, 1, bnp, s, y, true,
                        dbeta, dgamma);
}

TDL_API int tdl_conv_wgrad(const void* dy, const void* x, float* dw, float* ws, int N, int Hin, int Win, int Cin, int P,
                           int Q, int Cout, int R, int S, int stride, int pad, int num_cu, hipStream_t s) {
    return conv_wgrad_impl(dy, x, dw, ws, N, Hin, Win, Cin, P, Q, Cout, R, S, stride, pad, num_cu, nullptr, s);
}

// Weight gradient against relu(BN(y)) recomputed on load (pro as in tdl_conv_nt_pro).
TDL_API int tdl_conv_wgrad_pro(const void* dy, const void* x, float* dw, float* ws, int N, int Hin, int Win, int Cin,
                               int P, int Q, int Cout, int R, int S, int stride, int pad, int num_cu, const float* pro,
                               hipStream_t s) {
    if (pro == nullptr) return (int)hipErrorInvalidValue;
    return conv_wgrad_impl(dy, x, dw, ws, N, Hin, Win, Cin, P, Q, Cout, R, S, stride, pad, num_cu, pro, s);
}
