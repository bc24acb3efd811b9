// Causal flash attention for GPT-2 blocks, head dim 64, bf16 I/O, fp32 accumulate,
// gfx950 MFMA v_mfma_f32_32x32x16_bf16.
//
// Reads q/k/v straight out of the packed c_attn output [B, T, 3, H, D] and writes o as [B, T, H, D]
// (= the c_proj input), so no permute/contiguous copies exist around attention.
//
// Forward (per workgroup: 128 queries = 4 waves x 32; key blocks of 64 staged in LDS):
//   S^T = K . Q^T  ("swapped": each lane owns ONE query and 16 keys of every 32-key tile, so the
//   softmax row reductions are in-register + one cross-half shuffle).  The S^T accumulator is then
//   used directly as the B operand of O^T = V^T . P^T (cdna_hip_programming.md §3 "accumulator tile as
//   the next MFMA's operand"); V^T fragments come from a row-major LDS tile via ds_read_b64_tr_b16
//   (T10) in the matching permuted key order.  O^T keeps query on the lane, so the online-softmax
//   rescale is a per-lane scalar multiply.
// Backward = two atomic-free kernels (a first version that summed dQ with LDS + global fp32 atomics
// ran at ~27 TFLOP/s, 47% of the step, rocprof):
//   dK/dV: workgroup = 128 keys (key on the lane), double-buffered Q/dO tiles, S and dP
//          accumulators feed dV^T += dO^T.P and dK^T += Q^T.dS without leaving registers;
//   dQ:    workgroup = 128 queries (query on the lane, like the forward), S^T / dP^T recomputed,
//          dQ^T += K^T.dS^T with dS^T as the B operand.  +2 recomputed products, zero atomics.
#include "common.h"

#include <type_traits>

#include <cstdlib>
#include <cstring>

// Block-order mode: default = every head's block y dispatched together across heads (LPT over the
// whole grid); TDL_ATTN_MAP=xcd -> one head's blocks back to back on one XCD (head_xcd_map).
// dK/dV query-tile depth (32-row sub-tiles per barrier): TDL_ATTN_DKDV_NS=1|2 (default 1).  NS=2
// measured slower on MI355X (B=32 H=16 T=1024 causal bwd: 306.6 vs 327.6 TFLOP/s; the second
// staging register set and sub-tile loop cost more than the halved barrier count saves).  A
// software-pipelined form (two sub-tiles per barrier as straight-line S/dP(0), S/dP(1), [softmax |
// dV/dK](0), [softmax | dV/dK](1), dP started from -delta) needs 389 VGPRs = one wave per SIMD and
// measured 1220.7 vs 952.8 us for the whole backward at B=64 (profiles/r4_attn_dkdv_pipelined_ab.jsonl):
// the second wave per SIMD hides more than the in-wave interleave does.  Packing the score scaling
// into v_pk_fma (as the forward does) measured no change either (profiles/r4_attn_bwd_pkfma_ab.txt):
// the backward kernels wait on s_waitcnt / barriers, they are not VALU-bound.
static int dkdv_ns() {
    static int ns = [] {
        const char* e = std::getenv("TDL_ATTN_DKDV_NS");
        return (e && e[0] == '2') ? 2 : 1;
    }();
    return ns;
}

// dK/dV register prefetch depth (tiles ahead): TDL_ATTN_DKDV_PF=1|2 (default 2).
static int dkdv_pf() {   // read per call: in-process A/B
    const char* e = std::getenv("TDL_ATTN_DKDV_PF");
    return (e && e[0] == '1') ? 1 : 2;
}

// waves per workgroup of the attention kernels: TDL_ATTN_WAVES=4|8 (read per launch: in-process A/B)
// waves per workgroup of kernel i (0 forward, 1 dQ, 2 dK/dV): TDL_ATTN_WAVES = one digit for all
// three or three digits ("844"); 8 waves stage each K/V (Q/dO) tile once for twice the rows
// longest sequence the dK/dV kernel stages lse / delta for: 8 T bytes of dynamic LDS beside its
// 32-34 KiB of static tiles, at most the 160 KiB of a CU
#define ATTN_BWD_MAXT 16384
// s_waitcnt vmcnt(0) (expcnt / lgkmcnt left at their no-wait maxima), gfx9 encoding
#define VMCNT0 0x0F70

static int attn_waves(int i) {
    static const char dflt[] = "844";
    const char* e = std::getenv("TDL_ATTN_WAVES");
    if (e == nullptr || e[0] == 0) return dflt[i] - '0';
    const char c = (e[1] == 0) ? e[0] : (std::strlen(e) > (size_t)i ? e[i] : dflt[i]);
    return c == '8' ? 8 : 4;
}

static int attn_nbh_arg(int nbh) {
    const char* e = std::getenv("TDL_ATTN_MAP");
    return (e && std::strcmp(e, "xcd") == 0) ? -nbh : nbh;
}

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

__device__ __forceinline__ bf16x8_t as_bf16x8(uint4 u) { return __builtin_bit_cast(bf16x8_t, u); }

__device__ __forceinline__ short4_t tr_read(const bf16_t* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(p));
}
// 8-element operand fragment from two transposed 4x16 LDS reads (rows r..r+3 and r+8..r+11).
__device__ __forceinline__ bf16x8_t tr_pair(const bf16_t* p_lo, const bf16_t* p_hi) {
    const short4_t a = tr_read(p_lo), b = tr_read(p_hi);
    const short8_t c = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, c);
}
__device__ __forceinline__ bf16x8_t cvt8(const f32x16& v, int base) {
    bf16x8_t r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[base + j];
    return r;
}

constexpr int HD = 64;

// Element offset of (row, col) in a "plain" [rows][64] bf16 image read with ds_read_b64_tr_b16:
// the 64-B column half is XOR-flipped on every other row pair.  A transposed read takes 4 rows x
// 64 B per 32-lane group; at the natural 128-B row stride rows r and r + 2 hit the same 16 banks
// (2-way conflict on every read, PMC: 5.15 conflict cycles per LDS op in dK/dV).  With the flip the
// 4 rows cover the 64 banks once.  Writers store 16-B chunks through the same map.
__device__ __forceinline__ int swz_tr(int row, int col) { return row * HD + (col ^ (((row >> 1) & 1) << 5)); }

// 16-B chunk slot of logical chunk c in row `row` of a "row" image ([rows][64] bf16, 128-B rows)
// read with ds_read_b128, lane l -> row l & 31.  The bank slot of a chunk is (row & 1, slot): with
// slot = c ^ (row & 7) rows r and r + 8 share it and sit in one of ds_read_b128's 16-lane groups
// ({0-3,12-15,20-27}, ...) -> every row read was 2-way (PMC: 0.87-1.66 conflict cycles per LDS op
// in the three kernels).  Keyed on row >> 1 the 8 even and 8 odd rows of each group take distinct
// slots.  Also (row + 32 j) keeps the slot of row.
__device__ __forceinline__ int rsw(int row, int c) { return (c ^ ((row >> 1) & 7)) * 8; }

// Workgroup -> (batch*head, block) with the nb blocks of one head on ONE XCD, dispatched back to
// back (heaviest causal block first): the dispatcher sends workgroup L to XCD L % 8, so L = 8 j + x
// puts stream position j of XCD x on head 8 (j / nb) + x.  The head's K/V (fwd, dQ) or Q/dO (dK/dV)
// tiles are then fetched into that XCD's L2 once and shared by its co-resident workgroups — the
// earlier (B*H, T/128) grid streamed every head's K/V from HBM once per q-block wave.
__device__ __forceinline__ void head_xcd_map(int L, int nbh, int nb, bool causal, int& bh, int& blk) {
    const bool per_xcd = nbh < 0;  // sign carries the mapping mode (host: TDL_ATTN_MAP=xcd)
    nbh = per_xcd ? -nbh : nbh;
    if (per_xcd && (nbh & 7) == 0) {
        const int xcd = L & 7, j = L >> 3;
        const int hq = j % nb;
        bh = (j / nb) * 8 + xcd;
        blk = causal ? nb - 1 - hq : hq;
    } else {
        bh = L % nbh;
        const int y = L / nbh;
        blk = causal ? nb - 1 - y : y;
    }
}

// ============================================================================ forward
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// VALU helpers for the softmax of MFMA outputs, in forms hipcc understands (no inline asm: after
// every asm statement it pads an s_nop for hazards it cannot see).  Written as fmaxf / fmaf / +,
// -O3 emitted a canonicalising v_max_f32 x, x, x in front of every fmaxf of an MFMA result (32 per
// tile) and left the 32 score fmas unpacked (MI355X_MICROARCH issue costs: v_max / v_fma 4 cycles
// each, v_exp 8): the forward's softmax issued ~2x the cycles of its 16 MFMAs.  The scores are
// finite or -inf (masked), never NaN: fmax compiled without NaN semantics needs no canonicalize.
typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma clang fp contract(fast)
// (attention.hip is compiled with -fno-honor-nans: build_native.py)
__device__ __forceinline__ float vmax3(float a, float b, float c) { return __builtin_fmaxf(a, __builtin_fmaxf(b, c)); }
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 pk_add(f32x2 a, f32x2 b) { return a + b; }
// max over the 32 scores a lane holds (two 32x32 accumulators): 16 v_max3
__device__ __forceinline__ float max32(const f32x16& a, const f32x16& b) {
    float m = vmax3(a[0], b[0], a[1]);
#pragma unroll
    for (int i = 1; i < 16; ++i) m = vmax3(m, b[i], i + 1 < 16 ? a[i + 1] : b[i]);
    return m;
}

// 1-D grid of B*H*(T/128) workgroups mapped by head_xcd_map: one head's query blocks run back to
// back on one XCD, longest causal rows first (longest-processing-time-first inside each head).
// K / V are register-staged one tile ahead (tile t+1 loads during tile t; a second in-flight set
// measured flat in r4, profiles/r4_attn_fwd_valu_ab.txt).
// NW: waves per workgroup (32 queries each): 8 waves share every staged K / V tile between twice
// the queries (half the K / V traffic and LDS writes per MFMA of the 4-wave form)
template <bool CAUSAL, bool OPT = false, int NW = 4>
__global__ __launch_bounds__(64 * NW) void attn_fwd_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                           float* __restrict__ lse, int T, int H, int nbh, float scale_log2) {
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    constexpr int BM = 32 * NW, BN = 64;
    __shared__ __attribute__((aligned(16))) bf16_t Ks[2][BN * HD];
    __shared__ __attribute__((aligned(16))) bf16_t Vs[2][BN * HD];
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r = lane & 31;
    // wave-uniform (an SGPR): the causal tile tests become scalar branches, not exec-masked regions
    // (whose conservative wait bookkeeping drains in-flight loads)
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int bh, qb;
    head_xcd_map(blockIdx.x, nbh, T / BM, CAUSAL, bh, qb);
    const int b = bh / H, hd = bh - b * H;
    const int ldq = 3 * H * HD;
    const bf16_t* qbase = qkv + (size_t)b * T * ldq + hd * HD;
    const bf16_t* kbase = qbase + H * HD;
    const bf16_t* vbase = qbase + 2 * H * HD;
    const int qblk = qb * BM;
    const int q0 = qblk + 32 * w;
    const int qi = q0 + r;
    const int qrow = qi < T ? qi : T - 1;

    bf16x8_t qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = as_bf16x8(*(const uint4*)(qbase + (size_t)qrow * ldq + 16 * s + 8 * h));

    f32x16 o0 = {}, o1 = {};
    float m = -1e30f, l = 0.f;
    int nkb = T / BN;
    if (CAUSAL) {
        const int lim = (qblk + BM + BN - 1) / BN;
        nkb = lim < nkb ? lim : nkb;
    }
    // tr-read lane geometry (16-lane groups): lane 4q+p supplies row q, cols 4p..4p+3
    const int tq = (lane & 15) >> 2, tp = lane & 3, tcol = 16 * ((lane >> 4) & 1) + 4 * tp;
    // staging: 16 B of K and of V per thread and key row it stages (2 rows with 4 waves, 1 with 8)
    // per 64-key tile; the NEXT tile is loaded into registers while the current one computes (one
    // barrier per tile, LDS double-buffered); staging registers as named scalars (an indexed array
    // lands in scratch)
    uint4 kreg0 = {}, kreg1 = {}, vreg0 = {}, vreg1 = {};   // tile t+1 (PF = 1) / the set being stored
    const int srow0 = tid >> 3, sch = tid & 7, srow1 = srow0 + 32;
    auto gload_to = [&](int kb, uint4& k0, uint4& k1, uint4& v0, uint4& v1) {
        const size_t g0 = (size_t)(kb * BN + srow0) * ldq + sch * 8, g1 = g0 + (size_t)32 * ldq;
        k0 = *(const uint4*)(kbase + g0);
        v0 = *(const uint4*)(vbase + g0);
        if constexpr (NW == 4) {
            k1 = *(const uint4*)(kbase + g1);
            v1 = *(const uint4*)(vbase + g1);
        }
    };
    auto gload = [&](int kb) { gload_to(kb, kreg0, kreg1, vreg0, vreg1); };
    auto sstore = [&](int buf) {
        *(uint4*)(Ks[buf] + srow0 * HD + rsw(srow0, sch)) = kreg0;
        *(uint4*)(Vs[buf] + swz_tr(srow0, sch * 8)) = vreg0;
        if constexpr (NW == 4) {
            *(uint4*)(Ks[buf] + srow1 * HD + rsw(srow1, sch)) = kreg1;
            *(uint4*)(Vs[buf] + swz_tr(srow1, sch * 8)) = vreg1;
        }
    };
    gload(0);
    sstore(0);
    __syncthreads();
    // the Q fragments have landed before the loop (an empty asm consuming them pins their loads
    // and the wait here): otherwise the compiler sinks the loads into the loop's first tile and,
    // unsure of them, drains every K / V prefetch before a tile's first MFMA (s_waitcnt vmcnt(0))
    asm volatile("" ::"v"(qf[0]), "v"(qf[1]), "v"(qf[2]), "v"(qf[3]));
    // the tile of keys kb, staged in LDS buffer `buf`
    auto compute_tile = [&](int kb, int buf) {
        const bf16_t* K_ = Ks[buf];
        const bf16_t* V_ = Vs[buf];
        const bool active = !CAUSAL || (kb * BN <= q0 + 31);
        if (active) {
            f32x16 s0 = {}, s1 = {};
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int r1 = 32 + r;
                const bf16x8_t a0 = as_bf16x8(*(const uint4*)(K_ + r * HD + rsw(r, 2 * s + h)));
                const bf16x8_t a1 = as_bf16x8(*(const uint4*)(K_ + r1 * HD + rsw(r1, 2 * s + h)));
                s0 = MFMA32(a0, qf[s], s0);
                s1 = MFMA32(a1, qf[s], s1);
            }
            // row max on the raw scores (scale > 0 commutes with max); the scale folds into the
            // exponent's fma: p = exp2(s * scale_log2 - m) -> one fma + one v_exp per score
            float mx = -INFINITY;
            if (CAUSAL && kb * BN + BN - 1 > q0) {  // diagonal tile of this wave: mask keys > query
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key0 = kb * BN + (i & 3) + 8 * (i >> 2) + 4 * h;
                    const float v0 = key0 > qi ? -INFINITY : s0[i];
                    const float v1 = key0 + 32 > qi ? -INFINITY : s1[i];
                    s0[i] = v0;
                    s1[i] = v1;
                    if (!OPT) mx = fmaxf(mx, fmaxf(v0, v1));
                }
                if (OPT) mx = max32(s0, s1);
            } else if (OPT) {
                mx = max32(s0, s1);
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) mx = fmaxf(mx, fmaxf(s0[i], s1[i]));
            }
            if (OPT) {
                const float o = __shfl_xor(mx, 32, 64);
                mx = vmax3(mx, o, o);
            } else {
                mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
            }
            const float mn = fmaxf(m, mx * scale_log2);
            // exact skip of the O / l rescale when no row of the wave raised its running max
            // (alpha == 1 for every lane): the common case once the first tiles have been seen
            if (__any(mn > m)) {
                const float alpha = fast_exp2(m - mn);
                l *= alpha;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    o0[i] *= alpha;
                    o1[i] *= alpha;
                }
            }
            float rs = 0.f;
            if (OPT) {
                // p = exp2(s * scale - m) on register pairs: 16 v_pk_fma + 32 v_exp + 16 v_pk_add
                const f32x2 sc2 = {scale_log2, scale_log2}, nm2 = {-mn, -mn};
                f32x2 acc = {0.f, 0.f};
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    f32x2 a = {s0[i], s0[i + 1]}, b = {s1[i], s1[i + 1]};
                    a = pk_fma(a, sc2, nm2);
                    b = pk_fma(b, sc2, nm2);
                    a.x = fast_exp2(a.x);
                    a.y = fast_exp2(a.y);
                    b.x = fast_exp2(b.x);
                    b.y = fast_exp2(b.y);
                    acc = pk_add(acc, a);
                    acc = pk_add(acc, b);
                    s0[i] = a.x;
                    s0[i + 1] = a.y;
                    s1[i] = b.x;
                    s1[i + 1] = b.y;
                }
                rs = acc.x + acc.y;
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    s0[i] = fast_exp2(fmaf(s0[i], scale_log2, -mn));
                    s1[i] = fast_exp2(fmaf(s1[i], scale_log2, -mn));
                    rs += s0[i] + s1[i];
                }
            }
            rs += __shfl_xor(rs, 32, 64);
            l += rs;
            m = mn;
            const bf16x8_t p00 = cvt8(s0, 0), p01 = cvt8(s0, 8), p10 = cvt8(s1, 0), p11 = cvt8(s1, 8);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const bf16x8_t pf = t == 0 ? (s2 == 0 ? p00 : p01) : (s2 == 0 ? p10 : p11);
                    const int kr = 32 * t + 16 * s2 + 4 * h + tq;
                    const bf16x8_t v0 = tr_pair(V_ + swz_tr(kr, tcol), V_ + swz_tr(kr + 8, tcol));
                    const bf16x8_t v1 = tr_pair(V_ + swz_tr(kr, 32 + tcol), V_ + swz_tr(kr + 8, 32 + tcol));
                    o0 = MFMA32(v0, pf, o0);
                    o1 = MFMA32(v1, pf, o1);
                }
        }
    };
    for (int kb = 0; kb < nkb; ++kb) {
        const int buf = kb & 1;
        const bool has_next = kb + 1 < nkb;
        if (has_next) gload(kb + 1);
        compute_tile(kb, buf);
        if (has_next) sstore(buf ^ 1);
        __syncthreads();
    }
    if (qi < T) {
        const float inv_l = 1.f / l;
        bf16_t* orow = out + ((size_t)b * T + qi) * (H * HD) + hd * HD;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int d = 8 * g + 4 * h;
            float v[4] = {o0[4 * g] * inv_l, o0[4 * g + 1] * inv_l, o0[4 * g + 2] * inv_l, o0[4 * g + 3] * inv_l};
            *(uint2*)(orow + d) = pack4(v);
            float u[4] = {o1[4 * g] * inv_l, o1[4 * g + 1] * inv_l, o1[4 * g + 2] * inv_l, o1[4 * g + 3] * inv_l};
            *(uint2*)(orow + 32 + d) = pack4(u);
        }
        if (h == 0) lse[(size_t)bh * T + qi] = (m + log2f(l)) * 0.6931471805599453f;
    }
}

TDL_API int tdl_attn_fwd(const void* qkv, void* out, float* lse, void* unused, int B, int T, int H, int D, float scale,
                         int causal, hipStream_t s) {
    (void)unused;
    if (D != HD || T % 64 != 0) return (int)hipErrorInvalidValue;
    if (T % 128 != 0) return (int)hipErrorInvalidValue;
    const float sl2 = scale * 1.4426950408889634f;
    const char* ope = std::getenv("TDL_ATTN_FWD_OPT");   // packed softmax (default); 0 = scalar form
    const bool opt = !(ope && ope[0] == '0');
    auto Q = (const bf16_t*)qkv;
    auto O = (bf16_t*)out;
    const int nb = attn_nbh_arg(B * H);
    if (causal && opt && attn_waves(0) == 8 && T % 256 == 0) {
        attn_fwd_kernel<true, true, 8><<<B * H * (T / 256), 512, 0, s>>>(Q, O, lse, T, H, nb, sl2);
        TDL_LAUNCH_CHECK();
    }
    const int grid = B * H * (T / 128);
    if (causal) {
        if (opt) attn_fwd_kernel<true, true><<<grid, 256, 0, s>>>(Q, O, lse, T, H, nb, sl2);
        else attn_fwd_kernel<true><<<grid, 256, 0, s>>>(Q, O, lse, T, H, nb, sl2);
    } else {
        attn_fwd_kernel<false><<<grid, 256, 0, s>>>(Q, O, lse, T, H, nb, sl2);
    }
    TDL_LAUNCH_CHECK();
}

// ============================================================================ backward
// ---------------------------------------------------------------------------- dK, dV (key-owned)
// Workgroup = 128 keys (4 waves x 32, key on the MFMA lane); walks query tiles of BQ = 32 NS rows
// with a double-buffered LDS pipeline: the next tile's Q / dO / lse / delta are loaded into
// registers while the current tile computes, then written to the other buffer -> ONE barrier per
// tile.  NS = 2 halves the barriers per MFMA (16 -> 32 MFMAs per wave between barriers) at twice
// the LDS (64 KB, still 2 workgroups per CU) but measures slower (see dkdv_ns).
// Products per 32-row sub-tile and wave: S = Q.K^T, dP = dO.V^T (row-read A, K/V fragments
// resident in registers), dV^T += dO^T.P and dK^T += Q^T.dS (tr-read A, S/dP accumulators as B).
// ---- fused qkv-bias gradient (column sums of dqkv over tokens, SURVEY 2.8: no colsum pass over
// the [tokens, 3 * width] gradient).  Each workgroup reduces the bf16-rounded values it stores over
// its 128 rows and writes them to its own row of a partial matrix [B * T / 128][3 * H * HD]
// (every entry written once, fixed order: deterministic); tdl_colsum_f32 reduces the rows.
// Butterfly over the 32 lanes of a half-wave: at each step a lane keeps one half of its values
// (by its lane bit) and adds the partner's copy of that half, so N values cost N - N/32 shuffles
// instead of 5 N.  Afterwards lane r holds the sums of values (N / 32) * r + j, j < N / 32.
template <int N>
__device__ __forceinline__ void half_wave_colsum(float (&v)[N], int r) {
    static_assert(N % 32 == 0, "N multiple of 32");
    auto step = [&](auto oc) {
        constexpr int O = decltype(oc)::value, M = N * O / 32;   // values still held: 2 M -> M
        const bool up = (r & O) != 0;
#pragma unroll
        for (int i = 0; i < M; ++i) {
            const float send = up ? v[i] : v[i + M];
            const float keep = up ? v[i + M] : v[i];
            v[i] = keep + __shfl_xor(send, O, 64);
        }
    };
    step(std::integral_constant<int, 16>{});
    step(std::integral_constant<int, 8>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 1>{});
}
__device__ __forceinline__ float bf16_round(float x) {
    float a[4] = {x, 0.f, 0.f, 0.f}, b[4];
    unpack4(pack4(a), b);
    return b[0];
}

// NW = 8: 256 keys per workgroup, every staged Q / dO tile shared by twice the keys (waves 0-3
// stage Q, waves 4-7 dO)
template <bool CAUSAL, int NS, int PF, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_bwd_dkdv_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                            const float* __restrict__ lse, const float* __restrict__ delta,
                                                            bf16_t* __restrict__ dqkv, int T, int H, int nbh, float scale,
                                                            float* __restrict__ bias_part) {
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    constexpr int BK = 32 * NW, BQ = 32 * NS;
    // plain images (transposed tr-reads) + XOR-swizzled images (row reads: 32 rows x 128 B with
    // the 16-B chunk slot rsw(row, c) -> conflict-free ds_read_b128 across the 32 row lanes)
    // two buffers x four images: Q / dO, plain (transposed reads) and row-swizzled (row reads)
    constexpr int IMG = BQ * HD;
    __shared__ __attribute__((aligned(16))) bf16_t tiles[8 * IMG];
    auto Qs = [&](int b) { return tiles + b * IMG; };
    auto dOs = [&](int b) { return tiles + (2 + b) * IMG; };
    auto Qw = [&](int b) { return tiles + (4 + b) * IMG; };
    auto dOw = [&](int b) { return tiles + (6 + b) * IMG; };
    // lse (pre-scaled by log2(e)) and delta of every query this workgroup visits, staged once in the
    // prologue: no per-tile scalar loads in the loop (their waits drained the operand prefetch)
    // (dynamic LDS: 2 x T floats, sized at launch — dkdv_lds_bytes)
    extern __shared__ __attribute__((aligned(16))) float lse_dyn[];
    float* lse_s = lse_dyn;
    float* delta_s = lse_dyn + T;

    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r = lane & 31;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: tile-level branches stay scalar
    int bh, kbi;
    // causal dK/dV: key block 0 sees every query -> it is the heavy one; reverse the LPT order
    head_xcd_map(blockIdx.x, nbh, T / BK, CAUSAL, bh, kbi);
    if (CAUSAL) kbi = T / BK - 1 - kbi;
    const int b = bh / H, hd = bh - b * H;
    const int ldq = 3 * H * HD, ldo = H * HD;
    const bf16_t* qbase = qkv + (size_t)b * T * ldq + hd * HD;
    const bf16_t* kbase = qbase + H * HD;
    const bf16_t* vbase = qbase + 2 * H * HD;
    const bf16_t* dobase = dout + (size_t)b * T * ldo + hd * HD;
    const float* lse_row = lse + (size_t)bh * T;
    const float* delta_row = delta + (size_t)bh * T;
    const int kblk = kbi * BK;
    const int k0 = kblk + 32 * w;
    const int kj = k0 + r;

    bf16x8_t kf[4], vf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        kf[s] = as_bf16x8(*(const uint4*)(kbase + (size_t)kj * ldq + 16 * s + 8 * h));
        vf[s] = as_bf16x8(*(const uint4*)(vbase + (size_t)kj * ldq + 16 * s + 8 * h));
    }
    f32x16 dv0 = {}, dv1 = {}, dk0 = {}, dk1 = {};
    const int tq = (lane & 15) >> 2, tp = lane & 3, tcol = 16 * ((lane >> 4) & 1) + 4 * tp;
    const int q_start = CAUSAL ? kblk : 0;   // multiple of 128, so BQ (32 or 64) tiles end at T
    const int srow = (tid & 255) >> 3, sch = tid & 7;  // staging: 256 x 16 B = one 32 x 64 slab per operand
    const int swz = rsw(srow, sch);  // rsw(srow + 32 j, .) == rsw(srow, .)
    // which operand this thread stages: both (4 waves), Q (waves 0-3) or dO (waves 4-7) with 8
    const bool stq = NW == 4 || tid < 256, std_ = NW == 4 || tid >= 256;
    constexpr float LOG2E = 1.4426950408889634f;
    const float sl2 = scale * LOG2E;
    // prologue: tile q_start -> buffer 0
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const int row = srow + 32 * j;
        if (stq) {
            const uint4 q = *(const uint4*)(qbase + (size_t)(q_start + row) * ldq + sch * 8);
            *(uint4*)(Qs(0) + swz_tr(row, sch * 8)) = q;
            *(uint4*)(Qw(0) + row * HD + swz) = q;
        }
        if (std_) {
            const uint4 d = *(const uint4*)(dobase + (size_t)(q_start + row) * ldo + sch * 8);
            *(uint4*)(dOs(0) + swz_tr(row, sch * 8)) = d;
            *(uint4*)(dOw(0) + row * HD + swz) = d;
        }
    }
    for (int i = tid; i < T - q_start; i += 64 * NW) {
        lse_s[i] = lse_row[q_start + i] * LOG2E;
        delta_s[i] = -delta_row[q_start + i];   // negated: the dP accumulator starts from it
    }
    // every prologue load (K / V fragments included) has landed before the loop: the compiler's
    // wait bookkeeping then never has to drain the loop's prefetches on their account
    __builtin_amdgcn_s_waitcnt(VMCNT0);
    __syncthreads();

    // Register staging of the next tiles.  A tile's global loads land in a register set that is
    // stored to LDS one iteration later (PF = 1) or two (PF = 2).  With PF = 2 the loop is unrolled
    // by two and the two register sets swap roles statically: a copy from the "loaded" set into the
    // "to store" set would make the wave wait for the loads it just issued (ISA of the r4 form:
    // s_waitcnt vmcnt before the v_mov rotation, so the loads had one tile to land, not two).  The
    // lse scaling is applied when the value is stored to LDS, not when it arrives, for the same
    // reason (a multiply of the just-loaded lse made wave 0 wait for it every tile).
    auto load_tile = [&](int t0, uint4 (&q)[NS], uint4 (&d)[NS]) {
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            if (stq) q[j] = *(const uint4*)(qbase + (size_t)(t0 + srow + 32 * j) * ldq + sch * 8);
            if (std_) d[j] = *(const uint4*)(dobase + (size_t)(t0 + srow + 32 * j) * ldo + sch * 8);
        }
    };
    auto store_tile = [&](int nb, const uint4 (&q)[NS], const uint4 (&d)[NS]) {
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            const int row = srow + 32 * j;
            if (stq) {
                *(uint4*)(Qs(nb) + swz_tr(row, sch * 8)) = q[j];
                *(uint4*)(Qw(nb) + row * HD + swz) = q[j];
            }
            if (std_) {
                *(uint4*)(dOs(nb) + swz_tr(row, sch * 8)) = d[j];
                *(uint4*)(dOw(nb) + row * HD + swz) = d[j];
            }
        }
    };
    // the tile at query offset qt, staged in LDS buffer `buf`
    auto compute_tile = [&](int qt, int buf) {
#pragma unroll
            for (int j = 0; j < NS; ++j) {
                const int qs = qt + 32 * j;   // this sub-tile's first query
                if (CAUSAL && qs + 31 < k0) continue;
                const bf16_t* Qb = Qs(buf) + 32 * j * HD;
                const bf16_t* dOb = dOs(buf) + 32 * j * HD;
                const bf16_t* Qr = Qw(buf) + 32 * j * HD;
                const bf16_t* dOr = dOw(buf) + 32 * j * HD;
                const float* lsb = lse_s + (qs - q_start);
                const float* dlb = delta_s + (qs - q_start);
                // dP starts from -delta (row constants as the initial accumulator): the MFMA chain
                // leaves dP - delta, and dS = P * (dP - delta) is one multiply per score
                f32x16 sacc = {}, dpacc;
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    const float4 c = *(const float4*)(dlb + 8 * g4 + 4 * h);
                    dpacc[4 * g4] = c.x; dpacc[4 * g4 + 1] = c.y; dpacc[4 * g4 + 2] = c.z; dpacc[4 * g4 + 3] = c.w;
                }
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int c = rsw(r, 2 * s + h);
                    const bf16x8_t aq = as_bf16x8(*(const uint4*)(Qr + r * HD + c));
                    const bf16x8_t ad = as_bf16x8(*(const uint4*)(dOr + r * HD + c));
                    sacc = MFMA32(aq, kf[s], sacc);
                    dpacc = MFMA32(ad, vf[s], dpacc);
                }
                // the causal mask matters only on the tiles that straddle this wave's diagonal (a few
                // of T / 32): elsewhere the per-element compare + select is dropped (VALU-bound loop)
                // lse / delta of the lane's 16 query rows: 4 groups of 4 consecutive rows -> 4 + 4
                // 16-byte LDS reads instead of 32 scalar ones
                float lsv[16];
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    const float4 a = *(const float4*)(lsb + 8 * g4 + 4 * h);
                    lsv[4 * g4] = a.x; lsv[4 * g4 + 1] = a.y; lsv[4 * g4 + 2] = a.z; lsv[4 * g4 + 3] = a.w;
                }
                if (CAUSAL && qs < k0 + 31) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int ql = (i & 3) + 8 * (i >> 2) + 4 * h;
                        float p = fast_exp2(fmaf(sacc[i], sl2, -lsv[i]));
                        if (kj > qs + ql) p = 0.f;
                        sacc[i] = p;
                        dpacc[i] = p * dpacc[i];
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const float p = fast_exp2(fmaf(sacc[i], sl2, -lsv[i]));
                        sacc[i] = p;
                        dpacc[i] = p * dpacc[i];
                    }
                }
                const bf16x8_t pb0 = cvt8(sacc, 0), pb1 = cvt8(sacc, 8);
                const bf16x8_t db0 = cvt8(dpacc, 0), db1 = cvt8(dpacc, 8);
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int qr = 16 * s2 + 4 * h + tq;
                    const bf16x8_t pb = s2 == 0 ? pb0 : pb1;
                    const bf16x8_t dsb = s2 == 0 ? db0 : db1;
                    const bf16x8_t ado0 = tr_pair(dOb + swz_tr(qr, tcol), dOb + swz_tr(qr + 8, tcol));
                    const bf16x8_t ado1 = tr_pair(dOb + swz_tr(qr, 32 + tcol), dOb + swz_tr(qr + 8, 32 + tcol));
                    dv0 = MFMA32(ado0, pb, dv0);
                    dv1 = MFMA32(ado1, pb, dv1);
                    const bf16x8_t aq0 = tr_pair(Qb + swz_tr(qr, tcol), Qb + swz_tr(qr + 8, tcol));
                    const bf16x8_t aq1 = tr_pair(Qb + swz_tr(qr, 32 + tcol), Qb + swz_tr(qr + 8, 32 + tcol));
                    dk0 = MFMA32(aq0, dsb, dk0);
                    dk1 = MFMA32(aq1, dsb, dk1);
                }
            }
    };
    uint4 qa[NS], da[NS];
    if constexpr (PF == 2) {
        // two register sets, the loop unrolled by two so they swap roles statically: set A holds
        // tile qt + BQ (stored at the end of tile qt), set B receives tile qt + 2 BQ.  (An LDS-DMA
        // ring was tried: the compiler drains every in-flight copy before the first LDS read of a
        // tile — it cannot tell the ring's buffers apart — so it gained nothing.)
        uint4 qb[NS], db[NS];
        if (q_start + BQ < T) load_tile(q_start + BQ, qa, da);
        for (int qt = q_start; qt < T; qt += 2 * BQ) {
            if (qt + 2 * BQ < T) load_tile(qt + 2 * BQ, qb, db);
            compute_tile(qt, 0);
            if (qt + BQ < T) store_tile(1, qa, da);
            __syncthreads();
            if (qt + BQ >= T) break;
            if (qt + 3 * BQ < T) load_tile(qt + 3 * BQ, qa, da);
            compute_tile(qt + BQ, 1);
            if (qt + 2 * BQ < T) store_tile(0, qb, db);
            __syncthreads();
        }
    } else {
        int buf = 0;
        for (int qt = q_start; qt < T; qt += BQ) {
            const bool has_next = qt + BQ < T;
            if (has_next) load_tile(qt + BQ, qa, da);
            compute_tile(qt, buf);
            if (has_next) store_tile(buf ^ 1, qa, da);
            __syncthreads();
            buf ^= 1;
        }
    }
    bf16_t* dkrow = dqkv + ((size_t)b * T + kj) * ldq + H * HD + hd * HD;
    bf16_t* dvrow = dkrow + H * HD;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int d = 8 * g + 4 * h;
        float a[4] = {dk0[4 * g] * scale, dk0[4 * g + 1] * scale, dk0[4 * g + 2] * scale, dk0[4 * g + 3] * scale};
        *(uint2*)(dkrow + d) = pack4(a);
        float a2[4] = {dk1[4 * g] * scale, dk1[4 * g + 1] * scale, dk1[4 * g + 2] * scale, dk1[4 * g + 3] * scale};
        *(uint2*)(dkrow + 32 + d) = pack4(a2);
        float v[4] = {dv0[4 * g], dv0[4 * g + 1], dv0[4 * g + 2], dv0[4 * g + 3]};
        *(uint2*)(dvrow + d) = pack4(v);
        float v2[4] = {dv1[4 * g], dv1[4 * g + 1], dv1[4 * g + 2], dv1[4 * g + 3]};
        *(uint2*)(dvrow + 32 + d) = pack4(v2);
    }
    if (bias_part != nullptr) {
        // value i = 16 kind + 4 g + e, kind 0/1: dK columns (32 kind + 8 g + 4 h + e), 2/3: dV
        __shared__ float cs[NW][2][64];
        float v[64];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[4 * g + e] = bf16_round(dk0[4 * g + e] * scale);
                v[16 + 4 * g + e] = bf16_round(dk1[4 * g + e] * scale);
                v[32 + 4 * g + e] = bf16_round(dv0[4 * g + e]);
                v[48 + 4 * g + e] = bf16_round(dv1[4 * g + e]);
            }
        half_wave_colsum<64>(v, r);
        cs[w][h][2 * r] = v[0];
        cs[w][h][2 * r + 1] = v[1];
        __syncthreads();
        if (tid < 128) {
            const int hh = tid >> 6, i = tid & 63;
            float t = 0.f;
#pragma unroll
            for (int k = 0; k < NW; ++k) t += cs[k][hh][i];   // fixed order: deterministic
            const int kind = i >> 4, g = (i >> 2) & 3, e = i & 3;
            const int c = 32 * (kind & 1) + 8 * g + 4 * hh + e;
            const int col = (kind < 2 ? H * HD : 2 * H * HD) + hd * HD + c;
            // partial rows are per 128 tokens: an 8-wave workgroup (256 keys) fills two, the second with 0
            const size_t row = (size_t)b * (T / 128) + kbi * (BK / 128);
            bias_part[row * (3 * H * HD) + col] = t;
            if (BK == 256) bias_part[(row + 1) * (3 * H * HD) + col] = 0.f;
        }
    }
}

// ---------------------------------------------------------------------------- dQ (query-owned)
// Mirrors the forward: workgroup = 128 queries (query on the lane), key tiles of 64 staged in LDS.
// dP^T = V.dO^T and S^T = K.Q^T (row-read A), dS^T = P^T * (dP^T - delta) in registers, then
// dQ^T += K^T.dS^T with K^T from the transposed read of a plain K image and dS^T as the B operand.
// No atomics, no LDS round trip for dS.
// (a second in-flight K / V set — two tiles of prefetch — spills at 256 VGPRs: one set)
template <bool CAUSAL, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout,
                                                          const float* __restrict__ lse, const bf16_t* __restrict__ out,
                                                          float* __restrict__ delta,
                                                          bf16_t* __restrict__ dqkv, int T, int H, int nbh, float scale,
                                                          float* __restrict__ bias_part) {
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    constexpr int BM = 32 * NW, BN = 64;
    __shared__ __attribute__((aligned(16))) bf16_t Kr[2][BN * HD];  // swizzled, row reads
    __shared__ __attribute__((aligned(16))) bf16_t Kp[2][BN * HD];  // plain, transposed reads
    __shared__ __attribute__((aligned(16))) bf16_t Vr[2][BN * HD];  // swizzled, row reads
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, r = lane & 31;
    // wave-uniform (an SGPR): the causal tile tests become scalar branches, not exec-masked regions
    // (whose conservative wait bookkeeping drains in-flight loads)
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    int bh, qb;
    head_xcd_map(blockIdx.x, nbh, T / BM, CAUSAL, bh, qb);  // heavy (late) query blocks first
    const int b = bh / H, hd = bh - b * H;
    const int ldq = 3 * H * HD, ldo = H * HD;
    const bf16_t* qbase = qkv + (size_t)b * T * ldq + hd * HD;
    const bf16_t* kbase = qbase + H * HD;
    const bf16_t* vbase = qbase + 2 * H * HD;
    const bf16_t* dobase = dout + (size_t)b * T * ldo + hd * HD;
    const int qblk = qb * BM;
    const int q0 = qblk + 32 * w;
    const int qi = q0 + r;
    const float lse_q = lse[(size_t)bh * T + qi] * 1.4426950408889634f;
    const float sl2 = scale * 1.4426950408889634f;

    // delta = rowsum(dO * O) of this lane's query, from the dO fragments the lane loads anyway plus
    // the same slice of O (the two half-waves h hold the two halves of the row); written for the
    // dK/dV kernel, which runs after this one (no separate delta pass over O and dO)
    bf16x8_t qf[4], df[4];
    float dl_q = 0.f;
    const bf16_t* obase = out + (size_t)b * T * ldo + hd * HD;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        qf[s] = as_bf16x8(*(const uint4*)(qbase + (size_t)qi * ldq + 16 * s + 8 * h));
        const uint4 dr = *(const uint4*)(dobase + (size_t)qi * ldo + 16 * s + 8 * h);
        df[s] = as_bf16x8(dr);
        float gv[8], ov[8];
        unpack8(dr, gv);
        unpack8(*(const uint4*)(obase + (size_t)qi * ldo + 16 * s + 8 * h), ov);
#pragma unroll
        for (int k = 0; k < 8; ++k) dl_q += gv[k] * ov[k];
    }
    dl_q += __shfl_xor(dl_q, 32, 64);
    if (h == 0) delta[(size_t)bh * T + qi] = dl_q;
    f32x16 dq0 = {}, dq1 = {};
    // -delta as the dP^T chains' initial accumulator (the lane's query is fixed): the chain leaves
    // dP^T - delta and dS^T = P^T * (dP^T - delta) is one multiply per score
    f32x16 ndl;
#pragma unroll
    for (int i = 0; i < 16; ++i) ndl[i] = -dl_q;
    const int tq = (lane & 15) >> 2, tp = lane & 3, tcol = 16 * ((lane >> 4) & 1) + 4 * tp;
    int nkb = T / BN;
    if (CAUSAL) {
        const int lim = (qblk + BM + BN - 1) / BN;
        nkb = lim < nkb ? lim : nkb;
    }
    // staging registers as named scalars (an indexed array lands in scratch)
    uint4 kreg0 = {}, kreg1 = {}, vreg0 = {}, vreg1 = {};
    const int srow0 = tid >> 3, sch = tid & 7, srow1 = srow0 + 32;
    auto gload_to = [&](int kb, uint4& k0, uint4& k1, uint4& v0, uint4& v1) {
        const size_t g0 = (size_t)(kb * BN + srow0) * ldq + sch * 8, g1 = g0 + (size_t)32 * ldq;
        k0 = *(const uint4*)(kbase + g0);
        v0 = *(const uint4*)(vbase + g0);
        if constexpr (NW == 4) {
            k1 = *(const uint4*)(kbase + g1);
            v1 = *(const uint4*)(vbase + g1);
        }
    };
    auto gload = [&](int kb) { gload_to(kb, kreg0, kreg1, vreg0, vreg1); };
    auto sstore = [&](int buf) {
        *(uint4*)(Kr[buf] + srow0 * HD + rsw(srow0, sch)) = kreg0;
        *(uint4*)(Kp[buf] + swz_tr(srow0, sch * 8)) = kreg0;
        *(uint4*)(Vr[buf] + srow0 * HD + rsw(srow0, sch)) = vreg0;
        if constexpr (NW == 4) {
            *(uint4*)(Kr[buf] + srow1 * HD + rsw(srow1, sch)) = kreg1;
            *(uint4*)(Kp[buf] + swz_tr(srow1, sch * 8)) = kreg1;
            *(uint4*)(Vr[buf] + srow1 * HD + rsw(srow1, sch)) = vreg1;
        }
    };
    // the tile of keys kb, staged in LDS buffer `buf`
    auto compute_tile = [&](int kb, int buf) {
        const bf16_t* Kr_ = Kr[buf];
        const bf16_t* Kp_ = Kp[buf];
        const bf16_t* Vr_ = Vr[buf];
        if (!CAUSAL || kb * BN <= q0 + 31) {
            f32x16 s0 = {}, s1 = {}, p0, p1;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int r1 = 32 + r;
                const int c0 = rsw(r, 2 * s + h), c1 = rsw(r1, 2 * s + h);
                const bf16x8_t ak0 = as_bf16x8(*(const uint4*)(Kr_ + r * HD + c0));
                const bf16x8_t ak1 = as_bf16x8(*(const uint4*)(Kr_ + r1 * HD + c1));
                const bf16x8_t av0 = as_bf16x8(*(const uint4*)(Vr_ + r * HD + c0));
                const bf16x8_t av1 = as_bf16x8(*(const uint4*)(Vr_ + r1 * HD + c1));
                s0 = MFMA32(ak0, qf[s], s0);
                s1 = MFMA32(ak1, qf[s], s1);
                p0 = MFMA32(av0, df[s], s == 0 ? ndl : p0);
                p1 = MFMA32(av1, df[s], s == 0 ? ndl : p1);
            }
            if (CAUSAL && kb * BN + BN - 1 > q0) {  // diagonal tile: mask keys > query
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key0 = kb * BN + (i & 3) + 8 * (i >> 2) + 4 * h;
                    const float e0 = key0 > qi ? 0.f : fast_exp2(s0[i] * sl2 - lse_q);
                    const float e1 = key0 + 32 > qi ? 0.f : fast_exp2(s1[i] * sl2 - lse_q);
                    s0[i] = e0 * p0[i];  // dS^T
                    s1[i] = e1 * p1[i];
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    s0[i] = fast_exp2(s0[i] * sl2 - lse_q) * p0[i];
                    s1[i] = fast_exp2(s1[i] * sl2 - lse_q) * p1[i];
                }
            }
            const bf16x8_t d00 = cvt8(s0, 0), d01 = cvt8(s0, 8), d10 = cvt8(s1, 0), d11 = cvt8(s1, 8);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const bf16x8_t ds = t == 0 ? (s2 == 0 ? d00 : d01) : (s2 == 0 ? d10 : d11);
                    const int kr = 32 * t + 16 * s2 + 4 * h + tq;
                    const bf16x8_t a0 = tr_pair(Kp_ + swz_tr(kr, tcol), Kp_ + swz_tr(kr + 8, tcol));
                    const bf16x8_t a1 = tr_pair(Kp_ + swz_tr(kr, 32 + tcol), Kp_ + swz_tr(kr + 8, 32 + tcol));
                    dq0 = MFMA32(a0, ds, dq0);
                    dq1 = MFMA32(a1, ds, dq1);
                }
        }
    };
    gload(0);
    sstore(0);
    __syncthreads();
    for (int kb = 0; kb < nkb; ++kb) {
        const int buf = kb & 1;
        const bool has_next = kb + 1 < nkb;
        if (has_next) gload(kb + 1);
        compute_tile(kb, buf);
        if (has_next) sstore(buf ^ 1);
        __syncthreads();
    }
    bf16_t* qrow = dqkv + ((size_t)b * T + qi) * ldq + hd * HD;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int d = 8 * g + 4 * h;
        float a[4] = {dq0[4 * g] * scale, dq0[4 * g + 1] * scale, dq0[4 * g + 2] * scale, dq0[4 * g + 3] * scale};
        *(uint2*)(qrow + d) = pack4(a);
        float a2[4] = {dq1[4 * g] * scale, dq1[4 * g + 1] * scale, dq1[4 * g + 2] * scale, dq1[4 * g + 3] * scale};
        *(uint2*)(qrow + 32 + d) = pack4(a2);
    }
    if (bias_part != nullptr) {
        // value i = 16 kind + 4 g + e: dQ column 32 kind + 8 g + 4 h + e
        __shared__ float cs[NW][2][32];
        float v[32];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[4 * g + e] = bf16_round(dq0[4 * g + e] * scale);
                v[16 + 4 * g + e] = bf16_round(dq1[4 * g + e] * scale);
            }
        half_wave_colsum<32>(v, r);
        cs[w][h][r] = v[0];
        __syncthreads();
        if (tid < 64) {
            const int hh = tid >> 5, i = tid & 31;
            float t = 0.f;
#pragma unroll
            for (int k = 0; k < NW; ++k) t += cs[k][hh][i];   // fixed order: deterministic
            const int kind = i >> 4, g = (i >> 2) & 3, e = i & 3;
            const int col = hd * HD + 32 * kind + 8 * g + 4 * hh + e;
            const size_t row = (size_t)b * (T / 128) + qb * (BM / 128);
            bias_part[row * (3 * H * HD) + col] = t;
            if (BM == 256) bias_part[(row + 1) * (3 * H * HD) + col] = 0.f;
        }
    }
}

// launch a dK/dV kernel with `dl` bytes of dynamic LDS (raising the kernel's limit past the 64 KiB
// default once, for T > 8192)
template <typename Kern, typename... Args>
static void dkdv_launch(Kern kern, int grid, int threads, size_t dl, hipStream_t s, Args... args) {
    if (dl > 64 * 1024) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dl);
    kern<<<grid, threads, dl, s>>>(args...);
}

TDL_API int tdl_colsum_f32(const float* part, int G, int N, int ld, float* acc, hipStream_t s);  // norm_act.hip

// bias_acc (nullable): fp32 [3 H HD] accumulator of the qkv bias gradient (+= column sums of dqkv,
// computed inside the two kernels); bias_part: workspace of (B T / 128) x 3 H HD floats.
TDL_API int tdl_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv, float* bias_acc,
                         float* bias_part, float* delta, int B, int T, int H, int D, float scale, int causal,
                         hipStream_t s) {
    if (D != HD || T % 128 != 0 || T > ATTN_BWD_MAXT) return (int)hipErrorInvalidValue;
    const size_t dl = (size_t)2 * T * sizeof(float);   // dK/dV dynamic LDS: lse + delta of T queries
    if ((bias_acc == nullptr) != (bias_part == nullptr)) return (int)hipErrorInvalidValue;
    // the dQ kernel also produces delta = rowsum(dO * O) for the dK/dV kernel, so it runs first
    const int grid = B * H * (T / 128);
    auto Ob = (const bf16_t*)out;
    auto Q = (const bf16_t*)qkv;
    auto dO = (const bf16_t*)dout;
    auto dQKV = (bf16_t*)dqkv;
    const int nb = attn_nbh_arg(B * H);
    float* bp = bias_part;
    const int g8 = B * H * (T / 256);
    const bool w8 = causal && T % 256 == 0;
    if (causal) {
        if (w8 && attn_waves(1) == 8) attn_bwd_dq_kernel<true, 8><<<g8, 512, 0, s>>>(Q, dO, lse, Ob, delta, dQKV, T, H, nb, scale, bp);
        else attn_bwd_dq_kernel<true><<<grid, 256, 0, s>>>(Q, dO, lse, Ob, delta, dQKV, T, H, nb, scale, bp);
        if (w8 && attn_waves(2) == 8) dkdv_launch(attn_bwd_dkdv_kernel<true, 1, 2, 8>, g8, 512, dl, s, Q, dO, lse, delta, dQKV, T, H, nb, scale, bp);
        else if (dkdv_ns() == 2) dkdv_launch(attn_bwd_dkdv_kernel<true, 2, 1>, grid, 256, dl, s, Q, dO, lse, delta, dQKV, T, H, nb, scale, bp);
        else if (dkdv_pf() == 2) dkdv_launch(attn_bwd_dkdv_kernel<true, 1, 2>, grid, 256, dl, s, Q, dO, lse, delta, dQKV, T, H, nb, scale, bp);
        else dkdv_launch(attn_bwd_dkdv_kernel<true, 1, 1>, grid, 256, dl, s, Q, dO, lse, delta, dQKV, T, H, nb, scale, bp);
    } else {
        attn_bwd_dq_kernel<false><<<grid, 256, 0, s>>>(Q, dO, lse, Ob, delta, dQKV, T, H, nb, scale, bp);
        if (dkdv_ns() == 2) dkdv_launch(attn_bwd_dkdv_kernel<false, 2, 1>, grid, 256, dl, s, Q, dO, lse, delta, dQKV, T, H, nb, scale, bp);
        else if (dkdv_pf() == 2) dkdv_launch(attn_bwd_dkdv_kernel<false, 1, 2>, grid, 256, dl, s, Q, dO, lse, delta, dQKV, T, H, nb, scale, bp);
        else dkdv_launch(attn_bwd_dkdv_kernel<false, 1, 1>, grid, 256, dl, s, Q, dO, lse, delta, dQKV, T, H, nb, scale, bp);
    }
    if (bias_acc != nullptr) {
        const int rc = (int)hipGetLastError();
        if (rc) return rc;
        return tdl_colsum_f32(bias_part, B * (T / 128), 3 * H * HD, 3 * H * HD, bias_acc, s);
    }
    TDL_LAUNCH_CHECK();
}
