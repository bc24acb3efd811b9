// bf16 MFMA GEMM for gfx950 with fused epilogues: the projection GEMMs of the GPT-2 blocks and the
// tied LM head (reference call sites: the GPT2Block stages built at
// /root/reference/distributed_trainer.py:124-135 and the loss at :435-439).
//
//   C[m][n] = sum_k A(m, k) * B(n, k)      fp32 accumulate, bf16 operands
//
// Operand storage (template flags):
//   TA = false : A stored [M][lda]  (k contiguous)       TA = true : A stored [K][lda]  (m contiguous)
//   TB = false : B stored [N][ldb]  (k contiguous)       TB = true : B stored [K][ldb]  (n contiguous)
// so one kernel covers every product of a linear layer y = x W (W stored [in, out], HF Conv1D):
//   forward  y  = x  W     : A = x  [M][in]  (TA=0), B = W [in][out]  (TB=1)  (or W^T copy, TB=0)
//   dgrad    dx = dy W^T   : A = dy [M][out] (TA=0), B = W [in][out]  (TB=0: rows = in, k = out)
//   wgrad    dW = x^T dy   : A = x  [M][in]  (TA=1: rows = in, k = M), B = dy [M][out] (TB=1)
//
// Two kernels, both on a 256 x 256 x 64 workgroup tile of v_mfma_f32_16x16x32_bf16 (the 16x16
// shape holds a higher clock than 32x32x16 on random data, cdna_hip_programming.md rule 28):
//   gemm_p4  persistent grid (one workgroup per CU walks its tiles), 4 waves of 128 x 128 with the
//            256 accumulators per lane in AGPRs, operands register-staged two K steps ahead;
//   gemm_pp  one tile per workgroup, 8 waves of 128 x 64 in two groups staggered by one barrier,
//            operands staged by LDS-DMA (buffer_load ... lds), optional LDS-staged epilogue.
// In both, the MFMA "A" operand is the B tile and the MFMA "B" operand the A tile, so the
// accumulator of a tile holds D[n][m]: lane l owns output row m = l & 15 and FOUR CONSECUTIVE
// columns n = 4 (l >> 4) + 0..3 — one 8-byte bf16 / 16-byte fp32 vector store per (tile, lane).
//
// LDS images (16-byte chunks, conflict-free fragment reads):
//   k-contiguous tile [rows][64 k] : 128-B rows, 16-B chunk c of row r stored at c ^ (r & 7)
//       (source-address permutation, cdna_hip_programming.md rule 21); fragments via ds_read_b128.
//   row-contiguous tile [64 k][rows] : 32-B block b of k-row k stored at b ^ f(k),
//       f(k) = (k & 3) | ((k >> 1) & 4); fragments via ds_read_b64_tr_b16 (T10).
//
// Epilogues (EPI):
//   0 BF16      C = bf16(acc (+ bias[n]))
//   1 GELU      pre = acc + bias -> aux = bf16(pre), C = bf16(gelu_tanh(pre))
//   2 RESADD    C = bf16(C + acc (+ bias[n]))            (residual stream accumulate, in place)
//   3 DGELU     d = acc * gelu'(aux) -> C = bf16(d); colsum[n] += sum_m d   (fp32 atomics)
//   4 F32       C32[split][m][n] = acc                     (split-K slab / plain fp32 store)
//   5 F32ACC    C32[m][n] += acc                           (fp32 main_grad accumulate, split = 1)
//   6 F32ATOM   atomicAdd(C32[m][n], acc)                  (split-K straight into main_grad)
#include "common.h"

#include <cstdlib>
#include <type_traits>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 512;
constexpr int TILE_BYTES = BM * BK * 2;        // one operand, one K step: 32 KiB
constexpr int STAGE_BYTES = 2 * TILE_BYTES;    // A + B
constexpr int LDS_BYTES = 2 * STAGE_BYTES;     // two stages: 128 KiB

enum { EPI_BF16 = 0, EPI_GELU = 1, EPI_RESADD = 2, EPI_DGELU = 3, EPI_F32 = 4, EPI_F32ACC = 5, EPI_F32ATOM = 6 };

struct GemmParams {
    const bf16_t* A;
    const bf16_t* B;
    void* C;
    const bf16_t* bias;  // [N] or null
    bf16_t* aux;         // GELU: pre-activation out; DGELU: pre-activation in (both [M][ldc])
    float* colsum;       // DGELU: bias-gradient accumulator [N] or null
    int M, N, K;
    int lda, ldb, ldc;
    int k_per_split;      // K range of one blockIdx.y slice (multiple of BK)
    long long split_stride;  // EPI_F32: elements between split slabs
    int tiles_n, tiles;
    int splits;
    int group_m;          // tile order: 0 = row-major over (tm, tn); G > 0 = groups of G tile rows, tn-major
    unsigned long long* ts;  // diagnostics (tdl_gemm_set_timestamps): per-workgroup s_memrealtime stamps
    // gemm_pd GROUPED (weight gradients): a second product sharing K and the split, its items
    // numbered after the first product's items1 = tiles x splits
    struct Second {
        const bf16_t* A;
        const bf16_t* B;
        void* C;
        int M, N, lda, ldb, ldc, tiles_n, tiles;
        long long split_stride;
    } g2;
    int items1;
};

// timestamp slot `k` of this workgroup (wave 0, lane 0; 64 slots per workgroup)
__device__ __forceinline__ void stamp(const GemmParams& p, int k) {
    if (p.ts != nullptr && threadIdx.x == 0 && k < 64)
        p.ts[(size_t)(blockIdx.x + gridDim.x * blockIdx.y) * 64 + k] = __builtin_amdgcn_s_memrealtime();
}

// tile index (after the XCD remap) -> (tm, tn).  Grouped order (G tile rows per group, the tile
// column advancing slowest inside a group): the CUs of one XCD that run concurrently then share a
// G x (32 / G) block of A / B panels instead of ~3 A panels x every B panel (L2 reuse).
__device__ __forceinline__ void tile_coords(const GemmParams& p, int wg, int& tm, int& tn) {
    const int G = p.group_m;
    if (G <= 0) {
        tm = wg / p.tiles_n;
        tn = wg - tm * p.tiles_n;
        return;
    }
    const int tiles_m = p.tiles / p.tiles_n;
    const int per = G * p.tiles_n;
    const int grp = wg / per, in = wg - grp * per;
    const int first = grp * G;
    const int gs = tiles_m - first < G ? tiles_m - first : G;
    tn = in / gs;
    tm = first + (in - tn * gs);
}

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// 32-byte block swizzle of the row-contiguous (transposed-read) image
__device__ __forceinline__ int fsw(int k) { return (k & 3) | ((k >> 1) & 4); }

// Global -> LDS copies of one operand tile: 4 pieces of 1 KiB per wave, buffer_load ... lds through
// a per-K-step buffer resource whose base is the tile origin (uniform), so each lane keeps only its
// 4 loop-invariant 32-bit byte offsets.  (A layout with 64-B rows, one image per 32-deep k-half,
// was measured 7 % slower on every shape: the DMA then moves half cache lines.)
//   !TR: G = [rows][ld], LDS image [256 rows][64 k] (128-B rows, 16-B chunk c at c ^ (r & 7)).
//        Rows >= rmax fall outside the resource's num_records and read as zeros (ragged M / N).
//    TR: G = [K][ld], LDS image [64 k][256 rows] (512-B k-rows, 32-B block b at b ^ fsw(k));
//        column chunks clamped to rmax-8.
template <bool TR, int NW = 8>
struct Stager {
    static constexpr int NP = 32 / NW;  // 1-KiB pieces per wave per operand tile
    // piece i's lane offset = base[i & 1] + i * delta (delta uniform): two VGPRs per operand instead
    // of NP (the one-wave-per-SIMD kernel has no registers to hold them)
    uint32_t base[2];
    uint32_t delta;
    __device__ __forceinline__ void init(int ld, int r0, int rmax, int w, int lane) {
        if (!TR) {
            const int row = 8 * w + (lane >> 3);
            const int c = (lane & 7) ^ (lane >> 3);
            base[0] = base[1] = (uint32_t)(row * ld + 8 * c) * 2u;
            delta = (uint32_t)(8 * NW * ld) * 2u;
        } else {
#pragma unroll
            for (int par = 0; par < 2; ++par) {
                const int kr = 2 * (w + NW * par) + (lane >> 5);  // k-row of piece `par`
                const int c = (lane & 31) ^ (fsw(kr) << 1);
                int gc = 8 * c;
                gc = r0 + gc < rmax ? gc : rmax - 8 - r0;
                base[par] = (uint32_t)(kr * ld + gc) * 2u - (uint32_t)(par * 2 * NW * ld) * 2u;
            }
            delta = (uint32_t)(2 * NW * ld) * 2u;
        }
    }
    __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const bf16_t* G, int ld, int r0, int rmax, int k0) const {
        const bf16_t* b;
        uint32_t nrec;
        if (!TR) {
            b = G + (size_t)r0 * ld + k0;
            const long long rem = ((long long)(rmax - r0) * ld - k0) * 2;
            nrec = rem > 0x7fffffffll ? 0x7fffffffu : (uint32_t)rem;
        } else {
            b = G + (size_t)k0 * ld + r0;
            nrec = 0x7fffffffu;
        }
        return __builtin_amdgcn_make_buffer_rsrc((void*)b, 0, nrec, 0x00020000);
    }
    // piece i of this wave
    __device__ __forceinline__ void piece(__amdgpu_buffer_rsrc_t r, char* lds_tile, int w, int i) const {
        // opaque copy of the base: keeps the compiler from hoisting all NP offsets out of the K loop
        // (it did, and spilled them: a scratch reload + vmcnt(0) in front of every copy)
        uint32_t b = base[TR ? (i & 1) : 0];
        asm volatile("" : "+v"(b));
        const uint32_t off = b + (uint32_t)i * delta;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(lds_tile + (w + NW * i) * 1024), 16, off, 0, 0, 0);
    }
    __device__ __forceinline__ void issue(const bf16_t* G, int ld, int r0, int rmax, int k0, char* lds_tile, int w) const {
        const __amdgpu_buffer_rsrc_t r = rsrc(G, ld, r0, rmax, k0);
#pragma unroll
        for (int i = 0; i < NP; ++i) piece(r, lds_tile, w, i);
    }
    // register staging: the same copies as plain 16-byte loads into VGPRs, written to the same
    // lane-linear LDS image later (ds_write_b128)
    __device__ __forceinline__ void load_regs(const bf16_t* G, int ld, int r0, int rmax, int k0, u32x4_t (&v)[NP]) const {
        const __amdgpu_buffer_rsrc_t r = rsrc(G, ld, r0, rmax, k0);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            uint32_t b = base[TR ? (i & 1) : 0];
            asm volatile("" : "+v"(b));
            v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, b + (uint32_t)i * delta, 0, 0);
        }
    }
    __device__ __forceinline__ void write_regs(char* lds_tile, int w, int lane, const u32x4_t (&v)[NP]) const {
#pragma unroll
        for (int i = 0; i < NP; ++i) *(u32x4_t*)(lds_tile + (w + NW * i) * 1024 + lane * 16) = v[i];
    }
};

__device__ __forceinline__ short4_t tr_read(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(p));
}

// MFMA operand fragment (16 rows x 32 k) of a tile: lane l gets row rb + (l & 15),
// k = 32 ks + 8 (l >> 4) + 0..7.
template <bool TR>
__device__ __forceinline__ bf16x8_t frag(const char* tile, int rb, int ks, int lane) {
    if (!TR) {
        const int r = rb + (lane & 15);
        const int c = 4 * ks + (lane >> 4);
        return *(const bf16x8_t*)(tile + r * 128 + ((c ^ (r & 7)) << 4));
    } else {
        // ds_read_b64_tr_b16: lane 4q+p of a 16-lane group supplies k-row q, columns 4p..4p+3
        const int q = (lane & 15) >> 2, p = lane & 3;
        const int col = rb + 4 * p;
        const int kb = 32 * ks + 8 * (lane >> 4) + q;
        const int k2 = kb + 4;
        const char* a1 = tile + kb * 512 + ((((col >> 3) ^ (fsw(kb) << 1))) << 4) + ((col & 7) << 1);
        const char* a2 = tile + k2 * 512 + ((((col >> 3) ^ (fsw(k2) << 1))) << 4) + ((col & 7) << 1);
        const short4_t x = tr_read(a1), y = tr_read(a2);
        return __builtin_bit_cast(bf16x8_t, (short8_t)__builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
    }
}

// ============================================================================ 4-wave helpers
// Shared by the 4-wave persistent kernel (gemm_p4) and the ping-pong kernel's epilogue: 256-thread
// workgroups, one wave per SIMD, each wave a 128 x 128 block = 8 x 8 MFMA tiles whose 256
// accumulator registers live in AGPRs.
constexpr int PNTHR = 256;

// Fragments of the 4-wave kernel: the B fragments of both k-halves (the next half's are read while
// the current half's MFMAs use all eight), and ONE set of A fragments — row i of the next half is
// read into a[i] as soon as the current half's MFMAs of row i are done.
struct PFrags {
    bf16x8_t b[2][8], a[8];
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
    const uint32_t n = bytes <= 0 ? 0u : bytes > 0x7fffffffll ? 0x7fffffffu : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, n, 0x00020000);
}

// Epilogue of one wave's 128 x 128 block (rows from mw, columns from nw), branch-free: every access
// goes through a buffer resource whose num_records ends at row M, and columns >= N get an offset
// beyond it, so ragged edges are dropped (stores) or read as zero (loads) by the range check.
// (A per-tile `if` made hipcc hoist all 256 accumulator reads ahead of the stores: 256 VGPRs,
// spills, and a reload with vmcnt(0) at the head of the K loop.)
template <int T, class F>
__device__ __forceinline__ void for_tiles(F& fn) {
    if constexpr (T < 64) {
        fn(std::integral_constant<int, T>{});
        for_tiles<T + 1>(fn);
    }
}

// Epilogue of one wave's 128 x 128 block (rows from mw, columns from nw), tile by tile (T = 8 i + j
// in j-major order, the accumulators fetched by `get` only when the tile is stored), branch-free:
// every access goes through a buffer resource whose num_records ends at row M, and columns >= N
// get an offset beyond it, so ragged edges are dropped (stores) or read as zero (loads) by the range
// check.  (Per-tile `if`s made hipcc hoist ~100 accumulator reads ahead of the stores.)
template <int EPI, int NJ, class Get>
__device__ __forceinline__ void epilogue_store(const GemmParams& p, Get& get, int mw, int nw, int sp, int lane) {
    constexpr bool F32OUT = EPI >= EPI_F32;
    constexpr int ESZ = F32OUT ? 4 : 2;
    const int g = lane >> 4;
    const size_t row0 = (size_t)(EPI == EPI_F32 ? (long long)sp * p.split_stride : 0) + (size_t)mw * p.ldc;
    const long long rem = (long long)(p.M - mw) * p.ldc * ESZ;
    const __amdgpu_buffer_rsrc_t rc = make_rsrc((const char*)p.C + row0 * ESZ, rem);
    __amdgpu_buffer_rsrc_t rx = rc;
    if (EPI == EPI_GELU || EPI == EPI_DGELU) rx = make_rsrc((const char*)p.aux + row0 * ESZ, rem);
    const __amdgpu_buffer_rsrc_t rbias = make_rsrc(p.bias, p.bias != nullptr ? (long long)p.N * 2 : 0);
    const uint32_t lrow = (uint32_t)(lane & 15) * (uint32_t)p.ldc * ESZ;
    float csum[4];
    float bv[4];
    auto tile = [&](auto tc) {
        constexpr int T = decltype(tc)::value;
        constexpr int j = T / 8, i = T % 8;  // j-major: the bias / column sums of column block j
        if constexpr (j < NJ) {
        const int n = nw + 16 * j + 4 * g;
        const bool nok = n < p.N;
        if constexpr (i == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) csum[r] = 0.f, bv[r] = 0.f;
            if (EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_RESADD) {
                const u32x2_t b = __builtin_amdgcn_raw_buffer_load_b64(rbias, nok ? (uint32_t)n * 2u : 0x80000000u, 0, 0);
                unpack4(make_uint2(b.x, b.y), bv);
            }
        }
        const f32x4 a = get(std::integral_constant<int, i>{}, std::integral_constant<int, j>{});
        const uint32_t off = nok ? lrow + (uint32_t)(16 * i) * (uint32_t)p.ldc * ESZ + (uint32_t)n * ESZ : 0x80000000u;
        float v[4] = {a[0] + bv[0], a[1] + bv[1], a[2] + bv[2], a[3] + bv[3]};
        if constexpr (EPI == EPI_BF16) {
            const uint2 q = pack4(v);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{q.x, q.y}, rc, off, 0, 0);
        } else if constexpr (EPI == EPI_GELU) {
            const uint2 q = pack4(v);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{q.x, q.y}, rx, off, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
            const uint2 f = pack4(v);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{f.x, f.y}, rc, off, 0, 0);
        } else if constexpr (EPI == EPI_RESADD) {
            const u32x2_t o2 = __builtin_amdgcn_raw_buffer_load_b64(rc, off, 0, 0);
            float o[4];
            unpack4(make_uint2(o2.x, o2.y), o);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += o[r];
            const uint2 q = pack4(v);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{q.x, q.y}, rc, off, 0, 0);
        } else if constexpr (EPI == EPI_DGELU) {
            const u32x2_t u2 = __builtin_amdgcn_raw_buffer_load_b64(rx, off, 0, 0);
            float u[4];
            unpack4(make_uint2(u2.x, u2.y), u);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = a[r] * gelu_tanh_grad(u[r]);
                csum[r] += v[r];
            }
            const uint2 q = pack4(v);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{q.x, q.y}, rc, off, 0, 0);
        } else if constexpr (EPI == EPI_F32) {
            __builtin_amdgcn_raw_buffer_store_b128(
                u32x4_t{__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])}, rc,
                off, 0, 0);
        } else if constexpr (EPI == EPI_F32ACC) {
            const u32x4_t o = __builtin_amdgcn_raw_buffer_load_b128(rc, off, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(
                u32x4_t{__float_as_uint(v[0] + __uint_as_float(o.x)), __float_as_uint(v[1] + __uint_as_float(o.y)),
                        __float_as_uint(v[2] + __uint_as_float(o.z)), __float_as_uint(v[3] + __uint_as_float(o.w))},
                rc, off, 0, 0);
        } else {  // EPI_F32ATOM
#pragma unroll
            for (int r = 0; r < 4; ++r) __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(v[r], rc, off + 4u * r, 0, 0);
        }
        if constexpr (EPI == EPI_DGELU && i == 7) {
            if (p.colsum != nullptr) {
                // rows past M / columns past N had zero operands: they add nothing
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float t = csum[r];
                    t += __shfl_xor(t, 1, 64);
                    t += __shfl_xor(t, 2, 64);
                    t += __shfl_xor(t, 4, 64);
                    t += __shfl_xor(t, 8, 64);
                    csum[r] = t;
                }
                const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.colsum, (long long)p.N * 4);
                const int r = lane & 3;
                const float t = r == 0 ? csum[0] : r == 1 ? csum[1] : r == 2 ? csum[2] : csum[3];
                const bool writer = (lane & 15) < 4 && n + r < p.N;
                __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(t, rs, writer ? (uint32_t)(n + r) * 4u : 0x80000000u, 0, 0);
            }
        }
        // one tile at a time (keeps the accumulator read-out from being hoisted)
        __builtin_amdgcn_sched_barrier(0);
        }
    };
    for_tiles<0>(tile);
}

// ---- AGPR accumulators: tile T = 8 i + j (i: A tile, j: B tile) is acc[T].  The MFMAs are inline
// asm with "+a" operands: the 256 accumulator registers stay in AGPRs for the whole K loop and the
// register allocator knows they are live (with builtins hipcc shuffled 256 loop-carried accumulators
// through VGPRs; with a bare AGPR clobber it reused "free" AGPRs for its own values).
typedef f32x4 Acc[64];
template <int T>
__device__ __forceinline__ void amfma(Acc& acc, const bf16x8_t& b, const bf16x8_t& a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[T]) : "v"(b), "v"(a));
}
template <int T>
__device__ __forceinline__ void amfma0(Acc& acc, const bf16x8_t& b, const bf16x8_t& a) {  // C = 0: first K step
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc[T]) : "v"(b), "v"(a));
}
// an empty asm that reads and "writes" accumulators B..B+15 (ordering fence for their readers)
template <int B>
__device__ __forceinline__ void acc_fence(Acc& acc) {
    asm volatile("" : "+a"(acc[B + 0]), "+a"(acc[B + 1]), "+a"(acc[B + 2]), "+a"(acc[B + 3]), "+a"(acc[B + 4]),
                 "+a"(acc[B + 5]), "+a"(acc[B + 6]), "+a"(acc[B + 7]), "+a"(acc[B + 8]), "+a"(acc[B + 9]),
                 "+a"(acc[B + 10]), "+a"(acc[B + 11]), "+a"(acc[B + 12]), "+a"(acc[B + 13]), "+a"(acc[B + 14]),
                 "+a"(acc[B + 15]));
}
// 64 MFMAs of one 32-deep k-half in tile order T = 0..63; after MFMA T the hook issues that
// slot's companion instructions (global loads / LDS reads and writes), pinned by a scheduling fence
template <int H, int T, bool ZERO, class Hook>
__device__ __forceinline__ void mfma_run(Acc& acc, PFrags& f, Hook& hook) {
    if constexpr (T < 64) {
        if constexpr (ZERO) amfma0<T>(acc, f.b[H][T % 8], f.a[T / 8]);
        else amfma<T>(acc, f.b[H][T % 8], f.a[T / 8]);
        hook(std::integral_constant<int, T>{});
        __builtin_amdgcn_sched_barrier(0);
        mfma_run<H, T + 1, ZERO>(acc, f, hook);
    }
}

// ============================================================================ ping-pong kernel
// 256 x 256 x 64 tile, 8 waves as 2 (m) x 4 (n), 128 x 64 per wave (as gemm_kernel), but the two
// wave groups (wr = 0: waves 0-3, wr = 1: waves 4-7; one wave of each per SIMD) run STAGGERED by one
// barrier: while one wave of a SIMD runs its 16-MFMA cluster, its partner issues the next phase's
// fragment reads and LDS-DMA copies, so the copy-issue cost (the limiter of gemm_kernel /
// gemm_persistent8: profiles/r2_gemm_variants.jsonl) hides behind the partner's MFMAs
// (cdna_hip_programming.md, "The 256² 8-phase template").
//
// A K step is four phases, one output quadrant (4 m-tiles x 2 n-tiles x K 64 = 16 MFMAs) each:
//   P1 q(mh0, nh0): read A(mh0), B(nh0)   issue UB1(t+1)
//   P2 q(mh0, nh1): read B(nh1)           issue UA1(t+1)
//   P3 q(mh1, nh1): read A(mh1)           issue UA0(t+2)
//   P4 q(mh1, nh0): (B(nh0) still held)   issue UB0(t+2)
// LDS holds each operand tile as quarter units of 128 rows x 64 k (16 KiB, same swizzled 128-B
// rows as gemm_kernel), double-buffered PER UNIT (t & 1):
//   UA0 = A rows {0-63, 128-191} (each group's m-half 0), UA1 = A rows {64-127, 192-255},
//   UB0 = B rows {64 wc + 0..31}, UB1 = B rows {64 wc + 32..63}.
// Ordering (global phase index g; group 0 reads phase g between barriers 2g-2 and 2g-1, group 1
// between 2g-1 and 2g; both retire their reads with lgkmcnt(0) after the next barrier):
//   WAR: a copy issued in phase g may overwrite data last read in phase <= g-2 — each unit of
//        tile t+1 / t+2 above overwrites its tile-(t-1) / tile-t copy >= 2 phases after that read;
//   RAW: each wave keeps the copies of its last 4 phases in flight (s_waitcnt vmcnt(2 x issued
//        copies in phases g-3..g) before phase g's first barrier), so a unit issued in phase g is
//        readable from phase g+5 on — every unit is read >= 5 phases after its issue.
// copies allowed in flight at phase q's wait: 2 per issuing phase among q-3..q (PM / MK: issue
// masks of the previous / this K step)
constexpr int pp_vm_allow(int PM, int MK, int q) {
    int n = 0;
    for (int d = 0; d < 4; ++d) {
        const int x = q - d;  // <= 0: phase x + 4 of the previous step
        n += (x >= 1 ? (MK >> (x - 1)) & 1 : (PM >> (x + 3)) & 1) ? 2 : 0;
    }
    return n;
}
template <int N>
__device__ __forceinline__ void wait_vmc() {
    asm volatile("s_waitcnt vmcnt(%c0)" ::"n"(N) : "memory");
}

// LEPI (EPI_BF16 / EPI_GELU, one tile per workgroup): LDS-staged epilogue — after the K loop each
// wave writes its 128 x 64 bf16 block into its own 16 KiB of the (then idle) operand LDS (16-B chunks
// XOR-swizzled by row) and reads it back row-contiguous, so every store instruction writes 8 whole
// 128-B row segments (1 KiB) instead of 16 rows x 32 B: a quarter of the store instructions and
// L2 requests of the direct MFMA-layout store.
// LDS-staged epilogue of the 8-wave ping-pong kernel (EPI_BF16 / GELU / RESADD / DGELU):
// each wave writes its 128 x 64 bf16 block into its own 16 KiB of the (then idle) operand LDS
// (16-B chunks XOR-swizzled by row) and reads it back row-contiguous, so every store instruction
// writes 8 whole 128-B row segments (1 KiB) instead of 16 rows x 32 B: a quarter of the store
// instructions and L2 requests of the direct MFMA-layout store.  RESADD / DGELU bring their
// operand tile (residual C / pre-activation aux) in the same way reversed.
template <int EPI>
__device__ __forceinline__ void pp_lds_epilogue(const GemmParams& p, f32x4 (&acc)[8][4], char* smem, int m0, int n0,
                                                int wr, int wc, int w, int lane) {
    char* ws = smem + w * 16384;
    const int g = lane >> 4, rl = lane & 15;
    const int mw = m0 + wr * 128, nw = n0 + wc * 64;
    const long long rem = (long long)(p.M - mw) * p.ldc * 2;
    const __amdgpu_buffer_rsrc_t rc = make_rsrc((const bf16_t*)p.C + (size_t)mw * p.ldc, rem);
    const __amdgpu_buffer_rsrc_t rx =
        EPI == EPI_GELU || EPI == EPI_DGELU ? make_rsrc(p.aux + (size_t)mw * p.ldc, rem) : rc;
    const __amdgpu_buffer_rsrc_t rbias = make_rsrc(p.bias, p.bias != nullptr ? (long long)p.N * 2 : 0);
    float bv[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = nw + 16 * j + 4 * g;
        const u32x2_t b = __builtin_amdgcn_raw_buffer_load_b64(rbias, n < p.N ? (uint32_t)n * 2u : 0x80000000u, 0, 0);
        unpack4(make_uint2(b.x, b.y), bv[j]);
    }
    // read-back: lane -> row 8 q + (lane >> 3), 16-B chunk lane & 7 (columns nw + 8 c ..+7)
    const int cb = lane & 7;
    const uint32_t coff = nw + 8 * cb < p.N ? (uint32_t)(nw + 8 * cb) * 2u : 0x80000000u;
    auto pass = [&](bool post, __amdgpu_buffer_rsrc_t dst) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[i][j][r] + bv[j][r];
                    if (post) v[r] = gelu_tanh(v[r]);
                }
                const int row = 16 * i + rl, ch = 2 * j + (g >> 1);
                *(uint2*)(ws + row * 128 + ((ch ^ (row & 7)) << 4) + ((g & 1) << 3)) = pack4(v);
            }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row = 8 * q + (lane >> 3);
            const uint4 val = *(const uint4*)(ws + row * 128 + ((cb ^ (row & 7)) << 4));
            const uint32_t off = coff == 0x80000000u ? coff : (uint32_t)row * (uint32_t)p.ldc * 2u + coff;
            __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{val.x, val.y, val.z, val.w}, dst, off, 0, 0);
        }
    };
    if constexpr (EPI == EPI_RESADD || EPI == EPI_DGELU) {
        // the operand tile (residual C / pre-activation aux) comes in the same way reversed:
        // row-contiguous 16-B loads -> swizzled LDS -> each lane's MFMA-layout 4-vectors, which
        // the lane combines with its accumulators in fp32 and writes back to the same 8 bytes
        const __amdgpu_buffer_rsrc_t rs = EPI == EPI_RESADD ? rc : rx;
        uint4 ld[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row = 8 * q + (lane >> 3);
            const uint32_t off = coff == 0x80000000u ? coff : (uint32_t)row * (uint32_t)p.ldc * 2u + coff;
            const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
            ld[q] = make_uint4(v[0], v[1], v[2], v[3]);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row = 8 * q + (lane >> 3);
            *(uint4*)(ws + row * 128 + ((cb ^ (row & 7)) << 4)) = ld[q];
        }
        float csum[4][4];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = 16 * i + rl, ch = 2 * j + (g >> 1);
                char* a8 = ws + row * 128 + ((ch ^ (row & 7)) << 4) + ((g & 1) << 3);
                float o[4], v[4];
                unpack4(*(const uint2*)a8, o);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (EPI == EPI_RESADD) {
                        v[r] = acc[i][j][r] + bv[j][r] + o[r];
                    } else {
                        v[r] = acc[i][j][r] * gelu_tanh_grad(o[r]);
                        csum[j][r] = (i == 0 ? 0.f : csum[j][r]) + v[r];
                    }
                }
                *(uint2*)a8 = pack4(v);
            }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row = 8 * q + (lane >> 3);
            const uint4 val = *(const uint4*)(ws + row * 128 + ((cb ^ (row & 7)) << 4));
            const uint32_t off = coff == 0x80000000u ? coff : (uint32_t)row * (uint32_t)p.ldc * 2u + coff;
            __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{val.x, val.y, val.z, val.w}, rc, off, 0, 0);
        }
        if constexpr (EPI == EPI_DGELU) {
            if (p.colsum != nullptr) {  // rows past M / columns past N had zero operands
                const __amdgpu_buffer_rsrc_t rsum = make_rsrc(p.colsum, (long long)p.N * 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float t = csum[j][r];
                        t += __shfl_xor(t, 1, 64);
                        t += __shfl_xor(t, 2, 64);
                        t += __shfl_xor(t, 4, 64);
                        t += __shfl_xor(t, 8, 64);
                        csum[j][r] = t;
                    }
                    const int n = nw + 16 * j + 4 * g, r = lane & 3;
                    const float t = r == 0 ? csum[j][0] : r == 1 ? csum[j][1] : r == 2 ? csum[j][2] : csum[j][3];
                    const bool writer = (lane & 15) < 4 && n + r < p.N;
                    __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(t, rsum, writer ? (uint32_t)(n + r) * 4u : 0x80000000u, 0, 0);
                }
            }
        }
    } else if constexpr (EPI == EPI_GELU) {
        pass(false, rx);  // the pre-activation
        pass(true, rc);
    } else {
        pass(false, rc);
    }
}

template <bool TA, bool TB, int EPI, bool LEPI = false>
__global__ __launch_bounds__(NTHR, 1) void gemm_pp(GemmParams p) {
    static_assert(!LEPI || EPI <= EPI_DGELU, "LDS epilogue: bf16 outputs");
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];  // [buf 2][UA0 UA1 UB0 UB1][16 KiB]
    constexpr int UNIT = 16384, BUF = 4 * UNIT;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 2, wc = w & 3;
    auto coords = [&](int item, int& mm, int& nn) {
        const int wg = xcd_remap(item, p.tiles);
        int tm, tn;
        tile_coords(p, wg, tm, tn);
        mm = tm * BM;
        nn = tn * BN;
    };
    int m0, n0;
    coords(blockIdx.x, m0, n0);
    const int kbeg = blockIdx.y * p.k_per_split;
    const int nk = p.k_per_split / BK;  // >= 2 (host)
    stamp(p, 0);

    // Per-lane byte offsets of piece 0 of each unit (piece 1 adds the uniform di_a / di_b).
    //  k-contiguous operand: unit image [128 unit-rows][64 k], 128-B rows, 16-B chunk c of row r at
    //    c ^ (r & 7); piece = 8 rows; wave w copies unit-rows 8 w + (lane >> 3) (+ 64 for piece 1).
    //    A unit mh: unit-row u -> A row mh*64 + u (+ 64 when u >= 64)
    //    B unit nh: unit-row u -> B row 64 (u >> 5) + 32 nh + (u & 31)
    //  row-contiguous operand (TA / TB: stored [K][ld]): unit image [64 k][128 unit-rows], 256-B
    //    k-rows (one LDS bank row), 32-B window v of k-row k stored at v ^ fsw(k) (conflict-free
    //    ds_read_b64_tr_b16: the 8 k-rows a 32-lane half reads land in 8 distinct windows); piece =
    //    4 k-rows; wave w copies k-rows 4 w + (lane >> 4) (+ 32 for piece 1); a lane's 16-B chunk c
    //    holds unit-rows 8c..8c+7, clamped into [0, rmax - 8] for ragged M / N.
    uint32_t uoff[4];
    uint32_t di_a, di_b;
    {
        const int lr = lane >> 3, ch = (lane & 7) ^ lr;
        const int kr = 4 * w + (lane >> 4);
        const int cs = (lane & 15) ^ (((lane >> 4) | ((w & 2) << 1)) << 1);  // chunk whose slot is lane & 15
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool isA = u < 2;
            const bool tr = isA ? TA : TB;
            const int ld = isA ? p.lda : p.ldb;
            const int h = isA ? u : u - 2;
            if (!tr) {
                const int row = isA ? h * 64 + 8 * w + lr : 64 * (w >> 2) + 32 * h + 8 * (w & 3) + lr;
                uoff[u] = (uint32_t)(row * ld + 8 * ch) * 2u;
            } else {
                const int r0 = isA ? m0 : n0, rmax = isA ? p.M : p.N;
                int col = isA ? h * 64 + 8 * cs + (cs >= 8 ? 64 : 0) : 64 * (cs >> 2) + 32 * h + 8 * (cs & 3);
                col = r0 + col + 8 <= rmax ? col : rmax - 8 - r0;
                uoff[u] = (uint32_t)(kr * ld + col) * 2u;
            }
        }
        di_a = TA ? 32u * (uint32_t)p.lda * 2u : 128u * (uint32_t)p.lda * 2u;
        di_b = TB ? 32u * (uint32_t)p.ldb * 2u : 128u * (uint32_t)p.ldb * 2u;
    }
    auto rsrc = [&](const bf16_t* G, int ld, int r0, int rmax, int k0, bool tr) {
        if (tr) return make_rsrc(G + (size_t)k0 * ld + r0, 0x7fffffffll);
        const long long rem = ((long long)(rmax - r0) * ld - k0) * 2;
        return make_rsrc(G + (size_t)r0 * ld + k0, rem);
    };
    // unit u (0 UA0, 1 UA1, 2 UB0, 3 UB1) of K step t -> LDS buffer t & 1
    auto issue = [&](int u, int t) {
        const int mm = m0, nn = n0;
        const int k0 = kbeg + t * BK;
        char* dst = smem + (t & 1) * BUF + u * UNIT + w * 1024;
        const bool isA = u < 2;
        const __amdgpu_buffer_rsrc_t r = isA ? rsrc(p.A, p.lda, mm, p.M, k0, TA) : rsrc(p.B, p.ldb, nn, p.N, k0, TB);
        uint32_t o = uoff[u];
        const uint32_t di = isA ? di_a : di_b;
        asm volatile("" : "+v"(o));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)dst, 16, o, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(dst + 8 * 1024), 16, o + di, 0, 0, 0);
    };
    // MFMA operand fragment (16 unit-rows from rb x 32 k) of a unit: lane l gets unit-row
    // rb + (l & 15), k = 32 ks + 8 (l >> 4) + 0..7
    auto frag_ = [&](const char* U, int rb, int ks, auto trc) -> bf16x8_t {
        if constexpr (!decltype(trc)::value) {
            const int r = rb + (lane & 15);
            const int c = 4 * ks + (lane >> 4);
            return *(const bf16x8_t*)(U + r * 128 + ((c ^ (r & 7)) << 4));
        } else {
            // ds_read_b64_tr_b16: lane 4q+p of a 16-lane group supplies k-row q, columns 4p..4p+3
            const int q = (lane & 15) >> 2, pp = lane & 3;
            const int col = rb + 4 * pp;
            const int kb = 32 * ks + 8 * (lane >> 4) + q, k2 = kb + 4;
            const short4_t x = tr_read(U + kb * 256 + ((((col >> 3) ^ (fsw(kb) << 1))) << 4) + ((col & 7) << 1));
            const short4_t y = tr_read(U + k2 * 256 + ((((col >> 3) ^ (fsw(k2) << 1))) << 4) + ((col & 7) << 1));
            return __builtin_bit_cast(bf16x8_t, (short8_t)__builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
        }
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8_t FA[4][2], FB0[2][2], FB1[2][2];

    auto readA = [&](int buf, int mh) {
        const char* U = smem + buf * BUF + mh * UNIT;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) FA[i][ks] = frag_(U, wr * 64 + 16 * i, ks, std::integral_constant<bool, TA>{});
    };
    auto readB = [&](bf16x8_t (&F)[2][2], int buf, int nh) {
        const char* U = smem + buf * BUF + (2 + nh) * UNIT;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) F[j][ks] = frag_(U, wc * 32 + 16 * j, ks, std::integral_constant<bool, TB>{});
    };
    auto quad = [&](const bf16x8_t (&F)[2][2], int mh, int nh) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[4 * mh + i][2 * nh + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(F[j][ks], FA[i][ks], acc[4 * mh + i][2 * nh + j], 0, 0, 0);
    };
    // one phase: [reads] [copies] vmcnt(n) barrier lgkmcnt(0) | MFMA cluster | barrier
    auto phase_sync = [&](auto nc) {
        __builtin_amdgcn_sched_barrier(0);
        wait_vmc<decltype(nc)::value>();
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
    };
    auto phase_end = [&]() {
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // K step t with this step's / the previous step's issue masks (bit q-1: phase q issues)
    auto step = [&](int t, auto pmc, auto mc) {
        constexpr int PM = decltype(pmc)::value, MK = decltype(mc)::value;
        using V1 = std::integral_constant<int, pp_vm_allow(PM, MK, 1)>;
        using V2 = std::integral_constant<int, pp_vm_allow(PM, MK, 2)>;
        using V3 = std::integral_constant<int, pp_vm_allow(PM, MK, 3)>;
        using V4 = std::integral_constant<int, pp_vm_allow(PM, MK, 4)>;
        const int cur = t & 1;
        // P1
        readA(cur, 0);
        readB(FB0, cur, 0);
        if (MK & 1) issue(3, t + 1);
        phase_sync(V1{});
        quad(FB0, 0, 0);
        phase_end();
        // P2
        readB(FB1, cur, 1);
        if (MK & 2) issue(1, t + 1);
        phase_sync(V2{});
        quad(FB1, 0, 1);
        phase_end();
        // P3
        readA(cur, 1);
        if (MK & 4) issue(0, t + 2);
        phase_sync(V3{});
        quad(FB1, 1, 1);
        phase_end();
        // P4
        if (MK & 8) issue(2, t + 2);
        phase_sync(V4{});
        quad(FB0, 1, 0);
        phase_end();
    };

    // prologue: UA0(0) UB0(0) UB1(0) UA1(0) UA0(1) UB0(1) (the copies of "phases" -5..0)
    issue(0, 0);
    issue(2, 0);
    issue(3, 0);
    issue(1, 0);
    issue(0, 1);
    issue(2, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // UA0(0), UB0(0) landed
    __builtin_amdgcn_s_barrier();
    if (wr) __builtin_amdgcn_s_barrier();  // stagger: group 1 runs one barrier behind
    using I15 = std::integral_constant<int, 15>;
    using I3 = std::integral_constant<int, 3>;
    using I0 = std::integral_constant<int, 0>;
    auto epilogue = [&]() {
        auto get = [&](auto ic, auto jc) { return acc[decltype(ic)::value][decltype(jc)::value]; };
        epilogue_store<EPI, 4>(p, get, m0 + wr * 128, n0 + wc * 64, blockIdx.y, lane);
    };
    if constexpr (LEPI) {
        int t = 0;
#pragma clang loop unroll(disable)
        for (; t < nk - 2; ++t) step(t, I15{}, I15{});
        step(t, I15{}, I3{});
        step(t + 1, I3{}, I0{});
        stamp(p, 1);
        // group 0's extra barrier first: past it every wave has retired its last fragment reads and
        // waited its last copies (vmcnt(0) in the final phase), so the operand LDS is free
        if (!wr) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");  // no LDS access of the epilogue moves above that barrier
        __builtin_amdgcn_sched_barrier(0);
        pp_lds_epilogue<EPI>(p, acc, smem, m0, n0, wr, wc, w, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(p, 2);
        return;
    } else {
        int t = 0;
#pragma clang loop unroll(disable)
        for (; t < nk - 2; ++t) step(t, I15{}, I15{});
        step(t, I15{}, I3{});      // t = nk-2: P3 / P4 have no step t+2
        step(t + 1, I3{}, I0{});   // t = nk-1: nothing left to stage
        epilogue();
    }
    if (!wr) __builtin_amdgcn_s_barrier();  // match group 1's extra barrier
}


template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, I + 1>(f);
    }
}

// LDS-staged epilogue of one wave's 128 x 128 block with bf16 outputs (EPI_BF16 / GELU / RESADD /
// DGELU), in two passes of 64 rows through the wave's own 16 KiB of an idle LDS stage: the MFMA-layout
// accumulators (lane: row l & 15, 4 consecutive columns) go to LDS as 8-byte pieces and come back
// row-contiguous, so each store instruction writes 4 whole 256-B row segments instead of 16 rows x
// 32 B (a quarter of the store instructions, full-line writes).  Staging rows are 272 B apart (the
// 16 rows one 8-byte store instruction touches hit distinct banks) and every address is a per-lane
// base plus an immediate.
// Operand tiles of RESADD (C) / DGELU (aux) come in the same way reversed.
constexpr int P4_EPI_PITCH = 272, P4_EPI_WAVE = 64 * P4_EPI_PITCH;
template <int EPI>
__device__ __forceinline__ void p4_lds_epilogue(const GemmParams& p, Acc& acc, char* ws, int mw, int nw, int lane) {
    const int g = lane >> 4, rl = lane & 15;
    const long long rem = (long long)(p.M - mw) * p.ldc * 2;
    const __amdgpu_buffer_rsrc_t rc = make_rsrc((const bf16_t*)p.C + (size_t)mw * p.ldc, rem);
    const __amdgpu_buffer_rsrc_t rx =
        EPI == EPI_GELU || EPI == EPI_DGELU ? make_rsrc(p.aux + (size_t)mw * p.ldc, rem) : rc;
    const __amdgpu_buffer_rsrc_t rbias = make_rsrc(p.bias, p.bias != nullptr ? (long long)p.N * 2 : 0);
    // row-contiguous side: lane -> row 4 q + (lane >> 4) of the pass, 16-B chunk lane & 15
    const int cb = lane & 15;
    const uint32_t coff = nw + 8 * cb < p.N ? (uint32_t)(nw + 8 * cb) * 2u : 0x80000000u;
    auto goff = [&](int row) { return coff == 0x80000000u ? coff : (uint32_t)row * (uint32_t)p.ldc * 2u + coff; };
    auto lrow = [&](int row, int ch) { return ws + row * P4_EPI_PITCH + ch * 16; };
    const __amdgpu_buffer_rsrc_t rsum = make_rsrc(p.colsum, p.colsum != nullptr ? (long long)p.N * 4 : 0);
#pragma unroll
    for (int hr = 0; hr < 2; ++hr) {
        if constexpr (EPI == EPI_RESADD || EPI == EPI_DGELU) {
            // operand tile rows -> LDS (row-contiguous), then each lane picks its MFMA-layout 8 bytes
#pragma unroll
            for (int h = 0; h < 2; ++h) {  // 8 rows of 16 B per lane in flight at a time
                uint4 ld[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(EPI == EPI_RESADD ? rc : rx,
                                                                          goff(64 * hr + 4 * (8 * h + q) + g), 0, 0);
                    ld[q] = make_uint4(v[0], v[1], v[2], v[3]);
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) *(uint4*)lrow(4 * (8 * h + q) + g, cb) = ld[q];
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float bv[4] = {0.f, 0.f, 0.f, 0.f}, csum[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (EPI != EPI_DGELU) {
                const int n = nw + 16 * j + 4 * g;
                const u32x2_t b = __builtin_amdgcn_raw_buffer_load_b64(rbias, n < p.N ? (uint32_t)n * 2u : 0x80000000u, 0, 0);
                unpack4(make_uint2(b.x, b.y), bv);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const f32x4 a = acc[8 * (4 * hr + i) + j];
                const int row = 16 * i + rl, ch = 2 * j + (g >> 1);
                char* a8 = lrow(row, ch) + ((g & 1) << 3);
                float v[4];
                if constexpr (EPI == EPI_RESADD) {
                    float o[4];
                    unpack4(*(const uint2*)a8, o);
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = a[r] + bv[r] + o[r];
                } else if constexpr (EPI == EPI_DGELU) {
                    float u[4];
                    unpack4(*(const uint2*)a8, u);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v[r] = a[r] * gelu_tanh_grad(u[r]);
                        csum[r] += v[r];
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = a[r] + bv[r];
                }
                *(uint2*)a8 = pack4(v);
                __builtin_amdgcn_sched_barrier(0);  // one tile at a time (no hoisted accumulator reads)
            }
            if constexpr (EPI == EPI_DGELU) {
                // this pass's 64-row column sums of column block j: over the 16 lanes of a group,
                // one atomic per column (rows past M read aux as zero and had zero accumulators)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float t = csum[r];
                    t += __shfl_xor(t, 1, 64);
                    t += __shfl_xor(t, 2, 64);
                    t += __shfl_xor(t, 4, 64);
                    t += __shfl_xor(t, 8, 64);
                    csum[r] = t;
                }
                const int n = nw + 16 * j + 4 * g, r = lane & 3;
                const float t = r == 0 ? csum[0] : r == 1 ? csum[1] : r == 2 ? csum[2] : csum[3];
                const bool writer = p.colsum != nullptr && (lane & 15) < 4 && n + r < p.N;
                __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(t, rsum, writer ? (uint32_t)(n + r) * 4u : 0x80000000u, 0, 0);
            }
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint4 v = *(const uint4*)lrow(4 * q + g, cb);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, EPI == EPI_GELU ? rx : rc,
                                                   goff(64 * hr + 4 * q + g), 0, 0);
            if (q % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // at most 4 rows in registers
        }
        if constexpr (EPI == EPI_GELU) {  // the stored pre-activation -> gelu -> C
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                uint4 v = *(const uint4*)lrow(4 * q + g, cb);
                float f[8];
                unpack8(v, f);
#pragma unroll
                for (int r = 0; r < 8; ++r) f[r] = gelu_tanh(f[r]);
                v = pack8(f);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{v.x, v.y, v.z, v.w}, rc, goff(64 * hr + 4 * q + g), 0, 0);
                if (q % 4 == 3) __builtin_amdgcn_sched_barrier(0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // pass hr's reads before pass hr+1 rewrites
        __builtin_amdgcn_sched_barrier(0);
    }
}

// ============================================================================ persistent 4-wave, register staged
// hipBLASLt's fastest gfx950 kernels for these products (MT256x256x64, MIWT8_8, WG 256, stream-K
// persistent grid, register-staged global reads two K steps ahead: their kernel names in
// profiles/r3_baseline_rocprof_summary.txt) use ONE wave per SIMD owning a 128 x 128 block.  That
// reads a third less LDS per MFMA than 8 waves of 128 x 64, and the 128 MFMAs of a K step leave
// 128 issue gaps for the step's 32 fragment reads + 16 global loads + 16 LDS writes.
// Versus gemm_persistent (same geometry, LDS-DMA staging: 60-185 issue cycles per 1-KiB copy with
// no partner wave to hide them) the operands come through VGPRs (global_load_dwordx4 -> ds_write_b128).
//
// Per K step s (LDS buffer cur = s & 1 holds step s, F0 = its k-half 0 fragments, R = the global
// data of step s + 1, loaded during step s - 1):
//   half 0: 64 MFMAs on F0 | read F1 (k-half 1 of cur) ; write R -> buffer cur ^ 1 ; load R <- step s + 2
//   half 1: [own LDS reads / writes retired] barrier | 64 MFMAs on F1 | read F0 (k-half 0 of cur ^ 1)
// One barrier per step covers both hazards: after it every wave's writes of step s + 1 are visible,
// and every wave has finished reading buffer cur ^ 1's previous contents (step s - 1) long before
// (its last reads were in half 0 of step s - 1, before the previous barrier).
// The K-step sequence runs on across the tiles of the persistent walk, so the next tile's first
// steps are loaded while the current tile finishes; only the epilogue stalls the matrix pipe.
template <bool TA, bool TB, int EPI, bool LEPI = false>
__global__ __launch_bounds__(PNTHR, 1) void gemm_p4(GemmParams p) {
    static_assert(!LEPI || EPI <= EPI_DGELU, "LDS epilogue: bf16 outputs");
    __shared__ __attribute__((aligned(16))) char smem[LEPI ? LDS_BYTES + 32768 : LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 1, wn = w & 1;
    const int G = gridDim.x;
    const int lb = xcd_remap(blockIdx.x, G);
    const int nk = p.k_per_split / BK;
    const int n_items = p.tiles * p.splits;
    const int n_mine = lb < n_items ? (n_items - 1 - lb) / G + 1 : 0;
    const int total = n_mine * nk;
    if (total == 0) return;
    auto coords = [&](int i, int& m0, int& n0, int& sp) {
        const int item = lb + i * G;
        sp = item / p.tiles;
        const int tile = item - sp * p.tiles;
        int tm, tn;
        tile_coords(p, tile, tm, tn);
        m0 = tm * BM;
        n0 = tn * BN;
    };

    // ---- producer: the (item, k step) it loads next; after the last step it repeats that step
    // (its data then goes to a buffer nobody reads)
    int pi = 0, pt = 0, pm0, pn0, psp, pleft = total;
    coords(0, pm0, pn0, psp);
    Stager<TA, 4> sa;
    Stager<TB, 4> sb;
    sa.init(p.lda, pm0, p.M, w, lane);
    sb.init(p.ldb, pn0, p.N, w, lane);
    u32x4_t R[16];  // one K step of this wave's share: pieces 0-7 of A, 8-15 of B
    __amdgpu_buffer_rsrc_t qa, qb;
    auto produce_rsrc = [&]() {
        const int k0 = psp * p.k_per_split + pt * BK;
        qa = sa.rsrc(p.A, p.lda, pm0, p.M, k0);
        qb = sb.rsrc(p.B, p.ldb, pn0, p.N, k0);
    };
    auto produce_advance = [&]() {
        if (--pleft > 0) {
            if (++pt == nk) {
                pt = 0;
                ++pi;
                coords(pi, pm0, pn0, psp);
                sa.init(p.lda, pm0, p.M, w, lane);
                sb.init(p.ldb, pn0, p.N, w, lane);
            }
        } else {
            pleft = 0;
        }
    };
    auto load_piece = [&](auto ic) {
        constexpr int i = decltype(ic)::value;
        // per-lane base in the VGPR offset, the piece's uniform offset in the SGPR offset: no VALU
        if constexpr (i < 8) {
            R[i] = __builtin_amdgcn_raw_buffer_load_b128(qa, sa.base[TA ? (i & 1) : 0], (uint32_t)i * sa.delta, 0);
        } else {
            R[i] = __builtin_amdgcn_raw_buffer_load_b128(qb, sb.base[TB ? (i & 1) : 0], (uint32_t)(i - 8) * sb.delta, 0);
        }
    };
    auto write_piece = [&](char* buf, auto ic) {
        constexpr int i = decltype(ic)::value;
        char* t = buf + (i < 8 ? 0 : TILE_BYTES);
        *(u32x4_t*)(t + (w + 4 * (i & 7)) * 1024 + lane * 16) = R[i];
    };
    // fragment reads: a per-lane base (lane part + buffer + wave block, one VGPR per operand and
    // k-half, recomputed per half step) plus the tile's constant offset as the ds_read immediate
    auto frag_base = [&](bool isB, int buf, int ks) -> uint32_t {
        uint32_t v;
        if constexpr (true) {
            const bool tr = isB ? TB : TA;
            const int wb = isB ? wn : wm;
            if (!tr) {
                v = (uint32_t)((lane & 15) * 128 + (((4 * ks + (lane >> 4)) ^ (lane & 7)) << 4) + wb * 128 * 128);
            } else {
                v = 0;  // transposed images: frag<> computes the full address
            }
            v += (uint32_t)(buf * STAGE_BYTES + (isB ? TILE_BYTES : 0));
        }
        asm volatile("" : "+v"(v));
        return v;
    };
    auto frag_at = [&](uint32_t base, bool isB, int t, int buf, int ks) -> bf16x8_t {
        const bool tr = isB ? TB : TA;
        if (!tr) return *(const bf16x8_t*)(smem + base + t * 16 * 128);
        return isB ? frag<TB>(smem + buf * STAGE_BYTES + TILE_BYTES, wn * 128 + 16 * t, ks, lane)
                   : frag<TA>(smem + buf * STAGE_BYTES, wm * 128 + 16 * t, ks, lane);
    };

    PFrags F;
    Acc acc;
    stamp(p, 0);
    {   // prologue: step 0 -> LDS buffer 0, step 1 -> R, F = step 0's k-half 0
        produce_rsrc();
        static_for<16>(load_piece);
        produce_advance();
        static_for<16>([&](auto ic) { write_piece(smem, ic); });
        produce_rsrc();
        static_for<16>(load_piece);
        produce_advance();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t bb = frag_base(true, 0, 0), ba = frag_base(false, 0, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) F.b[0][j] = frag_at(bb, true, j, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) F.a[i] = frag_at(ba, false, i, 0, 0);
    }

    int s = 0;
    // one K step; ZERO: the tile's first (accumulators start from C = 0); LAST: the tile's last (the
    // next step's k-half 0 fragments are read after the epilogue, so they are not live across it)
    auto read_half0 = [&](int buf) {
        const uint32_t bb = frag_base(true, buf, 0), ba = frag_base(false, buf, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) F.b[0][j] = frag_at(bb, true, j, buf, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) F.a[i] = frag_at(ba, false, i, buf, 0);
    };
    auto kstep = [&](auto zc, auto lc) {
        constexpr bool ZERO = decltype(zc)::value, LAST = decltype(lc)::value;
        const int cur = s & 1, nxt = cur ^ 1;
        char* wbuf = smem + nxt * STAGE_BYTES;
        produce_rsrc();
        // ---- half 0 (MFMAs on b[0], a = k-half 0 of step s):
        //   b[1][j] <- k-half 1 of cur after MFMAs 1, 3, .., 15;  a[i] <- k-half 1 after row i (MFMA 8i + 7);
        //   R piece i -> LDS buffer nxt after MFMA 17 + 3i, then the next load into R[i] after 18 + 3i
        {
            const uint32_t bb = frag_base(true, cur, 1), ba = frag_base(false, cur, 1);
            auto hook = [&](auto tc) {
                constexpr int T = decltype(tc)::value;
                if constexpr (T < 16 && T % 2 == 1) F.b[1][T / 2] = frag_at(bb, true, T / 2, cur, 1);
                if constexpr (T % 8 == 7) F.a[T / 8] = frag_at(ba, false, T / 8, cur, 1);
                if constexpr (T >= 17 && (T - 17) % 3 == 0) write_piece(wbuf, std::integral_constant<int, (T - 17) / 3>{});
                if constexpr (T >= 18 && (T - 18) % 3 == 0) load_piece(std::integral_constant<int, (T - 18) / 3>{});
            };
            mfma_run<0, 0, ZERO>(acc, F, hook);
        }
        produce_advance();
        // ---- half 1: every wave's writes of step s + 1 and reads of step s landed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        {
            const uint32_t bb = frag_base(true, nxt, 0), ba = frag_base(false, nxt, 0);
            auto hook = [&](auto tc) {
                constexpr int T = decltype(tc)::value;
                if constexpr (!LAST && T < 16 && T % 2 == 1) F.b[0][T / 2] = frag_at(bb, true, T / 2, nxt, 0);
                if constexpr (!LAST && T % 8 == 7) F.a[T / 8] = frag_at(ba, false, T / 8, nxt, 0);
            };
            mfma_run<1, 0, false>(acc, F, hook);
        }
        ++s;
    };
    for (int ci = 0; ci < n_mine; ++ci) {
        int cm0, cn0, csp;
        coords(ci, cm0, cn0, csp);
        kstep(std::true_type{}, std::false_type{});
#pragma clang loop unroll(disable)
        for (int ct = 1; ct < nk - 1; ++ct) kstep(std::false_type{}, std::false_type{});
        kstep(std::false_type{}, std::true_type{});  // nk >= 2 (host)
        stamp(p, 1 + 2 * ci);
        // ---- epilogue: the last MFMAs' results must be written before the accumulator reads.
        // Inline-asm MFMAs are opaque to the hazard recognizer, and hipcc copied finished
        // accumulators to VGPRs right behind their last MFMA (stale values): after the nop sled,
        // empty asm statements "redefine" every accumulator, so no read can move above them.
        asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
        acc_fence<0>(acc);
        acc_fence<16>(acc);
        acc_fence<32>(acc);
        acc_fence<48>(acc);
        __builtin_amdgcn_sched_barrier(0);
        auto get = [&](auto ic, auto jc) { return acc[8 * decltype(ic)::value + decltype(jc)::value]; };
        if constexpr (LEPI) {
            // the stage the last step read is idle until the next step's writes: waves 0-2 stage
            // through 17 KiB each of it, wave 3 through the spare 32 KiB past the two stages; a
            // barrier keeps the next step's writes behind every wave's epilogue reads
            char* ws = w < 3 ? smem + (s & 1 ? 0 : STAGE_BYTES) + w * P4_EPI_WAVE : smem + LDS_BYTES;
            p4_lds_epilogue<EPI>(p, acc, ws, cm0 + wm * 128, cn0 + wn * 128, lane);
            __builtin_amdgcn_s_barrier();
        } else {
            epilogue_store<EPI, 8>(p, get, cm0 + wm * 128, cn0 + wn * 128, csp, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
        stamp(p, 2 + 2 * ci);
        read_half0(s & 1);  // the next tile's first k-half (step s, staged in buffer s & 1)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ============================================================================ persistent 4-wave, LDS-DMA
// gemm_p4's geometry (one wave per SIMD owning 128 x 128, AGPR accumulators, persistent grid) with
// the operands copied by LDS-DMA (buffer_load ... lds, no VGPR staging) into two 64-KiB stages, on
// the schedule of the library kernel our step profiles name for these products (its disassembly: a
// K step = 128 MFMAs, 16 one-KiB copies spread one per ~5 MFMAs, three barriers, ONE vmcnt wait):
//   half 0 (64 MFMAs on F0 = k-half 0 of step s, read at the end of step s - 1):
//     T 0..15 : read F1 = k-half 1 of step s from stage cur, one fragment per MFMA
//     T 18    : own LDS reads retired + barrier: no wave reads stage cur any more
//     T 20..62: copies 0-6 of step s + 2 into stage cur, one every 7 MFMAs (spread: a copy's issue
//               costs ~60 cycles, MI355X_MICROARCH.md; denser placements measured slower)
//   half 1 (64 MFMAs on F1):
//     T 5..33 : copies 7-11
//     T 36    : vmcnt(12) — every copy of step s + 1 (issued during step s - 1) landed, the 12
//               issued since stay in flight — + barrier: all waves' copies of step s + 1 visible
//     T 37..52: read F0 = k-half 0 of step s + 1 from stage nxt; copies 12-15 at T 40..61
// (variants of these slots: TDL_PD_SCHED, profiles/r5_gemm_pd_sched_ab.jsonl)
// So a copy has about a K step to land and the wave waits for copies once per step (gemm_p4 waits
// for each staged register ahead of its LDS write, inside the MFMA stream: 46 % of its wave cycles).
// NT operands only (TA = TB = false: the forward / input-gradient products).
// ORD 0: MFMA T = (A tile T / 8, B tile T % 8) — the MFMA's second source (an A fragment) held for
// 8 MFMAs; ORD 1: (A tile T % 8, B tile T / 8) — its first source (a B fragment) held, as in the
// library kernel.  Either way accumulator 8 i + j is tile (i, j).
template <int T, bool ZERO, int ORD, class Hook>
__device__ __forceinline__ void mfma_run_pd(Acc& acc, const bf16x8_t (&a)[8], const bf16x8_t (&b)[8], Hook& hook) {
    if constexpr (T < 64) {
        constexpr int i = ORD == 0 ? T / 8 : T % 8, j = ORD == 0 ? T % 8 : T / 8;
        if constexpr (ZERO) amfma0<8 * i + j>(acc, b[j], a[i]);
        else amfma<8 * i + j>(acc, b[j], a[i]);
        hook(std::integral_constant<int, T>{});
        __builtin_amdgcn_sched_barrier(0);
        mfma_run_pd<T + 1, ZERO, ORD>(acc, a, b, hook);
    }
}

// bf16 (+ bias) epilogue with 16-byte stores (cdna_hip_programming.md T21): the accumulator gives
// a lane 4 consecutive columns of a 16 x 16 tile; v_permlane16_swap trades tile j's columns 4-7
// (held by the odd 16-lane rows) for tile j + 1's columns 0-3 (held by the even rows), so every lane
// stores 8 consecutive columns of one tile: 32 dwordx4 stores per wave instead of 64 dwordx2 (half
// the store issue, and few enough VMEM ops that the next tile's first copy wait can count past
// them instead of waiting for the stores, PD_X4_VMEM).  The bias values come in `braw`, loaded by
// pd_bias_load at the start of the tile's last K step: a load inside the epilogue would make the
// in-order vmcnt wait for every copy and store issued before it (the per-tile-row epilogue waits
// that way once per column block).  Needs N % 8 == 0, ldc % 8 == 0.
// VMEM instructions of pd_store_x4 per wave: 32 stores (bf16), 64 (GELU: pre-activation + output)
constexpr int pd_x4_vmem(int epi) { return epi == EPI_GELU ? 64 : epi == EPI_DGELU ? 68 : 32; }
__device__ __forceinline__ void pd_bias_load(const GemmParams& p, int nw, int lane, u32x2_t (&braw)[8]) {
    const __amdgpu_buffer_rsrc_t rbias = make_rsrc(p.bias, p.bias != nullptr ? (long long)p.N * 2 : 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int n = nw + 16 * j + 4 * (lane >> 4);
        braw[j] = __builtin_amdgcn_raw_buffer_load_b64(rbias, n < p.N ? (uint32_t)n * 2u : 0x80000000u, 0, 0);
    }
}
// BIAS = false (no bias): no adds of zeros.  At K = 1024 this epilogue is 27-37 % of the kernel
// (the K loop alone runs 1.50-1.55 PF/s, profiles/r6_pd_epilogue_ab.jsonl); neither deferring half
// of its stores into the next tile's first K step, nor staggering the workgroups' start, nor a
// third fewer VALU moved it: the stores delay the next tile's copies queued behind them.
template <int EPI, bool BIAS = true, class Get>
__device__ __forceinline__ void pd_store_x4(const GemmParams& p, Get& get, int mw, int nw, int lane,
                                            const u32x2_t (&braw)[8]) {
    static_assert(EPI == EPI_BF16 || EPI == EPI_GELU, "16-byte store epilogue: bf16 (+ bias), bias + GELU");
    const int g = lane >> 4;
    const __amdgpu_buffer_rsrc_t rc = make_rsrc((const char*)p.C + (size_t)mw * p.ldc * 2, (long long)(p.M - mw) * p.ldc * 2);
    const __amdgpu_buffer_rsrc_t rx =
        EPI == EPI_GELU ? make_rsrc((const char*)p.aux + (size_t)mw * p.ldc * 2, (long long)(p.M - mw) * p.ldc * 2) : rc;
    const uint32_t lrow = (uint32_t)(lane & 15) * (uint32_t)p.ldc * 2u;
    auto pair = [&](auto jc) {
        constexpr int j = 2 * decltype(jc)::value;
        float ba[4], bb[4];   // bias of this lane's columns in tiles j, j + 1
        unpack4(make_uint2(braw[j].x, braw[j].y), ba);
        unpack4(make_uint2(braw[j + 1].x, braw[j + 1].y), bb);
        const int nt = nw + 16 * (j + (g & 1)) + 8 * (g >> 1);   // the 8 columns this lane stores
        const uint32_t col = nt < p.N ? (uint32_t)nt * 2u : 0x80000000u;
        auto row = [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const f32x4 a = get(std::integral_constant<int, i>{}, std::integral_constant<int, j>{});
            const f32x4 b = get(std::integral_constant<int, i>{}, std::integral_constant<int, j + 1>{});
            float va[4] = {a[0], a[1], a[2], a[3]};
            float vb[4] = {b[0], b[1], b[2], b[3]};
            if constexpr (BIAS) {   // (BIAS = false: no bias, no adds of zeros)
#pragma unroll
                for (int r = 0; r < 4; ++r) va[r] += ba[r], vb[r] += bb[r];
            }
            const uint32_t off = col == 0x80000000u ? col : lrow + (uint32_t)(16 * i) * (uint32_t)p.ldc * 2u + col;
            auto store8 = [&](const float (&xa)[4], const float (&xb)[4], const __amdgpu_buffer_rsrc_t& r) {
                const uint2 qa = pack4(xa), qb = pack4(xb);
                const auto s0 = __builtin_amdgcn_permlane16_swap(qa.x, qb.x, false, false);
                const auto s1 = __builtin_amdgcn_permlane16_swap(qa.y, qb.y, false, false);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{s0[0], s1[0], s0[1], s1[1]}, r, off, 0, 0);
            };
            if constexpr (EPI == EPI_GELU) {
                store8(va, vb, rx);   // the pre-activation
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    va[r] = gelu_tanh(va[r]);
                    vb[r] = gelu_tanh(vb[r]);
                }
            }
            store8(va, vb, rc);
            __builtin_amdgcn_sched_barrier(0);
        };
        static_for<8>(row);
    };
    static_for<4>(pair);
}

// dGELU epilogue with 16-byte accesses: d = acc * gelu'(pre), pre read from aux, bias-gradient
// column sums of d into colsum (fp32 atomics).  The accumulators are swapped in fp32 (4 swaps per
// tile pair and row block) so each lane holds 8 consecutive columns; all 32 pre-activation loads of
// the wave are issued before the first store (one in-order wait for them, none behind the stores).
// VMEM per wave: 32 loads + 32 stores + 4 atomics.
template <class Get>
__device__ __forceinline__ void pd_store_x4_dgelu(const GemmParams& p, Get& get, int mw, int nw, int lane) {
    const int g = lane >> 4;
    const __amdgpu_buffer_rsrc_t rc = make_rsrc((const char*)p.C + (size_t)mw * p.ldc * 2, (long long)(p.M - mw) * p.ldc * 2);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc((const char*)p.aux + (size_t)mw * p.ldc * 2, (long long)(p.M - mw) * p.ldc * 2);
    const uint32_t lrow = (uint32_t)(lane & 15) * (uint32_t)p.ldc * 2u;
    auto coloff = [&](int j) -> uint32_t {   // this lane's 8 columns of tile pair (j, j + 1)
        const int nt = nw + 16 * (j + (g & 1)) + 8 * (g >> 1);
        return nt < p.N ? (uint32_t)nt * 2u : 0x80000000u;
    };
    auto offset = [&](uint32_t col, int i) -> uint32_t {
        return col == 0x80000000u ? col : lrow + (uint32_t)(16 * i) * (uint32_t)p.ldc * 2u + col;
    };
    u32x4_t pre[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) pre[q] = __builtin_amdgcn_raw_buffer_load_b128(rx, offset(coloff(2 * (q >> 3)), q & 7), 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    auto pair = [&](auto jc) {
        constexpr int j = 2 * decltype(jc)::value;
        const uint32_t col = coloff(j);
        float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        auto row = [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            const f32x4 a = get(std::integral_constant<int, i>{}, std::integral_constant<int, j>{});
            const f32x4 b = get(std::integral_constant<int, i>{}, std::integral_constant<int, j + 1>{});
            float v[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[k]), __float_as_uint(b[k]), false, false);
                v[k] = __uint_as_float(sw[0]);       // columns 0-3 of the lane's 8
                v[4 + k] = __uint_as_float(sw[1]);   // columns 4-7
            }
            const u32x4_t u = pre[4 * j + i];   // (j / 2) * 8 + i
            float pu[8];
            unpack4(make_uint2(u.x, u.y), pu);
            unpack4(make_uint2(u.z, u.w), pu + 4);
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                v[c] *= gelu_tanh_grad(pu[c]);
                cs[c] += v[c];
            }
            const uint2 lo = pack4(v), hi = pack4(v + 4);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{lo.x, lo.y, hi.x, hi.y}, rc, offset(col, i), 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        };
        static_for<8>(row);
        if (p.colsum != nullptr) {
            // the 16 lanes of a row group hold the same 8 columns for 16 rows: sum over them
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                float t = cs[c];
                t += __shfl_xor(t, 1, 64);
                t += __shfl_xor(t, 2, 64);
                t += __shfl_xor(t, 4, 64);
                t += __shfl_xor(t, 8, 64);
                cs[c] = t;
            }
            const int c = lane & 7;
            float t = cs[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) t = c == k ? cs[k] : t;
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(p.colsum, (long long)p.N * 4);
            const bool writer = (lane & 15) < 8 && col != 0x80000000u;
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(t, rs, writer ? col * 2u + (uint32_t)c * 4u : 0x80000000u, 0, 0);
        }
    };
    static_for<4>(pair);
}

// s_waitcnt vmcnt(n) with expcnt / lgkmcnt at their no-wait maxima (gfx9 encoding)
constexpr int vmcnt_enc(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }
// copies of a step issued before global MFMA slot wg (slots ds + dp i, i < 16)
constexpr int copies_before(int ds, int dp, int wg) {
    int n = 0;
    for (int i = 0; i < 16; ++i) n += (ds + dp * i < wg) ? 1 : 0;
    return n;
}

// Schedule (global MFMA slot g = 64 half + T of a K step): RP = MFMAs per F1 fragment read at the
// head of half 0, then lgkmcnt(0) + barrier; copy i at slot DS + DP i; the vmcnt wait + barrier at
// slot WG; F0 reads after it.
template <int EPI, int RP = 1, int DS = 20, int DP = 7, int WG = 100, bool X4 = false, int ORD = 0, int B1 = 16 * RP + 2,
          bool TA = false, bool TB = false, bool NOEPI = false, bool NOBIAS = false, bool GROUPED = false>
__global__ __launch_bounds__(PNTHR, 1) void gemm_pd(GemmParams p) {
    static_assert(B1 >= 16 * RP + 2 && DS > B1 && DS + 15 * DP <= 127 && WG + 16 <= 127, "schedule must fit one K step");
    constexpr int NB = copies_before(DS, DP, WG);          // this step's copies in flight at the wait
    constexpr int RP2 = 127 - WG >= 32 ? 2 : 1;          // MFMAs per F0 fragment read
    static_assert(!X4 || EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_DGELU, "16-byte epilogues: bf16, GELU, dGELU");
    // the first wait after an epilogue: the copies it waits for precede the epilogue's VMEM ops
    // (>= 64 per wave for the per-tile-row epilogue, exactly PD_X4_VMEM for pd_store_x4) and the NB
    // copies issued since; vmcnt counts in issue order, so vmcnt(that sum) retires exactly the copies
    constexpr int EV = NOEPI ? 0 : X4 ? pd_x4_vmem(EPI) : 64;
    constexpr int NB_EPI = EV + NB < 63 ? EV + NB : 63;
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 1, wn = w & 1;
    const int G = gridDim.x;
    const int lb = xcd_remap(blockIdx.x, G);
    const int nk = p.k_per_split / BK;
    // GROUPED: one item per workgroup (host: items <= CUs), so a workgroup's product is fixed: the
    // ones past the first product's items switch every operand / output field to the second product
    // once, here, and the rest of the kernel is the plain one
    int ioff = 0;
    const int n_items = GROUPED ? p.items1 + p.g2.tiles * p.splits : p.tiles * p.splits;
    if constexpr (GROUPED) {
        if (lb >= p.items1) {
            p.A = p.g2.A;
            p.B = p.g2.B;
            p.C = p.g2.C;
            p.M = p.g2.M;
            p.N = p.g2.N;
            p.lda = p.g2.lda;
            p.ldb = p.g2.ldb;
            p.ldc = p.g2.ldc;
            p.tiles_n = p.g2.tiles_n;
            p.tiles = p.g2.tiles;
            p.split_stride = p.g2.split_stride;
            ioff = p.items1;
        }
    }
    const int n_mine = lb < n_items ? (GROUPED ? 1 : (n_items - 1 - lb) / G + 1) : 0;
    const int total = n_mine * nk;
    if (total == 0) return;
    auto coords = [&](int i, int& m0, int& n0, int& sp) {
        const int item = lb + i * G - ioff;
        sp = item / p.tiles;
        const int tile = item - sp * p.tiles;
        int tm, tn;
        tile_coords(p, tile, tm, tn);
        m0 = tm * BM;
        n0 = tn * BN;
    };
    // ---- producer: the (item, k step) it copies next, two steps ahead of the MFMAs; after the last
    // step it repeats that step (into a stage nobody reads any more)
    int pi = 0, pt = 0, pm0, pn0, psp, pleft = total;
    coords(0, pm0, pn0, psp);
    // k-contiguous images: lane offsets independent of the tile; row-contiguous (TA / TB: the weight
    // gradients) ones clamp ragged columns per tile, so the producer re-inits them with each tile
    Stager<TA, 4> sa;
    Stager<TB, 4> sb;
    sa.init(p.lda, pm0, p.M, w, lane);
    sb.init(p.ldb, pn0, p.N, w, lane);
    __amdgpu_buffer_rsrc_t qa, qb;
    auto produce_rsrc = [&]() {
        const int k0 = psp * p.k_per_split + pt * BK;
        qa = sa.rsrc(p.A, p.lda, pm0, p.M, k0);
        qb = sb.rsrc(p.B, p.ldb, pn0, p.N, k0);
    };
    auto produce_advance = [&]() {
        if constexpr (GROUPED) {   // one item: the producer never moves to another tile
            if (--pleft > 0) ++pt;
            else pleft = 0;
            return;
        }
        if (--pleft > 0) {
            if (++pt == nk) {
                pt = 0;
                ++pi;
                coords(pi, pm0, pn0, psp);
                if constexpr (TA) sa.init(p.lda, pm0, p.M, w, lane);
                if constexpr (TB) sb.init(p.ldb, pn0, p.N, w, lane);
            }
        } else {
            pleft = 0;
        }
    };
    // copy i (< 8: A piece i, else B piece i - 8): the lane's base offset in the VGPR operand, the
    // piece's uniform offset in the SGPR one (no per-copy address arithmetic in the K loop)
    auto copy_piece = [&](char* stage, auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int j = i & 7;
        constexpr bool TR = i < 8 ? TA : TB;
        const uint32_t vo = i < 8 ? sa.base[TR ? (j & 1) : 0] : sb.base[TR ? (j & 1) : 0];
        const uint32_t dl = i < 8 ? sa.delta : sb.delta;
        char* dst = stage + (i < 8 ? 0 : TILE_BYTES) + (w + 4 * j) * 1024;
        if constexpr (TR) {
            // Row-contiguous images are read with ds_read_b64_tr_b16, whose builtin hipcc cannot tell
            // apart from the DMA's destination: it drained every copy in flight (s_waitcnt vmcnt(0))
            // in front of the transposed reads, 10 times per K step — 62 % of the wave cycles parked,
            // 0.62x gemm_p4 (profiles/r6_pmc_wgrad_pd.txt).  Issued from asm, the copy is invisible
            // to that alias check; its completion is still counted by the explicit vmcnt waits.
            const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lds_void_t*)dst);
            const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)j * dl);
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                         :: "s"(la), "v"(vo), "s"(i < 8 ? qa : qb), "s"(so) : "memory", "m0");
        } else {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(i < 8 ? qa : qb, (lds_void_t*)dst, 16, vo,
                                                     __builtin_amdgcn_readfirstlane((uint32_t)j * dl), 0, 0);
        }
    };
    auto frag_base = [&](bool isB, int buf, int ks) -> uint32_t {
        const int wb = isB ? wn : wm;
        uint32_t v = (uint32_t)((lane & 15) * 128 + (((4 * ks + (lane >> 4)) ^ (lane & 7)) << 4) + wb * 128 * 128);
        v += (uint32_t)(buf * STAGE_BYTES + (isB ? TILE_BYTES : 0));
        asm volatile("" : "+v"(v));
        return v;
    };
    auto frag_at = [&](uint32_t base, int t) -> bf16x8_t { return *(const bf16x8_t*)(smem + base + t * 16 * 128); };
    // fragment t of operand B (isB) / A, k-half ks, stage buf: the k-contiguous image through a
    // per-lane base + immediate offsets, the row-contiguous one through the transposing read
    auto frag_x = [&](bool isB, uint32_t base, int buf, int t, int ks) -> bf16x8_t {
        if (isB ? TB : TA)
            return isB ? frag<TB>(smem + buf * STAGE_BYTES + TILE_BYTES, wn * 128 + 16 * t, ks, lane)
                       : frag<TA>(smem + buf * STAGE_BYTES, wm * 128 + 16 * t, ks, lane);
        return frag_at(base, t);
    };

    bf16x8_t a0[8], b0[8], a1[8], b1[8];
    Acc acc;
    auto read_f0 = [&](int buf) {
        const uint32_t bb = frag_base(true, buf, 0), ba = frag_base(false, buf, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) b0[j] = frag_x(true, bb, buf, j, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) a0[i] = frag_x(false, ba, buf, i, 0);
    };
    {   // prologue: steps 0 and 1 -> stages 0 and 1; F0 = step 0's k-half 0
        produce_rsrc();
        static_for<16>([&](auto ic) { copy_piece(smem, ic); });
        produce_advance();
        produce_rsrc();
        static_for<16>([&](auto ic) { copy_piece(smem + STAGE_BYTES, ic); });
        produce_advance();
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        read_f0(0);
    }
    int s = 0;
    u32x2_t braw[8];   // X4: the bias of the wave's columns (pd_bias_load)
    int bias_n0 = 0;
    // after_epi: the first step after a tile's epilogue, whose VMEM ops were issued between the
    // copies this step waits for and the NB issued since: vmcnt(NB_EPI) retires those copies without
    // waiting for all of the epilogue's stores (vmcnt(NB) stalled on them every tile)
    auto kstep = [&](auto zc, auto lc, bool after_epi) {
        constexpr bool ZERO = decltype(zc)::value, LAST = decltype(lc)::value;
        const int cur = s & 1, nxt = cur ^ 1;
        char* cstage = smem + cur * STAGE_BYTES;
        if constexpr (X4 && LAST && EPI != EPI_DGELU && !NOBIAS) pd_bias_load(p, bias_n0, lane, braw);   // ahead of this step's copies
        produce_rsrc();
        auto slot = [&](auto gc, const uint32_t* fb) {
            constexpr int g = decltype(gc)::value;
            if constexpr (g < 16 * RP && g % RP == RP - 1) {   // F1 = k-half 1 of step s (stage cur)
                constexpr int k = g / RP;
                if constexpr ((k < 8) == (ORD == 0)) b1[k & 7] = frag_x(true, fb[0], cur, k & 7, 1);
                else a1[k & 7] = frag_x(false, fb[1], cur, k & 7, 1);
            }
            if constexpr (g == B1) {   // own reads of stage cur retired; then all waves'
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            if constexpr (g >= DS && (g - DS) % DP == 0 && (g - DS) / DP < 16)
                copy_piece(cstage, std::integral_constant<int, (g - DS) / DP>{});
            if constexpr (g == WG) {   // copies of step s + 1 landed (this step's NB stay in flight)
                if (ZERO && after_epi) __builtin_amdgcn_s_waitcnt(vmcnt_enc(NB_EPI));
                else __builtin_amdgcn_s_waitcnt(vmcnt_enc(NB));
                __builtin_amdgcn_s_barrier();
            }
            if constexpr (!LAST && g > WG && (g - WG - 1) % RP2 == 0 && (g - WG - 1) / RP2 < 16) {
                constexpr int k = (g - WG - 1) / RP2;   // F0 = k-half 0 of step s + 1 (stage nxt)
                if constexpr ((k < 8) == (ORD == 0)) b0[k & 7] = frag_x(true, fb[2], nxt, k & 7, 0);
                else a0[k & 7] = frag_x(false, fb[3], nxt, k & 7, 0);
            }
        };
        const uint32_t fb[4] = {frag_base(true, cur, 1), frag_base(false, cur, 1), frag_base(true, nxt, 0),
                                frag_base(false, nxt, 0)};
        {
            auto hook = [&](auto tc) { slot(tc, fb); };
            mfma_run_pd<0, ZERO, ORD>(acc, a0, b0, hook);
        }
        {
            auto hook = [&](auto tc) { slot(std::integral_constant<int, 64 + decltype(tc)::value>{}, fb); };
            mfma_run_pd<0, false, ORD>(acc, a1, b1, hook);
        }
        produce_advance();
        ++s;
    };
    for (int ci = 0; ci < (GROUPED ? 1 : n_mine); ++ci) {
        int cm0, cn0, csp;
        coords(ci, cm0, cn0, csp);
        bias_n0 = cn0 + wn * 128;
        kstep(std::true_type{}, std::false_type{}, ci > 0);
#pragma clang loop unroll(disable)
        for (int ct = 1; ct < nk - 1; ++ct) kstep(std::false_type{}, std::false_type{}, false);
        kstep(std::false_type{}, std::true_type{}, false);  // nk >= 2 (host)
        // epilogue (as gemm_p4): results of the opaque asm MFMAs written before any accumulator read
        asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
        acc_fence<0>(acc);
        acc_fence<16>(acc);
        acc_fence<32>(acc);
        acc_fence<48>(acc);
        __builtin_amdgcn_sched_barrier(0);
        auto get = [&](auto ic, auto jc) { return acc[8 * decltype(ic)::value + decltype(jc)::value]; };
        if constexpr (NOEPI) {   // diagnostics only (TDL_PD_SCHED=10): the K loop without the epilogue
        } else if constexpr (X4 && EPI == EPI_DGELU) pd_store_x4_dgelu(p, get, cm0 + wm * 128, cn0 + wn * 128, lane);
        else if constexpr (X4) pd_store_x4<EPI, !NOBIAS>(p, get, cm0 + wm * 128, cn0 + wn * 128, lane, braw);
        else epilogue_store<EPI, 8>(p, get, cm0 + wm * 128, cn0 + wn * 128, csp, lane);
        __builtin_amdgcn_sched_barrier(0);
        read_f0(s & 1);  // the next tile's first k-half (its copies were waited for in the last step)
    }
    // no copy may still be landing when the workgroup's LDS is handed to the next one
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

// C = epilogue(A x B^T) (see the header for the storage flags and epilogue codes).
// Requirements: K % 64 == 0, N % 4 == 0; TA needs M % 8 == 0, TB N % 8 == 0; 16-byte aligned rows
// (lda/ldb % 8 == 0), ldc % 4 == 0.  split > 1 only with EPI 4 (slab i at C + i * split_stride) or
// 6 (atomics); the split is reduced until it divides K / 64 (every slice the same depth).
// `kernel` (epi bits 8..15): 0 = the persistent 4-wave kernel (gemm_p4), 1 = the staggered
// ping-pong kernel (gemm_pp; LDS-staged row-contiguous epilogue on NT operands with bf16 outputs).
static unsigned long long* g_gemm_ts = nullptr;   // diagnostics: stamps of every GEMM launch
TDL_API int tdl_gemm_set_timestamps(void* buf) {
    g_gemm_ts = (unsigned long long*)buf;
    return 0;
}

static int num_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

TDL_API int tdl_gemm(const void* A, const void* B, void* C, const void* bias, void* aux, float* colsum, int M, int N,
                     int K, int lda, int ldb, int ldc, int ta, int tb, int epi, int split, long long split_stride,
                     hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0 || K % BK || N % 4 || lda % 8 || ldb % 8 || ldc % 4) return (int)hipErrorInvalidValue;
    if ((ta && M % 8) || (tb && N % 8)) return (int)hipErrorInvalidValue;
    int kernel = (epi >> 8) & 0xff;
    epi &= 0xff;
    if (epi < 0 || epi > 6 || kernel > 3) return (int)hipErrorInvalidValue;
    const bool lds_epi = kernel == 2;  // p4 with the LDS-staged epilogue (NT, bf16 outputs)
    if (kernel == 2) kernel = 0;
    // the dGELU column sums assume rows past M read as zero, which a transposed A cannot give
    if (epi == EPI_DGELU && ta) return (int)hipErrorInvalidValue;
    if (split < 1) split = 1;
    if (split > (K / BK) / 2) split = (K / BK) / 2 > 1 ? (K / BK) / 2 : 1;
    while (split > 1 && (K / BK) % split) --split;
    if (split > 1 && epi != EPI_F32 && epi != EPI_F32ATOM) return (int)hipErrorInvalidValue;
    const int kps = K / split;
    GemmParams p{(const bf16_t*)A, (const bf16_t*)B, C, (const bf16_t*)bias, (bf16_t*)aux, colsum, M, N, K,
                 lda, ldb, ldc, kps, split_stride, (N + BN - 1) / BN, 0, split, 0, g_gemm_ts};
    {
        // tile order: groups of 8 tile rows, so the 32 CUs of an XCD share a block of at most 8 A
        // panels x 4 B panels (fc forward +7-8 %, profiles/r5_gemm_order_ring_ab.jsonl; the
        // weight gradients: qkv / out / fc +2-4 %, profiles/r6_wgrad_ab.jsonl — with 4 tile rows
        // the row-major walk spans every B panel).  TDL_GEMM_GROUPM overrides (read per launch:
        // in-process A/B)
        const char* g = std::getenv("TDL_GEMM_GROUPM");
        p.group_m = g ? std::atoi(g) : 8;
    }
    p.tiles = ((M + BM - 1) / BM) * p.tiles_n;
#ifdef TDL_GEMM_ISA_ONLY  // inspection builds: one instantiation (scripts/isa_p4.sh)
#ifndef P4_TA
#define P4_TA false
#define P4_TB false
#define P4_EPI 0
#endif
#ifndef P4_LEPI
#define P4_LEPI false
#endif
#ifdef PD_ISA   // the 16-byte-store gemm_pd epilogues instead (register / spill inspection)
    gemm_pd<EPI_BF16, 1, 20, 7, 100, true><<<256, PNTHR, 0, s>>>(p);
    gemm_pd<EPI_BF16, 1, 20, 7, 100, true, 0, 18, false, false, false, true><<<256, PNTHR, 0, s>>>(p);
    gemm_pd<EPI_GELU, 1, 20, 7, 100, true><<<256, PNTHR, 0, s>>>(p);
    gemm_pd<EPI_DGELU, 1, 20, 7, 100, true><<<256, PNTHR, 0, s>>>(p);
    gemm_pd<EPI_F32, 1, 20, 7, 100, false, 0, 18, true, true><<<256, PNTHR, 0, s>>>(p);
#else
    gemm_p4<P4_TA, P4_TB, P4_EPI, P4_LEPI><<<256, PNTHR, 0, s>>>(p);
#endif
    TDL_LAUNCH_CHECK();
#else
    if (kernel == 3) {  // gemm_pd: NT operands, or TT (the weight gradients) with fp32 outputs
        if (ta != tb || kps / BK < 2 || (ta && epi < EPI_F32)) return (int)hipErrorInvalidValue;
        const int items = p.tiles * split;
        const int grid = items < num_cus() ? items : num_cus();
        if (ta) {
            switch (epi) {
                case EPI_F32: gemm_pd<EPI_F32, 1, 20, 7, 100, false, 0, 18, true, true><<<grid, PNTHR, 0, s>>>(p); break;
                case EPI_F32ACC: gemm_pd<EPI_F32ACC, 1, 20, 7, 100, false, 0, 18, true, true><<<grid, PNTHR, 0, s>>>(p); break;
                default: gemm_pd<EPI_F32ATOM, 1, 20, 7, 100, false, 0, 18, true, true><<<grid, PNTHR, 0, s>>>(p); break;
            }
            TDL_LAUNCH_CHECK();
        }
        // schedule variants (plain bf16 epilogue only): TDL_PD_SCHED, read per launch (in-process A/B)
        const char* sv = std::getenv("TDL_PD_SCHED");
        const int v = (sv && epi == EPI_BF16) ? std::atoi(sv) : 0;
        if (v > 0) {
            switch (v) {
                case 1: gemm_pd<0, 2, 36, 6, 110><<<grid, PNTHR, 0, s>>>(p); break;
                case 2: gemm_pd<0, 2, 40, 5, 96><<<grid, PNTHR, 0, s>>>(p); break;
                case 3: gemm_pd<0, 2, 36, 6, 100><<<grid, PNTHR, 0, s>>>(p); break;
                case 4: gemm_pd<0, 1, 19, 7, 104><<<grid, PNTHR, 0, s>>>(p); break;
                case 6: gemm_pd<0, 1, 20, 7, 100, true, 1><<<grid, PNTHR, 0, s>>>(p); break;
                case 7: gemm_pd<0, 1, 26, 6, 100, true, 0, 24><<<grid, PNTHR, 0, s>>>(p); break;
                case 8: gemm_pd<0, 1, 24, 6, 100, true, 0, 22><<<grid, PNTHR, 0, s>>>(p); break;
                case 9: gemm_pd<0, 1, 30, 6, 104, true, 0, 28><<<grid, PNTHR, 0, s>>>(p); break;
                case 10: gemm_pd<0, 1, 20, 7, 100, true, 0, 18, false, false, true><<<grid, PNTHR, 0, s>>>(p); break;
                default: gemm_pd<0, 1, 20, 7, 108><<<grid, PNTHR, 0, s>>>(p); break;
            }
            TDL_LAUNCH_CHECK();
        }
        const char* xe = std::getenv("TDL_PD_X4");   // "0": per-tile-row stores (A/B)
        const bool x4 = (N % 8 == 0) && (ldc % 8 == 0) && ((uintptr_t)C % 16 == 0) && !(xe && xe[0] == '0');
        if ((epi == EPI_BF16 || epi == EPI_GELU || epi == EPI_DGELU) && x4 && (epi == EPI_BF16 || (uintptr_t)aux % 16 == 0)) {
            // (a bias / no-bias branch inside one kernel pushed it past 256 VGPRs: 13 spills whose
            // reloads drained every copy in flight, so the two are separate instantiations)
            if (epi == EPI_BF16 && bias == nullptr)
                gemm_pd<EPI_BF16, 1, 20, 7, 100, true, 0, 18, false, false, false, true><<<grid, PNTHR, 0, s>>>(p);
            else if (epi == EPI_BF16) gemm_pd<EPI_BF16, 1, 20, 7, 100, true><<<grid, PNTHR, 0, s>>>(p);
            else if (epi == EPI_GELU) gemm_pd<EPI_GELU, 1, 20, 7, 100, true><<<grid, PNTHR, 0, s>>>(p);
            else gemm_pd<EPI_DGELU, 1, 20, 7, 100, true><<<grid, PNTHR, 0, s>>>(p);
            TDL_LAUNCH_CHECK();
        }
        switch (epi) {
            case 0: gemm_pd<0><<<grid, PNTHR, 0, s>>>(p); break;
            case 1: gemm_pd<1><<<grid, PNTHR, 0, s>>>(p); break;
            case 2: gemm_pd<2><<<grid, PNTHR, 0, s>>>(p); break;
            case 3: gemm_pd<3><<<grid, PNTHR, 0, s>>>(p); break;
            case 4: gemm_pd<4><<<grid, PNTHR, 0, s>>>(p); break;
            case 5: gemm_pd<5><<<grid, PNTHR, 0, s>>>(p); break;
            default: gemm_pd<6><<<grid, PNTHR, 0, s>>>(p); break;
        }
        TDL_LAUNCH_CHECK();
    }
    if (kernel == 0) {
        if (kps / BK < 2) return (int)hipErrorInvalidValue;  // a tile's first and last K step differ
        const int items = p.tiles * split;
        const int grid = items < num_cus() ? items : num_cus();
#define P4_EPI(TA_, TB_)                                                 \
    switch (epi) {                                                       \
        case 0: gemm_p4<TA_, TB_, 0><<<grid, PNTHR, 0, s>>>(p); break;  \
        case 1: gemm_p4<TA_, TB_, 1><<<grid, PNTHR, 0, s>>>(p); break;  \
        case 2: gemm_p4<TA_, TB_, 2><<<grid, PNTHR, 0, s>>>(p); break;  \
        case 3: gemm_p4<TA_, TB_, 3><<<grid, PNTHR, 0, s>>>(p); break;  \
        case 4: gemm_p4<TA_, TB_, 4><<<grid, PNTHR, 0, s>>>(p); break;  \
        case 5: gemm_p4<TA_, TB_, 5><<<grid, PNTHR, 0, s>>>(p); break;  \
        default: gemm_p4<TA_, TB_, 6><<<grid, PNTHR, 0, s>>>(p); break; \
    }
        // the LDS-staged epilogue (NT, bf16 outputs; dGELU keeps the direct stores: its column sums
        // and pre-activation tile pushed the staged form past the register file)
        if (lds_epi && !ta && !tb && epi <= EPI_RESADD && p.ldc % 8 == 0) {
            switch (epi) {
                case EPI_BF16: gemm_p4<false, false, EPI_BF16, true><<<grid, PNTHR, 0, s>>>(p); break;
                case EPI_GELU: gemm_p4<false, false, EPI_GELU, true><<<grid, PNTHR, 0, s>>>(p); break;
                default: gemm_p4<false, false, EPI_RESADD, true><<<grid, PNTHR, 0, s>>>(p); break;
            }
            TDL_LAUNCH_CHECK();
        }
        if (!ta && !tb) { P4_EPI(false, false) }
        else if (!ta && tb) { P4_EPI(false, true) }
        else if (ta && !tb) { P4_EPI(true, false) }
        else { P4_EPI(true, true) }
#undef P4_EPI
        TDL_LAUNCH_CHECK();
    }
    if (kps / BK < 2) return (int)hipErrorInvalidValue;  // the ping-pong schedule needs two K steps
    const dim3 grid(p.tiles, split);
    if (!ta && !tb && epi <= EPI_DGELU && split == 1 && p.ldc % 8 == 0) {
        switch (epi) {
            case EPI_BF16: gemm_pp<false, false, EPI_BF16, true><<<grid, NTHR, 0, s>>>(p); break;
            case EPI_GELU: gemm_pp<false, false, EPI_GELU, true><<<grid, NTHR, 0, s>>>(p); break;
            case EPI_RESADD: gemm_pp<false, false, EPI_RESADD, true><<<grid, NTHR, 0, s>>>(p); break;
            default: gemm_pp<false, false, EPI_DGELU, true><<<grid, NTHR, 0, s>>>(p); break;
        }
        TDL_LAUNCH_CHECK();
    }
#define PP_LAUNCH(TA_, TB_, E_) gemm_pp<TA_, TB_, E_><<<grid, NTHR, 0, s>>>(p)
#define PP_EPI(TA_, TB_)                       \
    switch (epi) {                             \
        case 0: PP_LAUNCH(TA_, TB_, 0); break; \
        case 1: PP_LAUNCH(TA_, TB_, 1); break; \
        case 2: PP_LAUNCH(TA_, TB_, 2); break; \
        case 3: PP_LAUNCH(TA_, TB_, 3); break; \
        case 4: PP_LAUNCH(TA_, TB_, 4); break; \
        case 5: PP_LAUNCH(TA_, TB_, 5); break; \
        default: PP_LAUNCH(TA_, TB_, 6); break; \
    }
    if (!ta && !tb) { PP_EPI(false, false) }
    else if (!ta && tb) { PP_EPI(false, true) }
    else if (ta && !tb) { PP_EPI(true, false) }
    else { PP_EPI(true, true) }
#undef PP_EPI
#undef PP_LAUNCH
    TDL_LAUNCH_CHECK();
#endif
}

// Two weight gradients in ONE launch (gemm_pd, both operands row-contiguous, fp32 split-K slabs):
// C1[s] = A1^T B1 over slice s, C2[s] = A2^T B2, sharing M (the weights' input width) and K (the
// tokens).  The qkv (48 tiles) and out-projection (16 tiles) weight gradients of a GPT-2-medium
// block fill the 256 CUs in one round at split 4 together, where apart they need split 16 (three
// rounds of 16 fp32 slabs for qkv) to do so.  A stored [K][lda], B [K][ldb]; slabs [split][M][N].
TDL_API int tdl_gemm_wgrad_grouped(const void* A1, const void* B1, float* C1, int M1, int N1, int lda1, int ldb1,
                                   const void* A2, const void* B2, float* C2, int M2, int N2, int lda2, int ldb2, int K,
                                   int split, hipStream_t s) {
    if (M1 <= 0 || M2 <= 0 || N1 <= 0 || N2 <= 0 || K <= 0 || split < 1 || K % (BK * split) || K / BK / split < 2)
        return (int)hipErrorInvalidValue;
    if (M1 % 8 || M2 % 8 || N1 % 8 || N2 % 8 || lda1 % 8 || ldb1 % 8 || lda2 % 8 || ldb2 % 8) return (int)hipErrorInvalidValue;
    GemmParams p{(const bf16_t*)A1, (const bf16_t*)B1, C1, nullptr, nullptr, nullptr, M1, N1, K, lda1, ldb1, N1,
                 K / split, (long long)M1 * N1, (N1 + BN - 1) / BN, 0, split, 0, g_gemm_ts};
    const char* g = std::getenv("TDL_GEMM_GROUPM");
    p.group_m = g ? std::atoi(g) : 8;
    p.tiles = ((M1 + BM - 1) / BM) * p.tiles_n;
    p.g2.A = (const bf16_t*)A2;
    p.g2.B = (const bf16_t*)B2;
    p.g2.C = C2;
    p.g2.M = M2;
    p.g2.N = N2;
    p.g2.lda = lda2;
    p.g2.ldb = ldb2;
    p.g2.ldc = N2;
    p.g2.tiles_n = (N2 + BN - 1) / BN;
    p.g2.tiles = ((M2 + BM - 1) / BM) * p.g2.tiles_n;
    p.g2.split_stride = (long long)M2 * N2;
    p.items1 = p.tiles * split;
    const int items = p.items1 + p.g2.tiles * split;
    if (items > num_cus()) return (int)hipErrorInvalidValue;   // one item per workgroup (the caller splits less)
    const int grid = items;
    gemm_pd<EPI_F32, 1, 20, 7, 100, false, 0, 18, true, true, false, false, true><<<grid, PNTHR, 0, s>>>(p);
    TDL_LAUNCH_CHECK();
}
