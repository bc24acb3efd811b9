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
// Geometry: workgroup tile 256 x 256, K step 64, 512 threads = 8 waves as 2 (m) x 4 (n); each wave
// owns a 128 x 64 output block = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 (the 16x16 shape holds a
// higher clock than 32x32x16 on random data, cdna_hip_programming.md rule 28).  The MFMA "A"
// operand is the B tile and the MFMA "B" operand the A tile, so the accumulator of a tile holds
// D[n][m]: lane l owns output row m = l & 15 and FOUR CONSECUTIVE columns n = 4 (l >> 4) + 0..3 —
// one 8-byte bf16 / 16-byte fp32 vector store per (tile, lane), no shuffles.
//
// Staging: both operands go global -> LDS with global_load_lds_dwordx4 (1 KiB per wave
// instruction, lane-linear LDS image), two LDS stages of 64 KiB (one K step of A and B each).
//   k-contiguous tile [256 rows][64 k] : 128-B rows, 16-B chunk c of row r stored at c ^ (r & 7)
//       (source-address permutation, cdna_hip_programming.md rule 21); fragments read with
//       ds_read_b128 — every 16-lane group of a read hits 16 distinct bank slots.
//   row-contiguous tile [64 k][256 rows] : 512-B k-rows, 32-B block b of k-row k stored at
//       b ^ f(k), f(k) = (k & 3) | ((k >> 1) & 4); fragments read with ds_read_b64_tr_b16 (T10):
//       the 8 k-rows a 32-lane half touches map to 8 distinct 32-B bank blocks (conflict-free).
// The tile for K step t+1 is issued at the top of step t and waited for (vmcnt(0) + barrier) at
// its end, so each DMA has a whole step of MFMA work (~2k cycles per SIMD) to land.
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
    int rotate;  // persistent kernels: rotate the K order per XCD group
};

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

template <bool TA, bool TB, int EPI, int SCHED>
__global__ __launch_bounds__(NTHR, 2) void gemm_kernel(GemmParams p) {
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 2, wn = w & 3;
    const int wg = xcd_remap(blockIdx.x, p.tiles);
    const int tm = wg / p.tiles_n, tn = wg - tm * p.tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = blockIdx.y * p.k_per_split;
    const int kend = min(p.K, kbeg + p.k_per_split);
    const int nk = (kend - kbeg) / BK;

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    Stager<TA> sa;
    Stager<TB> sb;
    sa.init(p.lda, m0, p.M, w, lane);
    sb.init(p.ldb, n0, p.N, w, lane);
    auto stage_a = [&](int t, int buf) { sa.issue(p.A, p.lda, m0, p.M, kbeg + t * BK, smem + buf * STAGE_BYTES, w); };
    auto stage_b = [&](int t, int buf) {
        sb.issue(p.B, p.ldb, n0, p.N, kbeg + t * BK, smem + buf * STAGE_BYTES + TILE_BYTES, w);
    };
    // fragments: B tiles j = 0..3 (MFMA A operand) of one 32-deep sub-step; A tiles in two halves
    auto load_b = [&](bf16x8_t (&f)[4], int buf, int ks) {
        const char* Bt = smem + buf * STAGE_BYTES + TILE_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = frag<TB>(Bt, wn * 64 + 16 * j, ks, lane);
    };
    auto load_a = [&](bf16x8_t (&f)[4], int buf, int ks, int half) {
        const char* At = smem + buf * STAGE_BYTES;
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = frag<TA>(At, wm * 128 + 64 * half + 16 * i, ks, lane);
    };
    auto mma = [&](const bf16x8_t (&fb)[4], const bf16x8_t (&fa)[4], int half) {
        if (SCHED & 16) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[4 * half + i][j] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[4 * half + i][j], 0, 0, 0);
        if (SCHED & 16) __builtin_amdgcn_s_setprio(0);
    };
    // Quarter-step scheduling region: with SCHED bit 5 the reads / DMAs issued in the region are
    // spread between its 16 MFMAs (one after each of the first ones) instead of issued up front.
    constexpr int RD = TA ? 2 : 1, RDB = TB ? 2 : 1;  // LDS read instructions per fragment
    auto region_end = [&](int n_ds, int n_vm) {
        if (SCHED & 32) {
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);             // 1 MFMA
                if (k < n_vm) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // 1 DMA (VMEM read)
                if (2 * k < n_ds) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 LDS reads
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto vm_wait = [&](int n) {  // s_waitcnt vmcnt(n) lgkmcnt(0), n in {0, 4, 8}
        if (SCHED & 4) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if (n >= 8) {
            asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        } else if (n >= 4) {
            asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        }
    };
    auto barrier = [&]() {
        if (!(SCHED & 8)) __builtin_amdgcn_s_barrier();
    };

    if (SCHED == 0) {
        if (nk > 0) {
            stage_a(0, 0);
            stage_b(0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
        for (int t = 0; t < nk; ++t) {
            const int cur = t & 1;
            if (t + 1 < nk) {
                stage_a(t + 1, cur ^ 1);
                stage_b(t + 1, cur ^ 1);
            }
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8_t fb[4], fa0[4], fa1[4];
                load_b(fb, cur, ks);
                load_a(fa0, cur, ks, 0);
                load_a(fa1, cur, ks, 1);
                mma(fb, fa0, 0);
                mma(fb, fa1, 1);
            }
            // tile t+1 landed (own DMAs) and this wave's reads of stage `cur` retired, then the
            // barrier publishes both to the other waves (stage `cur` is restaged at step t+1)
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
    } else {
        // Software pipeline in quarter steps (16 MFMAs per wave each):
        //   Q1 (t,ks0): MFMA B0 x Alo   | read Ahi(t,0)            [| DMA B of tile t+1 (default)]
        //   Q2 (t,ks0): MFMA B0 x Ahi   | read B1(t,1), Alo(t,1)
        //   Q3 (t,ks1): MFMA B1 x Alo   | read Ahi(t,1)            [| bit 1: barrier, DMA B of t+2]
        //   Q4 (t,ks1): [own DMAs of tile t+1 done, own reads of stage t&1 done] barrier |
        //               DMA A of tile t+2 into stage t&1; read B0(t+1,0), Alo(t+1,0);  MFMA B1 x Ahi
        // Every fragment read has a quarter step (16 MFMAs per wave) to land, every DMA 3-5 quarters.
        constexpr bool B_EARLY = (SCHED & 2) != 0;
        bf16x8_t B0[4], B1[4], Alo[4], Ahi[4];
        if (nk > 0) {
            stage_a(0, 0);
            stage_b(0, 0);
            if (nk > 1) {
                if (B_EARLY) stage_b(1, 1);
                stage_a(1, 1);
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // tile 0 landed
                if (!B_EARLY) {
                    __builtin_amdgcn_s_barrier();
                } else {
                    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                }
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            load_b(B0, 0, 0);
            load_a(Alo, 0, 0, 0);
        }
        for (int t = 0; t < nk; ++t) {
            const int cur = t & 1;
            // Q1
            const bool b_now = !B_EARLY && t + 1 < nk;
            if (b_now) stage_b(t + 1, cur ^ 1);
            load_a(Ahi, cur, 0, 1);
            mma(B0, Alo, 0);
            region_end(4 * RD, b_now ? 4 : 0);
            // Q2
            load_b(B1, cur, 1);
            load_a(Alo, cur, 1, 0);
            mma(B0, Ahi, 1);
            region_end(4 * RD + 4 * RDB, 0);
            // Q3
            bool b3 = false;
            if (B_EARLY) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                barrier();
                if (t + 2 < nk) {
                    stage_b(t + 2, cur);
                    b3 = true;
                }
            }
            load_a(Ahi, cur, 1, 1);
            mma(B1, Alo, 0);
            region_end(4 * RD, b3 ? 4 : 0);
            // Q4: default order of DMA groups: A(t+1)@Q4(t-1), B(t+1)@Q1(t) -> wait all (vmcnt 0);
            //     B_EARLY: B(t+1)@Q3(t-1), A(t+1)@Q4(t-1), B(t+2)@Q3(t) -> vmcnt(4)
            vm_wait(B_EARLY && b3 ? 4 : 0);
            barrier();
            const bool a4 = t + 2 < nk;
            if (a4) stage_a(t + 2, cur);
            if (t + 1 < nk) {
                load_b(B0, cur ^ 1, 0);
                load_a(Alo, cur ^ 1, 0, 0);
            }
            mma(B1, Ahi, 1);
            region_end(t + 1 < nk ? 4 * RD + 4 * RDB : 0, a4 ? 4 : 0);
        }
    }

    // ---------------------------------------------------------------- epilogue
    const int g = lane >> 4;
    float csum[4][4];
    if (EPI == EPI_DGELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) csum[j][r] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + 16 * j + 4 * g;
        const bool nok = n < p.N;
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if ((EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_RESADD) && p.bias != nullptr && nok)
            unpack4(*(const uint2*)(p.bias + n), bv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int m = m0 + wm * 128 + 16 * i + (lane & 15);
            if (!(nok && m < p.M)) continue;
            float v[4] = {acc[i][j][0] + bv[0], acc[i][j][1] + bv[1], acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]};
            const size_t off = (size_t)m * p.ldc + n;
            if (EPI == EPI_BF16) {
                *(uint2*)((bf16_t*)p.C + off) = pack4(v);
            } else if (EPI == EPI_GELU) {
                *(uint2*)(p.aux + off) = pack4(v);
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
                *(uint2*)((bf16_t*)p.C + off) = pack4(v);
            } else if (EPI == EPI_RESADD) {
                float o[4];
                unpack4(*(const uint2*)((const bf16_t*)p.C + off), o);
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += o[r];
                *(uint2*)((bf16_t*)p.C + off) = pack4(v);
            } else if (EPI == EPI_DGELU) {
                float u[4];
                unpack4(*(const uint2*)(p.aux + off), u);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[r] = acc[i][j][r] * gelu_tanh_grad(u[r]);
                    csum[j][r] += v[r];
                }
                *(uint2*)((bf16_t*)p.C + off) = pack4(v);
            } else if (EPI == EPI_F32) {
                float* c = (float*)p.C + (size_t)blockIdx.y * p.split_stride + off;
                *(float4*)c = make_float4(v[0], v[1], v[2], v[3]);
            } else if (EPI == EPI_F32ACC) {
                float4* c = (float4*)((float*)p.C + off);
                float4 o = *c;
                *c = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
            } else {  // EPI_F32ATOM
                float* c = (float*)p.C + off;
#pragma unroll
                for (int r = 0; r < 4; ++r) atomicAdd(c + r, v[r]);
            }
        }
    }
    if (EPI == EPI_DGELU && p.colsum != nullptr) {
        // sum over the 16 lanes of a group (rows), then one atomic per column per wave
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float s = csum[j][r];
                s += __shfl_xor(s, 1, 64);
                s += __shfl_xor(s, 2, 64);
                s += __shfl_xor(s, 4, 64);
                s += __shfl_xor(s, 8, 64);
                csum[j][r] = s;
            }
        if ((lane & 15) < 4) {
            const int r = lane & 3;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int n = n0 + wn * 64 + 16 * j + 4 * g + r;
                const float s = r == 0 ? csum[j][0] : r == 1 ? csum[j][1] : r == 2 ? csum[j][2] : csum[j][3];
                if (n < p.N) atomicAdd(p.colsum + n, s);
            }
        }
    }
}


// ============================================================================ persistent kernel
// One workgroup per CU walks its share of the output tiles (and split-K slices): 256 threads =
// 4 waves as 2 (m) x 2 (n), one wave per SIMD, each wave a 128 x 128 block = 8 x 8 MFMA tiles, so
// the 256 accumulator registers live in AGPRs and the 512-entry register file is one wave's.
// Versus 8 waves of 128 x 64 this reads a third less LDS per MFMA (hipBLASLt's fastest gfx950
// kernels for these shapes use the same geometry and a persistent grid: rocprofv3 SQ_WAVES).
//
// The DMA pipeline runs across tile boundaries: step s = (item, k step) is staged into LDS stage
// s & 1 two steps ahead, so the next tile's first K steps land while the current tile finishes and
// only the epilogue itself (accumulator read-out + stores) interrupts the MFMA stream.
// Per step, two phases of 64 MFMAs:
//   A (k-half 0): MFMAs on F0                      | read F1 = frags(s, k-half 1)
//   B (k-half 1): [DMA(s+1) landed, own reads of stage s&1 retired] barrier |
//                 DMA step s+2 -> stage s&1; read F0 = frags(s+1, k-half 0) | MFMAs on F1
// The DMA copies and fragment reads are spread between the MFMAs (sched_group_barrier), so the
// single wave of a SIMD keeps its matrix pipe fed while it issues them.
constexpr int PNTHR = 256;

struct PFrags {
    bf16x8_t b[8], a[8];
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

// ---- asm-owned accumulators: tile T = 8 i + j (i: A tile, j: B tile) lives in a[4T : 4T+3].
// hipcc cannot keep 256 loop-carried MFMA accumulators in place (it shuffled them through VGPRs
// inside the K loop, with spills); the MFMAs are therefore inline asm on fixed AGPRs, and one
// empty asm statement clobbering a0..a255 makes the kernel descriptor allocate them.
template <int T>
__device__ __forceinline__ void amfma(const bf16x8_t& b, const bf16x8_t& a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" ::"v"(b), "v"(a), "i"(4 * T), "i"(4 * T + 3));
}
template <int T>
__device__ __forceinline__ void amfma0(const bf16x8_t& b, const bf16x8_t& a) {  // C = 0: first K step
    asm volatile("v_mfma_f32_16x16x32_bf16 a[%c2:%c3], %0, %1, 0" ::"v"(b), "v"(a), "i"(4 * T), "i"(4 * T + 3));
}
template <int T>
__device__ __forceinline__ f32x4 aread() {
    float x, y, z, w;
    asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\tv_accvgpr_read_b32 %2, a%c6\n\t"
                 "v_accvgpr_read_b32 %3, a%c7"
                 : "=v"(x), "=v"(y), "=v"(z), "=v"(w)
                 : "i"(4 * T), "i"(4 * T + 1), "i"(4 * T + 2), "i"(4 * T + 3));
    return f32x4{x, y, z, w};
}
// 64 MFMAs of one 32-deep k-half in tile order T = 0..63; after MFMA T the hook issues that
// slot's companion instructions (DMA copies / fragment reads), pinned by a scheduling fence
template <int T, bool ZERO, class Hook>
__device__ __forceinline__ void mfma_run(const PFrags& f, Hook& hook) {
    if constexpr (T < 64) {
        if constexpr (ZERO) amfma0<T>(f.b[T % 8], f.a[T / 8]);
        else amfma<T>(f.b[T % 8], f.a[T / 8]);
        hook(std::integral_constant<int, T>{});
        __builtin_amdgcn_sched_barrier(0);
        mfma_run<T + 1, ZERO>(f, hook);
    }
}
template <bool TA, bool TB, int EPI>
__global__ __launch_bounds__(PNTHR, 1) void gemm_persistent(GemmParams p) {
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    asm volatile("" ::: "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63", "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79", "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95", "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111", "a112", "a113", "a114", "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127", "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143", "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159", "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", "a172", "a173", "a174", "a175", "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191", "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207", "a208", "a209", "a210", "a211", "a212", "a213", "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223", "a224", "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", "a236", "a237", "a238", "a239", "a240", "a241", "a242", "a243", "a244", "a245", "a246", "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255");
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

    // item i of this workgroup -> tile origin and split slice (split-major: the items running at
    // the same time are consecutive tiles of one slice, which share operand panels in L2)
    auto coords = [&](int i, int& m0, int& n0, int& sp) {
        const int item = lb + i * G;
        sp = item / p.tiles;
        const int tile = item - sp * p.tiles;
        const int tm = tile / p.tiles_n;
        m0 = tm * BM;
        n0 = (tile - tm * p.tiles_n) * BN;
    };

    Stager<TA, 4> sa;
    Stager<TB, 4> sb;
    // ---- producer (DMA) state: the step it stages next; after the last step it repeats it into
    // the free stage (harmless, keeps the copy count per K step constant)
    int pi = 0, pt = 0, pm0, pn0, psp;
    coords(0, pm0, pn0, psp);
    sa.init(p.lda, pm0, p.M, w, lane);
    sb.init(p.ldb, pn0, p.N, w, lane);
    int prod_left = total;
    auto produce_rsrc = [&](__amdgpu_buffer_rsrc_t& ra, __amdgpu_buffer_rsrc_t& rb) {
        const int k0 = psp * p.k_per_split + pt * BK;
        ra = sa.rsrc(p.A, p.lda, pm0, p.M, k0);
        rb = sb.rsrc(p.B, p.ldb, pn0, p.N, k0);
    };
    auto produce_advance = [&]() {
        if (--prod_left > 0) {
            if (++pt == nk) {
                pt = 0;
                ++pi;
                coords(pi, pm0, pn0, psp);
                sa.init(p.lda, pm0, p.M, w, lane);
                sb.init(p.ldb, pn0, p.N, w, lane);
            }
        } else {
            prod_left = 0;
        }
    };
    auto frag_b = [&](int buf, int j, int ks) {
        return frag<TB>(smem + buf * STAGE_BYTES + TILE_BYTES, wn * 128 + 16 * j, ks, lane);
    };
    auto frag_a = [&](int buf, int i, int ks) { return frag<TA>(smem + buf * STAGE_BYTES, wm * 128 + 16 * i, ks, lane); };

    PFrags F0, F1;
    {   // prologue: steps 0 and 1 in flight, step 0's first k-half in registers
        __amdgpu_buffer_rsrc_t ra, rb;
        for (int st = 0; st < 2; ++st) {
            produce_rsrc(ra, rb);
            char* base = smem + st * STAGE_BYTES;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                sa.piece(ra, base, w, i);
                sb.piece(rb, base + TILE_BYTES, w, i);
            }
            produce_advance();
        }
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // step 0 landed, step 1 in flight
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int j = 0; j < 8; ++j) F0.b[j] = frag_b(0, j, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) F0.a[i] = frag_a(0, i, 0);
    }

    int s = 0;
    bool prev_epi = false;
    for (int ci = 0; ci < n_mine; ++ci) {
        int cm0, cn0, csp;
        coords(ci, cm0, cn0, csp);
        int ct = 0;
#pragma clang loop unroll(disable)
        do {
            const int cur = s & 1;
            // ---- phase A: MFMAs on F0 (k-half 0 of step s); F1 = k-half 1 of step s, one
            // fragment read after every 4th MFMA
            {
                auto hook = [&](auto tc) {
                    constexpr int T = decltype(tc)::value;
                    if constexpr (T % 4 == 0) {
                        constexpr int q = T / 4;
                        if constexpr (q < 8) F1.b[q] = frag_b(cur, q, 1);
                        else F1.a[q - 8] = frag_a(cur, q - 8, 1);
                    }
                };
                if (ct == 0) mfma_run<0, true>(F0, hook);
                else mfma_run<0, false>(F0, hook);
            }
            // ---- phase B: step s+1 must have landed (staged two phases ago, before any epilogue
            // stores: vmcnt(63) then covers it), every wave's reads of stage `cur` retired
            if (prev_epi) asm volatile("s_waitcnt vmcnt(63) lgkmcnt(0)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            prev_epi = false;
            {
                __amdgpu_buffer_rsrc_t ra, rb;
                produce_rsrc(ra, rb);
                char* base = smem + cur * STAGE_BYTES;
                const int nxt = cur ^ 1;
                // slots 0..15: the 16 DMA copies of step s+2 into stage `cur`; slots 16..61: the
                // 16 fragment reads of step s+1's k-half 0, one every 3 MFMAs
                auto hook = [&](auto tc) {
                    constexpr int T = decltype(tc)::value;
                    if constexpr (T < 16) {
                        if constexpr (T % 2 == 0) sa.piece(ra, base, w, T / 2);
                        else sb.piece(rb, base + TILE_BYTES, w, T / 2);
                    } else if constexpr ((T - 16) % 3 == 0 && (T - 16) / 3 < 16) {
                        constexpr int q = (T - 16) / 3;
                        if constexpr (q < 8) F0.b[q] = frag_b(nxt, q, 0);
                        else F0.a[q - 8] = frag_a(nxt, q - 8, 0);
                    }
                };
                mfma_run<0, false>(F1, hook);
            }
            produce_advance();
            ++s;
        } while (++ct < nk);
        // ---- epilogue: the last MFMAs' results must be written before the accumulator reads
        asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
        auto get = [&](auto ic, auto jc) { return aread<8 * decltype(ic)::value + decltype(jc)::value>(); };
        epilogue_store<EPI, 8>(p, get, cm0 + wm * 128, cn0 + wn * 128, csp, lane);
        prev_epi = true;
    }
    // no LDS-DMA may still be landing when the workgroup's LDS is handed to the next one
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ============================================================================ persistent, 8 waves
// The 8-wave geometry of gemm_kernel (2 waves per SIMD, 128 x 64 per wave, accumulators in
// VGPRs) on a persistent grid.  Two waves per SIMD are what hides the LDS-DMA issue cost (60-185
// cycles per 1-KiB copy): the partner wave's MFMAs keep the matrix pipe busy meanwhile.  With one
// wave per SIMD (gemm_persistent) the 16 copies per K step stall the pipe and it ran 10-20 % slower.
// Quarter-step schedule as gemm_kernel's pipeline; the DMA producers run ahead ACROSS items (A two
// steps ahead, B one), so a tile's first K steps land while the previous tile finishes.
template <bool TA, bool TB, int EPI, int ABL = 0>
__global__ __launch_bounds__(NTHR, 2) void gemm_persistent8(GemmParams p) {
    // ABL (benchmark ablations, wrong results): 1 = no operand staging in the K loop, 2 = no
    // fragment reads in the K loop, 4 = no waits / barriers in the K loop
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = w >> 2, wn = w & 3;
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
        const int tm = tile / p.tiles_n;
        m0 = tm * BM;
        n0 = (tile - tm * p.tiles_n) * BN;
    };
    // K-order rotation per XCD group (blockIdx % 8; speed only)
    const int rot = p.rotate ? ((int)(blockIdx.x & 7) * nk) >> 3 : 0;
    auto kstep = [&](int t) { return t + rot < nk ? t + rot : t + rot - nk; };

    // ---- producer: the (item, k step) whose operands it loads next (after the last step it repeats
    // that step; its copies then go to a stage nobody reads any more)
    int pi = 0, pt = 0, pm0, pn0, psp, pleft = total;
    coords(0, pm0, pn0, psp);
    Stager<TA, 8> sa;
    Stager<TB, 8> sb;
    sa.init(p.lda, pm0, p.M, w, lane);
    sb.init(p.ldb, pn0, p.N, w, lane);
    u32x4_t ra[4], rb[4];  // one K step of this wave's share of the operand tiles, in flight
    auto produce_load = [&]() {
        const int k0 = psp * p.k_per_split + kstep(pt) * BK;
        sa.load_regs(p.A, p.lda, pm0, p.M, k0, ra);
        sb.load_regs(p.B, p.ldb, pn0, p.N, k0, rb);
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
    auto produce_write = [&](int buf) {
        char* base = smem + buf * STAGE_BYTES;
        sa.write_regs(base, w, lane, ra);
        sb.write_regs(base + TILE_BYTES, w, lane, rb);
    };
    auto load_b = [&](bf16x8_t (&f)[4], int buf, int ks) {
        const char* Bt = smem + buf * STAGE_BYTES + TILE_BYTES;
#pragma unroll
        for (int j = 0; j < 4; ++j) f[j] = frag<TB>(Bt, wn * 64 + 16 * j, ks, lane);
    };
    auto load_a = [&](bf16x8_t (&f)[4], int buf, int ks, int half) {
        const char* At = smem + buf * STAGE_BYTES;
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = frag<TA>(At, wm * 128 + 64 * half + 16 * i, ks, lane);
    };
    f32x4 acc[8][4];
    auto mma = [&](const bf16x8_t (&fb)[4], const bf16x8_t (&fa)[4], int half) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[4 * half + i][j] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[4 * half + i][j], 0, 0, 0);
    };

    // prologue: steps 0 and 1 into stages 0 and 1, step 2's operands in flight into registers
    produce_load();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    produce_write(0);
    produce_load();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    produce_write(1);
    produce_load();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    bf16x8_t B0[4], B1[4], Alo[4], Ahi[4];
    load_b(B0, 0, 0);
    load_a(Alo, 0, 0, 0);
    if (ABL & 2) {  // ablation: fragments read once
        load_b(B1, 0, 1);
        load_a(Ahi, 0, 1, 1);
    }

    int s = 0;
    for (int ci = 0; ci < n_mine; ++ci) {
        int cm0, cn0, csp;
        coords(ci, cm0, cn0, csp);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        int ct = 0;
#pragma clang loop unroll(disable)
        do {
            const int cur = s & 1;
            // Q1
            if (!(ABL & 2)) load_a(Ahi, cur, 0, 1);
            __builtin_amdgcn_sched_barrier(0);
            mma(B0, Alo, 0);
            __builtin_amdgcn_sched_barrier(0);
            // Q2
            if (!(ABL & 2)) {
                load_b(B1, cur, 1);
                load_a(Alo, cur, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            mma(B0, Ahi, 1);
            __builtin_amdgcn_sched_barrier(0);
            // Q3
            if (!(ABL & 2)) load_a(Ahi, cur, 1, 1);
            __builtin_amdgcn_sched_barrier(0);
            mma(B1, Alo, 0);
            __builtin_amdgcn_sched_barrier(0);
            // Q4: step s+2's operands arrived in registers; this wave's LDS writes (step s+1) and
            // reads of stage `cur` retired; after the barrier stage `cur` is free and step s+1 visible
            if (!(ABL & 4)) {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            }
            if (!(ABL & 1)) {
                produce_write(cur);  // step s+2 -> stage `cur`
                produce_load();      // step s+3 -> registers (one K step to arrive)
            }
            if (!(ABL & 2)) {
                load_b(B0, cur ^ 1, 0);
                load_a(Alo, cur ^ 1, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            mma(B1, Ahi, 1);
            __builtin_amdgcn_sched_barrier(0);
            ++s;
        } while (++ct < nk);
        auto get = [&](auto ic, auto jc) { return acc[decltype(ic)::value][decltype(jc)::value]; };
        epilogue_store<EPI, 4>(p, get, cm0 + wm * 128, cn0 + wn * 64, csp, lane);
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
// Vector-memory operations one wave's epilogue_store<EPI, 4> issues, counted LOW (stores and
// operand loads only): the persistent form lets that many more ops stay in flight at the waits of
// the first K step after an epilogue (vmcnt retires in issue order: MI355X_MICROARCH.md, vmcnt),
// so the next tile's MFMAs start while the stores drain.  Under-counting only waits longer.
template <int EPI>
constexpr int pp_epi_vmem() {
    return EPI == EPI_BF16 || EPI == EPI_F32 ? 32 : EPI == EPI_F32ATOM ? 128 : 64;
}
// copies allowed in flight at phase q's wait: 2 per issuing phase among q-3..q (PM / MK: issue
// masks of the previous / this K step), plus EX, capped at the 6-bit vmcnt field
constexpr int pp_vm_allow(int PM, int MK, int q, int EX) {
    int n = 0;
    for (int d = 0; d < 4; ++d) {
        const int x = q - d;  // <= 0: phase x + 4 of the previous step
        n += (x >= 1 ? (MK >> (x - 1)) & 1 : (PM >> (x + 3)) & 1) ? 2 : 0;
    }
    n += EX;
    return n > 63 ? 63 : n;
}
template <int N>
__device__ __forceinline__ void wait_vmc() {
    asm volatile("s_waitcnt vmcnt(%c0)" ::"n"(N) : "memory");
}

// PERS: persistent form (NT only): gridDim.x (a multiple of 8) workgroups walk the tiles
// blockIdx.x, + gridDim.x, ...; the copies of the next tile's first two K steps are issued during
// the current tile's last two (the K-step sequence runs on across tiles, nk even keeps the LDS
// buffer parity), so neither the pipeline fill nor the store drain of a tile is exposed.
// LEPI (EPI_BF16 / EPI_GELU, one tile per workgroup): LDS-staged epilogue — after the K loop each
// wave writes its 128 x 64 bf16 block into its own 16 KiB of the (then idle) operand LDS (16-B chunks
// XOR-swizzled by row) and reads it back row-contiguous, so every store instruction writes 8 whole
// 128-B row segments (1 KiB) instead of 16 rows x 32 B: a quarter of the store instructions and
// L2 requests of the direct MFMA-layout store.
template <bool TA, bool TB, int EPI, int ABL = 0, bool PERS = false, bool LEPI = false>
__global__ __launch_bounds__(NTHR, 1) void gemm_pp(GemmParams p) {
    static_assert(!LEPI || (!PERS && EPI <= EPI_DGELU), "LDS epilogue: bf16 outputs, one tile");
    // ABL (timing-only ablations, wrong results): 1 = no copies in the K loop, 2 = no fragment
    // reads in the K loop, 4 = no waits / barriers in the K loop, 8 = no epilogue stores
    static_assert(!PERS || (!TA && !TB), "persistent ping-pong: k-contiguous operands only");
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];  // [buf 2][UA0 UA1 UB0 UB1][16 KiB]
    constexpr int UNIT = 16384, BUF = 4 * UNIT;
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = w >> 2, wc = w & 3;
    auto coords = [&](int item, int& mm, int& nn) {
        const int wg = xcd_remap(item, p.tiles);
        const int tm = wg / p.tiles_n;
        mm = tm * BM;
        nn = (wg - tm * p.tiles_n) * BN;
    };
    int item = blockIdx.x;
    int m0, n0, m1 = 0, n1 = 0;
    coords(item, m0, n0);
    bool has_next = PERS && item + (int)gridDim.x < p.tiles;
    if (has_next) coords(item + gridDim.x, m1, n1);
    const int kbeg = blockIdx.y * p.k_per_split;
    const int nk = p.k_per_split / BK;  // >= 2 (host); PERS: even and >= 4

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
    auto issue_at = [&](int u, int t, int mm, int nn) {
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
    auto issue = [&](int u, int t) {  // K step t of this tile, or t - nk of the next one
        if (!PERS || t < nk) issue_at(u, t, m0, n0);
        else issue_at(u, t - nk, m1, n1);
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
    // ex (persistent form, first step after an epilogue): the epilogue's ops may stay in flight
    auto phase_sync = [&](auto nc, auto nxc, bool ex) {
        __builtin_amdgcn_sched_barrier(0);
        if (!(ABL & 4)) {
            if (PERS && ex) wait_vmc<decltype(nxc)::value>();
            else wait_vmc<decltype(nc)::value>();
            __builtin_amdgcn_s_barrier();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
    };
    auto phase_end = [&]() {
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (!(ABL & 4)) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // K step t with this step's / the previous step's issue masks (bit q-1: phase q issues)
    // ex: the first K step after a persistent epilogue (EX more ops allowed in flight)
    constexpr int EX = pp_epi_vmem<EPI>();
    auto step = [&](int t, auto pmc, auto mc, bool ex) {
        constexpr int PM = decltype(pmc)::value, MK = decltype(mc)::value;
        using V1 = std::integral_constant<int, pp_vm_allow(PM, MK, 1, 0)>;
        using V2 = std::integral_constant<int, pp_vm_allow(PM, MK, 2, 0)>;
        using V3 = std::integral_constant<int, pp_vm_allow(PM, MK, 3, 0)>;
        using V4 = std::integral_constant<int, pp_vm_allow(PM, MK, 4, 0)>;
        using X1 = std::integral_constant<int, pp_vm_allow(PM, MK, 1, EX)>;
        using X2 = std::integral_constant<int, pp_vm_allow(PM, MK, 2, EX)>;
        using X3 = std::integral_constant<int, pp_vm_allow(PM, MK, 3, EX)>;
        using X4 = std::integral_constant<int, pp_vm_allow(PM, MK, 4, EX)>;
        const int cur = t & 1;
        constexpr bool RD = !(ABL & 2), CP = !(ABL & 1);
        // P1
        if (RD) readA(cur, 0);
        if (RD) readB(FB0, cur, 0);
        if (CP && (MK & 1)) issue(3, t + 1);
        phase_sync(V1{}, X1{}, ex);
        quad(FB0, 0, 0);
        phase_end();
        // P2
        if (RD) readB(FB1, cur, 1);
        if (CP && (MK & 2)) issue(1, t + 1);
        phase_sync(V2{}, X2{}, ex);
        quad(FB1, 0, 1);
        phase_end();
        // P3
        if (RD) readA(cur, 1);
        if (CP && (MK & 4)) issue(0, t + 2);
        phase_sync(V3{}, X3{}, ex);
        quad(FB1, 1, 1);
        phase_end();
        // P4
        if (CP && (MK & 8)) issue(2, t + 2);
        phase_sync(V4{}, X4{}, ex);
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
    if (wr && !(ABL & 4)) __builtin_amdgcn_s_barrier();  // stagger: group 1 runs one barrier behind
    if (ABL & 2) {
        readA(0, 0);
        readB(FB0, 0, 0);
        readB(FB1, 0, 1);
    }
    using I15 = std::integral_constant<int, 15>;
    using I3 = std::integral_constant<int, 3>;
    using I0 = std::integral_constant<int, 0>;
    auto epilogue = [&]() {
        if (ABL & 8) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
        } else {
            auto get = [&](auto ic, auto jc) { return acc[decltype(ic)::value][decltype(jc)::value]; };
            GemmParams q = p;
            if (ABL & 16) q.M = 0;  // ablation: every store falls outside the buffer (issued, dropped)
            epilogue_store<EPI, 4>(q, get, m0 + wr * 128, n0 + wc * 64, blockIdx.y, lane);
        }
    };
    if constexpr (LEPI) {
        int t = 0;
#pragma clang loop unroll(disable)
        for (; t < nk - 2; ++t) step(t, I15{}, I15{}, false);
        step(t, I15{}, I3{}, false);
        step(t + 1, I3{}, I0{}, false);
        // group 0's extra barrier first: past it every wave has retired its last fragment reads and
        // waited its last copies (vmcnt(0) in the final phase), so the operand LDS is free
        if (!wr && !(ABL & 4)) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");  // no LDS access of the epilogue moves above that barrier
        __builtin_amdgcn_sched_barrier(0);
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
        return;
    } else if constexpr (!PERS) {
        int t = 0;
#pragma clang loop unroll(disable)
        for (; t < nk - 2; ++t) step(t, I15{}, I15{}, false);
        step(t, I15{}, I3{}, false);      // t = nk-2: P3 / P4 have no step t+2
        step(t + 1, I3{}, I0{}, false);   // t = nk-1: nothing left to stage
        epilogue();
    } else {
        // ONE step instantiation (a loop of several spilled the accumulators): every step stages
        // (the last tile's last two re-stage its own first steps, never read), and step 0 may leave
        // the previous epilogue's ops in flight — for the first tile the prologue wait below already
        // retired everything step 0 reads.
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // UB1(0), UA1(0) landed too
        if (!has_next) {
            m1 = m0;
            n1 = n0;
        }
        int t = 0;
#pragma clang loop unroll(disable)
        while (true) {
            step(t, I15{}, I15{}, t == 0);
            if (++t < nk) continue;
            epilogue();
            if (!has_next) break;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            item += gridDim.x;
            m0 = m1;
            n0 = n1;
            has_next = item + (int)gridDim.x < p.tiles;
            if (has_next) coords(item + gridDim.x, m1, n1);
            t = 0;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the unread re-staged copies
    }
    if (!wr && !(ABL & 4)) __builtin_amdgcn_s_barrier();  // match group 1's extra barrier
}

}  // namespace

// C = epilogue(A x B^T) (see the header for the storage flags and epilogue codes).
// Requirements: K % 64 == 0, N % 4 == 0; TA needs M % 8 == 0, TB N % 8 == 0; 16-byte aligned rows
// (lda/ldb % 8 == 0), ldc % 4 == 0.  split > 1 only with EPI 4 (slab i at C + i * split_stride) or
// 6 (atomics); the split is reduced until it divides K / 64 (every slice the same depth).
// epi bits 8..15 select a benchmark variant: 0 (and 10) = the 8-wave kernel with its pipelined
// schedule (default: the fastest of these on MI355X, profiles/r2_gemm_variants.jsonl), 1 = its plain
// schedule, 2..9 = its NT bf16 schedule variants, 11 = the persistent 4-wave kernel, 12 = the
// persistent 8-wave kernel (register-staged producer), 13..18 its timing-only ablations, 19 = 12
// without the per-XCD K rotation (11..19: NT bf16 only), 20 = the ping-pong kernel (NT, every
// epilogue), 21..28 its timing-only ablations (NT bf16).
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
    int variant = (epi >> 8) & 0xff;
    epi &= 0xff;
    if (epi < 0 || epi > 6) return (int)hipErrorInvalidValue;
    if (split < 1) split = 1;
    while (split > 1 && (K / BK) % split) --split;
    if (split > 1 && epi != EPI_F32 && epi != EPI_F32ATOM) return (int)hipErrorInvalidValue;
    const int kps = K / split;
    GemmParams p{(const bf16_t*)A, (const bf16_t*)B, C, (const bf16_t*)bias, (bf16_t*)aux, colsum, M, N, K,
                 lda, ldb, ldc, kps, split_stride, (N + BN - 1) / BN, 0, split, 1};
    p.tiles = ((M + BM - 1) / BM) * p.tiles_n;
    if (variant >= 11 && variant <= 19) {  // benchmark-only persistent kernels (NT, bf16 out)
        if (ta || tb || epi != 0) return (int)hipErrorInvalidValue;
        const int items = p.tiles * split;
        const int grid = items < num_cus() ? items : num_cus();
        if (variant == 11) {
            gemm_persistent<false, false, 0><<<grid, PNTHR, 0, s>>>(p);
        } else {
            p.rotate = variant != 19;
            switch (variant - 12) {
                case 1: gemm_persistent8<false, false, 0, 1><<<grid, NTHR, 0, s>>>(p); break;  // no staging
                case 2: gemm_persistent8<false, false, 0, 2><<<grid, NTHR, 0, s>>>(p); break;  // no LDS reads
                case 4: gemm_persistent8<false, false, 0, 4><<<grid, NTHR, 0, s>>>(p); break;  // no waits
                case 5: gemm_persistent8<false, false, 0, 5><<<grid, NTHR, 0, s>>>(p); break;
                case 6: gemm_persistent8<false, false, 0, 7><<<grid, NTHR, 0, s>>>(p); break;  // MFMA only
                default: gemm_persistent8<false, false, 0, 0><<<grid, NTHR, 0, s>>>(p); break;
            }
        }
        TDL_LAUNCH_CHECK();
    }
    const dim3 grid(p.tiles, split);
    if (variant >= 21 && variant <= 28 && !ta && !tb && epi == 0 && kps / BK >= 2) {  // pp ablations
        switch (variant) {
            case 21: gemm_pp<false, false, 0, 1><<<grid, NTHR, 0, s>>>(p); break;   // no copies
            case 22: gemm_pp<false, false, 0, 2><<<grid, NTHR, 0, s>>>(p); break;   // no frag reads
            case 23: gemm_pp<false, false, 0, 3><<<grid, NTHR, 0, s>>>(p); break;   // MFMA + sync
            case 24: gemm_pp<false, false, 0, 7><<<grid, NTHR, 0, s>>>(p); break;   // MFMA only
            case 25: gemm_pp<false, false, 0, 8><<<grid, NTHR, 0, s>>>(p); break;   // no epilogue
            case 26: gemm_pp<false, false, 0, 15><<<grid, NTHR, 0, s>>>(p); break;  // MFMA only, no epilogue
            case 28: gemm_pp<false, false, 0, 16><<<grid, NTHR, 0, s>>>(p); break;  // stores dropped
            default: gemm_pp<false, false, 0, 4><<<grid, NTHR, 0, s>>>(p); break;   // no sync
        }
        TDL_LAUNCH_CHECK();
    }
    if (variant == 36 && !ta && !tb && epi <= EPI_DGELU && split == 1 && kps / BK >= 2 && p.ldc % 8 == 0) {
        switch (epi) {
            case EPI_BF16: gemm_pp<false, false, EPI_BF16, 0, false, true><<<grid, NTHR, 0, s>>>(p); break;
            case EPI_GELU: gemm_pp<false, false, EPI_GELU, 0, false, true><<<grid, NTHR, 0, s>>>(p); break;
            case EPI_RESADD: gemm_pp<false, false, EPI_RESADD, 0, false, true><<<grid, NTHR, 0, s>>>(p); break;
            default: gemm_pp<false, false, EPI_DGELU, 0, false, true><<<grid, NTHR, 0, s>>>(p); break;
        }
        TDL_LAUNCH_CHECK();
    }
    if (variant == 36) variant = 20;  // other epilogues / layouts: the direct-store ping-pong
    if (variant == 35 && !ta && !tb && kps / BK >= 4 && (kps / BK) % 2 == 0) {  // persistent ping-pong
        const int g8 = num_cus() & ~7;
        const dim3 pgrid(p.tiles < g8 ? p.tiles : g8, split);
        switch (epi) {
            case 0: gemm_pp<false, false, 0, 0, true><<<pgrid, NTHR, 0, s>>>(p); break;
            case 1: gemm_pp<false, false, 1, 0, true><<<pgrid, NTHR, 0, s>>>(p); break;
            case 2: gemm_pp<false, false, 2, 0, true><<<pgrid, NTHR, 0, s>>>(p); break;
            case 3: gemm_pp<false, false, 3, 0, true><<<pgrid, NTHR, 0, s>>>(p); break;
            case 4: gemm_pp<false, false, 4, 0, true><<<pgrid, NTHR, 0, s>>>(p); break;
            case 5: gemm_pp<false, false, 5, 0, true><<<pgrid, NTHR, 0, s>>>(p); break;
            default: gemm_pp<false, false, 6, 0, true><<<pgrid, NTHR, 0, s>>>(p); break;
        }
        TDL_LAUNCH_CHECK();
    }
    if (variant == 20 && kps / BK >= 2) {  // ping-pong kernel
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
    }
    if (variant >= 2 && variant <= 9) {  // schedule variants of the 8-wave kernel (NT, bf16 out only)
        if (ta || tb || epi != 0) return (int)hipErrorInvalidValue;
        switch (variant) {
            case 2: gemm_kernel<false, false, 0, 1><<<grid, NTHR, 0, s>>>(p); break;            // base pipeline
            case 3: gemm_kernel<false, false, 0, 1 | 32><<<grid, NTHR, 0, s>>>(p); break;       // interleave
            case 4: gemm_kernel<false, false, 0, 1 | 2><<<grid, NTHR, 0, s>>>(p); break;        // B early
            case 5: gemm_kernel<false, false, 0, 1 | 2 | 32><<<grid, NTHR, 0, s>>>(p); break;
            case 6: gemm_kernel<false, false, 0, 1 | 4><<<grid, NTHR, 0, s>>>(p); break;        // ablation: no vmcnt
            case 7: gemm_kernel<false, false, 0, 1 | 4 | 8><<<grid, NTHR, 0, s>>>(p); break;    // ablation: no vm/barrier
            case 8: gemm_kernel<false, false, 0, 1 | 16><<<grid, NTHR, 0, s>>>(p); break;       // setprio
            default: gemm_kernel<false, false, 0, 1 | 16 | 32><<<grid, NTHR, 0, s>>>(p); break;
        }
        TDL_LAUNCH_CHECK();
    }
    if (variant == 1) {  // plain (unpipelined) schedule, benchmark reference
        if (epi != 0) return (int)hipErrorInvalidValue;
        if (!ta && !tb) gemm_kernel<false, false, 0, 0><<<grid, NTHR, 0, s>>>(p);
        else if (!ta && tb) gemm_kernel<false, true, 0, 0><<<grid, NTHR, 0, s>>>(p);
        else if (ta && !tb) gemm_kernel<true, false, 0, 0><<<grid, NTHR, 0, s>>>(p);
        else gemm_kernel<true, true, 0, 0><<<grid, NTHR, 0, s>>>(p);
        TDL_LAUNCH_CHECK();
    }
#define G_LAUNCH(TA_, TB_, E_) gemm_kernel<TA_, TB_, E_, 1><<<grid, NTHR, 0, s>>>(p)
#define G_EPI(TA_, TB_)                                  \
    switch (epi) {                                       \
        case 0: G_LAUNCH(TA_, TB_, 0); break;            \
        case 1: G_LAUNCH(TA_, TB_, 1); break;            \
        case 2: G_LAUNCH(TA_, TB_, 2); break;            \
        case 3: G_LAUNCH(TA_, TB_, 3); break;            \
        case 4: G_LAUNCH(TA_, TB_, 4); break;            \
        case 5: G_LAUNCH(TA_, TB_, 5); break;            \
        default: G_LAUNCH(TA_, TB_, 6); break;           \
    }
    if (!ta && !tb) { G_EPI(false, false) }
    else if (!ta && tb) { G_EPI(false, true) }
    else if (ta && !tb) { G_EPI(true, false) }
    else { G_EPI(true, true) }
#undef G_EPI
#undef G_LAUNCH
    TDL_LAUNCH_CHECK();
}
