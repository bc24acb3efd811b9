// Backward-audit primitives of the commit / key / open gradient protocol (security/grad_audit.py,
// parallel/commitments.py, parallel/audit.py).  Reference: the gradient check there is a host
// z-score (/root/reference/attack_detector.py:109-141) that a sign flip passes, and the optimizer
// step it is meant to guard (/root/reference/distributed_trainer.py:197-205, :441-446) applies
// whatever gradient the node holds.
//
//  * BLAKE2s Merkle hash — a collision-resistant 256-bit commitment to a range of 32-bit words:
//      leaf j   = BLAKE2s(words [256 j, 256 j + 256) ; node_offset = j, node_depth = 0)
//      node l,j = BLAKE2s(child digests [32 j, 32 j + 32) of level l - 1 ; node_offset = j, node_depth = l)
//    up to one root per segment (at least one node level), then one combine over the segments'
//    roots (node_depth = 255, last_node).  Bit-identical to Python's hashlib.blake2s with the same
//    node parameters (the CPU path and the GPU tests use it as the oracle).  One thread per leaf /
//    node: 16 compressions of 10 rounds each, integer VALU only.  Two launches per segment: leaves
//    + level 1 (each workgroup's 8 level-1 nodes from its 256 leaf digests in LDS), then the rest of
//    the tree in one workgroup per batch entry (levels >= 3 in LDS); a batch dimension (grid.y)
//    hashes the M per-micro-batch contributions of a step in the same two launches.
//  * keyed sketch — K = 4 full-coverage random-sign projections sum_j s_k(key, j) a_j with the
//    signs derived from a PRIVATE per-step key revealed only after the commitments were received;
//    two-pass, fixed-order reduction (deterministic: the auditor recomputes the auditee's value
//    bit for bit).  Batched over contributions (grid.y).
//  * contribution snapshot — c_i = g - prev, prev = g after micro-batch i's weight gradients.
//
// (r5 used an additive mix32 word hash: a sum of invertible 32-bit mixes, so a second preimage
// cost O(1) — set one word to mix^-1 of the difference — and it travelled folded to 32 bits.)
#include "common.h"

namespace {

// ============================================================================ BLAKE2s
__constant__ uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};

constexpr uint8_t kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

constexpr int LEAF_WORDS = 256;   // 1 KiB leaves: 16 compressions per thread
constexpr int FANOUT = 32;        // 32 child digests (1 KiB) per internal node

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

template <int R>
__device__ __forceinline__ void b2s_round(uint32_t* v, const uint32_t* m) {
#define B2S_G(a, b, c, d, x, y)                 \
    v[a] = v[a] + v[b] + (x);                   \
    v[d] = rotr(v[d] ^ v[a], 16);               \
    v[c] = v[c] + v[d];                         \
    v[b] = rotr(v[b] ^ v[c], 12);               \
    v[a] = v[a] + v[b] + (y);                   \
    v[d] = rotr(v[d] ^ v[a], 8);                \
    v[c] = v[c] + v[d];                         \
    v[b] = rotr(v[b] ^ v[c], 7);
    B2S_G(0, 4, 8, 12, m[kSigma[R][0]], m[kSigma[R][1]]);
    B2S_G(1, 5, 9, 13, m[kSigma[R][2]], m[kSigma[R][3]]);
    B2S_G(2, 6, 10, 14, m[kSigma[R][4]], m[kSigma[R][5]]);
    B2S_G(3, 7, 11, 15, m[kSigma[R][6]], m[kSigma[R][7]]);
    B2S_G(0, 5, 10, 15, m[kSigma[R][8]], m[kSigma[R][9]]);
    B2S_G(1, 6, 11, 12, m[kSigma[R][10]], m[kSigma[R][11]]);
    B2S_G(2, 7, 8, 13, m[kSigma[R][12]], m[kSigma[R][13]]);
    B2S_G(3, 4, 9, 14, m[kSigma[R][14]], m[kSigma[R][15]]);
#undef B2S_G
}

// one compression of block m (t: bytes hashed so far including this block; last: final block)
__device__ __forceinline__ void b2s_compress(uint32_t* h, const uint32_t* m, uint32_t t, bool last, bool last_node) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = h[i];
        v[i + 8] = kIV[i];
    }
    v[12] ^= t;
    v[14] ^= last ? 0xFFFFFFFFu : 0u;
    v[15] ^= last_node ? 0xFFFFFFFFu : 0u;
    b2s_round<0>(v, m);
    b2s_round<1>(v, m);
    b2s_round<2>(v, m);
    b2s_round<3>(v, m);
    b2s_round<4>(v, m);
    b2s_round<5>(v, m);
    b2s_round<6>(v, m);
    b2s_round<7>(v, m);
    b2s_round<8>(v, m);
    b2s_round<9>(v, m);
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

// parameter block of a 32-byte, unkeyed digest with fanout 1, depth 1 (hashlib's defaults) and the
// given node offset (< 2^32 here) / node depth
__device__ __forceinline__ void b2s_init(uint32_t* h, uint32_t node_offset, uint32_t node_depth) {
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = kIV[i];
    h[0] ^= 32u | (1u << 16) | (1u << 24);
    h[2] ^= node_offset;
    h[3] ^= node_depth << 16;
}

// hash `nw` >= 1 words read by `load(block, m)` (block b: words [16 b, 16 b + 16), zero padded)
template <class Load>
__device__ __forceinline__ void b2s_words(uint32_t* h, int nw, bool last_node, Load load) {
    const int nblk = (nw + 15) >> 4;
    uint32_t m[16];
    for (int b = 0; b < nblk; ++b) {
        load(b, m);
        const bool last = b == nblk - 1;
        const uint32_t t = last ? (uint32_t)nw * 4u : (uint32_t)(b + 1) * 64u;
        b2s_compress(h, m, t, last, last_node);
    }
}

// leaves AND their level-1 parents in one launch: out[y][q] = level-1 node q (over leaves
// [32 q, 32 q + 32)) of x[y * stride + lo : ... + hi); each 256-thread workgroup hashes 256 leaves
// into LDS, then 8 of its threads hash the 8 level-1 nodes they form.
// Loads: a thread hashes one 1 KiB leaf, so direct loads put its 64 lanes on 64 different cache
// lines per instruction (the address path, not HBM, bounded the r6 kernel at ~0.6 TB/s).  A full,
// aligned workgroup instead stages its 256 leaves through LDS two blocks (128 B per leaf) at a
// time: 8 consecutive lanes load one leaf's 128 B line, so a wave's uint4 load covers 8 whole lines;
// the next stage's loads are in flight (registers) while the current two compressions run.  Rows
// are padded to 36 words: each lane's 16-byte LDS reads of its own row hit distinct banks.
constexpr int STG_ROW4 = 9;                 // uint4 per padded LDS row (32 words + 4 pad)
constexpr int STAGES = LEAF_WORDS / 32;     // 8 stages of 2 blocks per leaf

template <bool ALIGNED>
__global__ __launch_bounds__(256) void b2s_leaf_l1_kernel(const uint32_t* __restrict__ x, long long stride,
                                                         long long lo, long long hi, long long nleaf,
                                                         uint32_t* __restrict__ out, long long out_stride) {
    __shared__ uint4 stg[256 * STG_ROW4];   // 36 KiB staging; reused for the 256 leaf digests
    uint32_t* dig = reinterpret_cast<uint32_t*>(stg);
    const int tid = threadIdx.x;
    const long long j = (long long)blockIdx.x * 256 + tid;
    const bool full = ALIGNED && (long long)(blockIdx.x + 1) * 256 * LEAF_WORDS <= hi - lo;
    if (full) {
        const uint4* base = reinterpret_cast<const uint4*>(x + (long long)blockIdx.y * stride + lo +
                                                           (long long)blockIdx.x * 256 * LEAF_WORDS);
        // piece p = i * 256 + tid of a stage: leaf p >> 3, 16-byte part p & 7; named registers (an
        // array carried around the stage loop was put in scratch)
        const uint4* src = base + (tid >> 3) * (LEAF_WORDS / 4) + (tid & 7);
        constexpr int LS = 32 * (LEAF_WORDS / 4);     // 32 leaves further: the next 256 pieces
        uint4 r0 = src[0], r1 = src[LS], r2 = src[2 * LS], r3 = src[3 * LS];
        uint4 r4 = src[4 * LS], r5 = src[5 * LS], r6 = src[6 * LS], r7 = src[7 * LS];
        uint4* dst = stg + (tid >> 3) * STG_ROW4 + (tid & 7);
        constexpr int DS = 32 * STG_ROW4;
        uint32_t h[8];
        b2s_init(h, (uint32_t)j, 0u);
        for (int st = 0; st < STAGES; ++st) {
            __syncthreads();                 // every lane is done reading the previous stage
            dst[0] = r0; dst[DS] = r1; dst[2 * DS] = r2; dst[3 * DS] = r3;
            dst[4 * DS] = r4; dst[5 * DS] = r5; dst[6 * DS] = r6; dst[7 * DS] = r7;
            __syncthreads();
            // the next stage's loads in flight during this stage's compressions (the last stage
            // reloads its own data: a uniform, in-bounds no-op)
            const uint4* nx = src + (st + 1 < STAGES ? st + 1 : st) * 8;
            r0 = nx[0]; r1 = nx[LS]; r2 = nx[2 * LS]; r3 = nx[3 * LS];
            r4 = nx[4 * LS]; r5 = nx[5 * LS]; r6 = nx[6 * LS]; r7 = nx[7 * LS];
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                uint32_t m[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint4 u = stg[tid * STG_ROW4 + b * 4 + q];
                    m[4 * q] = u.x;
                    m[4 * q + 1] = u.y;
                    m[4 * q + 2] = u.z;
                    m[4 * q + 3] = u.w;
                }
                const int blk = st * 2 + b;
                b2s_compress(h, m, (uint32_t)(blk + 1) * 64u, blk == 2 * STAGES - 1, false);
            }
        }
        __syncthreads();                     // staging reads done before it holds digests
#pragma unroll
        for (int i = 0; i < 8; ++i) dig[tid * 8 + i] = h[i];
    } else if (j < nleaf) {
        const uint32_t* src = x + (long long)blockIdx.y * stride + lo + j * LEAF_WORDS;
        const long long rem = hi - lo - j * LEAF_WORDS;
        const int nw = rem < LEAF_WORDS ? (int)rem : LEAF_WORDS;
        uint32_t h[8];
        b2s_init(h, (uint32_t)j, 0u);
        b2s_words(h, nw, false, [&](int b, uint32_t* m) {
            const int w0 = b * 16;
            if (ALIGNED && w0 + 16 <= nw) {
                const uint4* s4 = reinterpret_cast<const uint4*>(src + w0);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint4 u = s4[q];
                    m[4 * q] = u.x;
                    m[4 * q + 1] = u.y;
                    m[4 * q + 2] = u.z;
                    m[4 * q + 3] = u.w;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 16; ++q) m[q] = w0 + q < nw ? src[w0 + q] : 0u;
            }
        });
#pragma unroll
        for (int i = 0; i < 8; ++i) dig[tid * 8 + i] = h[i];
    }
    __syncthreads();
    if (tid < 256 / FANOUT) {
        const long long q = (long long)blockIdx.x * (256 / FANOUT) + tid;
        const long long rem = nleaf - q * FANOUT;
        if (rem > 0) {
            const int nch = rem < FANOUT ? (int)rem : FANOUT;
            const uint32_t* src = dig + tid * FANOUT * 8;
            uint32_t h[8];
            b2s_init(h, (uint32_t)q, 1u);
            b2s_words(h, nch * 8, false, [&](int b, uint32_t* m) {
                const int w0 = b * 16;
#pragma unroll
                for (int i = 0; i < 16; ++i) m[i] = w0 + i < nch * 8 ? src[w0 + i] : 0u;
            });
            uint32_t* o = out + (long long)blockIdx.y * out_stride + q * 8;
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = h[i];
        }
    }
}

constexpr int TOP_MAX = 1024;   // level-(d0+1) digests the top kernel keeps in LDS (32 KiB)

// the rest of a segment's tree in ONE workgroup per batch entry: in[y] holds n_in >= 1 digests of
// level d0 - 1; levels d0, d0 + 1, ... until one digest remains (levels >= d0 + 1 live in LDS).
// root[y * root_stride] = the segment root; with `combine`, the tree's final node over this single
// segment's root (node_depth 255, last_node) instead.  n_in <= FANOUT * TOP_MAX.
__global__ __launch_bounds__(256) void b2s_top_kernel(const uint32_t* __restrict__ in, long long in_stride,
                                                     int n_in, int d0, int combine, uint32_t* __restrict__ root,
                                                     long long root_stride) {
    __shared__ uint32_t buf[2][TOP_MAX * 8];
    const uint32_t* src_g = in + (long long)blockIdx.y * in_stride;
    uint32_t* dst = root + (long long)blockIdx.y * root_stride;
    auto node = [&](const uint32_t* src, int n, long long q, uint32_t depth, uint32_t* o) {
        const long long rem = n - q * FANOUT;
        const int nch = rem < FANOUT ? (int)rem : FANOUT;
        const uint32_t* c = src + q * FANOUT * 8;
        uint32_t h[8];
        b2s_init(h, (uint32_t)q, depth);
        b2s_words(h, nch * 8, false, [&](int b, uint32_t* m) {
            const int w0 = b * 16;
#pragma unroll
            for (int i = 0; i < 16; ++i) m[i] = w0 + i < nch * 8 ? c[w0 + i] : 0u;
        });
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = h[i];
    };
    int n = n_in;
    const uint32_t* cur = src_g;
    int which = 0;
    uint32_t depth = (uint32_t)d0;
    if (n > 1) {
        while (true) {
            const int n_out = (n + FANOUT - 1) / FANOUT;
            for (int q = threadIdx.x; q < n_out; q += 256) node(cur, n, q, depth, buf[which] + q * 8);
            __syncthreads();
            cur = buf[which];
            which ^= 1;
            n = n_out;
            ++depth;
            if (n == 1) break;
        }
    }
    if (threadIdx.x == 0) {
        uint32_t r[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = cur[i];
        if (combine) {
            uint32_t h[8];
            b2s_init(h, 0u, 255u);
            b2s_words(h, 8, true, [&](int, uint32_t* m) {
#pragma unroll
                for (int i = 0; i < 8; ++i) m[i] = r[i];
#pragma unroll
                for (int i = 8; i < 16; ++i) m[i] = 0u;
            });
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = h[i];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) dst[i] = r[i];
    }
}

// internal nodes: out[y][j] = node j over children [F j, F j + F) of in[y] (n_in digests)
__global__ __launch_bounds__(256) void b2s_node_kernel(const uint32_t* __restrict__ in, long long in_stride,
                                                      long long n_in, int fan, uint32_t depth, int last_node,
                                                      uint32_t* __restrict__ out, long long out_stride,
                                                      long long n_out) {
    const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
    if (j >= n_out) return;
    const uint32_t* src = in + (long long)blockIdx.y * in_stride + j * fan * 8;
    const long long rem = n_in - j * fan;
    const int nch = rem < fan ? (int)rem : fan;
    uint32_t h[8];
    b2s_init(h, (uint32_t)j, depth);
    b2s_words(h, nch * 8, last_node != 0, [&](int b, uint32_t* m) {
        const int w0 = b * 16;
        const int nw = nch * 8;
        if (w0 + 16 <= nw) {
            const uint4* s4 = reinterpret_cast<const uint4*>(src + w0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 u = s4[q];
                m[4 * q] = u.x;
                m[4 * q + 1] = u.y;
                m[4 * q + 2] = u.z;
                m[4 * q + 3] = u.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) m[q] = w0 + q < nw ? src[w0 + q] : 0u;
        }
    });
    uint32_t* o = out + (long long)blockIdx.y * out_stride + j * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = h[i];
}

// ============================================================================ keyed sketch
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x6c8e9cf5u;
    x ^= x >> 16;
    return x;
}

constexpr int HB = 256;

// part[y][block][k] = sum over this block's j of s_k(key, j) * (a[y][j] - b[j])   (b nullable)
__global__ __launch_bounds__(HB) void keyed_sketch_partial_kernel(const float* __restrict__ a, long long stride,
                                                                 const float* __restrict__ b, long long lo,
                                                                 long long hi, uint32_t k0, uint32_t k1,
                                                                 float* __restrict__ part) {
    __shared__ float red[HB / 64][4];
    a += (long long)blockIdx.y * stride;
    part += (long long)blockIdx.y * gridDim.x * 4;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    const long long step = (long long)gridDim.x * HB;
    for (long long j = lo + (long long)blockIdx.x * HB + threadIdx.x; j < hi; j += step) {
        const float v = b != nullptr ? a[j] - b[j] : a[j];
        const uint32_t h = mix32(mix32((uint32_t)j ^ k0) ^ k1);
#pragma unroll
        for (int k = 0; k < 4; ++k) s[k] += (h >> (28 + k)) & 1u ? -v : v;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = wave_sum(s[k]);
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) red[threadIdx.x >> 6][k] = s[k];
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < HB / 64; ++i) t += red[i][threadIdx.x];
        part[blockIdx.x * 4 + threadIdx.x] = t;
    }
}

// out[y][k] (+)= sum over blocks of part[y][.][k], in block order (one wave per k, one block per y)
__global__ __launch_bounds__(256) void keyed_sketch_final_kernel(const float* __restrict__ part, int nb,
                                                                float* __restrict__ out, int accumulate) {
    const int k = threadIdx.x >> 6, lane = threadIdx.x & 63;
    part += (long long)blockIdx.x * nb * 4;
    out += blockIdx.x * 4;
    float t = 0.f;
    for (int i = lane; i < nb; i += 64) t += part[i * 4 + k];
    t = wave_sum(t);
    if (lane == 0) out[k] = accumulate ? out[k] + t : t;
}

int grid_for(long long n, int cap) {
    const long long b = (n + HB * 8 - 1) / (HB * 8);   // ~8 elements per thread
    return (int)(b < 1 ? 1 : b > cap ? cap : b);
}

// ============================================================================ contribution snapshot
// c = g - prev ; prev = g   (fp32, elementwise; the subtraction the CPU path does in torch)
__global__ __launch_bounds__(256) void contrib_snap_kernel(const float* __restrict__ g, float* __restrict__ prev,
                                                          float* __restrict__ c, long long n) {
    const long long step = (long long)gridDim.x * 256;
    for (long long j = (long long)blockIdx.x * 256 + threadIdx.x; j < n; j += step) {
        const float v = g[j];
        c[j] = v - prev[j];
        prev[j] = v;
    }
}

// out[0] = max |a - b|, out[1] = max |b| over [lo, hi) (fp32 bits of non-negative values compare as
// unsigned integers; a NaN's bits exceed +inf's, so a NaN anywhere reads as the largest error).
// out must be zeroed by the caller.  No temporaries (the torch form allocated two n-sized ones).
__global__ __launch_bounds__(256) void absdiff_max_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         long long lo, long long hi, unsigned int* __restrict__ out) {
    float d = 0.f, r = 0.f;
    const long long step = (long long)gridDim.x * 256;
    for (long long j = lo + (long long)blockIdx.x * 256 + threadIdx.x; j < hi; j += step) {
        const float x = a[j], y = b[j];
        const float e = fabsf(x - y), m = fabsf(y);
        d = (e > d || e != e) ? e : d;
        r = (m > r || m != m) ? m : r;
    }
    unsigned int ud = __float_as_uint(d), ur = __float_as_uint(r);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        ud = max(ud, (unsigned int)__shfl_xor((int)ud, o, 64));
        ur = max(ur, (unsigned int)__shfl_xor((int)ur, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(out, ud);
        atomicMax(out + 1, ur);
    }
}

}  // namespace

// out (uint32[2], zeroed) = bits of (max |a - b|, max |b|) over [lo, hi)
TDL_API int tdl_absdiff_max(const float* a, const float* b, long long lo, long long hi, unsigned int* out,
                            hipStream_t s) {
    if (hi <= lo) return 0;
    long long nb = (hi - lo + 256 * 8 - 1) / (256 * 8);
    if (nb > 2048) nb = 2048;
    absdiff_max_kernel<<<(int)nb, 256, 0, s>>>(a, b, lo, hi, out);
    TDL_LAUNCH_CHECK();
}

// ---- BLAKE2s Merkle levels (the Python side walks the tree: grad_audit.merkle_roots)
TDL_API long long tdl_b2s_leaf_words() { return LEAF_WORDS; }
TDL_API long long tdl_b2s_fanout() { return FANOUT; }

// out[y][0..ceil(nleaf / 32)) = level-1 nodes of x[y * stride + lo : ... + hi), y < batch
TDL_API int tdl_b2s_leaves_l1(const void* x, long long stride, int batch, long long lo, long long hi, void* out,
                              long long out_stride, hipStream_t s) {
    if (hi <= lo || batch <= 0) return 0;
    const long long nleaf = (hi - lo + LEAF_WORDS - 1) / LEAF_WORDS;
    const dim3 grid((unsigned)((nleaf + 255) / 256), (unsigned)batch);
    const bool aligned = ((reinterpret_cast<uintptr_t>(x) & 15) == 0) && ((lo & 3) == 0) && ((stride & 3) == 0);
    if (aligned)
        b2s_leaf_l1_kernel<true><<<grid, 256, 0, s>>>((const uint32_t*)x, stride, lo, hi, nleaf, (uint32_t*)out,
                                                      out_stride);
    else
        b2s_leaf_l1_kernel<false><<<grid, 256, 0, s>>>((const uint32_t*)x, stride, lo, hi, nleaf, (uint32_t*)out,
                                                       out_stride);
    TDL_LAUNCH_CHECK();
}

TDL_API long long tdl_b2s_top_max_in() { return (long long)FANOUT * TOP_MAX; }

// root[y] = the rest of the tree over in[y][0..n_in) (level d0 - 1 digests); combine: the final node too
TDL_API int tdl_b2s_top(const void* in, long long in_stride, int n_in, int batch, int d0, int combine, void* root,
                        long long root_stride, hipStream_t s) {
    if (n_in <= 0 || batch <= 0 || n_in > FANOUT * TOP_MAX) return (int)hipErrorInvalidValue;
    b2s_top_kernel<<<dim3(1, (unsigned)batch), 256, 0, s>>>((const uint32_t*)in, in_stride, n_in, d0, combine,
                                                           (uint32_t*)root, root_stride);
    TDL_LAUNCH_CHECK();
}

// out[y][0..n_out) = nodes over in[y][0..n_in), fan children each (in / out strides in uint32 words)
TDL_API int tdl_b2s_nodes(const void* in, long long in_stride, long long n_in, int batch, int fan, int depth,
                          int last_node, void* out, long long out_stride, hipStream_t s) {
    if (n_in <= 0 || batch <= 0) return 0;
    const long long n_out = (n_in + fan - 1) / fan;
    const dim3 grid((unsigned)((n_out + 255) / 256), (unsigned)batch);
    b2s_node_kernel<<<grid, 256, 0, s>>>((const uint32_t*)in, in_stride, n_in, fan, (uint32_t)depth, last_node,
                                         (uint32_t*)out, out_stride, n_out);
    TDL_LAUNCH_CHECK();
}

// number of partial rows the keyed sketch uses per batch entry (workspace: 4 floats each)
TDL_API long long tdl_keyed_sketch_ws_floats(long long n) { return 4LL * grid_for(n, 1024); }

// out[y][0..3] (+)= keyed sketch of (a[y] - b)[lo:hi) (b nullable) under key (k0, k1), y < batch;
// ws >= batch * ws_floats(hi - lo)
TDL_API int tdl_keyed_sketch(const float* a, long long stride, int batch, const float* b, long long lo, long long hi,
                             unsigned int k0, unsigned int k1, float* ws, float* out, int accumulate, hipStream_t s) {
    if (batch <= 0) return 0;
    if (hi <= lo) {
        if (!accumulate) hipMemsetAsync(out, 0, 4 * sizeof(float) * batch, s);
        TDL_LAUNCH_CHECK();
    }
    const int nb = grid_for(hi - lo, 1024);
    keyed_sketch_partial_kernel<<<dim3(nb, batch), HB, 0, s>>>(a, stride, b, lo, hi, k0, k1, ws);
    keyed_sketch_final_kernel<<<batch, 256, 0, s>>>(ws, nb, out, accumulate);
    TDL_LAUNCH_CHECK();
}

// c = g - prev; prev = g  (n fp32)
TDL_API int tdl_contrib_snap(const float* g, float* prev, float* c, long long n, hipStream_t s) {
    if (n <= 0) return 0;
    long long nb = (n + 256 * 8 - 1) / (256 * 8);
    if (nb > 4096) nb = 4096;
    contrib_snap_kernel<<<(int)nb, 256, 0, s>>>(g, prev, c, n);
    TDL_LAUNCH_CHECK();
}
