// Host (CPU) BLAKE2s Merkle commitments: the same tree as the gfx950 kernels of csrc/audit.hip
// (leaves of 256 32-bit words with node_offset = leaf index / node_depth 0, internal nodes over 32
// child digests with node_depth = level, one root per segment, a combine node over the segment
// roots with node_depth 255 + last_node).  Used by CPU ranks (gloo) and CPU tests; Python's
// hashlib.blake2s with the same node parameters is the oracle (tests/test_lying_rank.py), and the
// GPU test compares the kernels against this.  Leaves are hashed by a pool of std::threads.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t kIV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
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
constexpr long long kLeaf = 256;
constexpr long long kFan = 32;

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

inline void compress(uint32_t* h, const uint32_t* m, uint32_t t, bool last, bool last_node) {
    uint32_t v[16];
    for (int i = 0; i < 8; ++i) {
        v[i] = h[i];
        v[i + 8] = kIV[i];
    }
    v[12] ^= t;
    if (last) v[14] = ~v[14];
    if (last_node) v[15] = ~v[15];
    auto G = [&](int a, int b, int c, int d, uint32_t x, uint32_t y) {
        v[a] = v[a] + v[b] + x;
        v[d] = rotr(v[d] ^ v[a], 16);
        v[c] = v[c] + v[d];
        v[b] = rotr(v[b] ^ v[c], 12);
        v[a] = v[a] + v[b] + y;
        v[d] = rotr(v[d] ^ v[a], 8);
        v[c] = v[c] + v[d];
        v[b] = rotr(v[b] ^ v[c], 7);
    };
    for (int r = 0; r < 10; ++r) {
        const uint8_t* s = kSigma[r];
        G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

// BLAKE2s-256 (fanout 1, depth 1, unkeyed) of nw >= 0 little-endian words
void hash_words(const uint32_t* w, long long nw, uint32_t node_offset, uint32_t depth, bool last_node, uint32_t* out) {
    uint32_t h[8];
    for (int i = 0; i < 8; ++i) h[i] = kIV[i];
    h[0] ^= 32u | (1u << 16) | (1u << 24);
    h[2] ^= node_offset;
    h[3] ^= depth << 16;
    const long long nblk = nw > 0 ? (nw + 15) / 16 : 1;
    uint32_t m[16];
    for (long long b = 0; b < nblk; ++b) {
        const long long w0 = b * 16;
        const long long k = std::min<long long>(16, std::max<long long>(0, nw - w0));
        std::memset(m, 0, sizeof(m));
        if (k > 0) std::memcpy(m, w + w0, (size_t)k * 4);
        const bool last = b == nblk - 1;
        compress(h, m, last ? (uint32_t)(nw * 4) : (uint32_t)((b + 1) * 64), last, last_node);
    }
    std::memcpy(out, h, 32);
}

template <class F>
void parallel_for(long long n, int threads, F f) {
    if (threads <= 1 || n < 64) {
        for (long long i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> pool;
    const long long per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const long long lo = t * per, hi = std::min(n, lo + per);
        if (lo >= hi) break;
        pool.emplace_back([=] {
            for (long long i = lo; i < hi; ++i) f(i);
        });
    }
    for (auto& th : pool) th.join();
}

void segment_root(const uint32_t* x, long long nw, int threads, uint32_t* out) {
    long long n = (nw + kLeaf - 1) / kLeaf;
    if (n < 1) n = 1;
    std::vector<uint32_t> cur((size_t)n * 8), nxt;
    parallel_for(n, threads, [&](long long j) {
        const long long len = std::min(kLeaf, nw - j * kLeaf);
        hash_words(x + j * kLeaf, len < 0 ? 0 : len, (uint32_t)j, 0u, false, cur.data() + j * 8);
    });
    uint32_t depth = 1;
    while (true) {
        const long long n_out = (n + kFan - 1) / kFan;
        nxt.assign((size_t)n_out * 8, 0u);
        parallel_for(n_out, threads, [&](long long j) {
            const long long nch = std::min(kFan, n - j * kFan);
            hash_words(cur.data() + j * kFan * 8, nch * 8, (uint32_t)j, depth, false, nxt.data() + j * 8);
        });
        cur.swap(nxt);
        n = n_out;
        ++depth;
        if (n == 1) break;
    }
    std::memcpy(out, cur.data(), 32);
}

}  // namespace

// out[y][8] = Merkle root of x[y * stride + seg_lo[k] : y * stride + seg_hi[k]) over the nseg segments
extern "C" __attribute__((visibility("default"))) int tdl_host_merkle(const uint32_t* x, long long stride, int batch,
                                                                      const long long* seg_lo, const long long* seg_hi,
                                                                      int nseg, int threads, uint32_t* out) {
    if (threads < 1) threads = 1;
    std::vector<uint32_t> roots((size_t)std::max(nseg, 1) * 8);
    for (int y = 0; y < batch; ++y) {
        for (int k = 0; k < nseg; ++k)
            segment_root(x + (long long)y * stride + seg_lo[k], seg_hi[k] - seg_lo[k], threads, roots.data() + k * 8);
        hash_words(roots.data(), (long long)nseg * 8, 0u, 255u, true, out + (long long)y * 8);
    }
    return 0;
}
