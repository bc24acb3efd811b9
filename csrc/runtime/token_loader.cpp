// Native token-window data loader (the data layer of SURVEY §1 L2 / phantom get_dataloader).
//
// Language-model batches are windows of T+1 tokens cut from a memory-mapped token corpus (raw
// uint16 or uint32 little-endian ids, e.g. a GPT-2-tokenised OpenWebText dump) or, without a
// corpus, synthetic ids from a counter-based hash.  Worker threads fill a ring of caller-owned
// (pinned) int64 slots ahead of the training loop; batch k is a pure function of (seed, rank, k),
// so the stream is identical whatever the thread count and the consumer sees batches in order.
//
//   h = tdl_loader_create(path|NULL, token_bytes, vocab, B, T, seed, slots, threads, rank, world)
//   tdl_loader_bind_slot(h, s, input[B*T], target[B*T])    for every slot, then tdl_loader_start(h)
//   s = tdl_loader_next(h, &k)      blocks until batch k (the next in order) is ready in slot s
//   tdl_loader_release(h, s)        slot s may be refilled (caller: after its H2D copy completed)
//   tdl_loader_destroy(h)
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#define TDL_API extern "C" __attribute__((visibility("default")))

namespace {

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

enum SlotState { FREE = 0, FILLING = 1, READY = 2, IN_USE = 3 };

struct Slot {
    int64_t* input = nullptr;
    int64_t* target = nullptr;
    int64_t batch = -1;
    SlotState state = FREE;
};

struct Loader {
    // corpus
    const uint8_t* map = nullptr;
    size_t map_bytes = 0;
    int token_bytes = 2;
    int64_t ntok = 0;
    // shape / stream
    int64_t vocab = 50257;
    int B = 1, T = 1;
    uint64_t seed = 0;
    int rank = 0, world = 1;
    std::vector<Slot> slots;
    // scheduling
    std::mutex mu;
    std::condition_variable cv_work, cv_ready;
    int64_t next_to_fill = 0;     // batch index the next worker claims
    int64_t next_to_serve = 0;    // batch index the consumer gets next
    bool stop = false;
    bool started = false;
    std::vector<std::thread> threads;
    int nthreads = 1;

    int64_t token_at(int64_t i) const {
        if (token_bytes == 2) {
            uint16_t v;
            std::memcpy(&v, map + (size_t)i * 2, 2);
            return v;
        }
        uint32_t v;
        std::memcpy(&v, map + (size_t)i * 4, 4);
        return v;
    }

    void fill(Slot& s, int64_t k) {
        // the global batch index interleaves ranks so data-parallel replicas read disjoint batches
        const uint64_t gk = (uint64_t)k * (uint64_t)world + (uint64_t)rank;
        for (int b = 0; b < B; ++b) {
            const uint64_t h = splitmix64(seed ^ splitmix64(gk * 1315423911ull + (uint64_t)b));
            int64_t* in = s.input + (size_t)b * T;
            int64_t* tg = s.target + (size_t)b * T;
            if (map) {
                const int64_t span = ntok - T - 1;
                const int64_t start = span > 0 ? (int64_t)(h % (uint64_t)span) : 0;
                int64_t prev = token_at(start);
                for (int t = 0; t < T; ++t) {
                    const int64_t nxt = token_at(start + t + 1);
                    in[t] = prev;
                    tg[t] = nxt;
                    prev = nxt;
                }
            } else {
                uint64_t st = h;
                int64_t prev = (int64_t)(splitmix64(st) % (uint64_t)vocab);
                for (int t = 0; t < T; ++t) {
                    st += 0x9E3779B97F4A7C15ull;
                    const int64_t nxt = (int64_t)(splitmix64(st) % (uint64_t)vocab);
                    in[t] = prev;
                    tg[t] = nxt;
                    prev = nxt;
                }
            }
        }
    }

    void worker() {
        for (;;) {
            int si = -1;
            int64_t k = -1;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_work.wait(lk, [&] {
                    if (stop) return true;
                    // claim a free slot only for a batch within the ring window of the consumer
                    if (next_to_fill >= next_to_serve + (int64_t)slots.size()) return false;
                    for (auto& s : slots)
                        if (s.state == FREE) return true;
                    return false;
                });
                if (stop) return;
                for (size_t i = 0; i < slots.size(); ++i)
                    if (slots[i].state == FREE) {
                        si = (int)i;
                        break;
                    }
                k = next_to_fill++;
                slots[si].state = FILLING;
                slots[si].batch = k;
            }
            fill(slots[si], k);
            {
                std::lock_guard<std::mutex> lk(mu);
                slots[si].state = READY;
            }
            cv_ready.notify_all();
        }
    }
};

}  // namespace

TDL_API void* tdl_loader_create(const char* path, int token_bytes, int64_t vocab, int batch, int seq_len, uint64_t seed,
                                int num_slots, int num_threads, int rank, int world) {
    if (batch <= 0 || seq_len <= 0 || num_slots < 2 || (token_bytes != 2 && token_bytes != 4)) return nullptr;
    auto* L = new Loader();
    L->token_bytes = token_bytes;
    L->vocab = vocab > 0 ? vocab : 50257;
    L->B = batch;
    L->T = seq_len;
    L->seed = seed;
    L->rank = rank;
    L->world = world > 0 ? world : 1;
    L->slots.resize(num_slots);
    L->nthreads = num_threads > 0 ? num_threads : 1;
    if (path && path[0]) {
        const int fd = open(path, O_RDONLY);
        if (fd < 0) {
            delete L;
            return nullptr;
        }
        struct stat st;
        if (fstat(fd, &st) != 0 || st.st_size < (off_t)((seq_len + 2) * token_bytes)) {
            close(fd);
            delete L;
            return nullptr;
        }
        void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE | MAP_NORESERVE, fd, 0);
        close(fd);
        if (p == MAP_FAILED) {
            delete L;
            return nullptr;
        }
        madvise(p, (size_t)st.st_size, MADV_RANDOM);
        L->map = (const uint8_t*)p;
        L->map_bytes = (size_t)st.st_size;
        L->ntok = (int64_t)(st.st_size / token_bytes);
    }
    return L;
}

TDL_API int tdl_loader_bind_slot(void* h, int slot, int64_t* input, int64_t* target) {
    auto* L = (Loader*)h;
    if (!L || L->started || slot < 0 || slot >= (int)L->slots.size() || !input || !target) return 1;
    L->slots[slot].input = input;
    L->slots[slot].target = target;
    return 0;
}

TDL_API int tdl_loader_start(void* h) {
    auto* L = (Loader*)h;
    if (!L || L->started) return 1;
    for (auto& s : L->slots)
        if (!s.input || !s.target) return 2;
    L->started = true;
    for (int i = 0; i < L->nthreads; ++i) L->threads.emplace_back([L] { L->worker(); });
    return 0;
}

// Returns the slot holding the next batch in order (blocking); *batch_index receives its index.
TDL_API int tdl_loader_next(void* h, int64_t* batch_index) {
    auto* L = (Loader*)h;
    if (!L || !L->started) return -1;
    std::unique_lock<std::mutex> lk(L->mu);
    const int64_t want = L->next_to_serve;
    int found = -1;
    L->cv_ready.wait(lk, [&] {
        for (size_t i = 0; i < L->slots.size(); ++i)
            if (L->slots[i].state == READY && L->slots[i].batch == want) {
                found = (int)i;
                return true;
            }
        return L->stop;
    });
    if (found < 0) return -1;
    L->slots[found].state = IN_USE;
    L->next_to_serve++;
    if (batch_index) *batch_index = want;
    lk.unlock();
    L->cv_work.notify_all();
    return found;
}

TDL_API int tdl_loader_release(void* h, int slot) {
    auto* L = (Loader*)h;
    if (!L || slot < 0 || slot >= (int)L->slots.size()) return 1;
    {
        std::lock_guard<std::mutex> lk(L->mu);
        if (L->slots[slot].state != IN_USE) return 2;
        L->slots[slot].state = FREE;
        L->slots[slot].batch = -1;
    }
    L->cv_work.notify_all();
    return 0;
}

TDL_API int64_t tdl_loader_num_tokens(void* h) {
    auto* L = (Loader*)h;
    return L ? L->ntok : 0;
}

TDL_API void tdl_loader_destroy(void* h) {
    auto* L = (Loader*)h;
    if (!L) return;
    {
        std::lock_guard<std::mutex> lk(L->mu);
        L->stop = true;
    }
    L->cv_work.notify_all();
    L->cv_ready.notify_all();
    for (auto& t : L->threads) t.join();
    if (L->map) munmap((void*)L->map, L->map_bytes);
    delete L;
}
