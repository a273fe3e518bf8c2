// host_mem.cpp — registry of page-locked host ranges (decds_host_register / decds_host_alloc),
// the host thread pool for staging copies, and the pinned bounce rings (host_mem.h).
#include "host_mem.h"
#include "hip_status.h"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/decds_rlnc.h"
#include "capi_internal.h"

namespace decds {

namespace {

// ---- registry ---------------------------------------------------------------------------------
// A range stays page-locked while it has a registration (regs) or an in-flight use (uses); the last
// of the two to drop it unlocks it. Ranges never overlap (a partial overlap is refused: locking the
// same pages twice and unlocking one of them is exactly the hazard this replaces).
struct Entry {
    size_t len;
    int regs;
    int uses;
    bool alloc;  // from decds_host_alloc (host_pinned_alloc): freed, not unregistered
};
std::mutex g_reg_mu;
std::map<uintptr_t, Entry> g_reg;

// caller holds g_reg_mu
void finalize_if_idle(std::map<uintptr_t, Entry>::iterator it) {
    if (it->second.regs > 0 || it->second.uses > 0) return;
    void *p = reinterpret_cast<void *>(it->first);
    if (it->second.alloc)
        host_pinned_free(p, it->second.len);
    else
        hip_tolerate(hipHostUnregister(p), "hipHostUnregister");
    g_reg.erase(it);
}

// entry whose range contains [p, p+n), or end()
std::map<uintptr_t, Entry>::iterator find_containing(uintptr_t p, size_t n) {
    auto it = g_reg.upper_bound(p);
    if (it == g_reg.begin()) return g_reg.end();
    --it;
    if (p + n <= it->first + it->second.len) return it;
    return g_reg.end();
}

bool overlaps(uintptr_t p, size_t n) {
    auto it = g_reg.upper_bound(p);
    if (it != g_reg.end() && it->first < p + n) return true;
    if (it != g_reg.begin()) {
        --it;
        if (it->first + it->second.len > p) return true;
    }
    return false;
}

// ---- host pool --------------------------------------------------------------------------------
class Pool {
   public:
    static Pool &get() {
        static Pool p;
        return p;
    }
    void run(size_t n, const std::function<void(size_t)> &fn) {
        if (n == 0) return;
        if (n == 1 || workers_.empty()) {
            for (size_t i = 0; i < n; i++) fn(i);
            return;
        }
        Job job{&fn, n};
        {
            std::lock_guard<std::mutex> g(mu_);
            jobs_.push_back(&job);
        }
        cv_.notify_all();
        work(job);
        std::unique_lock<std::mutex> g(mu_);
        auto it = std::find(jobs_.begin(), jobs_.end(), &job);
        if (it != jobs_.end()) jobs_.erase(it);
        done_cv_.wait(g, [&] { return job.finished.load() == n && job.attached == 0; });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : workers_) t.join();
    }

   private:
    struct Job {
        const std::function<void(size_t)> *fn;
        size_t n;
        std::atomic<size_t> next{0};
        std::atomic<size_t> finished{0};
        int attached = 0;  // workers holding a pointer to the job (under mu_)
    };
    Pool() {
        unsigned t = std::thread::hardware_concurrency();
        t = t ? std::min(8u, t) : 4u;
        if (const char *e = std::getenv("DECDS_HOST_THREADS")) t = (unsigned)std::max(1, std::atoi(e));
        for (unsigned i = 1; i < t; i++) workers_.emplace_back([this] { loop(); });
    }
    void work(Job &j) {
        for (size_t i; (i = j.next.fetch_add(1)) < j.n;) {
            (*j.fn)(i);
            j.finished.fetch_add(1);
        }
    }
    void loop() {
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || !jobs_.empty(); });
            if (stop_) return;
            Job *j = jobs_.front();
            if (j->next.load() >= j->n) {  // fully handed out: drop it from the queue
                jobs_.pop_front();
                continue;
            }
            j->attached++;
            g.unlock();
            work(*j);
            g.lock();
            j->attached--;
            done_cv_.notify_all();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<Job *> jobs_;
    bool stop_ = false;
};

}  // namespace

HostUse::HostUse(const void *p, size_t n) {
    if (!p || !n) return;
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = find_containing(reinterpret_cast<uintptr_t>(p), n);
    if (it == g_reg.end() || it->second.regs == 0) return;
    it->second.uses++;
    key_ = it->first;
}

HostUse::~HostUse() {
    if (!key_) return;
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg.find(key_);
    if (it == g_reg.end()) return;
    it->second.uses--;
    finalize_if_idle(it);
}

// ---- page-locked block cache ---------------------------------------------------------------------
// Page-locking costs ~0.25 s per GiB on the GPU box (hipHostMalloc of a Blob's 1.6 GiB coded store
// 0.08-0.16 s, its hipHostFree 0.07 s): blocks of at least CACHE_MIN bytes are kept on free, up to
// DECDS_PINNED_CACHE_MB in total (default 8 GiB: a 4 GiB Blob's coded store is 6.4 GiB, the largest
// size of the reference's build_blob bench), and handed out again for requests of 80-100 % of
// their size. decds_host_cache_trim() returns them to the system; so does destroying the process's
// last context (capi.cpp), so an idle process holds no cached page-locked memory.
namespace {
constexpr size_t CACHE_MIN = (size_t)64 << 20;
std::mutex g_cache_mu;
std::multimap<size_t, void *> g_cache;  // free blocks by size
std::deque<void *> g_order;             // the same blocks, longest cached first
std::map<void *, size_t> g_block;       // every block >= CACHE_MIN, live or cached -> its size
size_t g_cached = 0;
size_t cache_cap() {
    static const size_t cap = [] {
        const char *v = std::getenv("DECDS_PINNED_CACHE_MB");
        return v ? (size_t)std::strtoull(v, nullptr, 10) << 20 : (size_t)8 << 30;
    }();
    return cap;
}
}  // namespace

hipError_t host_pinned_alloc(size_t n, void **out) {
    *out = nullptr;
    if (n >= CACHE_MIN) {
        std::lock_guard<std::mutex> g(g_cache_mu);
        auto it = g_cache.lower_bound(n);
        if (it != g_cache.end() && it->first - n <= it->first / 5) {
            *out = it->second;
            g_cached -= it->first;
            g_cache.erase(it);
            g_order.erase(std::find(g_order.begin(), g_order.end(), *out));
            return hipSuccess;
        }
    }
    hipError_t e = hipHostMalloc(out, n ? n : 1, DECDS_HOST_MALLOC_FLAGS);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // this call's own error, returned
        return e;
    }
    if (n >= CACHE_MIN) {
        std::lock_guard<std::mutex> g(g_cache_mu);
        g_block[*out] = n;
    }
    return e;
}

void host_pinned_free(void *p, size_t) {
    if (!p) return;
    std::vector<void *> evicted;
    {
        std::lock_guard<std::mutex> g(g_cache_mu);
        auto b = g_block.find(p);
        if (b != g_block.end()) {
            if (b->second <= cache_cap()) {
                // the block just freed is the likeliest to be asked for again (the next Blob of the same
                // size): blocks cached longest are released to make room for it (a 4 GiB Blob's 6.4 GiB
                // store behind a 1 GiB one's 1.6 GiB was refused by the cap and page-locked anew per call:
                // Blob::new at 4 GiB 0.66 s, r09e)
                while (g_cached + b->second > cache_cap() && !g_order.empty()) {
                    void *old = g_order.front();
                    g_order.pop_front();
                    for (auto it = g_cache.begin(); it != g_cache.end(); ++it)
                        if (it->second == old) {
                            g_cached -= it->first;
                            g_cache.erase(it);
                            break;
                        }
                    g_block.erase(old);
                    evicted.push_back(old);
                }
                g_cache.emplace(b->second, p);
                g_order.push_back(p);
                g_cached += b->second;
                p = nullptr;
            } else {
                g_block.erase(b);
            }
        }
    }
    for (void *q : evicted) hip_tolerate(hipHostFree(q), "hipHostFree");
    if (p) hip_tolerate(hipHostFree(p), "hipHostFree");
}

size_t host_cache_trim() {
    std::lock_guard<std::mutex> g(g_cache_mu);
    const size_t freed = g_cached;
    for (auto &kv : g_cache) {
        g_block.erase(kv.second);
        hip_tolerate(hipHostFree(kv.second), "hipHostFree");
    }
    g_cache.clear();
    g_order.clear();
    g_cached = 0;
    return freed;
}

void host_parallel(size_t n, const std::function<void(size_t)> &fn) { Pool::get().run(n, fn); }

void par_memcpy(void *dst, const void *src, size_t n) {
    constexpr size_t PART = (size_t)2 << 20;
    if (n < 2 * PART) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t parts = std::min<size_t>(16, n / PART);
    const size_t step = (n / parts + 63) & ~(size_t)63;
    host_parallel(parts, [&](size_t i) {
        const size_t lo = i * step;
        if (lo >= n) return;
        std::memcpy(static_cast<uint8_t *>(dst) + lo, static_cast<const uint8_t *>(src) + lo, std::min(step, n - lo));
    });
}

// ---- bounce rings -----------------------------------------------------------------------------
hipError_t BounceRing::init() {
    for (int i = 0; i < R; i++) {
        hipError_t e;
        if (!buf[i] && (e = host_pinned_alloc(PIECE, reinterpret_cast<void **>(&buf[i])))) return e;
        if (!ev[i] && (e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming))) return e;
    }
    return hipSuccess;
}

hipError_t BounceRing::settle(int i) {
    if (used[i]) {
        hipError_t e = hipEventSynchronize(ev[i]);
        if (e) return e;
        used[i] = false;
    }
    if (pend_dst[i]) {
        par_memcpy(pend_dst[i], buf[i], pend_len[i]);
        pend_dst[i] = nullptr;
    }
    return hipSuccess;
}

hipError_t BounceRing::h2d(uint8_t *ddst, const uint8_t *hsrc, size_t n, hipStream_t s) {
    hipError_t e;
    if ((e = init())) return e;
    for (size_t o = 0; o < n; o += PIECE) {
        const int i = next;
        next = (next + 1) % R;
        if ((e = settle(i))) return e;
        const size_t len = std::min(PIECE, n - o);
        par_memcpy(buf[i], hsrc + o, len);
        if ((e = hipMemcpyAsync(ddst + o, buf[i], len, hipMemcpyHostToDevice, s)) || (e = hipEventRecord(ev[i], s)))
            return e;
        used[i] = true;
    }
    return hipSuccess;
}

hipError_t BounceRing::stage(int *idx, uint8_t **piece) {
    hipError_t e;
    if ((e = init())) return e;
    const int i = next;
    next = (next + 1) % R;
    if ((e = settle(i))) return e;
    *idx = i;
    *piece = buf[i];
    return hipSuccess;
}

hipError_t BounceRing::commit(int i, uint8_t *ddst, size_t n, hipStream_t s) {
    hipError_t e;
    if (n > PIECE) return hipErrorInvalidValue;
    if ((e = hipMemcpyAsync(ddst, buf[i], n, hipMemcpyHostToDevice, s)) || (e = hipEventRecord(ev[i], s))) return e;
    used[i] = true;
    return hipSuccess;
}

hipError_t BounceRing::d2h(uint8_t *hdst, const uint8_t *dsrc, size_t n, hipStream_t s) {
    hipError_t e;
    if ((e = init())) return e;
    for (size_t o = 0; o < n; o += PIECE) {
        const int i = next;
        next = (next + 1) % R;
        if ((e = settle(i))) return e;
        const size_t len = std::min(PIECE, n - o);
        if ((e = hipMemcpyAsync(buf[i], dsrc + o, len, hipMemcpyDeviceToHost, s)) || (e = hipEventRecord(ev[i], s)))
            return e;
        used[i] = true;
        pend_dst[i] = hdst + o;
        pend_len[i] = len;
    }
    return hipSuccess;
}

hipError_t BounceRing::flush() {
    for (int k = 0; k < R; k++) {  // oldest piece first
        hipError_t e = settle((next + k) % R);
        if (e) return e;
    }
    return hipSuccess;
}

void BounceRing::abandon() {
    for (int i = 0; i < R; i++) {
        pend_dst[i] = nullptr;  // an abandoned call's copy-outs are dropped, never written late
        if (used[i]) hip_tolerate(hipEventSynchronize(ev[i]), "hipEventSynchronize");
        used[i] = false;
    }
}

void BounceRing::retire() {
    for (int i = 0; i < R; i++)
        if (!pend_dst[i]) used[i] = false;
}

BounceRing::~BounceRing() {
    abandon();
    for (int i = 0; i < R; i++) {
        if (ev[i]) hip_tolerate(hipEventDestroy(ev[i]), "hipEventDestroy");
        if (buf[i]) host_pinned_free(buf[i], PIECE);
    }
}

hipError_t copy_h2d(uint8_t *d, const uint8_t *h, size_t n, bool pinned, BounceRing &ring, hipStream_t s) {
    if (n == 0) return hipSuccess;
    return pinned ? hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s) : ring.h2d(d, h, n, s);
}

// Device -> page-locked host copies of more than a few tens of MB are split into D2H_PIECE pieces: one
// hipMemcpyAsync of 270 MB (a 16-chunkset batch of coded rows) ran at 30 GB/s on the box whatever the
// host memory (hipHostMalloc coherent or not, hipHostRegister'd), one of 16 MiB at 54 GB/s, and a
// kernel storing straight into the host buffer at 55 GB/s (tools/d2hbench.hip, r07j); a trace of the
// blob encode showed the large copy executed as 8 MiB blit kernels with gaps as long as the kernels
// between them (r07b). Pieces of 64 MiB (round 6): blob encode −1 % at 1 GiB and −3 % at 2 GiB against
// 16 MiB, repair unchanged (three interleaved pairs each, r09k). DECDS_D2H_PIECE_MB overrides the piece
// (0: one copy, round 4's behaviour).
static size_t d2h_piece() {
    static const size_t piece = [] {
        const char *v = std::getenv("DECDS_D2H_PIECE_MB");
        return v && *v ? (size_t)std::strtoull(v, nullptr, 10) << 20 : (size_t)64 << 20;
    }();
    return piece;
}

hipError_t d2h_pieces(uint8_t *h, const uint8_t *d, size_t n, hipStream_t s) {
    const size_t piece = d2h_piece();
    if (piece == 0 || n <= piece) return hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s);
    for (size_t o = 0; o < n; o += piece)
        if (hipError_t e = hipMemcpyAsync(h + o, d + o, std::min(piece, n - o), hipMemcpyDeviceToHost, s)) return e;
    return hipSuccess;
}

hipError_t copy_d2h(uint8_t *h, const uint8_t *d, size_t n, bool pinned, BounceRing &ring, hipStream_t s) {
    if (n == 0) return hipSuccess;
    return pinned ? d2h_pieces(h, d, n, s) : ring.d2h(h, d, n, s);
}

}  // namespace decds

using namespace decds;

extern "C" {

int decds_host_register(const void *ptr, size_t len) {
    if (!ptr || !len) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null or empty buffer");
    const uintptr_t p = reinterpret_cast<uintptr_t>(ptr);
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg.find(p);
    if (it != g_reg.end() && it->second.len == len && !it->second.alloc) {
        it->second.regs++;  // the same range again: one more registration to undo
        return DECDS_OK;
    }
    if (overlaps(p, len))
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT,
                               "range [%p, +%zu) overlaps a range already registered with this library", ptr, len);
    hipError_t e = hipHostRegister(const_cast<void *>(ptr), len, hipHostRegisterDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // the failed call's own error, reported below
        return decds_hip_error(e, "hipHostRegister");
    }
    g_reg.emplace(p, Entry{len, 1, 0, false});
    return DECDS_OK;
}

int decds_host_unregister(const void *ptr) {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == g_reg.end() || it->second.alloc || it->second.regs == 0)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "%p was not registered with decds_host_register", ptr);
    it->second.regs--;
    finalize_if_idle(it);  // deferred while a call still uses the range
    return DECDS_OK;
}

int decds_host_alloc(size_t len, void **out) {
    if (!out || !len) return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "null out pointer or empty size");
    *out = nullptr;
    void *p = nullptr;
    hipError_t e = host_pinned_alloc(len, &p);
    if (e != hipSuccess) return decds_hip_error(e, "page-locked allocation");
    std::lock_guard<std::mutex> g(g_reg_mu);
    g_reg.emplace(reinterpret_cast<uintptr_t>(p), Entry{len, 1, 0, true});
    *out = p;
    return DECDS_OK;
}

int decds_host_free(void *ptr) {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == g_reg.end() || !it->second.alloc || it->second.regs == 0)
        return decds_set_error(DECDS_ERR_INVALID_ARGUMENT, "%p was not allocated with decds_host_alloc", ptr);
    it->second.regs--;
    finalize_if_idle(it);
    return DECDS_OK;
}

size_t decds_host_cache_trim(void) { return host_cache_trim(); }

int decds_host_is_registered(const void *ptr, size_t len) {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = find_containing(reinterpret_cast<uintptr_t>(ptr), len ? len : 1);
    return it != g_reg.end() && it->second.regs > 0;
}

}  // extern "C"
