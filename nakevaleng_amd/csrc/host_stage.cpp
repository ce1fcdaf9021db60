// host_stage.cpp -- worker pool and pipelined pinned staging (host_stage.hpp).
#include "host_stage.hpp"

#include <string.h>

#include <algorithm>
#include <cstdlib>

namespace nkv {

int default_host_threads() {
    if (const char* e = std::getenv("NKV_HOST_THREADS")) {
        const int v = std::atoi(e);
        if (v >= 1) return std::min(v, 256);
    }
    const unsigned hw = std::thread::hardware_concurrency();
    // the GPU boxes give one GPU 16 cores; more threads only contend for DRAM
    return int(std::max(1u, std::min(hw ? hw : 1u, 16u)));
}

// ---------------------------------------------------------------------------
// HostPool

HostPool::~HostPool() { stop(); }

void HostPool::stop() {
    {
        std::lock_guard<std::mutex> g(m_);
        quit_ = true;
    }
    go_.notify_all();
    for (auto& t : workers_) t.join();
    workers_.clear();
    quit_ = false;
}

void HostPool::resize(int threads) {
    threads = std::max(1, threads);
    if (this->threads() == threads) return;
    stop();
    for (int i = 0; i + 1 < threads; ++i) workers_.emplace_back([this] { loop(); });
}

void HostPool::loop() {
    uint64_t seen = 0;
    for (;;) {
        const std::function<void(int)>* fn;
        int nj;
        {
            std::unique_lock<std::mutex> lk(m_);
            go_.wait(lk, [&] { return quit_ || gen_ != seen; });
            if (quit_) return;
            seen = gen_;
            fn = fn_;
            nj = njobs_;
        }
        for (int j = next_.fetch_add(1); j < nj; j = next_.fetch_add(1)) (*fn)(j);
        std::lock_guard<std::mutex> g(m_);
        if (--busy_ == 0) done_.notify_one();
    }
}

void HostPool::run(int njobs, const std::function<void(int)>& fn) {
    if (njobs <= 0) return;
    if (njobs == 1 || workers_.empty()) {
        for (int j = 0; j < njobs; ++j) fn(j);
        return;
    }
    {
        std::lock_guard<std::mutex> g(m_);
        fn_ = &fn;
        njobs_ = njobs;
        next_.store(0);
        busy_ = int(workers_.size());
        ++gen_;
    }
    go_.notify_all();
    for (int j = next_.fetch_add(1); j < njobs; j = next_.fetch_add(1)) fn(j);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return busy_ == 0; });
    fn_ = nullptr;
}

// ---------------------------------------------------------------------------
// Stager

Stager::~Stager() {
    (void)drain();
    release();
}

void Stager::release() {
    for (int k = 0; k < kStageSlots; ++k) {
        if (slot[k]) (void)hipHostFree(slot[k]);
        if (ev[k]) (void)hipEventDestroy(ev[k]);
        slot[k] = nullptr;
        ev[k] = nullptr;
        pending[k] = false;
    }
    slot_bytes = 0;
}

hipError_t Stager::wait_slot(int k) {
    if (!pending[k]) return hipSuccess;
    pending[k] = false;
    return hipEventSynchronize(ev[k]);
}

hipError_t Stager::drain() {
    hipError_t r = hipSuccess;
    for (int k = 0; k < kStageSlots; ++k) {
        const hipError_t e = wait_slot(k);
        if (r == hipSuccess) r = e;
    }
    return r;
}

hipError_t Stager::ready() {
    pool.resize(want_threads > 0 ? want_threads : default_host_threads());
    if (slot_bytes == chunk && slot[0]) return hipSuccess;
    hipError_t e = drain();
    if (e != hipSuccess) return e;
    release();
    for (int k = 0; k < kStageSlots; ++k) {
        e = hipHostMalloc(&slot[k], chunk, hipHostMallocDefault);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            release();
            return e;
        }
    }
    slot_bytes = chunk;
    return hipSuccess;
}

namespace {

// pieces of a chunk: at most one per thread, none smaller than min_piece
int pieces_of(uint64_t bytes, int threads, uint64_t chunk) {
    const uint64_t min_piece = std::max<uint64_t>(4096, std::min<uint64_t>(256 << 10, chunk / threads));
    return int(std::max<uint64_t>(1, std::min<uint64_t>(uint64_t(threads), bytes / min_piece)));
}

// copy packed bytes [a, b) of the segments into out (out[0] = packed byte a)
void gather(const Segments& s, uint64_t a, uint64_t b, uint8_t* out) {
    // last segment starting at or before a
    uint64_t i = uint64_t(std::upper_bound(s.dst, s.dst + s.n, a) - s.dst);
    i = i ? i - 1 : 0;
    for (; i < s.n && s.dst[i] < b; ++i) {
        const uint64_t lo = std::max(a, s.dst[i]);
        const uint64_t hi = std::min(b, s.dst[i] + s.len[i]);
        if (hi > lo) memcpy(out + (lo - a), s.src + s.off[i] + (lo - s.dst[i]), hi - lo);
    }
}

}  // namespace

hipError_t Stager::upload(const Segments& seg, uint64_t total, uint8_t* d_dst, hipStream_t s) {
    if (total == 0) return hipSuccess;
    hipError_t e = ready();
    if (e != hipSuccess) return e;
    const int T = pool.threads();
    uint64_t k = 0;
    for (uint64_t a = 0; a < total; a += chunk, ++k) {
        const int sl = int(k % kStageSlots);
        if ((e = wait_slot(sl)) != hipSuccess) return e;
        const uint64_t b = std::min<uint64_t>(total, a + chunk);
        uint8_t* buf = static_cast<uint8_t*>(slot[sl]);
        const int np = pieces_of(b - a, T, chunk);
        pool.run(np, [&](int j) {
            const uint64_t pa = a + (b - a) * uint64_t(j) / uint64_t(np);
            const uint64_t pb = a + (b - a) * uint64_t(j + 1) / uint64_t(np);
            gather(seg, pa, pb, buf + (pa - a));
        });
        if ((e = hipMemcpyAsync(d_dst + a, buf, b - a, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
        if ((e = hipEventRecord(ev[sl], s)) != hipSuccess) return e;
        pending[sl] = true;
    }
    return hipSuccess;
}

hipError_t Stager::upload(const uint8_t* src, uint64_t bytes, uint8_t* d_dst, hipStream_t s) {
    const uint64_t zero = 0;
    const Segments seg{src, &zero, &bytes, &zero, 1};
    return upload(seg, bytes, d_dst, s);
}

hipError_t Stager::download(uint8_t* h_dst, const uint8_t* d_src, uint64_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    hipError_t e = ready();
    if (e != hipSuccess) return e;
    const int T = pool.threads();
    const uint64_t nch = (bytes + chunk - 1) / chunk;
    auto issue = [&](uint64_t k) -> hipError_t {
        const int sl = int(k % kStageSlots);
        hipError_t r = wait_slot(sl);
        if (r != hipSuccess) return r;
        const uint64_t a = k * chunk, b = std::min<uint64_t>(bytes, a + chunk);
        if ((r = hipMemcpyAsync(slot[sl], d_src + a, b - a, hipMemcpyDeviceToHost, s)) != hipSuccess) return r;
        if ((r = hipEventRecord(ev[sl], s)) != hipSuccess) return r;
        pending[sl] = true;
        return hipSuccess;
    };
    for (uint64_t k = 0; k < std::min<uint64_t>(nch, kStageSlots); ++k)
        if ((e = issue(k)) != hipSuccess) return e;
    for (uint64_t k = 0; k < nch; ++k) {
        const int sl = int(k % kStageSlots);
        if ((e = wait_slot(sl)) != hipSuccess) return e;
        const uint64_t a = k * chunk, b = std::min<uint64_t>(bytes, a + chunk);
        const uint8_t* buf = static_cast<const uint8_t*>(slot[sl]);
        const int np = pieces_of(b - a, T, chunk);
        pool.run(np, [&](int j) {
            const uint64_t pa = (b - a) * uint64_t(j) / uint64_t(np);
            const uint64_t pb = (b - a) * uint64_t(j + 1) / uint64_t(np);
            memcpy(h_dst + a + pa, buf + pa, pb - pa);
        });
        if (k + kStageSlots < nch && (e = issue(k + kStageSlots)) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace nkv
