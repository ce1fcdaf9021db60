// nkv_merkletree.hpp -- C++ mirror of the reference's ds/merkletree API over the
// C-ABI in nkv_merkle.h (header-only; link libnkvmerkle.so).
//
// The reference is Go; this header is the same shim a cgo package would be
// (INTEGRATION.md), written in C++ so it can be compiled and tested here.
// Names and behaviour follow magley/nakevaleng (paths relative to its root):
//
//   MerkleNode, MERKLE_NODE_EMPTY   ds/merkletree/merklenode.go:11-19
//   MerkleNode::String              merklenode.go:22-24
//   NewLeaf                         merklenode.go:27-34  -- deferred: the value's copy into
//                                   a pinned arena is handed to a pool of copy threads
//                                   and the value is hashed on the GPU by New() (or on
//                                   first Resolve()), batched with its neighbours.
//                                   Contract: a value handed to NewLeaf must not change
//                                   until New returns (both callers, sstable.go:61-63 and
//                                   lsmtree.go:211, pass values they never mutate)
//   MerkleNode::Serialize           merklenode.go:37-63
//   MerkleNode::Deserialize         merklenode.go:67-96  (returns true at EOF)
//   MerkleTree, New                 merkletree.go:13-25  ("cannot build Merkle Tree from 0 nodes")
//   MerkleTree::Serialize           merkletree.go:67-92  (O_WRONLY|O_CREAT, no O_TRUNC)
//   MerkleTree::Deserialize         merkletree.go:97-157 (root only, as the reference)
//   MerkleTree::Validate            merkletree.go:162-171 + merklenode.go:99-108
//   CompactRoots                    lsmtree.go:71-128,211 + sstable.go:35-47: the Merkle
//                                   step of several output tables, one thread per GPU
//
// Errors the reference panics on are thrown as std::runtime_error.  There is
// no CPU hashing path: without a HIP device every hashing call throws.
#pragma once

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#if defined(__SSE2__)
#include <emmintrin.h>
#endif

#include "nkv_merkle.h"

namespace nkv {
namespace merkletree {

constexpr uint8_t MERKLE_NODE_EMPTY = NKV_MERKLE_NODE_EMPTY;

inline void check(int rc, const char* what) {
    if (rc != NKV_OK) throw std::runtime_error(std::string(what) + ": " + nkv_strerror(rc));
}

// NewLeaf's arena copies off the caller's thread: the
// caller only records (arena place, value pointer, length); a pool of threads
// copies whole jobs of consecutive places.  settled() is the arena prefix whose
// copies have all finished (jobs finish out of order), which the caller streams
// to the device (nkv_host_stream) while the NewLeaf loop goes on.
class CopyPool {
   public:
    struct Task {
        uint64_t at;
        const uint8_t* src;
        size_t n;
    };
    struct Job {
        uint8_t* base = nullptr;  // the arena the places are in
        uint64_t end = 0;         // arena bytes [0, end) are covered once this job is done
        std::vector<Task> tasks;
        std::atomic<bool> done{false};
    };
    using CopyFn = void (*)(uint8_t*, const uint8_t*, size_t);

    explicit CopyPool(int threads, CopyFn copy) : copy_(copy) {
        for (int i = 0; i < threads; ++i) th_.emplace_back([this] { Work(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    CopyPool(const CopyPool&) = delete;
    CopyPool& operator=(const CopyPool&) = delete;
    int threads() const { return int(th_.size()); }

    void Submit(std::unique_ptr<Job> j) {
        Job* raw = j.get();
        {
            std::lock_guard<std::mutex> g(mu_);
            jobs_.push_back(std::move(j));
            queue_.push_back(raw);
        }
        cv_.notify_one();
    }
    // the arena prefix whose copies are all done (caller thread only)
    uint64_t Settled() {
        std::lock_guard<std::mutex> g(mu_);
        while (!jobs_.empty() && jobs_.front()->done.load(std::memory_order_acquire)) Retire();
        return settled_;
    }
    // a job to fill: a retired one with its task vector's capacity (no fresh
    // allocation, and no page faults, per job once a flush of that size ran)
    std::unique_ptr<Job> Fresh() {
        std::lock_guard<std::mutex> g(mu_);
        std::unique_ptr<Job> j;
        if (!free_.empty()) {
            j = std::move(free_.back());
            free_.pop_back();
            j->tasks.clear();
            j->done.store(false);
        } else {
            j.reset(new Job());
        }
        return j;
    }
    // a job that was filled but copied by its owner instead (Session::Settle)
    void Recycle(std::unique_ptr<Job> j) {
        if (!j) return;
        std::lock_guard<std::mutex> g(mu_);
        j->tasks.clear();
        free_.push_back(std::move(j));
    }
    CopyFn copy_fn() const { return copy_; }
    // wait for every submitted job (their stores are fenced by the workers)
    void Drain() {
        std::unique_lock<std::mutex> g(mu_);
        idle_.wait(g, [this] { return queue_.empty() && busy_ == 0; });
        while (!jobs_.empty()) Retire();
    }
    // a new batch starts at arena byte 0
    void Reset() {
        Drain();
        settled_ = 0;
    }

   private:
    void Retire() {  // the front job is done (mu_ held)
        settled_ = jobs_.front()->end;
        free_.push_back(std::move(jobs_.front()));
        jobs_.pop_front();
    }
    void Work() {
        std::unique_lock<std::mutex> g(mu_);
        while (true) {
            cv_.wait(g, [this] { return stop_ || !queue_.empty(); });
            if (queue_.empty()) return;  // stop_
            Job* j = queue_.front();
            queue_.pop_front();
            ++busy_;
            g.unlock();
            for (const Task& t : j->tasks) copy_(j->base + t.at, t.src, t.n);
#if defined(__SSE2__)
            _mm_sfence();  // this thread's non-temporal stores, before done is seen
#endif
            j->done.store(true, std::memory_order_release);
            g.lock();
            if (--busy_ == 0 && queue_.empty()) idle_.notify_all();
        }
    }

    CopyFn copy_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, idle_;
    std::deque<std::unique_ptr<Job>> jobs_;  // submitted, in arena order, not yet settled
    std::vector<std::unique_ptr<Job>> free_;  // retired, for Fresh()
    std::deque<Job*> queue_;                 // not yet taken by a worker
    int busy_ = 0;
    bool stop_ = false;
    uint64_t settled_ = 0;
};

// A small persistent team of host threads for New's materialization and
// Serialize's walk: Run(parts, fn) calls fn(0 .. parts - 1) on the team and the
// calling thread, and returns when every part is done.
class TaskTeam {
   public:
    explicit TaskTeam(int threads) {
        for (int i = 1; i < threads; ++i) th_.emplace_back([this] { Work(); });
    }
    ~TaskTeam() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    TaskTeam(const TaskTeam&) = delete;
    TaskTeam& operator=(const TaskTeam&) = delete;
    int size() const { return int(th_.size()) + 1; }

    // Safe from several threads at once: one run holds the team, and a caller
    // that finds it busy (another thread's Serialize or New) runs its parts
    // itself (two trees serialized or destroyed on two threads, as
    // Go allows).
    void Run(int parts, const std::function<void(int)>& fn) {
        struct Hold {  // the team for this run, released however the run ends
            std::atomic<bool>* f;
            bool own;
            ~Hold() {
                if (own) f->store(false, std::memory_order_release);
            }
        } held{&busy_, false};
        if (parts > 1 && !th_.empty()) held.own = !busy_.exchange(true, std::memory_order_acq_rel);
        if (!held.own) {  // every part runs, as on the team
            std::exception_ptr e;
            for (int k = 0; k < parts; ++k) {
                try {
                    fn(k);
                } catch (...) {
                    if (!e) e = std::current_exception();
                }
            }
            if (e) std::rethrow_exception(e);
            return;
        }
        std::unique_lock<std::mutex> g(mu_);
        fn_ = &fn;
        parts_ = parts;
        next_.store(0);
        left_ = parts;
        ++gen_;
        g.unlock();
        cv_.notify_all();
        Claim(fn, parts);
        g.lock();
        // every part done and no worker still inside Claim (a late fetch_add of
        // a finished run must not take a part of the next one)
        done_.wait(g, [this] { return left_ == 0 && active_ == 0; });
        fn_ = nullptr;
        // a part that threw (on any thread): rethrown here, once every thread
        // has left fn, which lives in the caller's frame
        if (err_) {
            std::exception_ptr e = err_;
            err_ = nullptr;
            g.unlock();
            std::rethrow_exception(e);
        }
    }

   private:
    void Claim(const std::function<void(int)>& fn, int parts) {  // take parts until none is left
        for (int k; (k = next_.fetch_add(1)) < parts;) {
            std::exception_ptr e;
            try {
                fn(k);
            } catch (...) {
                e = std::current_exception();
            }
            std::lock_guard<std::mutex> g(mu_);
            if (e && !err_) err_ = e;
            if (--left_ == 0) done_.notify_all();
        }
    }
    void Work() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> g(mu_);
        while (true) {
            cv_.wait(g, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            if (!fn_) continue;  // that run already finished without this thread
            const std::function<void(int)>* fn = fn_;
            const int parts = parts_;
            ++active_;
            g.unlock();
            Claim(*fn, parts);
            g.lock();
            if (--active_ == 0 && left_ == 0) done_.notify_all();
        }
    }

    std::vector<std::thread> th_;
    std::atomic<bool> busy_{false};  // a run owns the team
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int parts_ = 0, left_ = 0, active_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
    std::exception_ptr err_;  // the first part that threw in the current run
};

struct MerkleNode;

// One device context + the pinned arena that deferred NewLeaf values go to.
//
// Threads: NewLeaf and New of one session are one thread at a time (the
// caller's flush or compaction loop; the Go shim holds a mutex).  Serialize,
// Deserialize and the destruction of finished trees may run on several threads
// at once: the recycled node storage is locked and the host team runs one
// caller's parts at a time.
class Session {
   public:
    // The device context is created on first use (ctx()), so trees that never
    // hash (Deserialize, Serialize of a read tree) need no GPU.
    explicit Session(int device = 0) : device_(device) {}
    ~Session();  // below MerkleNode (it frees the recycled node storage)
    Session(const Session&) = delete;
    Session& operator=(const Session&) = delete;

    nkv_ctx* ctx() {
        std::call_once(ctx_once_, [this] {
            check(nkv_ctx_create(device_, &ctx_), "nkv_ctx_create");
            // NKV_ARENA_COHERENT=0: the arena in default pinned memory (A/B runs)
            if (const char* e = std::getenv("NKV_ARENA_COHERENT"))
                check(nkv_ctx_set_option(ctx_, NKV_OPT_ARENA_COHERENT, std::atoi(e) ? 1 : 0), "NKV_ARENA_COHERENT");
        });
        return ctx_;
    }

    // The process-wide default session on device 0 (Go's package-level state).
    // Never destroyed: a tree with static storage may outlive any other static,
    // and its destructor recycles into this session.
    static Session& Default() {
        static Session* s = new Session(0);
        return *s;
    }

    // Size the pinned arena for a flush of up to `bytes` of values (plus their
    // 16-byte alignment) before the first NewLeaf, e.g. from the memtable's
    // threshold at engine start (coreconf MEMTABLE_THRESHOLD): the first flush
    // then neither grows nor copies the arena.
    void Reserve(uint64_t bytes) { Grow(bytes, false); }

    // ---- deferred leaves ----
    struct Batch {
        uint64_t epoch;
        std::vector<uint64_t> off, len;
        std::vector<uint8_t> digests;  // filled when resolved
        bool resolved = false;
    };

    // Places `data` in the arena at a 16-byte aligned place (the leaf kernel's
    // aligned path reads the values where they lie: the library copies the
    // arena to the device in one DMA, nkv_merkle.h); returns (batch, index).
    // With copy threads (default) the copy itself is queued for the pool in
    // jobs of kJobBytes and `data` must stay unchanged until New returns;
    // with 0 threads it is copied here.  Every settled kStreamChunk of the
    // arena starts its device copy at once (nkv_host_stream), so the copy
    // overlaps the rest of the NewLeaf loop.
    static constexpr uint64_t kStreamChunk = uint64_t(32) << 20;
    static constexpr uint64_t kJobBytes = uint64_t(2) << 20;
    // Values of at least kStreamCopy bytes go to the arena with non-temporal
    // stores: the arena is written once and then read by the DMA engine, so
    // pulling its lines into the cache first (the read-for-ownership of a
    // plain store) only costs memory bandwidth.  Fence() orders them before
    // any DMA that reads the arena.
    static constexpr size_t kStreamCopy = 256;
    // defer = false: copied on the caller's thread now (for values the caller
    // may free at once: NewLeaf's std::string / std::vector forms, often
    // temporaries in C++, where Go's garbage collector keeps a slice alive)
    // Returns the value's index in the current batch (batch()).
    uint64_t AddLeaf(const uint8_t* data, size_t n, bool defer = true) {
        if (!batch_ || batch_->resolved) {
            // a sealed batch nobody else holds is reused: its vectors keep their
            // capacity (sized for the last flush, no regrowth per flush)
            const size_t hint = batch_ ? batch_->off.size() : 0;
            if (batch_ && batch_.use_count() == 1) {
                batch_->off.clear();
                batch_->len.clear();
                batch_->digests.clear();
                batch_->resolved = false;
            } else {
                auto nb = std::make_shared<Batch>();
                if (batch_ && batch_->resolved) {
                    // a sealed batch's places are never read again (its leaves
                    // hold their digests or read them from `digests`): the new
                    // batch takes its vectors, capacity and all
                    nb->off.swap(batch_->off);
                    nb->len.swap(batch_->len);
                    nb->off.clear();
                    nb->len.clear();
                }
                nb->off.reserve(hint);
                nb->len.reserve(hint);
                batch_ = std::move(nb);
            }
            batch_->epoch = ++epoch_;
            Settle();
            used_ = 0;
            streamed_ = 0;
            if (pool_) pool_->Reset();
        }
        const uint64_t at = (used_ + 15) & ~uint64_t(15);
        Grow(at + n, true);
        batch_->off.push_back(at);
        batch_->len.push_back(n);
        used_ = at + n;
        if (defer && Pool()) {
            if (!job_) {
                job_ = pool_->Fresh();
                job_->base = static_cast<uint8_t*>(arena_);
                if (job_->tasks.capacity() == 0) job_->tasks.reserve(kJobBytes / 4096 + 1);
            }
            if (n) job_->tasks.push_back({at, data, n});
            job_bytes_ += n;
            if (job_bytes_ >= kJobBytes) {
                SubmitJob();
                if (stream_) {  // checked once per job, not per value
                    const uint64_t s = pool_->Settled();
                    if (s >= streamed_ + kStreamChunk) {
                        streamed_ = s - s % kStreamChunk;
                        Fence();  // values this thread copied itself (the std::string forms)
                        check(nkv_host_stream(ctx(), arena_, streamed_), "nkv_host_stream");
                    }
                }
            }
        } else {
            if (nt_) CopyIn(static_cast<uint8_t*>(arena_) + at, data, n);
            else if (n) std::memcpy(static_cast<uint8_t*>(arena_) + at, data, n);
            if (!pool_ && stream_ && used_ >= streamed_ + kStreamChunk) {
                streamed_ = used_ - used_ % kStreamChunk;
                Fence();
                check(nkv_host_stream(ctx(), arena_, streamed_), "nkv_host_stream");
            }
        }
        return batch_->off.size() - 1;
    }
    const std::shared_ptr<Batch>& batch() const { return batch_; }
    // Every queued arena copy done (New and every other reader of the arena
    // call this first).
    // A job of at most kInlineJob bytes still being filled (a small flush's
    // whole batch, or the tail of a large one) is copied here instead: handing
    // it to a pool thread and waiting for it costs two thread wake-ups, more
    // than the copy (the reference's default flush is ~2 KB).
    static constexpr uint64_t kInlineJob = uint64_t(256) << 10;
    // A larger last job (a flush under kJobBytes, e.g. 1 Ki x 1 KiB) goes to the
    // pool in pieces of about kInlineJob, one per copy thread.
    void Settle() {
        if (!pool_) return;
        if (job_ && job_bytes_ <= kInlineJob) {
            const CopyPool::CopyFn copy = pool_->copy_fn();
            for (const CopyPool::Task& t : job_->tasks) copy(job_->base + t.at, t.src, t.n);
            pool_->Recycle(std::move(job_));
            job_.reset();
            job_bytes_ = 0;
        } else if (job_ && pool_->threads() > 1) {
            const uint64_t parts = std::min<uint64_t>(uint64_t(pool_->threads()), job_bytes_ / kInlineJob + 1);
            const uint64_t per = job_bytes_ / parts + 1;
            std::unique_ptr<CopyPool::Job> big = std::move(job_);
            std::unique_ptr<CopyPool::Job> piece;
            uint64_t bytes = 0;
            for (const CopyPool::Task& t : big->tasks) {
                if (!piece) {
                    piece = pool_->Fresh();
                    piece->base = big->base;
                }
                piece->tasks.push_back(t);
                piece->end = t.at + t.n;  // tasks are in arena order
                bytes += t.n;
                if (bytes >= per) {
                    pool_->Submit(std::move(piece));
                    bytes = 0;
                }
            }
            if (piece) {
                piece->end = used_;
                pool_->Submit(std::move(piece));
            }
            pool_->Recycle(std::move(big));
            job_bytes_ = 0;
        } else {
            SubmitJob();
        }
        pool_->Drain();
    }
    // NewLeaf's copy threads: 0 = copy on the caller's thread; default
    // min(16, cores), or the NKV_COPY_THREADS environment variable
    void SetCopyThreads(int k) {
        Settle();
        pool_.reset();
        copy_threads_ = std::max(0, k);
        if (copy_threads_) pool_.reset(new CopyPool(copy_threads_, nt_ ? &CopyIn : &PlainCopy));
    }
    int CopyThreads() { return Pool() ? pool_->threads() : 0; }
    // NewLeaf streams settled arena chunks ahead of New (default on)
    void SetStreaming(bool on) { stream_ = on; }
    // NewLeaf copies values of kStreamCopy bytes or more with non-temporal
    // stores (default on; off: memcpy)
    void SetNonTemporal(bool on) {
        nt_ = on;
        if (pool_) SetCopyThreads(pool_->threads());
    }

    const uint8_t* arena() const { return static_cast<const uint8_t*>(arena_); }
    // nkv_host_alloc calls so far: a sealed batch's arena is reused by the next
    // batch (flush after flush), so this grows only when a batch outgrows it
    uint64_t arena_allocs() const { return allocs_; }

    void ResolveBatch(Batch& b) {
        if (b.resolved) return;
        const uint64_t n = b.off.size();
        b.digests.assign(20 * n, 0);
        Settle();
        Fence();
        check(nkv_leaf_hash(ctx(), arena(), b.off.data(), b.len.data(), n, b.digests.data()), "NewLeaf");
        b.resolved = true;
    }

    // makes the arena's non-temporal stores visible to the DMA engine
    static void Fence() {
#if defined(__SSE2__)
        _mm_sfence();
#endif
    }

    // NewLeaf's arena copy (public for its CPU test); dst is 16-byte aligned
    // (AddLeaf's places)
    static void CopyIn(uint8_t* dst, const uint8_t* src, size_t n) {
#if defined(__SSE2__)
        if (n >= kStreamCopy) {
            const size_t body = n & ~size_t(63);
            for (size_t i = 0; i < body; i += 64) {
                const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
                const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
                const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
                const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
                _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
                _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
                _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
                _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
            }
            if (n > body) std::memcpy(dst + body, src + body, n - body);
            return;
        }
#endif
        if (n) std::memcpy(dst, src, n);
    }
    static void PlainCopy(uint8_t* dst, const uint8_t* src, size_t n) {
        if (n) std::memcpy(dst, src, n);
    }

    // New's pointer tree reuses the node storage of trees already destroyed
    // (no per-node allocation once a flush of that size has run)
    std::vector<MerkleNode>* TakeNodes();
    void GiveNodes(std::vector<MerkleNode>* v);
    // the host thread team (lazily: min(8, cores) threads)
    TaskTeam& Team() {
        std::call_once(team_once_, [this] {
            team_.reset(new TaskTeam(int(std::min<unsigned>(8, std::max(1u, std::thread::hardware_concurrency())))));
        });
        return *team_;
    }
    // New's level arrays, recycled the same way (no 20 * (2n - 1)-byte zero
    // fill and page faults per flush)
    std::vector<uint8_t> TakeLevels() {
        std::vector<uint8_t> v;
        std::lock_guard<std::mutex> g(spare_mu_);
        v.swap(spare_levels_);
        return v;
    }
    void GiveLevels(std::vector<uint8_t>&& v) {
        std::lock_guard<std::mutex> g(spare_mu_);
        if (v.capacity() > spare_levels_.capacity()) spare_levels_.swap(v);
    }
    // the host team (Team()) is created once even when two threads ask at once
    std::once_flag team_once_;

   private:
    CopyPool* Pool() {
        if (!pool_ && copy_threads_ < 0) {
            const char* e = std::getenv("NKV_COPY_THREADS");
            const int hw = int(std::thread::hardware_concurrency());
            SetCopyThreads(e ? std::atoi(e) : std::min(16, std::max(1, hw)));
        }
        return pool_.get();
    }
    void SubmitJob() {
        if (job_) {
            job_->end = used_;
            pool_->Submit(std::move(job_));
        }
        job_.reset();
        job_bytes_ = 0;
    }
    // A block of at least `bytes`: exactly that for Reserve, else (NewLeaf
    // outgrowing the block) twice the old size, from kFirstArena.  The open
    // batch's values move with it.  A process that only flushes the engine's
    // default 10-value memtables pins 1 MiB (and, since its values take the
    // small path, no HBM mirror: nkv_host_alloc mirrors blocks of >= 64 MiB
    // up front, smaller ones on first use).
    static constexpr uint64_t kFirstArena = uint64_t(1) << 20;
    void Grow(uint64_t bytes, bool doubling) {
        if (bytes <= cap_) return;
        Settle();  // no queued copy may land in the old block
        uint64_t want = bytes;
        if (doubling) {
            want = cap_ ? cap_ * 2 : kFirstArena;
            while (want < bytes) want *= 2;
        }
        void* p = nullptr;
        check(nkv_host_alloc(ctx(), want, &p), "nkv_host_alloc");
        ++allocs_;
        if (arena_) {
            Fence();
            if (used_) std::memcpy(p, arena_, used_);
            nkv_host_free(ctx(), arena_);
        }
        arena_ = p;
        cap_ = want;
        streamed_ = 0;  // a new block: its device copy starts from byte 0
    }

    int device_ = 0;
    std::once_flag ctx_once_;
    nkv_ctx* ctx_ = nullptr;
    std::mutex spare_mu_;  // spare_ and spare_levels_ (trees end on any thread)
    void* arena_ = nullptr;
    uint64_t cap_ = 0, used_ = 0, epoch_ = 0, allocs_ = 0, streamed_ = 0;
    bool stream_ = true, nt_ = true;
    std::shared_ptr<Batch> batch_;
    std::unique_ptr<CopyPool> pool_;
    std::unique_ptr<CopyPool::Job> job_;  // the job NewLeaf is filling
    uint64_t job_bytes_ = 0;
    int copy_threads_ = -1;  // -1: not chosen yet (Pool())
    std::vector<std::vector<MerkleNode>*> spare_;
    std::vector<uint8_t> spare_levels_;
    std::unique_ptr<TaskTeam> team_;
};

struct MerkleNode {  // merklenode.go:15-19
    std::vector<uint8_t> Data;
    MerkleNode* Left = nullptr;
    MerkleNode* Right = nullptr;

    // deferred NewLeaf digest (resolved by New or Resolve).  New marks its
    // leaves resolved with pend_idx = kResolved instead of dropping pend (no
    // atomic reference-count update per leaf on New's path).
    static constexpr uint64_t kResolved = ~uint64_t(0);
    std::shared_ptr<Session::Batch> pend;
    uint64_t pend_idx = 0;
    bool pending() const { return pend && pend_idx != kResolved; }

    MerkleNode() = default;
    explicit MerkleNode(std::vector<uint8_t> d) : Data(std::move(d)) {}

    const std::vector<uint8_t>& Resolve() {
        if (pending()) {
            Session::Default().ResolveBatch(*pend);
            Data.assign(pend->digests.begin() + 20 * pend_idx, pend->digests.begin() + 20 * pend_idx + 20);
            pend.reset();
        }
        return Data;
    }

    std::string String() {  // merklenode.go:22-24 (hex)
        static const char* hx = "0123456789abcdef";
        Resolve();
        std::string s;
        for (uint8_t b : Data) {
            s.push_back(hx[b >> 4]);
            s.push_back(hx[b & 15]);
        }
        return s;
    }

    void Serialize(std::vector<uint8_t>& w) {  // merklenode.go:37-63
        Resolve();
        if (Data.empty()) {
            w.push_back(MERKLE_NODE_EMPTY);
        } else {
            w.push_back(0);
            w.insert(w.end(), Data.begin(), Data.end());
        }
    }

    // merklenode.go:67-96: true at EOF (a truncated node counts as EOF)
    bool Deserialize(const uint8_t*& p, const uint8_t* end) {
        if (p >= end) return true;
        const uint8_t flags = *p++;
        if (flags & MERKLE_NODE_EMPTY) {
            Data.clear();
        } else {
            if (end - p < 20) return true;
            Data.assign(p, p + 20);
            p += 20;
        }
        pend.reset();
        return false;
    }
};

// merklenode.go:27-34.  The pointer form defers the copy to the session's copy
// threads: data[0, n) must stay unchanged until New returns (the flush and
// compaction callers hand over values they never mutate).  The std::vector /
// std::string forms copy at once (their argument may be a temporary).
// Data stays empty until the batch is resolved (New, or Resolve / String /
// Serialize / Validate on the node): one allocation fewer on the caller's
// thread per value; New fills the leaves' Data on several threads.
inline MerkleNode NewLeafAt(const uint8_t* data, size_t n, bool defer) {
    MerkleNode m;
    Session& S = Session::Default();
    m.pend_idx = S.AddLeaf(data, n, defer);
    m.pend = S.batch();
    return m;
}
inline MerkleNode NewLeaf(const uint8_t* data, size_t n) { return NewLeafAt(data, n, true); }
inline MerkleNode NewLeaf(const std::vector<uint8_t>& v) { return NewLeafAt(v.data(), v.size(), false); }
inline MerkleNode NewLeaf(const std::string& v) {
    return NewLeafAt(reinterpret_cast<const uint8_t*>(v.data()), v.size(), false);
}

inline Session::~Session() {
    team_.reset();
    pool_.reset();
    for (auto* v : spare_) delete v;
    if (arena_) nkv_host_free(ctx_, arena_);
    if (ctx_) nkv_ctx_destroy(ctx_);
}

inline std::vector<MerkleNode>* Session::TakeNodes() {
    std::lock_guard<std::mutex> g(spare_mu_);
    if (spare_.empty()) return new std::vector<MerkleNode>();
    auto* v = spare_.back();
    spare_.pop_back();
    return v;
}

inline void Session::GiveNodes(std::vector<MerkleNode>* v) {
    if (!v) return;
    std::unique_lock<std::mutex> g(spare_mu_);
    if (spare_.size() >= 2) {  // two trees' worth (a flush and the one before)
        g.unlock();
        delete v;
        return;
    }
    spare_.push_back(v);
}

inline std::vector<std::vector<uint8_t>> Sha1Many(const std::vector<std::vector<uint8_t>>& msgs);

class MerkleTree {  // merkletree.go:13-15
   public:
    MerkleNode* Root = nullptr;

    MerkleTree() = default;
    ~MerkleTree() {
        Session::Default().GiveNodes(inner_);
        Session::Default().GiveLevels(std::move(levels_));
    }
    MerkleTree(const MerkleTree&) = delete;
    MerkleTree& operator=(const MerkleTree&) = delete;

    // merkletree.go:67-92: write the BFS image; O_WRONLY|O_CREAT without O_TRUNC.
    // (A per-thread image buffer kept across flushes measured no faster: the
    // walk's time is the pointer chase, not the buffer.)
    void Serialize(const std::string& fname) {
        std::vector<uint8_t> buf;
        const auto t0 = std::chrono::steady_clock::now();
        const uint64_t total = WalkInto(buf);
        const auto t1 = std::chrono::steady_clock::now();
        check(nkv_write_file(fname.c_str(), buf.data(), total), ("Serialize(" + fname + ")").c_str());
        const auto t2 = std::chrono::steady_clock::now();
        ser_timing_.walk_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        ser_timing_.write_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
        ser_timing_.bytes = total;
    }
    // where the last Serialize's time went (bench.py --config api_flush)
    struct SerializeTiming {
        double walk_ms = 0, write_ms = 0;
        uint64_t bytes = 0;
    };
    const SerializeTiming& LastSerializeTiming() const { return ser_timing_; }

    // The image as bytes (the same walk into a fresh vector).
    std::vector<uint8_t> SerializeBytes() {
        std::vector<uint8_t> w;
        w.resize(WalkInto(w));
        return w;
    }

   private:
    // The queue walk (merkletree.go:75-89).  A FIFO queue visits every node of
    // depth d, in order, before any of depth d + 1, so the walk goes level by
    // level: each level's children and byte counts in parallel chunks (the host
    // team), then the image (merklenode.go:37-63) written in place, chunk by
    // chunk, at offsets known from the counts.  The same bytes as the queue.
    // Writes the image to w[0, total) (w grows if it is smaller, and is never
    // shrunk or cleared) and returns total.
    uint64_t WalkInto(std::vector<uint8_t>& w) {
        struct Level {
            std::vector<MerkleNode*> v;
            std::vector<uint64_t> cut, bytes;  // chunk bounds (parts + 1), chunk byte counts
        };
        std::vector<Level> lv(1);
        lv[0].v.push_back(Root);
        TaskTeam& team = Session::Default().Team();
        for (size_t d = 0; !lv[d].v.empty(); ++d) {
            Level& L = lv[d];
            const uint64_t m = L.v.size();
            const int parts = m >= (uint64_t(1) << 15) ? 4 * team.size() : 1;
            L.cut.resize(parts + 1);
            for (int k = 0; k <= parts; ++k) L.cut[k] = m * uint64_t(k) / parts;
            L.bytes.assign(parts, 0);
            std::vector<uint64_t> kids(parts, 0);
            std::vector<char> pend(parts, 0);
            team.Run(parts, [&](int k) {
                uint64_t c = 0, b = 0;
                for (uint64_t i = L.cut[k]; i < L.cut[k + 1]; ++i) {
                    const MerkleNode* x = L.v[i];
                    c += (x->Left != nullptr) + (x->Right != nullptr);
                    if (x->pending()) pend[k] = 1;
                    b += x->Data.empty() ? 1 : 1 + x->Data.size();
                }
                kids[k] = c;
                L.bytes[k] = b;
            });
            if (std::find(pend.begin(), pend.end(), 1) != pend.end()) {
                // deferred NewLeaf digests (a device call): resolve on this thread
                for (int k = 0; k < parts; ++k) {
                    uint64_t b = 0;
                    for (uint64_t i = L.cut[k]; i < L.cut[k + 1]; ++i) {
                        const size_t sz = L.v[i]->Resolve().size();
                        b += sz ? 1 + sz : 1;
                    }
                    L.bytes[k] = b;
                }
            }
            std::vector<uint64_t> at(parts + 1, 0);
            for (int k = 0; k < parts; ++k) at[k + 1] = at[k] + kids[k];
            lv.emplace_back();
            Level& N = lv.back();
            Level& P = lv[d];  // (emplace_back may have moved the levels)
            N.v.resize(at[parts]);
            team.Run(parts, [&](int k) {
                uint64_t o = at[k];
                for (uint64_t i = P.cut[k]; i < P.cut[k + 1]; ++i) {
                    MerkleNode* x = P.v[i];
                    if (x->Left) N.v[o++] = x->Left;
                    if (x->Right) N.v[o++] = x->Right;
                }
            });
        }
        uint64_t total = 0;
        for (const Level& L : lv)
            for (uint64_t b : L.bytes) total += b;
        if (w.size() < total) w.resize(total);
        uint64_t base = 0;
        for (const Level& L : lv) {
            const int parts = int(L.bytes.size());
            std::vector<uint64_t> at(parts + 1, base);
            for (int k = 0; k < parts; ++k) at[k + 1] = at[k] + L.bytes[k];
            team.Run(parts, [&](int k) {
                uint8_t* o = w.data() + at[k];
                for (uint64_t i = L.cut[k]; i < L.cut[k + 1]; ++i) {
                    const MerkleNode* x = L.v[i];
                    const size_t sz = x->Data.size();
                    if (!sz) {
                        *o++ = MERKLE_NODE_EMPTY;
                    } else {
                        *o++ = 0;
                        std::memcpy(o, x->Data.data(), sz);
                        o += sz;
                    }
                }
            });
            base = at[parts];
        }
        return total;
    }

   public:
    // merkletree.go:97-157, including its quirk: the loop compares the node
    // counter against the just-emptied queue and stops, so only the root is
    // linked into the tree.
    void Deserialize(const std::string& fname) {
        FILE* f = std::fopen(fname.c_str(), "rb");
        if (!f) throw std::runtime_error("open " + fname);
        std::vector<uint8_t> blob;
        uint8_t buf[1 << 16];
        size_t k;
        while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) blob.insert(blob.end(), buf, buf + k);
        std::fclose(f);
        leaves_.clear();
        if (!inner_) inner_ = Session::Default().TakeNodes();
        inner_->clear();
        const uint8_t* p = blob.data();
        const uint8_t* end = p + blob.size();
        while (true) {
            MerkleNode n;
            if (n.Deserialize(p, end)) break;
            inner_->push_back(std::move(n));
        }
        Root = inner_->empty() ? nullptr : &inner_->front();
        n_ = 0;  // no longer a tree New built
    }

    // merkletree.go:162-171: recompute the root from the leaves' Data.  When the
    // pointer tree under Root has exactly the shape New builds for its n leaves
    // (checked link by link: NewShapedLeaves), rehash (merklenode.go:99-108)
    // equals the tree rebuilt from the leaves' current Data -- one device call,
    // nkv_tree_validate.  Any other tree (Deserialize's root-only tree, a
    // hand-built or relinked one) is rehashed per depth.
    bool Validate() {
        if (!Root) throw std::runtime_error("Validate: nil root");
        std::vector<MerkleNode*> leaves;
        if (n_ && NewShapedLeaves(Root, n_, &leaves)) {
            if (Root->Resolve().size() < 20) throw std::runtime_error("Validate: index out of range");
            std::vector<uint8_t> flat;
            std::vector<uint64_t> off, len;
            for (MerkleNode* x : leaves) {
                const auto& d = x->Resolve();
                off.push_back(flat.size());
                len.push_back(d.size());
                flat.insert(flat.end(), d.begin(), d.end());
            }
            flat.push_back(0);
            int ok = 0;
            check(nkv_tree_validate(Session::Default().ctx(), flat.data(), off.data(), len.data(), leaves.size(),
                                    Root->Data.data(), &ok),
                  "Validate");
            return ok != 0;
        }
        std::vector<uint8_t> h = Rehash(Root);
        if (Root->Resolve().size() < 20 || h.size() < 20)
            throw std::runtime_error("Validate: index out of range");
        for (int i = 0; i < 20; ++i)
            if (Root->Data[i] != h[i]) return false;
        return true;
    }

    // every digest, level-major bottom-up (as the C-ABI returns it)
    const std::vector<uint8_t>& Levels() const { return levels_; }

    // where New's time went (bench.py --config api_flush): the device call
    // (values to HBM, kernels, digests back) and the pointer-tree materialization
    struct NewTiming {
        double call_ms = 0, materialize_ms = 0;
    };
    const NewTiming& LastNewTiming() const { return timing_; }

    friend std::unique_ptr<MerkleTree> New(std::vector<MerkleNode> level, std::string* err);

   private:
    // The n level-0 nodes under root when the tree has New's shape for n leaves
    // (merkletree.go:31-64): every internal node has two children, each odd level
    // below the top ends in an empty childless pad, level-0 nodes are childless.
    static bool NewShapedLeaves(MerkleNode* root, uint64_t n, std::vector<MerkleNode*>* out) {
        const int top = nkv_num_levels(n) - 1;
        std::vector<MerkleNode*> cur{root};
        auto pad_ok = [](const MerkleNode* p) { return !p->Left && !p->Right && p->Data.empty() && !p->pending(); };
        for (int L = top; L >= 0; --L) {
            const uint64_t real = nkv_level_count(n, L);
            const bool pad = (real & 1) && L < top;
            if (cur.size() != real + (pad ? 1 : 0)) return false;
            if (pad && !pad_ok(cur.back())) return false;
            if (L == 0) {
                for (uint64_t i = 0; i < real; ++i)
                    if (cur[i]->Left || cur[i]->Right) return false;
                out->assign(cur.begin(), cur.begin() + real);
                return true;
            }
            std::vector<MerkleNode*> nxt;
            nxt.reserve(2 * real);
            for (uint64_t i = 0; i < real; ++i) {
                if (!cur[i]->Left || !cur[i]->Right) return false;
                nxt.push_back(cur[i]->Left);
                nxt.push_back(cur[i]->Right);
            }
            cur.swap(nxt);
        }
        return false;
    }

    // merklenode.go:99-108 by depth on the device (pads make the tree ragged)
    static std::vector<uint8_t> Rehash(MerkleNode* root) {
        std::vector<std::vector<MerkleNode*>> lv{{root}};
        while (true) {
            std::vector<MerkleNode*> nx;
            for (MerkleNode* n : lv.back()) {
                if ((n->Left == nullptr) != (n->Right == nullptr))
                    throw std::runtime_error("Validate: nil pointer dereference");
                if (n->Left) {
                    nx.push_back(n->Left);
                    nx.push_back(n->Right);
                }
            }
            if (nx.empty()) break;
            lv.push_back(std::move(nx));
        }
        std::unordered_map<MerkleNode*, std::vector<uint8_t>> val;
        for (size_t d = lv.size(); d-- > 0;) {
            std::vector<std::vector<uint8_t>> msgs;
            std::vector<MerkleNode*> owners;
            for (MerkleNode* n : lv[d]) {
                if (!n->Left) {
                    val[n] = n->Resolve();
                } else {
                    std::vector<uint8_t> m = val[n->Left];
                    const auto& r = val[n->Right];
                    m.insert(m.end(), r.begin(), r.end());
                    msgs.push_back(std::move(m));
                    owners.push_back(n);
                }
            }
            if (!msgs.empty()) {
                auto dg = Sha1Many(msgs);
                for (size_t i = 0; i < owners.size(); ++i) val[owners[i]] = std::move(dg[i]);
            }
        }
        return val[root];
    }

    // the tree's nodes (stable addresses): New's leaves, and the internal nodes +
    // pads in storage recycled from destroyed trees (Deserialize: every node)
    std::vector<MerkleNode> leaves_;
    std::vector<MerkleNode>* inner_ = nullptr;
    std::vector<uint8_t> levels_;
    uint64_t n_ = 0;  // leaves New built the tree from
    NewTiming timing_;
    SerializeTiming ser_timing_;
};

inline std::vector<std::vector<uint8_t>> Sha1Many(const std::vector<std::vector<uint8_t>>& msgs) {
    std::vector<uint8_t> flat;
    std::vector<uint64_t> off, len;
    for (const auto& m : msgs) {
        off.push_back(flat.size());
        len.push_back(m.size());
        flat.insert(flat.end(), m.begin(), m.end());
    }
    flat.push_back(0);
    std::vector<uint8_t> out(20 * msgs.size());
    check(nkv_leaf_hash(Session::Default().ctx(), flat.data(), off.data(), len.data(), msgs.size(),
                        out.data()),
          "Validate");
    std::vector<std::vector<uint8_t>> r;
    for (size_t i = 0; i < msgs.size(); ++i) r.emplace_back(out.begin() + 20 * i, out.begin() + 20 * i + 20);
    return r;
}

// merkletree.go:18-25 (+ build, :31-64).  Returns nullptr and sets *err to the
// reference's error text for an empty level.
inline std::unique_ptr<MerkleTree> New(std::vector<MerkleNode> level, std::string* err = nullptr) {
    const uint64_t n = level.size();
    if (n == 0) {
        if (err) *err = "cannot build Merkle Tree from 0 nodes";
        return nullptr;
    }
    using clk = std::chrono::steady_clock;
    const auto c0 = clk::now();
    nkv_ctx* ctx = Session::Default().ctx();
    std::unique_ptr<MerkleTree> t(new MerkleTree());
    const uint64_t total = nkv_total_nodes(n);
    Session& S = Session::Default();
    t->levels_ = S.TakeLevels();
    t->levels_.resize(20 * total);  // recycled: every byte is written below (level 0 zeroed for generic leaves)
    uint8_t* nodes = t->levels_.data();

    // the flush / compaction pattern: n NewLeaf calls of one batch, in order
    const std::shared_ptr<Session::Batch> b0 = level[0].pend;
    bool same_batch = level[0].pending() && !b0->resolved && b0->off.size() == n;
    for (uint64_t i = 0; same_batch && i < n; ++i)
        same_batch = level[i].pend == b0 && level[i].pend_idx == i && !level[i].Left && !level[i].Right;
    if (same_batch) {
        S.Settle();
        Session::Fence();
        check(nkv_tree_from_values(ctx, S.arena(), b0->off.data(), b0->len.data(), n, nullptr, nodes, nullptr),
              "New");
        // other copies of these leaves (the caller kept the slice) resolve later
        // from the batch; New's own leaves are filled below
        if (b0.use_count() > 2 + int64_t(n)) b0->digests.assign(nodes, nodes + 20 * n);
        b0->resolved = true;
    } else {
        bool all20 = true;
        for (auto& x : level) all20 = all20 && x.Resolve().size() == 20;
        if (all20) {
            std::vector<uint8_t> leaf20;
            for (auto& x : level) leaf20.insert(leaf20.end(), x.Data.begin(), x.Data.end());
            check(nkv_tree_build(ctx, leaf20.data(), n, nullptr, nodes, nullptr), "New");
        } else {
            std::vector<uint8_t> flat;
            std::vector<uint64_t> off, len;
            for (auto& x : level) {
                off.push_back(flat.size());
                len.push_back(x.Data.size());
                flat.insert(flat.end(), x.Data.begin(), x.Data.end());
            }
            flat.push_back(0);
            // leaves of any length have no 20-byte level 0: zero it, as a fresh
            // array was (a recycled one holds the last tree's digests)
            std::memset(nodes, 0, 20 * n);
            check(nkv_tree_generic(ctx, flat.data(), off.data(), len.data(), n, nullptr, nodes + 20 * n,
                                   nullptr),
                  "New");
        }
    }
    const auto c1 = clk::now();
    // Materialize the pointer tree: the given leaves (Go copies `l := level[i]`:
    // `level` is New's own copy, kept as the tree's leaves), then the parents of
    // every level with the empty pad node (merkletree.go:32-34), in node storage
    // recycled from destroyed trees.  Every node's place is known up front, so
    // the fill runs on several threads.
    t->leaves_ = std::move(level);
    auto& leaves = t->leaves_;
    t->n_ = n;
    const int lv = nkv_num_levels(n);
    // pool layout: [level 0's pad], then for L = 1 .. top: level L, [level L's
    // pad] (a level below the top with an odd count has one)
    std::vector<uint64_t> lbase(lv + 1, 0), lpad(lv, ~uint64_t(0)), lcnt(lv), lstart(lv);
    for (int L = 0; L < lv; ++L) {
        lcnt[L] = nkv_level_count(n, L);
        lstart[L] = nkv_level_start(n, L);
    }
    uint64_t inner = 0;
    if (lcnt[0] & 1) lpad[0] = inner++;
    for (int L = 1; L < lv; ++L) {
        lbase[L] = inner;
        inner += lcnt[L];
        if (L + 1 < lv && (lcnt[L] & 1)) lpad[L] = inner++;
    }
    lbase[lv] = inner;
    t->inner_ = S.TakeNodes();
    std::vector<MerkleNode>& pool = *t->inner_;
    pool.resize(inner);
    auto node_at = [&](int L, uint64_t j) -> MerkleNode* {
        if (j == lcnt[L]) return &pool[lpad[L]];
        return L == 0 ? &leaves[j] : &pool[lbase[L] + j];
    };
    auto fill = [&](uint64_t lo, uint64_t hi) {  // items [lo, hi): leaves, then pool slots
        for (uint64_t x = lo; x < hi && x < n; ++x) {
            if (same_batch) {
                leaves[x].Data.assign(nodes + 20 * x, nodes + 20 * x + 20);
                leaves[x].pend_idx = MerkleNode::kResolved;
            }
        }
        int L = 1;
        for (uint64_t x = std::max(lo, n); x < hi; ++x) {
            const uint64_t k = x - n;
            while (k >= lbase[L + 1]) ++L;
            MerkleNode& m = pool[k];
            const uint64_t j = k - lbase[L];
            if (k < lbase[L] || j >= lcnt[L]) {  // a pad: MerkleNode{Data: []byte{}}
                m.Data.clear();
                m.Left = m.Right = nullptr;
            } else {
                const uint64_t i = lstart[L] + j;
                m.Data.assign(nodes + 20 * i, nodes + 20 * i + 20);
                m.Left = node_at(L - 1, 2 * j);
                m.Right = node_at(L - 1, 2 * j + 1);
            }
            if (m.pend) m.pend.reset();
            m.pend_idx = 0;
        }
    };
    const uint64_t items = n + inner;
    const int nt = items >= (uint64_t(1) << 16) ? 4 * S.Team().size() : 1;
    S.Team().Run(nt, [&](int k) { fill(items * uint64_t(k) / nt, items * uint64_t(k + 1) / nt); });
    MerkleNode* root = lv == 1 ? &leaves[0] : &pool[lbase[lv - 1]];
    t->Root = root;
    t->timing_.call_ms = std::chrono::duration<double, std::milli>(c1 - c0).count();
    t->timing_.materialize_ms = std::chrono::duration<double, std::milli>(clk::now() - c1).count();
    return t;
}

// The Merkle step of several compaction output tables (lsmtree.go:71-128 merges
// a level's runs; MakeTableSecondaries builds each output table's tree,
// sstable.go:35-47) over several GPUs of one process: table t goes to devices[t %
// g], one host thread per device drives that device's context of a group
// (nkv_group_create: one context per GPU and one RCCL communicator), and each
// table's values are located in its serialized Data table on the device
// (nkv_tree_from_records, record.go:191-199).  Returns the roots in table order.
struct DataTable {
    std::vector<uint8_t> data;       // the Data-table bytes (record.Serialize, record.go:191-199)
    std::vector<uint64_t> rec_size;  // KeyContext.RecSize of each record (record.go:38-41)
};

class Group {  // RAII over nkv_group
   public:
    explicit Group(const std::vector<int>& devices) {
        check(nkv_group_create(devices.data(), int(devices.size()), &g_), "nkv_group_create");
    }
    ~Group() { nkv_group_destroy(g_); }
    Group(const Group&) = delete;
    Group& operator=(const Group&) = delete;
    nkv_group* get() const { return g_; }
    int size() const { return nkv_group_size(g_); }
    nkv_ctx* ctx(int i) const {
        nkv_ctx* c = nullptr;
        check(nkv_group_ctx(g_, i, &c), "nkv_group_ctx");
        return c;
    }

   private:
    nkv_group* g_ = nullptr;
};

inline std::vector<std::array<uint8_t, 20>> CompactRoots(Group& grp, const std::vector<DataTable>& tables) {
    const int g = grp.size();
    std::vector<std::array<uint8_t, 20>> roots(tables.size());
    std::vector<std::exception_ptr> err(g);
    auto work = [&](int m) {
        try {
            nkv_ctx* c = grp.ctx(m);
            for (size_t t = size_t(m); t < tables.size(); t += size_t(g)) {
                const DataTable& d = tables[t];
                if (d.rec_size.empty()) throw std::runtime_error("cannot build Merkle Tree from 0 nodes");
                check(nkv_tree_from_records(c, d.data.data(), d.data.size(), d.rec_size.data(), d.rec_size.size(),
                                            roots[t].data(), nullptr, nullptr),
                      "CompactRoots");
            }
        } catch (...) {
            err[m] = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    for (int m = 1; m < g; ++m) th.emplace_back(work, m);
    work(0);
    for (auto& x : th) x.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    return roots;
}

inline std::vector<std::array<uint8_t, 20>> CompactRoots(const std::vector<int>& devices,
                                                         const std::vector<DataTable>& tables) {
    Group grp(devices);
    return CompactRoots(grp, tables);
}

}  // namespace merkletree
}  // namespace nkv
