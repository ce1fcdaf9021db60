// host_stage.hpp -- the host half of the host-buffer API: a worker pool and the
// pipelined pinned staging that moves caller memory to HBM and back.
//
// The reference's path starts and ends in host memory (memtable records on
// flush, Data-table bytes on compaction; core/sstable/sstable.go:58-74,
// core/lsmtree/lsmtree.go:146,211).  A synchronous host call therefore costs
// gather + H2D + compute + D2H.  The gather (caller bytes -> pinned staging)
// is split across a pool of host threads and overlapped with the DMA of the
// previous chunk, so the call runs at the PCIe rate instead of one core's
// memcpy rate.  No caller pointer is kept once a call returns (cgo rule): the
// DMA reads only library-owned pinned slots.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace nkv {

// Fixed set of worker threads; run() executes fn(0..njobs-1) on them and on the
// calling thread, and returns when every job is done.
class HostPool {
  public:
    HostPool() = default;
    ~HostPool();
    HostPool(const HostPool&) = delete;
    HostPool& operator=(const HostPool&) = delete;
    // total threads including the caller (>= 1); restarts the workers
    void resize(int threads);
    int threads() const { return int(workers_.size()) + 1; }
    void run(int njobs, const std::function<void(int)>& fn);

  private:
    void stop();
    void loop();
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable go_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int njobs_ = 0;
    std::atomic<int> next_{0};
    int busy_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

// Byte segments scattered over host memory and packed into one destination
// range: segment i is src + off[i] .. + len[i], destined for [dst[i], dst[i] +
// len[i]) of the packed range.  dst must be non-decreasing.
struct Segments {
    const uint8_t* src;
    const uint64_t* off;
    const uint64_t* len;
    const uint64_t* dst;
    uint64_t n;
};

constexpr int kStageSlots = 3;

// Pinned ring of kStageSlots chunks; each slot's DMA is tracked by an event.
struct Stager {
    void* slot[kStageSlots] = {nullptr, nullptr, nullptr};
    hipEvent_t ev[kStageSlots] = {nullptr, nullptr, nullptr};
    bool pending[kStageSlots] = {false, false, false};
    size_t slot_bytes = 0;
    size_t chunk = size_t(32) << 20;  // NKV_OPT_STAGE_CHUNK
    HostPool pool;
    int want_threads = 0;  // NKV_OPT_HOST_THREADS (0 = default)

    ~Stager();
    // (re)allocate slots of `chunk` bytes and start the pool; hipSuccess or an error
    hipError_t ready();
    // Gather the segments into packed bytes [0, total) of d_dst (device), chunk
    // by chunk: the pool fills a slot while the previous slots' DMA runs on
    // stream s.  Returns after the last gather; the DMA may still run.
    hipError_t upload(const Segments& seg, uint64_t total, uint8_t* d_dst, hipStream_t s);
    // Contiguous host bytes -> device.
    hipError_t upload(const uint8_t* src, uint64_t bytes, uint8_t* d_dst, hipStream_t s);
    // Device bytes -> host, synchronously (DMA into the slots, the pool copies out).
    hipError_t download(uint8_t* h_dst, const uint8_t* d_src, uint64_t bytes, hipStream_t s);
    // wait for every slot's DMA (before the slots are freed or resized)
    hipError_t drain();

  private:
    hipError_t wait_slot(int k);
    void release();
};

int default_host_threads();

}  // namespace nkv
