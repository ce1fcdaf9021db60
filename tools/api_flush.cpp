// api_flush -- the memtable-flush Merkle step end to end through the C++ mirror
// of the Go API (include/nkv_merkletree.hpp), driven exactly as
// sstable.makeMetadata drives ds/merkletree (core/sstable/sstable.go:58-74):
//
//   for each record: leaves = append(leaves, NewLeaf(rec.Value))   merklenode.go:27-34
//   tree := New(leaves)                                             merkletree.go:18-25
//   tree.Serialize(metadata file)                                   merkletree.go:67-92
//
// plus Root.String() (the caller's view of the root).  The values start in host
// memory (the memtable), one contiguous buffer of n x vlen bytes.  Every cycle
// is a fresh flush into a fresh file; cycle 0 also allocates the pinned arena,
// later cycles reuse it (steady state).  One JSON line per cycle:
//   newleaf_ms    the NewLeaf loop: arena places recorded and the copies queued
//                 for the copy threads (COPY_THREADS = 0: the copies themselves);
//                 streaming on, the DMA of every settled 32 MiB chunk starts
//                 inside it
//   new_call_ms   New's device call: the copy threads' last jobs, the rest of
//                 the values to HBM, leaf + tree kernels, every digest back
//     upload_ms / kernels_ms / download_ms   its HIP-event split
//   materialize_ms  New's pointer tree (2n - 1 nodes + pads)
//   root_ms       Root.String()
//   walk_ms / write_ms   Serialize(file): BFS walk of the live tree, the file
//                 write (MerkleTree::LastSerializeTiming)
//
// Usage: api_flush N VLEN CYCLES DIR [STREAMING=1] [SEED] [NONTEMPORAL=1] [COPY_THREADS=-1] [RETAIN_HEAP=1]
//                  [RESERVE=1]
// (RESERVE 1: Session::Reserve sizes the pinned arena before the first flush,
// as an engine does once from its memtable capacity; 0: the first flush grows
// it by doubling.)
// (COPY_THREADS -1: the mirror's default, min(16, cores) or NKV_COPY_THREADS.
// RETAIN_HEAP 1: the process keeps freed memory mapped between flushes, as a Go
// process's garbage-collected heap does; glibc's default hands every block over
// 32 MiB back to the kernel on free, so each flush would page-fault its
// 64 MiB leaves slice and the tree's node storage afresh.  0: glibc defaults.)
#include <fcntl.h>
#include <malloc.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "nkv_merkletree.hpp"

using namespace nkv::merkletree;
using clk = std::chrono::steady_clock;

static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

// byte j = byte (j % 8) of splitmix64(seed, j / 8), as oracle/merkle_oracle.c
static void fill(uint8_t* out, uint64_t n, uint64_t seed, int threads) {
    std::vector<std::thread> th;
    const uint64_t words = (n + 7) / 8, per = (words + threads - 1) / threads;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([=] {
            for (uint64_t w = uint64_t(t) * per; w < std::min(words, uint64_t(t + 1) * per); ++w) {
                uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
                z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
                z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
                z ^= z >> 31;
                for (uint64_t b = 0; b < 8 && 8 * w + b < n; ++b) out[8 * w + b] = uint8_t(z >> (8 * b));
            }
        });
    for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s N VLEN CYCLES DIR [STREAMING] [SEED] [NONTEMPORAL]\n", argv[0]);
        return 2;
    }
    const uint64_t n = std::strtoull(argv[1], nullptr, 10), vlen = std::strtoull(argv[2], nullptr, 10);
    const int cycles = std::atoi(argv[3]);
    const std::string dir = argv[4];
    const bool streaming = argc > 5 ? std::atoi(argv[5]) != 0 : true;
    const uint64_t seed = argc > 6 ? std::strtoull(argv[6], nullptr, 0) : 0x6E616B65ull;
    const bool nontemporal = argc > 7 ? std::atoi(argv[7]) != 0 : true;
    const int copy_threads = argc > 8 ? std::atoi(argv[8]) : -1;
    const bool retain_heap = argc > 9 ? std::atoi(argv[9]) != 0 : true;
    const bool reserve = argc > 10 ? std::atoi(argv[10]) != 0 : true;
    if (retain_heap) {
        mallopt(M_MMAP_THRESHOLD, 1 << 30);  // large blocks from the heap, not fresh mappings
        mallopt(M_TRIM_THRESHOLD, -1);       // and the heap is not trimmed on free
    }
    std::vector<uint8_t> memtable(n * vlen);
    fill(memtable.data(), memtable.size(), seed, 16);
    Session& S = Session::Default();
    S.SetStreaming(streaming);
    S.SetNonTemporal(nontemporal);
    if (copy_threads >= 0) S.SetCopyThreads(copy_threads);
    check(nkv_ctx_set_timing(S.ctx(), NKV_TIMING_EVENTS), "timing");
    // RESERVE 1: the engine sizes the arena once at start from the memtable's
    // capacity (what the Go shim's merkletree.Reserve does from coreconf's
    // MEMTABLE_THRESHOLD), outside any flush; 0: the first flush grows it
    const auto r0 = clk::now();
    if (reserve) S.Reserve(n * ((vlen + 15) & ~uint64_t(15)));
    const double reserve_ms = ms(r0, clk::now());
    for (int cyc = 0; cyc < cycles; ++cyc) {
        const std::string fname = dir + "/api_flush-1-" + std::to_string(cyc) + "-metadata.db";
        unlink(fname.c_str());
        const auto t0 = clk::now();
        std::vector<MerkleNode> leaves;
        leaves.reserve(n);
        for (uint64_t i = 0; i < n; ++i) leaves.push_back(NewLeaf(memtable.data() + i * vlen, vlen));
        const auto t1 = clk::now();
        std::string err;
        auto tree = New(std::move(leaves), &err);
        if (!tree) {
            std::fprintf(stderr, "New: %s\n", err.c_str());
            return 1;
        }
        const auto t2 = clk::now();
        const std::string root = tree->Root->String();
        const auto t3 = clk::now();
        tree->Serialize(fname);  // the walk of the live tree + the file write
        const auto t5 = clk::now();
        const auto& st = tree->LastSerializeTiming();
        float up = -1, ker = -1, down = -1;
        if (nkv_ctx_last_host_timing(S.ctx(), &up, &ker, &down) != NKV_OK) up = ker = down = -1;
        const double total = ms(t0, t5);
        std::printf(
            "{\"cycle\": %d, \"n\": %llu, \"value_bytes\": %llu, \"streaming\": %d, \"nontemporal\": %d, "
            "\"copy_threads\": %d, \"retain_heap\": %d, \"gib_s\": %.3f, "
            "\"total_ms\": %.3f, \"newleaf_ms\": %.3f, \"new_call_ms\": %.3f, \"upload_ms\": %.3f, "
            "\"kernels_ms\": %.3f, \"download_ms\": %.3f, \"materialize_ms\": %.3f, \"root_ms\": %.3f, "
            "\"walk_ms\": %.3f, \"write_ms\": %.3f, \"image_bytes\": %zu, \"arena_allocs\": %llu, "
            "\"reserve\": %d, \"reserve_ms\": %.3f, \"root\": \"%s\"}\n",
            cyc, (unsigned long long)n, (unsigned long long)vlen, int(streaming), int(nontemporal), S.CopyThreads(), int(retain_heap),
            double(n * vlen) / (total * 1e-3) / double(1ull << 30), total, ms(t0, t1),
            tree->LastNewTiming().call_ms, up, ker, down, tree->LastNewTiming().materialize_ms, ms(t2, t3),
            st.walk_ms, st.write_ms, size_t(st.bytes), (unsigned long long)S.arena_allocs(), int(reserve),
            reserve_ms, root.c_str());
        std::fflush(stdout);
    }
    return 0;
}
