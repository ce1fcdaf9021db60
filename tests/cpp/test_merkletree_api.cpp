// Drives the C++ ds/merkletree mirror (include/nkv_merkletree.hpp) through the
// C-ABI on the GPU and prints "key value" lines that tests/test_cpp_api.py checks
// against the golden fixtures and the oracle.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "nkv_merkletree.hpp"

using nkv::merkletree::MerkleNode;
using nkv::merkletree::MerkleTree;
using nkv::merkletree::New;
using nkv::merkletree::NewLeaf;

static std::string hex(const std::vector<uint8_t>& v) {
    static const char* h = "0123456789abcdef";
    std::string s;
    for (uint8_t b : v) {
        s.push_back(h[b >> 4]);
        s.push_back(h[b & 15]);
    }
    return s;
}

static std::vector<uint8_t> splitmix64_bytes(size_t n, uint64_t seed) {
    std::vector<uint8_t> out(n);
    for (size_t j = 0; j < n; j += 8) {
        uint64_t z = seed + (j / 8 + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        for (size_t b = 0; b < 8 && j + b < n; ++b) out[j + b] = uint8_t(z >> (8 * b));
    }
    return out;
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    // README example (ds/merkletree/README.md:44-57)
    {
        std::vector<MerkleNode> lv;
        for (int i = 1; i <= 7; ++i) lv.emplace_back(std::vector<uint8_t>{uint8_t('0' + i)});
        auto t = New(lv);
        std::printf("readme_root %s\n", t->Root->String().c_str());
        std::printf("readme_bfs %s\n", hex(t->SerializeBytes()).c_str());
        std::printf("readme_validate %d\n", int(t->Validate()));
        t->Serialize(dir + "/readme-1-0-metadata.db");
        MerkleTree t2;
        t2.Deserialize(dir + "/readme-1-0-metadata.db");
        std::printf("readme_deser_root %s\n", t2.Root->String().c_str());
        std::printf("readme_deser_children %d\n", int(t2.Root->Left != nullptr || t2.Root->Right != nullptr));
        std::printf("readme_deser_validate %d\n", int(t2.Validate()));
    }
    // empty level: the reference's error
    {
        std::string err;
        auto t = New({}, &err);
        std::printf("empty_null %d\n", int(t == nullptr));
        std::printf("empty_err %s\n", err.c_str());
    }
    // the flush pattern: NewLeaf per value, then New, then Serialize
    for (uint64_t n : {1ull, 2ull, 3ull, 255ull, 256ull, 257ull, 1000ull, 1025ull, 70001ull}) {
        const size_t vlen = n > 300 ? 64 : 100;
        auto data = splitmix64_bytes(n * vlen, 0x6E616B65ull + n);
        std::vector<MerkleNode> leaves;
        for (uint64_t i = 0; i < n; ++i) leaves.push_back(NewLeaf(data.data() + i * vlen, vlen));
        auto t = New(leaves);
        auto img = t->SerializeBytes();
        std::printf("tree%llu_root %s\n", (unsigned long long)n, t->Root->String().c_str());
        std::printf("tree%llu_bfs_len %zu\n", (unsigned long long)n, img.size());
        std::printf("tree%llu_bfs_head %s\n", (unsigned long long)n,
                    hex(std::vector<uint8_t>(img.begin(), img.begin() + std::min<size_t>(64, img.size()))).c_str());
        std::printf("tree%llu_validate %d\n", (unsigned long long)n, int(t->Validate()));
        if (n == 70001) {  // past the threshold of New's multi-threaded materialization
            FILE* f = std::fopen((dir + "/tree70001.img").c_str(), "wb");
            std::fwrite(img.data(), 1, img.size(), f);
            std::fclose(f);
        }
        // Serialize(file) walks into a reused per-thread buffer (larger after the
        // bigger trees): the file must hold exactly this tree's image
        {
            const std::string fn = dir + "/tree" + std::to_string(n) + "-1-0-metadata.db";
            std::remove(fn.c_str());
            t->Serialize(fn);
            FILE* f = std::fopen(fn.c_str(), "rb");
            std::vector<uint8_t> got(img.size() + 1);
            const size_t k = f ? std::fread(got.data(), 1, got.size(), f) : 0;
            if (f) std::fclose(f);
            got.resize(k);
            std::printf("tree%llu_file_eq %d\n", (unsigned long long)n, int(got == img));
        }
        if (n == 1000) {
            // corrupt one leaf of the materialized tree: Validate must fail
            MerkleNode* leaf = t->Root;
            while (leaf->Left) leaf = leaf->Left;
            leaf->Data.assign(20, 0);
            std::printf("tree1000_corrupt_validate %d\n", int(t->Validate()));
        }
    }
    // leaf Data read before New resolves the pending batch on the GPU
    {
        std::vector<MerkleNode> lv;
        for (int i = 0; i < 10; ++i) lv.push_back(NewLeaf(std::string(size_t(i) * 7, char('a' + i))));
        std::printf("early_leaf3 %s\n", lv[3].String().c_str());
        auto t = New(lv);
        std::printf("early_root %s\n", t->Root->String().c_str());
    }
    // three flush cycles of one memtable size: the pinned arena is allocated by
    // the first and reused by the next two (no nkv_host_alloc after the first)
    {
        auto& S = nkv::merkletree::Session::Default();
        for (int k = 0; k < 3; ++k) {
            const uint64_t n = 4096;
            const size_t vlen = 512;
            auto data = splitmix64_bytes(n * vlen, 0xF1u + uint64_t(k));
            std::vector<MerkleNode> leaves;
            for (uint64_t i = 0; i < n; ++i) leaves.push_back(NewLeaf(data.data() + i * vlen, vlen));
            const uint64_t before = S.arena_allocs();
            auto t = New(leaves);
            std::printf("flush%d_allocs_during %llu\n", k, (unsigned long long)(S.arena_allocs() - before));
            std::printf("flush%d_allocs_total %llu\n", k, (unsigned long long)S.arena_allocs());
            std::printf("flush%d_root %s\n", k, t->Root->String().c_str());
            std::printf("flush%d_validate %d\n", k, int(t->Validate()));
            // children swapped: still New's shape, leaves re-collected in the new order
            std::swap(t->Root->Left, t->Root->Right);
            std::printf("flush%d_swapped_validate %d\n", k, int(t->Validate()));
            std::swap(t->Root->Left, t->Root->Right);
            t->Root->Data[0] ^= 1;  // the stored root no longer matches the leaves
            std::printf("flush%d_bad_root_validate %d\n", k, int(t->Validate()));
        }
    }
    // Serialize walks the live tree (merkletree.go:75-89): Data changed after New
    // (a leaf and an interior node) is what the file holds
    {
        const uint64_t n = 37;
        auto data = splitmix64_bytes(n * 50, 0xAB);
        std::vector<MerkleNode> leaves;
        for (uint64_t i = 0; i < n; ++i) leaves.push_back(NewLeaf(data.data() + i * 50, 50));
        auto t = New(leaves);
        MerkleNode* leaf = t->Root;
        while (leaf->Left) leaf = leaf->Left;
        leaf->Data.assign(20, 0xAB);
        t->Root->Right->Data[0] ^= 0xFF;
        const auto mimg = t->SerializeBytes();
        std::printf("mut_img %s\n", hex(mimg).c_str());
        // Serialize(file) after the 70001-leaf tree: the reused buffer is larger
        // than this image, the file holds only this image's bytes
        const std::string fn = dir + "/mut-1-0-metadata.db";
        std::remove(fn.c_str());
        t->Serialize(fn);
        FILE* f = std::fopen(fn.c_str(), "rb");
        std::vector<uint8_t> got(mimg.size() + 64);
        const size_t k = f ? std::fread(got.data(), 1, got.size(), f) : 0;
        if (f) std::fclose(f);
        got.resize(k);
        std::printf("mut_file_eq %d\n", int(got == mimg));
    }
    // flushes larger than the arena's stream chunk (32 MiB): settled chunks are
    // copied to the device during the NewLeaf loop; odd value sizes land at
    // 16-byte aligned places; streaming off gives the same tree
    {
        auto& S = nkv::merkletree::Session::Default();
        const uint64_t n = 20000;
        std::printf("default_copy_threads %d\n", S.CopyThreads());
        // copy threads: the default pool, the caller's thread (0), a 3-thread
        // pool; the first 4096-byte flush also grows the arena mid-loop with
        // copies queued (Reserve settles them first)
        for (int threads : {-1, 0, 3}) {
            if (threads >= 0) S.SetCopyThreads(threads);
            for (size_t vlen : {size_t(4096), size_t(1001)}) {
                auto data = splitmix64_bytes(n * vlen, 0x5EED + vlen);
                for (int streaming = 1; streaming >= 0; --streaming) {
                    S.SetStreaming(streaming != 0);
                    std::vector<MerkleNode> leaves;
                    for (uint64_t i = 0; i < n; ++i) leaves.push_back(NewLeaf(data.data() + i * vlen, vlen));
                    auto t = New(leaves);
                    std::printf("big%zu_t%d_s%d_root %s\n", vlen, threads, streaming, t->Root->String().c_str());
                }
                S.SetStreaming(true);
            }
            // ragged values 0..4999 bytes (jobs cut mid-run, empty values) and a
            // leaf resolved before New (String() settles the pool first)
            auto data = splitmix64_bytes(uint64_t(5000) * 9000, 0xBADu);
            std::vector<MerkleNode> leaves;
            for (uint64_t i = 0; i < 9000; ++i) leaves.push_back(NewLeaf(data.data() + i * 5000, (i * 37) % 5000));
            std::printf("ragged_t%d_leaf77 %s\n", threads, leaves[77].String().c_str());
            auto t = New(leaves);
            std::printf("ragged_t%d_root %s\n", threads, t->Root->String().c_str());
        }
        S.SetCopyThreads(16);
    }
    // CompactRoots: five Data tables (record.go:191-199) over a group of one GPU
    // (RCCL) and of device 0 twice (copy transport), one host thread per member
    {
        std::vector<nkv::merkletree::DataTable> tabs;
        for (int t = 0; t < 5; ++t) {
            nkv::merkletree::DataTable d;
            const uint64_t recs = 300 + 77 * uint64_t(t), ks = 16, vs = 100 + 13 * uint64_t(t);
            auto bytes = splitmix64_bytes(recs * (ks + vs), 0xC0 + uint64_t(t));
            for (uint64_t r = 0; r < recs; ++r) {
                uint8_t hdr[30] = {};
                std::memcpy(hdr + 14, &ks, 8);
                std::memcpy(hdr + 22, &vs, 8);
                d.data.insert(d.data.end(), hdr, hdr + 30);
                d.data.insert(d.data.end(), bytes.begin() + long(r * (ks + vs)), bytes.begin() + long((r + 1) * (ks + vs)));
                d.rec_size.push_back(30 + ks + vs);
            }
            FILE* f = std::fopen((dir + "/table" + std::to_string(t) + ".bin").c_str(), "wb");
            std::fwrite(d.data.data(), 1, d.data.size(), f);
            std::fclose(f);
            tabs.push_back(std::move(d));
        }
        for (const std::vector<int>& devs : {std::vector<int>{0}, std::vector<int>{0, 0}}) {
            auto roots = nkv::merkletree::CompactRoots(devs, tabs);
            for (size_t t = 0; t < roots.size(); ++t)
                std::printf("compact_g%zu_root%zu %s\n", devs.size(), t,
                            hex(std::vector<uint8_t>(roots[t].begin(), roots[t].end())).c_str());
        }
        nkv::merkletree::Group g1({0});
        std::printf("group1_transport %d\n", nkv_group_transport(g1.get()));
        // every visible GPU (a multi-GPU box): ncclCommInitAll over distinct
        // devices with /opt/rocm's RCCL, as a C++ or Go host loads it
        int cnt = 0;
        if (nkv_device_count(&cnt) == NKV_OK && cnt > 1) {
            std::vector<int> all;
            for (int d = 0; d < cnt; ++d) all.push_back(d);
            nkv::merkletree::Group ga(all);
            std::printf("groupall_size %d\ngroupall_transport %d\n", ga.size(), nkv_group_transport(ga.get()));
            auto roots = nkv::merkletree::CompactRoots(ga, tabs);
            for (size_t t = 0; t < roots.size(); ++t)
                std::printf("compact_gall_root%zu %s\n", t,
                            hex(std::vector<uint8_t>(roots[t].begin(), roots[t].end())).c_str());
        }
    }
    return 0;
}
