// CPU test: the C++ mirror's process-wide Session is shared by
// every tree, so finished trees may be serialized and destroyed on several
// threads at once, as Go allows.  Two or more threads each, many times:
// Deserialize a tree from an image file (no device needed: the session's
// context is created on first use only), Serialize it to a file of its own,
// check the bytes, destroy the tree (its node storage and level array go back
// to the session); meanwhile they call the host team directly with runs of
// many parts.  Every part of every run must execute exactly once.  Built with
// and without ThreadSanitizer (tests/test_cpp_api.py).
//
// Usage: test_session_threads DIR ITERATIONS
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <string>
#include <thread>
#include <vector>

#include "nkv_merkletree.hpp"

using namespace nkv::merkletree;

static std::vector<uint8_t> read_file(const std::string& f) {
    std::ifstream in(f, std::ios::binary);
    return std::vector<uint8_t>(std::istreambuf_iterator<char>(in), {});
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const std::string dir = argv[1];
    const int iters = std::atoi(argv[2]);
    // a BFS image of a 3-leaf tree: root, level 1 (2 nodes), level 0 (3 nodes +
    // the pad byte); Deserialize links the root only (merkletree.go:97-157)
    std::vector<uint8_t> img;
    for (int node = 0; node < 6; ++node) {
        img.push_back(0);
        for (int b = 0; b < 20; ++b) img.push_back(uint8_t(node * 20 + b));
    }
    img.push_back(MERKLE_NODE_EMPTY);
    const std::string src = dir + "/session-src-metadata.db";
    {
        std::ofstream out(src, std::ios::binary);
        out.write(reinterpret_cast<const char*>(img.data()), std::streamsize(img.size()));
    }
    std::vector<uint8_t> root_img(img.begin(), img.begin() + 21);  // the root-only tree writes its root
    const int nthreads = 4;
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        th.emplace_back([&, t] {
            const std::string dst = dir + "/session-" + std::to_string(t) + "-metadata.db";
            std::vector<std::atomic<int>> hits(97);
            for (int i = 0; i < iters; ++i) {
                {
                    MerkleTree tree;
                    tree.Deserialize(src);
                    if (!tree.Root || tree.Root->Left) {
                        bad.fetch_add(1);
                        return;
                    }
                    std::remove(dst.c_str());
                    tree.Serialize(dst);
                    if (read_file(dst) != root_img) bad.fetch_add(1);
                    if (tree.SerializeBytes() != root_img) bad.fetch_add(1);
                }  // destroyed: storage back to the session
                const int parts = 1 + (i * 7 + t) % 96;
                for (int k = 0; k < parts; ++k) hits[k].store(0);
                Session::Default().Team().Run(parts, [&](int k) { hits[k].fetch_add(1); });
                for (int k = 0; k < parts; ++k)
                    if (hits[k].load() != 1) bad.fetch_add(1);
                std::vector<uint8_t> lv = Session::Default().TakeLevels();
                lv.resize(64 + 16 * size_t(t));
                Session::Default().GiveLevels(std::move(lv));
            }
        });
    }
    for (auto& x : th) x.join();
    if (bad.load()) {
        std::printf("bad: %d failures\n", bad.load());
        return 1;
    }
    std::printf("ok %d threads x %d\n", nthreads, iters);
    return 0;
}
