// small_flush -- the Merkle step at the reference engine's own default sizes,
// through the C++ mirror of the Go API (include/nkv_merkletree.hpp), driven as
// sstable.makeMetadata drives ds/merkletree (core/sstable/sstable.go:58-74):
//
//   for each record: leaves = append(leaves, NewLeaf(rec.Value))   merklenode.go:27-34
//   tree := New(leaves)                                             merkletree.go:18-25
//   root := tree.Root.String(); image := the Serialize bytes        merkletree.go:67-92
//
// The default engine flushes a memtable of MEMTABLE_CAPACITY = 10 records under
// a 2 KB threshold (engine/coreconf/coreconf.go:33-34) and compacts
// LSM_RUN_MAX = 4 such runs (:39), so a flush hashes ~10 values of <= 200 B.
// For each shape, every repetition is one flush; the line reports microseconds
// per flush (median, p10, p90) for:
//   mirror_us   NewLeaf x n + New + Root.String() + the image bytes (no file)
//   file_us     the same + Serialize(fname) (open without O_TRUNC, write, close)
//   abi_us      one nkv_tree_from_values call (root, nodes, image) on the values
//               as they lie in the memtable: the C-ABI's own floor
// with the context's NKV_OPT_SMALL_PATH set to MODE (0 = the grid path, 1 = the
// one-launch kernel reading pinned host memory, 2 = the one launch through HBM,
// 3 = the resident service: no launch per flush; 3h = the same with its
// requests in host memory, NKV_OPT_SERVICE_MAILBOX 1).
//
// Usage: small_flush MODE REPS DIR SHAPE...   SHAPE = N:MINLEN:MAXLEN[:SEED]
// One JSON line per shape; roots in hex so the caller checks them against the
// oracle.
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "nkv_merkletree.hpp"

using namespace nkv::merkletree;
using clk = std::chrono::steady_clock;

static double us(clk::time_point a, clk::time_point b) {
    return std::chrono::duration<double, std::micro>(b - a).count();
}

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Stats {
    double med, p10, p90;
};
static Stats stats(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    auto at = [&](double q) { return v[std::min(v.size() - 1, size_t(q * double(v.size() - 1) + 0.5))]; };
    return {at(0.5), at(0.1), at(0.9)};
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s MODE REPS DIR N:MINLEN:MAXLEN[:SEED]...\n", argv[0]);
        return 2;
    }
    const int mode = std::atoi(argv[1]);
    // "3h": the service with its requests in host memory (NKV_OPT_SERVICE_MAILBOX 1)
    const bool host_mailbox = std::string(argv[1]).find('h') != std::string::npos;
    const int reps = std::max(3, std::atoi(argv[2]));
    const std::string dir = argv[3];
    Session& S = Session::Default();
    check(nkv_ctx_set_option(S.ctx(), NKV_OPT_SMALL_PATH, mode), "NKV_OPT_SMALL_PATH");
    check(nkv_ctx_set_option(S.ctx(), NKV_OPT_SERVICE_MAILBOX, host_mailbox ? 1 : 0), "NKV_OPT_SERVICE_MAILBOX");
    for (int a = 4; a < argc; ++a) {
        unsigned long long n = 0, lo = 0, hi = 0, seed = 0x6E616B67ull;
        if (std::sscanf(argv[a], "%llu:%llu:%llu:%llx", &n, &lo, &hi, &seed) < 3 || n == 0 || hi < lo) {
            std::fprintf(stderr, "bad shape %s\n", argv[a]);
            return 2;
        }
        // the memtable's values: lengths uniform in [lo, hi], splitmix64 bytes,
        // back to back (the caller's own memory, as Go's rec.Value slices)
        uint64_t s = seed;
        std::vector<uint64_t> off(n), len(n);
        uint64_t total = 0;
        for (uint64_t i = 0; i < n; ++i) {
            len[i] = lo + (hi > lo ? splitmix(s) % (hi - lo + 1) : 0);
            off[i] = total;
            total += len[i];
        }
        std::vector<uint8_t> mem(total + 8);
        for (uint64_t j = 0; j < total; j += 8) {
            const uint64_t v = splitmix(s);
            std::memcpy(mem.data() + j, &v, 8);
        }
        const std::string fname = dir + "/small_flush-" + std::to_string(a) + "-metadata.db";
        std::vector<double> t_mirror, t_file, t_abi;
        std::string root_hex;
        std::vector<uint8_t> img_last;
        int path = -1;
        for (int r = 0; r < reps + 3; ++r) {  // 3 warm-up flushes
            const bool keep = r >= 3;
            for (int with_file = 0; with_file < 2; ++with_file) {
                const auto t0 = clk::now();
                std::vector<MerkleNode> leaves;
                leaves.reserve(n);
                for (uint64_t i = 0; i < n; ++i) leaves.push_back(NewLeaf(mem.data() + off[i], len[i]));
                std::string err;
                auto tree = New(std::move(leaves), &err);
                if (!tree) {
                    std::fprintf(stderr, "New: %s\n", err.c_str());
                    return 1;
                }
                root_hex = tree->Root->String();
                if (with_file) {
                    unlink(fname.c_str());
                    tree->Serialize(fname);
                } else {
                    img_last = tree->SerializeBytes();
                }
                const auto t1 = clk::now();
                check(nkv_ctx_last_path(S.ctx(), &path), "nkv_ctx_last_path");
                if (keep) (with_file ? t_file : t_mirror).push_back(us(t0, t1));
            }
            uint8_t root[20];
            const uint64_t tot = nkv_total_nodes(n);
            std::vector<uint8_t> nodes(20 * tot), img(nkv_bfs_size(n));
            const auto a0 = clk::now();
            check(nkv_tree_from_values(S.ctx(), mem.data(), off.data(), len.data(), n, root, nodes.data(),
                                       img.data()),
                  "nkv_tree_from_values");
            const auto a1 = clk::now();
            if (keep) t_abi.push_back(us(a0, a1));
            if (img != img_last) {
                std::fprintf(stderr, "image of the C-ABI call differs from the mirror's\n");
                return 1;
            }
        }
        const Stats m = stats(t_mirror), f = stats(t_file), c = stats(t_abi);
        std::printf(
            "{\"n\": %llu, \"min_len\": %llu, \"max_len\": %llu, \"seed\": \"%#llx\", \"payload_bytes\": %llu, "
            "\"mode\": %d, \"path\": %d, \"reps\": %d, "
            "\"mirror_us\": %.2f, \"mirror_us_p10\": %.2f, \"mirror_us_p90\": %.2f, "
            "\"file_us\": %.2f, \"file_us_p10\": %.2f, \"file_us_p90\": %.2f, "
            "\"abi_us\": %.2f, \"abi_us_p10\": %.2f, \"abi_us_p90\": %.2f, "
            "\"image_bytes\": %zu, \"root\": \"%s\"}\n",
            n, lo, hi, seed, (unsigned long long)total, mode, path, reps, m.med, m.p10, m.p90, f.med, f.p10, f.p90,
            c.med, c.p10, c.p90, img_last.size(), root_hex.c_str());
        std::fflush(stdout);
    }
    return 0;
}
