// CPU test of the C++ mirror's host thread team (include/nkv_merkletree.hpp,
// TaskTeam): every part of every Run is executed exactly once, runs of any
// size back to back (a worker that wakes late for a finished run must not
// touch the next one), and the team shuts down cleanly.
#include <atomic>
#include <cstdio>
#include <vector>

#include "nkv_merkletree.hpp"

#include <cstdlib>

int main(int argc, char** argv) {
    const int runs = argc > 1 ? std::atoi(argv[1]) : 20000;
    for (int threads : {1, 2, 3, 8}) {
        nkv::merkletree::TaskTeam team(threads);
        std::vector<std::atomic<int>> hits(257);
        for (int run = 0; run < runs; ++run) {
            const int parts = run % 257;
            for (int k = 0; k < parts; ++k) hits[k].store(0);
            team.Run(parts, [&](int k) { hits[k].fetch_add(1); });
            for (int k = 0; k < parts; ++k)
                if (hits[k].load() != 1) {
                    std::printf("bad: threads %d run %d part %d hit %d times\n", threads, run, k, hits[k].load());
                    return 1;
                }
        }
    }
    std::printf("ok\n");
    return 0;
}
