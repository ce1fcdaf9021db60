// CPU test of the C++ mirror's host thread team (include/nkv_merkletree.hpp,
// TaskTeam): every part of every Run is executed exactly once, runs of any
// size back to back (a worker that wakes late for a finished run must not
// touch the next one), a part that throws (on whichever thread) reaches the
// caller of Run once every part is done, and the team shuts down cleanly.
#include <atomic>
#include <cstdio>
#include <stdexcept>
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
        // parts 3 and 40 throw: Run still runs every part, then rethrows one of
        // them; the team stays usable
        for (int rep = 0; rep < 200; ++rep) {
            for (int k = 0; k < 64; ++k) hits[k].store(0);
            bool caught = false;
            try {
                team.Run(64, [&](int k) {
                    hits[k].fetch_add(1);
                    if (k == 3 || k == 40) throw std::runtime_error("part failed");
                });
            } catch (const std::runtime_error&) {
                caught = true;
            }
            for (int k = 0; k < 64; ++k)
                if (hits[k].load() != 1) {
                    std::printf("bad: threads %d throwing run part %d hit %d times\n", threads, k, hits[k].load());
                    return 1;
                }
            if (!caught) {
                std::printf("bad: threads %d: the exception was not rethrown\n", threads);
                return 1;
            }
            team.Run(5, [&](int k) { hits[k].fetch_add(1); });
        }
    }
    std::printf("ok\n");
    return 0;
}
