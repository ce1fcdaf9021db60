// CPU check of the C++ mirror's arena copy (Session::CopyIn: non-temporal
// stores for values of kStreamCopy bytes or more, memcpy below): every length
// 0..1100 and a 64 KiB value, from every source offset 0..15, into 16-byte
// aligned places; the bytes after each copy stay untouched.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "nkv_merkletree.hpp"

int main() {
    using nkv::merkletree::Session;
    std::vector<uint8_t> src(70000 + 64);
    for (size_t i = 0; i < src.size(); ++i) src[i] = uint8_t(i * 131u + 7u);
    alignas(64) static uint8_t dst[70000 + 256];
    std::vector<size_t> lens;
    for (size_t n = 0; n <= 1100; ++n) lens.push_back(n);
    lens.push_back(4096);
    lens.push_back(65536);
    lens.push_back(65536 + 13);
    for (size_t n : lens)
        for (size_t so = 0; so < 16; ++so)
            for (size_t dof = 0; dof < 64; dof += 16) {
                std::memset(dst, 0xEE, sizeof dst);
                Session::CopyIn(dst + dof, src.data() + so, n);
                Session::Fence();
                if (std::memcmp(dst + dof, src.data() + so, n) != 0) {
                    std::printf("FAIL copy n=%zu src+%zu dst+%zu\n", n, so, dof);
                    return 1;
                }
                for (size_t k = 0; k < 64; ++k)
                    if (dst[dof + n + k] != 0xEE || (dof && dst[dof - 1] != 0xEE)) {
                        std::printf("FAIL bounds n=%zu src+%zu dst+%zu\n", n, so, dof);
                        return 1;
                    }
            }
    std::printf("ok %zu\n", lens.size());
    return 0;
}
