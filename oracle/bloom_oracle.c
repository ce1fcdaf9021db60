/* bloom_oracle.c -- TEST INFRASTRUCTURE ONLY (tests/, bench tools' CPU leg).
 * Never linked into or called by the product path.
 *
 * CPU restatement of the SSTable filter build of magley/nakevaleng:
 *   sstable.makeFilter        core/sstable/sstable.go:49-56  bloomfilter.New(len(keyctx), 0.01),
 *                                                            Insert(kc.Key) for every key
 *   calculateM / calculateK   ds/bloomfilter/bloomfilter.go:18-24
 *   createHashFunctions       ds/bloomfilter/bloomfilter.go:28-39  seeds t, t+1, .., t+k-1
 *   (*BloomFilter).Insert     ds/bloomfilter/bloomfilter.go:76-91  bit murmur3(seed_i, key) % M,
 *                                                            Contents[idx/8] |= 1 << (idx%8)
 *   (*BloomFilter).Query      ds/bloomfilter/bloomfilter.go:93-111
 * The hash is the third-party github.com/spaolacci/murmur3 v1.1.0 (go.mod:7,
 * not under /root/reference): New32WithSeed + Write + Sum32 is MurmurHash3_x86_32
 * (Austin Appleby's published algorithm), restated here.  Pinned by the
 * published MurmurHash3_x86_32 vectors and by scikit-learn's murmurhash3_32
 * (Appleby's C code) in tests/test_oracle.py.  The reference's seed t is
 * uint32(time.Now().UnixNano()), so a filter is reproducible only with the
 * seed given explicitly (here and in the C-ABI).  calculateM/K use C's libm
 * log/pow where Go uses its own math.Log/math.Pow: equal except possibly in
 * the last ulp, which matters only if a product lands exactly on an integer.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

uint32_t nkvo_murmur3_32(const uint8_t *data, uint64_t len, uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h = seed;
    const uint64_t nblocks = len / 4;
    for (uint64_t i = 0; i < nblocks; ++i) {
        uint32_t k;
        memcpy(&k, data + 4 * i, 4); /* little endian */
        k *= c1;
        k = rotl32(k, 15);
        k *= c2;
        h ^= k;
        h = rotl32(h, 13);
        h = h * 5 + 0xe6546b64u;
    }
    const uint8_t *tail = data + 4 * nblocks;
    uint32_t k1 = 0;
    switch (len & 3) {
        case 3: k1 ^= (uint32_t)tail[2] << 16; /* fall through */
        case 2: k1 ^= (uint32_t)tail[1] << 8;  /* fall through */
        case 1:
            k1 ^= tail[0];
            k1 *= c1;
            k1 = rotl32(k1, 15);
            k1 *= c2;
            h ^= k1;
    }
    h ^= (uint32_t)len; /* Go: h1 ^= uint32(d.clen) */
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

/* bloomfilter.New sizing (bloomfilter.go:18-24).  n must be > 0. */
void nkvo_bloom_params(uint64_t n, double p, uint32_t *m, uint32_t *k) {
    const double ln2 = log(2.0);
    *m = (uint32_t)ceil((double)n * fabs(log(p)) / pow(ln2, 2.0));
    *k = (uint32_t)ceil(((double)*m / (double)n) * ln2);
}

/* Insert every key (base + off[i], len[i]) with k hashes seeded seed0 + j into
 * bits (ceil(m / 8) bytes, OR-ed). */
void nkvo_bloom_insert(const uint8_t *base, const uint64_t *off, const uint64_t *len, uint64_t n, uint32_t m,
                       uint32_t k, uint32_t seed0, uint8_t *bits) {
    for (uint64_t i = 0; i < n; ++i)
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t idx = nkvo_murmur3_32(base + off[i], len[i], seed0 + j) % m;
            bits[idx / 8] |= (uint8_t)(1u << (idx % 8));
        }
}

/* Query (bloomfilter.go:93-111): out[i] = 1 if every bit of key i is set. */
void nkvo_bloom_query(const uint8_t *base, const uint64_t *off, const uint64_t *len, uint64_t n, uint32_t m,
                      uint32_t k, uint32_t seed0, const uint8_t *bits, uint8_t *out) {
    for (uint64_t i = 0; i < n; ++i) {
        uint8_t hit = 1;
        for (uint32_t j = 0; j < k && hit; ++j) {
            const uint32_t idx = nkvo_murmur3_32(base + off[i], len[i], seed0 + j) % m;
            if (!(bits[idx / 8] & (1u << (idx % 8)))) hit = 0;
        }
        out[i] = hit;
    }
}
