/*
 * merkle_oracle.c -- CPU restatement of magley/nakevaleng ds/merkletree.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (nakevaleng_amd/, include/)
 * links, loads or calls this file.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * Parity status: the SHA-1 primitive is pinned by FIPS 180-4 known answers
 * (tests/test_oracle.py).  The tree layer is "parity unpinned": the reference
 * is Go, no Go toolchain exists in this image, and the reference ships no
 * tests, fixtures or golden vectors for ds/merkletree (SURVEY.md section 4,
 * 8c).  This file is cross-checked against an independent literal Python
 * restatement of the Go pointer tree (oracle/merkle_ref.py, hashlib SHA-1).
 *
 * What each function restates (paths relative to the reference root):
 *   nkvo_sha1                 Go stdlib crypto/sha1 Sum, as called by
 *                             ds/merkletree/merklenode.go:27-34 (NewLeaf) and
 *                             ds/merkletree/merkletree.go:44-46 (build).
 *   nkvo_tree_from_digests    ds/merkletree/merkletree.go:18-64 (New + build):
 *                             odd level -> append an EMPTY node (:32-34), so a
 *                             lone node's parent is SHA-1(left || "") ; recurse
 *                             until the NEW level has one node (:59-63), hence
 *                             at least one level above the leaves.
 *   nkvo_tree_generic         the same with leaves of arbitrary Data length
 *                             (README example ds/merkletree/README.md:44-57).
 *   nkvo_bfs_image            ds/merkletree/merkletree.go:67-92 + merklenode.go:37-63
 *                             (BFS order, 0x00+Data for real nodes, 0x01 alone
 *                             for an empty node, MERKLE_NODE_EMPTY merklenode.go:11).
 *   nkvo_splitmix64_fill      synthetic input generator shared with the GPU
 *                             bench (not a reference function).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

/* ---------------- portable FIPS 180-4 SHA-1 ---------------- */

static inline uint32_t rol32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* Scalar FIPS 180-4 compression with a rolling 16-word schedule and the 80
 * rounds fully unrolled (a restatement, written independently of Go's
 * crypto/sha1 block function). */
static inline uint32_t ld_be32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return __builtin_bswap32(v);
}

#define SHA1_W(t) (w[(t) & 15] = rol32(w[((t) + 13) & 15] ^ w[((t) + 8) & 15] ^ w[((t) + 2) & 15] ^ w[(t) & 15], 1))
#define SHA1_R(a, b, c, d, e, f, k, x)                 \
    do {                                             \
        e += rol32(a, 5) + (f) + (k) + (x);          \
        b = rol32(b, 30);                            \
    } while (0)
#define F1(b, c, d) (d ^ (b & (c ^ d)))
#define F2(b, c, d) (b ^ c ^ d)
#define F3(b, c, d) ((b & c) | (d & (b | c)))

static void sha1_compress(uint32_t h[5], const uint8_t blk[64]) {
    uint32_t w[16];
    for (int t = 0; t < 16; t++) w[t] = ld_be32(blk + 4 * t);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#define R5(F, K, X0, X1, X2, X3, X4)            \
    SHA1_R(a, b, c, d, e, F(b, c, d), K, X0);    \
    SHA1_R(e, a, b, c, d, F(a, b, c), K, X1);    \
    SHA1_R(d, e, a, b, c, F(e, a, b), K, X2);    \
    SHA1_R(c, d, e, a, b, F(d, e, a), K, X3);    \
    SHA1_R(b, c, d, e, a, F(c, d, e), K, X4)
    R5(F1, 0x5A827999u, w[0], w[1], w[2], w[3], w[4]);
    R5(F1, 0x5A827999u, w[5], w[6], w[7], w[8], w[9]);
    R5(F1, 0x5A827999u, w[10], w[11], w[12], w[13], w[14]);
    R5(F1, 0x5A827999u, w[15], SHA1_W(16), SHA1_W(17), SHA1_W(18), SHA1_W(19));
    R5(F2, 0x6ED9EBA1u, SHA1_W(20), SHA1_W(21), SHA1_W(22), SHA1_W(23), SHA1_W(24));
    R5(F2, 0x6ED9EBA1u, SHA1_W(25), SHA1_W(26), SHA1_W(27), SHA1_W(28), SHA1_W(29));
    R5(F2, 0x6ED9EBA1u, SHA1_W(30), SHA1_W(31), SHA1_W(32), SHA1_W(33), SHA1_W(34));
    R5(F2, 0x6ED9EBA1u, SHA1_W(35), SHA1_W(36), SHA1_W(37), SHA1_W(38), SHA1_W(39));
    R5(F3, 0x8F1BBCDCu, SHA1_W(40), SHA1_W(41), SHA1_W(42), SHA1_W(43), SHA1_W(44));
    R5(F3, 0x8F1BBCDCu, SHA1_W(45), SHA1_W(46), SHA1_W(47), SHA1_W(48), SHA1_W(49));
    R5(F3, 0x8F1BBCDCu, SHA1_W(50), SHA1_W(51), SHA1_W(52), SHA1_W(53), SHA1_W(54));
    R5(F3, 0x8F1BBCDCu, SHA1_W(55), SHA1_W(56), SHA1_W(57), SHA1_W(58), SHA1_W(59));
    R5(F2, 0xCA62C1D6u, SHA1_W(60), SHA1_W(61), SHA1_W(62), SHA1_W(63), SHA1_W(64));
    R5(F2, 0xCA62C1D6u, SHA1_W(65), SHA1_W(66), SHA1_W(67), SHA1_W(68), SHA1_W(69));
    R5(F2, 0xCA62C1D6u, SHA1_W(70), SHA1_W(71), SHA1_W(72), SHA1_W(73), SHA1_W(74));
    R5(F2, 0xCA62C1D6u, SHA1_W(75), SHA1_W(76), SHA1_W(77), SHA1_W(78), SHA1_W(79));
#undef R5
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

void nkvo_sha1(const uint8_t *data, uint64_t len, uint8_t out[20]) {
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    uint64_t full = len / 64;
    for (uint64_t i = 0; i < full; i++) sha1_compress(h, data + 64 * i);
    uint8_t tail[128];
    uint64_t rem = len - 64 * full;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, data + 64 * full, rem);
    tail[rem] = 0x80;
    uint64_t tl = (rem < 56) ? 64 : 128;
    uint64_t bits = len * 8;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha1_compress(h, tail);
    if (tl == 128) sha1_compress(h, tail + 64);
    for (int i = 0; i < 5; i++) {
        out[4 * i] = (uint8_t)(h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8);
        out[4 * i + 3] = (uint8_t)h[i];
    }
}

/* ---------------- synthetic input generator ---------------- */

static inline uint64_t splitmix64_at(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* byte j of the stream = byte (j % 8) (little endian) of splitmix64_at(seed, j / 8) */
void nkvo_splitmix64_fill(uint8_t *buf, uint64_t nbytes, uint64_t seed) {
    uint64_t nw = nbytes / 8;
    for (uint64_t k = 0; k < nw; k++) {
        uint64_t v = splitmix64_at(seed, k);
        memcpy(buf + 8 * k, &v, 8); /* host is little endian (x86-64) */
    }
    if (nbytes % 8) {
        uint64_t v = splitmix64_at(seed, nw);
        memcpy(buf + 8 * nw, &v, nbytes % 8);
    }
}

/* the same stream from byte `first` (a multiple of 8) on: bytes [first, first + nbytes) */
void nkvo_splitmix64_fill_at(uint8_t *buf, uint64_t nbytes, uint64_t seed, uint64_t first) {
    const uint64_t k0 = first / 8, nw = nbytes / 8;
    for (uint64_t k = 0; k < nw; k++) {
        uint64_t v = splitmix64_at(seed, k0 + k);
        memcpy(buf + 8 * k, &v, 8);
    }
    if (nbytes % 8) {
        uint64_t v = splitmix64_at(seed, k0 + nw);
        memcpy(buf + 8 * nw, &v, nbytes % 8);
    }
}

/* ---------------- leaf hashing (NewLeaf) ---------------- */

typedef struct {
    const uint8_t *base;
    const uint64_t *off, *len;
    uint64_t stride, L;
    uint64_t lo, hi;
    uint8_t *out;
} leaf_job;

static void *leaf_worker(void *p) {
    leaf_job *j = (leaf_job *)p;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        if (j->off)
            nkvo_sha1(j->base + j->off[i], j->len[i], j->out + 20 * i);
        else
            nkvo_sha1(j->base + j->stride * i, j->L, j->out + 20 * i);
    }
    return NULL;
}

static void run_leaf_jobs(leaf_job proto, uint64_t n, int threads) {
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > n) threads = n ? (int)n : 1;
    pthread_t *tid = calloc(threads, sizeof *tid);
    leaf_job *jobs = calloc(threads, sizeof *jobs);
    for (int t = 0; t < threads; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * t / threads;
        jobs[t].hi = n * (t + 1) / threads;
        if (threads == 1) leaf_worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, leaf_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid);
    free(jobs);
}

/* NewLeaf over n values: value i = base[off[i] .. off[i]+len[i]) */
void nkvo_leaf_hashes(const uint8_t *base, const uint64_t *off, const uint64_t *len, uint64_t n,
                      uint8_t *out, int threads) {
    leaf_job p = {base, off, len, 0, 0, 0, 0, out};
    run_leaf_jobs(p, n, threads);
}

/* NewLeaf over n values of length L at base + i*stride */
void nkvo_leaf_hashes_strided(const uint8_t *base, uint64_t stride, uint64_t L, uint64_t n,
                              uint8_t *out, int threads) {
    leaf_job p = {base, NULL, NULL, stride, L, 0, 0, out};
    run_leaf_jobs(p, n, threads);
}

/* ---------------- tree shape (merkletree.go:31-64) ---------------- */

/* Number of levels including the leaf level.  build() always produces at
 * least one level above the leaves (the loop tests the NEW level, :59). */
int nkvo_num_levels(uint64_t n) {
    if (n == 0) return 0;
    int lv = 1;
    uint64_t c = n;
    do { c = (c + 1) / 2; lv++; } while (c > 1);
    return lv;
}

/* counts[L] = real nodes at level L (pads excluded), L = 0 is the leaf level */
int nkvo_level_counts(uint64_t n, uint64_t *counts, int cap) {
    int lv = nkvo_num_levels(n);
    if (lv > cap) return -1;
    uint64_t c = n;
    for (int L = 0; L < lv; L++) { counts[L] = c; c = (c + 1) / 2; }
    return lv;
}

uint64_t nkvo_total_nodes(uint64_t n) {
    uint64_t counts[72];
    int lv = nkvo_level_counts(n, counts, 72);
    uint64_t s = 0;
    for (int L = 0; L < lv; L++) s += counts[L];
    return s;
}

/* parent from two 20-byte children, or from a lone one (the empty pad adds
 * nothing to the concatenation, merkletree.go:44-46) */
static void parent20(const uint8_t *l, const uint8_t *r, uint8_t *out) {
    uint8_t buf[40];
    memcpy(buf, l, 20);
    if (r) { memcpy(buf + 20, r, 20); nkvo_sha1(buf, 40, out); }
    else nkvo_sha1(buf, 20, out);
}

/* nodes: level-major, bottom-up; level 0 (n digests) must already be filled.
 * Levels 1..top are written after it.  Returns the number of levels. */
int nkvo_tree_from_digests(uint8_t *nodes, uint64_t n) {
    uint64_t counts[72];
    int lv = nkvo_level_counts(n, counts, 72);
    if (lv <= 0) return -1; /* merkletree.go:19-21: cannot build from 0 nodes */
    uint64_t base = 0;
    for (int L = 1; L < lv; L++) {
        uint64_t pc = counts[L - 1];
        uint8_t *prev = nodes + 20 * base;
        uint8_t *cur = prev + 20 * pc;
        for (uint64_t i = 0; i < counts[L]; i++)
            parent20(prev + 40 * i, (2 * i + 1 < pc) ? prev + 40 * i + 20 : NULL, cur + 20 * i);
        base += pc;
    }
    return lv;
}

/* The same tree with each level of at least 4096 parents split over `threads`
 * (the all-cores CPU baseline, SURVEY.md 8(d) variant 2: "std::thread over
 * leaf ranges + parallel levels").  Same bytes as nkvo_tree_from_digests. */
typedef struct {
    const uint8_t *prev;
    uint8_t *cur;
    uint64_t pc, lo, hi;
} level_job;

static void *level_worker(void *p) {
    level_job *j = (level_job *)p;
    for (uint64_t i = j->lo; i < j->hi; i++)
        parent20(j->prev + 40 * i, (2 * i + 1 < j->pc) ? j->prev + 40 * i + 20 : NULL, j->cur + 20 * i);
    return NULL;
}

int nkvo_tree_from_digests_mt(uint8_t *nodes, uint64_t n, int threads) {
    uint64_t counts[72];
    int lv = nkvo_level_counts(n, counts, 72);
    if (lv <= 0) return -1;
    if (threads < 1) threads = 1;
    pthread_t *tid = calloc((size_t)threads, sizeof *tid);
    level_job *jobs = calloc((size_t)threads, sizeof *jobs);
    uint64_t base = 0;
    for (int L = 1; L < lv; L++) {
        const uint64_t pc = counts[L - 1], cc = counts[L];
        uint8_t *prev = nodes + 20 * base;
        const int t = cc >= 4096 ? threads : 1;
        for (int k = 0; k < t; k++) {
            jobs[k] = (level_job){prev, prev + 20 * pc, pc, cc * (uint64_t)k / (uint64_t)t,
                                  cc * (uint64_t)(k + 1) / (uint64_t)t};
            if (t == 1) level_worker(&jobs[k]);
            else pthread_create(&tid[k], NULL, level_worker, &jobs[k]);
        }
        if (t > 1)
            for (int k = 0; k < t; k++) pthread_join(tid[k], NULL);
        base += pc;
    }
    free(tid);
    free(jobs);
    return lv;
}

/* New() with leaves of arbitrary Data: leaf i = data[off[i] .. +len[i]).
 * upper: levels 1..top (20 bytes each), level-major bottom-up. */
int nkvo_tree_generic(const uint8_t *data, const uint64_t *off, const uint64_t *len, uint64_t n,
                      uint8_t *upper) {
    uint64_t counts[72];
    int lv = nkvo_level_counts(n, counts, 72);
    if (lv <= 0) return -1;
    uint64_t maxlen = 0;
    for (uint64_t i = 0; i < n; i++) if (len[i] > maxlen) maxlen = len[i];
    uint8_t *buf = malloc(2 * maxlen + 1);
    for (uint64_t i = 0; i < counts[1]; i++) {
        uint64_t l = 2 * i, r = 2 * i + 1, m = len[l];
        memcpy(buf, data + off[l], len[l]);
        if (r < n) { memcpy(buf + m, data + off[r], len[r]); m += len[r]; }
        nkvo_sha1(buf, m, upper + 20 * i);
    }
    free(buf);
    uint64_t base = 0;
    for (int L = 2; L < lv; L++) {
        uint64_t pc = counts[L - 1];
        uint8_t *prev = upper + 20 * base;
        uint8_t *cur = prev + 20 * pc;
        for (uint64_t i = 0; i < counts[L]; i++)
            parent20(prev + 40 * i, (2 * i + 1 < pc) ? prev + 40 * i + 20 : NULL, cur + 20 * i);
        base += pc;
    }
    return lv;
}

/* BFS image size for 20-byte leaves: every real node 21 bytes, one 0x01 pad
 * byte for every odd level below the top. */
uint64_t nkvo_bfs_size(uint64_t n) {
    uint64_t counts[72];
    int lv = nkvo_level_counts(n, counts, 72);
    if (lv <= 0) return 0;
    uint64_t s = 0;
    for (int L = 0; L < lv; L++) {
        s += 21 * counts[L];
        if (L < lv - 1 && (counts[L] & 1)) s += 1;
    }
    return s;
}

/* ---------------- CPU timing of one small flush (bench.py small_flush) ----------------
 * `reps` flushes of the n values on the calling thread, each the whole Merkle
 * step of sstable.makeMetadata (core/sstable/sstable.go:58-74) in memory:
 * NewLeaf per value, New/build, the Serialize image -- fresh buffers per
 * flush, as Go allocates them.  fn: the SHA-1 to use (NULL: this file's
 * portable one; bench.py passes OpenSSL's from liboracle_ossl.so).  Returns the
 * total seconds; root20: the last flush's root. */
typedef void (*nkvo_sha1_fn)(const uint8_t *, uint64_t, uint8_t *);
uint64_t nkvo_bfs_image(const uint8_t *nodes, uint64_t n, uint8_t *img);

double nkvo_flush_reps(const uint8_t *base, const uint64_t *off, const uint64_t *len, uint64_t n, int reps,
                       nkvo_sha1_fn fn, uint8_t *root20) {
    if (n == 0 || reps < 1) return 0.0;
    if (!fn) fn = nkvo_sha1;
    const uint64_t total = nkvo_total_nodes(n), isz = nkvo_bfs_size(n);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) {
        uint8_t *nodes = malloc(20 * total), *img = malloc(isz);
        for (uint64_t i = 0; i < n; i++) fn(base + off[i], len[i], nodes + 20 * i);
        uint64_t b = 0, pc = n;
        do {
            const uint64_t cc = (pc + 1) / 2;
            uint8_t *prev = nodes + 20 * b, *cur = prev + 20 * pc;
            for (uint64_t i = 0; i < cc; i++) fn(prev + 40 * i, 2 * i + 1 < pc ? 40 : 20, cur + 20 * i);
            b += pc;
            pc = cc;
        } while (pc > 1);
        nkvo_bfs_image(nodes, n, img);
        if (r == reps - 1 && root20) memcpy(root20, nodes + 20 * (total - 1), 20);
        free(nodes);
        free(img);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* BFS image from level-major nodes (20-byte leaves).  Returns bytes written. */
uint64_t nkvo_bfs_image(const uint8_t *nodes, uint64_t n, uint8_t *img) {
    uint64_t counts[72], start[72];
    int lv = nkvo_level_counts(n, counts, 72);
    if (lv <= 0) return 0;
    uint64_t s = 0;
    for (int L = 0; L < lv; L++) { start[L] = s; s += counts[L]; }
    uint64_t p = 0;
    for (int L = lv - 1; L >= 0; L--) {
        for (uint64_t i = 0; i < counts[L]; i++) {
            img[p++] = 0x00;
            memcpy(img + p, nodes + 20 * (start[L] + i), 20);
            p += 20;
        }
        if (L < lv - 1 && (counts[L] & 1)) img[p++] = 0x01;
    }
    return p;
}
