/*
 * merkle_openssl.c -- the CPU baseline's strongest variant: ds/merkletree's
 * leaf hash and tree build with OpenSSL's SHA-1 (libcrypto, SHA-NI where the
 * host has it), on one thread or on every core this process may use.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (nakevaleng_amd/, include/)
 * links, loads or calls this file.  Only tests/ and bench.py's cpu_baseline leg
 * use it: as the fastest CPU comparator SURVEY.md 8(d) asks for ("SHA-1 via
 * the portable scalar oracle and via OpenSSL EVP (SHA-NI if present)", single
 * thread and all host cores).  Go's crypto/sha1 (the reference's hash,
 * ds/merkletree/merklenode.go:28, merkletree.go:46) is assembly on amd64, so a
 * library SHA-1 is the honest stand-in for the reference's per-core rate.
 *
 * The tree follows the same statements as merkle_oracle.c
 * (ds/merkletree/merkletree.go:31-64: an odd level's lone node is hashed with
 * the empty pad, i.e. SHA-1 of its 20 bytes; at least one level above the
 * leaves); tests/test_oracle.py checks both files against each other and the
 * FIPS 180-4 known answers.
 */
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* The low-level SHA1_Init / _Update / _Final: straight into libcrypto's block
 * function (SHA-NI where present).  The one-shot SHA1() of OpenSSL 3 goes
 * through EVP_Q_digest, which fetches the algorithm from the provider on every
 * call under a library lock: measured on the GPU host, 16 threads then hashed
 * no faster than one (1.88 GiB/s) and a 200-byte message cost 3 us more. */
static inline void sha1_ll(const uint8_t *data, size_t len, uint8_t out[20]) {
    SHA_CTX c;
    SHA1_Init(&c);
    SHA1_Update(&c, data, len);
    SHA1_Final(out, &c);
}

void nkvo_ossl_sha1(const uint8_t *data, uint64_t len, uint8_t out[20]) { sha1_ll(data, (size_t)len, out); }

typedef struct {
    const uint8_t *base;
    const uint64_t *off, *len; /* off NULL: strided */
    uint64_t stride, L;
    uint8_t *out;
    uint64_t lo, hi;
    /* tree level job */
    const uint8_t *prev;
    uint64_t pc;
} job;

static void *leaf_worker(void *p) {
    job *j = (job *)p;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        if (j->off)
            sha1_ll(j->base + j->off[i], (size_t)j->len[i], j->out + 20 * i);
        else
            sha1_ll(j->base + j->stride * i, (size_t)j->L, j->out + 20 * i);
    }
    return NULL;
}

/* parents [lo, hi) of one level: SHA-1(l || r), or SHA-1(l) for the lone node
 * whose sibling is the empty pad (merkletree.go:32-34, :44-46) */
static void *level_worker(void *p) {
    job *j = (job *)p;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const int pair = 2 * i + 1 < j->pc;
        sha1_ll(j->prev + 40 * i, pair ? 40 : 20, j->out + 20 * i);
    }
    return NULL;
}

static void run(job proto, uint64_t n, int threads, void *(*fn)(void *)) {
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > n) threads = n ? (int)n : 1;
    if (threads == 1) {
        proto.lo = 0;
        proto.hi = n;
        fn(&proto);
        return;
    }
    pthread_t *tid = calloc((size_t)threads, sizeof *tid);
    job *jobs = calloc((size_t)threads, sizeof *jobs);
    for (int t = 0; t < threads; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        pthread_create(&tid[t], NULL, fn, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid);
    free(jobs);
}

/* NewLeaf over n values: value i = base[off[i] .. off[i]+len[i]) */
void nkvo_ossl_leaf_hashes(const uint8_t *base, const uint64_t *off, const uint64_t *len, uint64_t n,
                           uint8_t *out, int threads) {
    job p = {base, off, len, 0, 0, out, 0, 0, NULL, 0};
    run(p, n, threads, leaf_worker);
}

/* NewLeaf over n values of L bytes at base + i * stride */
void nkvo_ossl_leaf_hashes_strided(const uint8_t *base, uint64_t stride, uint64_t L, uint64_t n, uint8_t *out,
                                   int threads) {
    job p = {base, NULL, NULL, stride, L, out, 0, 0, NULL, 0};
    run(p, n, threads, leaf_worker);
}

/* New + build over level 0 already in nodes (n digests); levels 1..top are
 * written after it, level-major bottom-up (the layout of merkle_oracle.c).
 * Levels of at least 4096 parents are split over the threads.  Returns the
 * number of levels, or -1 for n == 0 (merkletree.go:19-21). */
int nkvo_ossl_tree_from_digests(uint8_t *nodes, uint64_t n, int threads) {
    if (n == 0) return -1;
    uint64_t base = 0, pc = n;
    int lv = 1;
    do {
        const uint64_t cc = (pc + 1) / 2;
        job p = {NULL, NULL, NULL, 0, 0, nodes + 20 * (base + pc), 0, 0, nodes + 20 * base, pc};
        run(p, cc, cc >= 4096 ? threads : 1, level_worker);
        base += pc;
        pc = cc;
        lv++;
    } while (pc > 1);
    return lv;
}
