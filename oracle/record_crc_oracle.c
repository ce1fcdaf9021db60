/* record_crc_oracle.c -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py's
 * cpu_baseline leg).  Never linked into or called by the product path.
 *
 * CPU restatement of the record checksum of magley/nakevaleng:
 *   record.New            core/record/record.go:49-52   Crc = crc32.ChecksumIEEE(key ++ value)
 *   (*Record).Deserialize core/record/record.go:163-169 recompute, compare with the stored Crc
 *   byte layout           core/record/record.go:191-204 Crc u32 | Timestamp i64 | Status u8 |
 *                         TypeInfo u8 | KeySize u64 | ValueSize u64 | Key | Value (all LE)
 * The arithmetic is Go's standard library hash/crc32 ChecksumIEEE (not under
 * /root/reference): reflected CRC-32, polynomial 0xEDB88320, init and final XOR
 * 0xFFFFFFFF (ISO-HDLC).  Parity is pinned by the published check value
 * CRC-32("123456789") = 0xCBF43926 and by Python's zlib.crc32 (same algorithm)
 * in tests/test_oracle.py.  Bitwise form on purpose: no table shared with the
 * device code.
 */
#include <stdint.h>
#include <string.h>

uint32_t nkvo_crc32_update(uint32_t crc, const uint8_t *p, uint64_t n) {
    crc = ~crc;
    for (uint64_t i = 0; i < n; ++i) {
        crc ^= p[i];
        for (int k = 0; k < 8; ++k) crc = (crc >> 1) ^ (0xEDB88320u & (0u - (crc & 1u)));
    }
    return ~crc;
}

uint32_t nkvo_crc32(const uint8_t *p, uint64_t n) { return nkvo_crc32_update(0u, p, n); }

static uint64_t ld_le64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

/* Records at stream + rec_off[i]: out_crc[i] = CRC-32 of key ++ value (the
 * contiguous span at +30 of KeySize + ValueSize bytes), out_ok[i] = (it equals
 * the stored Crc at +0).  Returns the number of records whose checksum does not
 * match (record.go:166 panics on the first). */
uint64_t nkvo_record_crcs(const uint8_t *stream, const uint64_t *rec_off, uint64_t n, uint32_t *out_crc,
                          uint8_t *out_ok) {
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t *r = stream + rec_off[i];
        const uint64_t span = ld_le64(r + 14) + ld_le64(r + 22);
        const uint32_t c = nkvo_crc32(r + 30, span);
        uint32_t stored;
        memcpy(&stored, r, 4);
        out_crc[i] = c;
        out_ok[i] = c == stored;
        bad += c != stored;
    }
    return bad;
}

/* ---------------- CPU baseline of the compaction read (bench.py) ----------------
 * The fast CRC forms below time the reference's per-record check on the host
 * (bench.py cpu_baseline for records_verify); the checker above stays the
 * bitwise statement.  Both are pinned against zlib.crc32 and the bitwise form
 * in tests/test_oracle.py.  Go's hash/crc32 ChecksumIEEE runs a PCLMULQDQ
 * folding loop on amd64 (ieeeCLMUL) when the CPU has it, so the "openssl"
 * variant of the baseline uses the same technique (crc32_clmul); the "port"
 * variant uses slicing-by-8 tables (portable C). */
#include <pthread.h>
#include <immintrin.h>

static uint32_t s8_tab[8][256];
static pthread_once_t s8_once = PTHREAD_ONCE_INIT;

static void s8_init(void) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
        s8_tab[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
        for (int t = 1; t < 8; ++t) s8_tab[t][i] = (s8_tab[t - 1][i] >> 8) ^ s8_tab[0][s8_tab[t - 1][i] & 0xFFu];
}

/* the CRC register (already inverted) advanced over n bytes, 8 at a time */
static uint32_t crc_reg_s8(uint32_t reg, const uint8_t *p, uint64_t n) {
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= reg;
        reg = s8_tab[7][lo & 0xFFu] ^ s8_tab[6][(lo >> 8) & 0xFFu] ^ s8_tab[5][(lo >> 16) & 0xFFu] ^
              s8_tab[4][lo >> 24] ^ s8_tab[3][hi & 0xFFu] ^ s8_tab[2][(hi >> 8) & 0xFFu] ^
              s8_tab[1][(hi >> 16) & 0xFFu] ^ s8_tab[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) reg = (reg >> 8) ^ s8_tab[0][(reg ^ *p++) & 0xFFu];
    return reg;
}

uint32_t nkvo_crc32_s8(const uint8_t *p, uint64_t n) {
    pthread_once(&s8_once, s8_init);
    return ~crc_reg_s8(0xFFFFFFFFu, p, n);
}

/* PCLMULQDQ folding of the reflected CRC-32 (Gopal et al., "Fast CRC
 * Computation for Generic Polynomials Using PCLMULQDQ", Intel 2009): four
 * 128-bit lanes folded 64 bytes at a time by x^(512+-32) mod P, folded to one
 * lane, reduced to 64 then 32 bits, Barrett reduction to the register.  The
 * constants are the bit-reflected x^k mod P (P = 0x104C11DB7) and
 * floor(x^64 / P); n >= 64. */
__attribute__((target("pclmul,sse4.1"))) static uint32_t crc_reg_clmul(uint32_t reg, const uint8_t *p,
                                                                        uint64_t n) {
    const __m128i k12 = _mm_set_epi64x(0x1c6e41596LL, 0x154442bd4LL);
    const __m128i k34 = _mm_set_epi64x(0x0ccaa009eLL, 0x1751997d0LL);
    const __m128i k5 = _mm_set_epi64x(0, 0x163cd6124LL);
    const __m128i pmu = _mm_set_epi64x(0x1f7011641LL, 0x1db710641LL);
    const __m128i mask32 = _mm_set_epi32(0, 0, 0, -1);
    __m128i x1 = _mm_loadu_si128((const __m128i *)p), x2 = _mm_loadu_si128((const __m128i *)(p + 16)),
            x3 = _mm_loadu_si128((const __m128i *)(p + 32)), x4 = _mm_loadu_si128((const __m128i *)(p + 48));
    x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)reg));
    p += 64;
    n -= 64;
#define NKVO_FOLD(x, k, d) \
    x = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), d)
    while (n >= 64) {
        NKVO_FOLD(x1, k12, _mm_loadu_si128((const __m128i *)p));
        NKVO_FOLD(x2, k12, _mm_loadu_si128((const __m128i *)(p + 16)));
        NKVO_FOLD(x3, k12, _mm_loadu_si128((const __m128i *)(p + 32)));
        NKVO_FOLD(x4, k12, _mm_loadu_si128((const __m128i *)(p + 48)));
        p += 64;
        n -= 64;
    }
    NKVO_FOLD(x1, k34, x2);
    NKVO_FOLD(x1, k34, x3);
    NKVO_FOLD(x1, k34, x4);
    while (n >= 16) {
        NKVO_FOLD(x1, k34, _mm_loadu_si128((const __m128i *)p));
        p += 16;
        n -= 16;
    }
#undef NKVO_FOLD
    /* 128 -> 64 bits (R4 x low half), then 64 -> 32 (R5) */
    x2 = _mm_clmulepi64_si128(k34, x1, 0x01);
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x2);
    x2 = _mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k5, 0x00);
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 4), x2);
    /* Barrett */
    x2 = _mm_and_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, mask32), pmu, 0x10), mask32);
    x2 = _mm_clmulepi64_si128(x2, pmu, 0x00);
    x1 = _mm_xor_si128(x1, x2);
    reg = (uint32_t)_mm_extract_epi32(x1, 1);
    return crc_reg_s8(reg, p, n);
}

uint32_t nkvo_crc32_clmul(const uint8_t *p, uint64_t n) {
    pthread_once(&s8_once, s8_init);
    return ~(n >= 64 ? crc_reg_clmul(0xFFFFFFFFu, p, n) : crc_reg_s8(0xFFFFFFFFu, p, n));
}

typedef void (*nkvo_sha1_fn)(const uint8_t *, uint64_t, uint8_t *);
void nkvo_sha1(const uint8_t *data, uint64_t len, uint8_t out[20]);

typedef struct {
    const uint8_t *stream;
    const uint64_t *rec_off;
    uint8_t *out20;
    nkvo_sha1_fn sha1; /* NULL: seal (store each record's Crc, no digest) */
    int clmul;
    uint64_t lo, hi, bad;
} verify_job;

/* merge's per-record work (lsmtree.go:210-211 after record.go:163-169): parse
 * the header, CRC-32 of Key ++ Value against the stored Crc, SHA-1 of the Value */
static void *verify_worker(void *arg) {
    verify_job *j = (verify_job *)arg;
    uint64_t bad = 0;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        const uint8_t *r = j->stream + j->rec_off[i];
        const uint64_t ks = ld_le64(r + 14), vs = ld_le64(r + 22);
        const uint32_t c = j->clmul && ks + vs >= 64 ? ~crc_reg_clmul(0xFFFFFFFFu, r + 30, ks + vs)
                                                     : ~crc_reg_s8(0xFFFFFFFFu, r + 30, ks + vs);
        if (!j->sha1) {
            memcpy((uint8_t *)r, &c, 4);
            continue;
        }
        uint32_t stored;
        memcpy(&stored, r, 4);
        bad += c != stored;
        j->sha1(r + 30 + ks, vs, j->out20 + 20 * i);
    }
    j->bad = bad;
    return NULL;
}

/* The compaction read of n records on `threads` host threads: every stored Crc
 * checked, every Value's leaf digest into out20.  sha1: NULL = the portable
 * SHA-1 of merkle_oracle.c (bench.py passes OpenSSL's); clmul: the PCLMULQDQ
 * CRC (else slicing-by-8).  Returns the number of records whose Crc fails. */
static uint64_t run_verify(const uint8_t *stream, const uint64_t *rec_off, uint64_t n, uint8_t *out20, int threads,
                           nkvo_sha1_fn sha1, int clmul) {
    pthread_once(&s8_once, s8_init);
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > n) threads = n ? (int)n : 1;
    verify_job jobs[256];
    pthread_t tid[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (verify_job){stream, rec_off, out20, sha1, clmul, n * (uint64_t)t / (uint64_t)threads,
                               n * (uint64_t)(t + 1) / (uint64_t)threads, 0};
        if (threads == 1) verify_worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, verify_worker, &jobs[t]);
    }
    uint64_t bad = 0;
    for (int t = 0; t < threads; ++t) {
        if (threads > 1) pthread_join(tid[t], NULL);
        bad += jobs[t].bad;
    }
    return bad;
}

uint64_t nkvo_verify_records(const uint8_t *stream, const uint64_t *rec_off, uint64_t n, uint8_t *out20,
                             int threads, nkvo_sha1_fn sha1, int clmul) {
    return run_verify(stream, rec_off, n, out20, threads, sha1 ? sha1 : nkvo_sha1, clmul);
}

/* Store each record's Crc of Key ++ Value at +0 (record.go:51), on `threads`
 * threads: the synthetic Data table of the baseline's sample. */
void nkvo_seal_records(uint8_t *stream, const uint64_t *rec_off, uint64_t n, int threads) {
    run_verify(stream, rec_off, n, NULL, threads, NULL, 1);
}
