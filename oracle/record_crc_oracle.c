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
