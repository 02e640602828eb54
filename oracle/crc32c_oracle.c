/*
 * CPU oracle (TEST INFRASTRUCTURE ONLY -- never linked into libjfsgpu.so):
 * CRC-32C (Castagnoli) as JuiceFS computes it.
 *
 *   pkg/object/checksum.go:30-45   crc32c = crc32.MakeTable(crc32.Castagnoli);
 *                                  crc32.Update(0, crc32c, data) -> object checksum
 *   pkg/chunk/disk_cache_file.go:139-152
 *                                  checksum(data): crc32.Checksum of every
 *                                  csBlock (32 KiB, :35) piece, each written with
 *                                  utils.Buffer.Put32 = big-endian (buffer.go:42,102);
 *                                  buffer size ((len-1)/csBlock+1)*4 with Go's
 *                                  truncating division (4 zero bytes for len 0)
 *
 * Go's hash/crc32 is the reflected CRC with polynomial 0x82F63B78, initial
 * value ~0 and final xor ~0 (crc32.Update(crc, tab, p) = ~update(~crc, p)).
 * This restatement is byte-at-a-time from a 256-entry table (the textbook
 * form), pinned in tests/test_crc32c.py by the check value "123456789" ->
 * 0xE3069283 and the RFC 3720 (iSCSI) B.4 vectors.
 */
#include <stdint.h>
#include <stddef.h>

#define CRC32C_POLY 0x82F63B78u

static uint32_t tab[256];
static int tab_ready;

static void build(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ CRC32C_POLY : c >> 1;
        tab[i] = c;
    }
    tab_ready = 1;
}

/* crc32.Update(crc, crc32c, p) */
uint32_t oracle_crc32c_update(uint32_t crc, const uint8_t *p, size_t n) {
    if (!tab_ready) build();
    uint32_t c = ~crc;
    for (size_t i = 0; i < n; i++) c = tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

/* disk_cache_file.go checksum(): big-endian CRC-32C of every seg-byte piece.
 * out must hold ((n-1)/seg+1)*4 bytes (Go division; 4 for n == 0).
 * Returns the number of bytes written. */
int64_t oracle_crc32c_segments(const uint8_t *p, int64_t n, int64_t seg, uint8_t *out) {
    int64_t words = (n - 1) / seg + 1; /* C and Go both truncate toward zero */
    for (int64_t w = 0; w < words; w++) out[4 * w] = out[4 * w + 1] = out[4 * w + 2] = out[4 * w + 3] = 0;
    int64_t k = 0;
    for (int64_t s = 0; s < n; s += seg, k++) {
        int64_t e = s + seg < n ? s + seg : n;
        uint32_t v = oracle_crc32c_update(0, p + s, (size_t)(e - s));
        out[4 * k] = (uint8_t)(v >> 24);
        out[4 * k + 1] = (uint8_t)(v >> 16);
        out[4 * k + 2] = (uint8_t)(v >> 8);
        out[4 * k + 3] = (uint8_t)v;
    }
    return words * 4;
}
