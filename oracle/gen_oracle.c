/*
 * gen_oracle.c — CPU twin of the synthetic segment generators used by
 * bench.py and the parity tests (TEST INFRASTRUCTURE; see packed_oracle.c).
 *
 * The device generator (capnproto-rust_amd/csrc/gen.hip) must produce the
 * same words bit for bit; tests/test_gen.py checks that on the GPU.
 *
 * Workloads (BASELINE.json configs):
 *   kind 0 "iid":   each word all-zero with probability pz; otherwise each
 *                   byte zero with probability 111/256 (~0.435, the carsales
 *                   byte statistic), values uniform non-zero; an all-zero
 *                   draw is redrawn.  pz = 0.30 (config 2), 0.80 (config 3).
 *   kind 1 "zero-runs": long all-zero runs (mean ~600 words) broken by one
 *                   iid non-zero word (config 4, 10 % of segments).
 *   kind 2 "literal-runs": words with no zero byte, broken every ~500 words
 *                   by a word with two zero bytes (config 4, 10 %).
 * Seeds: splitmix64(0xCA95A1E5 ^ chunk_id).
 */
#include <stdint.h>
#include <stddef.h>

static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

#define GEN_SEED_BASE 0xCA95A1E5ULL
#define ZERO_BYTE_THRESH 111u

static inline uint64_t nonzero_bytes(uint64_t v) {
    uint64_t w = 0;
    for (int j = 0; j < 8; j++) {
        uint64_t b = (v >> (8 * j)) & 0xFF;
        if (b == 0) b = 0x5A;
        w |= b << (8 * j);
    }
    return w;
}

static inline uint64_t iid_nonzero_word(uint64_t seed, uint64_t k) {
    for (uint64_t a = 0;; a++) {
        uint64_t m = splitmix64(seed + 4 * k + 1 + (a << 40));
        uint64_t v = splitmix64(seed + 4 * k + 2 + (a << 40));
        uint64_t w = 0;
        for (int j = 0; j < 8; j++) {
            uint64_t keep = ((m >> (8 * j)) & 0xFF) >= ZERO_BYTE_THRESH;
            uint64_t b = (v >> (8 * j)) & 0xFF;
            if (b == 0) b = 0x5A;
            if (keep) w |= b << (8 * j);
        }
        if (w != 0) return w;
    }
}

uint64_t gen_word(int kind, uint32_t pz_thresh, uint64_t chunk, uint64_t k) {
    uint64_t seed = splitmix64(GEN_SEED_BASE ^ chunk);
    uint64_t u = splitmix64(seed + 4 * k);
    if (kind == 0) {
        if ((uint32_t)u < pz_thresh) return 0;
        return iid_nonzero_word(seed, k);
    } else if (kind == 1) {
        if ((u >> 32) % 600 != 0) return 0;
        return iid_nonzero_word(seed, k);
    } else {
        uint64_t v = splitmix64(seed + 4 * k + 3);
        uint64_t w = nonzero_bytes(v);
        if ((u >> 32) % 500 == 0) w &= 0xFFFF0000FFFFFFFFULL; /* two zero bytes */
        return w;
    }
}

/* Fills words [offs[c], offs[c+1]) for chunks c in [c0, c1) with chunk ids
 * id0 + c; kinds[c] (may be NULL => all `kind0`) selects the generator. */
void gen_fill(uint64_t* words, const uint64_t* offs, size_t c0, size_t c1, uint64_t id0,
              const uint8_t* kinds, int kind0, uint32_t pz_thresh) {
    for (size_t c = c0; c < c1; c++) {
        int kind = kinds ? kinds[c] : kind0;
        for (uint64_t k = 0; k < offs[c + 1] - offs[c]; k++)
            words[offs[c] + k] = gen_word(kind, pz_thresh, id0 + c, k);
    }
}
