/*
 * carsales_oracle.c — CPU restatement of the reference benchmark's carsales
 * request (BASELINE.json configs[0]).
 *
 * TEST INFRASTRUCTURE ONLY (like packed_oracle.c): loaded by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
 * product library.  The device twin is capnproto-rust_amd/csrc/gen.hip
 * (gen_carsales_kernel); tests/test_gpu_carsales.py checks it word for word.
 *
 * What is restated
 *   FastRand               benchmark/common.rs:22-70 (xorshift128, default
 *                          seed :33-36; next_less_than :57-59, next_bool
 *                          :62-64, next_double :67-69)
 *   random_car             benchmark/carsales.rs:84-131
 *   setup_request          benchmark/carsales.rs:140-150 (one FastRand for
 *                          the whole run, benchmark.rs:220)
 *   car_value              benchmark/carsales.rs:32-72 (the expectation)
 * into the words of the request's one segment, as message::Builder with the
 * `reuse` scratch allocator (benchmark.rs:155-185: 128 Ki words, so every
 * request fits the first segment) lays them out:
 *   allocation order = call order; arena.allocate bumps the segment
 *   (layout.rs:432-480); struct pointer (layout.rs:295-298 upper half),
 *   list pointer (:324-336), inline-composite tag (:247-254, :1305-1337),
 *   text = byte list with NUL (:1752-1779); offset = target - ptr - 1
 *   (:210-220).
 *
 * Struct layouts (derived by hand from carsales.capnp:28-81 with capnp's
 * field-placement rule: fields in ordinal order, each in the first free
 * hole of its size, else a new data word; no generated code ships in the
 * reference, it is produced by capnpc at build time):
 *   ParkingLot  0 data, 1 ptr   (cars)
 *   Car         3 data, 4 ptrs  color u16 @0, seats u8 @2, doors u8 @3,
 *               length u16 @4, width u16 @6, height u16 @8, hasPowerWindows
 *               bit 80, hasPowerSteering bit 81, hasCruiseControl bit 82,
 *               hasNavSystem bit 83, cupHolders u8 @11, weight u32 @12,
 *               fuelCapacity f32 @16, fuelLevel f32 @20; ptrs make, model,
 *               wheels, engine
 *   Wheel       1 data          diameter u16 @0, snowTires bit 16,
 *               airPressure f32 @4
 *   Engine      1 data          horsepower u16 @0, cylinders u8 @2,
 *               usesGas bit 24, usesElectric bit 25, cc u32 @4
 * Request with n cars = 3 + 15 n words:
 *   [root ptr][ParkingLot][list tag][n cars x 7]
 *   then per car: make text, model text (1 word each: every name is <= 7
 *   bytes + NUL), wheels tag + 4 wheels, engine.
 *
 * Pinning: the reference cannot be run here (no cargo/rustc); the derived
 * layout is checked for internal consistency (carsales_value re-reads every
 * request through its pointers and must give setup_request's expectation,
 * tests/test_carsales.py) and against the published totals of the reference
 * benchmark (blog/_posts/2013-11-16-benchmark.md:38-41: ~125 MB unpacked,
 * ~81 MB packed per 10 000 carsales iterations).  Byte identity with the
 * Rust builder is therefore "parity unpinned" beyond those checks.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

typedef struct fastrand {
    uint32_t x, y, z, w;
} fastrand;

/* benchmark/common.rs:30-39 */
void carsales_seed(uint32_t st[4]) {
    st[0] = 0x1d2acd47u;
    st[1] = 0x58ca3e14u;
    st[2] = 0xf563f232u;
    st[3] = 0x0bc76199u;
}

/* common.rs:46-54 */
static inline uint32_t fr_next(fastrand* r) {
    uint32_t tmp = r->x ^ (r->x << 11);
    r->x = r->y;
    r->y = r->z;
    r->z = r->w;
    r->w = r->w ^ (r->w >> 19) ^ tmp ^ (tmp >> 8);
    return r->w;
}
static inline uint32_t fr_less(fastrand* r, uint32_t range) { return fr_next(r) % range; }
static inline int fr_bool(fastrand* r) { return (fr_next(r) % 2) == 1; }
/* common.rs:67-69: next_u32() as f64 * range / (u32::MAX as f64) */
static inline double fr_double(fastrand* r, double range) {
    return (double)fr_next(r) * range / 4294967295.0;
}

static const char* const kMakes[5] = {"Toyota", "GM", "Ford", "Honda", "Tesla"};
static const char* const kModels[6] = {"Camry", "Prius", "Volt", "Accord", "Leaf", "Model S"};

static inline uint64_t struct_ptr(uint64_t at, uint64_t target, uint32_t data, uint32_t ptrs) {
    uint32_t lo = (uint32_t)((int32_t)(target - at - 1) << 2);
    return (uint64_t)lo | ((uint64_t)(data | (ptrs << 16)) << 32);
}
static inline uint64_t list_ptr(uint64_t at, uint64_t target, uint32_t esize, uint32_t count) {
    uint32_t lo = (uint32_t)((int32_t)(target - at - 1) << 2) | 1u;
    return (uint64_t)lo | ((uint64_t)((count << 3) | esize) << 32);
}
static inline uint64_t text_word(const char* s) {
    uint64_t w = 0;
    for (size_t i = 0; s[i]; i++) w |= (uint64_t)(uint8_t)s[i] << (8 * i);
    return w;
}
static inline void put16(uint64_t* w, unsigned byte, uint16_t v) {
    w[byte / 8] |= (uint64_t)v << (8 * (byte % 8));
}
static inline void put8(uint64_t* w, unsigned byte, uint8_t v) {
    w[byte / 8] |= (uint64_t)v << (8 * (byte % 8));
}
static inline void put32(uint64_t* w, unsigned byte, uint32_t v) {
    w[byte / 8] |= (uint64_t)v << (8 * (byte % 8));
}
static inline void putbit(uint64_t* w, unsigned bit, int v) {
    if (v) w[bit / 64] |= 1ull << (bit % 64);
}
static inline uint32_t f32_bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

/* setup_request (carsales.rs:140-150) + random_car (:84-131) for one
 * request; writes 3 + 15 n words to seg (seg must hold 3 + 15*199 words) and
 * returns the word count; *expected = the sum of car_value (:32-72). */
size_t carsales_request(uint32_t st[4], uint64_t* seg, uint64_t* expected) {
    fastrand r = {st[0], st[1], st[2], st[3]};
    const uint32_t n = fr_less(&r, 200);
    const size_t nw = 3 + 15 * (size_t)n;
    memset(seg, 0, nw * 8);
    seg[0] = struct_ptr(0, 1, 0, 1);        /* root -> ParkingLot */
    seg[1] = list_ptr(1, 2, 7, 7 * n);      /* cars: inline composite */
    seg[2] = ((uint64_t)n << 2) | ((uint64_t)(3u | (4u << 16)) << 32);  /* tag */
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t c = 3 + 7ull * i;          /* the car's struct */
        const uint64_t b = 3 + 7ull * n + 8ull * i;  /* its out-of-line objects */
        uint64_t* d = seg + c;
        const char* make = kMakes[fr_less(&r, 5)];
        seg[b] = text_word(make);
        seg[c + 3] = list_ptr(c + 3, b, 2, (uint32_t)strlen(make) + 1);
        const char* model = kModels[fr_less(&r, 6)];
        seg[b + 1] = text_word(model);
        seg[c + 4] = list_ptr(c + 4, b + 1, 2, (uint32_t)strlen(model) + 1);
        const uint16_t color = (uint16_t)fr_less(&r, 9);
        const uint8_t seats = (uint8_t)(2 + fr_less(&r, 6));
        const uint8_t doors = (uint8_t)(2 + fr_less(&r, 3));
        put16(d, 0, color);
        put8(d, 2, seats);
        put8(d, 3, doors);
        seg[c + 5] = list_ptr(c + 5, b + 2, 7, 4);
        seg[b + 2] = (4ull << 2) | ((uint64_t)1u << 32);  /* 4 wheels, 1 data word */
        uint64_t value = (uint64_t)seats * 200 + (uint64_t)doors * 350;
        for (int k = 0; k < 4; k++) {
            uint64_t* wd = seg + b + 3 + k;
            const uint16_t diam = (uint16_t)(25 + fr_less(&r, 15));
            const float air = (float)(30.0 + fr_double(&r, 20.0));
            const int snow = fr_less(&r, 16) == 0;
            put16(wd, 0, diam);
            put32(wd, 4, f32_bits(air));
            putbit(wd, 16, snow);
            value += (uint64_t)diam * diam + (snow ? 100 : 0);
        }
        const uint16_t length = (uint16_t)(170 + fr_less(&r, 150));
        const uint16_t width = (uint16_t)(48 + fr_less(&r, 36));
        const uint16_t height = (uint16_t)(54 + fr_less(&r, 48));
        put16(d, 4, length);
        put16(d, 6, width);
        put16(d, 8, height);
        put32(d, 12, (uint32_t)length * width * height / 200);
        value += (uint64_t)length * width * height / 50;
        seg[c + 6] = struct_ptr(c + 6, b + 7, 1, 0);
        uint64_t* ed = seg + b + 7;
        const uint16_t hp = (uint16_t)(100 * (uint16_t)fr_less(&r, 400));
        const uint8_t cyl = (uint8_t)(4 + 2 * (uint8_t)fr_less(&r, 3));
        const uint32_t cc = 800 + fr_less(&r, 10000);
        const int electric = fr_bool(&r);
        put16(ed, 0, hp);
        put8(ed, 2, cyl);
        put32(ed, 4, cc);
        putbit(ed, 24, 1);  /* usesGas = true */
        putbit(ed, 25, electric);
        value += (uint64_t)hp * 40 + (electric ? 5000 : 0);  /* uses gas: hybrid */
        const float fuel_cap = (float)(10.0 + fr_double(&r, 30.0));
        const float fuel_lvl = (float)fr_double(&r, (double)fuel_cap);
        put32(d, 16, f32_bits(fuel_cap));
        put32(d, 20, f32_bits(fuel_lvl));
        const int windows = fr_bool(&r), steering = fr_bool(&r), cruise = fr_bool(&r);
        const uint8_t cups = (uint8_t)fr_less(&r, 12);
        const int nav = fr_bool(&r);
        putbit(d, 80, windows);
        putbit(d, 81, steering);
        putbit(d, 82, cruise);
        put8(d, 11, cups);
        putbit(d, 83, nav);
        value += (windows ? 100 : 0) + (steering ? 200 : 0) + (cruise ? 400 : 0) +
                 (nav ? 2000 : 0) + (uint64_t)cups * 25;
        total += value;
    }
    st[0] = r.x;
    st[1] = r.y;
    st[2] = r.z;
    st[3] = r.w;
    if (expected) *expected = total;
    return nw;
}

/* handle_request (carsales.rs:152-163) on a request segment, through its
 * pointers: the sum of car_value (:32-72).  Returns UINT64_MAX if a pointer
 * does not have the shape setup_request gives it. */
static inline int64_t ptr_off(uint64_t p) { return (int64_t)(int32_t)(uint32_t)p >> 2; }
uint64_t carsales_value(const uint64_t* seg, size_t nw) {
    const uint64_t bad = UINT64_MAX;
    if (nw < 3 || (seg[0] & 3) != 0) return bad;
    const int64_t pl = 1 + ptr_off(seg[0]);
    if (pl < 0 || (uint64_t)pl >= nw || (seg[0] >> 32) != 0x10000u) return bad;
    const uint64_t lp = seg[pl];
    if ((lp & 3) != 1 || ((lp >> 32) & 7) != 7) return bad;
    const int64_t tagi = pl + 1 + ptr_off(lp);
    if (tagi < 0 || (uint64_t)tagi >= nw) return bad;
    const uint64_t tag = seg[tagi];
    const uint32_t n = (uint32_t)tag >> 2;
    if ((tag >> 32) != (3u | (4u << 16)) || 7ull * n != (lp >> 35)) return bad;
    if ((uint64_t)tagi + 1 + 7ull * n > nw) return bad;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t c = (uint64_t)tagi + 1 + 7ull * i;
        const uint64_t* d = seg + c;
        const uint64_t seats = (d[0] >> 16) & 0xFF, doors = (d[0] >> 24) & 0xFF;
        uint64_t v = seats * 200 + doors * 350;
        const uint64_t wp = seg[c + 5];
        const int64_t wt = (int64_t)c + 5 + 1 + ptr_off(wp);
        if ((wp & 3) != 1 || wt < 0 || (uint64_t)wt + 5 > nw) return bad;
        const uint32_t nwheels = (uint32_t)seg[wt] >> 2;
        for (uint32_t k = 0; k < nwheels; k++) {
            const uint64_t wd = seg[wt + 1 + k];
            const uint64_t diam = wd & 0xFFFF;
            v += diam * diam + (((wd >> 16) & 1) ? 100 : 0);
        }
        const uint64_t length = (d[0] >> 32) & 0xFFFF, width = (d[0] >> 48) & 0xFFFF;
        const uint64_t height = d[1] & 0xFFFF;
        v += length * width * height / 50;
        const uint64_t ep = seg[c + 6];
        const int64_t et = (int64_t)c + 6 + 1 + ptr_off(ep);
        if ((ep & 3) != 0 || et < 0 || (uint64_t)et >= nw) return bad;
        const uint64_t e = seg[et];
        v += (e & 0xFFFF) * 40;
        if ((e >> 25) & 1) v += ((e >> 24) & 1) ? 5000 : 3000;
        v += ((d[1] >> 16) & 1) ? 100 : 0;
        v += ((d[1] >> 17) & 1) ? 200 : 0;
        v += ((d[1] >> 18) & 1) ? 400 : 0;
        v += ((d[1] >> 19) & 1) ? 2000 : 0;
        v += ((d[1] >> 24) & 0xFF) * 25;
        total += v;
    }
    return total;
}

/* The request stream of one benchmark run: requests `skip`, skip+1, ... of
 * the FastRand chain that starts at `st` (benchmark.rs:220-229), their
 * segments back to back in `words` until `target_words` are covered (the
 * last request may be cut).  msg_off[i] = first word of request i (at most
 * max_msgs + 1 entries, msg_off[nmsgs] = the words written in full).
 * Returns the number of requests started; st is advanced past them. */
size_t carsales_stream(uint32_t st[4], uint64_t skip, uint64_t* words, uint64_t target_words,
                       uint64_t* msg_off, size_t max_msgs) {
    uint64_t tmp[3 + 15 * 199];
    for (uint64_t i = 0; i < skip; i++) carsales_request(st, tmp, NULL);
    uint64_t w = 0;
    size_t m = 0;
    while (w < target_words && m < max_msgs) {
        const size_t nw = carsales_request(st, tmp, NULL);
        const uint64_t take = (w + nw <= target_words) ? nw : target_words - w;
        memcpy(words + w, tmp, take * 8);
        if (msg_off) msg_off[m] = w;
        w += nw;
        m++;
    }
    if (msg_off) msg_off[m] = w;
    return m;
}
