// gen.hip — device generators of the synthetic segment workloads (bench and
// parity tests).  Bit-identical twin of oracle/gen_oracle.c; see that file
// for the workload definitions.
#include "common.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

constexpr uint64_t kSeedBase = 0xCA95A1E5ull;
constexpr uint32_t kZeroByteThresh = 111u;

__device__ __forceinline__ uint64_t nonzero_bytes(uint64_t v) {
    uint64_t w = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        uint64_t b = (v >> (8 * j)) & 0xFF;
        if (b == 0) b = 0x5A;
        w |= b << (8 * j);
    }
    return w;
}

__device__ __forceinline__ uint64_t iid_nonzero_word(uint64_t seed, uint64_t k) {
    for (uint64_t a = 0;; a++) {
        const uint64_t m = splitmix64(seed + 4 * k + 1 + (a << 40));
        const uint64_t v = splitmix64(seed + 4 * k + 2 + (a << 40));
        uint64_t w = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const bool keep = ((m >> (8 * j)) & 0xFF) >= kZeroByteThresh;
            uint64_t b = (v >> (8 * j)) & 0xFF;
            if (b == 0) b = 0x5A;
            if (keep) w |= b << (8 * j);
        }
        if (w != 0) return w;
    }
}

__device__ __forceinline__ uint64_t gen_word(uint32_t kind, uint32_t pz, uint64_t seed,
                                             uint64_t k) {
    const uint64_t u = splitmix64(seed + 4 * k);
    if (kind == 0) {
        if ((uint32_t)u < pz) return 0;
        return iid_nonzero_word(seed, k);
    } else if (kind == 1) {
        if ((u >> 32) % 600 != 0) return 0;
        return iid_nonzero_word(seed, k);
    }
    const uint64_t v = splitmix64(seed + 4 * k + 3);
    uint64_t w = nonzero_bytes(v);
    if ((u >> 32) % 500 == 0) w &= 0xFFFF0000FFFFFFFFull;
    return w;
}

// One wave per chunk, grid-stride over chunks.
__global__ void __launch_bounds__(256)
gen_kernel(uint64_t* __restrict__ words, const uint64_t* __restrict__ offs, uint64_t nchunks,
           uint64_t id0, const uint8_t* __restrict__ kinds, uint32_t kind0, uint32_t pz) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t c = wave0; c < nchunks; c += nwaves) {
        const uint64_t a = offs[c], b = offs[c + 1];
        const uint32_t kind = kinds ? kinds[c] : kind0;
        const uint64_t seed = splitmix64(kSeedBase ^ (id0 + c));
        for (uint64_t k = lane; k < b - a; k += 64) words[a + k] = gen_word(kind, pz, seed, k);
    }
}

// ---- carsales requests (BASELINE.json configs[0]) --
// Device twin of oracle/carsales_oracle.c, which documents the restated
// reference lines (benchmark/common.rs:22-70 FastRand, benchmark/carsales.rs
// :84-150 random_car / setup_request) and the derived segment layout:
//   [root][ParkingLot][cars tag][n cars x 7] + per car [make][model]
//   [wheels tag][4 wheels][engine], 3 + 15 n words.
// The FastRand chain is serial across requests (one generator for the whole
// run, benchmark.rs:220), so the host walks it once (capnp_carsales_plan) and
// hands every request its starting state; one thread per request then
// writes the request's words.

struct FastRand {
    uint32_t x, y, z, w;
    __host__ __device__ __forceinline__ uint32_t next() {
        const uint32_t t = x ^ (x << 11);
        x = y;
        y = z;
        z = w;
        w = w ^ (w >> 19) ^ t ^ (t >> 8);
        return w;
    }
    __host__ __device__ __forceinline__ uint32_t less(uint32_t r) { return next() % r; }
    __device__ __forceinline__ bool flip() { return (next() % 2) == 1; }
    // next_u32() as f64 * range / (u32::MAX as f64), common.rs:67-69
    __device__ __forceinline__ double dbl(double range) {
#pragma clang fp contract(off)
        return (double)next() * range / 4294967295.0;
    }
};

// Names as the little-endian words of their NUL-padded text (all <= 7 bytes).
__device__ constexpr uint64_t kMakeWord[5] = {
    0x61746f796f54ull /* Toyota */, 0x4d47ull /* GM */, 0x64726f46ull /* Ford */,
    0x61646e6f48ull /* Honda */, 0x616c736554ull /* Tesla */};
__device__ constexpr uint32_t kMakeLen[5] = {6, 2, 4, 5, 5};
__device__ constexpr uint64_t kModelWord[6] = {
    0x79726d6143ull /* Camry */, 0x7375697250ull /* Prius */, 0x746c6f56ull /* Volt */,
    0x64726f636341ull /* Accord */, 0x6661654cull /* Leaf */,
    0x53206c65646f4dull /* Model S */};
__device__ constexpr uint32_t kModelLen[6] = {5, 5, 4, 6, 4, 7};

__device__ __forceinline__ uint64_t cs_struct_ptr(uint64_t at, uint64_t to, uint32_t data,
                                                  uint32_t ptrs) {
    return (uint64_t)(uint32_t)((int32_t)(to - at - 1) << 2) |
           ((uint64_t)(data | (ptrs << 16)) << 32);
}
__device__ __forceinline__ uint64_t cs_list_ptr(uint64_t at, uint64_t to, uint32_t esize,
                                                uint32_t count) {
    return (uint64_t)((uint32_t)((int32_t)(to - at - 1) << 2) | 1u) |
           ((uint64_t)((count << 3) | esize) << 32);
}

__global__ void __launch_bounds__(256)
gen_carsales_kernel(uint64_t* __restrict__ words, uint64_t total_words,
                    const uint32_t* __restrict__ states, const uint64_t* __restrict__ req_off,
                    uint64_t nreq) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nreq) return;
    FastRand r{states[4 * i], states[4 * i + 1], states[4 * i + 2], states[4 * i + 3]};
    const uint64_t base = req_off[i];
    // every word of the request is written exactly once, in address order
    // within each object; words at or past total_words are dropped
    auto put = [&](uint64_t k, uint64_t v) {
        if (base + k < total_words) words[base + k] = v;
    };
    const uint32_t n = r.less(200);
    put(0, cs_struct_ptr(0, 1, 0, 1));
    put(1, cs_list_ptr(1, 2, 7, 7 * n));
    put(2, ((uint64_t)n << 2) | ((uint64_t)(3u | (4u << 16)) << 32));
    for (uint32_t j = 0; j < n; j++) {
        const uint64_t c = 3 + 7ull * j, b = 3 + 7ull * n + 8ull * j;
        const uint32_t mk = r.less(5);
        put(b, kMakeWord[mk]);
        put(c + 3, cs_list_ptr(c + 3, b, 2, kMakeLen[mk] + 1));
        const uint32_t md = r.less(6);
        put(b + 1, kModelWord[md]);
        put(c + 4, cs_list_ptr(c + 4, b + 1, 2, kModelLen[md] + 1));
        const uint64_t color = r.less(9);
        const uint64_t seats = 2 + r.less(6);
        const uint64_t doors = 2 + r.less(3);
        put(c + 5, cs_list_ptr(c + 5, b + 2, 7, 4));
        put(b + 2, (4ull << 2) | (1ull << 32));
        for (int k = 0; k < 4; k++) {
            const uint64_t diam = 25 + r.less(15);
            const float air = (float)(30.0 + r.dbl(20.0));
            const uint64_t snow = r.less(16) == 0;
            put(b + 3 + k, diam | (snow << 16) | ((uint64_t)__float_as_uint(air) << 32));
        }
        const uint64_t length = 170 + r.less(150);
        const uint64_t width = 48 + r.less(36);
        const uint64_t height = 54 + r.less(48);
        const uint64_t weight = (uint32_t)(length * width * height / 200);
        put(c + 6, cs_struct_ptr(c + 6, b + 7, 1, 0));
        const uint64_t hp = (uint16_t)(100 * (uint16_t)r.less(400));
        const uint64_t cyl = (uint8_t)(4 + 2 * (uint8_t)r.less(3));
        const uint64_t cc = 800 + r.less(10000);
        const uint64_t electric = r.flip();
        put(b + 7, hp | (cyl << 16) | (1ull << 24) | (electric << 25) | (cc << 32));
        const float fuel_cap = (float)(10.0 + r.dbl(30.0));
        const float fuel_lvl = (float)r.dbl((double)fuel_cap);
        const uint64_t windows = r.flip(), steering = r.flip(), cruise = r.flip();
        const uint64_t cups = r.less(12);
        const uint64_t nav = r.flip();
        put(c, color | (seats << 16) | (doors << 24) | (length << 32) | (width << 48));
        put(c + 1, height | (windows << 16) | (steering << 17) | (cruise << 18) | (nav << 19) |
                       (cups << 24) | (weight << 32));
        put(c + 2, (uint64_t)__float_as_uint(fuel_cap) |
                       ((uint64_t)__float_as_uint(fuel_lvl) << 32));
    }
}

}  // namespace

// Walks the benchmark's FastRand chain on the host: skips `skip` requests,
// then records the starting state (4 x u32) and first word of each request
// until `target_words` are covered or max_req requests are planned.
// req_off[nreq] = the words of those requests in full.  Returns nreq.
extern "C" uint64_t capnp_carsales_plan(const uint32_t seed[4], uint64_t skip,
                                        uint64_t target_words, uint32_t* states,
                                        uint64_t* req_off, uint64_t max_req) {
    FastRand r{seed[0], seed[1], seed[2], seed[3]};
    auto skip_request = [&r]() {
        const uint32_t n = r.less(200);
        for (uint32_t d = 0; d < 31 * n; d++) r.next();  // 31 draws per car
        return 3 + 15ull * n;
    };
    for (uint64_t i = 0; i < skip; i++) skip_request();
    uint64_t w = 0, m = 0;
    while (w < target_words && m < max_req) {
        states[4 * m] = r.x;
        states[4 * m + 1] = r.y;
        states[4 * m + 2] = r.z;
        states[4 * m + 3] = r.w;
        req_off[m] = w;
        w += skip_request();
        m++;
    }
    req_off[m] = w;
    return m;
}

extern "C" hipError_t capnp_launch_gen_carsales(uint64_t* d_words, uint64_t total_words,
                                                const uint32_t* d_states,
                                                const uint64_t* d_req_off, uint64_t nreq,
                                                hipStream_t stream) {
    if (nreq == 0) return hipSuccess;
    hipLaunchKernelGGL(gen_carsales_kernel, dim3((uint32_t)((nreq + 255) / 256)), dim3(256), 0,
                       stream, d_words, total_words, d_states, d_req_off, nreq);
    return hipGetLastError();
}

extern "C" hipError_t capnp_launch_gen(uint64_t* d_words, const uint64_t* d_offs,
                                       uint64_t nchunks, uint64_t id0, const uint8_t* d_kinds,
                                       uint32_t kind0, uint32_t pz, hipStream_t stream) {
    if (nchunks == 0) return hipSuccess;
    uint64_t blocks = (nchunks + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(gen_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, d_words,
                       d_offs, nchunks, id0, d_kinds, kind0, pz);
    return hipGetLastError();
}
