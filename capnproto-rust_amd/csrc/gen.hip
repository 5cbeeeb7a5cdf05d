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

}  // namespace

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
