// Diagnostic: HBM write bandwidth of lane-segmented 8-byte stores (lane l of a
// wave writes words [16 l, 16 l + 16) of its wave's 1024-word block, one word
// per instruction) against coalesced stores of the same block.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ void __launch_bounds__(256) st(uint64_t* out, uint64_t nblocks) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint64_t blk = (uint64_t)blockIdx.x * 4 + wave; blk < nblocks; blk += (uint64_t)gridDim.x * 4) {
        uint64_t* o = out + blk * 1024;
        if (MODE == 0) {  // coalesced: instruction j writes words 64 j + lane
#pragma unroll
            for (int j = 0; j < 16; j++) o[64 * j + lane] = blk + j;
        } else if (MODE == 1) {  // segmented 8-byte stores
#pragma unroll
            for (int j = 0; j < 16; j++) o[16 * lane + j] = blk + j;
        } else {  // segmented 16-byte stores
#pragma unroll
            for (int j = 0; j < 16; j += 2)
                *reinterpret_cast<ulonglong2*>(o + 16 * lane + j) = make_ulonglong2(blk + j, blk);
        }
    }
}

int main() {
    const uint64_t words = 1ull << 27;  // 1 GiB
    uint64_t* d;
    hipMalloc(&d, words * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int mode = 0; mode < 3; mode++) {
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(a);
            if (mode == 0) hipLaunchKernelGGL(st<0>, dim3(8192), dim3(256), 0, 0, d, words / 1024);
            if (mode == 1) hipLaunchKernelGGL(st<1>, dim3(8192), dim3(256), 0, 0, d, words / 1024);
            if (mode == 2) hipLaunchKernelGGL(st<2>, dim3(8192), dim3(256), 0, 0, d, words / 1024);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            if (rep == 2) printf("mode %d (%s): %.1f us, %.0f GB/s\n", mode,
                                 mode == 0 ? "coalesced 8B" : mode == 1 ? "segmented 8B" : "segmented 16B",
                                 ms * 1e3, words * 8 / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
