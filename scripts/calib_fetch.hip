// calib_fetch.hip — FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the
// access widths the codec kernels use (1 B, 8 B and 16 B per lane reads;
// 16 B per lane writes).  Each kernel touches exactly `bytes` bytes once.
//   hipcc -O3 --offload-arch=gfx950 -o build/calib scripts/calib_fetch.hip
//   rocprofv3 --pmc FETCH_SIZE -- ./build/calib
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <typename T>
__global__ void read_kernel(const T* __restrict__ p, size_t n, uint64_t* sink) {
    uint64_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const T v = p[i];
        if constexpr (sizeof(T) >= 8) {
            uint64_t w[sizeof(T) / 8];
            __builtin_memcpy(w, &v, sizeof(T));
            for (unsigned k = 0; k < sizeof(T) / 8; k++) acc ^= w[k];
        } else {
            acc += (uint64_t)v;
        }
    }
    if (acc == 0x123456789ull) *sink = acc;  // keeps the loads alive
}

__global__ void write_kernel(uint4* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main() {
    const size_t bytes = size_t(1) << 30;
    uint8_t* d = nullptr;
    uint64_t* sink = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
    if (hipMemset(d, 1, bytes) != hipSuccess) return 1;
    const int grid = 256 * 32, block = 256;
    for (int rep = 0; rep < 2; rep++) {
        read_kernel<uint8_t><<<grid, block>>>(d, bytes, sink);
        read_kernel<uint64_t><<<grid, block>>>(reinterpret_cast<uint64_t*>(d), bytes / 8, sink);
        read_kernel<uint4><<<grid, block>>>(reinterpret_cast<uint4*>(d), bytes / 16, sink);
        write_kernel<<<grid, block>>>(reinterpret_cast<uint4*>(d), bytes / 16);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("calib: each kernel touches %zu bytes\n", bytes);
    return 0;
}
