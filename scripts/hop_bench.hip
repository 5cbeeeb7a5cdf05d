// Diagnostic: cycles per dependent hop of the packed-tag walk in LDS, for a
// few loop bodies, at 1 wave per SIMD and at 8.  (scripts/hop_bench)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int V>
__global__ void hop(uint64_t* out, int iters) {
    __shared__ uint8_t B[16384];
    __shared__ uint16_t D[4096 + 256];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < 16384; i += blockDim.x) {
        uint32_t x = i * 2654435761u;
        x ^= x >> 13;
        uint8_t v = (uint8_t)(x >> 7);
        if (v == 0 || v == 0xFF) v = 0x5A;
        B[i] = v;
    }
    __syncthreads();
    const uint32_t lane = t & 63;
    uint32_t q = 1 + (t * 61) % 8000, w = t * 16;
    uint32_t tag = B[q - 1], b1 = B[q], b9 = B[q + 8];
    const uint32_t cpe1 = 16000;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        if (V == 0) {  // full hop: position, words, descriptor store
            const bool isz = tag == 0, isf = tag == 0xFF;
            const uint32_t fx = isf ? 8u * b9 + 1u : 0u;
            const uint32_t qe = __builtin_popcount(tag) + q + (isz ? 1u : 0u) + fx + 1u;
            const uint32_t qn = (qe < cpe1 ? qe : cpe1) & 8191;
            const uint32_t ntag = B[qn - 1], nb1 = B[qn], nb9 = B[qn + 8];
            const uint32_t cnt = isz ? b1 : (isf ? b9 : 0u);
            D[(w & 4095)] = (uint16_t)q;
            w = w + 1 + cnt;
            q = qn + 1;
            tag = ntag; b1 = nb1; b9 = nb9;
        } else if (V == 1) {  // position chain only, one byte read
            q = (q + __builtin_popcount(tag) + 1) & 8191;
            tag = B[q];
        } else if (V == 2) {  // position chain, u16 + u8 reads
            q = (q + __builtin_popcount(tag) + 1) & 8191;
            const uint32_t v = *reinterpret_cast<const uint16_t*>(B + q);  // aligned? no
            tag = v & 0xFF; b9 += B[q + 8];
        } else {  // V == 3: position chain + descriptor store
            D[(w++ & 4095)] = (uint16_t)q;
            q = (q + __builtin_popcount(tag) + 1) & 8191;
            tag = B[q];
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + (t >> 6)] = t1 - t0;
    if (q == 0xFFFFFFFF) out[0] = tag + b1 + b9 + w;
}

int main() {
    uint64_t* d;
    hipMalloc(&d, 256 * 16 * 8 * 8);
    uint64_t h[256 * 16];
    const int iters = 1000;
    for (int v = 0; v < 4; v++) {
        for (int blocks : {256, 2048}) {
            hipMemset(d, 0, sizeof(h));
            if (v == 0) hipLaunchKernelGGL(hop<0>, dim3(blocks), dim3(256), 0, 0, d, iters);
            if (v == 1) hipLaunchKernelGGL(hop<1>, dim3(blocks), dim3(256), 0, 0, d, iters);
            if (v == 2) hipLaunchKernelGGL(hop<2>, dim3(blocks), dim3(256), 0, 0, d, iters);
            if (v == 3) hipLaunchKernelGGL(hop<3>, dim3(blocks), dim3(256), 0, 0, d, iters);
            hipDeviceSynchronize();
            hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
            double s = 0; int n = 0;
            for (int i = 0; i < 256 * 4; i++) if (h[(i / 4) * 16 + i % 4]) { s += h[(i / 4) * 16 + i % 4]; n++; }
            printf("variant %d blocks %d: %.1f cycles/hop\n", v, blocks, s / n / iters);
        }
    }
    return 0;
}
