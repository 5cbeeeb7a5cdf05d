// Diagnostic: are byte-misaligned 2/8/16-byte LDS reads and writes exact on
// this device (SH_MEM_CONFIG alignment mode)?  And what do they cost?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

// forced instructions (the compiler would split a misaligned access)
__device__ __forceinline__ uint64_t ld64(const uint8_t* p) {
    uint64_t v;
    asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
    return v;
}
__device__ __forceinline__ uint16_t ld16(const uint8_t* p) {
    uint32_t v;
    asm volatile("ds_read_u16 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
    return (uint16_t)v;
}
__device__ __forceinline__ uint4 ld128(const uint8_t* p) {
    uint4 v;
    asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((uint32_t)(uintptr_t)p));
    return v;
}
__device__ __forceinline__ void st64(uint8_t* p, uint64_t v) {
    asm volatile("ds_write_b64 %0, %1" :: "v"((uint32_t)(uintptr_t)p), "v"(v) : "memory");
}
__device__ __forceinline__ void st16(uint8_t* p, uint32_t v) {
    asm volatile("ds_write_b16 %0, %1" :: "v"((uint32_t)(uintptr_t)p), "v"(v) : "memory");
}

__global__ void probe(uint32_t* err, uint64_t* cyc) {
    __shared__ __attribute__((aligned(16))) uint8_t b[8192];
    __shared__ __attribute__((aligned(16))) uint8_t c[8192];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < 8192; i += blockDim.x) { b[i] = (uint8_t)(i * 131 + 7); c[i] = 0; }
    __syncthreads();
    uint32_t bad = 0;
    // reads: u64 and u16 at every misalignment
    for (uint32_t k = 0; k < 16; k++) {
        const uint32_t p = t * 17 + k;
        uint64_t v = ld64(b + p);
        uint64_t ref = 0;
        for (int j = 7; j >= 0; j--) ref = (ref << 8) | (uint8_t)((p + j) * 131 + 7);
        if (v != ref) bad |= 1;
        uint16_t h = ld16(b + p);
        if (h != (uint16_t)(ref & 0xFFFF)) bad |= 2;
        uint4 q = ld128(b + p);
        uint64_t r2 = 0;
        for (int j = 15; j >= 8; j--) r2 = (r2 << 8) | (uint8_t)((p + j) * 131 + 7);
        if (q.x != (uint32_t)ref || q.y != (uint32_t)(ref >> 32) || q.z != (uint32_t)r2 ||
            q.w != (uint32_t)(r2 >> 32)) bad |= 4;
    }
    // writes: lane t writes 10 bytes at 10 t + 3 (neighbours share dwords)
    {
        const uint32_t p = 10 * t + 3;
        uint64_t v = 0;
        for (int j = 7; j >= 0; j--) v = (v << 8) | (uint8_t)(p + j + 1);
        st64(c + p, v);
        st16(c + p + 8, (uint16_t)(((p + 9 + 1) & 0xFF) << 8 | ((p + 8 + 1) & 0xFF)));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (uint32_t i = t; i < 10 * blockDim.x; i += blockDim.x) {
        const uint32_t p = i + 3;
        if (c[p] != (uint8_t)(p + 1)) bad |= 8;
    }
    // timing: dependent chains of misaligned vs aligned u64 reads
    uint32_t pos = t * 8 + 1;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 256; i++) {
        uint64_t v = ld64(b + (pos & 4095));
        pos = (uint32_t)(v & 7) + pos + 9;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t pa = t * 8;
    for (int i = 0; i < 256; i++) {
        uint64_t v = ld64(b + (pa & 4088));
        pa = ((uint32_t)(v & 7) << 3) + pa + 8;
    }
    uint64_t t2 = __builtin_amdgcn_s_memtime();
    uint32_t pb = t * 8 + 1;
    for (int i = 0; i < 256; i++) {
        uint32_t v = b[pb & 4095];
        pb = (v & 7) + pb + 9;
    }
    uint64_t t3 = __builtin_amdgcn_s_memtime();
    atomicOr(err, bad);
    if (t == 0) { cyc[0] = (t1 - t0); cyc[1] = (t2 - t1); cyc[2] = t3 - t2; cyc[3] = pos + pa + pb; }
}

int main() {
    uint32_t* err; uint64_t* cyc;
    hipMalloc(&err, 4); hipMalloc(&cyc, 32); hipMemset(err, 0, 4);
    hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, err, cyc);
    uint32_t h; uint64_t c[4];
    hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost);
    hipMemcpy(c, cyc, 32, hipMemcpyDeviceToHost);
    printf("unaligned LDS errors mask=%u (1 u64 read, 2 u16 read, 4 u128 read, 8 write)\n", h);
    printf("256 dependent u64 reads: misaligned %llu, aligned %llu, u8 %llu s_memtime ticks\n",
           (unsigned long long)c[0], (unsigned long long)c[1], (unsigned long long)c[2]);
    return 0;
}
