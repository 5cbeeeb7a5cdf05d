// Diagnostic: the per-call floor of a one-launch call against a resident
// service workgroup that polls a pinned doorbell.  Each "call" moves a small
// request through pinned host memory the way capnp_packed_read_message does:
// the host writes `in_bytes` of payload, the GPU reads it, writes `out_bytes`
// back and stores a completion flag (system-scope release); the host spins
// on the flag.  Modes:
//   launch  one kernel launch per call (the shipped design)
//   service one resident wave polls the doorbell (system-scope loads) and
//           serves each new sequence number; it exits on a stop value or
//           after `idle` microseconds without a request (bounded: it never
//           outlives the process by more than that)
// Prints the median / p10 microseconds per call for each mode and size.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/doorbell_probe.hip -o build/doorbell_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

__device__ __forceinline__ void serve_one(const uint8_t* in, uint32_t in_bytes, uint8_t* out,
                                          uint32_t out_bytes, uint32_t* flag, uint32_t seq) {
    const uint32_t lane = threadIdx.x;
    uint4 acc = make_uint4(seq, 0, 0, 0);
    for (uint32_t o = 16 * lane; o < in_bytes; o += 16 * 64) {
        const uint4 v = *reinterpret_cast<const uint4*>(in + o);
        acc.x ^= v.x;
        acc.y ^= v.y;
        acc.z ^= v.z;
        acc.w ^= v.w;
    }
    for (uint32_t o = 16 * lane; o < out_bytes; o += 16 * 64)
        *reinterpret_cast<uint4*>(out + o) = acc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (system scope: the writes are visible first)
    if (lane == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(64) k_launch(const uint8_t* in, uint32_t in_bytes, uint8_t* out,
                                               uint32_t out_bytes, uint32_t* flag, uint32_t seq) {
    serve_one(in, in_bytes, out, out_bytes, flag, seq);
}

// The resident wave.  Exit conditions every path reaches: the stop value, an
// idle period with no new request, or a hard cap on the total time.
__global__ void __launch_bounds__(64) k_service(const uint32_t* bell, const uint8_t* in,
                                                uint32_t in_bytes, uint8_t* out, uint32_t out_bytes,
                                                uint32_t* flag, uint64_t idle_ticks,
                                                uint64_t cap_ticks, uint32_t* served) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t t_last = t0;
    uint32_t last = 0, n = 0;
    for (;;) {
        uint32_t b = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (b == 0xFFFFFFFFu) break;
        if (b != last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // (system scope: the payload is fresh)
            serve_one(in, in_bytes, out, out_bytes, flag, b);
            last = b;
            t_last = now;
            n++;
            continue;
        }
        if (now - t_last > idle_ticks || now - t0 > cap_ticks) break;
        __builtin_amdgcn_s_sleep(1);
    }
    if (threadIdx.x == 0) served[0] = n;
}

static double pct(std::vector<double>& v, double p) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(p * (v.size() - 1))];
}

static inline void spin_eq(volatile uint32_t* f, uint32_t seq) {
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(f, __ATOMIC_ACQUIRE) != seq) {
        __builtin_ia32_pause();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) {
            fprintf(stderr, "flag timeout at seq %u\n", seq);
            break;
        }
    }
}

int main() {
    uint8_t *h_in, *h_out, *d_in, *d_out;
    uint32_t *h_bell, *h_flag, *d_bell, *d_flag, *d_served;
    CK(hipHostMalloc(&h_in, 1 << 20, 0));
    CK(hipHostMalloc(&h_out, 1 << 20, 0));
    CK(hipHostMalloc(&h_bell, 4096, 0));
    CK(hipHostMalloc(&h_flag, 4096, 0));
    CK(hipHostGetDevicePointer((void**)&d_in, h_in, 0));
    CK(hipHostGetDevicePointer((void**)&d_out, h_out, 0));
    CK(hipHostGetDevicePointer((void**)&d_bell, h_bell, 0));
    CK(hipHostGetDevicePointer((void**)&d_flag, h_flag, 0));
    CK(hipMalloc(&d_served, 64));
    hipStream_t s, ss;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
    std::vector<uint8_t> payload(1 << 20);
    for (size_t i = 0; i < payload.size(); i++) payload[i] = (uint8_t)(i * 131 + 7);
    const int reps = 4000;
    struct Sz {
        uint32_t in, out;
    } sizes[] = {{0, 0}, {600, 1024}, {6600, 12288}};
    uint32_t seq = 0;
    for (const Sz& z : sizes) {
        // launch mode
        std::vector<double> tl;
        for (int r = 0; r < reps + 200; r++) {
            const auto a = std::chrono::steady_clock::now();
            if (z.in) memcpy(h_in, payload.data(), z.in);
            ++seq;
            hipLaunchKernelGGL(k_launch, dim3(1), dim3(64), 0, s, d_in, z.in, d_out, z.out, d_flag, seq);
            spin_eq(h_flag, seq);
            const auto b = std::chrono::steady_clock::now();
            if (r >= 200) tl.push_back(std::chrono::duration<double, std::micro>(b - a).count());
        }
        CK(hipStreamSynchronize(s));
        // service mode
        *(volatile uint32_t*)h_bell = 0;
        __atomic_store_n(h_flag, 0u, __ATOMIC_RELEASE);
        hipLaunchKernelGGL(k_service, dim3(1), dim3(64), 0, ss, d_bell, d_in, z.in, d_out, z.out,
                           d_flag, (uint64_t)100 * 2000 /* 2 ms idle */,
                           (uint64_t)100 * 1000 * 10000 /* 10 s cap */, d_served);
        std::vector<double> tsv;
        uint32_t bseq = 0;
        for (int r = 0; r < reps + 200; r++) {
            const auto a = std::chrono::steady_clock::now();
            if (z.in) memcpy(h_in, payload.data(), z.in);
            ++bseq;
            __atomic_store_n(h_bell, bseq, __ATOMIC_RELEASE);
            spin_eq(h_flag, bseq);
            const auto b = std::chrono::steady_clock::now();
            if (r >= 200) tsv.push_back(std::chrono::duration<double, std::micro>(b - a).count());
        }
        __atomic_store_n(h_bell, 0xFFFFFFFFu, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(ss));
        uint32_t served = 0;
        CK(hipMemcpy(&served, d_served, 4, hipMemcpyDeviceToHost));
        // relaunch cost of the service after an idle exit (first call after launch)
        std::vector<double> tr;
        for (int r = 0; r < 200; r++) {
            __atomic_store_n(h_bell, 0u, __ATOMIC_RELEASE);
            __atomic_store_n(h_flag, 0u, __ATOMIC_RELEASE);
            const auto a = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_service, dim3(1), dim3(64), 0, ss, d_bell, d_in, z.in, d_out, z.out,
                               d_flag, (uint64_t)100 * 2000, (uint64_t)100 * 1000 * 10000, d_served);
            if (z.in) memcpy(h_in, payload.data(), z.in);
            __atomic_store_n(h_bell, 1u, __ATOMIC_RELEASE);
            spin_eq(h_flag, 1u);
            const auto b = std::chrono::steady_clock::now();
            tr.push_back(std::chrono::duration<double, std::micro>(b - a).count());
            __atomic_store_n(h_bell, 0xFFFFFFFFu, __ATOMIC_RELEASE);
            CK(hipStreamSynchronize(ss));
        }
        printf("{\"in_bytes\": %u, \"out_bytes\": %u, \"launch_us_median\": %.2f, \"launch_us_p10\": %.2f, "
               "\"service_us_median\": %.2f, \"service_us_p10\": %.2f, \"served\": %u, "
               "\"cold_service_us_median\": %.2f}\n",
               z.in, z.out, pct(tl, 0.5), pct(tl, 0.1), pct(tsv, 0.5), pct(tsv, 0.1), served,
               pct(tr, 0.5));
        fflush(stdout);
    }
    return 0;
}
