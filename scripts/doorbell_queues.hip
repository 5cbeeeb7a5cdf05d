// Diagnostic: two resident service waves (one per kind of per-message call)
// on their own streams, with the process's other streams created first, so
// that the runtime's hardware queues (GPU_MAX_HW_QUEUES) may be shared.  A
// resident kernel blocks every later packet of its hardware queue, so the
// services must not share one with each other or with other work.  Modes:
//   plain   hipStreamCreateWithFlags streams
//   masked  hipExtStreamCreateWithCUMask streams (all CUs)
//   prio    non-blocking streams at the highest stream priority
// For each: requests alternate between the two services (median us, and how
// many waited > 500 us), then an empty kernel on every other stream while
// both services are resident (us until each completes).
//
//   hipcc --offload-arch=gfx950 -O3 scripts/doorbell_queues.hip -o build/doorbell_queues
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

using clk = std::chrono::steady_clock;

__global__ void k_empty(uint32_t* p) {
    if (threadIdx.x == 0 && p) p[0] = 1;
}

// One resident wave: serves each new bell value (flag = bell), exits on the
// stop value or after idle_ticks of the 100 MHz clock without a request.
__global__ void __launch_bounds__(64) k_service(const uint32_t* bell, uint32_t* flag,
                                                uint64_t idle_ticks) {
    uint64_t t_last = __builtin_amdgcn_s_memrealtime();
    uint32_t last = 0;
    for (;;) {
        uint32_t b = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        b = (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (b == 0xFFFFFFFFu) break;
        if (b != last) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (threadIdx.x == 0) __hip_atomic_store(flag, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = b;
            t_last = now;
            continue;
        }
        if (now - t_last > idle_ticks) break;
        __builtin_amdgcn_s_sleep(1);
    }
}

static double pct(std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0 : v[(size_t)(p * (v.size() - 1))];
}

static bool spin_eq(volatile uint32_t* f, uint32_t seq, double limit_us) {
    const auto t0 = clk::now();
    while (__atomic_load_n(f, __ATOMIC_ACQUIRE) != seq) {
        __builtin_ia32_pause();
        if (std::chrono::duration<double, std::micro>(clk::now() - t0).count() > limit_us) return false;
    }
    return true;
}

int main() {
    uint32_t *h, *d;
    CK(hipHostMalloc(&h, 4096, 0));
    CK(hipHostGetDevicePointer((void**)&d, h, 0));
    uint32_t* dz;
    CK(hipMalloc(&dz, 64));
    // the process's other streams first (torch's, the context's own, ...)
    std::vector<hipStream_t> other(6);
    for (auto& s : other) {
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, dz);
        CK(hipStreamSynchronize(s));
    }
    int prio_lo = 0, prio_hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    printf("{\"priority_range\": [%d, %d]}\n", prio_lo, prio_hi);
    for (int mode = 2; mode >= 0; mode--) {
        hipStream_t sa, sb;
        if (mode == 0) {
            CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
            CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
        } else if (mode == 2) {
            CK(hipStreamCreateWithPriority(&sa, hipStreamNonBlocking, prio_hi));
            CK(hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, prio_hi));
        } else {
            std::vector<uint32_t> mask(8, 0xFFFFFFFFu);
            CK(hipExtStreamCreateWithCUMask(&sa, (uint32_t)mask.size(), mask.data()));
            CK(hipExtStreamCreateWithCUMask(&sb, (uint32_t)mask.size(), mask.data()));
        }
        uint32_t *bell_a = h, *flag_a = h + 16, *bell_b = h + 32, *flag_b = h + 48;
        memset(h, 0, 4096);
        const uint64_t idle = 100 * 2000;  // 2 ms
        hipLaunchKernelGGL(k_service, dim3(1), dim3(64), 0, sa, d, d + 16, idle);
        hipLaunchKernelGGL(k_service, dim3(1), dim3(64), 0, sb, d + 32, d + 48, idle);
        std::vector<double> t;
        int slow = 0, lost = 0;
        for (uint32_t r = 1; r <= 2000; r++) {
            const bool a = r & 1;
            const auto t0 = clk::now();
            __atomic_store_n(a ? bell_a : bell_b, r, __ATOMIC_RELEASE);
            if (!spin_eq(a ? flag_a : flag_b, r, 1500.0)) {  // (< the idle exit: both still resident)
                lost++;
                break;
            }
            const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
            if (us > 500) slow++;
            t.push_back(us);
        }
        // other streams while both services are resident
        std::vector<double> te;
        for (size_t i = 0; i <= other.size(); i++) {
            hipStream_t s = i < other.size() ? other[i] : (hipStream_t)0;
            const auto t0 = clk::now();
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, dz);
            CK(hipStreamSynchronize(s));
            te.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
            // keep the services busy (a request each) so they do not idle out
            __atomic_store_n(bell_a, 100000u + (uint32_t)i, __ATOMIC_RELEASE);
            spin_eq(flag_a, 100000u + (uint32_t)i, 3000.0);
            __atomic_store_n(bell_b, 100000u + (uint32_t)i, __ATOMIC_RELEASE);
            spin_eq(flag_b, 100000u + (uint32_t)i, 3000.0);
        }
        __atomic_store_n(bell_a, 0xFFFFFFFFu, __ATOMIC_RELEASE);
        __atomic_store_n(bell_b, 0xFFFFFFFFu, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(sa));
        CK(hipStreamSynchronize(sb));
        printf("{\"mode\": \"%s\", \"alternating_us_median\": %.2f, \"p90\": %.2f, \"slow\": %d, "
               "\"lost\": %d, \"served\": %zu, \"other_stream_us\": [",
               mode == 2 ? "prio" : (mode ? "masked" : "plain"), pct(t, 0.5), pct(t, 0.9), slow, lost, t.size());
        for (size_t i = 0; i < te.size(); i++) printf("%s%.1f", i ? ", " : "", te[i]);
        printf("]}\n");
        fflush(stdout);
        CK(hipStreamDestroy(sa));
        CK(hipStreamDestroy(sb));
    }
    return 0;
}
