// capi.hip — the C ABI (include/capnp_packed.h, include/capnp_packed_bench.h).
//
// Host entry points stage through device memory and run the gfx950 kernels;
// there is no CPU implementation of the codec in this library.
#ifndef CAPNP_STATE_ALLOC
// pack look-back records: 1 uncached device memory (default; see pack.hip),
// 0 hipMalloc, 2 fine-grained (diagnostic builds)
#define CAPNP_STATE_ALLOC 1
#endif
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <cmath>
#include <mutex>
#include <vector>

#include "../../include/capnp_packed.h"
#include "../../include/capnp_packed_bench.h"
#include "common.h"
#include "frame.h"

extern "C" hipError_t capnp_launch_pack(const uint64_t*, const uint64_t*, uint64_t, uint32_t,
                                        uint8_t*, uint64_t, uint64_t*, uint64_t*, uint32_t*,
                                        hipStream_t);
extern "C" hipError_t capnp_launch_pack_gap(const uint64_t*, const uint64_t*, uint64_t, uint32_t,
                                            uint8_t*, uint64_t, uint64_t*, uint64_t*,
                                            const uint32_t*, hipStream_t);
extern "C" uint32_t capnp_pack_tile_words(void);
extern "C" hipError_t capnp_launch_msg_gap(const uint64_t*, const uint64_t*, uint64_t, uint64_t,
                                           uint32_t*, uint32_t*, hipStream_t);
extern "C" hipError_t capnp_launch_msg_tables(const uint64_t*, const uint64_t*, uint64_t,
                                              const uint64_t*, uint8_t*, uint64_t, uint64_t*,
                                              hipStream_t);
extern "C" hipError_t capnp_msg_scan_bytes(uint64_t, size_t*);
extern "C" hipError_t capnp_launch_msg_prepare(const uint64_t*, const uint64_t*, const uint64_t*,
                                               uint64_t, uint64_t*, uint64_t*, uint64_t*,
                                               uint64_t*, void*, size_t, uint64_t*, uint64_t*,
                                               hipStream_t);
extern "C" hipError_t capnp_launch_msg_offsets(const uint64_t*, const uint64_t*, uint64_t,
                                               uint64_t*, hipStream_t);
extern "C" hipError_t capnp_launch_msg_frame(const uint8_t*, const uint64_t*, uint64_t, int,
                                             uint64_t, int, uint64_t*, uint64_t*, int32_t*,
                                             uint64_t*, void*, size_t, uint64_t*, uint64_t*,
                                             hipStream_t);
extern "C" hipError_t capnp_launch_msg_segs(const uint8_t*, const uint64_t*, uint64_t, int,
                                            uint64_t, int, const int32_t*, const uint64_t*,
                                            const uint64_t*, const uint64_t*, uint64_t*,
                                            uint64_t*, uint64_t*, hipStream_t);
extern "C" hipError_t capnp_launch_msg_status(uint64_t, const int32_t*, const uint64_t*,
                                              const int32_t*, const uint64_t*, int32_t*,
                                              uint64_t*, hipStream_t);
extern "C" hipError_t capnp_launch_flat_frame(const uint8_t*, const uint64_t*, uint64_t, int,
                                              uint64_t, int, uint64_t*, int32_t*, uint64_t*,
                                              uint64_t*, void*, size_t, uint64_t*, hipStream_t);
extern "C" hipError_t capnp_launch_flat_segs(const uint8_t*, const uint64_t*, uint64_t, int,
                                             uint64_t, int, const int32_t*, const uint64_t*,
                                             uint32_t*, hipStream_t);
extern "C" size_t capnp_pack_state_bytes(uint64_t, uint32_t);
extern "C" hipError_t capnp_launch_unpack(const uint8_t*, const uint64_t*, uint64_t, uint32_t,
                                          uint64_t*, const uint64_t*, int32_t*, uint64_t*,
                                          const uint32_t*, hipStream_t);
extern "C" hipError_t capnp_launch_gen(uint64_t*, const uint64_t*, uint64_t, uint64_t,
                                       const uint8_t*, uint32_t, uint32_t, hipStream_t);
extern "C" uint64_t capnp_carsales_plan(const uint32_t*, uint64_t, uint64_t, uint32_t*, uint64_t*,
                                        uint64_t);
extern "C" hipError_t capnp_launch_gen_carsales(uint64_t*, uint64_t, const uint32_t*,
                                                const uint64_t*, uint64_t, hipStream_t);
extern "C" size_t capnp_resync_ws_bytes(uint64_t n, uint64_t total_bytes);
extern "C" size_t capnp_msg_chain_ws_bytes(uint64_t words_cap);
extern "C" hipError_t capnp_resync_read_stream(const uint8_t*, uint64_t, uint64_t, uint64_t*,
                                               uint64_t*, uint64_t, uint64_t*, uint64_t*,
                                               uint64_t*, int*, void*, size_t, hipStream_t,
                                               uint64_t*);
extern "C" hipError_t capnp_launch_msg_meta(const uint64_t*, const uint64_t*, uint64_t, uint64_t,
                                            int, uint64_t*, uint64_t*, uint64_t*, hipStream_t);
extern "C" hipError_t capnp_launch_msg_seglist(const uint64_t*, const uint64_t*, uint64_t,
                                               const uint64_t*, uint64_t*, hipStream_t);
extern "C" hipError_t capnp_scan_counts(const uint64_t*, uint64_t, uint64_t*, void*, size_t,
                                        hipStream_t);
extern "C" size_t capnp_scan_counts_tmp_bytes(uint64_t n);
extern "C" size_t capnp_unpack_wt_ws_bytes(uint64_t wlo, uint64_t whi);
extern "C" uint64_t capnp_pack_wt_tiles(uint64_t wlo, uint64_t whi);
extern "C" size_t capnp_pack_wt_ws_bytes(uint64_t wlo, uint64_t whi);
extern "C" hipError_t capnp_launch_pack_wt(const uint64_t*, const uint64_t*, uint64_t, uint8_t*,
                                           uint64_t, uint64_t*, uint64_t*, void*, size_t,
                                           uint32_t*, uint64_t, uint64_t, hipStream_t);
extern "C" hipError_t capnp_launch_unpack_wt(const uint8_t*, const uint64_t*, uint64_t, uint64_t*,
                                             const uint64_t*, int32_t*, uint64_t*,
                                             const uint32_t*, uint64_t, uint64_t, void*, size_t,
                                             hipStream_t);
extern "C" hipError_t capnp_resync_find_messages(const uint8_t* d_in, uint64_t nbytes,
                                                 uint64_t max_msgs, uint64_t* d_pos,
                                                 uint64_t* d_words, uint64_t words_cap,
                                                 uint64_t* nmsg, int* clean, void* d_ws,
                                                 size_t ws_bytes, hipStream_t s,
                                                 uint64_t* words_needed);
extern "C" hipError_t capnp_resync_decode_prefix(const uint8_t* d_in, uint64_t nbytes,
                                                 uint64_t max_words, uint64_t* d_out, void* d_ws,
                                                 size_t ws_bytes, hipStream_t s, uint64_t* bytes,
                                                 uint64_t* words);
extern "C" hipError_t capnp_resync_prefix(const uint8_t* d_in, uint64_t nbytes, void* d_ws,
                                          size_t ws_bytes, hipStream_t s, uint64_t* bytes,
                                          uint64_t* words);
extern "C" hipError_t capnp_resync_unpack(const uint8_t* d_in, const uint64_t* d_in_off, uint64_t n,
                                          uint64_t total_bytes, uint64_t* d_out,
                                          const uint64_t* d_out_off, int32_t* d_status,
                                          uint64_t* d_consumed, void* d_ws, size_t ws_bytes,
                                          hipStream_t s, int* passes, int* serial,
                                          const int32_t** failed_flag);
extern "C" hipError_t capnp_launch_msg_read(const uint8_t*, uint64_t, uint32_t, uint32_t, uint64_t,
                                            uint32_t, uint64_t, uint64_t, FrameResult*, uint64_t*,
                                            uint64_t*, uint32_t*, uint32_t, hipStream_t);
extern "C" uint32_t capnp_msg_pack_words(void);
extern "C" hipError_t capnp_launch_msg_pack(const uint64_t*, const uint64_t*, uint32_t, uint32_t,
                                            uint8_t*, uint64_t, uint64_t*, uint32_t*, uint32_t,
                                            uint8_t*, hipStream_t);
extern "C" hipError_t capnp_launch_frame(const uint8_t*, uint64_t, uint32_t, uint32_t, uint64_t,
                                         uint32_t, uint64_t, uint64_t, FrameResult*, hipStream_t);
extern "C" hipError_t capnp_launch_msg_read_service(const uint64_t*, uint64_t*, uint32_t, uint64_t,
                                                    FrameResult*, uint32_t*, hipStream_t);
extern "C" hipError_t capnp_launch_msg_pack_service(const uint64_t*, uint64_t*, uint32_t, uint64_t,
                                                    uint32_t*, hipStream_t);

namespace {

constexpr uint32_t kDefaultTileChunks = 16;
constexpr uint32_t kMaxTileChunks = 64;

size_t round16(size_t x) { return (x + 15) & ~size_t(15); }

}  // namespace

constexpr size_t kTablePrefixBytes = 4096;  // >= 10 bytes x (1 + 256) table words
// message bodies of at least this many words decode in parallel (read_body)
#ifndef PARALLEL_BODY_WORDS
#define PARALLEL_BODY_WORDS 65536  // (32768: a 256 KiB read 224 us; 65536: 174; 131072: a 512 KiB read 353 vs 237)
#endif
constexpr uint64_t kParallelBodyWords = PARALLEL_BODY_WORDS;

// A resident service for one kind of one-launch call (0: msg_read_kernel,
// 1: msg_pack_kernel): one workgroup on its own stream polls a pinned
// request line and serves each request without a launch (common.h,
// svc_next).  Pinned block: [0, 8) the request line (bell, six arguments,
// check), [8] the exit mark (the last generation that exited).
struct CallSvc {
    hipStream_t s = nullptr;
    uint64_t* h = nullptr;
    uint64_t* d = nullptr;
    // The request line: h, or with CAPNP_SVC_LINE_BAR=1 device memory the
    // host writes through the BAR (req_buf; the service then polls HBM
    // instead of reading across PCIe: profiles/r06q_bar_probe.txt "fgfg").
    uint64_t* line = nullptr;         // the host's view
    const uint64_t* line_d = nullptr;  // the service's
    bool line_dev = false;
    uint64_t args[kSvcArgs] = {};     // the current request's (the check is made from these)
    uint64_t bell = 0;                // the last bell rung
    uint32_t gen = 0;
    bool live = false;  // a service of `gen` was started and may still run
    std::chrono::steady_clock::time_point last{};  // its last completed request
};

struct capnp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint8_t* d_state = nullptr;   // pack look-back records (tiles, groups)
    size_t state_cap = 0;
    uint8_t* d_stage = nullptr;   // staging for the host APIs (inputs)
    size_t stage_cap = 0;
    uint8_t* d_body = nullptr;    // staging for decoded message bodies
    size_t body_cap = 0;
    FrameResult* d_frame = nullptr;
    FrameResult* h_frame = nullptr;  // pinned
    // streaming host batch (capnp_stream_*): copy-in, compute and copy-out
    // streams, two device staging slots and their events
    hipStream_t sstream[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_in[2] = {}, ev_comp[2] = {}, ev_off[2] = {}, ev_out[2] = {};
    uint8_t* d_slot[2] = {nullptr, nullptr};
    size_t slot_cap = 0;
    uint64_t* h_slot_off[2] = {nullptr, nullptr};  // pinned: a slice's packed offsets
    size_t h_slot_off_cap = 0;
    uint8_t* d_msg = nullptr;  // batch message framing: staging words and tables
    size_t msg_cap = 0;
    uint8_t* d_resync = nullptr;  // index-free decode: per-block chain state
    size_t resync_cap = 0;
    uint8_t* d_wt = nullptr;  // word-tile unpack: per-tile plans and piece flags
    size_t wt_cap = 0;
    uint8_t* d_pwt = nullptr;  // word-tile pack: range map and tile offsets
    size_t pwt_cap = 0;
    uint8_t* d_stream_words = nullptr;  // message discovery: the stream decoded to words
    size_t stream_words_cap = 0;
    int resync_passes = 0, resync_serial = 0;  // last capnp_gpu_unpack_batch_resync
    const int32_t* resync_failed = nullptr;     // its device "a chunk failed" flag (read on demand)
    hipStream_t resync_stream = nullptr;
    hipEvent_t ev_resync = nullptr;  // orders a resync decode after the previous one
    uint32_t* d_bad = nullptr;  // offset validation: flag, then each array's ends (check_offsets)
    uint32_t* h_bad = nullptr;  // pinned copy (kCheckBytes)
    uint8_t* h_pin = nullptr;   // pinned staging of the small host calls (kPinnedCall)
    uint8_t* d_pin = nullptr;   // ... its device address (the one-launch calls read and write it)
    size_t pin_cap = 0;
    FrameResult* d_hframe = nullptr;  // h_frame's device address
    uint8_t* d_req = nullptr;    // per-message calls' inputs, written by the host through the BAR
    int req_ok = -1;             // ... whether the device allows that (-1: not asked yet)
    uint32_t* h_flag = nullptr;  // pinned: the one-launch calls' completion flag
    uint32_t* d_flag = nullptr;  // ... its device address
    uint32_t call_seq = 0;
    CallSvc svc[2];  // resident services of the per-message calls (read, write)
    std::chrono::steady_clock::time_point percall_last{};  // the last per-message call
    bool percall_any = false;
    // Caller streams that ran this context's device work: an event recorded on
    // each after its last call, so a workspace that has to grow waits for that
    // work only (not for every stream of the device), and destroy too.
    static constexpr int kUseSlots = 8;
    hipStream_t use_s[kUseSlots] = {};
    hipEvent_t use_ev[kUseSlots] = {};
    int use_next = 0;
    std::string err;
};

// Host calls whose staging fits this many bytes go through a pinned buffer:
// one copy in and one copy out, each a plain DMA (a pageable copy is staged
// by the runtime in pieces, and each costs a synchronisation).  That is the
// drop-in's per-message cost (write_message / read_message at the
// reference's call granularity).
constexpr size_t kPinnedCall = size_t(4) << 20;
// write_message past the one-launch kernel's size goes through the pinned
// buffer up to this many staged bytes (its host copies are not pipelined
// with the DMA, the runtime's pageable path is: larger messages take that)
#ifndef WRITE_PIN_MAX
#define WRITE_PIN_MAX kPinnedCall  // (1 MiB message: 137 vs 165 us pageable, 64 KiB 69 vs 85)
#endif
constexpr size_t kWritePinMax = WRITE_PIN_MAX;

namespace {

// Offset-array validation for the synchronising entry points: off[0..n] must
// be non-decreasing and off[n] <= limit.  A kernel handed backwards offsets
// would read or write outside the caller's buffers (a chunk of "negative"
// length), so these calls return CAPNP_E_INVALID_ARGUMENT before any kernel
// touches the data.  (The reference takes slices, which cannot be backwards:
// serialize.rs:53-97, serialize_packed.rs:300-304.)
// ends = {off[0], off[n]}: the array's range, copied back with the verdict
// (the callers that size their launches from it read no more).
__global__ void __launch_bounds__(256) k_check_offsets(const uint64_t* __restrict__ off,
                                                       uint64_t n, uint64_t limit,
                                                       uint32_t* __restrict__ bad,
                                                       uint64_t* __restrict__ ends) {
    const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i0 == 0) {
        ends[0] = off[0];
        ends[1] = off[n];
    }
    for (uint64_t i = i0; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = off[i], b = off[i + 1];
        if (b < a || b > limit) atomicOr(bad, 1u);  // (vector atomic, rare)
    }
}

// check_offsets' device record: the flag (8 bytes with its pad), then
// {first, last} of up to kCheckArrays arrays.
constexpr size_t kCheckArrays = 3;
constexpr size_t kCheckBytes = 8 + 16 * kCheckArrays;

}  // namespace

namespace {

capnp_status fail(capnp_ctx* ctx, hipError_t e, const char* what) {
    if (ctx) ctx->err = std::string(what) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? CAPNP_E_OUT_OF_MEMORY : CAPNP_E_HIP;
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return fail(ctx, e_, #expr); \
    } while (0)

// Device batch APIs are ordered on the caller's stream; NULL is the HIP null
// (default) stream, as everywhere in HIP.
hipStream_t pick(capnp_ctx*, void* s) { return (hipStream_t)s; }

// Records that `s` now holds work of this context (called when a call that
// enqueued on a caller's stream returns).  Work under stream capture is the
// caller's graph: it is not tracked.
void mark_use(capnp_ctx* ctx, hipStream_t s) {
    if (s == ctx->stream) return;  // (ctx->stream is synchronised directly)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
    int k = 0;
    while (k < capnp_ctx::kUseSlots && !(ctx->use_ev[k] && ctx->use_s[k] == s)) k++;
    if (k == capnp_ctx::kUseSlots) {
        k = ctx->use_next;
        ctx->use_next = (k + 1) % capnp_ctx::kUseSlots;
        if (ctx->use_ev[k]) {
            (void)hipEventSynchronize(ctx->use_ev[k]);  // (the slot's stream drops out)
        } else if (hipEventCreateWithFlags(&ctx->use_ev[k], hipEventDisableTiming) != hipSuccess) {
            ctx->use_ev[k] = nullptr;
            (void)hipStreamSynchronize(s);  // (no event: wait now instead)
            return;
        }
    }
    ctx->use_s[k] = s;
    if (hipEventRecord(ctx->use_ev[k], s) != hipSuccess) (void)hipStreamSynchronize(s);
}

struct UseMark {
    capnp_ctx* ctx;
    hipStream_t s;
    ~UseMark() {
        if (ctx) mark_use(ctx, s);
    }
};

// Waits for every piece of work this context has queued: its own streams and
// the caller streams marked above (before a workspace is freed).
void svc_stop_all(capnp_ctx* ctx);

hipError_t wait_uses(capnp_ctx* ctx) {
    svc_stop_all(ctx);  // (a resident per-call service: stopped before buffers move)
    hipError_t e = hipSuccess, r;
    if (ctx->stream && (r = hipStreamSynchronize(ctx->stream)) != hipSuccess) e = r;
    for (int k = 0; k < capnp_ctx::kUseSlots; k++)
        if (ctx->use_ev[k] && ctx->use_s[k] && (r = hipEventSynchronize(ctx->use_ev[k])) != hipSuccess)
            e = r;
    for (int k = 0; k < 3; k++)
        if (ctx->sstream[k] && (r = hipStreamSynchronize(ctx->sstream[k])) != hipSuccess) e = r;
    return e;
}

capnp_status ensure_state(capnp_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->state_cap) return CAPNP_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    if (ctx->d_state) {
        HIP_TRY(wait_uses(ctx));
        HIP_TRY(hipFree(ctx->d_state));
        ctx->d_state = nullptr;
        ctx->state_cap = 0;
    }
    size_t cap = std::max<size_t>(bytes, 1 << 16);
#if CAPNP_STATE_ALLOC == 1
    HIP_TRY(hipExtMallocWithFlags(reinterpret_cast<void**>(&ctx->d_state), cap,
                                  hipDeviceMallocUncached));
#elif CAPNP_STATE_ALLOC == 2
    HIP_TRY(hipExtMallocWithFlags(reinterpret_cast<void**>(&ctx->d_state), cap,
                                  hipDeviceMallocFinegrained));
#else
    HIP_TRY(hipMalloc(&ctx->d_state, cap));
#endif
    ctx->state_cap = cap;
    return CAPNP_OK;
}

// The last index-free decode's "a chunk failed its check" flag lives in the
// resync workspace and is read on demand (capnp_resync_stats), or here before
// the workspace is reused or reallocated.
capnp_status settle_resync(capnp_ctx* ctx) {
    if (!ctx->resync_failed) return CAPNP_OK;
    int32_t f = 0;
    HIP_TRY(hipStreamSynchronize(ctx->resync_stream));
    HIP_TRY(hipMemcpy(&f, ctx->resync_failed, 4, hipMemcpyDeviceToHost));
    if (f) ctx->resync_serial = 3;
    ctx->resync_failed = nullptr;
    return CAPNP_OK;
}

capnp_status ensure_buf(capnp_ctx* ctx, uint8_t** buf, size_t* cap_io, size_t bytes) {
    if (buf == &ctx->d_resync) {
        const capnp_status st = settle_resync(ctx);
        if (st != CAPNP_OK) return st;
    }
    if (bytes <= *cap_io) return CAPNP_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    if (*buf) {
        // (work queued on a caller's stream, not only ctx->stream, may still
        // use the buffer: the device batch calls run on the caller's stream
        // and are marked there, mark_use)
        HIP_TRY(wait_uses(ctx));
        HIP_TRY(hipFree(*buf));
        *buf = nullptr;
        *cap_io = 0;
    }
    size_t cap = std::max<size_t>(round16(bytes) + 64, 1 << 20);
    HIP_TRY(hipMalloc(buf, cap));
    *cap_io = cap;
    return CAPNP_OK;
}

capnp_status ensure_stage(capnp_ctx* ctx, size_t bytes) {
    return ensure_buf(ctx, &ctx->d_stage, &ctx->stage_cap, bytes);
}

capnp_status ensure_pin(capnp_ctx* ctx, size_t bytes) {
    if (bytes <= ctx->pin_cap) return CAPNP_OK;
    HIP_TRY(hipSetDevice(ctx->device));
    if (ctx->h_pin) {
        svc_stop_all(ctx);
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        HIP_TRY(hipHostFree(ctx->h_pin));
        ctx->h_pin = nullptr;
        ctx->pin_cap = 0;
    }
    const size_t cap = std::max<size_t>(round16(bytes) + 64, 1 << 16);
    HIP_TRY(hipHostMalloc(&ctx->h_pin, cap, 0));
    ctx->pin_cap = cap;
    void* dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, ctx->h_pin, 0));
    ctx->d_pin = static_cast<uint8_t*>(dp);
    return CAPNP_OK;
}

// The per-message calls' inputs (the staged read prefix, the laid-out write
// words and offsets) go to device memory that the host writes through the
// PCI BAR, on devices whose whole memory is mapped there (large BAR): the
// host's stores are posted writes and the kernel reads HBM, where from
// pinned memory every fetch was a PCIe read round trip
// (scripts/bar_probe.hip, profiles/r06q_bar_probe.txt: a 12 KB request
// 8.98 -> 5.6 us, 6.6 KB 6.62 -> 4.7).  Fine-grained memory: the kernel's
// system-scope acquire (the service) or its launch sees the bytes.  Outputs
// stay in pinned memory (host reads through the BAR are uncached).  Inputs
// past kReqBytes, devices without a large BAR and CAPNP_PERCALL_BAR=0 use
// the pinned buffer.
constexpr size_t kReqBytes = size_t(1) << 20;

uint8_t* req_buf(capnp_ctx* ctx, size_t bytes) {
    if (bytes > kReqBytes) return nullptr;
    if (ctx->req_ok < 0) {
        static const bool enabled = [] {
            const char* e = getenv("CAPNP_PERCALL_BAR");
            return !(e && e[0] == '0');
        }();
        int large = 0;
        ctx->req_ok = 0;
        if (enabled && hipSetDevice(ctx->device) == hipSuccess &&
            hipDeviceGetAttribute(&large, hipDeviceAttributeIsLargeBar, ctx->device) == hipSuccess &&
            large == 1 &&
            hipExtMallocWithFlags(reinterpret_cast<void**>(&ctx->d_req), kReqBytes + 64,
                                  hipDeviceMallocFinegrained) == hipSuccess)
            ctx->req_ok = 1;
        else
            ctx->d_req = nullptr;
    }
    return ctx->req_ok ? ctx->d_req : nullptr;
}

// The host's stores into req_buf reach the device before what follows them
// (a service's bell, a launch's doorbell).
inline void req_done() { __builtin_ia32_sfence(); }

// Waits for a one-launch call (msg_read_kernel / msg_pack_kernel) by its
// completion flag in pinned memory: the kernel stores `seq` there after its
// results, and polling the flag returns a few microseconds sooner than the
// runtime's stream wait (the per-message calls are latency-bound).  A call
// that has not finished within ~5 ms, or failed, falls to that wait, which
// reports the error.
capnp_status wait_call(capnp_ctx* ctx, uint32_t seq, hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; i++) {
        if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE) == seq) return CAPNP_OK;
        __builtin_ia32_pause();
        if ((i & 1023) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(5))
            break;
    }
    HIP_TRY(hipStreamSynchronize(s));
    if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE) != seq) {
        ctx->err = "one-launch call finished without its completion flag";
        return CAPNP_E_HIP;
    }
    return CAPNP_OK;
}

// ---- resident per-call services (CallSvc) ----
// A per-message call within kSvcWarm of the previous one goes to the resident
// service of its kind instead of a launch (profiles/r06j_doorbell*.txt: a
// request's round trip 2.9 vs 7.2 us for an empty call, 4.9 vs 9.2 for a
// 1 KiB one).  A service that completed a request within kSvcTrust is rung
// directly; otherwise a new generation starts (an older one, if still
// polling, exits when it sees the new bell).  The workgroup exits after
// kSvcIdleTicks without a request: while resident it holds its hardware
// queue, so it must not outlive a burst of calls by long.  Its streams are
// non-blocking and of the highest priority (the normal-priority streams'
// queues are not shared with it: profiles/r06j_doorbell_queues.txt).
constexpr auto kSvcWarm = std::chrono::microseconds(1000);
constexpr auto kSvcTrust = std::chrono::microseconds(150);
constexpr uint64_t kSvcIdleTicks = 100 * 250;  // 250 us of the 100 MHz clock
constexpr auto kSvcCheck = std::chrono::microseconds(100);
constexpr auto kSvcGiveUp = std::chrono::milliseconds(200);

std::mutex g_svc_mu;
std::vector<capnp_ctx*>* g_svc_ctxs = nullptr;  // contexts that started a service

void svc_bell(CallSvc& v, uint64_t b) {
    // (the arguments, the check and the payload before the bell, non-temporal
    // and write-combined stores included)
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    __atomic_store_n(&v.line[0], b, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    v.bell = b;
}

// The request line for bell b (the arguments from v.args; the line is only
// written: host reads through the BAR are uncached), then the bell.
void svc_ring(CallSvc& v, uint64_t b) {
    for (uint32_t i = 0; i < kSvcArgs; i++) v.line[1 + i] = v.args[i];
    v.line[7] = svc_mix(b, v.args);
    svc_bell(v, b);
}

// Stops service k (it exits at its next poll) and waits for it.
void svc_stop(capnp_ctx* ctx, int k) {
    CallSvc& v = ctx->svc[k];
    if (!v.s || !v.live) return;
    svc_bell(v, 0);  // (generation 0 is never started)
    (void)hipStreamSynchronize(v.s);
    v.live = false;
}

void svc_stop_all(capnp_ctx* ctx) {
    svc_stop(ctx, 0);
    svc_stop(ctx, 1);
}

// Process exit with a service still resident (a context never destroyed):
// the stop bell, then a bounded wait for its exit mark (no runtime calls).
void svc_atexit() {
    std::lock_guard<std::mutex> g(g_svc_mu);
    if (!g_svc_ctxs) return;
    for (capnp_ctx* ctx : *g_svc_ctxs)
        for (CallSvc& v : ctx->svc) {
            if (!v.live || !v.line) continue;
            svc_bell(v, 0);
            const auto t0 = std::chrono::steady_clock::now();
            while (__atomic_load_n(&v.h[8], __ATOMIC_ACQUIRE) != v.gen &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(20))
                __builtin_ia32_pause();
        }
}

capnp_status svc_init(capnp_ctx* ctx, int k) {
    CallSvc& v = ctx->svc[k];
    if (v.s) return CAPNP_OK;
    HIP_TRY(hipSetDevice(ctx->device));  // (the stream and the line are this device's)
    int lo = 0, hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_TRY(hipHostMalloc(&v.h, 256, 0));
    memset(v.h, 0, 256);
    void* dp = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dp, v.h, 0));
    v.d = static_cast<uint64_t*>(dp);
    v.line = v.h;
    v.line_d = v.d;
    void* ld = nullptr;
    // (off by default: measured no faster -- carsales pair 35.3 / 35.4 vs
    // 35.2 / 35.1 us, writes 0.3-0.5 us slower, reads 0.1-0.3 faster,
    // profiles/r06q_line_ab.txt; CAPNP_SVC_LINE_BAR=1 turns it on)
    static const bool line_bar = [] {
        const char* e = getenv("CAPNP_SVC_LINE_BAR");
        return e && e[0] == '1';
    }();
    if (line_bar && req_buf(ctx, 0) &&
        hipExtMallocWithFlags(&ld, 256, hipDeviceMallocFinegrained) == hipSuccess) {
        v.line = static_cast<uint64_t*>(ld);
        v.line_d = v.line;
        v.line_dev = true;
        for (int i = 0; i < 8; i++) v.line[i] = 0;
        __builtin_ia32_sfence();
    }
    HIP_TRY(hipStreamCreateWithPriority(&v.s, hipStreamNonBlocking, hi));
    std::lock_guard<std::mutex> g(g_svc_mu);
    if (!g_svc_ctxs) {
        g_svc_ctxs = new std::vector<capnp_ctx*>();
        atexit(svc_atexit);
    }
    if (std::find(g_svc_ctxs->begin(), g_svc_ctxs->end(), ctx) == g_svc_ctxs->end())
        g_svc_ctxs->push_back(ctx);
    return CAPNP_OK;
}

// A new generation of service k, rung for request `seq` before its launch.
capnp_status svc_start(capnp_ctx* ctx, int k, uint32_t seq) {
    CallSvc& v = ctx->svc[k];
    if (++v.gen == 0) v.gen = 1;
    svc_ring(v, ((uint64_t)v.gen << 32) | seq);
    v.live = true;
    HIP_TRY(k == 0 ? capnp_launch_msg_read_service(v.line_d, v.d + 8, v.gen, kSvcIdleTicks,
                                                   ctx->d_hframe, ctx->d_flag, v.s)
                   : capnp_launch_msg_pack_service(v.line_d, v.d + 8, v.gen, kSvcIdleTicks,
                                                   ctx->d_flag, v.s));
    return CAPNP_OK;
}

// One request to service k: the arguments (kSvcArgs), the request line, the
// wait for the completion flag (`seq`).  A service that has exited before
// seeing the bell (its stream is idle and the flag not set) is started again.
capnp_status svc_call(capnp_ctx* ctx, int k, const uint64_t* args, uint32_t seq) {
    capnp_status st = svc_init(ctx, k);
    if (st != CAPNP_OK) return st;
    CallSvc& v = ctx->svc[k];
    memcpy(v.args, args, kSvcArgs * sizeof(uint64_t));
    const auto t0 = std::chrono::steady_clock::now();
    if (v.live && t0 - v.last <= kSvcTrust) {
        svc_ring(v, ((uint64_t)v.gen << 32) | seq);
    } else if ((st = svc_start(ctx, k, seq)) != CAPNP_OK) {
        return st;
    }
    auto check = t0;
    for (uint32_t i = 1;; i++) {
        if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE) == seq) {
            v.last = std::chrono::steady_clock::now();
            return CAPNP_OK;
        }
        __builtin_ia32_pause();
        if ((i & 255) == 0) {
            const auto t = std::chrono::steady_clock::now();
            if (t - check > kSvcCheck) {
                check = t;
                if (hipStreamQuery(v.s) == hipSuccess &&
                    __atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE) != seq &&
                    (st = svc_start(ctx, k, seq)) != CAPNP_OK)
                    return st;
            }
            if (t - t0 > kSvcGiveUp) break;
        }
    }
    const hipError_t q = hipStreamQuery(v.s);
    char diag[200];
    snprintf(diag, sizeof diag, " (kind %d, bell %llx, exit mark %llu, flag %u, seq %u, stream %d)",
             k, (unsigned long long)v.bell, (unsigned long long)v.h[8],
             __atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE), seq, (int)q);
    svc_stop(ctx, k);
    if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE) == seq) return CAPNP_OK;
    ctx->err = std::string("the per-call service did not complete the request") + diag;
    return CAPNP_E_HIP;
}

// The next call's completion value (never 0: a new service has served none).
uint32_t next_seq(capnp_ctx* ctx) {
    if (++ctx->call_seq == 0) ++ctx->call_seq;
    return ctx->call_seq;
}

// Whether this per-message call goes to a resident service (the previous one
// was recent); percall_done notes when the call ended.
bool percall_warm(capnp_ctx* ctx) {
    // (CAPNP_PERCALL_SERVICE=0: every call launches, for A/B measurements)
    static const bool enabled = [] {
        const char* e = getenv("CAPNP_PERCALL_SERVICE");
        return !(e && e[0] == '0');
    }();
    if (!enabled) return false;
    const auto now = std::chrono::steady_clock::now();
    const bool warm = ctx->percall_any && now - ctx->percall_last <= kSvcWarm;
    ctx->percall_any = true;
    return warm;
}
void percall_done(capnp_ctx* ctx) { ctx->percall_last = std::chrono::steady_clock::now(); }

// Enqueues the checks of `arrays` (device offset arrays of n + 1 entries with
// their limits) on `s`, copies the verdict to the pinned flag and waits for
// it.  CAPNP_OK, CAPNP_E_INVALID_ARGUMENT or a HIP error.
struct OffCheck {
    const uint64_t* off;
    size_t n;
    uint64_t limit;
};
// With wait == false the verdict is only enqueued: the caller synchronises
// `s` itself (it has its own reason to) and then calls offsets_verdict().
capnp_status offsets_verdict(capnp_ctx* ctx) {
    if (*ctx->h_bad) {
        ctx->err = "offset array not non-decreasing or past its buffer";
        return CAPNP_E_INVALID_ARGUMENT;
    }
    return CAPNP_OK;
}
// After the wait: array k's {off[0], off[n]} (arrays with n > 0 only).
const uint64_t* checked_ends(const capnp_ctx* ctx, size_t k) {
    return reinterpret_cast<const uint64_t*>(ctx->h_bad + 2) + 2 * k;
}
capnp_status check_offsets(capnp_ctx* ctx, hipStream_t s, std::initializer_list<OffCheck> arrays,
                           bool wait = true) {
    if (arrays.size() > kCheckArrays) return CAPNP_E_INVALID_ARGUMENT;
    HIP_TRY(hipMemsetAsync(ctx->d_bad, 0, 4, s));
    size_t k = 0;
    for (const OffCheck& a : arrays) {
        uint64_t* ends = reinterpret_cast<uint64_t*>(ctx->d_bad + 2) + 2 * k++;
        if (a.n == 0 || !a.off) continue;
        const uint64_t blocks = std::min<uint64_t>((a.n + 255) / 256, 2048);
        hipLaunchKernelGGL(k_check_offsets, dim3((uint32_t)blocks), dim3(256), 0, s, a.off,
                           (uint64_t)a.n, a.limit, ctx->d_bad, ends);
        HIP_TRY(hipGetLastError());
    }
    // the verdict and the ranges in one copy (pinned: no staging)
    HIP_TRY(hipMemcpyAsync(ctx->h_bad, ctx->d_bad, 8 + 16 * k, hipMemcpyDeviceToHost, s));
    if (!wait) return CAPNP_OK;
    HIP_TRY(hipStreamSynchronize(s));
    return offsets_verdict(ctx);
}


size_t state_bytes_for(size_t nchunks, uint32_t tc) {
    return capnp_pack_state_bytes(nchunks, tc) + 16;
}

// Chunks per pack tile: the staged path holds capnp_pack_tile_words() / 64
// steps of 64 words per tile, and a chunk takes whole steps, so the budget
// is counted in steps of the mean chunk (a 32-word chunk still takes one).
uint32_t tile_chunks_for(uint64_t total_words, size_t n) {
    if (n == 0) return kDefaultTileChunks;
    const double mean = (double)total_words / (double)n;
    const double steps = std::max(1.0, std::ceil(mean / 64.0));
    double t = (double)(capnp_pack_tile_words() / 64) / steps;
    uint32_t tc = (uint32_t)std::max(1.0, std::min(t, (double)kMaxTileChunks));
    return tc;
}

// Diagnostics: CAPNP_WORD_TILES=1 takes the word tiles for every tc == 0 call.
bool force_word_tiles() {
    static const bool v = [] {
        const char* e = getenv("CAPNP_WORD_TILES");
        return e && e[0] == '1';
    }();
    return v;
}

// Batches whose mean chunk is at least this many words pack (and, with the
// record sync index, unpack) in word tiles.
constexpr uint64_t kWordTileMean = 512;
// index-free batches of at least kLongUnitsMin units whose mean is in
// [kLongUnitWords, kBlockDecodeWords) decode one unit per workgroup
constexpr uint64_t kLongUnitsMin = 256;
constexpr uint64_t kLongUnitWords = 2048;
constexpr uint64_t kBlockDecodeWords = 32768;

// tc == 0: the launch is sized from the batch's word range (one
// synchronisation to read it): word tiles (capnp_launch_pack_wt: chunks of
// any length) for a mean chunk of at least kWordTileMean words, else chunk
// tiles of about capnp_pack_tile_words() words.
// host_wr: the batch's word range when the caller already knows it (and has
// validated the offsets on the host): no synchronisation at all.
capnp_status pack_batch_dev(capnp_ctx* ctx, const uint64_t* d_words, const uint64_t* d_off,
                            size_t n, uint8_t* d_out, size_t cap, uint64_t* d_out_off,
                            uint32_t tc, hipStream_t s, uint32_t* d_sync = nullptr,
                            const uint64_t* host_wr = nullptr) {
    if (n > 0 && !d_off) return CAPNP_E_INVALID_ARGUMENT;
    if (!d_out_off) return CAPNP_E_INVALID_ARGUMENT;
    UseMark um{ctx, s};
    if (tc == 0 && n > 0) {
        uint64_t wr[2];
        if (host_wr) {
            wr[0] = host_wr[0];
            wr[1] = host_wr[1];
        } else {
            capnp_status vst = check_offsets(ctx, s, {{d_off, n, ~0ull}});
            if (vst != CAPNP_OK) return vst;
            wr[0] = checked_ends(ctx, 0)[0];
            wr[1] = checked_ends(ctx, 0)[1];
        }
        if (wr[1] < wr[0]) return CAPNP_E_INVALID_ARGUMENT;
        const uint64_t words = wr[1] - wr[0];
        if (words && (words / n >= kWordTileMean || force_word_tiles())) {
            const uint64_t ntiles = capnp_pack_wt_tiles(wr[0], wr[1]);
            capnp_status st = ensure_state(ctx, capnp_pack_state_bytes(ntiles, 1) + 16);
            if (st != CAPNP_OK) return st;
            st = ensure_buf(ctx, &ctx->d_pwt, &ctx->pwt_cap, capnp_pack_wt_ws_bytes(wr[0], wr[1]));
            if (st != CAPNP_OK) return st;
            HIP_TRY(capnp_launch_pack_wt(d_words, d_off, n, d_out, cap, d_out_off,
                                         reinterpret_cast<uint64_t*>(ctx->d_state), ctx->d_pwt,
                                         ctx->pwt_cap, d_sync, wr[0], wr[1], s));
            return CAPNP_OK;
        }
        tc = tile_chunks_for(words, n);
    }
    if (tc == 0) tc = kDefaultTileChunks;
    if (tc > kMaxTileChunks) return CAPNP_E_INVALID_ARGUMENT;
    const size_t sb = state_bytes_for(n, tc);
    capnp_status st = ensure_state(ctx, sb);
    if (st != CAPNP_OK) return st;
    HIP_TRY(capnp_launch_pack(d_words, d_off, n, tc, d_out, cap, d_out_off,
                              reinterpret_cast<uint64_t*>(ctx->d_state), d_sync, s));
    return CAPNP_OK;
}

// Host batch pack through the staging buffer.  Returns the needed size in
// *total; writes min(total, out_cap) bytes to `out`.
capnp_status pack_host(capnp_ctx* ctx, const uint64_t* words, const uint64_t* off, size_t n,
                       uint8_t* out, size_t out_cap, uint64_t* out_off_host, uint64_t* total) {
    const uint64_t base = n ? off[0] : 0;
    const uint64_t nw = n ? off[n] - base : 0;
    std::vector<uint64_t> rel(n + 1);
    for (size_t i = 0; i <= n; i++) {
        rel[i] = n ? off[i] - base : 0;
        if (i && off[i] < off[i - 1]) return CAPNP_E_INVALID_ARGUMENT;  // (checked here, on the host)
    }
    const uint64_t wr[2] = {0, nw};
    const size_t bound = capnp_packed_batch_bound_bytes(nw, n);
    const size_t o_words = 0;
    const size_t o_off = round16(nw * 8);
    const size_t o_oo = o_off + round16((n + 1) * 8);
    const size_t o_out = o_oo + round16((n + 1) * 8);
    capnp_status st = ensure_stage(ctx, o_out + bound + 16);
    if (st != CAPNP_OK) return st;
    uint8_t* d = ctx->d_stage;
    hipStream_t s = ctx->stream;
    const uint32_t tc = (n && nw / n >= kWordTileMean) ? 0u : tile_chunks_for(nw, n);
    if (o_out + bound <= kPinnedCall) {
        // small call: words and offsets in, offsets and the bound's bytes
        // out, through the pinned buffer: one copy each way, one wait
        st = ensure_pin(ctx, o_out + bound + 16);
        if (st != CAPNP_OK) return st;
        uint8_t* h = ctx->h_pin;
        if (nw) memcpy(h + o_words, words + base, nw * 8);
        memcpy(h + o_off, rel.data(), (n + 1) * 8);
        HIP_TRY(hipMemcpyAsync(d, h, o_oo, hipMemcpyHostToDevice, s));
        st = pack_batch_dev(ctx, reinterpret_cast<uint64_t*>(d + o_words),
                            reinterpret_cast<uint64_t*>(d + o_off), n, d + o_out, bound,
                            reinterpret_cast<uint64_t*>(d + o_oo), tc, s, nullptr, wr);
        if (st != CAPNP_OK) return st;
        HIP_TRY(hipMemcpyAsync(h + o_oo, d + o_oo, o_out - o_oo + bound, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        const uint64_t* oo = reinterpret_cast<const uint64_t*>(h + o_oo);
        *total = oo[n];
        const size_t ncopy = std::min<uint64_t>(oo[n], out_cap);
        if (ncopy) memcpy(out, h + o_out, ncopy);
        if (out_off_host) memcpy(out_off_host, oo, (n + 1) * 8);
        return oo[n] > out_cap ? CAPNP_E_BUFFER_NOT_LARGE_ENOUGH : CAPNP_OK;
    }
    if (nw) HIP_TRY(hipMemcpyAsync(d + o_words, words + base, nw * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d + o_off, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
    st = pack_batch_dev(ctx, reinterpret_cast<uint64_t*>(d + o_words),
                        reinterpret_cast<uint64_t*>(d + o_off), n, d + o_out, bound,
                        reinterpret_cast<uint64_t*>(d + o_oo), tc, s, nullptr, wr);
    if (st != CAPNP_OK) return st;
    std::vector<uint64_t> oo(n + 1);
    HIP_TRY(hipMemcpyAsync(oo.data(), d + o_oo, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    *total = oo[n];
    const size_t ncopy = std::min<uint64_t>(oo[n], out_cap);
    if (ncopy) {
        HIP_TRY(hipMemcpyAsync(out, d + o_out, ncopy, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    if (out_off_host) memcpy(out_off_host, oo.data(), (n + 1) * 8);
    return oo[n] > out_cap ? CAPNP_E_BUFFER_NOT_LARGE_ENOUGH : CAPNP_OK;
}

// ---- streaming host batch ------------------------------------------------
constexpr size_t kDefaultSliceWords = size_t(4) << 20;  // 32 MiB of words (scripts/stream_sweep.py)
constexpr size_t kSlotPad = 64;  // staging slack: the kernels read whole aligned blocks

capnp_status stream_setup(capnp_ctx* ctx, size_t slot_bytes, size_t off_entries) {
    HIP_TRY(hipSetDevice(ctx->device));
    if (!ctx->sstream[0]) {
        for (int k = 0; k < 3; k++)
            HIP_TRY(hipStreamCreateWithFlags(&ctx->sstream[k], hipStreamNonBlocking));
        for (int k = 0; k < 2; k++) {
            HIP_TRY(hipEventCreateWithFlags(&ctx->ev_in[k], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&ctx->ev_comp[k], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&ctx->ev_off[k], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&ctx->ev_out[k], hipEventDisableTiming));
        }
    }
    if (slot_bytes > ctx->slot_cap) {
        for (int k = 0; k < 2; k++) {
            if (ctx->d_slot[k]) HIP_TRY(hipFree(ctx->d_slot[k]));
            ctx->d_slot[k] = nullptr;
        }
        ctx->slot_cap = 0;
        for (int k = 0; k < 2; k++) HIP_TRY(hipMalloc(&ctx->d_slot[k], slot_bytes));
        ctx->slot_cap = slot_bytes;
    }
    if (off_entries > ctx->h_slot_off_cap) {
        for (int k = 0; k < 2; k++) {
            if (ctx->h_slot_off[k]) HIP_TRY(hipHostFree(ctx->h_slot_off[k]));
            ctx->h_slot_off[k] = nullptr;
        }
        ctx->h_slot_off_cap = 0;
        for (int k = 0; k < 2; k++)
            HIP_TRY(hipHostMalloc(&ctx->h_slot_off[k], off_entries * 8, 0));
        ctx->h_slot_off_cap = off_entries;
    }
    return CAPNP_OK;
}

// Chunk-aligned slices of about slice_words words (at least one chunk each).
std::vector<size_t> make_slices(const uint64_t* off, size_t n, size_t slice_words) {
    std::vector<size_t> b{0};
    size_t s = 0;
    while (s < n) {
        size_t e = s + 1;
        while (e < n && off[e + 1] - off[s] <= slice_words) e++;
        b.push_back(e);
        s = e;
    }
    return b;
}

}  // namespace

extern "C" {

const char* capnp_version(void) { return "capnp-packed-mi355x 0.1.0 (gfx950)"; }

uint32_t capnp_abi_version(void) { return CAPNP_ABI_VERSION; }

capnp_reader_options capnp_default_reader_options(void) {
    capnp_reader_options o;
    o.traversal_limit_in_words = 8ull * 1024 * 1024;
    o.has_traversal_limit = 1;
    o.nesting_limit = 64;
    return o;
}

size_t capnp_packed_bound_bytes(size_t words) {
    return words ? 8 * words + (words + 1) / 2 + 2 : 0;
}

size_t capnp_packed_batch_bound_bytes(size_t total_words, size_t nchunks) {
    return 8 * total_words + (total_words + nchunks) / 2 + 2 * nchunks + 16;
}

capnp_ctx* capnp_ctx_create(int device, capnp_status* status) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) {
        if (status) *status = CAPNP_E_NO_DEVICE;
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess ||
        strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        if (status) *status = CAPNP_E_NO_DEVICE;
        return nullptr;
    }
    capnp_ctx* ctx = new capnp_ctx();
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&ctx->d_frame, sizeof(FrameResult));
    if (e == hipSuccess) e = hipHostMalloc(&ctx->h_frame, sizeof(FrameResult), 0);
    if (e == hipSuccess) {
        void* dp = nullptr;
        e = hipHostGetDevicePointer(&dp, ctx->h_frame, 0);
        ctx->d_hframe = static_cast<FrameResult*>(dp);
    }
    if (e == hipSuccess) e = hipHostMalloc(&ctx->h_flag, 64, 0);
    if (e == hipSuccess) {
        *ctx->h_flag = 0;
        void* dp = nullptr;
        e = hipHostGetDevicePointer(&dp, ctx->h_flag, 0);
        ctx->d_flag = static_cast<uint32_t*>(dp);
    }
    if (e == hipSuccess) e = hipMalloc(&ctx->d_bad, kCheckBytes);
    if (e == hipSuccess) e = hipHostMalloc(&ctx->h_bad, kCheckBytes, 0);
    if (e != hipSuccess) {
        if (status) *status = CAPNP_E_HIP;
        capnp_ctx_destroy(ctx);
        return nullptr;
    }
    if (status) *status = CAPNP_OK;
    return ctx;
}

// (internal: stream_io.hip's private contexts)
int capnp_ctx_device(const capnp_ctx* ctx) { return ctx ? ctx->device : 0; }

void capnp_ctx_destroy(capnp_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)wait_uses(ctx);  // (an index-free decode may still be running on its caller's stream)
    {
        std::lock_guard<std::mutex> g(g_svc_mu);
        if (g_svc_ctxs)
            g_svc_ctxs->erase(std::remove(g_svc_ctxs->begin(), g_svc_ctxs->end(), ctx),
                              g_svc_ctxs->end());
    }
    for (CallSvc& v : ctx->svc) {
        if (v.s) (void)hipStreamDestroy(v.s);
        if (v.h) (void)hipHostFree(v.h);
        if (v.line_dev) (void)hipFree(v.line);
    }
    if (ctx->d_state) (void)hipFree(ctx->d_state);
    if (ctx->d_stage) (void)hipFree(ctx->d_stage);
    if (ctx->d_body) (void)hipFree(ctx->d_body);
    if (ctx->d_frame) (void)hipFree(ctx->d_frame);
    if (ctx->h_frame) (void)hipHostFree(ctx->h_frame);
    if (ctx->d_bad) (void)hipFree(ctx->d_bad);
    if (ctx->h_bad) (void)hipHostFree(ctx->h_bad);
    if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
    if (ctx->d_req) (void)hipFree(ctx->d_req);
    if (ctx->h_flag) (void)hipHostFree(ctx->h_flag);
    if (ctx->d_msg) (void)hipFree(ctx->d_msg);
    if (ctx->d_resync) (void)hipFree(ctx->d_resync);
    if (ctx->d_wt) (void)hipFree(ctx->d_wt);
    if (ctx->d_pwt) (void)hipFree(ctx->d_pwt);
    if (ctx->ev_resync) (void)hipEventDestroy(ctx->ev_resync);
    for (int k = 0; k < capnp_ctx::kUseSlots; k++)
        if (ctx->use_ev[k]) (void)hipEventDestroy(ctx->use_ev[k]);
    for (int k = 0; k < 3; k++)
        if (ctx->sstream[k]) {
            (void)hipStreamSynchronize(ctx->sstream[k]);
            (void)hipStreamDestroy(ctx->sstream[k]);
        }
    for (int k = 0; k < 2; k++) {
        if (ctx->ev_in[k]) (void)hipEventDestroy(ctx->ev_in[k]);
        if (ctx->ev_comp[k]) (void)hipEventDestroy(ctx->ev_comp[k]);
        if (ctx->ev_off[k]) (void)hipEventDestroy(ctx->ev_off[k]);
        if (ctx->ev_out[k]) (void)hipEventDestroy(ctx->ev_out[k]);
        if (ctx->d_slot[k]) (void)hipFree(ctx->d_slot[k]);
        if (ctx->h_slot_off[k]) (void)hipHostFree(ctx->h_slot_off[k]);
    }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

void* capnp_ctx_stream(capnp_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

const char* capnp_ctx_last_error(capnp_ctx* ctx) { return ctx ? ctx->err.c_str() : ""; }

capnp_status capnp_ctx_reserve(capnp_ctx* ctx, size_t max_chunks) {
    if (!ctx) return CAPNP_E_INVALID_ARGUMENT;
    return ensure_state(ctx, state_bytes_for(max_chunks, 1));
}

capnp_status capnp_gpu_pack_batch(capnp_ctx* ctx, const uint64_t* d_words,
                                  const uint64_t* d_chunk_word_off, size_t nchunks,
                                  uint8_t* d_out, size_t out_cap, uint64_t* d_out_byte_off,
                                  void* stream) {
    if (!ctx) return CAPNP_E_INVALID_ARGUMENT;
    return pack_batch_dev(ctx, d_words, d_chunk_word_off, nchunks, d_out, out_cap,
                          d_out_byte_off, 0, pick(ctx, stream));
}

capnp_status capnp_gpu_pack_batch_tuned(capnp_ctx* ctx, const uint64_t* d_words,
                                        const uint64_t* d_chunk_word_off, size_t nchunks,
                                        uint8_t* d_out, size_t out_cap,
                                        uint64_t* d_out_byte_off, uint32_t chunks_per_tile,
                                        void* stream) {
    if (!ctx) return CAPNP_E_INVALID_ARGUMENT;
    return pack_batch_dev(ctx, d_words, d_chunk_word_off, nchunks, d_out, out_cap,
                          d_out_byte_off, chunks_per_tile, pick(ctx, stream));
}

// With the record sync index and chunks_per_tile == 0 the launch is sized
// from the batch's word range (one synchronisation to read it): batches whose
// mean chunk is at least kWordTileMean words decode in word tiles
// (capnp_launch_unpack_wt: chunks of any length, cut at sync points), others
// in chunk tiles of about capnp_unpack_tile_words() words.

static capnp_status unpack_resync_dev(capnp_ctx* ctx, const uint8_t* d_packed,
                                      const uint64_t* d_in_byte_off, size_t nchunks,
                                      uint64_t* d_words, const uint64_t* d_out_word_off,
                                      int32_t* d_status, uint64_t* d_consumed, hipStream_t s,
                                      const uint64_t* checked_byte_ends = nullptr);

static capnp_status unpack_batch_dev(capnp_ctx* ctx, const uint8_t* d_packed,
                                     const uint64_t* d_in_byte_off, size_t nchunks,
                                     uint64_t* d_words, const uint64_t* d_out_word_off,
                                     int32_t* d_status, uint64_t* d_consumed, uint32_t tc,
                                     void* stream, const uint32_t* d_sync = nullptr) {
    if (!ctx || (nchunks && (!d_in_byte_off || !d_out_word_off || !d_status)))
        return CAPNP_E_INVALID_ARGUMENT;
    if (tc > 256) return CAPNP_E_INVALID_ARGUMENT;
    UseMark um{ctx, pick(ctx, stream)};
    if (tc == 0 && nchunks) {
        hipStream_t s = pick(ctx, stream);
        uint64_t wr[2], br[2];
        capnp_status vst = check_offsets(
            ctx, s, {{d_in_byte_off, nchunks, ~0ull}, {d_out_word_off, nchunks, ~0ull}});
        if (vst != CAPNP_OK) return vst;
        br[0] = checked_ends(ctx, 0)[0];
        br[1] = checked_ends(ctx, 0)[1];
        wr[0] = checked_ends(ctx, 1)[0];
        wr[1] = checked_ends(ctx, 1)[1];
        if (wr[1] < wr[0]) return CAPNP_E_INVALID_ARGUMENT;
        const uint64_t words = wr[1] - wr[0];
        const bool longc = words && (words / nchunks >= kWordTileMean || force_word_tiles());
        const uint64_t mean = words / nchunks;
        if (longc && !d_sync && !force_word_tiles() && nchunks >= kLongUnitsMin &&
            mean >= kLongUnitWords && mean < kBlockDecodeWords) {
            // no index, enough units of a few thousand words each to fill the
            // chip: one workgroup per unit (the long-unit decode, unpack.hip
            // unpack_long) beats resolving blocks (scripts/long_unit_bench.py:
            // 256 x 8192 words 67 vs 152 us, 2300 x 8192 178 vs 292,
            // profiles/r06b_long_unit_auto.txt)
            tc = 1;
        } else if (longc && !d_sync) {
            // no index, few units or mixed sizes: the speculative block walk
            // spreads every unit over the chip (resync.hip; 2 x 1 Mi words 211 us
            // against 4.4 ms on two workgroups, config 4 1.65 ms against
            // 2.14-2.47 in chunk tiles, profiles/r06d_route_probe.txt); both offset
            // arrays were checked just above
            return unpack_resync_dev(ctx, d_packed, d_in_byte_off, nchunks, d_words,
                                     d_out_word_off, d_status, d_consumed, s, br);
        }
        if (longc && d_sync) {
            const size_t ws = capnp_unpack_wt_ws_bytes(wr[0], wr[1]);
            capnp_status st = ensure_buf(ctx, &ctx->d_wt, &ctx->wt_cap, ws);
            if (st != CAPNP_OK) return st;
            HIP_TRY(capnp_launch_unpack_wt(d_packed, d_in_byte_off, nchunks, d_words,
                                           d_out_word_off, d_status, d_consumed, d_sync, wr[0],
                                           wr[1], ctx->d_wt, ctx->wt_cap, s));
            return CAPNP_OK;
        }
        if (tc == 0) {
            const uint64_t m = mean ? mean : 1;
            const uint64_t t = capnp_unpack_tile_words() / m;
            tc = (uint32_t)(t < 1 ? 1 : (t > 64 ? 64 : t));
        }
    }
    HIP_TRY(capnp_launch_unpack(d_packed, d_in_byte_off, nchunks, tc, d_words, d_out_word_off,
                                d_status, d_consumed, d_sync, pick(ctx, stream)));
    return CAPNP_OK;
}

capnp_status capnp_gpu_unpack_batch(capnp_ctx* ctx, const uint8_t* d_packed,
                                    const uint64_t* d_in_byte_off, size_t nchunks,
                                    uint64_t* d_words, const uint64_t* d_out_word_off,
                                    int32_t* d_status, uint64_t* d_consumed, void* stream) {
    return unpack_batch_dev(ctx, d_packed, d_in_byte_off, nchunks, d_words, d_out_word_off,
                            d_status, d_consumed, 0, stream);
}

capnp_status capnp_gpu_unpack_batch_tuned(capnp_ctx* ctx, const uint8_t* d_packed,
                                          const uint64_t* d_in_byte_off, size_t nchunks,
                                          uint64_t* d_words, const uint64_t* d_out_word_off,
                                          int32_t* d_status, uint64_t* d_consumed,
                                          uint32_t chunks_per_tile, void* stream) {
    return unpack_batch_dev(ctx, d_packed, d_in_byte_off, nchunks, d_words, d_out_word_off,
                            d_status, d_consumed, chunks_per_tile, stream);
}

size_t capnp_sync_index_entries(size_t total_words) {
    return (total_words + CAPNP_SYNC_WORDS - 1) / CAPNP_SYNC_WORDS;
}

capnp_status capnp_gpu_pack_batch_sync(capnp_ctx* ctx, const uint64_t* d_words,
                                       const uint64_t* d_chunk_word_off, size_t nchunks,
                                       uint8_t* d_out, size_t out_cap, uint64_t* d_out_byte_off,
                                       uint32_t* d_sync, void* stream) {
    if (!ctx || !d_sync) return CAPNP_E_INVALID_ARGUMENT;
    return pack_batch_dev(ctx, d_words, d_chunk_word_off, nchunks, d_out, out_cap,
                          d_out_byte_off, 0, pick(ctx, stream), d_sync);
}

capnp_status capnp_gpu_unpack_batch_sync(capnp_ctx* ctx, const uint8_t* d_packed,
                                         const uint64_t* d_in_byte_off, size_t nchunks,
                                         uint64_t* d_words, const uint64_t* d_out_word_off,
                                         const uint32_t* d_sync, int32_t* d_status,
                                         uint64_t* d_consumed, void* stream) {
    if (!d_sync) return CAPNP_E_INVALID_ARGUMENT;
    return unpack_batch_dev(ctx, d_packed, d_in_byte_off, nchunks, d_words, d_out_word_off,
                            d_status, d_consumed, 0, stream, d_sync);
}

capnp_status capnp_gpu_pack_batch_sync_tuned(capnp_ctx* ctx, const uint64_t* d_words,
                                             const uint64_t* d_chunk_word_off, size_t nchunks,
                                             uint8_t* d_out, size_t out_cap,
                                             uint64_t* d_out_byte_off, uint32_t* d_sync,
                                             uint32_t chunks_per_tile, void* stream) {
    if (!ctx || !d_sync) return CAPNP_E_INVALID_ARGUMENT;
    return pack_batch_dev(ctx, d_words, d_chunk_word_off, nchunks, d_out, out_cap,
                          d_out_byte_off, chunks_per_tile, pick(ctx, stream), d_sync);
}

capnp_status capnp_gpu_unpack_batch_sync_tuned(capnp_ctx* ctx, const uint8_t* d_packed,
                                               const uint64_t* d_in_byte_off, size_t nchunks,
                                               uint64_t* d_words, const uint64_t* d_out_word_off,
                                               const uint32_t* d_sync, int32_t* d_status,
                                               uint64_t* d_consumed, uint32_t chunks_per_tile,
                                               void* stream) {
    if (!d_sync) return CAPNP_E_INVALID_ARGUMENT;
    return unpack_batch_dev(ctx, d_packed, d_in_byte_off, nchunks, d_words, d_out_word_off,
                            d_status, d_consumed, chunks_per_tile, stream, d_sync);
}

capnp_status capnp_gpu_unpack_batch_resync(capnp_ctx* ctx, const uint8_t* d_packed,
                                           const uint64_t* d_in_byte_off, size_t nchunks,
                                           uint64_t* d_words, const uint64_t* d_out_word_off,
                                           int32_t* d_status, uint64_t* d_consumed,
                                           void* stream) {
    if (!ctx || (nchunks && (!d_in_byte_off || !d_out_word_off || !d_status)))
        return CAPNP_E_INVALID_ARGUMENT;
    return unpack_resync_dev(ctx, d_packed, d_in_byte_off, nchunks, d_words, d_out_word_off,
                             d_status, d_consumed, pick(ctx, stream));
}

// checked_byte_ends: the caller has just checked both offset arrays (and read
// d_in_byte_off's first and last entries, given here); otherwise this call
// checks them.
static capnp_status unpack_resync_dev(capnp_ctx* ctx, const uint8_t* d_packed,
                                      const uint64_t* d_in_byte_off, size_t nchunks,
                                      uint64_t* d_words, const uint64_t* d_out_word_off,
                                      int32_t* d_status, uint64_t* d_consumed, hipStream_t s,
                                      const uint64_t* checked_byte_ends) {
    UseMark um{ctx, s};
    // The previous index-free decode returned with its kernels still queued on
    // its own stream, and they read and write the workspace this call is about
    // to reset: a call on another stream waits for them first (an event, no
    // host synchronisation); on the same stream, stream order already does.
    if (ctx->resync_failed && ctx->resync_stream != s) {
        if (!ctx->ev_resync)
            HIP_TRY(hipEventCreateWithFlags(&ctx->ev_resync, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ctx->ev_resync, ctx->resync_stream));
        HIP_TRY(hipStreamWaitEvent(s, ctx->ev_resync, 0));
    }
    ctx->resync_failed = nullptr;  // (a new call: the previous call's flag is moot)
    ctx->resync_passes = ctx->resync_serial = 0;
    if (nchunks == 0) return CAPNP_OK;
    uint64_t ends[2];
    if (checked_byte_ends) {
        ends[0] = checked_byte_ends[0];
        ends[1] = checked_byte_ends[1];
    } else {
        capnp_status vst = check_offsets(
            ctx, s, {{d_in_byte_off, nchunks, ~0ull}, {d_out_word_off, nchunks, ~0ull}});
        if (vst != CAPNP_OK) return vst;
        ends[0] = checked_ends(ctx, 0)[0];
        ends[1] = checked_ends(ctx, 0)[1];
    }
    if (ends[1] < ends[0]) return CAPNP_E_INVALID_ARGUMENT;
    const size_t ws = capnp_resync_ws_bytes(nchunks, ends[1] - ends[0]);
    capnp_status st = ensure_buf(ctx, &ctx->d_resync, &ctx->resync_cap, ws);
    if (st != CAPNP_OK) return st;
    HIP_TRY(capnp_resync_unpack(d_packed, d_in_byte_off, nchunks, ends[1] - ends[0], d_words,
                                d_out_word_off, d_status, d_consumed, ctx->d_resync,
                                ctx->resync_cap, s, &ctx->resync_passes, &ctx->resync_serial,
                                &ctx->resync_failed));
    ctx->resync_stream = s;
    return CAPNP_OK;
}

capnp_status capnp_resync_stats(capnp_ctx* ctx, int* passes, int* serial) {
    if (!ctx) return CAPNP_E_INVALID_ARGUMENT;
    const capnp_status st = settle_resync(ctx);  // (the decode did not wait for its flag)
    if (st != CAPNP_OK) return st;
    if (passes) *passes = ctx->resync_passes;
    if (serial) *serial = ctx->resync_serial;
    return CAPNP_OK;
}

capnp_status capnp_gpu_gen_batch(capnp_ctx* ctx, uint64_t* d_words, const uint64_t* d_offs,
                                 size_t nchunks, uint64_t id0, const uint8_t* d_kinds,
                                 uint32_t kind0, uint32_t pz_thresh, void* stream) {
    if (!ctx) return CAPNP_E_INVALID_ARGUMENT;
    HIP_TRY(capnp_launch_gen(d_words, d_offs, nchunks, id0, d_kinds, kind0, pz_thresh,
                             pick(ctx, stream)));
    return CAPNP_OK;
}

capnp_status capnp_gpu_gen_carsales(capnp_ctx* ctx, uint64_t* d_words, uint64_t total_words,
                                    uint64_t skip_requests, uint64_t* h_req_off,
                                    size_t max_req, size_t* nreq, void* stream) {
    if (!ctx || (total_words && !d_words)) return CAPNP_E_INVALID_ARGUMENT;
    // a request has at least 3 words: this many requests always cover it
    const uint64_t cap = std::min<uint64_t>(total_words / 3 + 2, max_req ? max_req : ~0ull);
    std::vector<uint32_t> states(4 * cap);
    std::vector<uint64_t> off(cap + 1);
    static const uint32_t seed[4] = {0x1d2acd47u, 0x58ca3e14u, 0xf563f232u, 0x0bc76199u};
    const uint64_t m = capnp_carsales_plan(seed, skip_requests, total_words, states.data(),
                                           off.data(), cap);
    if (nreq) *nreq = m;
    if (h_req_off) memcpy(h_req_off, off.data(), (m + 1) * 8);
    if (m == 0) return CAPNP_OK;
    const size_t o_off = round16(m * 16);
    capnp_status st = ensure_stage(ctx, o_off + (m + 1) * 8);
    if (st != CAPNP_OK) return st;
    hipStream_t s = pick(ctx, stream);
    HIP_TRY(hipMemcpyAsync(ctx->d_stage, states.data(), m * 16, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(ctx->d_stage + o_off, off.data(), (m + 1) * 8, hipMemcpyHostToDevice,
                           s));
    HIP_TRY(capnp_launch_gen_carsales(d_words, total_words,
                                      reinterpret_cast<uint32_t*>(ctx->d_stage),
                                      reinterpret_cast<uint64_t*>(ctx->d_stage + o_off), m, s));
    HIP_TRY(hipStreamSynchronize(s));  // the staging buffer is reused by later calls
    return CAPNP_OK;
}

capnp_status capnp_pack(capnp_ctx* ctx, const uint8_t* in, size_t len, uint8_t* out,
                        size_t cap, size_t* written) {
    if (!ctx || !written || (len && !in)) return CAPNP_E_INVALID_ARGUMENT;
    if (len % 8 != 0) return CAPNP_E_MISALIGNED_LEN;
    *written = 0;
    std::vector<uint64_t> words(len / 8);
    if (len) memcpy(words.data(), in, len);
    uint64_t off[2] = {0, len / 8};
    uint64_t total = 0;
    capnp_status st = pack_host(ctx, words.data(), off, 1, out, cap, nullptr, &total);
    *written = std::min<uint64_t>(total, cap);
    return st;
}

capnp_status capnp_pack_batch_host(capnp_ctx* ctx, const uint64_t* words,
                                   const uint64_t* chunk_word_off, size_t nchunks, uint8_t* out,
                                   size_t out_cap, uint64_t* out_byte_off) {
    if (!ctx || !chunk_word_off || !out_byte_off) return CAPNP_E_INVALID_ARGUMENT;
    uint64_t total = 0;
    return pack_host(ctx, words, chunk_word_off, nchunks, out, out_cap, out_byte_off, &total);
}

capnp_status capnp_unpack_batch_host(capnp_ctx* ctx, const uint8_t* packed,
                                     const uint64_t* in_byte_off, size_t nchunks,
                                     uint64_t* words, const uint64_t* out_word_off,
                                     int32_t* status, uint64_t* consumed) {
    if (!ctx || !in_byte_off || !out_word_off || !status) return CAPNP_E_INVALID_ARGUMENT;
    const size_t n = nchunks;
    const uint64_t ib = n ? in_byte_off[0] : 0, ie = n ? in_byte_off[n] : 0;
    const uint64_t ob = n ? out_word_off[0] : 0, oe = n ? out_word_off[n] : 0;
    std::vector<uint64_t> ri(n + 1), ro(n + 1);
    for (size_t i = 0; i <= n; i++) {
        ri[i] = n ? in_byte_off[i] - ib : 0;
        ro[i] = n ? out_word_off[i] - ob : 0;
    }
    const size_t o_in = 0;
    const size_t o_ri = round16(ie - ib + 16);
    const size_t o_ro = o_ri + round16((n + 1) * 8);
    const size_t o_st = o_ro + round16((n + 1) * 8);
    const size_t o_cs = o_st + round16(n * 4);
    const size_t o_out = o_cs + round16(n * 8);
    capnp_status st = ensure_stage(ctx, o_out + (oe - ob) * 8 + 16);
    if (st != CAPNP_OK) return st;
    uint8_t* d = ctx->d_stage;
    hipStream_t s = ctx->stream;
    if (ie > ib) HIP_TRY(hipMemcpyAsync(d + o_in, packed + ib, ie - ib, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d + o_ri, ri.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d + o_ro, ro.data(), (n + 1) * 8, hipMemcpyHostToDevice, s));
    // the device batch's own plan: long chunks (a stream reader's 1 MiB unit)
    // take the speculative block walk rather than one wave's serial walk
    if (n) {
        st = unpack_batch_dev(ctx, d + o_in, reinterpret_cast<uint64_t*>(d + o_ri), n,
                              reinterpret_cast<uint64_t*>(d + o_out),
                              reinterpret_cast<uint64_t*>(d + o_ro),
                              reinterpret_cast<int32_t*>(d + o_st),
                              reinterpret_cast<uint64_t*>(d + o_cs), 0, s);
        if (st != CAPNP_OK) return st;
    }
    if (oe > ob) HIP_TRY(hipMemcpyAsync(words + ob, d + o_out, (oe - ob) * 8, hipMemcpyDeviceToHost, s));
    if (n) HIP_TRY(hipMemcpyAsync(status, d + o_st, n * 4, hipMemcpyDeviceToHost, s));
    if (n && consumed) HIP_TRY(hipMemcpyAsync(consumed, d + o_cs, n * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return CAPNP_OK;
}

capnp_status capnp_unpack(capnp_ctx* ctx, const uint8_t* in, size_t in_len, size_t* consumed,
                          uint8_t* out, size_t out_len) {
    if (!ctx || !consumed || (in_len && !in) || (out_len && !out)) return CAPNP_E_INVALID_ARGUMENT;
    *consumed = 0;
    if (out_len == 0) return CAPNP_OK;                  // serialize_packed.rs:82-84
    if (out_len % 8 != 0) return CAPNP_E_MISALIGNED_LEN;  // :86 (panic)
    uint64_t io[2] = {0, in_len}, oo[2] = {0, out_len / 8};
    int32_t status = 0;
    uint64_t used = 0;
    std::vector<uint64_t> words(out_len / 8);
    capnp_status st = capnp_unpack_batch_host(ctx, in, io, 1, words.data(), oo, &status, &used);
    if (st != CAPNP_OK) return st;
    *consumed = used;
    if (status == CAPNP_OK) memcpy(out, words.data(), out_len);
    return (capnp_status)status;
}

// Streaming pack: slice i+1's copy in, slice i's kernel and slice i-1's copy
// out overlap.  The slots hold a slice's words, its (absolute) chunk offsets,
// its packed offsets and its packed bytes; the kernel sees the words through
// a pointer biased by the slice's first word, so the caller's offsets go
// over unchanged.  The host waits once per slice, for the slice's packed
// size (to place its bytes), while the next slice is already queued.
capnp_status capnp_stream_pack_batch(capnp_ctx* ctx, const uint64_t* words,
                                     const uint64_t* chunk_word_off, size_t nchunks,
                                     uint8_t* out, size_t out_cap, uint64_t* out_byte_off,
                                     size_t slice_words) {
    if (!ctx || !chunk_word_off || !out_byte_off || (out_cap && !out))
        return CAPNP_E_INVALID_ARGUMENT;
    const size_t n = nchunks;
    if (n == 0) {
        out_byte_off[0] = 0;
        return CAPNP_OK;
    }
    if (!words) return CAPNP_E_INVALID_ARGUMENT;
    for (size_t c = 0; c < n; c++)
        if (chunk_word_off[c + 1] < chunk_word_off[c]) return CAPNP_E_INVALID_ARGUMENT;
    const std::vector<size_t> sl = make_slices(chunk_word_off, n, slice_words ? slice_words
                                                                              : kDefaultSliceWords);
    const size_t ns = sl.size() - 1;
    size_t max_w = 0, max_n = 0, max_bound = 0;
    for (size_t i = 0; i < ns; i++) {
        const size_t w = chunk_word_off[sl[i + 1]] - chunk_word_off[sl[i]];
        const size_t c = sl[i + 1] - sl[i];
        max_w = std::max(max_w, w);
        max_n = std::max(max_n, c);
        max_bound = std::max(max_bound, capnp_packed_batch_bound_bytes(w, c));
    }
    const uint32_t tc = tile_chunks_for(chunk_word_off[n] - chunk_word_off[0], n);
    const size_t o_off = round16(max_w * 8 + kSlotPad);
    const size_t o_oo = o_off + round16((max_n + 1) * 8);
    const size_t o_out = o_oo + round16((max_n + 1) * 8);
    capnp_status st = stream_setup(ctx, o_out + max_bound + kSlotPad, max_n + 1);
    if (st != CAPNP_OK) return st;
    st = ensure_state(ctx, state_bytes_for(max_n, tc));
    if (st != CAPNP_OK) return st;
    hipStream_t s_in = ctx->sstream[0], s_comp = ctx->sstream[1], s_out = ctx->sstream[2];
    uint64_t base = 0;
    capnp_status result = CAPNP_OK;
    // places slice j's bytes once its packed size is known
    auto finalize = [&](size_t j) -> capnp_status {
        const int k = (int)(j & 1);
        const size_t c0 = sl[j], nj = sl[j + 1] - sl[j];
        HIP_TRY(hipEventSynchronize(ctx->ev_off[k]));
        const uint64_t* ho = ctx->h_slot_off[k];
        for (size_t c = 0; c < nj; c++) out_byte_off[c0 + c] = base + ho[c];
        const uint64_t total = ho[nj];
        const uint64_t ncopy = base >= out_cap ? 0 : std::min<uint64_t>(total, out_cap - base);
        if (ncopy)
            HIP_TRY(hipMemcpyAsync(out + base, ctx->d_slot[k] + o_out, ncopy,
                                   hipMemcpyDeviceToHost, s_out));
        HIP_TRY(hipEventRecord(ctx->ev_out[k], s_out));
        base += total;
        return CAPNP_OK;
    };
    for (size_t i = 0; i < ns; i++) {
        const int k = (int)(i & 1);
        const size_t c0 = sl[i], ni = sl[i + 1] - sl[i];
        const uint64_t w0 = chunk_word_off[c0], wi = chunk_word_off[sl[i + 1]] - w0;
        uint8_t* d = ctx->d_slot[k];
        if (i >= 2) HIP_TRY(hipStreamWaitEvent(s_in, ctx->ev_out[k], 0));
        if (wi)
            HIP_TRY(hipMemcpyAsync(d, words + w0, wi * 8, hipMemcpyHostToDevice, s_in));
        HIP_TRY(hipMemcpyAsync(d + o_off, chunk_word_off + c0, (ni + 1) * 8,
                               hipMemcpyHostToDevice, s_in));
        HIP_TRY(hipEventRecord(ctx->ev_in[k], s_in));
        HIP_TRY(hipStreamWaitEvent(s_comp, ctx->ev_in[k], 0));
        st = pack_batch_dev(ctx, reinterpret_cast<const uint64_t*>(d) - w0,
                            reinterpret_cast<const uint64_t*>(d + o_off), ni, d + o_out,
                            capnp_packed_batch_bound_bytes(wi, ni),
                            reinterpret_cast<uint64_t*>(d + o_oo), tc, s_comp);
        if (st != CAPNP_OK) return st;
        HIP_TRY(hipEventRecord(ctx->ev_comp[k], s_comp));
        if (i >= 1) {
            st = finalize(i - 1);
            if (st != CAPNP_OK) return st;
        }
        HIP_TRY(hipStreamWaitEvent(s_out, ctx->ev_comp[k], 0));
        HIP_TRY(hipMemcpyAsync(ctx->h_slot_off[k], d + o_oo, (ni + 1) * 8,
                               hipMemcpyDeviceToHost, s_out));
        HIP_TRY(hipEventRecord(ctx->ev_off[k], s_out));
    }
    st = finalize(ns - 1);
    if (st != CAPNP_OK) return st;
    HIP_TRY(hipStreamSynchronize(s_out));
    out_byte_off[n] = base;
    if (base > out_cap) result = CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;
    return result;
}

// Streaming unpack: every slice's sizes are known from the offsets, so the
// three streams run without any host wait until the end.
capnp_status capnp_stream_unpack_batch(capnp_ctx* ctx, const uint8_t* packed,
                                       const uint64_t* in_byte_off, size_t nchunks,
                                       uint64_t* words, const uint64_t* out_word_off,
                                       int32_t* status, uint64_t* consumed, size_t slice_words) {
    if (!ctx || !in_byte_off || !out_word_off || !status) return CAPNP_E_INVALID_ARGUMENT;
    const size_t n = nchunks;
    if (n == 0) return CAPNP_OK;
    for (size_t c = 0; c < n; c++)
        if (in_byte_off[c + 1] < in_byte_off[c] || out_word_off[c + 1] < out_word_off[c])
            return CAPNP_E_INVALID_ARGUMENT;
    if ((in_byte_off[n] > in_byte_off[0] && !packed) ||
        (out_word_off[n] > out_word_off[0] && !words))
        return CAPNP_E_INVALID_ARGUMENT;
    const std::vector<size_t> sl = make_slices(out_word_off, n, slice_words ? slice_words
                                                                            : kDefaultSliceWords);
    const size_t ns = sl.size() - 1;
    size_t max_w = 0, max_n = 0, max_b = 0;
    for (size_t i = 0; i < ns; i++) {
        max_w = std::max<size_t>(max_w, out_word_off[sl[i + 1]] - out_word_off[sl[i]]);
        max_b = std::max<size_t>(max_b, in_byte_off[sl[i + 1]] - in_byte_off[sl[i]]);
        max_n = std::max(max_n, sl[i + 1] - sl[i]);
    }
    const uint64_t tw = out_word_off[n] - out_word_off[0];
    const double mean = std::max((double)tw / (double)n, 1.0);
    const uint32_t utc = (uint32_t)std::max(1.0, std::min((double)capnp_unpack_tile_words() /
                                                              mean, 64.0));
    const size_t o_in = kSlotPad;
    const size_t o_io = o_in + round16(max_b + kSlotPad);
    const size_t o_oo = o_io + round16((max_n + 1) * 8);
    const size_t o_st = o_oo + round16((max_n + 1) * 8);
    const size_t o_cs = o_st + round16(max_n * 4);
    const size_t o_out = o_cs + round16(max_n * 8);
    capnp_status st = stream_setup(ctx, o_out + max_w * 8 + kSlotPad, 1);
    if (st != CAPNP_OK) return st;
    hipStream_t s_in = ctx->sstream[0], s_comp = ctx->sstream[1], s_out = ctx->sstream[2];
    for (size_t i = 0; i < ns; i++) {
        const int k = (int)(i & 1);
        const size_t c0 = sl[i], ni = sl[i + 1] - sl[i];
        const uint64_t b0 = in_byte_off[c0], bi = in_byte_off[sl[i + 1]] - b0;
        const uint64_t w0 = out_word_off[c0], wi = out_word_off[sl[i + 1]] - w0;
        uint8_t* d = ctx->d_slot[k];
        if (i >= 2) HIP_TRY(hipStreamWaitEvent(s_in, ctx->ev_out[k], 0));
        if (bi) HIP_TRY(hipMemcpyAsync(d + o_in, packed + b0, bi, hipMemcpyHostToDevice, s_in));
        HIP_TRY(hipMemcpyAsync(d + o_io, in_byte_off + c0, (ni + 1) * 8, hipMemcpyHostToDevice,
                               s_in));
        HIP_TRY(hipMemcpyAsync(d + o_oo, out_word_off + c0, (ni + 1) * 8,
                               hipMemcpyHostToDevice, s_in));
        HIP_TRY(hipEventRecord(ctx->ev_in[k], s_in));
        HIP_TRY(hipStreamWaitEvent(s_comp, ctx->ev_in[k], 0));
        HIP_TRY(capnp_launch_unpack(d + o_in - b0, reinterpret_cast<const uint64_t*>(d + o_io),
                                    ni, utc, reinterpret_cast<uint64_t*>(d + o_out) - w0,
                                    reinterpret_cast<const uint64_t*>(d + o_oo),
                                    reinterpret_cast<int32_t*>(d + o_st),
                                    reinterpret_cast<uint64_t*>(d + o_cs), nullptr, s_comp));
        HIP_TRY(hipEventRecord(ctx->ev_comp[k], s_comp));
        HIP_TRY(hipStreamWaitEvent(s_out, ctx->ev_comp[k], 0));
        if (wi)
            HIP_TRY(hipMemcpyAsync(words + w0, d + o_out, wi * 8, hipMemcpyDeviceToHost, s_out));
        HIP_TRY(hipMemcpyAsync(status + c0, d + o_st, ni * 4, hipMemcpyDeviceToHost, s_out));
        if (consumed)
            HIP_TRY(hipMemcpyAsync(consumed + c0, d + o_cs, ni * 8, hipMemcpyDeviceToHost,
                                   s_out));
        HIP_TRY(hipEventRecord(ctx->ev_out[k], s_out));
    }
    HIP_TRY(hipStreamSynchronize(s_out));
    return CAPNP_OK;
}

// Batch write_message on the device (msgbatch.hip): layout, scans and
// assembly into a staging array, one stream synchronisation for the totals,
// then the batch pack of the chunks and the message offsets.
capnp_status capnp_gpu_write_messages(capnp_ctx* ctx, const uint64_t* d_words,
                                      const uint64_t* d_seg_word_off,
                                      const uint64_t* d_msg_seg_off, size_t nmsg,
                                      size_t total_segs, size_t total_words, uint8_t* d_out,
                                      size_t out_cap, uint64_t* d_msg_byte_off, void* stream) {
    if (!ctx || !d_msg_byte_off || (nmsg && (!d_seg_word_off || !d_msg_seg_off)))
        return CAPNP_E_INVALID_ARGUMENT;
    hipStream_t s = pick(ctx, stream);
    UseMark um{ctx, s};
    if (nmsg == 0) {
        HIP_TRY(hipMemsetAsync(d_msg_byte_off, 0, sizeof(uint64_t), s));
        return CAPNP_OK;
    }
    if (total_segs < nmsg || (total_words && !d_words)) return CAPNP_E_INVALID_ARGUMENT;
    {
        // message m's segments [msg_seg_off[m], msg_seg_off[m+1]) within
        // [0, total_segs]; segment offsets non-decreasing and within the
        // total_words words of d_words (both paths read the segments at these
        // offsets before anything else would notice)
        capnp_status vst = check_offsets(ctx, s,
                                         {{d_msg_seg_off, nmsg, (uint64_t)total_segs},
                                          {d_seg_word_off, total_segs, (uint64_t)total_words}});
        if (vst != CAPNP_OK) return vst;
    }
    // Gap path: the segments are packed in place as the chunks, each
    // message's first chunk preceded by a gap of its packed table's size, and
    // the tables are written into the gaps afterwards.  Messages without
    // segments (or offsets that do not span the batch) take the staging path.
    {
        const size_t g_gap = 0;
        const size_t g_cboff = g_gap + round16(total_segs * 4);
        const size_t g_flag = g_cboff + round16((total_segs + 1) * 8);
        capnp_status st = ensure_buf(ctx, &ctx->d_msg, &ctx->msg_cap, g_flag + 64);
        if (st != CAPNP_OK) return st;
        uint8_t* d = ctx->d_msg;
        uint32_t* gap = reinterpret_cast<uint32_t*>(d + g_gap);
        uint64_t* cboff = reinterpret_cast<uint64_t*>(d + g_cboff);
        uint32_t* flag = reinterpret_cast<uint32_t*>(d + g_flag);
        HIP_TRY(capnp_launch_msg_gap(d_seg_word_off, d_msg_seg_off, nmsg, total_segs, gap, flag,
                                     s));
        uint32_t h_flag = 1;
        HIP_TRY(hipMemcpyAsync(&h_flag, flag, 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (h_flag == 0) {
            const uint32_t tc = tile_chunks_for(total_words, total_segs);
            st = ensure_state(ctx, state_bytes_for(total_segs, tc));
            if (st != CAPNP_OK) return st;
            HIP_TRY(capnp_launch_pack_gap(d_words, d_seg_word_off, total_segs, tc, d_out, out_cap,
                                          cboff, reinterpret_cast<uint64_t*>(ctx->d_state), gap,
                                          s));
            HIP_TRY(capnp_launch_msg_tables(d_seg_word_off, d_msg_seg_off, nmsg, cboff, d_out,
                                            out_cap, d_msg_byte_off, s));
            return CAPNP_OK;
        }
    }
    // bounds: table words <= nmsg + total_segs / 2 + nmsg, chunks <= 2 nmsg + total_segs
    const size_t max_words = total_words + 2 * nmsg + total_segs / 2 + 1;
    const size_t max_chunks = 2 * nmsg + total_segs;
    size_t scan_bytes = 0;
    HIP_TRY(capnp_msg_scan_bytes(nmsg + 1, &scan_bytes));
    const size_t o_cw = 0;
    const size_t o_cc = o_cw + round16((nmsg + 1) * 8);
    const size_t o_wofs = o_cc + round16((nmsg + 1) * 8);
    const size_t o_cofs = o_wofs + round16((nmsg + 1) * 8);
    const size_t o_tmp = o_cofs + round16((nmsg + 1) * 8);
    const size_t o_coff = o_tmp + round16(scan_bytes + 16);
    const size_t o_cboff = o_coff + round16((max_chunks + 1) * 8);
    const size_t o_stage = o_cboff + round16((max_chunks + 1) * 8);
    capnp_status st = ensure_buf(ctx, &ctx->d_msg, &ctx->msg_cap, o_stage + max_words * 8 + 64);
    if (st != CAPNP_OK) return st;
    uint8_t* d = ctx->d_msg;
    auto U = [&](size_t o) { return reinterpret_cast<uint64_t*>(d + o); };
    HIP_TRY(capnp_launch_msg_prepare(d_words, d_seg_word_off, d_msg_seg_off, nmsg, U(o_cw),
                                     U(o_cc), U(o_wofs), U(o_cofs), d + o_tmp, scan_bytes,
                                     U(o_stage), U(o_coff), s));
    uint64_t tot[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&tot[0], U(o_wofs) + nmsg, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&tot[1], U(o_cofs) + nmsg, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (tot[0] > max_words || tot[1] > max_chunks) return CAPNP_E_INVALID_ARGUMENT;
    st = pack_batch_dev(ctx, U(o_stage), U(o_coff), tot[1], d_out, out_cap, U(o_cboff),
                        tile_chunks_for(tot[0], tot[1]), s);
    if (st != CAPNP_OK) return st;
    HIP_TRY(capnp_launch_msg_offsets(U(o_cofs), U(o_cboff), nmsg, d_msg_byte_off, s));
    return CAPNP_OK;
}

// Batch read_message on the device (msgbatch.hip): table decode per
// message, scans into the caller's offset arrays, one synchronisation for
// the totals (capacity check), segment lengths and the interleaved chunk
// tables, the batch unpack of the bodies, then the per-message status.
capnp_status capnp_gpu_read_messages(capnp_ctx* ctx, const uint8_t* d_packed,
                                     const uint64_t* d_msg_byte_off, size_t nmsg,
                                     const capnp_reader_options* opts, int try_mode,
                                     uint64_t* d_words, size_t words_cap,
                                     uint64_t* d_msg_word_off, uint64_t* d_seg_words,
                                     size_t segs_cap, uint64_t* d_msg_seg_off,
                                     int32_t* d_status, uint64_t* d_consumed, void* stream) {
    if (!ctx || !d_msg_word_off || !d_msg_seg_off ||
        (nmsg && (!d_msg_byte_off || !d_status)))
        return CAPNP_E_INVALID_ARGUMENT;
    hipStream_t s = pick(ctx, stream);
    UseMark um{ctx, s};
    if (nmsg == 0) {
        HIP_TRY(hipMemsetAsync(d_msg_word_off, 0, 8, s));
        HIP_TRY(hipMemsetAsync(d_msg_seg_off, 0, 8, s));
        return CAPNP_OK;
    }
    {
        capnp_status vst = check_offsets(ctx, s, {{d_msg_byte_off, nmsg, ~0ull}});
        if (vst != CAPNP_OK) return vst;
    }
    const capnp_reader_options o = opts ? *opts : capnp_default_reader_options();
    size_t scan_bytes = 0;
    HIP_TRY(capnp_msg_scan_bytes(nmsg + 1, &scan_bytes));
    const size_t n1 = nmsg + 1, n2 = 2 * nmsg + 1;
    const size_t o_nseg = 0;
    const size_t o_words = o_nseg + round16(n1 * 8);
    const size_t o_tst = o_words + round16(n1 * 8);
    const size_t o_tused = o_tst + round16(n1 * 4);
    const size_t o_tmp = o_tused + round16(n1 * 8);
    const size_t o_in2 = o_tmp + round16(scan_bytes + 16);
    const size_t o_out2 = o_in2 + round16(n2 * 8);
    const size_t o_cst = o_out2 + round16(n2 * 8);
    const size_t o_ccons = o_cst + round16(n2 * 4);
    const size_t o_end = o_ccons + round16(n2 * 8);
    capnp_status st = ensure_buf(ctx, &ctx->d_msg, &ctx->msg_cap, o_end + 64);
    if (st != CAPNP_OK) return st;
    uint8_t* d = ctx->d_msg;
    auto U = [&](size_t off) { return reinterpret_cast<uint64_t*>(d + off); };
    auto I = [&](size_t off) { return reinterpret_cast<int32_t*>(d + off); };
    const uint64_t limit = o.traversal_limit_in_words;
    const int has_limit = o.has_traversal_limit != 0;
    HIP_TRY(capnp_launch_msg_frame(d_packed, d_msg_byte_off, nmsg, try_mode, limit, has_limit,
                                   U(o_nseg), U(o_words), I(o_tst), U(o_tused), d + o_tmp,
                                   scan_bytes, d_msg_seg_off, d_msg_word_off, s));
    uint64_t tot[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&tot[0], d_msg_word_off + nmsg, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&tot[1], d_msg_seg_off + nmsg, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (tot[0] > words_cap || tot[1] > segs_cap || (tot[0] && !d_words) ||
        (tot[1] && !d_seg_words))
        return CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;
    HIP_TRY(capnp_launch_msg_segs(d_packed, d_msg_byte_off, nmsg, try_mode, limit, has_limit,
                                  I(o_tst), U(o_tused), d_msg_seg_off, d_msg_word_off,
                                  d_seg_words, U(o_in2), U(o_out2), s));
    const double mean = std::max((double)tot[0] / (double)(2 * nmsg), 1.0);
    const uint32_t utc = (uint32_t)std::max(1.0, std::min((double)capnp_unpack_tile_words() /
                                                              mean, 64.0));
    HIP_TRY(capnp_launch_unpack(d_packed, U(o_in2), 2 * nmsg, utc, d_words, U(o_out2),
                                I(o_cst), U(o_ccons), nullptr, s));
    HIP_TRY(capnp_launch_msg_status(nmsg, I(o_tst), U(o_tused), I(o_cst), U(o_ccons), d_status,
                                    d_consumed, s));
    return CAPNP_OK;
}

// try_read_message in a loop over one packed stream with no byte index
// (serialize.rs:310-325): the byte where each message starts.  Each round
// resolves the rest of the stream as one read unit (resync.hip), decodes it,
// follows the message chain through the segment tables and places the
// starts; a round that stops early (max_msgs, or a resolution that did not
// settle) is continued from where it stopped.
capnp_status capnp_gpu_find_messages(capnp_ctx* ctx, const uint8_t* d_packed, size_t nbytes,
                                     size_t max_msgs, uint64_t* d_msg_byte_off, size_t* nmsg,
                                     void* stream) {
    if (!ctx || !nmsg || !d_msg_byte_off || (nbytes && !d_packed)) return CAPNP_E_INVALID_ARGUMENT;
    hipStream_t s = pick(ctx, stream);
    UseMark um{ctx, s};
    *nmsg = 0;
    size_t found = 0;
    uint64_t start = 0;
    for (;;) {
        const uint64_t rest = nbytes - start;
        if (rest == 0 || found == max_msgs) break;
        uint64_t words_cap = ctx->stream_words_cap / 8, need = 0, m = 0;
        const size_t ws = capnp_resync_ws_bytes(1, rest) + 8 * (max_msgs - found + 16) + 4096 +
                          capnp_msg_chain_ws_bytes(words_cap);
        capnp_status st = ensure_buf(ctx, &ctx->d_resync, &ctx->resync_cap, ws);
        if (st != CAPNP_OK) return st;
        int clean = 0;
        hipError_t e = capnp_resync_find_messages(d_packed + start, rest, max_msgs - found,
                                                  d_msg_byte_off + found,
                                                  reinterpret_cast<uint64_t*>(ctx->d_stream_words),
                                                  words_cap, &m, &clean, ctx->d_resync,
                                                  ctx->resync_cap, s, &need);
        if (e == hipErrorInvalidValue && need > words_cap) {
            st = ensure_buf(ctx, &ctx->d_stream_words, &ctx->stream_words_cap, need * 8 + 64);
            if (st != CAPNP_OK) return st;
            continue;
        }
        HIP_TRY(e);
        // the round's offsets are relative to `start`
        if (start && m + 1 > 0) {
            std::vector<uint64_t> h(m + 1);
            HIP_TRY(hipMemcpyAsync(h.data(), d_msg_byte_off + found, 8 * (m + 1),
                                   hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            for (auto& v : h) v += start;
            HIP_TRY(hipMemcpyAsync(d_msg_byte_off + found, h.data(), 8 * (m + 1),
                                   hipMemcpyHostToDevice, s));
        }
        uint64_t stop = 0;
        HIP_TRY(hipMemcpyAsync(&stop, d_msg_byte_off + found + m, 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        found += m;
        if (m == 0 || clean || stop >= nbytes) break;
        start = stop;
    }
    if (found == 0) HIP_TRY(hipMemcpyAsync(d_msg_byte_off, &start, 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    *nmsg = found;
    return CAPNP_OK;
}

// try_read_message in a loop over one packed stream, in one pass: the
// stream is resolved and decoded once into the caller's d_words
// (capnp_resync_read_stream: block walk, decode, message chain), and the
// messages are described in place from their tables.  See the header.
capnp_status capnp_gpu_read_message_stream(capnp_ctx* ctx, const uint8_t* d_packed,
                                           size_t nbytes, const capnp_reader_options* opts,
                                           uint64_t* d_words, size_t words_cap,
                                           uint64_t* d_msg_byte_off, uint64_t* d_body_word_off,
                                           size_t msgs_cap, uint64_t* d_seg_words,
                                           size_t segs_cap, uint64_t* d_msg_seg_off,
                                           size_t* nmsg, int32_t* clean, size_t* words_need,
                                           size_t* msgs_need, size_t* segs_need, void* stream) {
    if (!ctx || !nmsg || !clean || !d_msg_byte_off || !d_msg_seg_off || (nbytes && !d_packed) ||
        (msgs_cap && !d_body_word_off) || (words_cap && !d_words))
        return CAPNP_E_INVALID_ARGUMENT;
    hipStream_t s = pick(ctx, stream);
    UseMark um{ctx, s};
    *nmsg = 0;
    *clean = 0;
    if (words_need) *words_need = 0;
    if (msgs_need) *msgs_need = 0;
    if (segs_need) *segs_need = 0;
    const capnp_reader_options o = opts ? *opts : capnp_default_reader_options();
    // scratch: word starts [msgs_cap + 1], segment counts [msgs_cap], the
    // first message over the traversal limit, the scan's temporary
    const size_t scan_tmp = capnp_scan_counts_tmp_bytes(msgs_cap + 1);
    const size_t o_ustart = 0, o_nseg = round16(8 * (msgs_cap + 1));
    const size_t o_bad = o_nseg + round16(8 * (msgs_cap + 1));
    const size_t o_tmp = o_bad + 16, o_end = o_tmp + round16(scan_tmp);
    capnp_status st = ensure_buf(ctx, &ctx->d_stream_words, &ctx->stream_words_cap, o_end + 64);
    if (st != CAPNP_OK) return st;
    uint8_t* d = ctx->d_stream_words;
    uint64_t* ustart = reinterpret_cast<uint64_t*>(d + o_ustart);
    uint64_t* nseg = reinterpret_cast<uint64_t*>(d + o_nseg);
    uint64_t* bad = reinterpret_cast<uint64_t*>(d + o_bad);
    const size_t ws = capnp_resync_ws_bytes(1, nbytes) + 8 * (msgs_cap + 16) + 4096 +
                      capnp_msg_chain_ws_bytes(words_cap);
    st = ensure_buf(ctx, &ctx->d_resync, &ctx->resync_cap, ws);
    if (st != CAPNP_OK) return st;
    uint64_t m = 0, total = 0, wneed = 0;
    int cl = 0;
    hipError_t e = capnp_resync_read_stream(d_packed, nbytes, msgs_cap, d_msg_byte_off, d_words,
                                            words_cap, ustart, &m, &total, &cl, ctx->d_resync,
                                            ctx->resync_cap, s, &wneed);
    if (e == hipErrorInvalidValue && wneed > words_cap) {
        if (words_need) *words_need = wneed;
        return CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;
    }
    HIP_TRY(e);
    if (total > msgs_cap) {  // (the lists hold msgs_cap; the chain has more)
        if (words_need) *words_need = wneed;
        if (msgs_need) *msgs_need = total;
        return CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;
    }
    // tables; a message over the traversal limit ends the loop there
    const uint64_t none = ~0ull;
    HIP_TRY(hipMemcpyAsync(bad, &none, 8, hipMemcpyHostToDevice, s));
    HIP_TRY(capnp_launch_msg_meta(d_words, ustart, m, o.traversal_limit_in_words,
                                  o.has_traversal_limit != 0, d_body_word_off, nseg, bad, s));
    uint64_t hbad = ~0ull;
    HIP_TRY(hipMemcpyAsync(&hbad, bad, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (hbad < m) {
        m = hbad;
        cl = 0;
    }
    HIP_TRY(capnp_scan_counts(nseg, m, d_msg_seg_off, d + o_tmp, scan_tmp, s));
    uint64_t nsegs = 0;
    HIP_TRY(hipMemcpyAsync(&nsegs, d_msg_seg_off + m, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (nsegs > segs_cap || (nsegs && !d_seg_words)) {
        if (words_need) *words_need = wneed;
        if (segs_need) *segs_need = nsegs;
        return CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;
    }
    HIP_TRY(capnp_launch_msg_seglist(d_words, ustart, m, d_msg_seg_off, d_seg_words, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (words_need) *words_need = wneed;
    if (msgs_need) *msgs_need = m;
    if (segs_need) *segs_need = nsegs;
    *nmsg = m;
    *clean = cl;
    return CAPNP_OK;
}

// Streaming reader support (stream_io.hip; not part of the public header):
// the longest prefix of complete records of n host bytes, resolved on the
// device (capnp_resync_prefix).
capnp_status capnp_stream_complete_prefix(capnp_ctx* ctx, const uint8_t* host, size_t n,
                                          uint64_t* bytes, uint64_t* words) {
    if (!ctx || !bytes || !words || (n && !host)) return CAPNP_E_INVALID_ARGUMENT;
    *bytes = *words = 0;
    if (n == 0) return CAPNP_OK;
    capnp_status st = ensure_stage(ctx, round16(n) + 64);
    if (st != CAPNP_OK) return st;
    const size_t ws = capnp_resync_ws_bytes(1, n) + 4096;
    st = ensure_buf(ctx, &ctx->d_resync, &ctx->resync_cap, ws);
    if (st != CAPNP_OK) return st;
    hipStream_t s = ctx->stream;
    HIP_TRY(hipMemcpyAsync(ctx->d_stage, host, n, hipMemcpyHostToDevice, s));
    HIP_TRY(capnp_resync_prefix(ctx->d_stage, n, ctx->d_resync, ctx->resync_cap, s, bytes, words));
    return CAPNP_OK;
}

// ... and decoded: the longest prefix of complete records of n host bytes
// with at most max_words words, its words into out[0, *words) (host; NULL:
// the lengths only).
capnp_status capnp_stream_decode_prefix(capnp_ctx* ctx, const uint8_t* host, size_t n,
                                        uint64_t max_words, uint64_t* out, uint64_t* bytes,
                                        uint64_t* words) {
    if (!ctx || !bytes || !words || (n && !host)) return CAPNP_E_INVALID_ARGUMENT;
    *bytes = *words = 0;
    if (n == 0 || max_words == 0) return CAPNP_OK;
    const size_t o_out = round16(n) + 64;
    capnp_status st = ensure_stage(ctx, o_out + (out ? max_words * 8 : 0) + 16);
    if (st != CAPNP_OK) return st;
    const size_t ws = capnp_resync_ws_bytes(1, n) + 4096;
    st = ensure_buf(ctx, &ctx->d_resync, &ctx->resync_cap, ws);
    if (st != CAPNP_OK) return st;
    hipStream_t s = ctx->stream;
    uint64_t* d_out = out ? reinterpret_cast<uint64_t*>(ctx->d_stage + o_out) : nullptr;
    HIP_TRY(hipMemcpyAsync(ctx->d_stage, host, n, hipMemcpyHostToDevice, s));
    HIP_TRY(capnp_resync_decode_prefix(ctx->d_stage, n, max_words, d_out, ctx->d_resync,
                                       ctx->resync_cap, s, bytes, words));
    if (out && *words) {
        HIP_TRY(hipMemcpyAsync(out, d_out, *words * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return CAPNP_OK;
}

capnp_status capnp_unpack_prefix(capnp_ctx* ctx, const uint8_t* in, size_t in_len,
                                 uint64_t max_words, uint64_t* out, size_t* bytes,
                                 uint64_t* words) {
    if (!bytes || !words) return CAPNP_E_INVALID_ARGUMENT;
    uint64_t b = 0;
    capnp_status st = capnp_stream_decode_prefix(ctx, in, in_len, max_words, out, &b, words);
    *bytes = (size_t)b;
    return st;
}

capnp_status capnp_gpu_read_flat_messages(capnp_ctx* ctx, const uint8_t* d_buf, size_t buf_len,
                                          const uint64_t* d_slice_off, size_t nmsg,
                                          const capnp_reader_options* opts, int no_alloc,
                                          uint32_t* d_seg_words, size_t segs_cap,
                                          uint64_t* d_msg_seg_off, int32_t* d_status,
                                          uint64_t* d_body_off, uint64_t* d_consumed,
                                          void* stream) {
    // d_buf may be NULL when every slice is empty (an empty tensor has no storage)
    if (!ctx || !d_msg_seg_off || (nmsg && (!d_slice_off || !d_status)))
        return CAPNP_E_INVALID_ARGUMENT;
    hipStream_t s = pick(ctx, stream);
    UseMark um{ctx, s};
    if (nmsg == 0) {
        HIP_TRY(hipMemsetAsync(d_msg_seg_off, 0, 8, s));
        return CAPNP_OK;
    }
    {
        // slices [slice_off[m], slice_off[m+1]) inside d_buf[0, buf_len)
        capnp_status vst = check_offsets(ctx, s, {{d_slice_off, nmsg, (uint64_t)buf_len}});
        if (vst != CAPNP_OK) return vst;
    }
    const capnp_reader_options o = opts ? *opts : capnp_default_reader_options();
    size_t scan_bytes = 0;
    HIP_TRY(capnp_msg_scan_bytes(nmsg + 1, &scan_bytes));
    const size_t o_nseg = 0;
    const size_t o_tmp = o_nseg + round16((nmsg + 1) * 8);
    const size_t o_end = o_tmp + round16(scan_bytes + 16);
    capnp_status st = ensure_buf(ctx, &ctx->d_msg, &ctx->msg_cap, o_end + 64);
    if (st != CAPNP_OK) return st;
    uint8_t* d = ctx->d_msg;
    const uint64_t limit = o.traversal_limit_in_words;
    const int has_limit = o.has_traversal_limit != 0;
    HIP_TRY(capnp_launch_flat_frame(d_buf, d_slice_off, nmsg, no_alloc, limit, has_limit,
                                    reinterpret_cast<uint64_t*>(d + o_nseg), d_status,
                                    d_body_off, d_consumed, d + o_tmp, scan_bytes,
                                    d_msg_seg_off, s));
    uint64_t tot = 0;
    HIP_TRY(hipMemcpyAsync(&tot, d_msg_seg_off + nmsg, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (tot > segs_cap || (tot && !d_seg_words)) return CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;
    HIP_TRY(capnp_launch_flat_segs(d_buf, d_slice_off, nmsg, no_alloc, limit, has_limit,
                                   d_status, d_msg_seg_off, d_seg_words, s));
    return CAPNP_OK;
}

capnp_status capnp_packed_write_message(capnp_ctx* ctx, const uint64_t* const* segs,
                                        const uint32_t* seg_words, uint32_t nseg, uint8_t* out,
                                        size_t cap, size_t* written) {
    if (!ctx || !written || nseg == 0 || !seg_words || !segs) return CAPNP_E_INVALID_ARGUMENT;
    *written = 0;
    // chunks: word 0, the rest of the table, then one per segment
    // (serialize.rs:605-679)
    const size_t rest = nseg == 1 ? 0 : (nseg < 4 ? 8 : (size_t)(nseg & ~1u) * 4);
    const size_t tw = 1 + rest / 8;  // table words
    const size_t nch = 1 + (nseg > 1 ? 1 : 0) + nseg;
    uint64_t nw = tw;
    for (uint32_t i = 0; i < nseg; i++) {
        if (seg_words[i] && !segs[i]) return CAPNP_E_INVALID_ARGUMENT;
        nw += seg_words[i];
    }
    const size_t bound = capnp_packed_batch_bound_bytes(nw, nch);
    const size_t o_off = round16(nw * 8), o_tot = o_off + round16((nch + 1) * 8);
    const size_t o_out = o_tot + 16;
    hipStream_t s = ctx->stream;
    // the table words and the chunk offsets, written where `base` points
    auto lay_out = [&](uint64_t* w, uint64_t* off) {
        w[0] = (uint64_t)(nseg - 1) | ((uint64_t)seg_words[0] << 32);
        if (rest) {
            uint32_t* t = reinterpret_cast<uint32_t*>(w + 1);
            memset(t, 0, rest);
            for (uint32_t i = 1; i < nseg; i++) t[i - 1] = seg_words[i];
        }
        size_t k = 0;
        off[k++] = 0;
        off[k++] = 1;
        if (rest) off[k++] = tw;
        uint64_t o = tw;
        for (uint32_t i = 0; i < nseg; i++) off[k++] = (o += seg_words[i]);
    };
    if (nw <= capnp_msg_pack_words() && nch <= 515 && o_out + bound + 64 <= kPinnedCall) {
        // one launch (msg_pack_kernel): chunks and offsets laid out in pinned
        // memory, the kernel writes the packed bytes and their total there
        capnp_status st = ensure_pin(ctx, o_out + bound + 64);
        if (st == CAPNP_OK) st = ensure_stage(ctx, bound + 64);
        if (st != CAPNP_OK) return st;
        uint8_t* h = ctx->h_pin;
        uint8_t* dh = ctx->d_pin;
        // the words and offsets: through the BAR when the device allows it
        uint8_t* dr = req_buf(ctx, o_tot);
        uint8_t* hw = dr ? dr : h;
        uint64_t* w = reinterpret_cast<uint64_t*>(hw);
        lay_out(w, reinterpret_cast<uint64_t*>(hw + o_off));
        uint64_t o = tw;
        for (uint32_t i = 0; i < nseg; i++) {
            if (seg_words[i]) memcpy(w + o, segs[i], (size_t)seg_words[i] * 8);
            o += seg_words[i];
        }
        if (dr) req_done();
        uint8_t* dw = dr ? dr : dh;  // (the kernel's view of the words and offsets)
        const uint32_t seq = next_seq(ctx);
        if (percall_warm(ctx)) {
            SvcPackReq q;
            q.words = (uint64_t)dw;
            q.off = (uint64_t)(dw + o_off);
            q.out = (uint64_t)(dh + o_out);  // (*total at dh + o_tot = out - 16)
            q.counts = nch | ((uint64_t)nw << 32);
            q.out_cap = bound;
            q.scratch = (uint64_t)ctx->d_stage;
            st = svc_call(ctx, 1, reinterpret_cast<const uint64_t*>(&q), seq);
        } else {
            HIP_TRY(capnp_launch_msg_pack(reinterpret_cast<uint64_t*>(dw),
                                          reinterpret_cast<uint64_t*>(dw + o_off), (uint32_t)nch,
                                          (uint32_t)nw, dh + o_out, bound,
                                          reinterpret_cast<uint64_t*>(dh + o_tot), ctx->d_flag,
                                          seq, ctx->d_stage, s));
            st = wait_call(ctx, seq, s);
        }
        percall_done(ctx);
        if (st != CAPNP_OK) return st;
        const uint64_t total = *reinterpret_cast<volatile uint64_t*>(h + o_tot);
        const size_t ncopy = std::min<uint64_t>(total, cap);
        if (ncopy) memcpy(out, h + o_out, ncopy);
        *written = ncopy;
        return total > cap ? CAPNP_E_BUFFER_NOT_LARGE_ENOUGH : CAPNP_OK;
    }
    // a long message: each segment goes to the device staging buffer straight
    // from the caller's memory (no host gather), the table and offsets from a
    // small host array; the batch pack; the bytes straight back into `out`
    const size_t o_oo = o_tot;  // (device layout: words, offsets, out offsets, out)
    const size_t o_dout = o_oo + round16((nch + 1) * 8);
    capnp_status st = ensure_stage(ctx, o_dout + bound + 16);
    if (st != CAPNP_OK) return st;
    uint8_t* d = ctx->d_stage;
    if (o_dout + bound + 16 <= kWritePinMax) {
        // mid-sized: laid out in pinned memory, one DMA in, the batch pack, one
        // DMA back of the offsets and the output bound, one wait (the
        // pageable copies each went through the runtime's staging and its
        // own synchronisation)
        st = ensure_pin(ctx, o_dout + bound + 16);
        if (st != CAPNP_OK) return st;
        uint8_t* h = ctx->h_pin;
        uint64_t* w = reinterpret_cast<uint64_t*>(h);
        lay_out(w, reinterpret_cast<uint64_t*>(h + o_off));
        uint64_t o = tw;
        for (uint32_t i = 0; i < nseg; i++) {
            if (seg_words[i]) memcpy(w + o, segs[i], (size_t)seg_words[i] * 8);
            o += seg_words[i];
        }
        HIP_TRY(hipMemcpyAsync(d, h, o_oo, hipMemcpyHostToDevice, s));
        const uint64_t wr[2] = {0, nw};
        const uint32_t tc = nw / nch >= kWordTileMean ? 0u : tile_chunks_for(nw, nch);
        st = pack_batch_dev(ctx, reinterpret_cast<uint64_t*>(d),
                            reinterpret_cast<uint64_t*>(d + o_off), nch, d + o_dout, bound,
                            reinterpret_cast<uint64_t*>(d + o_oo), tc, s, nullptr, wr);
        if (st != CAPNP_OK) return st;
        HIP_TRY(hipMemcpyAsync(h + o_oo, d + o_oo, o_dout - o_oo + bound, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        const uint64_t total = reinterpret_cast<const uint64_t*>(h + o_oo)[nch];
        const size_t ncopy = std::min<uint64_t>(total, cap);
        if (ncopy) memcpy(out, h + o_dout, ncopy);
        *written = ncopy;
        return total > cap ? CAPNP_E_BUFFER_NOT_LARGE_ENOUGH : CAPNP_OK;
    }
    std::vector<uint64_t> small(tw);
    std::vector<uint64_t> off(nch + 1);
    lay_out(small.data(), off.data());
    HIP_TRY(hipMemcpyAsync(d, small.data(), tw * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(d + o_off, off.data(), (nch + 1) * 8, hipMemcpyHostToDevice, s));
    uint64_t o = tw;
    for (uint32_t i = 0; i < nseg; i++) {
        if (seg_words[i])
            HIP_TRY(hipMemcpyAsync(d + o * 8, segs[i], (size_t)seg_words[i] * 8,
                                   hipMemcpyHostToDevice, s));
        o += seg_words[i];
    }
    const uint64_t wr[2] = {0, nw};
    const uint32_t tc = nw / nch >= kWordTileMean ? 0u : tile_chunks_for(nw, nch);
    st = pack_batch_dev(ctx, reinterpret_cast<uint64_t*>(d), reinterpret_cast<uint64_t*>(d + o_off),
                        nch, d + o_dout, bound, reinterpret_cast<uint64_t*>(d + o_oo), tc, s,
                        nullptr, wr);
    if (st != CAPNP_OK) return st;
    uint64_t total = 0;
    HIP_TRY(hipMemcpyAsync(&total, d + o_oo + nch * 8, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const size_t ncopy = std::min<uint64_t>(total, cap);
    if (ncopy) {
        HIP_TRY(hipMemcpyAsync(out, d + o_dout, ncopy, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    *written = ncopy;
    return total > cap ? CAPNP_E_BUFFER_NOT_LARGE_ENOUGH : CAPNP_OK;
}

// A message whose body is short (< kParallelBodyWords words, and within the
// caller's capacity) in ONE launch: the input prefix that can hold the table
// and such a body (<= 10 bytes per word) is copied into the pinned buffer,
// and msg_read_kernel (unpack.hip) reads it there, checks the table, decodes
// the body with the workgroup's long-unit decode and writes the frame
// result, the body's status and consumed bytes and its words back into
// pinned memory (a body too long, or a failed table, is an empty unit): one
// launch and one wait.  *done = false when the body still has to be read the
// long way (read_body): it is longer than that, or its unit ran past the
// staged prefix of a longer input.  The reference's per-message cost
// (serialize_packed::read_message once per request, benchmark.rs:207-259) is
// this call.
static capnp_status read_message_fast(capnp_ctx* ctx, const uint8_t* in, size_t in_len,
                                      const capnp_reader_options* opts, int try_mode,
                                      int no_alloc, uint64_t buffer_len, uint64_t cap_words,
                                      FrameResult* fr, const uint8_t** words,
                                      uint64_t* body_consumed, bool* done) {
    capnp_reader_options o = opts ? *opts : capnp_default_reader_options();
    *done = false;
    *body_consumed = 0;
    const uint64_t cap = std::min<uint64_t>(cap_words, kParallelBodyWords - 1);
    const size_t stage = std::min<size_t>(in_len, kTablePrefixBytes + cap * 10 + 16);
    const size_t o_st = round16(cap * 8);  // body words, then status, pad, consumed
    const size_t h_out = round16(stage + 16);
    capnp_status st = ensure_pin(ctx, h_out + o_st + 64);
    if (st != CAPNP_OK) return st;
    uint8_t* h = ctx->h_pin;
    uint8_t* dh = ctx->d_pin;
    hipStream_t s = ctx->stream;
    // the staged input: through the BAR when the device allows it (req_buf)
    uint8_t* dr = req_buf(ctx, round16(stage) + 16);
    if (stage) memcpy(dr ? dr : h, in, stage);
    if (dr) req_done();
    uint8_t* din = dr ? dr : dh;
    // one launch: the kernel reads the staged bytes and writes the frame
    // record, the body's status and its words in pinned memory
    const uint32_t seq = next_seq(ctx);
    if (percall_warm(ctx)) {
        SvcReadReq q;
        q.in = (uint64_t)din;
        q.words = (uint64_t)(dh + h_out);  // (res at + o_st = round16(8 cap))
        q.flags = stage | ((uint64_t)(no_alloc != 0) << 32) | ((uint64_t)(try_mode != 0) << 33) |
                  ((uint64_t)(o.has_traversal_limit != 0) << 34);
        q.limit = o.traversal_limit_in_words;
        q.buffer_len = buffer_len;
        q.cap = cap;
        st = svc_call(ctx, 0, reinterpret_cast<const uint64_t*>(&q), seq);
    } else {
        HIP_TRY(capnp_launch_msg_read(din, stage, (uint32_t)no_alloc, (uint32_t)(try_mode != 0),
                                      o.traversal_limit_in_words,
                                      (uint32_t)(o.has_traversal_limit != 0), buffer_len, cap,
                                      ctx->d_hframe, reinterpret_cast<uint64_t*>(dh + h_out),
                                      reinterpret_cast<uint64_t*>(dh + h_out + o_st), ctx->d_flag,
                                      seq, s));
        st = wait_call(ctx, seq, s);
    }
    percall_done(ctx);
    if (st != CAPNP_OK) return st;
    *fr = *ctx->h_frame;
    if (fr->status != CAPNP_OK || fr->total_words > cap) return CAPNP_OK;  // (the caller decides)
    uint64_t res[3];
    memcpy(res, h + h_out + o_st, 24);  // status (low 32 bits), pad, consumed
    const int32_t bst = (int32_t)(uint32_t)res[0];
    if ((bst == CAPNP_E_PREMATURE_END_OF_PACKED_INPUT || bst == CAPNP_E_FAILED_TO_FILL_WHOLE_BUFFER) &&
        stage < in_len)
        return CAPNP_OK;  // the unit ran past the staged prefix: the long way
    *done = true;
    *words = h + h_out;  // (the caller copies them out, even on an error, as read_body does)
    if (bst != CAPNP_OK) return (capnp_status)bst;
    *body_consumed = res[2];
    return CAPNP_OK;
}

// Decodes the body unit (read_exact of total_words words after the table,
// serialize.rs:514-524) into host memory.  The stream decodes at most 10
// bytes per word, so at most 10 * words + 16 bytes after the table are
// staged; the result (status, consumed, words) comes back in one copy.
static capnp_status read_body(capnp_ctx* ctx, const FrameResult& fr, const uint8_t* in,
                              size_t in_len, uint8_t* host_out, uint64_t* body_consumed) {
    *body_consumed = 0;
    if (fr.total_words == 0) return CAPNP_OK;
    const size_t rem = in_len - std::min<size_t>(in_len, fr.table_consumed);
    const size_t take = std::min<size_t>(rem, fr.total_words * 10 + 16);
    const size_t o_in = 0, o_off = round16(take + 16), o_res = o_off + 32;
    capnp_status st = ensure_stage(ctx, o_res + 64);
    if (st != CAPNP_OK) return st;
    const size_t o_st = round16(fr.total_words * 8);
    st = ensure_buf(ctx, &ctx->d_body, &ctx->body_cap, o_st + 64);
    if (st != CAPNP_OK) return st;
    uint8_t* di = ctx->d_stage;
    uint8_t* d = ctx->d_body;
    hipStream_t s = ctx->stream;
    const uint64_t offs[4] = {0, take, 0, fr.total_words};
    // a small body: staged bytes and their unit offsets in, status and words
    // out, through the pinned buffer (one copy each way)
    const bool pinned = fr.total_words < kParallelBodyWords && o_res + o_st + 64 <= kPinnedCall;
    if (pinned) {
        st = ensure_pin(ctx, std::max<size_t>(o_res, o_st + 32) + 64);
        if (st != CAPNP_OK) return st;
        uint8_t* h = ctx->h_pin;
        if (take) memcpy(h + o_in, in + fr.table_consumed, take);
        memcpy(h + o_off, offs, sizeof(offs));
        HIP_TRY(hipMemcpyAsync(di, h, o_off + sizeof(offs), hipMemcpyHostToDevice, s));
        HIP_TRY(capnp_launch_unpack(di + o_in, reinterpret_cast<uint64_t*>(di + o_off), 1, 0,
                                    reinterpret_cast<uint64_t*>(d),
                                    reinterpret_cast<uint64_t*>(di + o_off + 16),
                                    reinterpret_cast<int32_t*>(d + o_st),
                                    reinterpret_cast<uint64_t*>(d + o_st + 16), nullptr, s));
        HIP_TRY(hipMemcpyAsync(h, d, o_st + 24, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        uint64_t res[3];
        memcpy(res, h + o_st, 24);  // status (low 32 bits), pad, consumed
        memcpy(host_out, h, fr.total_words * 8);  // (as below: the words even on an error)
        const int32_t status = (int32_t)(uint32_t)res[0];
        if (status != CAPNP_OK) return (capnp_status)status;
        *body_consumed = res[2];
        return CAPNP_OK;
    }
    if (take) HIP_TRY(hipMemcpyAsync(di + o_in, in + fr.table_consumed, take,
                                     hipMemcpyHostToDevice, s));
    if (fr.total_words >= kParallelBodyWords && take) {
        // A long body decodes in parallel: the whole records of the staged
        // bytes up to the body's words, resolved block by block
        // (capnp_resync_decode_prefix) instead of one lane walking the unit.
        // If they fill the body exactly, that is the read: read_exact stops
        // right after the record that fills its buffer
        // (serialize_packed.rs:222-225).  Otherwise the read fails, and the
        // exact unit decode below gives its status.
        st = ensure_buf(ctx, &ctx->d_resync, &ctx->resync_cap, capnp_resync_ws_bytes(1, take) + 4096);
        if (st != CAPNP_OK) return st;
        uint64_t pb = 0, pw = 0;
        HIP_TRY(capnp_resync_decode_prefix(di + o_in, take, fr.total_words,
                                           reinterpret_cast<uint64_t*>(d), ctx->d_resync,
                                           ctx->resync_cap, s, &pb, &pw));
        if (pw == fr.total_words) {
            HIP_TRY(hipMemcpyAsync(host_out, d, fr.total_words * 8, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            *body_consumed = pb;
            return CAPNP_OK;
        }
    }
    HIP_TRY(hipMemcpyAsync(di + o_off, offs, sizeof(offs), hipMemcpyHostToDevice, s));
    HIP_TRY(capnp_launch_unpack(di + o_in, reinterpret_cast<uint64_t*>(di + o_off), 1, 0,
                                reinterpret_cast<uint64_t*>(d),
                                reinterpret_cast<uint64_t*>(di + o_off + 16),
                                reinterpret_cast<int32_t*>(d + o_st),
                                reinterpret_cast<uint64_t*>(d + o_st + 16), nullptr, s));
    uint64_t res[3] = {0, 0, 0};  // status (low 32 bits), pad, consumed
    HIP_TRY(hipMemcpyAsync(res, d + o_st, 24, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(host_out, d, fr.total_words * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const int32_t status = (int32_t)(uint32_t)res[0];
    if (status != CAPNP_OK) return (capnp_status)status;
    *body_consumed = res[2];
    return CAPNP_OK;
}

capnp_status capnp_packed_read_message(capnp_ctx* ctx, const uint8_t* in, size_t in_len,
                                       const capnp_reader_options* opts, int try_mode,
                                       uint64_t* body, size_t body_cap_words,
                                       uint32_t* seg_words_out, uint32_t* nseg_out,
                                       size_t* consumed) {
    if (!ctx || !consumed || !nseg_out || !seg_words_out || (in_len && !in))
        return CAPNP_E_INVALID_ARGUMENT;
    *consumed = 0;
    *nseg_out = 0;
    FrameResult fr;
    uint64_t used = 0;
    bool done = false;
    const uint8_t* fw = nullptr;
    capnp_status st = read_message_fast(ctx, in, in_len, opts, try_mode, 0, 0, body_cap_words, &fr,
                                        &fw, &used, &done);
    if (done && fr.total_words) memcpy(body, fw, fr.total_words * 8);
    if (st != CAPNP_OK) return st;
    if (fr.status != CAPNP_OK) return (capnp_status)fr.status;
    if (fr.total_words > body_cap_words) {
        // the table is read: report it, so the caller can size the body
        memcpy(seg_words_out, fr.seg_words, fr.nseg * sizeof(uint32_t));
        *nseg_out = fr.nseg;
        return CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;
    }
    if (!done) st = read_body(ctx, fr, in, in_len, reinterpret_cast<uint8_t*>(body), &used);
    if (st != CAPNP_OK) return st;
    memcpy(seg_words_out, fr.seg_words, fr.nseg * sizeof(uint32_t));
    *nseg_out = fr.nseg;
    *consumed = fr.table_consumed + used;
    return CAPNP_OK;
}

capnp_status capnp_packed_read_message_no_alloc(capnp_ctx* ctx, const uint8_t* in,
                                                size_t in_len, const capnp_reader_options* opts,
                                                int try_mode, uint8_t* buffer, size_t buffer_len,
                                                uint32_t* nseg_out, size_t* table_bytes_out,
                                                size_t* body_bytes_out, size_t* consumed) {
    if (!ctx || !consumed || !nseg_out || !table_bytes_out || !body_bytes_out || (in_len && !in))
        return CAPNP_E_INVALID_ARGUMENT;
    *consumed = 0;
    *nseg_out = 0;
    if (((uintptr_t)buffer) % 8 != 0) return CAPNP_E_UNALIGNED_SEGMENT;  // serialize.rs:341-343
    if (buffer_len < 8) return CAPNP_E_BUFFER_NOT_LARGE_ENOUGH;          // :345-347
    FrameResult fr;
    uint64_t used = 0;
    bool done = false;
    // (the frame kernel checks the table plus body against buffer_len, so a
    // body it passes fits after the table)
    const uint64_t cap_words = buffer_len / 8;
    const uint8_t* fw = nullptr;
    capnp_status st = read_message_fast(ctx, in, in_len, opts, try_mode, 1, buffer_len, cap_words,
                                        &fr, &fw, &used, &done);
    if (st != CAPNP_OK && !done) return st;
    // the table bytes land in the caller's buffer as the reference reads them
    if (fr.status == CAPNP_OK) memcpy(buffer, fr.table, fr.table_bytes);
    if (fr.status != CAPNP_OK) return (capnp_status)fr.status;
    if (done) {  // (the words came back with the table)
        if (fr.total_words) memcpy(buffer + fr.table_bytes, fw, fr.total_words * 8);
    } else {
        st = read_body(ctx, fr, in, in_len, buffer + fr.table_bytes, &used);
    }
    if (st != CAPNP_OK) return st;
    *nseg_out = fr.nseg;
    *table_bytes_out = fr.table_bytes;
    *body_bytes_out = fr.total_words * 8;
    *consumed = fr.table_consumed + used;
    return CAPNP_OK;
}

}  // extern "C"
