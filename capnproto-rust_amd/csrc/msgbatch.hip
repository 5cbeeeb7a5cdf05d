// msgbatch.hip — device framing of many messages at once: the batched body of
// serialize_packed::write_message (serialize_packed.rs:446-453 ->
// serialize.rs:574-679), SURVEY §8f row 1.
//
// write_message packs a message as separate write_all calls: the segment
// table's first word, the rest of the table (when there is more than one
// segment), then every segment (serialize.rs:605-679), and a packed write_all
// never carries a run across calls.  So a batch of messages is a batch of
// chunks: msg_layout sizes each message (table words, chunk count), two
// exclusive scans place them, msg_assemble writes each message's table words
// and copies its segments into one staging array with the chunk offsets of
// the layout, and the regular batch pack kernel packs the chunks.  The
// message byte offsets are the chunk offsets of each message's first chunk.
#include "common.h"
#include "../../include/capnp_packed.h"
#include <hipcub/hipcub.hpp>

namespace {

constexpr int kThreads = 256;

// Per message: staging words (table + segments) and chunk count, into
// cw[m] / cc[m] (m < nmsg; entry nmsg is 0 so the exclusive scans end in the
// totals).  The table is 1 + nseg / 2 words: word 0 = (nseg - 1, len 0),
// then the other lengths as u32, padded to a word (serialize.rs:211-253).
__global__ void msg_layout(const uint64_t* __restrict__ seg_off,
                           const uint64_t* __restrict__ msg_seg_off, uint64_t nmsg,
                           uint64_t* __restrict__ cw, uint64_t* __restrict__ cc) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m > nmsg) return;
    if (m == nmsg) {
        cw[m] = 0;
        cc[m] = 0;
        return;
    }
    const uint64_t s0 = msg_seg_off[m], s1 = msg_seg_off[m + 1];
    const uint64_t nseg = s1 - s0;
    cw[m] = 1 + nseg / 2 + (seg_off[s1] - seg_off[s0]);
    cc[m] = 1 + (nseg > 1 ? 1 : 0) + nseg;
}

// One wave per message: table words, chunk offsets (staging-relative word
// offsets; chunk c ends where chunk c + 1 starts) and the segment words.
__global__ void msg_assemble(const uint64_t* __restrict__ words,
                             const uint64_t* __restrict__ seg_off,
                             const uint64_t* __restrict__ msg_seg_off, uint64_t nmsg,
                             const uint64_t* __restrict__ wofs, const uint64_t* __restrict__ cofs,
                             uint64_t* __restrict__ stage, uint64_t* __restrict__ chunk_off) {
    const uint64_t m = (uint64_t)blockIdx.x * (kThreads / CAPNP_WAVE) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (m >= nmsg) return;
    const uint64_t s0 = msg_seg_off[m], s1 = msg_seg_off[m + 1];
    const uint64_t nseg = s1 - s0;
    const uint64_t w = wofs[m], c = cofs[m];
    const uint64_t t = 1 + nseg / 2;  // table words
    uint64_t* dst = stage + w;
    uint32_t* tab = reinterpret_cast<uint32_t*>(dst);
    // table: u32 [nseg - 1, len 0, len 1, ..., pad]
    for (uint64_t i = lane; i < 2 * t; i += CAPNP_WAVE) {
        uint32_t v;
        if (i == 0) v = (uint32_t)(nseg - 1);
        else if (i - 1 < nseg) v = (uint32_t)(seg_off[s0 + i] - seg_off[s0 + i - 1]);
        else v = 0;
        tab[i] = v;
    }
    // chunks: table word 0, the rest of the table, each segment
    if (lane == 0) {
        chunk_off[c] = w;
        if (nseg > 1) chunk_off[c + 1] = w + 1;
    }
    const uint64_t cs = c + 1 + (nseg > 1 ? 1 : 0);
    const uint64_t base = seg_off[s0];
    for (uint64_t j = lane; j < nseg; j += CAPNP_WAVE)
        chunk_off[cs + j] = w + t + (seg_off[s0 + j] - base);
    if (m + 1 == nmsg && lane == 0) chunk_off[cs + nseg] = w + t + (seg_off[s1] - base);
    // segment words (contiguous in the input from seg_off[s0] on)
    const uint64_t n = seg_off[s1] - base;
    const uint64_t* src = words + base;
    for (uint64_t i = lane; i < n; i += CAPNP_WAVE) dst[t + i] = src[i];
}

__global__ void msg_offsets(const uint64_t* __restrict__ cofs,
                            const uint64_t* __restrict__ chunk_byte_off, uint64_t nmsg,
                            uint64_t* __restrict__ msg_byte_off) {
    const uint64_t m = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (m <= nmsg) msg_byte_off[m] = chunk_byte_off[cofs[m]];
}

}  // namespace

extern "C" hipError_t capnp_msg_scan_bytes(uint64_t n, size_t* bytes) {
    *bytes = 0;
    return hipcub::DeviceScan::ExclusiveSum(nullptr, *bytes, (const uint64_t*)nullptr,
                                            (uint64_t*)nullptr, (int)n);
}

// Layout, scans and assembly; the caller reads the totals (wofs[nmsg],
// cofs[nmsg]) before packing.  tmp: capnp_msg_scan_bytes(nmsg + 1) bytes.
extern "C" hipError_t capnp_launch_msg_prepare(const uint64_t* d_words, const uint64_t* d_seg_off,
                                               const uint64_t* d_msg_seg_off, uint64_t nmsg,
                                               uint64_t* cw, uint64_t* cc, uint64_t* wofs,
                                               uint64_t* cofs, void* tmp, size_t tmp_bytes,
                                               uint64_t* stage, uint64_t* chunk_off,
                                               hipStream_t s) {
    const uint32_t g1 = (uint32_t)((nmsg + 1 + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(msg_layout, dim3(g1), dim3(kThreads), 0, s, d_seg_off, d_msg_seg_off, nmsg,
                       cw, cc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cw, wofs, (int)(nmsg + 1), s);
    if (e != hipSuccess) return e;
    tb = tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cc, cofs, (int)(nmsg + 1), s);
    if (e != hipSuccess) return e;
    const uint32_t per = kThreads / CAPNP_WAVE;
    const uint32_t g2 = (uint32_t)((nmsg + per - 1) / per);
    if (g2)
        hipLaunchKernelGGL(msg_assemble, dim3(g2), dim3(kThreads), 0, s, d_words, d_seg_off,
                           d_msg_seg_off, nmsg, wofs, cofs, stage, chunk_off);
    return hipGetLastError();
}

extern "C" hipError_t capnp_launch_msg_offsets(const uint64_t* cofs,
                                               const uint64_t* chunk_byte_off, uint64_t nmsg,
                                               uint64_t* msg_byte_off, hipStream_t s) {
    const uint32_t g = (uint32_t)((nmsg + 1 + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(msg_offsets, dim3(g), dim3(kThreads), 0, s, cofs, chunk_byte_off, nmsg,
                       msg_byte_off);
    return hipGetLastError();
}
