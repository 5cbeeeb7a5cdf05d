// frame.hip — message framing on the device: the segment-table read units of
// serialize_packed::{read_message, try_read_message, read_message_no_alloc,
// try_read_message_no_alloc} (serialize_packed.rs:233-291 ->
// serialize.rs:287-420, 448-510).
//
// The table is tiny (<= 2 KiB) and its read units are sequential, so one
// lane decodes them with the same PackedRead semantics as the batch kernel
// (serialize_packed.rs:80-228), validates the table and leaves the packed
// range and unpacked length of the body unit in device memory, where the
// batch UNPACK kernel picks them up without a host round trip.
#include "common.h"
#include "frame.h"

namespace {

using namespace capnp_frame;

__global__ void frame_kernel(const uint8_t* __restrict__ in, uint64_t in_len, uint32_t no_alloc,
                             uint32_t try_mode, uint64_t limit, uint32_t has_limit,
                             uint64_t buffer_len, uint64_t body_cap,
                             FrameResult* __restrict__ r) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    frame_table(in, in_len, no_alloc, try_mode, limit, has_limit, buffer_len, body_cap, r);
}

}  // namespace

extern "C" hipError_t capnp_launch_frame(const uint8_t* d_in, uint64_t in_len, uint32_t no_alloc,
                                         uint32_t try_mode, uint64_t limit, uint32_t has_limit,
                                         uint64_t buffer_len, uint64_t body_cap,
                                         FrameResult* d_result, hipStream_t stream) {
    hipLaunchKernelGGL(frame_kernel, dim3(1), dim3(64), 0, stream, d_in, in_len, no_alloc,
                       try_mode, limit, has_limit, buffer_len, body_cap, d_result);
    return hipGetLastError();
}
