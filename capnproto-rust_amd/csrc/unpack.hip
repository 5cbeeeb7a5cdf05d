// unpack.hip — gfx950 UNPACK kernel: the batched body of PackedRead::read
// under read_exact (capnp/src/serialize_packed.rs:80-228, io.rs:16-31).
//
// The decode of one chunk is a serial chain: the position of tag k+1 depends
// on the value of tag k.  Parallelism therefore comes from independent
// chunks (the batch carries a side-band index: each chunk's packed range and
// unpacked length, produced by the encoder's offsets):
//
//   walk       lane l of a wave owns chunk 64g + l and follows its tag chain
//              for the next 64 output words, writing one 16-bit descriptor
//              per head word (kind + packed position relative to the round's
//              base) into an LDS table desc[chunk][word];
//   expand     the whole wave then takes the chunks one at a time, lane =
//              output word: the head covering each word is the highest
//              descriptor at or below it (ballot + clz), the word is rebuilt
//              from the tag and its non-zero bytes (v_perm with a SWAR rank
//              selector), zero-run words are 0, literal-run words are copied;
//              every chunk's 64 words leave as one 512-byte coalesced store.
//
// Status per chunk follows the reference exactly (first error in stream
// order): PrematureEndOfPackedInput when a tag, a tag's bytes or a run count
// is missing (:59-74, :109-145), DidNotEndCleanly when a run overruns the
// output (:166-170, :183-187; checked before copying), FailedToFill when a
// literal run's bytes are missing (:195-205 + io.rs:26-28) or the input is
// empty (read() returns 0, io.rs:26-28).
#include "common.h"

namespace {

constexpr int kWaves = 4;
constexpr int kThreads = kWaves * CAPNP_WAVE;

enum : uint32_t {
    KIND_NONE = 0,
    KIND_NORMAL = 1,   // head word with tag not in {0x00, 0xFF}
    KIND_ZERO = 2,     // tag 0x00 head
    KIND_LIT = 3,      // tag 0xFF head
    KIND_ZERO_CONT = 4,  // zero run carried in from an earlier round
    KIND_LIT_CONT = 5,   // literal run carried in; position = its next raw word
};

enum : int32_t {
    ST_OK = 0,
    ST_PREMATURE = 2,
    ST_NOT_CLEAN = 3,
    ST_FAILED_FILL = 4,
};

// Loads `len` (1..8) bytes at byte position `pos` of `base` with aligned
// 8-byte loads, touching only qwords that hold a requested byte.
__device__ __forceinline__ uint64_t load_bytes(const uint8_t* __restrict__ base, uint64_t pos,
                                               uint32_t len) {
    const uint64_t a = pos & ~7ull;
    const uint32_t s = (uint32_t)(pos & 7);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(base + a);
    uint64_t v = q[0] >> (8 * s);
    if (s + len > 8) v |= q[1] << (64 - 8 * s);
    return v;
}

__device__ __forceinline__ uint64_t expand_word(uint32_t tag, uint64_t packed) {
    const uint64_t sel = expand_selector(tag);
    const uint32_t lo = (uint32_t)packed, hi = (uint32_t)(packed >> 32);
    const uint32_t rlo = __builtin_amdgcn_perm(hi, lo, (uint32_t)sel);
    const uint32_t rhi = __builtin_amdgcn_perm(hi, lo, (uint32_t)(sel >> 32));
    return ((uint64_t)rhi << 32) | rlo;
}

__global__ void __launch_bounds__(kThreads)
unpack_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
              uint64_t nchunks, uint64_t* __restrict__ out,
              const uint64_t* __restrict__ out_off, int32_t* __restrict__ status,
              uint64_t* __restrict__ consumed) {
    __shared__ alignas(16) uint16_t desc_all[kWaves][CAPNP_WAVE][CAPNP_WAVE];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    uint16_t(*desc)[CAPNP_WAVE] = desc_all[wave];

    const uint64_t c = ((uint64_t)blockIdx.x * kWaves + wave) * CAPNP_WAVE + lane;
    const bool have = c < nchunks;
    uint64_t p = 0, in_end = 0, n = 0, obase = 0;
    if (have) {
        p = in_off[c];
        in_end = in_off[c + 1];
        obase = out_off[c];
        n = out_off[c + 1] - obase;
    }
    const uint64_t p_start = p;
    int32_t st = ST_OK;
    uint64_t w = 0;  // words decoded so far
    bool active = have && n > 0;
    if (active && p == in_end) {  // read() returns Ok(0): read_exact fails
        st = ST_FAILED_FILL;
        active = false;
    }
    uint32_t pend_kind = KIND_NONE;  // carried run
    uint64_t pend_rem = 0, pend_src = 0;

    for (uint64_t wbeg = 0; ballot64(active); wbeg += CAPNP_WAVE) {
        // clear this wave's descriptor table (8 KiB, 16 B per lane-store)
        {
            uint4* d4 = reinterpret_cast<uint4*>(&desc[0][0]);
#pragma unroll
            for (int k = 0; k < 8; k++) d4[k * CAPNP_WAVE + lane] = make_uint4(0, 0, 0, 0);
        }
        wave_lds_sync();

        // ---- walk: lane = chunk
        uint32_t cnt_round = 0;
        uint64_t pb = p;
        if (active) {
            const uint64_t wend = (wbeg + CAPNP_WAVE < n) ? wbeg + CAPNP_WAVE : n;
            if (pend_kind == KIND_LIT_CONT) pb = pend_src;
            if (pend_kind != KIND_NONE) {
                desc[lane][0] = (uint16_t)(pend_kind << 12);  // position = pb
                const uint64_t room = wend - w;
                const uint64_t take = pend_rem < room ? pend_rem : room;
                w += take;
                pend_rem -= take;
                if (pend_kind == KIND_LIT_CONT) pend_src += 8 * take;
                if (pend_rem == 0) pend_kind = KIND_NONE;
            }
            while (w < wend) {
                if (p >= in_end) { st = ST_PREMATURE; break; }
                const uint32_t tag = in[p];
                const uint32_t pop = __builtin_popcount(tag);
                if (p + 1 + pop > in_end) { st = ST_PREMATURE; break; }
                const uint32_t kind = tag == 0 ? KIND_ZERO : (tag == 0xFF ? KIND_LIT : KIND_NORMAL);
                desc[lane][w - wbeg] = (uint16_t)((kind << 12) | (uint32_t)(p - pb));
                uint64_t q = p + 1 + pop;
                w += 1;
                if (kind != KIND_NORMAL) {
                    if (q >= in_end) { st = ST_PREMATURE; break; }
                    const uint64_t cnt = in[q];
                    q += 1;
                    if (cnt > n - w) { st = ST_NOT_CLEAN; break; }
                    uint64_t src = q;
                    if (kind == KIND_LIT) {
                        if (in_end - q < 8 * cnt) { st = ST_FAILED_FILL; break; }
                        q += 8 * cnt;
                    }
                    const uint64_t room = wend - w;
                    const uint64_t take = cnt < room ? cnt : room;
                    w += take;
                    if (cnt > take) {
                        pend_kind = kind == KIND_LIT ? KIND_LIT_CONT : KIND_ZERO_CONT;
                        pend_rem = cnt - take;
                        pend_src = src + 8 * take;
                    }
                }
                p = q;
            }
            cnt_round = (uint32_t)(w - wbeg);
            if (st != ST_OK) { active = false; cnt_round = 0; }
            else if (w == n) active = false;
        }
        wave_lds_sync();

        // ---- expand: lane = word of one chunk at a time
        for (uint32_t s = 0; s < CAPNP_WAVE; s++) {
            const uint32_t cr = (uint32_t)__builtin_amdgcn_readlane((int)cnt_round, s);
            if (cr == 0) continue;
            const uint64_t pbs = readlane64(pb, s);
            const uint64_t ob = readlane64(obase, s);
            const bool valid = lane < cr;
            const uint32_t d = valid ? desc[s][lane] : 0u;
            const uint64_t heads = ballot64(d != 0);
            const uint64_t hm = heads & low_mask(lane + 1);
            const uint32_t h = hm ? 63u - (uint32_t)__builtin_clzll(hm) : 0u;
            const uint32_t dh = (h == lane) ? d : (uint32_t)desc[s][h];
            const uint32_t kind = dh >> 12;
            const uint64_t pos = pbs + (dh & 0xFFFu);
            uint64_t word = 0;
            if (valid) {
                if (kind == KIND_NORMAL) {
                    const uint32_t tag = in[pos];
                    const uint32_t pop = __builtin_popcount(tag);
                    const uint64_t pk = load_bytes(in, pos + 1, pop);
                    word = expand_word(tag, pk);
                } else if (kind == KIND_LIT) {
                    const uint64_t src = (h == lane) ? pos + 1 : pos + 10 + 8ull * (lane - h - 1);
                    word = load_bytes(in, src, 8);
                } else if (kind == KIND_LIT_CONT) {
                    word = load_bytes(in, pos + 8ull * (lane - h), 8);
                }
                out[ob + wbeg + lane] = word;
            }
        }
        wave_lds_sync();
    }
    if (have) {
        status[c] = st;
        // bytes used: all of them when a literal run ran dry (the reference
        // copies what is there before read_exact fails), none on other errors
        if (consumed)
            consumed[c] = st == ST_OK ? p - p_start : (st == ST_FAILED_FILL ? in_end - p_start : 0);
    }
}

}  // namespace

extern "C" hipError_t capnp_launch_unpack(const uint8_t* d_in, const uint64_t* d_in_off,
                                          uint64_t nchunks, uint64_t* d_out,
                                          const uint64_t* d_out_off, int32_t* d_status,
                                          uint64_t* d_consumed, hipStream_t stream) {
    if (nchunks == 0) return hipSuccess;
    const uint64_t per_block = (uint64_t)kWaves * CAPNP_WAVE;
    const uint64_t blocks = (nchunks + per_block - 1) / per_block;
    hipLaunchKernelGGL(unpack_kernel, dim3((uint32_t)blocks), dim3(kThreads), 0, stream, d_in,
                       d_in_off, nchunks, d_out, d_out_off, d_status, d_consumed);
    return hipGetLastError();
}
