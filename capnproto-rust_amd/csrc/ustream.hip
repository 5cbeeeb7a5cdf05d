// ustream.hip — gfx950 index-free UNPACK: the batched body of PackedRead::read
// under read_exact (capnp/src/serialize_packed.rs:80-228, io.rs:16-31) with
// one lane per chunk and no side-band index.
//
// The decode of a chunk is a serial chain (tag k+1's position depends on tag
// k), so the parallelism is across chunks: every lane of every wave walks its
// own chunk, one record (or one literal-run word) per hop, and all 64 lanes
// hop together.  Three per-wave LDS structures make that cheap:
//
//   input ring   each lane streams its chunk's packed bytes through a ring of
//                US_RB 16-byte blocks (+1 guard block mirroring block 0, so a
//                record's 16-byte window never wraps).  One aligned 16-byte
//                load per lane and hop, kept US_D hops in flight in registers
//                (the hop loop is unrolled US_D times, so the compiler waits
//                with vmcnt(US_D-1) for exactly the load it commits).  Lanes
//                with nothing to request load a dummy block (one shared line).
//   output ring  each lane writes its decoded words into an 8-word (64-byte)
//                group buffer; complete groups go out through a per-hop flush
//                queue, 8 lanes per group (coalesced 64-byte stores).  Words of
//                zero runs are never written to LDS: the group's written-mask
//                makes the flush store zeros for them, and whole zero groups
//                are stored by the lane directly.
//   chunk table  the wave's chunk offsets (relative 32-bit), loaded once; a
//                lane that finishes takes the next unassigned chunk of the
//                wave (dynamic assignment), and starts requesting its bytes
//                while it still decodes the previous one.
//
// Per hop a lane either decodes one record (tag, its data bytes, and the
// count byte of a 0x00/0xFF record) or one raw word of a literal run, with
// the reference's checks in the reference's order (first error in stream
// order): PrematureEndOfPackedInput when the tag, a data byte or the count is
// missing (:59-74, :109-145); DidNotEndCleanly when a run overruns the output
// (:166-170, :183-187); FailedToFillTheWholeBuffer when a literal run's bytes
// are missing (:195-205 + io.rs:26-28) or the input is empty (read() returns
// 0).  consumed = bytes used on success, the whole chunk on PrematureEnd and
// FailedToFill, 0 on DidNotEndCleanly (where the reference leaves a &[u8]
// reader; the oracle's read_exact, oracle/packed_oracle.c).
#include "common.h"

#ifndef US_D
#define US_D 4  // loads in flight per lane (hops between a load and its commit)
#endif
#ifndef US_RB
#define US_RB 8  // input ring blocks of 16 B per lane (power of two)
#endif
#ifndef US_CPW
#define US_CPW 256  // max chunks per wave range (LDS chunk table)
#endif
#ifndef US_WG
#define US_WG 4  // waves per workgroup (independent; they share the selector table)
#endif

namespace {

constexpr uint32_t kW = CAPNP_WAVE;
constexpr uint32_t kD = US_D;
constexpr uint32_t kRB = US_RB;
constexpr uint32_t kRingBytes = (kRB + 1) * 16;  // + guard block
constexpr uint32_t kMaxC = US_CPW;
constexpr uint32_t kWavesPerWG = US_WG;
static_assert((kRB & (kRB - 1)) == 0 && kRB >= 4, "ring blocks: power of two >= 4");

enum : int32_t { ST_OK = 0, ST_PREMATURE = 2, ST_NOT_CLEAN = 3, ST_FAILED_FILL = 4 };

struct ExpandTable {
    uint64_t s[256];
};
constexpr ExpandTable make_table() {
    ExpandTable t{};
    for (uint32_t tag = 0; tag < 256; tag++) t.s[tag] = expand_selector(tag);
    return t;
}
__device__ constexpr ExpandTable kSel = make_table();

struct alignas(16) WaveLds {
    uint8_t ring[kW][kRingBytes];  // input rings, lane-major
    uint64_t obuf[kW][9];          // output groups (8 words + pad: 72-B lane stride)
    uint2 q[2 * kW];               // flush queue: {group, src | lo | hi | mask}
    uint32_t cin[kMaxC + 1];       // chunk packed starts, bytes from the wave's block 0
    uint32_t cout[kMaxC + 1];      // chunk word starts, words from the wave's first word
};

struct alignas(16) Smem {
    uint64_t sel[256];
    WaveLds w[kWavesPerWG];
};

constexpr uint32_t kNone = 0xFFFFFFFFu;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// flush-queue entry flags: src lane (6 bits), lo (3), hi (4), written mask (8)
__device__ __forceinline__ uint32_t qent(uint32_t src, uint32_t lo, uint32_t hi, uint32_t m) {
    return src | (lo << 6) | (hi << 9) | (m << 13);
}

}  // namespace

// One wave per range of up to kMaxC consecutive chunks: [wave * cpw, ...).
// Requires `out` 16-byte aligned (whole zero groups leave as 16-byte stores).
__global__ void __launch_bounds__(kWavesPerWG * kW)
unpack_stream_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                     uint64_t nchunks, uint32_t cpw, uint64_t* __restrict__ out,
                     const uint64_t* __restrict__ out_off, int32_t* __restrict__ status,
                     uint64_t* __restrict__ consumed) {
    __shared__ Smem sm;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & (kW - 1);
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    for (uint32_t i = tid; i < 256; i += kWavesPerWG * kW) sm.sel[i] = kSel.s[i];
    __syncthreads();

    const uint64_t c_lo = ((uint64_t)blockIdx.x * kWavesPerWG + wave) * cpw;
    if (c_lo >= nchunks) return;
    const uint32_t nc = (uint32_t)((c_lo + cpw < nchunks ? c_lo + cpw : nchunks) - c_lo);
    WaveLds& L = sm.w[wave];

    // wave bases: A0 = the 16-byte block holding the range's first packed
    // byte; W0 = the range's first output word
    const uint64_t B0 = uniform64(in_off[c_lo]);
    const uint64_t W0 = uniform64(out_off[c_lo]);
    // (pointer arithmetic on `in`, not an integer cast, so the loads stay
    // global_load: a flat load would count in lgkmcnt too and force full waits)
    const uint32_t a0 = (uint32_t)(reinterpret_cast<uintptr_t>(in + B0) & 15u);
    const uint8_t* A0 = in + (B0 - a0);  // range start within block 0: a0
    for (uint32_t i = lane; i <= nc; i += kW) {
        L.cin[i] = (uint32_t)(in_off[c_lo + i] - B0) + a0;
        L.cout[i] = (uint32_t)(out_off[c_lo + i] - W0);
    }
    // (ring and group buffers need no clearing: every byte read was written)
    wave_lds_sync();
    if (uniform64(in_off[c_lo + nc]) == B0) {
        // no packed bytes at all (the buffer may even be empty): nothing to
        // load; every chunk with words fails as read() returns 0
        for (uint32_t i = lane; i < nc; i += kW) {
            status[c_lo + i] = L.cout[i + 1] > L.cout[i] ? ST_FAILED_FILL : ST_OK;
            if (consumed) consumed[c_lo + i] = 0;
        }
        return;
    }

    const uint64_t Wg0 = W0 >> 3;             // the wave's first output group
    const uint32_t wg0 = (uint32_t)(W0 & 7);  // W0's offset in it
    uint8_t* const ring = L.ring[lane];
    uint64_t* const obuf = L.obuf[lane];
    const v4u* const blocks = reinterpret_cast<const v4u*>(A0);
    v4u* const outg = reinterpret_cast<v4u*>(out + 8 * Wg0);  // 4 x 16 B per group

    // ---- per-lane state (bytes relative to A0, words relative to W0,
    // groups relative to Wg0)
    // decode chunk dc: position p (from p0, end pe), word w (from w0, end
    // we), literal words left, ring slot bias (seq of block b = b + dsb)
    uint32_t dc = kNone, p = 0, p0 = 0, pe = 0, w = 0, w0 = 0, we = 0, lit = 0, dsb = 0;
    // request chunk rc (the decode chunk, or the next one once the decode
    // chunk's blocks are all requested): next block r, end block rend, bias
    uint32_t rc = kNone, r = 0, rend = 0, rsb = 0;
    uint32_t nreq = 0, ncommit = 0;  // loads issued / committed by this lane
    uint32_t og = 0, omask = 0;      // open output group, its written-word mask
    uint32_t qn = 0;                 // next unassigned chunk (wave-uniform)
    v4u pend[kD];
    uint32_t pslot[kD];
    // (the pipeline starts full of dummy loads, issued in hop order, so the
    // loop is entered with the same vmcnt picture it has on its back edge and
    // every commit waits with vmcnt(kD - 1))
#pragma unroll
    for (uint32_t k = 0; k < kD; k++) {
        uint32_t i0 = 0;
        asm volatile("" : "+v"(i0));  // (kD distinct loads, not one)
        pend[k] = blocks[i0];
        pslot[k] = kNone;
    }

    for (;;) {
#pragma unroll
        for (uint32_t k = 0; k < kD; k++) {
            // ---- 1. commit the load issued kD hops ago
            if (pslot[k] != kNone) {
                *reinterpret_cast<v4u*>(ring + 16 * pslot[k]) = pend[k];
                if (pslot[k] == 0) *reinterpret_cast<v4u*>(ring + 16 * kRB) = pend[k];
                ncommit++;
            }

            // ---- 1b. request the next block (or a dummy block) into the register
            // set just committed (so it is never free for other values)
            {
                const bool room = dc == kNone || (int32_t)(nreq - ((p >> 4) + dsb)) < (int32_t)kRB;
                const bool issue = rc != kNone && r < rend && room;
                uint32_t bi = issue ? r : 0u;
                asm volatile("" : "+v"(bi));  // (one unconditional load, not two)
                pend[k] = blocks[bi];
                pslot[k] = issue ? (nreq & (kRB - 1)) : kNone;
                if (issue) {
                    nreq++;
                    r++;
                }
            }

            // ---- 2. decode one record / literal-run word
            bool e1v = false, e2v = false;  // flush entries of this hop
            uint32_t e1g = 0, e1 = 0, e2g = 0, e2 = 0;
            if (dc != kNone) {
                const uint32_t last = p + 9 < pe ? p + 9 : (pe > p ? pe - 1 : p);
                const bool ready = p >= pe || (int32_t)(ncommit - ((last >> 4) + dsb)) > 0;
                if (ready) {
                    int32_t st = ST_OK;
                    uint64_t word = 0;
                    uint32_t nw = 1;
                    if (p < pe) {
                        const uint32_t x = (((p >> 4) + dsb) & (kRB - 1)) * 16 + (p & 15);
                        const uint32_t* rd = reinterpret_cast<const uint32_t*>(ring + (x & ~3u));
                        const uint32_t d0 = rd[0], d1 = rd[1], d2 = rd[2], d3 = rd[3];
                        const uint32_t b0 = __builtin_amdgcn_alignbyte(d1, d0, x);
                        const uint32_t b1 = __builtin_amdgcn_alignbyte(d2, d1, x);
                        const uint32_t b2 = __builtin_amdgcn_alignbyte(d3, d2, x);
                        if (lit) {  // raw word of a literal run (bytes checked at its head)
                            word = ((uint64_t)b1 << 32) | b0;
                            p += 8;
                            lit--;
                        } else {
                            const uint32_t tag = b0 & 0xFFu;
                            const uint32_t lo = __builtin_amdgcn_alignbyte(b1, b0, 1);
                            const uint32_t hi = __builtin_amdgcn_alignbyte(b2, b1, 1);
                            const uint64_t sv = sm.sel[tag];
                            word = ((uint64_t)__builtin_amdgcn_perm(hi, lo, (uint32_t)(sv >> 32))
                                    << 32) |
                                   __builtin_amdgcn_perm(hi, lo, (uint32_t)sv);
                            const bool isz = tag == 0, isf = tag == 0xFFu;
                            const uint32_t q = p + 1 + __builtin_popcount(tag);
                            const uint32_t cnt =
                                isz ? ((b0 >> 8) & 0xFFu) : (isf ? ((b2 >> 8) & 0xFFu) : 0u);
                            const uint32_t end = q + ((isz || isf) ? 1u : 0u);
                            if (q > pe || ((isz || isf) && q >= pe)) st = ST_PREMATURE;
                            else if (cnt > we - w - 1) st = ST_NOT_CLEAN;
                            else if (isf && pe - end < 8 * cnt) st = ST_FAILED_FILL;
                            p = end;
                            nw = 1 + (isz ? cnt : 0u);
                            lit = isf ? cnt : 0u;
                        }
                    } else {
                        st = p0 == pe ? ST_FAILED_FILL : ST_PREMATURE;  // empty input: read() = 0
                    }
                    const uint32_t lo0 = og == ((w0 + wg0) >> 3) ? ((w0 + wg0) & 7) : 0u;
                    bool fin;
                    if (st == ST_OK) {
                        const uint32_t ws = (w + wg0) & 7;
                        obuf[ws] = word;
                        omask |= 1u << ws;
                        w += nw;
                        const uint32_t gn = (w + wg0) >> 3;
                        if (gn != og) {  // the open group is complete
                            e1v = true;
                            e1g = og;
                            e1 = qent(lane, lo0, 8, omask);
                            // whole groups inside a zero run: zeros, stored directly
                            for (uint32_t g = og + 1; g < gn; g++) {
                                v4u* o = outg + 4 * (uint64_t)g;
                                const v4u z = {0u, 0u, 0u, 0u};
                                o[0] = z;
                                o[1] = z;
                                o[2] = z;
                                o[3] = z;
                            }
                            og = gn;
                            omask = 0;
                        }
                        fin = w == we;
                    } else {
                        fin = true;
                    }
                    if (fin) {
                        // the last (partial) group: words produced in it
                        const uint32_t lo2 = og == ((w0 + wg0) >> 3) ? ((w0 + wg0) & 7) : 0u;
                        const uint32_t hi2 = (w + wg0) - 8 * og;
                        if (hi2 > lo2) {
                            e2v = true;
                            e2g = og;
                            e2 = qent(lane, lo2, hi2, omask);
                        }
                        const uint64_t c = c_lo + dc;
                        status[c] = st;
                        if (consumed)
                            consumed[c] = st == ST_OK ? p - p0 : (st == ST_NOT_CLEAN ? 0u : pe - p0);
                        if (rc == dc) rc = kNone;  // stop requesting its bytes
                        dc = kNone;
                    }
                }
            }

            // ---- 3. flush complete / final groups (8 lanes per group)
            {
                const uint64_t m1 = ballot64(e1v), m2 = ballot64(e2v);
                if (m1 | m2) {
                    const uint32_t n1 = popc64(m1);
                    const uint32_t nent = n1 + popc64(m2);
                    if (e1v) L.q[mask_rank(m1)] = make_uint2(e1g, e1);
                    if (e2v) L.q[n1 + mask_rank(m2)] = make_uint2(e2g, e2);
                    const uint32_t kk = lane & 7;
                    for (uint32_t b = 0; b < nent; b += 8) {
                        const uint32_t j = b + (lane >> 3);
                        const uint2 e = L.q[j < nent ? j : 0u];
                        const uint32_t src = e.y & 63u, lo = (e.y >> 6) & 7u, hi = (e.y >> 9) & 15u;
                        const uint32_t msk = e.y >> 13;
                        const uint64_t v = L.obuf[src][kk];
                        if (j < nent && kk >= lo && kk < hi)
                            out[8 * (Wg0 + e.x) + kk] = ((msk >> kk) & 1u) ? v : 0ull;
                    }
                }
            }

            // ---- 4. assignment: lanes whose request side is free take the
            // wave's next chunks (empty chunks finish at once)
            for (;;) {
                const bool want = rc == kNone || (rc == dc && r == rend);
                const uint64_t m = ballot64(want);
                if (m == 0 || qn >= nc) break;
                const uint32_t c = qn + mask_rank(m);
                qn = qn + popc64(m) < nc ? qn + popc64(m) : nc;
                if (want && c < nc) {
                    const uint32_t ci = L.cin[c], ce = L.cin[c + 1];
                    const uint32_t wi = L.cout[c], wz = L.cout[c + 1];
                    if (wz == wi) {  // nothing to read: Ok (read of 0 bytes)
                        status[c_lo + c] = ST_OK;
                        if (consumed) consumed[c_lo + c] = 0;
                    } else {
                        rc = c;
                        r = ci >> 4;
                        rend = (ce + 15) >> 4;
                        rsb = nreq - r;
                        if (dc == kNone) {  // idle lane: decode it next
                            dc = c;
                            p = p0 = ci;
                            pe = ce;
                            w = w0 = wi;
                            we = wz;
                            lit = 0;
                            dsb = rsb;
                            og = (wi + wg0) >> 3;
                            omask = 0;
                        }
                    }
                }
            }
            // a lane whose decode chunk finished picks up its request chunk
            if (dc == kNone && rc != kNone) {
                dc = rc;
                p = p0 = L.cin[rc];
                pe = L.cin[rc + 1];
                w = w0 = L.cout[rc];
                we = L.cout[rc + 1];
                lit = 0;
                dsb = rsb;
                og = (w + wg0) >> 3;
                omask = 0;
            }

        }
        // ---- 5. done when no lane has work and no chunk is left (checked once
        // per kD hops: an exit inside the unrolled hops would give the waitcnt
        // pass a path to the loop header that skips loads, and it would then
        // drain the pipeline with vmcnt(0..kD-2) at the first hops)
        if (ballot64(dc != kNone || rc != kNone) == 0 && qn >= nc) break;
    }
}

extern "C" hipError_t capnp_launch_unpack_stream(const uint8_t* d_in, const uint64_t* d_in_off,
                                                 uint64_t nchunks, uint32_t cpw, uint64_t* d_out,
                                                 const uint64_t* d_out_off, int32_t* d_status,
                                                 uint64_t* d_consumed, hipStream_t stream) {
    if (nchunks == 0) return hipSuccess;
    if (cpw == 0) cpw = kMaxC;
    if (cpw > kMaxC) cpw = kMaxC;
    if (reinterpret_cast<uintptr_t>(d_out) & 15u) return hipErrorInvalidValue;
    const uint64_t waves = (nchunks + cpw - 1) / cpw;
    const uint64_t blocks = (waves + kWavesPerWG - 1) / kWavesPerWG;
    hipLaunchKernelGGL(unpack_stream_kernel, dim3((uint32_t)blocks), dim3(kWavesPerWG * kW), 0,
                       stream, d_in, d_in_off, nchunks, cpw, d_out, d_out_off, d_status,
                       d_consumed);
    return hipGetLastError();
}

extern "C" uint32_t capnp_unpack_stream_chunks_per_wave(void) { return kMaxC; }
