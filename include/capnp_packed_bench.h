/*
 * capnp_packed_bench.h — workload helpers exported by the same library for
 * the benchmark and the parity tests (not part of the codec boundary).
 */
#ifndef CAPNP_PACKED_BENCH_H
#define CAPNP_PACKED_BENCH_H

#include <stddef.h>
#include <stdint.h>

#include "capnp_packed.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fills d_words[d_offs[c] .. d_offs[c+1]) for c < nchunks with the synthetic
 * workload of oracle/gen_oracle.c (bit-identical): chunk id = id0 + c,
 * generator kind = d_kinds[c] (or kind0 when d_kinds is NULL; 0 iid, 1 long
 * zero runs, 2 long literal runs), pz_thresh = P(zero word) * 2^32. */
capnp_status capnp_gpu_gen_batch(capnp_ctx* ctx, uint64_t* d_words, const uint64_t* d_offs,
                                 size_t nchunks, uint64_t id0, const uint8_t* d_kinds,
                                 uint32_t kind0, uint32_t pz_thresh, void* stream);

/* Fills d_words[0 .. total_words) with the carsales request stream of the
 * reference benchmark (BASELINE.json configs[0]; benchmark/carsales.rs:84-150
 * on benchmark/common.rs:22-70's FastRand from its default seed, one
 * generator for the whole run): the single segments of requests
 * skip_requests, skip_requests + 1, ... back to back, the last one cut at
 * total_words.  Bit-identical to oracle/carsales_oracle.c's carsales_stream.
 * *nreq = requests started; h_req_off (optional, host, nreq + 1 entries) =
 * each request's first word, then the end of the last one in full.  The
 * chain is walked on the host (serial by construction); the words are
 * written on the device, then the call synchronises `stream`. */
capnp_status capnp_gpu_gen_carsales(capnp_ctx* ctx, uint64_t* d_words, uint64_t total_words,
                                    uint64_t skip_requests, uint64_t* h_req_off,
                                    size_t max_req, size_t* nreq, void* stream);

/* (The explicit-tile-size batch calls, capnp_gpu_*_tuned, are declared in
 * capnp_packed.h: they are the stream-ordered variants of the boundary.) */

/* Output words per wave sub-tile of the record-sync-index unpack (the
 * chunks_per_tile of the _sync_ calls ~ this / mean chunk words). */
uint32_t capnp_unpack_sync_tile_words(void);

/* Output words per unpack tile the staged path is sized for. */
uint32_t capnp_unpack_tile_words(void);

/* Words per pack tile the staged path is sized for (4 waves x steps of 64
 * words); chunks_per_tile ~ this / mean chunk words. */
uint32_t capnp_pack_tile_words(void);

/* Diagnostics of the last capnp_gpu_unpack_batch_resync on ctx: fix passes
 * run; serial = 1 if the batch went to the serial batch unpack (fix passes
 * did not converge), 2 if its chunks were short enough to go there directly,
 * 3 if only the chunks that failed their check were decoded serially. */
capnp_status capnp_resync_stats(capnp_ctx* ctx, int* passes, int* serial);

/* Packed bytes per lane of the index-free decode. */
uint32_t capnp_resync_block_bytes(void);

/* Diagnostic: caps the rounds a tile of the index-free decode's resolution
 * may run before it gives up to the serial fallbacks (process-wide; 1 .. 258,
 * 0 restores the default 258, which the rounds' termination bound never
 * reaches; the name predates the round-4 look-back, which replaced the fix
 * passes).  Returns the previous cap (0 = default).  Lets the tests drive the
 * fallback paths (capnp_gpu_unpack_batch_resync's per-chunk serial decode,
 * the stream reader's serial whole-record cut) without adversarial input. */
int capnp_resync_max_passes(int passes);

/* Pre-sizes the context workspace for batches of up to max_chunks chunks so
 * that later calls allocate nothing (required before HIP graph capture). */
capnp_status capnp_ctx_reserve(capnp_ctx* ctx, size_t max_chunks);

#ifdef __cplusplus
}
#endif
#endif /* CAPNP_PACKED_BENCH_H */
