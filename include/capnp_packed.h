/*
 * capnp_packed.h — C ABI of the MI355X-native Cap'n Proto packed-stream codec.
 *
 * This is the drop-in boundary that replaces the bodies of the packed codec in
 * capnproto-rust (capnp 0.27.0).  Every entry point below names the reference
 * item it stands in for (paths relative to the capnproto-rust checkout):
 *
 *   PackedWrite::write_all      capnp/src/serialize_packed.rs:300-440
 *   PackedRead::read            capnp/src/serialize_packed.rs:76-229
 *   serialize_packed::write_message          serialize_packed.rs:446-453
 *   serialize_packed::read_message           serialize_packed.rs:233-242
 *   serialize_packed::try_read_message       serialize_packed.rs:246-255
 *   serialize_packed::read_message_no_alloc  serialize_packed.rs:263-273
 *   serialize_packed::try_read_message_no_alloc serialize_packed.rs:281-291
 *
 * Conventions
 *   - Plain pointers and sizes only; no HIP or torch types.  `stream` is a
 *     hipStream_t passed as void* (NULL = the HIP null stream; the context's
 *     own stream is returned by capnp_ctx_stream).
 *   - All buffers are caller-owned.  The library never frees caller memory.
 *   - Functions prefixed capnp_gpu_* take DEVICE pointers and enqueue their
 *     kernels on `stream`.  Those that size their launch from device data
 *     say so ("Synchronises"): they copy a few bytes back and wait for
 *     `stream` before returning, so they must not be captured into a
 *     hipGraph.  capnp_gpu_pack_batch, capnp_gpu_unpack_batch and their _sync
 *     forms do that (they read the batch's word range to pick the tiling);
 *     their _tuned forms with chunks_per_tile != 0 are fully asynchronous
 *     (stream ordered, capture-safe, no host wait).  All other functions take
 *     HOST pointers and are blocking; they stage through pinned memory and
 *     run the same HIP kernels.
 *   - There is no CPU implementation of the transform in this library: if no
 *     gfx950 device is present, capnp_ctx_create fails with CAPNP_E_NO_DEVICE.
 *   - Status codes map 1:1 onto capnp::ErrorKind (capnp/src/lib.rs:211-426).
 */
#ifndef CAPNP_PACKED_H
#define CAPNP_PACKED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum capnp_status {
    CAPNP_OK = 0,
    /* try_read_message* hit a clean EOF on a message boundary: Ok(None)
       (serialize.rs:458-461). */
    CAPNP_NONE = 1,
    /* ErrorKind::PrematureEndOfPackedInput (lib.rs:394). */
    CAPNP_E_PREMATURE_END_OF_PACKED_INPUT = 2,
    /* ErrorKind::PackedInputDidNotEndCleanlyOnASegmentBoundary (lib.rs:388). */
    CAPNP_E_DID_NOT_END_CLEANLY = 3,
    /* ErrorKind::FailedToFillTheWholeBuffer (lib.rs:271, io.rs:26-28). */
    CAPNP_E_FAILED_TO_FILL_WHOLE_BUFFER = 4,
    /* ErrorKind::PrematureEndOfFile (lib.rs:391). */
    CAPNP_E_PREMATURE_END_OF_FILE = 5,
    /* ErrorKind::InvalidNumberOfSegments (lib.rs:310). */
    CAPNP_E_INVALID_NUMBER_OF_SEGMENTS = 6,
    /* ErrorKind::MessageSizeOverflow (lib.rs:373). */
    CAPNP_E_MESSAGE_SIZE_OVERFLOW = 7,
    /* ErrorKind::MessageTooLarge (lib.rs:376). */
    CAPNP_E_MESSAGE_TOO_LARGE = 8,
    /* ErrorKind::BufferNotLargeEnough (lib.rs:232). */
    CAPNP_E_BUFFER_NOT_LARGE_ENOUGH = 9,
    /* ErrorKind::UnalignedSegment (lib.rs:419). */
    CAPNP_E_UNALIGNED_SEGMENT = 10,
    /* Replaces the panic "PackedRead reads must be word-aligned."
       (serialize_packed.rs:86) and non-word-multiple write_all input. */
    CAPNP_E_MISALIGNED_LEN = 11,
    /* ErrorKind::MessageEndsPrematurely (lib.rs:361): a flat slice shorter
       than its segment table claims (serialize.rs:66-70,
       no_alloc_buffer_segments.rs:253-258, :84-89). */
    CAPNP_E_MESSAGE_ENDS_PREMATURELY = 12,
    /* ErrorKind::EmptySlice (lib.rs:247): read_message_from_flat_slice on an
       empty slice (serialize.rs:60-62). */
    CAPNP_E_EMPTY_SLICE = 13,
    /* ErrorKind::MessageNotAlignedBy8BytesBoundary (lib.rs:370): the no-alloc
       flat reader's alignment check (no_alloc_buffer_segments.rs:234-248). */
    CAPNP_E_NOT_ALIGNED = 14,
    /* The inner stream of a streaming adaptor has nothing now: Poll::Pending
       (capnp-futures); call again. */
    CAPNP_PENDING = 15,
    /* Library-level errors (no counterpart in the reference). */
    CAPNP_E_INVALID_ARGUMENT = 64,
    CAPNP_E_NO_DEVICE = 65,
    CAPNP_E_HIP = 66,
    CAPNP_E_OUT_OF_MEMORY = 67,
    /* The inner stream of a streaming adaptor reported an I/O error (an
       io::Error, lib.rs:481-499) or took no bytes. */
    CAPNP_E_IO = 68
} capnp_status;

/* Mirror of capnp::message::ReaderOptions (message.rs:85-120).  Only the
   traversal limit is consulted by the framing reader (serialize.rs:501-507). */
typedef struct capnp_reader_options {
    uint64_t traversal_limit_in_words; /* default 8 Mi words (message.rs:117) */
    int32_t has_traversal_limit;       /* 0 => None (no limit)               */
    int32_t nesting_limit;             /* carried, not used by the codec      */
} capnp_reader_options;

/* Limit on segments per message (serialize.rs:39). */
#define CAPNP_SEGMENTS_COUNT_LIMIT 512u

typedef struct capnp_ctx capnp_ctx;

/* ---- context ----------------------------------------------------------- */
/* Creates a context bound to HIP device `device` (its own stream, workspace
   and pinned staging).  Returns NULL and sets *status on failure. */
capnp_ctx* capnp_ctx_create(int device, capnp_status* status);
void capnp_ctx_destroy(capnp_ctx* ctx);
/* hipStream_t owned by the context (as void*). */
void* capnp_ctx_stream(capnp_ctx* ctx);
/* Text of the last HIP error seen by this context ("" if none). */
const char* capnp_ctx_last_error(capnp_ctx* ctx);
/* Library / ABI version and the gfx target the kernels were built for. */
const char* capnp_version(void);
/* The ABI revision this header describes.  It changes whenever an exported
   signature changes in place (round 3 inserted buf_len into
   capnp_gpu_read_flat_messages under the same name); a binding checks
   capnp_abi_version() == CAPNP_ABI_VERSION once, before any other call. */
#define CAPNP_ABI_VERSION 6u
uint32_t capnp_abi_version(void);
/* Default ReaderOptions (message.rs:117-120). */
capnp_reader_options capnp_default_reader_options(void);

/* ---- sizes ------------------------------------------------------------- */
/* Upper bound on PACK output for a chunk of `words` words:
   8n + ceil(n/2) + 2 bytes (0 for n == 0). */
size_t capnp_packed_bound_bytes(size_t words);
/* Bound for a batch: sum of per-chunk bounds given the total words and the
   chunk count. */
size_t capnp_packed_batch_bound_bytes(size_t total_words, size_t nchunks);

/* ---- device batch API (the hot path) ----------------------------------- */
/* PACK every chunk c = words [d_chunk_word_off[c], d_chunk_word_off[c+1]) of
   d_words exactly as one PackedWrite::write_all call would
   (serialize_packed.rs:304-439), and concatenate the results in chunk order
   into d_out.  On completion d_out_byte_off[c] is chunk c's start in d_out
   and d_out_byte_off[nchunks] the total packed size.  If the total exceeds
   out_cap nothing at or past out_cap is written (the chunk that straddles
   out_cap may be partially written) and the total still reports the size
   that was needed (caller checks after the stream syncs).
   d_chunk_word_off: nchunks+1 non-decreasing word offsets, checked on the
   device first (CAPNP_E_INVALID_ARGUMENT, nothing launched, if one
   decreases).  Synchronises `stream` once (the check, and d_chunk_word_off[0]
   and [nchunks] to choose chunk tiles or word tiles);
   capnp_gpu_pack_batch_tuned below does neither. */
capnp_status capnp_gpu_pack_batch(capnp_ctx* ctx, const uint64_t* d_words,
                                  const uint64_t* d_chunk_word_off, size_t nchunks,
                                  uint8_t* d_out, size_t out_cap,
                                  uint64_t* d_out_byte_off, void* stream);

/* UNPACK every chunk c: decode packed bytes d_packed[d_in_byte_off[c] ..
   d_in_byte_off[c+1]) into words d_words[d_out_word_off[c] ..
   d_out_word_off[c+1]) exactly as one PackedRead::read_exact call of that
   many bytes would (serialize_packed.rs:80-228, io.rs:16-31).
   d_status[c] receives the capnp_status of the chunk; d_consumed[c] (may be
   NULL) the packed bytes the decode used.  Bytes of d_words that belong to a
   chunk with a non-OK status are unspecified.
   d_in_byte_off and d_out_word_off (nchunks+1 entries each) must be
   non-decreasing: checked on the device first (CAPNP_E_INVALID_ARGUMENT,
   nothing launched, otherwise).  Synchronises `stream` once (the check, and
   d_out_word_off[0] and [nchunks] to size the launch); a batch whose mean
   chunk is >= 512 words then takes the index-free block decode of
   capnp_gpu_unpack_batch_resync (one more synchronisation, before its
   decode), which spreads each unit over the whole chip -- except a batch of
   >= 256 units of 2048-32767 words on average, which fills the chip with one
   workgroup per unit.  The decode itself is only enqueued: d_words, d_status and
   d_consumed are ordered on `stream` (read them after a synchronisation of
   `stream`, or from work queued on it) -- never with a plain hipMemcpy or
   from another stream without an event.
   capnp_gpu_unpack_batch_tuned below does neither synchronisation. */
capnp_status capnp_gpu_unpack_batch(capnp_ctx* ctx, const uint8_t* d_packed,
                                    const uint64_t* d_in_byte_off, size_t nchunks,
                                    uint64_t* d_words, const uint64_t* d_out_word_off,
                                    int32_t* d_status, uint64_t* d_consumed,
                                    void* stream);

/* ---- record sync index (optional side-band of the device batch API) ---- */
/* The batch pack can also emit a record sync index: one uint32 entry per
   word index m = CAPNP_SYNC_WORDS * k of the batch's word space
   (k < ceil(total_words / CAPNP_SYNC_WORDS)).
   Entry k describes the chunk c that holds word m: bits 0-23 are the
   chunk-relative packed offset of the record (tag) that covers word m,
   bits 24-31 m minus that record's first word (a run covers at most 255
   words after its head).  0xFFFFFFFF = not provided (chunks packed by the
   streaming path, i.e. larger than the staged tile).  The packed bytes are
   unchanged: the index is metadata, like d_out_byte_off.
   An unpack given the index (with the same word offsets as the pack, as
   d_out_word_off) decodes CAPNP_SYNC_WORDS-word segments in parallel and checks
   that consecutive segments meet exactly; any mismatch (a corrupt or
   foreign index) falls back to the serial walk for that chunk, so results
   and statuses are always those of capnp_gpu_unpack_batch. */
#ifndef CAPNP_SYNC_WORDS /* (overridable for diagnostic builds only) */
#define CAPNP_SYNC_WORDS 8
#endif
size_t capnp_sync_index_entries(size_t total_words);
capnp_status capnp_gpu_pack_batch_sync(capnp_ctx* ctx, const uint64_t* d_words,
                                       const uint64_t* d_chunk_word_off, size_t nchunks,
                                       uint8_t* d_out, size_t out_cap, uint64_t* d_out_byte_off,
                                       uint32_t* d_sync, void* stream);
capnp_status capnp_gpu_unpack_batch_sync(capnp_ctx* ctx, const uint8_t* d_packed,
                                         const uint64_t* d_in_byte_off, size_t nchunks,
                                         uint64_t* d_words, const uint64_t* d_out_word_off,
                                         const uint32_t* d_sync, int32_t* d_status,
                                         uint64_t* d_consumed, void* stream);

/* Stream-ordered forms: the same calls with an explicit tile size and no
   host synchronisation (capture-safe).  Pack: chunks per 256-thread
   workgroup, 1..64, about capnp_pack_tile_words() / mean chunk words, for
   batches whose chunks fit a tile's staged steps (longer chunks are packed by
   the slower in-kernel streaming path; chunks_per_tile 0 = choose, which
   synchronises).  Unpack: 1..256 chunks per workgroup; a tile takes the
   LDS-staged path when it has <= 64 chunks, <= capnp_unpack_tile_words()
   output words and <= 4.5x that many packed bytes.  The offset arrays are
   not validated by these forms: the caller guarantees them non-decreasing
   (a decreasing offset is a chunk of negative length, read or written out
   of bounds). */
capnp_status capnp_gpu_pack_batch_tuned(capnp_ctx* ctx, const uint64_t* d_words,
                                        const uint64_t* d_chunk_word_off, size_t nchunks,
                                        uint8_t* d_out, size_t out_cap,
                                        uint64_t* d_out_byte_off, uint32_t chunks_per_tile,
                                        void* stream);

capnp_status capnp_gpu_unpack_batch_tuned(capnp_ctx* ctx, const uint8_t* d_packed,
                                          const uint64_t* d_in_byte_off, size_t nchunks,
                                          uint64_t* d_words, const uint64_t* d_out_word_off,
                                          int32_t* d_status, uint64_t* d_consumed,
                                          uint32_t chunks_per_tile, void* stream);

/* The record-sync-index batch calls with an explicit tile size. */
capnp_status capnp_gpu_pack_batch_sync_tuned(capnp_ctx* ctx, const uint64_t* d_words,
                                             const uint64_t* d_chunk_word_off, size_t nchunks,
                                             uint8_t* d_out, size_t out_cap,
                                             uint64_t* d_out_byte_off, uint32_t* d_sync,
                                             uint32_t chunks_per_tile, void* stream);
capnp_status capnp_gpu_unpack_batch_sync_tuned(capnp_ctx* ctx, const uint8_t* d_packed,
                                               const uint64_t* d_in_byte_off, size_t nchunks,
                                               uint64_t* d_words, const uint64_t* d_out_word_off,
                                               const uint32_t* d_sync, int32_t* d_status,
                                               uint64_t* d_consumed, uint32_t chunks_per_tile,
                                               void* stream);


/* ---- index-free decode of long read units ---------- */
/* The same transform, statuses and consumed counts as capnp_gpu_unpack_batch
   (PackedRead::read under read_exact, serialize_packed.rs:76-229, io.rs:16-31)
   for batches that carry no record sync index and whose chunks may be of any
   length (a foreign stream: a 64 KiB segment, or a whole message body read
   as one unit by read_message, serialize.rs:514-524).  Each chunk's packed
   bytes are split into fixed blocks decoded in parallel: a block's tag chain
   is walked speculatively from its first byte and resynchronised against
   its predecessor's exit (csrc/resync.hip).  A chunk whose chain does not
   end exactly at its packed end with exactly its word count is decoded
   serially on its own (in the same launch as the resolved blocks), so its
   status, consumed count and partial output are exactly what
   capnp_gpu_unpack_batch gives it.  The offset arrays are checked first as
   for capnp_gpu_unpack_batch: that check synchronises `stream` once, before
   any decode work.  The decode is then enqueued on `stream` and the call
   returns without waiting for it (so documented from ABI 5; the ABI-4 header
   said it waited): the results are
   ordered on `stream` only.  A later resync call on the same context but
   another stream waits for this one's kernels by an event (they share the
   context's workspace); capnp_resync_stats synchronises `stream`. */
capnp_status capnp_gpu_unpack_batch_resync(capnp_ctx* ctx, const uint8_t* d_packed,
                                           const uint64_t* d_in_byte_off, size_t nchunks,
                                           uint64_t* d_words, const uint64_t* d_out_word_off,
                                           int32_t* d_status, uint64_t* d_consumed,
                                           void* stream);

/* ---- host single-unit API (blocking; runs the same kernels) ------------ */
/* PackedWrite::write_all of one chunk (serialize_packed.rs:304-439) into a
   caller buffer; *written = packed length.  len must be a multiple of 8. */
capnp_status capnp_pack(capnp_ctx* ctx, const uint8_t* in, size_t len,
                        uint8_t* out, size_t cap, size_t* written);
/* PackedRead::read_exact of out_len bytes from a slice of in_len bytes
   (serialize_packed.rs:80-228 with io.rs:16-31); *consumed = bytes used. */
capnp_status capnp_unpack(capnp_ctx* ctx, const uint8_t* in, size_t in_len,
                          size_t* consumed, uint8_t* out, size_t out_len);

/* The longest prefix of whole records of the packed bytes in[0, in_len)
   that decodes to at most max_words words: *bytes its length, *words the
   words it decodes to, written to out (host, max_words words; NULL: the
   lengths only).  The primitive of a streaming read over a BufRead: a
   reader keeps only the incomplete record past *bytes when it must pull the
   next input buffer, instead of the whole unit seen so far (the records
   before it are final: PackedRead::read decodes left to right and consumes
   a buffer before refilling, serialize_packed.rs:59-74, :100-226).  Tags
   are not validated beyond their record lengths: the exact status comes
   from capnp_unpack. */
capnp_status capnp_unpack_prefix(capnp_ctx* ctx, const uint8_t* in, size_t in_len,
                                 uint64_t max_words, uint64_t* out, size_t* bytes,
                                 uint64_t* words);

/* ---- host batch API (end-to-end: pinned H2D -> kernel -> D2H) ---------- */
capnp_status capnp_pack_batch_host(capnp_ctx* ctx, const uint64_t* words,
                                   const uint64_t* chunk_word_off, size_t nchunks,
                                   uint8_t* out, size_t out_cap, uint64_t* out_byte_off);
capnp_status capnp_unpack_batch_host(capnp_ctx* ctx, const uint8_t* packed,
                                     const uint64_t* in_byte_off, size_t nchunks,
                                     uint64_t* words, const uint64_t* out_word_off,
                                     int32_t* status, uint64_t* consumed);

/* ---- streaming host batch API ----------------------- */
/* The same transforms and results as capnp_pack_batch_host /
   capnp_unpack_batch_host, pipelined over slices of about slice_words words
   (0 = 4 Mi words): the copy in of slice i+1, the kernel on slice i and the
   copy out of slice i-1 run concurrently on three streams with
   double-buffered device staging, so a host-to-host batch moves at the PCIe
   rate instead of the sum of the three phases.  This is the device side of
   the async PackedRead/PackedWrite adaptors
   (capnp-futures/src/serialize_packed.rs:83-226, 330-521) for whole batches.
   Host buffers should be pinned (hipHostMalloc / hipHostRegister) for the
   copies to overlap.  Blocking: returns when every byte has landed.
   Pack: out_byte_off (host, nchunks+1) receives the exclusive scan of packed
   sizes; CAPNP_E_BUFFER_NOT_LARGE_ENOUGH if the total exceeds out_cap
   (nothing at or past out_cap is written).  Unpack: per-chunk status and
   consumed (may be NULL) as capnp_unpack_batch_host. */
capnp_status capnp_stream_pack_batch(capnp_ctx* ctx, const uint64_t* words,
                                     const uint64_t* chunk_word_off, size_t nchunks,
                                     uint8_t* out, size_t out_cap, uint64_t* out_byte_off,
                                     size_t slice_words);
capnp_status capnp_stream_unpack_batch(capnp_ctx* ctx, const uint8_t* packed,
                                       const uint64_t* in_byte_off, size_t nchunks,
                                       uint64_t* words, const uint64_t* out_word_off,
                                       int32_t* status, uint64_t* consumed, size_t slice_words);

/* ---- device batch message framing ------------------ */
/* serialize_packed::write_message for nmsg messages at once
   (serialize_packed.rs:446-453 -> serialize.rs:574-679).  Message m owns
   segments [d_msg_seg_off[m], d_msg_seg_off[m+1]) (at least one), segment s
   is words [d_seg_word_off[s], d_seg_word_off[s+1]) of d_words, and a
   message's segments are consecutive in d_words.  The packed messages go
   back to back into d_out, message m at d_msg_byte_off[m] (nmsg+1 entries,
   the last is the total): each is exactly the byte stream write_message
   produces (the segment table's word 0, the rest of the table, then every
   segment, each packed by its own write_all).  total_segs is the batch's
   segment count and total_words the words d_words holds (host-side sizes):
   every d_seg_word_off entry must lie in [0, total_words].  The
   segments are packed in place with a gap before each message's first
   segment that then receives the packed table; a batch whose message offsets
   do not span [0, total_segs) goes through a staging copy instead.
   d_msg_seg_off must be non-decreasing and end at or before total_segs, and
   d_seg_word_off non-decreasing and end at or before total_words: checked
   on the device first, before any segment word is read
   (CAPNP_E_INVALID_ARGUMENT otherwise).  Synchronises the stream twice (the
   check; then to choose the path, or to size the staging pack); out_cap as
   in capnp_gpu_pack_batch. */
capnp_status capnp_gpu_write_messages(capnp_ctx* ctx, const uint64_t* d_words,
                                      const uint64_t* d_seg_word_off,
                                      const uint64_t* d_msg_seg_off, size_t nmsg,
                                      size_t total_segs, size_t total_words, uint8_t* d_out,
                                      size_t out_cap, uint64_t* d_msg_byte_off, void* stream);

/* serialize_packed::read_message / try_read_message (serialize_packed.rs:
   233-255 -> serialize.rs:287-325, 448-524) for nmsg messages at once, the
   messages delimited by a side-band byte index: message m is packed bytes
   [d_msg_byte_off[m], d_msg_byte_off[m+1]) of d_packed (as
   capnp_gpu_write_messages writes it).  Per message: the table's read units
   (8 bytes, then the rest of the table as one unit) with the reference's
   checks (segment count, traversal limit of opts, NULL = defaults;
   try_mode: an empty message yields CAPNP_NONE), then the body as one
   read_exact.  Outputs (device): the bodies back to back in d_words
   (message m's segments at words [d_msg_word_off[m], d_msg_word_off[m+1]),
   nmsg+1 entries), the segment lengths in d_seg_words (message m's at
   [d_msg_seg_off[m], d_msg_seg_off[m+1])), d_status[m] and d_consumed[m]
   (may be NULL; packed bytes the message used).  A message whose table
   fails gets no words and no segments.  d_msg_byte_off must be
   non-decreasing: checked on the device first (CAPNP_E_INVALID_ARGUMENT).
   Synchronises the stream twice (the check; the totals are checked against
   words_cap and segs_cap: CAPNP_E_BUFFER_NOT_LARGE_ENOUGH, with only the
   offset arrays written). */
capnp_status capnp_gpu_read_messages(capnp_ctx* ctx, const uint8_t* d_packed,
                                     const uint64_t* d_msg_byte_off, size_t nmsg,
                                     const capnp_reader_options* opts, int try_mode,
                                     uint64_t* d_words, size_t words_cap,
                                     uint64_t* d_msg_word_off, uint64_t* d_seg_words,
                                     size_t segs_cap, uint64_t* d_msg_seg_off,
                                     int32_t* d_status, uint64_t* d_consumed, void* stream);

/* Unpacked flat-slice framing for nmsg messages at once:
   serialize::read_message_from_flat_slice (serialize.rs:53-78) when
   no_alloc == 0, read_message_from_flat_slice_no_alloc /
   NoAllocSliceSegments::from_slice (serialize.rs:88-96,
   no_alloc_buffer_segments.rs:22-92, :152-162) when no_alloc != 0.  Message
   m is read from the slice d_buf[d_slice_off[m] .. d_slice_off[m+1]) (the
   slice may extend past the message, as in the reference).  Zero copy:
   nothing is moved, only the framing is validated and described.  Outputs
   (device): d_status[m]; d_body_off[m] the byte offset in d_buf of the first
   segment (slice start + table bytes); d_consumed[m] table + body bytes (the
   reference's `*slice` advance); segment lengths in words in d_seg_words,
   message m's at [d_msg_seg_off[m], d_msg_seg_off[m+1]) (nmsg+1 entries; a
   failed message has none).  On CAPNP_E_MESSAGE_ENDS_PREMATURELY,
   d_body_off[m] / d_consumed[m] carry the reference's
   MessageEndsPrematurely(header, body) payload instead (serialize.rs:67-71,
   no_alloc_buffer_segments.rs:77-80, :254-257).  d_buf holds buf_len
   bytes; d_slice_off must be non-decreasing with d_slice_off[nmsg] <=
   buf_len, checked on the device before anything is read
   (CAPNP_E_INVALID_ARGUMENT otherwise).  d_body_off / d_consumed may be NULL.
   Synchronises the stream twice (the offset check, then the segment total
   against segs_cap: CAPNP_E_BUFFER_NOT_LARGE_ENOUGH, with only d_msg_seg_off
   written). */
capnp_status capnp_gpu_read_flat_messages(capnp_ctx* ctx, const uint8_t* d_buf, size_t buf_len,
                                          const uint64_t* d_slice_off, size_t nmsg,
                                          const capnp_reader_options* opts, int no_alloc,
                                          uint32_t* d_seg_words, size_t segs_cap,
                                          uint64_t* d_msg_seg_off, int32_t* d_status,
                                          uint64_t* d_body_off, uint64_t* d_consumed,
                                          void* stream);

/* ---- host message API (mirrors serialize_packed) ----------------------- */
/* Latency of the per-message calls below: a message that fits the one-launch
   kernels (writes of <= 8448 words, reads of bodies < 64 Ki words) is served
   by one workgroup; the host writes its inputs into device memory through
   the PCI BAR on large-BAR devices (1 MiB per context; pinned memory
   otherwise, or with CAPNP_PERCALL_BAR=0) and its results land in pinned
   host memory.  A call within
   1 ms of the context's previous per-message call goes to a resident
   service workgroup of its kind instead of a launch: it polls a pinned
   request line, serves each request, and exits 250 us after its last one
   (so a device-wide synchronisation right after a burst of calls waits up to
   that long, and a context destroyed mid-burst stops it first).  The
   environment variable CAPNP_PERCALL_SERVICE=0 makes every call launch. */
/* serialize_packed::write_message (serialize_packed.rs:446-453 ->
   serialize.rs:574-582): packs the segment table word 0, the rest of the
   table, then each segment as separate write_all chunks
   (serialize.rs:605-679).  segs[i] points at seg_words[i] words. */
capnp_status capnp_packed_write_message(capnp_ctx* ctx, const uint64_t* const* segs,
                                        const uint32_t* seg_words, uint32_t nseg,
                                        uint8_t* out, size_t cap, size_t* written);

/* serialize_packed::read_message / try_read_message (serialize_packed.rs:
   233-255 -> serialize.rs:287-325, 448-524).  Read units: 8 bytes, the rest
   of the segment table, then the whole body.  try_mode != 0 returns
   CAPNP_NONE on an empty input instead of CAPNP_E_PREMATURE_END_OF_FILE.
   body receives the segments back to back (body_cap_words capacity);
   seg_words_out (capacity CAPNP_SEGMENTS_COUNT_LIMIT) the segment lengths;
   *consumed the packed bytes used. */
capnp_status capnp_packed_read_message(capnp_ctx* ctx, const uint8_t* in, size_t in_len,
                                       const capnp_reader_options* opts, int try_mode,
                                       uint64_t* body, size_t body_cap_words,
                                       uint32_t* seg_words_out, uint32_t* nseg_out,
                                       size_t* consumed);

/* serialize_packed::read_message_no_alloc / try_read_message_no_alloc
   (serialize_packed.rs:263-291 -> serialize.rs:333-440): the table rest is
   read 8 bytes at a time into `buffer` and the body follows it there.
   `buffer` must be 8-byte aligned (CAPNP_E_UNALIGNED_SEGMENT otherwise). */
capnp_status capnp_packed_read_message_no_alloc(capnp_ctx* ctx, const uint8_t* in,
                                                size_t in_len,
                                                const capnp_reader_options* opts,
                                                int try_mode, uint8_t* buffer,
                                                size_t buffer_len, uint32_t* nseg_out,
                                                size_t* table_bytes_out,
                                                size_t* body_bytes_out, size_t* consumed);

/* try_read_message in a loop over one packed stream in device memory with
   no byte index (serialize.rs:310-325, :448-524; serialize_packed.rs:246-255):
   writes the starts of the messages the loop reads completely,
   d_msg_byte_off[0..*nmsg), and d_msg_byte_off[*nmsg] = where the next
   try_read_message starts (== nbytes: it returns None, a clean end; else the
   rest of the stream is a message that fails, whose status
   capnp_gpu_read_messages over [d_msg_byte_off[*nmsg], nbytes) gives).
   d_msg_byte_off holds max_msgs + 1 entries; with *nmsg == max_msgs the loop
   may go on from d_msg_byte_off[*nmsg].  The messages' bytes are
   [d_msg_byte_off[k], d_msg_byte_off[k+1]): capnp_gpu_read_messages with
   that index decodes them (status, segments, consumed per message).
   Blocking.  The stream is resolved as one read unit by the speculative
   block walk (resync), the message chain is followed through the decoded
   segment tables on the device. */
capnp_status capnp_gpu_find_messages(capnp_ctx* ctx, const uint8_t* d_packed, size_t nbytes,
                                     size_t max_msgs, uint64_t* d_msg_byte_off, size_t* nmsg,
                                     void* stream);

/* try_read_message in a loop over one packed stream in device memory with
   no byte index, in ONE pass (serialize.rs:310-325, :448-524;
   serialize_packed.rs:246-255): the stream is resolved and decoded once (the
   block walk of capnp_gpu_find_messages) into d_words, the message chain is
   followed through the decoded segment tables in parallel, and the messages
   are described in place, with no second decode:
     d_words            the decoded stream (segment tables and bodies), words_cap words;
     d_msg_byte_off[m]  message m's first packed byte (nmsg + 1 entries: the
                        last is where the loop's next try_read_message starts);
     d_body_word_off[m] the word of d_words where message m's first segment
                        starts (its segments follow back to back);
     d_seg_words        segment lengths in words, message m's at
                        [d_msg_seg_off[m], d_msg_seg_off[m+1]) (nmsg + 1 entries).
   Messages are read while the loop reads them: a segment table the reader
   rejects (segment count, total words over opts' traversal limit; opts
   NULL = defaults), a message cut by the stream end, or one the resolution
   could not place, ends the list.  *clean = 1 if the loop ended at the end of
   the stream (the next try_read_message returns None); otherwise the
   message at d_msg_byte_off[*nmsg] is the one the loop tries next: its status
   (or, where the resolution stopped early, its contents, and the loop goes
   on after it) is what capnp_gpu_read_messages gives over
   [d_msg_byte_off[*nmsg], nbytes) in try mode.
   Capacities: msgs_cap messages (d_msg_byte_off and d_msg_seg_off hold
   msgs_cap + 1 entries, d_body_word_off msgs_cap), segs_cap segments,
   words_cap words.  CAPNP_E_BUFFER_NOT_LARGE_ENOUGH when one is short, with
   *words_need / *msgs_need / *segs_need (may be NULL) set to what is known
   to be needed so far (call again with at least those).  Blocking. */
capnp_status capnp_gpu_read_message_stream(capnp_ctx* ctx, const uint8_t* d_packed,
                                           size_t nbytes, const capnp_reader_options* opts,
                                           uint64_t* d_words, size_t words_cap,
                                           uint64_t* d_msg_byte_off, uint64_t* d_body_word_off,
                                           size_t msgs_cap, uint64_t* d_seg_words,
                                           size_t segs_cap, uint64_t* d_msg_seg_off,
                                           size_t* nmsg, int32_t* clean, size_t* words_need,
                                           size_t* msgs_need, size_t* segs_need, void* stream);

/* ---- Streaming adaptors over caller-supplied byte streams ----------------
 * The async PackedWrite / PackedRead of capnp-futures
 * (capnp-futures/src/serialize_packed.rs:34-225, :330-521) and its message
 * reader (capnp-futures/src/serialize_packed.rs:233-258 ->
 * capnp-futures/src/serialize.rs:31-137): input split at any byte, an inner
 * stream that returns short reads / partial writes or "pending".  The inner
 * stream is a function plus a user pointer:
 *   read:  bytes read into buf (0 = end of stream), CAPNP_IO_PENDING when
 *          nothing is available now, or another negative value on error;
 *   write: bytes accepted (1..len), CAPNP_IO_PENDING, or negative on error.
 * The transform runs in the GPU kernels (capnp_pack_batch_host /
 * capnp_unpack_batch_host); an adaptor is used by one thread at a time. */
#define CAPNP_IO_PENDING (-1)
typedef ptrdiff_t (*capnp_read_fn)(void* user, uint8_t* buf, size_t len);
typedef ptrdiff_t (*capnp_write_fn)(void* user, const uint8_t* buf, size_t len);
typedef struct capnp_packed_writer capnp_packed_writer;
typedef struct capnp_packed_reader capnp_packed_reader;

/* PackedWrite::new(inner) (capnp-futures serialize_packed.rs:336-348). */
capnp_packed_writer* capnp_packed_writer_new(capnp_ctx* ctx, capnp_write_fn fn, void* user);
void capnp_packed_writer_free(capnp_packed_writer* w);
/* poll_write (poll_write_aux, :350-504): takes all `len` bytes.  A word
   completed from carried bytes and the whole words of this call are one
   packed chunk (runs never reach past the call, as the reference's run scan
   of `inbuf`); trailing bytes of an incomplete word are carried.  Packed
   bytes are queued and handed to the inner writer on flush (or every
   1 MiB of input). */
capnp_status capnp_packed_writer_write(capnp_packed_writer* w, const uint8_t* buf, size_t len);
/* poll_flush / finish_pending_writes (:506-521): packs what is queued and
   drains it to the inner writer; CAPNP_PENDING if the inner writer pends
   (call again).  Carried bytes of an incomplete word stay carried. */
capnp_status capnp_packed_writer_flush(capnp_packed_writer* w);
/* Bytes of an incomplete word carried to the next write (0..7). */
size_t capnp_packed_writer_carried(const capnp_packed_writer* w);

/* PackedRead::new(inner) (:56-70). */
capnp_packed_reader* capnp_packed_reader_new(capnp_ctx* ctx, capnp_read_fn fn, void* user);
void capnp_packed_reader_free(capnp_packed_reader* r);
/* Bulk read-ahead (off by default): pull input in MiB units past what the
   current read can need, while the inner reader returns every byte asked
   (a file, a memory stream).  Off, a read first decodes what is staged and
   pulls only when no complete record is (a read may then return fewer bytes
   than asked, as poll_read does), so, as the reference reads no further than
   the current request, a blocking pipe or socket whose peer sent exactly one
   request's worth and awaits a reply is never read past it. */
void capnp_packed_reader_set_readahead(capnp_packed_reader* r, int on);
/* poll_read (:74-225): 1..len unpacked bytes in *nread, 0 at a clean end of
   the stream, CAPNP_PENDING when the inner reader pends, and
   CAPNP_E_PREMATURE_END_OF_FILE when the stream ends inside a record (the
   reference's UnexpectedEof). */
capnp_status capnp_packed_reader_read(capnp_packed_reader* r, uint8_t* out, size_t len,
                                      size_t* nread);
/* read_exact: reads until `len` bytes (retrying a pending inner reader);
   CAPNP_E_PREMATURE_END_OF_FILE if the stream ends first; *got (may be NULL)
   = bytes delivered. */
capnp_status capnp_packed_reader_read_exact(capnp_packed_reader* r, uint8_t* out, size_t len,
                                            size_t* got);
/* try_read_message / read_message (capnp-futures serialize.rs:31-137): the
   segment table then the body into `body`; CAPNP_NONE (try_mode) or
   CAPNP_E_PREMATURE_END_OF_FILE at a clean end; InvalidNumberOfSegments,
   MessageTooLarge as serialize.rs:467-507; BufferNotLargeEnough with
   *body_words = words needed when body_cap_words is short (the table has
   then been read and *nseg / seg_words hold it; read the body with
   capnp_packed_reader_read_exact). */
capnp_status capnp_packed_reader_read_message(capnp_packed_reader* r,
                                              const capnp_reader_options* opts, int try_mode,
                                              uint64_t* body, size_t body_cap_words,
                                              uint32_t* seg_words, uint32_t* nseg,
                                              uint64_t* body_words);
/* Bytes staged (packed, not yet decoded) plus decoded bytes not yet read. */
size_t capnp_packed_reader_buffered(const capnp_packed_reader* r);

#ifdef __cplusplus
}
#endif
#endif /* CAPNP_PACKED_H */
