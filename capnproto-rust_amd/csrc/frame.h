// frame.h — result record of the device framing kernel (frame.hip).
#pragma once
#include <stdint.h>

struct FrameResult {
    int32_t status;
    uint32_t nseg;
    uint64_t table_consumed;   // packed bytes used by the table read units
    uint64_t total_words;      // body words
    uint64_t table_bytes;      // bytes of the decoded table (no-alloc layout)
    uint64_t body_in_off[2];   // packed range of the body unit (chunk index)
    uint64_t body_out_off[2];  // {0, total_words}
    uint32_t seg_words[512];
    uint8_t table[2064];       // decoded table bytes
};
