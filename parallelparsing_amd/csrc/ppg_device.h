// ppg_device.h — host/device shared records of libppgpu (plain C layout, no HIP types).
#pragma once
#include <stdint.h>

// One inflate job per checkpoint chunk k (Point k -> Point k+1 of Common/Index.cs:51-82).
struct PpgInflateJob {
    uint64_t bit_start;   // 8*from.Input - from.Bits, relative to the device copy of the file range
    uint64_t bit_limit;   // 8*to.Input (relative): the slice LazyFileReader hands zlib ends there
    uint64_t out_off;     // from.Output - base output of the batch (byte offset into the out buffer)
    uint64_t out_len;     // to.Output - from.Output (Core.cs:140)
    uint64_t dict_off;    // byte offset of from.Window (32 KiB) in the dictionary buffer
    uint64_t expect_end;  // 8*to.Input - to.Bits (R-E5), or ~0 when not checkable (last chunk)
};

struct PpgInflateResult {
    uint64_t produced;    // bytes written (Core.cs:191: len - AvailOut)
    uint64_t end_bit;     // bit position after the chunk's trailing end-of-block code
    int32_t status;       // 0 or a ZResult error code (Interop/Conventions.cs:9-20)
    int32_t flags;        // PPG_FLAG_*
};

// offset_k bytes (Common/Index.cs:75) live concatenated in one device buffer
struct PpgOffsetRef {
    uint64_t start;
    uint32_t len;
    uint32_t pad;
};

struct PpgParseInfo {
    uint64_t records;     // FastqRecords emitted by Parsing.Parse for this chunk
    uint32_t newlines;    // '\n' bytes in raw
    uint32_t serial;      // 1: parsed by the exact serial state machine
};

#define PPG_FLAG_NO_EOB 1     // the symbol after the last output byte is not end-of-block
#define PPG_FLAG_OVERRUN 2    // decoding consumed bits past the chunk's compressed slice
