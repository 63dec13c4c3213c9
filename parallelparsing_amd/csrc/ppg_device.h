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
    // CreateIndex pass 1 only (ppg_inflate_kernel<.., IX = true>): decode whole blocks until one
    // ends at or past stop_bit (or the final block ends); block ends go to blk[blk_off, +blk_cap)
    uint64_t stop_bit;
    uint32_t blk_off;
    uint32_t blk_cap;
    // DecompressAll: the newline census fused into the output flush (ppg_inflate_kernel, nls != null).
    // Body newline m (chunk position p) is stored as raw_shift + p at nls[nl_off + m] while m < nl_cap.
    uint64_t nl_off;
    uint32_t nl_cap;
    uint32_t raw_shift;   // |offset_k|: raw index of the body's first byte
    uint32_t prev_byte;   // raw byte before the body: offset_k's last byte, or '\n' when offset_k is empty
    uint32_t pad;         // (raw[0] == '\n' is then an empty line, as in Parsing.Parse's view)
};

struct PpgInflateResult {
    uint64_t produced;    // bytes written (Core.cs:191: len - AvailOut)
    uint64_t end_bit;     // bit position after the chunk's trailing end-of-block code
    int32_t status;       // 0 or a ZResult error code (Interop/Conventions.cs:9-20)
    int32_t flags;        // PPG_FLAG_*
    uint32_t nblocks;     // CreateIndex pass 1: block ends recorded
    uint32_t last;        // CreateIndex pass 1: the final block (BFINAL) was decoded
    uint32_t newlines;    // census: '\n' bytes in the produced body
    uint32_t pflags;      // census: PPG_PF_* below
};

#define PPG_PF_SERIAL 1     // an empty line (incl. at the offset junction) or a NUL byte in the body
#define PPG_PF_OVERFLOW 2   // more body newlines than nl_cap: descriptors come from ppg_parse_emit
#define PPG_PF_NUL 4        // a NUL byte in the body (ppg_parse_chain declines the chunk)

// CreateIndex: one deflate block end (Core.cs:98 -- where inflate(Z_BLOCK) reports data_type & 128)
struct PpgBlockEnd {
    uint64_t end_bit;     // absolute bit position after the block (the next block's header)
    uint64_t out_end;     // output bytes of the piece up to the block end
};

// CreateIndex: '@' census of one block's output (Core.cs:79-96), positions relative to the block
struct PpgAtStats {
    uint32_t count;       // '@' bytes
    int32_t first;        // first '@' (-1: none)
    int32_t last;         // last '@' (-1: none)
    uint32_t max_gap;     // largest distance between consecutive '@' inside the block
};

// offset_k bytes (Common/Index.cs:75) live concatenated in one device buffer
// ppg_materialize_kernel: where a piece's pass-1 symbols and its exact starting history are
struct PpgMatInfo {
    uint64_t sym_off;     // first symbol (positions) in the pass-1 output buffer
    uint64_t win_off;     // its 32 KiB starting history in the window buffer (bytes)
    uint64_t end_bit;     // the piece's last block end (its result's end_bit)
    uint32_t nblocks;
    uint32_t last;        // the piece ends with the final block
    uint32_t prev;        // the census's previous byte, or > 255: the history's last byte
    uint32_t pad;
};

struct PpgOffsetRef {
    uint64_t start;
    uint32_t len;
    uint32_t nl;          // '\n' bytes in offset_k | PPG_OFF_SERIAL
};

#define PPG_OFF_SERIAL 0x80000000u   // offset_k alone has an empty line or a NUL (R-P3)
#define PPG_OFF_NUL 0x40000000u      // offset_k has a NUL
#define PPG_OFF_COUNT 0x3FFFFFFFu    // the '\n' count

struct PpgParseInfo {
    uint64_t records;     // FastqRecords emitted by Parsing.Parse for this chunk
    uint32_t newlines;    // '\n' bytes in raw
    uint16_t serial;      // 1: parsed by the exact serial state machine
    uint16_t emit;        // 1: census overflowed; descriptors by the ppg_parse_emit scan
};

// CreateIndex: a 32 KiB history ending at output position `end` of a piece (ppg_gather_kernel)
struct PpgGather {
    uint64_t out_off;     // position p >= 0 of the piece is out[out_off + (p & mask)]
    uint64_t dict_off;    // position p < 0 is dicts[dict_off + 32768 + p]
    uint64_t end;
    uint64_t mask;        // 0xFFFF for pass-1 rings, ~0 for plain output
    uint64_t ref_off;     // with a reference buffer: compare against ref[ref_off, +32768)
};

struct PpgSpan {          // byte range [lo, hi) of an output buffer
    uint64_t lo, hi;
};

#define PPG_FLAG_NO_EOB 1     // the symbol after the last output byte is not end-of-block
#define PPG_FLAG_OVERRUN 2    // decoding consumed bits past the chunk's compressed slice
#define PPG_FLAG_BLK_FULL 16  // CreateIndex pass 1: more block ends than blk_cap

// CRC-32 of the GPU CreateIndex's exact output (ppg_crc_kernel): one lane per kCrcSub bytes, one
// wave (64 lanes) per kCrcSeg bytes
constexpr uint32_t kCrcSub = 16384;
constexpr uint32_t kCrcSeg = 64 * kCrcSub;
