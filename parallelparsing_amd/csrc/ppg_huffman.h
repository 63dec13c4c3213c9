// ppg_huffman.h — device-side DEFLATE (RFC 1951) Huffman machinery shared by the inflate kernel:
// canonical table build by 64 lanes, the zlib 1.2.11 validity rules, and the bit-serial slow path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef PPG_DB
#define PPG_DB 8
#endif
#define DB PPG_DB        // distance root table bits
#define CB 7             // code-length-code table bits (complete: max code length is 7)

// Root-table entries (the lane-parallel decoder's format).  Every field is placed so that one
// VALU op extracts or applies it: bits [4:0] are the code length (bit 4 always 0), so
// v_alignbit / v_lshrrev consume the code straight from the entry.
//  litlen: a literal's entry is its finished token word (the decoder's format: [7:0] bits = L,
//          [16:8] bytes = 1, [31:17] 0x100 | byte), and an entry to decode bit-serially (end-of-
//          block, invalid symbol, or a code longer than the root table) the special token word
//          (bits 128, bytes 0, field 0x100); both have bit 6 clear.  A length symbol's entry:
//          [3:0] code length L, [6] set, [15:8] L + length extra bits, [24:16] length base, so
//          e >> 8 is the token word's bits + bytes part before the extra bits' value, and
//          ((e >> 8) - e)[4:0] the number of extra bits.  (r03: the decoder selects a literal's word
//          instead of assembling it from fields, ~10 VALU fewer per candidate; r03 v4: this length
//          layout, 3 VALU fewer per candidate.)
//  dist:   [3:0] L2, [9:5] L2 + extra bits, [14:10] extra bits, [31:16] base - 1 (the token
//          word's field is distance - 1); all ones = decode bit-serially (its sign bit is the test)
//  code-length code: [3:0] L, [15:8] symbol

__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                     35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385,
                                     513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum { TAB_LIT = 0, TAB_DST = 1, TAB_CL = 2 };

// the decoder's token word of a token its root tables cannot resolve: 128 bits (ends the walk),
// 0 bytes, field 0x100
#define PPG_SPECIAL_TOKEN (128u | (0x100u << 17))

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | (uint64_t)uni((uint32_t)x);
}

__device__ __forceinline__ uint32_t rdlane_u(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

__device__ __forceinline__ uint32_t make_entry(uint32_t sym, uint32_t len, int kind) {
    if (kind == TAB_CL) return len | (sym << 8);
    if (kind == TAB_LIT) {
        if (sym < 256) return len | (1u << 8) | ((0x100u | sym) << 17);
        if (sym == 256 || sym >= 286) return PPG_SPECIAL_TOKEN;
        const uint32_t x = c_lext[sym - 257];
        return len | 0x40u | ((len + x) << 8) | ((uint32_t)c_lbase[sym - 257] << 16);
    }
    if (sym >= 30) return ~0u;
    const uint32_t x = c_dext[sym];
    return len | ((len + x) << 5) | (x << 10) | ((uint32_t)(c_dbase[sym] - 1) << 16);
}

// Builds a canonical-Huffman root table of 2^TB entries from n code lengths (all 64 lanes).
// Codes longer than TB (and unused patterns of an incomplete code) get the bit-serial entry (0; the
// special token word in a litlen table, all ones in a distance table) -> bit-serial path,
// which decodes bit-by-bit from count[]/sorted[].  Validity follows zlib 1.2.11 inflate_table:
// over-subscribed -> error; incomplete -> error unless exactly one code of length 1 (not for
// the code-length code); no codes at all -> accepted (decoding then fails).  Returns 0 / -1.
// Per-lane canonical-code description (lane l = code length l, 1..15): number of codes, first
// code (MSB-first), and index of that length's first symbol in `sorted`.  canon_decode uses it.
struct Canon {
    uint32_t count, first, index;
};

// copy_to (may be NULL): where the sorted symbols are kept for canon_decode when `sorted` is only
// LDS scratch of the build (ppg_inflate_kernel, PPG_GSORT: global memory, written once per table)
template <int TB>
__device__ int build_table(const uint8_t *lens, int n, uint32_t *table, Canon *canon, uint16_t *sorted, int kind,
                           int lane, uint16_t *copy_to = nullptr) {
    // Runs once per block, so it is written for few registers, not speed: per-length counts,
    // offsets and running ranks live one per lane (lane l holds length l), loops stay rolled.
    uint32_t cnt = 0;
    for (int g = 0; g < n; g += 64) {
        const int s = g + lane;
        const uint32_t L = s < n ? lens[s] : 0u;
#pragma unroll 1
        for (uint32_t l = 1; l < 16; l++) {
            const uint32_t c = (uint32_t)__popcll(__ballot(L == l));
            if ((uint32_t)lane == l) cnt += c;
        }
    }
    int left = 1, maxl = 0;
    uint32_t offs = 0, run = 0, first = 0, code = 0;
#pragma unroll 1
    for (uint32_t l = 1; l < 16; l++) {
        const uint32_t c = rdlane_u(cnt, l);
        left = left * 2 - (int)c;       // stays negative once over-subscribed
        if (c) maxl = (int)l;
        if ((uint32_t)lane == l) { offs = run; first = code; }
        run += c;
        code = (code + c) << 1;         // first code of length l+1 (RFC 1951 3.2.2)
    }
    if (maxl != 0) {
        if (left < 0) return -1;
        if (left > 0 && (kind == TAB_CL || maxl != 1)) return -1;
    } else if (kind == TAB_CL) {
        return -1;  // zlib accepts the empty set, then fails with "missing end-of-block"
    }
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t seen = 0;
    for (int g = 0; g < n; g += 64) {
        const int s = g + lane;
        const uint32_t L = s < n ? lens[s] : 0u;
        uint32_t mypos = 0;
#pragma unroll 1
        for (uint32_t l = 1; l < 16; l++) {
            const uint64_t m = __ballot(L == l);
            if (m) {
                const uint32_t base = rdlane_u(offs, l) + rdlane_u(seen, l);
                if (L == l) mypos = base + (uint32_t)__popcll(m & lt);
                if ((uint32_t)lane == l) seen += (uint32_t)__popcll(m);
            }
        }
        if (L) sorted[mypos] = (uint16_t)s;
    }
    if (canon) *canon = Canon{lane == 0 || lane > 15 ? 0u : cnt, first, offs};
    __syncthreads();
    for (int e0 = 0; e0 < (1 << TB); e0 += 64) {   // uniform trip count (see ppg_inflate_kernel)
        const int e = e0 + lane;
        // not found (longer than TB, or an unused pattern of an incomplete code): bit-serial
        uint32_t code = 0, first = 0, index = 0,
                 entry = kind == TAB_LIT ? PPG_SPECIAL_TOKEN : kind == TAB_DST ? ~0u : 0u;
        bool found = false;
#pragma unroll 1
        for (int l = 1; l <= TB; l++) {
            code |= ((uint32_t)e >> (l - 1)) & 1u;
            const uint32_t c = rdlane_u(cnt, (uint32_t)l);
            if (!found && code - first < c) {
                entry = make_entry(sorted[index + code - first], (uint32_t)l, kind);
                found = true;
            }
            index += c;
            first = (first + c) << 1;
            code <<= 1;
        }
        table[e] = entry;
    }
    if (copy_to)
        for (int i = lane; i < n; i += 64) copy_to[i] = sorted[i];
    __syncthreads();
    return 0;
}

// Consume n (<= 32) bits from a reader's bit buffer (fields bb / bn).
template <class R>
__device__ __forceinline__ uint32_t br_take(R &b, uint32_t n) {
    uint32_t v = (uint32_t)(b.bb & ((1ull << n) - 1ull));
    b.bb >>= n;
    b.bn -= n;
    return v;
}

// Canonical decode of the next code, all 15 lengths at once: lane l reverses the next l bits
// (DEFLATE codes are MSB-first in an LSB-first stream) and tests them against the range of codes
// of length l.  For a prefix code exactly one length matches; ballot + ff1 finds it.  Returns the
// symbol and consumes the code, or -1 (no code matches: invalid).  Needs bn >= 15.
template <class R>
__device__ __forceinline__ int canon_decode(R &b, const Canon &c, const uint16_t *sorted, int lane) {
    const uint32_t bits = __builtin_bitreverse32((uint32_t)b.bb);   // next bit in the MSB
    const uint32_t l = (uint32_t)lane;
    const uint32_t code = (l >= 1 && l <= 15) ? bits >> (32 - l) : 0u;
    const uint64_t hit = __ballot(l >= 1 && l <= 15 && code - c.first < c.count);
    if (!hit) return -1;
    const uint32_t L = (uint32_t)__builtin_ctzll(hit);
    const uint32_t idx = rdlane_u(c.index + code - c.first, L);
    const int sym = (int)__builtin_amdgcn_readfirstlane(sorted[idx]);
    b.bb >>= L;
    b.bn -= L;
    return sym;
}

// status codes (ZResult, Interop/Conventions.cs:9-20)
#define ST_OK 0
#define ST_DATA_ERROR (-3)

