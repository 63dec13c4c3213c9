// ppg_kernels.hip — gfx950 (MI355X / CDNA4) kernels for the chunked-gzip DecompressAll path.
//
//   ppg_inflate_kernel   one 64-lane wavefront per checkpoint chunk: raw DEFLATE inflate seeded
//                        with the Point's 32 KiB window and bit offset.  Replaces the zlib calls of
//                        Core.ExtractDeflateIndex (Decompressor/Core.cs:133-192): inflateInit2(-15)
//                        + inflatePrime + inflateSetDictionary + inflate(Z_NO_FLUSH) until
//                        to.Output-from.Output bytes exist.
//   ppg_parse_count      per-chunk newline census of raw = offset ++ chunk (Parsing.cs:11-69 fast
//                        path) + the conditions under which it equals the serial
//                        state machine.
//   ppg_parse_serial     the exact Parsing.Parse state machine for chunks the fast path declines.
//   ppg_scan_counts      exclusive scan of per-chunk record counts -> record bases.
//   ppg_parse_emit       per-record descriptors (n1..n4 newline positions) for fast chunks.
//
// Design: the decoder state (bit buffer, counters, positions) is wave-uniform and
// lives in SGPRs; compressed words are fetched with scalar loads; Huffman tables are built by all
// 64 lanes in LDS and read with one uniform ds_read per symbol; the 32 KiB history is an LDS ring
// indexed by the GLOBAL output address mod 32 KiB, so back-references are lane-parallel LDS copies
// and every completed 4 KiB unit leaves the ring as 16-B-per-lane coalesced stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "ppg_device.h"

#define RING_BITS 15
#define RING (1u << RING_BITS)
#define RMASK (RING - 1u)
#define LB 10            // litlen root table bits
#define DB 8             // distance root table bits
#define CB 7             // code-length-code table bits (complete: max code length is 7)
#define UNIT 4096        // flush unit (bytes, global-address aligned)

// table entry: [3:0] code length (0 = slow path) [5:4] kind [15:8] literal / extra bits [31:16] base
#define K_LIT 0u
#define K_BASE 1u
#define K_EOB 2u
#define K_BAD 3u

struct __attribute__((aligned(16))) InflateLds {
    uint8_t ring[RING];
    uint32_t lit[1 << LB];
    uint32_t dst[1 << DB];
    uint32_t cl[1 << CB];
    uint16_t lit_sorted[288];
    uint16_t dst_sorted[32];
    uint16_t cl_sorted[20];
    uint16_t lit_count[16];
    uint16_t dst_count[16];
    uint8_t lens[320];
};

__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                     35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385,
                                     513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

enum { TAB_LIT = 0, TAB_DST = 1, TAB_CL = 2 };

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint32_t make_entry(uint32_t sym, uint32_t len, int kind) {
    if (kind == TAB_CL) return len | (sym << 8);
    if (kind == TAB_LIT) {
        if (sym < 256) return len | (K_LIT << 4) | (sym << 8);
        if (sym == 256) return len | (K_EOB << 4);
        if (sym < 286) return len | (K_BASE << 4) | ((uint32_t)c_lext[sym - 257] << 8) | ((uint32_t)c_lbase[sym - 257] << 16);
        return len | (K_BAD << 4);
    }
    if (sym < 30) return len | (K_BASE << 4) | ((uint32_t)c_dext[sym] << 8) | ((uint32_t)c_dbase[sym] << 16);
    return len | (K_BAD << 4);
}

// Builds a canonical-Huffman root table of 2^TB entries from n code lengths (all 64 lanes).
// Codes longer than TB (and unused patterns of an incomplete code) get entry 0 -> slow path,
// which decodes bit-by-bit from count[]/sorted[].  Validity follows zlib 1.2.11 inflate_table:
// over-subscribed -> error; incomplete -> error unless exactly one code of length 1 (not for
// the code-length code); no codes at all -> accepted (decoding then fails).  Returns 0 / -1.
template <int TB>
__device__ int build_table(const uint8_t *lens, int n, uint32_t *table, uint16_t *count_lds, uint16_t *sorted,
                           int kind, int lane) {
    uint32_t cnt[16];
#pragma unroll
    for (int l = 0; l < 16; l++) cnt[l] = 0;
    for (int g = 0; g < n; g += 64) {
        int s = g + lane;
        uint32_t L = s < n ? lens[s] : 0u;
#pragma unroll
        for (int l = 1; l < 16; l++) cnt[l] += (uint32_t)__popcll(__ballot(L == (uint32_t)l));
    }
    int left = 1, maxl = 0;
#pragma unroll
    for (int l = 1; l < 16; l++) {
        left = left * 2 - (int)cnt[l];
        if (cnt[l]) maxl = l;
    }
    if (maxl != 0) {
        if (left < 0) return -1;
        if (left > 0 && (kind == TAB_CL || maxl != 1)) return -1;
    } else if (kind == TAB_CL) {
        return -1;  // zlib accepts the empty set, then fails with "missing end-of-block"
    }
    uint32_t offs[16], seen[16];
    offs[0] = 0;
    offs[1] = 0;
#pragma unroll
    for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + cnt[l];
#pragma unroll
    for (int l = 0; l < 16; l++) seen[l] = 0;
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    for (int g = 0; g < n; g += 64) {
        int s = g + lane;
        uint32_t L = s < n ? lens[s] : 0u;
        uint32_t mypos = 0;
#pragma unroll
        for (int l = 1; l < 16; l++) {
            uint64_t m = __ballot(L == (uint32_t)l);
            if (L == (uint32_t)l) mypos = offs[l] + seen[l] + (uint32_t)__popcll(m & lt);
            seen[l] += (uint32_t)__popcll(m);
        }
        if (L) sorted[mypos] = (uint16_t)s;
    }
    if (count_lds) {
        uint32_t c = 0;
#pragma unroll
        for (int l = 0; l < 16; l++) c = (lane == l) ? cnt[l] : c;
        if (lane < 16) count_lds[lane] = (uint16_t)c;
    }
    __syncthreads();
    for (int e = lane; e < (1 << TB); e += 64) {
        uint32_t code = 0, first = 0, index = 0, entry = 0;
#pragma unroll
        for (int l = 1; l <= TB; l++) {
            code |= ((uint32_t)e >> (l - 1)) & 1u;
            uint32_t c = cnt[l];
            if (entry == 0 && code - first < c) entry = make_entry(sorted[index + code - first], (uint32_t)l, kind);
            index += c;
            first = (first + c) << 1;
            code <<= 1;
        }
        table[e] = entry;
    }
    __syncthreads();
    return 0;
}

struct BitReader {
    uint64_t bb;   // bit buffer (LSB = next bit)
    uint32_t bn;   // valid bits in bb
    uint64_t wi;   // next 32-bit word to load
};

__device__ __forceinline__ void br_init(BitReader &b, const uint32_t *comp, uint64_t nwords, uint64_t bit) {
    b.wi = bit >> 5;
    uint32_t sh = (uint32_t)(bit & 31);
    uint32_t w = b.wi < nwords ? comp[b.wi] : 0u;
    b.wi++;
    b.bb = (uint64_t)(w >> sh);
    b.bn = 32 - sh;
}

// guarantees bn >= 32
__device__ __forceinline__ void br_refill(BitReader &b, const uint32_t *comp, uint64_t nwords) {
    if (b.bn <= 32) {
        uint32_t w = b.wi < nwords ? comp[b.wi] : 0u;
        b.wi++;
        b.bb |= (uint64_t)w << b.bn;
        b.bn += 32;
    }
}

__device__ __forceinline__ uint32_t br_take(BitReader &b, uint32_t n) {
    uint32_t v = (uint32_t)(b.bb & ((1ull << n) - 1ull));
    b.bb >>= n;
    b.bn -= n;
    return v;
}

__device__ __forceinline__ uint64_t br_pos(const BitReader &b) { return b.wi * 32 - b.bn; }

// Canonical bit-by-bit decode (codes longer than the root table, or invalid patterns).
// Returns symbol, or -1 for an invalid code.  Needs bn >= 15.
__device__ int slow_decode(BitReader &b, const uint16_t *count, const uint16_t *sorted) {
    uint32_t code = 0, first = 0, index = 0;
    for (uint32_t l = 1; l < 16; l++) {
        code |= (uint32_t)(b.bb >> (l - 1)) & 1u;
        uint32_t c = uni(count[l]);
        if (code - first < c) {
            uint32_t sym = uni(sorted[index + code - first]);
            b.bb >>= l;
            b.bn -= l;
            return (int)sym;
        }
        index += c;
        first = (first + c) << 1;
        code <<= 1;
    }
    return -1;
}

// Copies ring bytes [glo, ghi) (global output addresses) to out; head/tail bytes singly, the
// 16-B-aligned middle as one ds_read_b128 + global_store_dwordx4 per lane per KiB.
__device__ __forceinline__ void flush_range(const uint8_t *ring, uint8_t *out, uint64_t glo, uint64_t ghi, int lane) {
    if (ghi <= glo) return;
    uint64_t a = (glo + 15) & ~15ull, z = ghi & ~15ull;
    if (a >= z) {
        for (uint64_t g = glo + lane; g < ghi; g += 64) out[g] = ring[g & RMASK];
        return;
    }
    if (lane < (int)(a - glo)) out[glo + lane] = ring[(glo + lane) & RMASK];
    if (lane < (int)(ghi - z)) out[z + lane] = ring[(z + lane) & RMASK];
    for (uint64_t g = a + (uint64_t)lane * 16; g < z; g += 1024) {
        uint4 v = *(const uint4 *)(ring + (g & RMASK));
        *(uint4 *)(out + g) = v;
    }
}

// status codes (ZResult, Interop/Conventions.cs:9-20)
#define ST_OK 0
#define ST_DATA_ERROR (-3)

extern "C" __global__ __launch_bounds__(64) void ppg_inflate_kernel(
    const uint32_t *__restrict__ comp, uint64_t nwords, const PpgInflateJob *__restrict__ jobs,
    const uint8_t *__restrict__ dicts, uint8_t *__restrict__ out, PpgInflateResult *__restrict__ res, int njobs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    InflateLds &S = *reinterpret_cast<InflateLds *>(smem);
    const int lane = threadIdx.x;
    const int k = blockIdx.x;
    if (k >= njobs) return;
    const PpgInflateJob J = jobs[k];
    const uint64_t out_off = J.out_off, out_len = J.out_len;

    // history: dictionary byte i is output position i-32768 -> ring slot (out_off + i) mod 32 KiB
    {
        const uint32_t *d32 = (const uint32_t *)(dicts + J.dict_off);
        for (int w = lane; w < (int)(RING / 4); w += 64) {
            uint32_t v = d32[w];
            uint64_t g = out_off + (uint64_t)w * 4;
#pragma unroll
            for (int q = 0; q < 4; q++) S.ring[(g + q) & RMASK] = (uint8_t)(v >> (8 * q));
        }
    }
    __syncthreads();

    BitReader br;
    br_init(br, comp, nwords, J.bit_start);
    const uint64_t word_limit = (J.bit_limit >> 5) + 4;   // runaway guard for corrupt streams
    uint64_t gend = out_off;                              // global address of the next output byte
    const uint64_t gstop = out_off + out_len;
    uint64_t gflushed = out_off;
    int status = ST_OK;
    int flags = 0;
    int last = 0;
    int in_block = 0;   // 1 while a Huffman block is open (tables valid)

    while (gend < gstop && !last) {
        br_refill(br, comp, nwords);
        last = (int)br_take(br, 1);
        uint32_t type = br_take(br, 2);
        if (type == 0) {
            // ---- stored block ----
            br_take(br, br.bn & 7);
            br_refill(br, comp, nwords);
            uint32_t len = br_take(br, 16), nlen = br_take(br, 16);
            if ((len ^ 0xFFFFu) != nlen) { status = ST_DATA_ERROR; break; }
            uint64_t bytepos = br_pos(br) >> 3;
            const uint8_t *c8 = (const uint8_t *)comp;
            uint64_t remain = len;
            if (remain > gstop - gend) remain = gstop - gend;
            if (bytepos + remain > nwords * 4) { status = ST_DATA_ERROR; break; }
            uint64_t copied = 0;
            while (copied < remain) {
                uint64_t piece = remain - copied;
                if (piece > UNIT) piece = UNIT;
                for (uint64_t j = lane; j < piece; j += 64) S.ring[(gend + j) & RMASK] = c8[bytepos + copied + j];
                gend += piece;
                copied += piece;
                if (gend - (gflushed & ~(uint64_t)(UNIT - 1)) >= UNIT) {
                    uint64_t to = gend & ~(uint64_t)(UNIT - 1);
                    flush_range(S.ring, out, gflushed, to, lane);
                    gflushed = to;
                }
            }
            br_init(br, comp, nwords, (bytepos + copied) * 8);
            if (copied < len) break;   // output full mid-block (zlib stops at avail_out == 0)
            in_block = 0;
            continue;
        }
        if (type == 3) { status = ST_DATA_ERROR; break; }
        if (type == 1) {
            // ---- fixed Huffman tables (RFC 1951 3.2.6) ----
            for (int s = lane; s < 320; s += 64) {
                uint8_t L;
                if (s < 144) L = 8; else if (s < 256) L = 9; else if (s < 280) L = 7; else if (s < 288) L = 8;
                else L = 5;   // 288..319 -> the 32 distance codes
                S.lens[s] = L;
            }
            __syncthreads();
            build_table<LB>(S.lens, 288, S.lit, S.lit_count, S.lit_sorted, TAB_LIT, lane);
            build_table<DB>(S.lens + 288, 32, S.dst, S.dst_count, S.dst_sorted, TAB_DST, lane);
        } else {
            // ---- dynamic Huffman tables (RFC 1951 3.2.7) ----
            br_refill(br, comp, nwords);
            uint32_t hlit = br_take(br, 5) + 257, hdist = br_take(br, 5) + 1, hclen = br_take(br, 4) + 4;
            if (hlit > 286 || hdist > 30) { status = ST_DATA_ERROR; break; }
            for (int s = lane; s < 19; s += 64) S.lens[s] = 0;
            __syncthreads();
            for (uint32_t i = 0; i < hclen; i++) {
                br_refill(br, comp, nwords);
                uint32_t v = br_take(br, 3);
                if (lane == 0) S.lens[c_clorder[i]] = (uint8_t)v;
            }
            __syncthreads();
            if (build_table<CB>(S.lens, 19, S.cl, nullptr, S.cl_sorted, TAB_CL, lane) != 0) { status = ST_DATA_ERROR; break; }
            uint32_t idx = 0, total = hlit + hdist;
            bool bad = false;
            while (idx < total) {
                br_refill(br, comp, nwords);
                uint32_t e = uni(S.cl[br.bb & ((1u << CB) - 1)]);
                uint32_t L = e & 15;
                if (L == 0) { bad = true; break; }
                br_take(br, L);
                uint32_t sym = e >> 8;
                uint32_t val, rep;
                if (sym < 16) { val = sym; rep = 1; }
                else if (sym == 16) {
                    if (idx == 0) { bad = true; break; }
                    val = uni(S.lens[idx - 1]);
                    rep = 3 + br_take(br, 2);
                } else if (sym == 17) { val = 0; rep = 3 + br_take(br, 3); }
                else { val = 0; rep = 11 + br_take(br, 7); }
                if (idx + rep > total) { bad = true; break; }
                for (uint32_t j = lane; j < rep; j += 64) S.lens[idx + j] = (uint8_t)val;
                idx += rep;
            }
            __syncthreads();
            if (bad) { status = ST_DATA_ERROR; break; }
            if (uni(S.lens[256]) == 0) { status = ST_DATA_ERROR; break; }
            // distance lengths move to their own slots so both tables read from S.lens
            if (build_table<LB>(S.lens, (int)hlit, S.lit, S.lit_count, S.lit_sorted, TAB_LIT, lane) != 0) { status = ST_DATA_ERROR; break; }
            if (build_table<DB>(S.lens + hlit, (int)hdist, S.dst, S.dst_count, S.dst_sorted, TAB_DST, lane) != 0) { status = ST_DATA_ERROR; break; }
        }
        in_block = 1;

        // ---- token loop ----
        for (;;) {
            if (gend >= gstop) break;
            if (br.wi > word_limit) { status = ST_DATA_ERROR; break; }
            br_refill(br, comp, nwords);
            uint32_t e = uni(S.lit[br.bb & ((1u << LB) - 1)]);
            uint32_t L = e & 15;
            uint32_t kind;
            uint32_t sym_lit = 0, len = 0;
            if (L != 0) {
                br.bb >>= L;
                br.bn -= L;
                kind = (e >> 4) & 3;
                if (kind == K_LIT) sym_lit = (e >> 8) & 0xFF;
                else if (kind == K_BASE) len = (e >> 16) + br_take(br, (e >> 8) & 15);
            } else {
                int sym = slow_decode(br, S.lit_count, S.lit_sorted);
                if (sym < 0 || sym > 285) { status = ST_DATA_ERROR; break; }
                if (sym < 256) { kind = K_LIT; sym_lit = (uint32_t)sym; }
                else if (sym == 256) kind = K_EOB;
                else {
                    kind = K_BASE;
                    len = c_lbase[sym - 257];
                    len += br_take(br, c_lext[sym - 257]);
                }
            }
            if (kind == K_LIT) {
                if (lane == 0) S.ring[gend & RMASK] = (uint8_t)sym_lit;
                gend++;
            } else if (kind == K_BASE) {
                br_refill(br, comp, nwords);
                uint32_t d = uni(S.dst[br.bb & ((1u << DB) - 1)]);
                uint32_t dist;
                uint32_t DL = d & 15;
                if (DL != 0) {
                    if (((d >> 4) & 3) != K_BASE) { status = ST_DATA_ERROR; break; }
                    br.bb >>= DL;
                    br.bn -= DL;
                    dist = (d >> 16) + br_take(br, (d >> 8) & 15);
                } else {
                    int ds = slow_decode(br, S.dst_count, S.dst_sorted);
                    if (ds < 0 || ds > 29) { status = ST_DATA_ERROR; break; }
                    dist = c_dbase[ds];
                    dist += br_take(br, c_dext[ds]);
                }
                uint64_t room = gstop - gend;
                uint32_t n = len < room ? len : (uint32_t)room;
                if (dist >= n) {
                    for (uint32_t j = lane; j < n; j += 64) {
                        uint8_t v = S.ring[(gend - dist + j) & RMASK];
                        S.ring[(gend + j) & RMASK] = v;
                    }
                } else {
                    for (uint32_t j = lane; j < n; j += 64) {
                        uint8_t v = S.ring[(gend - dist + (j % dist)) & RMASK];
                        S.ring[(gend + j) & RMASK] = v;
                    }
                }
                gend += n;
            } else if (kind == K_EOB) {
                in_block = 0;
                break;
            } else {
                status = ST_DATA_ERROR;
                break;
            }
            if (gend - (gflushed & ~(uint64_t)(UNIT - 1)) >= UNIT) {
                uint64_t to = gend & ~(uint64_t)(UNIT - 1);
                flush_range(S.ring, out, gflushed, to, lane);
                gflushed = to;
            }
        }
        if (status != ST_OK) break;
    }
    flush_range(S.ring, out, gflushed, gend, lane);

    // R-E5 integrity: the chunk should end right before its block's end-of-block code.
    uint64_t end_bit = br_pos(br);
    if (status == ST_OK && in_block && gend == gstop) {
        br_refill(br, comp, nwords);
        uint32_t e = uni(S.lit[br.bb & ((1u << LB) - 1)]);
        bool eob;
        if ((e & 15) != 0) {
            eob = ((e >> 4) & 3) == K_EOB;
            if (eob) br_take(br, e & 15);
        } else {
            eob = slow_decode(br, S.lit_count, S.lit_sorted) == 256;   // EOB is often a long code
        }
        if (eob) end_bit = br_pos(br);
        else flags |= PPG_FLAG_NO_EOB;
    }
    if (end_bit > J.bit_limit) flags |= PPG_FLAG_OVERRUN;
    if (lane == 0) {
        res[k].produced = gend - out_off;
        res[k].end_bit = end_bit;
        res[k].status = status;
        res[k].flags = flags;
    }
}

// ------------------------------------------------------------------------------------------
// FASTQ record scan.  raw_k = offset_k ++ out[out_off, out_off+produced).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint8_t raw_at(const uint8_t *off, uint32_t off_len, const uint8_t *body, uint64_t blen,
                                          uint64_t i) {
    if (i < off_len) return off[i];
    i -= off_len;
    return i < blen ? body[i] : (uint8_t)0;
}

// Newline census: per chunk the '\n' count and whether the 4-newline grouping could differ
// from Parsing.Parse: an empty line anywhere ("\n\n" or raw[0]=='\n'), or a '\0' byte.  Those
// chunks go to ppg_parse_serial.  256 threads per chunk, 16 B per thread per 4 KiB tile.
extern "C" __global__ __launch_bounds__(256) void ppg_parse_count(
    const uint8_t *__restrict__ out, const PpgInflateJob *__restrict__ jobs, const PpgInflateResult *__restrict__ ires,
    const uint8_t *__restrict__ offs, const PpgOffsetRef *__restrict__ oref, PpgParseInfo *__restrict__ info, int nchunks) {
    const int k = blockIdx.x;
    if (k >= nchunks) return;
    const int t = threadIdx.x;
    __shared__ uint32_t red_nl[4], red_flag[4];
    const uint64_t g0 = jobs[k].out_off;
    const uint64_t blen = ires[k].status == 0 ? ires[k].produced : 0;
    const uint8_t *off = offs + oref[k].start;
    const uint32_t olen = oref[k].len;
    uint32_t nl = 0, flag = 0;
    // offset prefix (short): byte-wise; pair check spans into the body's first byte
    for (uint32_t i = t; i < olen; i += 256) {
        uint8_t c = off[i];
        uint8_t p = i ? off[i - 1] : (uint8_t)0;
        if (c == '\n') { nl++; if (i == 0 || p == '\n') flag = 1; }
        if (c == 0) flag = 1;
    }
    // body: 16-B aligned words over [g0, g0+blen)
    const uint64_t g1 = g0 + blen;
    const uint64_t a0 = g0 & ~15ull;
    for (uint64_t w = a0 + (uint64_t)t * 16; w < g1; w += 4096) {
        uint4 v = *(const uint4 *)(out + w);
        uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        // previous byte in raw order: out[g-1] inside the body; at g0 the last offset byte, or
        // "raw start" (a leading '\n' is itself an empty line) when the offset is empty
        uint8_t prev = w > g0 ? out[w - 1] : (uint8_t)0;
        const uint8_t at_g0 = olen ? off[olen - 1] : (uint8_t)'\n';
#pragma unroll
        for (int q = 0; q < 16; q++) {
            uint8_t c = (uint8_t)(wd[q >> 2] >> (8 * (q & 3)));
            uint64_t g = w + q;
            uint8_t p = g == g0 ? at_g0 : prev;
            if (g >= g0 && g < g1) {
                if (c == '\n') { nl++; if (p == '\n') flag = 1; }
                if (c == 0) flag = 1;
            }
            prev = c;
        }
    }
    // reduce over 256 threads (4 waves)
    for (int o = 32; o > 0; o >>= 1) { nl += __shfl_down(nl, o); flag |= __shfl_down(flag, o); }
    if ((t & 63) == 0) { red_nl[t >> 6] = nl; red_flag[t >> 6] = flag; }
    __syncthreads();
    if (t == 0) {
        uint32_t n = red_nl[0] + red_nl[1] + red_nl[2] + red_nl[3];
        uint32_t f = red_flag[0] | red_flag[1] | red_flag[2] | red_flag[3];
        info[k].newlines = n;
        info[k].serial = f;
        info[k].records = (ires[k].status == 0 && !f) ? n / 4 : 0;
    }
}

// Parsing.Parse (Parsing.cs:11-69) exactly, one lane per chunk that the census declined.
// mode 0: count into info[k].records; mode 1: also write descriptors at base[k].
extern "C" __global__ __launch_bounds__(64) void ppg_parse_serial(
    const uint8_t *__restrict__ out, const PpgInflateJob *__restrict__ jobs, const PpgInflateResult *__restrict__ ires,
    const uint8_t *__restrict__ offs, const PpgOffsetRef *__restrict__ oref, PpgParseInfo *__restrict__ info,
    const uint64_t *__restrict__ base, uint32_t *__restrict__ recs, int nchunks, int mode) {
    const int k = blockIdx.x;
    if (k >= nchunks || threadIdx.x != 0) return;
    if (!info[k].serial || ires[k].status != 0) return;
    const uint8_t *body = out + jobs[k].out_off;
    const uint64_t blen = ires[k].produced;
    const uint8_t *off = offs + oref[k].start;
    const uint32_t olen = oref[k].len;
    const uint64_t total = olen + blen;
    uint64_t i = 0, n = 0;
    uint32_t *dst = mode ? recs + 4 * base[k] : nullptr;
    while (i <= total) {
        if (raw_at(off, olen, body, blen, i) == 0) break;
        i++;
        uint64_t nn[4];
        bool ok = true;
        for (int f = 0; f < 4; f++) {
            if (f == 2) i++;   // skip '+' (Parsing.cs:30)
            for (;;) {
                uint8_t b = raw_at(off, olen, body, blen, i);
                if (b == '\n' || b == 0) break;
                i++;
            }
            if (raw_at(off, olen, body, blen, i) == 0) { ok = false; break; }
            nn[f] = i;
            i++;
        }
        if (!ok) break;
        if (dst) {
            dst[4 * n + 0] = (uint32_t)nn[0];
            dst[4 * n + 1] = (uint32_t)nn[1];
            dst[4 * n + 2] = (uint32_t)nn[2];
            dst[4 * n + 3] = (uint32_t)nn[3];
        }
        n++;
    }
    if (!mode) info[k].records = n;
}

// Exclusive scan of info[].records -> base[] and total (single workgroup; chunks <= a few 1e5).
extern "C" __global__ __launch_bounds__(1024) void ppg_scan_counts(const PpgParseInfo *__restrict__ info,
                                                                   uint64_t *__restrict__ base, uint64_t *__restrict__ total,
                                                                   int nchunks) {
    __shared__ uint64_t part[1024];
    const int t = threadIdx.x;
    const int per = (nchunks + 1023) / 1024;
    const int lo = t * per, hi = min(nchunks, lo + per);
    uint64_t s = 0;
    for (int k = lo; k < hi; k++) s += info[k].records;
    part[t] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        uint64_t v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = t ? part[t - 1] : 0;
    for (int k = lo; k < hi; k++) { base[k] = run; run += info[k].records; }
    if (t == 1023) *total = part[1023];
}

// Descriptors for fast-path chunks: newline m (m < 4*records) is field m%4 of record m/4.
extern "C" __global__ __launch_bounds__(256) void ppg_parse_emit(
    const uint8_t *__restrict__ out, const PpgInflateJob *__restrict__ jobs, const PpgInflateResult *__restrict__ ires,
    const uint8_t *__restrict__ offs, const PpgOffsetRef *__restrict__ oref, const PpgParseInfo *__restrict__ info,
    const uint64_t *__restrict__ base, uint32_t *__restrict__ recs, int nchunks) {
    const int k = blockIdx.x;
    if (k >= nchunks) return;
    if (info[k].serial || ires[k].status != 0) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    __shared__ uint32_t wsum[4];
    const uint64_t nrec = info[k].records;
    if (nrec == 0) return;
    const uint64_t limit = 4 * nrec;
    uint32_t *dst = recs + 4 * base[k];
    const uint8_t *off = offs + oref[k].start;
    const uint32_t olen = oref[k].len;
    const uint64_t g0 = jobs[k].out_off, g1 = g0 + ires[k].produced;
    uint64_t carry = 0;   // newlines before the current tile
    // offset prefix: a few hundred bytes -> thread 0 walks it
    if (olen) {
        if (t == 0) {
            uint64_t m = 0;
            for (uint32_t i = 0; i < olen; i++)
                if (off[i] == '\n') { if (m < limit) dst[m] = i; m++; }
            wsum[0] = (uint32_t)m;
        }
        __syncthreads();
        carry = wsum[0];
        __syncthreads();
    }
    const uint64_t a0 = g0 & ~15ull;
    for (uint64_t tile = a0; tile < g1; tile += 4096) {
        uint64_t w = tile + (uint64_t)t * 16;
        uint32_t mask = 0;
        if (w < g1) {
            uint4 v = *(const uint4 *)(out + w);
            uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 16; q++) {
                uint8_t c = (uint8_t)(wd[q >> 2] >> (8 * (q & 3)));
                uint64_t g = w + q;
                if (c == '\n' && g >= g0 && g < g1) mask |= 1u << q;
            }
        }
        uint32_t c = (uint32_t)__popc(mask);
        // wave inclusive scan
        uint32_t inc = c;
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        if (lane == 63) wsum[wv] = inc;
        __syncthreads();
        uint32_t before = 0, tile_total = 0;
        for (int q = 0; q < 4; q++) { if (q < wv) before += wsum[q]; tile_total += wsum[q]; }
        uint64_t m = carry + before + inc - c;
        while (mask) {
            int q = __ffs(mask) - 1;
            mask &= mask - 1;
            if (m < limit) dst[m] = (uint32_t)(olen + (w + q - g0));
            m++;
        }
        carry += tile_total;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// Host-side launchers (called from ppg_api.cpp; keep <<<>>> inside this translation unit).
// ------------------------------------------------------------------------------------------
size_t ppg_inflate_lds_bytes() { return sizeof(InflateLds); }

hipError_t ppg_launch_inflate(hipStream_t s, const uint32_t *comp, uint64_t nwords, const PpgInflateJob *jobs,
                              const uint8_t *dicts, uint8_t *out, PpgInflateResult *res, int njobs) {
    if (njobs <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_inflate_kernel, dim3(njobs), dim3(64), sizeof(InflateLds), s, comp, nwords, jobs, dicts,
                       out, res, njobs);
    return hipGetLastError();
}

hipError_t ppg_launch_parse_count(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                  const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                  PpgParseInfo *info, uint64_t *base, uint64_t *total, int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_parse_count, dim3(n), dim3(256), 0, s, out, jobs, ires, offs, oref, info, n);
    hipLaunchKernelGGL(ppg_parse_serial, dim3(n), dim3(64), 0, s, out, jobs, ires, offs, oref, info,
                       (const uint64_t *)nullptr, (uint32_t *)nullptr, n, 0);
    hipLaunchKernelGGL(ppg_scan_counts, dim3(1), dim3(1024), 0, s, info, base, total, n);
    return hipGetLastError();
}

hipError_t ppg_launch_parse_emit(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                 const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                 PpgParseInfo *info, const uint64_t *base, uint32_t *recs, int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_parse_emit, dim3(n), dim3(256), 0, s, out, jobs, ires, offs, oref, info, base, recs, n);
    hipLaunchKernelGGL(ppg_parse_serial, dim3(n), dim3(64), 0, s, out, jobs, ires, offs, oref, info, base, recs, n, 1);
    return hipGetLastError();
}
