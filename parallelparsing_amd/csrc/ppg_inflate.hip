// ppg_inflate.hip — gfx950 (MI355X / CDNA4) DEFLATE inflate for checkpoint chunks.
//
// Replaces the zlib calls of Core.ExtractDeflateIndex (Decompressor/Core.cs:133-192):
// inflateInit2(-15) + inflatePrime(from.Bits) + inflateSetDictionary(from.Window, 32768) +
// inflate(Z_NO_FLUSH) until to.Output - from.Output bytes exist.  One 64-lane wavefront decodes
// one chunk; chunks are independent because every Point carries its 32 KiB history.
//
// DEFLATE is a serial bit stream, and a single wave issues roughly one instruction per ~8
// cycles on gfx950, so the kernel is organised to need few instructions per token and to keep
// many waves per CU:
//   * speculative lane-parallel decode: in each round every lane decodes one whole token
//     (litlen code, length extra bits, distance code, distance extra bits) as if a token
//     started at bit bp + lane, using 10/8-bit LDS root tables whose entries are laid out for
//     single-op extraction; a scalar walk then follows the real chain of tokens through the
//     lanes (lane s -> lane s + bits(s)), recording each token at its output offset;
//   * byte-parallel emit: each lane produces one output byte of the round (its token found by
//     mask + clz, the token's info fetched with ds_bpermute); sources inside the round are
//     resolved by pointer doubling, so one ds_write commits up to 64 bytes;
//   * codes longer than the root tables, end-of-block and invalid codes end the walk and are
//     decoded bit-serially (canonical decode from the per-length counts);
//   * the compressed stream streams into an LDS ring by global_load_lds (two segments ahead) and
//     lanes read their words from it directly;
//   * history is an LDS ring of 2^RB bytes (4-32 KiB) indexed by the GLOBAL output
//     address; references further back read the already flushed output (or the Point's window)
//     from HBM; completed 4 KiB units leave the ring as 16-B-per-lane coalesced stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <type_traits>
#include "ppg_device.h"
#include "ppg_huffman.h"
#include <atomic>
#include <mutex>
#define PPG_SORT_SLOT 320   // u16 per wave in global scratch: litlen sorted symbols 288, distance 32

// CreateIndex pass 1 (IX): each job's output lives in a ring of 64 Ki positions of the out buffer
// (only the last 32 KiB + REACH are ever read back).  Pass 1 does not know a piece's starting
// history, so its output is SYMBOLIC, 16 bits per position: 0x8000 | byte for a byte the piece's
// own literals determine, or i (0..32767) for a copy of byte i of the unknown 32 KiB history
// (position i - 32768) -- one decode gives what two decodes over two synthetic histories gave
// before r03; ppg_resolve_kernel turns the tails into exact histories.
#define IX_RING_BYTES 65536u
#define IX_RING_MASK (IX_RING_BYTES - 1u)
// Wave priority (s_setprio) by phase of the token round: 2 for the serial walk, 1 after it until
// the round's bytes are written and through the round's tail (pos/carry/flush), 0 again before the
// next round's decode.  A wave that has walked its round finishes it ahead of waves still decoding
// theirs: the walk and the emit are one serial chain of dependent LDS / lane / far-load latencies,
// the decode is VALU-dense and latency-tolerant.  Measured on the 50 GB step (tools/ab_bench.sh,
// r02): none 840.4 ms; walk 2: 815-818; walk 2 + emit 1: 794.7; + tail: 793.3; walk 1 + emit 1:
// 795.2; decode 1 as well: 846.4 (priority on the decode costs what it gains).  The other serial
// stretches -- a bit-serial token (long code, end-of-block) and a dynamic block header -- run at 2:
// 810.1 -> 805.9 ms (r02, near noise).  (r03 re-tried emit 2 / walk 3: no gain,
// profiles/r03_ab_walk_prio_variants.txt.)

template <int RB, int LBT, typename RingT = uint8_t>
struct __attribute__((aligned(16))) InflateLds {
    // first: the decode's five-word reads address it with ds_read2 offsets (8-bit dword fields)
    uint32_t stream[132];          // compressed words: segment g (32 words) at slot g & 3; [128,132) mirror [0,4)
    // bytes (DecompressAll) or 16-bit symbols (CreateIndex pass 1)
    RingT ring[1u << RB];
    union {                        // the code-length code is dead once the litlen table is built
        uint32_t lit[1 << LBT];
        uint32_t cl[1 << CB];
    };
    uint32_t dst[1 << DB];
    // (the canonical codes' sorted symbols are in global scratch: see ppg_inflate_kernel)
    uint8_t lens[320];
    uint32_t cen[8];               // newline census: count, previous byte was '\n', PPG_PF_* flags, cap, shift, dst
    uint16_t dsort[32];            // the distance code's sorted symbols (bit-serial distance codes read them here, r06)
};

#ifdef PPG_IX_STATS
// diagnostic build only (EXTRA=-DPPG_IX_STATS): CreateIndex pass 1's history-symbol output -- how
// many output bytes are copies of the piece's unknown starting history, and how far into the piece
// the last one lies ([0] symbols, [1] sum of last positions + 1, [2] bytes, [3] jobs, [4..13] jobs
// by last position / bytes in tenths, [14] the largest last position)
__device__ unsigned long long ppg_ixstat[16];
#endif

#ifdef PPG_STAMPS
// diagnostic build only (EXTRA=-DPPG_STAMPS): s_memtime stamps at the phase boundaries of every
// token round, summed per wave and added to these totals at the end of each chunk; the launcher
// prints them (cycles per phase, rounds) after each launch.  Perturbs the schedule (+~10%).
// [0..7]: the general rounds (one_round); [8..15]: the pipelined rounds (hot_pipe, r05)
__device__ unsigned long long ppg_stamp_acc[25];
// [15..24] (r06): per-wave totals over the whole job -- wave cycles, bit-serial tokens (cycles,
// count), flushes + census (cycles, count), block headers + table builds (cycles, count), jobs
#define PPG_STAMP(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#else
#define PPG_STAMP(t)
#endif

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// v_writelane_b32 (value, lane, old) — the LLVM intrinsic, not exposed as a clang builtin
extern "C" __device__ int llvm_writelane(int, int, int) __asm("llvm.amdgcn.writelane");

__device__ __forceinline__ uint32_t bperm(uint32_t byte_addr, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)byte_addr, (int)v);
}

// Compressed stream of one chunk: word i (chunk-relative) is base[i].  Words move to an LDS ring
// of four 32-word segments by global_load_lds (straight to LDS, no VGPR in flight).  While the
// decoder reads segment g, segments g and g+1 are resident and g+2 is loading; entering g+1
// issues g+3 and waits for everything but that newest load (s_waitcnt vmcnt(1)) — once per
// 128 B of input.  The compiler does not track LDS-DMA, so every wait is explicit.
struct Reader {
    const uint32_t *base;
    uint32_t nw;            // readable words from base (>= 1)
    uint32_t sg;            // segment the decoder is in
    uint32_t wi;            // next word to append to bb
    uint64_t bb;            // bit buffer, LSB = next bit
    uint32_t bn;            // valid bits in bb
};

// global_load_lds_dword as inline asm: with the builtin the compiler waits for the DMA (vmcnt) before
// every later LDS read that may alias the ring — each round would stall on the prefetch issued two
// segments ahead and on any pending output stores.  Invisible to the compiler, the DMA is ordered
// only by st_enter's explicit s_waitcnt; an untracked VMEM op can only make the compiler's own
// vmcnt waits stricter, never looser.  (s_nop: SALU write of M0 -> LDS DMA needs one wait state.)
__device__ __forceinline__ void lds_dma_dword(const uint32_t *src, const uint32_t *lds_base) {
    asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "{m0}"((uint32_t)(uintptr_t)lds_base)
                 : "memory");
}

__device__ __forceinline__ void st_issue(const Reader &r, uint32_t *stream, uint32_t g, int lane) {
    const uint32_t i = min(g * 32 + (uint32_t)lane, r.nw - 1);   // past the end: any valid word
    if (lane < 32) lds_dma_dword(r.base + i, stream + (g & 3) * 32);
    // slot 0's first words again after slot 3, so a lane's consecutive words never wrap
    if ((g & 3) == 0 && lane < 4) lds_dma_dword(r.base + i, stream + 128);
}

// make segments g and g+1 resident (g+2 loading).  g == sg - 1 is resident too (the bit reader
// runs up to two words ahead of the decode position and may have entered sg already).
__device__ __forceinline__ void st_enter(Reader &r, uint32_t *stream, uint32_t g, int lane) {
    if (g == r.sg || g + 1 == r.sg) return;
    if (g != r.sg + 1) {
        st_issue(r, stream, g, lane);
        st_issue(r, stream, g + 1, lane);
    }
    st_issue(r, stream, g + 2, lane);
    r.sg = g;
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
}

__device__ __forceinline__ uint32_t rd_word(Reader &r, uint32_t *stream, uint32_t w, int lane) {
    st_enter(r, stream, w >> 5, lane);
    return uni(stream[w & 127]);
}

// position the bit buffer at chunk-relative bit `bit`
__device__ __forceinline__ void rd_seek(Reader &r, uint32_t *stream, uint32_t bit, int lane) {
    r.wi = bit >> 5;
    const uint32_t w = rd_word(r, stream, r.wi, lane);
    r.wi++;
    const uint32_t sh = bit & 31;
    r.bb = (uint64_t)(w >> sh);
    r.bn = 32 - sh;
}

// guarantees bn >= 32
__device__ __forceinline__ void rd_refill(Reader &r, uint32_t *stream, int lane) {
    if (r.bn <= 32) {
        const uint32_t w = rd_word(r, stream, r.wi, lane);
        r.wi++;
        r.bb |= (uint64_t)w << r.bn;
        r.bn += 32;
    }
}

__device__ __forceinline__ uint32_t rd_pos(const Reader &r) { return r.wi * 32 - r.bn; }

// Ring bytes of global output addresses [glo, ghi) -> out; unaligned head/tail singly, the
// 16-B-aligned middle as ds_read_b128 + global_store_dwordx4 (1 KiB per wave instruction).
template <int RB>
__device__ __forceinline__ void flush_range(const uint8_t *ring, uint8_t *out, uint64_t glo, uint64_t ghi, int lane) {
    constexpr uint64_t RM = (1ull << RB) - 1;
    if (ghi <= glo) return;
    const uint64_t a = (glo + 15) & ~15ull, z = ghi & ~15ull;
    if (a >= z) {
        for (uint64_t g0 = glo; g0 < ghi; g0 += 64) {
            const uint64_t g = g0 + lane;
            if (g < ghi) out[g] = ring[g & RM];
        }
        return;
    }
    if (lane < (int)(a - glo)) out[glo + lane] = ring[(glo + lane) & RM];
    if (lane < (int)(ghi - z)) out[z + lane] = ring[(z + lane) & RM];
    for (uint64_t g0 = a; g0 < z; g0 += 1024) {
        const uint64_t g = g0 + (uint64_t)lane * 16;
        if (g < z) {
            uint4 v = *(const uint4 *)(ring + (g & RM));
            *(uint4 *)(out + g) = v;
        }
    }
}

// flush_range for CreateIndex pass 1's 16-bit symbols: ring positions [glo, ghi) -> out16 (8 per
// 16-B store)
template <int RB>
__device__ __forceinline__ void flush_range_sym(const uint16_t *ring, uint16_t *out, uint64_t glo, uint64_t ghi,
                                                int lane) {
    constexpr uint64_t RM = (1ull << RB) - 1;
    if (ghi <= glo) return;
    const uint64_t a = (glo + 7) & ~7ull, z = ghi & ~7ull;
    if (a >= z) {
        for (uint64_t g0 = glo; g0 < ghi; g0 += 64) {
            const uint64_t g = g0 + lane;
            if (g < ghi) out[g] = ring[g & RM];
        }
        return;
    }
    if (lane < (int)(a - glo)) out[glo + lane] = ring[(glo + lane) & RM];
    if (lane < (int)(ghi - z)) out[z + lane] = ring[(z + lane) & RM];
    for (uint64_t g0 = a; g0 < z; g0 += 512) {
        const uint64_t g = g0 + (uint64_t)lane * 8;
        if (g < z) *(uint4 *)(out + g) = *(const uint4 *)(ring + (g & RM));
    }
}

// ---- FASTQ newline census, fused into the output flush (DecompressAll; Parsing.cs:11-69) ----
// Every flushed byte passes here once, in output order, as up to 16 bytes per lane (lanes in
// increasing position, contiguous).  Per chunk it counts '\n', stores each newline's raw index
// (the record descriptors of SURVEY A.3 R-P3 are newlines 4j..4j+3), and flags what makes the
// 4-newline grouping differ from the serial state machine: an empty line (a '\n' right after a
// '\n', or raw[0] == '\n') or a NUL byte.  Filler bytes ('A') pad lanes that hold fewer bytes.
#define PPG_FILL 0x41414141u

// 0x80 in every byte of x that is zero, exactly (no borrow between bytes)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}

// bit j = byte j of the 16-byte little-endian word (w0..w3) is '\n'
__device__ __forceinline__ uint32_t nl_mask16(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    const uint32_t n0 = zero_bytes(w0 ^ 0x0A0A0A0Au) >> 7, n1 = zero_bytes(w1 ^ 0x0A0A0A0Au) >> 7;
    const uint32_t n2 = zero_bytes(w2 ^ 0x0A0A0A0Au) >> 7, n3 = zero_bytes(w3 ^ 0x0A0A0A0Au) >> 7;
    // bytes are 0/1 now: a dot product with (1,2,4,8) / (16,32,64,128) packs four of them
    const uint32_t lo = __builtin_amdgcn_udot4(n1, 0x80402010u, __builtin_amdgcn_udot4(n0, 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(n3, 0x80402010u, __builtin_amdgcn_udot4(n2, 0x08040201u, 0u, false), false);
    return lo | (hi << 8);
}

// inclusive prefix sum over the wave (DPP row shifts + row broadcasts, GFX9 encodings)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return x;
}

struct CensusOut {
    uint32_t *dst;          // nls + nl_off
    uint32_t cap;           // nl_cap
    uint32_t shift;         // raw_shift
};

// One census step: lanes [0, nact) hold bytes at chunk positions p_lane + j; `lastbit` = index of
// a lane's last byte (15 for 16-byte lanes, 0 for single bytes); state in LDS (cen).
__device__ __forceinline__ void census_step(uint32_t *cen, const CensusOut &co, uint32_t w0, uint32_t w1, uint32_t w2,
                                            uint32_t w3, uint32_t p_lane, uint32_t lastbit, uint32_t nact, int lane) {
    const uint32_t m = nl_mask16(w0, w1, w2, w3);
    const uint32_t z = zero_bytes(w0) | zero_bytes(w1) | zero_bytes(w2) | zero_bytes(w3);
    const uint64_t L = __ballot((m >> lastbit) & 1u);   // lanes whose last byte is '\n'
    const uint64_t F = __ballot(m & 1u);                // lanes whose first byte is '\n'
    const uint64_t B = __ballot((m & (m << 1)) != 0u);
    const uint64_t Z = __ballot(z != 0u);
    uint32_t cnt = uni(cen[0]);
    const uint32_t prevnl = uni(cen[1]);
    uint32_t flags = uni(cen[2]);
    if (B | Z | (F & ((L << 1) | prevnl))) flags |= PPG_PF_SERIAL;
    if (Z) flags |= PPG_PF_NUL;
    const uint32_t c = (uint32_t)__builtin_popcount(m);
    const uint32_t incl = wave_incl_scan(c);
    const uint32_t total = rdlane(incl, 63);
    if (total) {
        uint32_t idx = cnt + incl - c;
        uint32_t mm = m;
        while (__ballot(mm != 0u)) {
            if (mm) {
                const uint32_t b = (uint32_t)__builtin_ctz(mm);
                mm &= mm - 1u;
                if (idx < co.cap) ((__attribute__((address_space(1))) uint32_t *)co.dst)[idx] = co.shift + p_lane + b;
                idx++;
            }
        }
        cnt += total;
        if (cnt > co.cap) flags |= PPG_PF_OVERFLOW;
    }
    if (lane == 0) {
        cen[0] = cnt;
        cen[1] = (uint32_t)(L >> (nact - 1)) & 1u;
        cen[2] = flags;
    }
}

__device__ __forceinline__ CensusOut census_out(const uint32_t *cen) {
    CensusOut co;
    co.cap = uni(cen[3]);
    co.shift = uni(cen[4]);
    co.dst = (uint32_t *)(((uint64_t)uni(cen[6]) << 32) | uni(cen[5]));
    return co;
}

// flush_range + census for DecompressAll chunks: chunk positions [lo, hi) at out + out_off, as
// steps of either aligned 16-B words (up to 1 KiB) or single bytes (an unaligned head, a tail
// under 16 B), in output order.  One census_step per step: a single inlined instance per call
// site.  The census parameters live in LDS (cen[3..6]), not in SGPRs the token loop keeps.
template <int RB>
__device__ __forceinline__ void flush_census(const uint8_t *ring, uint8_t *out, uint64_t out_off, uint32_t lo,
                                             uint32_t hi, int lane, uint32_t *cen) {
    constexpr uint32_t RM = (1u << RB) - 1;
    const CensusOut co = census_out(cen);
    for (uint32_t p = lo; p < hi;) {
        const uint64_t g = out_off + p;
        const uint32_t left = hi - p;
        const uint32_t head = (uint32_t)(-g & 15);
        uint32_t w0 = PPG_FILL, w1 = PPG_FILL, w2 = PPG_FILL, w3 = PPG_FILL, lastbit, nact;
        if (head == 0 && left >= 16) {
            nact = min(left / 16, 64u);
            if ((uint32_t)lane < nact) {
                const uint4 v = *(const uint4 *)(ring + ((uint32_t)(g + 16 * lane) & RM));
                *(uint4 *)(out + g + 16 * lane) = v;
                w0 = v.x; w1 = v.y; w2 = v.z; w3 = v.w;
            }
            lastbit = 15;
            nact *= 16;
        } else {
            nact = min(head ? head : 64u, left);
            if ((uint32_t)lane < nact) {
                const uint8_t c = ring[(uint32_t)(g + lane) & RM];
                out[g + lane] = c;
                w0 = (PPG_FILL & ~255u) | c;
            }
            lastbit = 0;
        }
        census_step(cen, co, w0, w1, w2, w3, p + (lastbit ? 16 : 1) * (uint32_t)lane, lastbit,
                    lastbit ? nact / 16 : nact, lane);
        p += nact;
    }
}

// Byte at chunk position p older than the ring: the flushed output (p >= 0; this wave's own
// earlier stores — a wave's accesses to one address are ordered) or the Point's window.  Read as
// an aligned dword from a uniform base + 32-bit lane offset (global_load saddr form; never merged
// with an LDS byte load into a flat load).  ob: out + (out_off & ~3), oa: out_off & 3.
// IX (CreateIndex pass 1): the job's output is a 64 KiB ring, position p at ob[p & 0xFFFF].
template <bool IX = false, uint32_t IXM = IX_RING_MASK>
__device__ __forceinline__ uint32_t far_byte(const uint8_t *ob, uint32_t oa, const uint8_t *dict, int32_t p) {
    if constexpr (IX) {   // 16-bit symbols: the job's ring (IXM; ~0: its whole output), or the history index itself
        if (p >= 0) return ((const uint16_t *)ob)[(uint32_t)p & IXM];
        return 32768u + (uint32_t)p;
    } else {
        // the two loads differ in width so the compiler cannot fold them into one per-lane base select
        if (p >= 0) {
            const uint32_t q = oa + (uint32_t)p;
            return (*(const uint32_t *)(ob + (q & ~3u)) >> (8 * (q & 3))) & 255u;
        }
        return dict[32768u + (uint32_t)p];   // p >= -32768; only the chunk's first 32 KiB
    }
}

// One dword per lane from a uniform base + 32-bit lane offset, as global_load_dword's saddr form,
// waited for in the same asm statement (so no copy of the register can be read while the load is
// in flight).  Written out because the compiler turns the emit's far-byte load into exec-mask
// juggling (~9 SALU per round) or a 64-bit per-lane address.  The wait also covers the stream's
// LDS-DMA issued before it, as any vmcnt wait here did.
// No wait states precede the load: the base pair must not be written by a VALU (a spill restore)
// just before it -- tools/hazard_lint.py checks the compiled kernel for that at every build (with
// amdgpu_num_sgpr(64) the base was spilled and the load faulted; padding costs 0.6%).
__device__ __forceinline__ uint32_t far_load(const uint8_t *base, uint32_t off) {
    uint32_t v;
    asm volatile("global_load_dword %0, %1, %2\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(off), "s"(base) : "memory");
    return v;
}
// the byte itself (DecompressAll's emit): no alignment mask, no bit-field extract (r03 v4:
// 707 -> 698.5 ms per 50 GB step, same-box A/B)
__device__ __forceinline__ uint32_t far_load_u8(const uint8_t *base, uint32_t off) {
    uint32_t v;
    asm volatile("global_load_ubyte %0, %1, %2\n\ts_waitcnt vmcnt(0)" : "=&v"(v) : "v"(off), "s"(base) : "memory");
    return v;
}

// One LZ77 copy of n bytes from dist back, at chunk position pos (all 64 lanes, uniform args).
template <int RB, bool IX, typename RingT, uint32_t IXM = IX_RING_MASK>
__device__ __forceinline__ void copy_match(RingT *ring, const uint8_t *ob, uint32_t oa, const uint8_t *dict,
                                           uint32_t rb0, uint32_t pos, uint32_t dist, uint32_t n, int lane) {
    constexpr uint32_t RM = (1u << RB) - 1;
    constexpr uint32_t REACH = (1u << RB) - 64;   // ring bytes a reference may use (see the emit)
    const uint32_t dst0 = rb0 + pos;   // ring slot of the first output byte
    if (dist + n <= REACH) {
        // source entirely in the ring and never overwritten by this copy; every source byte
        // precedes pos, so no 64-byte group reads another group's output
        const uint32_t src0 = dst0 - dist;
        if (dist >= n) {
            for (uint32_t j0 = 0; j0 < n; j0 += 64) {
                const uint32_t j = j0 + lane;
                if (j < n) ring[(dst0 + j) & RM] = ring[(src0 + j) & RM];
            }
        } else {
            // overlapping run: byte j repeats byte j mod dist
            for (uint32_t j0 = 0; j0 < n; j0 += 64) {
                const uint32_t j = j0 + lane;
                if (j < n) ring[(dst0 + j) & RM] = ring[(src0 + j % dist) & RM];
            }
        }
    } else {
        // far reference (dist > REACH - n >= n)
        for (uint32_t j0 = 0; j0 < n; j0 += 64) {
            const uint32_t j = j0 + lane;
            if (j < n) {
                const uint32_t back = dist - j;                 // source = pos - back
                const int32_t rel = (int32_t)pos - (int32_t)back;
                uint32_t v;
                if (back + n <= REACH) v = ring[(dst0 - back) & RM];
                else v = far_byte<IX, IXM>(ob, oa, dict, rel);
                ring[(dst0 + j) & RM] = (RingT)v;
            }
        }
    }
}

// One speculative token from the 64 stream bits (lo, hi) at some bit offset, decoded with the
// root tables.  Token word: [7:0] the token's bits, [16:8] output bytes (1: literal), [31:17]
// distance - 1 (match) or 0x100 | byte (literal: then lane - 1 - field lies in [-512, -194]:
// negative and, for any ring >= 1 KiB, never "far", see the emit).  The walk adds whole words to
// its state (see Round), so [7:0] and [16:8] must not carry into each other: bits <= 48, bytes <= 258.
// A special token (a code the root tables do not resolve: end-of-block, invalid, long) is
// 128 | 0x100 << 17: bits 128 set bit 7 of the walk's candidate index, which ends the walk; 0
// bytes; the field keeps the emit's source for lanes past it negative and near.  Never 0 (the
// emit finds tokens by that).
template <int LBT>
__device__ __forceinline__ uint32_t spec_token(const uint32_t *lit, const uint32_t *dst, uint32_t lo, uint32_t hi,
                                               uint32_t lane) {
    // a literal's (or a special code's) root entry is already its token word; only a length
    // symbol's entry (bit 6) is assembled from the two tables (ppg_huffman.h, r03)
    const uint32_t e = lit[lo & ((1u << LBT) - 1)];
    // length entry: e >> 8 = [7:0] L + x, [16:8] length base; (e >> 8) - e has x in its low 5 bits
    const uint32_t e2 = e >> 8;
    const uint32_t xs = e2 - e;
    const uint32_t y = __builtin_amdgcn_alignbit(hi, lo, e2);      // past the code and its extra bits
    uint32_t tke;   // bits and bytes of the length (one v_lshl_add; the compiler split it in two)
    asm("v_lshl_add_u32 %0, %1, 8, %2" : "=v"(tke) : "v"(__builtin_amdgcn_ubfe(lo, e, xs)), "v"(e2));
    const uint32_t d = dst[y & ((1u << DB) - 1)];
    const uint32_t dm1 = (d >> 16) + __builtin_amdgcn_ubfe(y, d, d >> 10);
    const uint32_t tlen = tke + ((d >> 5) & 31) + (dm1 << 17);
    const uint32_t lm = (uint32_t)((int32_t)(e << 25) >> 31);       // bit 6: a length symbol
    const uint32_t sd = (uint32_t)((int32_t)d >> 31);
    uint32_t t2, tok;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(t2) : "v"(sd), "v"(PPG_SPECIAL_TOKEN), "v"(tlen));
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(tok) : "v"(lm), "v"(t2), "v"(e));
    return tok;
}
// The walk loop of the decoder (see Round) over both 64-candidate spans in one asm block: per
// token v_readlane (candidate X[5:0]), v_writelane (at output offset (X >> 8)[5:0]), one s_add,
// and s_and's SCC as the loop test; span b (candidates 64..127, X rebased by -64, half = 64) only
// when span a ended at s >= 64 with output left and no special token (s_and's SCC again).  Written
// out because the compiler adds an s_cmp_eq 0 after each s_and (one more SALU per token, and SALU
// issue is what bounds this kernel); one block for both spans (r04: 642.3 -> 638.8 ms per 50 GB
// step, same box, profiles/r04v2_ab_walk2_cw0_prio.json).  t: the last token word walked.
__device__ __forceinline__ void walk2_asm(uint32_t va, uint32_t vb, uint32_t &vtin, uint32_t &X, uint32_t &t,
                                          uint32_t &half) {
    uint32_t tmp;   // (the order is the compiler's own hazard-clean one for these instructions)
    // each span's loop unrolled by two: one taken branch per two tokens (r04, on the pipelined
    // kernel: 559.5 -> 553.8 ms, profiles/r04o_ab_lean_unrolled.json)
    asm volatile(
        "1:\n\t"
        "v_readlane_b32 %[t], %[va], %[X]\n\t"
        "s_lshr_b32 m0, %[X], 8\n\t"
        "s_add_u32 %[X], %[t], %[X]\n\t"
        "s_and_b32 %[tmp], %[X], 0x1c0c0\n\t"
        "v_writelane_b32 %[vtin], %[t], m0\n\t"
        "s_cbranch_scc1 4f\n\t"
        "v_readlane_b32 %[t], %[va], %[X]\n\t"
        "s_lshr_b32 m0, %[X], 8\n\t"
        "s_add_u32 %[X], %[t], %[X]\n\t"
        "s_and_b32 %[tmp], %[X], 0x1c0c0\n\t"
        "v_writelane_b32 %[vtin], %[t], m0\n\t"
        "s_cbranch_scc0 1b\n"
        "4:\n\t"
        "s_mov_b32 %[h], 0\n\t"
        "s_and_b32 %[tmp], %[X], 0x1c080\n\t"
        "s_cbranch_scc1 3f\n\t"
        "s_sub_u32 %[X], %[X], 64\n\t"
        "s_mov_b32 %[h], 64\n"
        "2:\n\t"
        "v_readlane_b32 %[t], %[vb], %[X]\n\t"
        "s_lshr_b32 m0, %[X], 8\n\t"
        "s_add_u32 %[X], %[t], %[X]\n\t"
        "s_and_b32 %[tmp], %[X], 0x1c0c0\n\t"
        "v_writelane_b32 %[vtin], %[t], m0\n\t"
        "s_cbranch_scc1 3f\n\t"
        "v_readlane_b32 %[t], %[vb], %[X]\n\t"
        "s_lshr_b32 m0, %[X], 8\n\t"
        "s_add_u32 %[X], %[t], %[X]\n\t"
        "s_and_b32 %[tmp], %[X], 0x1c0c0\n\t"
        "v_writelane_b32 %[vtin], %[t], m0\n\t"
        "s_cbranch_scc0 2b\n"
        "3:"
        : [vtin] "+v"(vtin), [X] "+s"(X), [t] "=&s"(t), [tmp] "=&s"(tmp), [h] "=&s"(half)
        : [va] "v"(va), [vb] "v"(vb)
        : "m0", "scc");
}
// the round loop's latch limit: 0 after a special token (bit 7 of the walk state), else lim -- as
// one opaque s_bitcmp1 + s_cselect, so the latch stays one s_cmp + s_cbranch (the compiler turned
// "spec ? 0 : lim" into 64-bit lane-mask logic: 5 SALU)
__device__ __forceinline__ uint32_t latch_limit(uint32_t x, uint32_t lim) {
    uint32_t r;
    asm("s_bitcmp1_b32 %1, 7\n\ts_cselect_b32 %0, 0, %2" : "=s"(r) : "s"(uni(x)), "s"(uni(lim)) : "scc");
    return r;
}

// (r03 tried a walk taking two tokens per step -- each candidate's following token gathered by one
// ds_bpermute per span, the v_readlane -> s_add -> v_readlane chain paid once per two tokens:
// 829.1 vs 802.0 ms; an unrolled two-token loop: 799.4 vs 802.4.  DESIGN.md §4.)

// IX = false: Core.ExtractDeflateIndex of checkpoint chunks (out_len bytes each).
// IX = true:  CreateIndex pass 1 (ppg_index_gpu.cpp): decode whole blocks from a candidate block
//             start until a block ends at or past stop_bit, recording every block end.
// SGPR budget: a wave holds ceil(sgpr/16)*16 + 16 of the SIMD's 800 SGPRs, so .sgpr_count <= 80 is
// needed for 8 waves per SIMD (97 gives 6; MI355X_MICROARCH.md, occupancy formula)
// r03 v4: the token rounds as an inner loop with one latch, and the emit's token-start address as
// one v_mad_i32_i24 -- together 694.5 -> 682.2 ms per 50 GB step (each alone: 695.1 / 701.0;
// profiles/r03_ab_latch_sj.txt).
// amdgpu_waves_per_eu(8, 8): the VGPRs held to 64 (r04: the round loop's carry state took the
// compiler to 65, 7 waves per SIMD)
// IXF (CreateIndex-style pass 1 with IX = true): each job's symbolic output is kept whole at
// out + 2 * out_off (J.out_len = its capacity in positions; past it the job fails) instead of a
// 64 Ki-position ring -- the lone-chunk Decompress materialises its pieces from it
// (ppg_materialize_kernel) instead of decoding them a second time
template <int RB, int LBT, bool IX, bool CEN, bool IXF = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(8, 8))) void ppg_inflate_kernel(const uint32_t *__restrict__ comp, uint64_t nwords,
                                                         const PpgInflateJob *__restrict__ jobs,
                                                         const uint8_t *__restrict__ dicts, uint8_t *__restrict__ out,
                                                         PpgInflateResult *__restrict__ res, int njobs,
                                                         PpgBlockEnd *__restrict__ blk, uint32_t *__restrict__ nls,
                                                         uint16_t *__restrict__ gsort) {
    constexpr uint32_t RING = 1u << RB;
    constexpr uint32_t RM = RING - 1;
    // flush unit: far references (older than REACH = RING - 64) must already be flushed; a round
    // adds at most 64 + 258 bytes, so UNIT <= RING - 386 keeps them flushed (see copy_match)
    constexpr uint32_t UNIT = RB >= 13 ? 4096u : RING / 2;
    static_assert(RB >= 10 && RB <= 15, "ring of 1..32 KiB");
    using RingT = typename std::conditional<IX, uint16_t, uint8_t>::type;   // IX: 16-bit symbols
    constexpr uint32_t IXM = IXF ? 0xFFFFFFFFu : IX_RING_MASK;             // IX output: ring or whole
    static_assert(!IXF || IX, "IXF is a pass-1 (IX) form");
    // static LDS: every address is a link-time constant the compiler folds into the instructions'
    // offsets (a dynamic extern array cost one v_add of its base per ring access, r03)
    __shared__ InflateLds<RB, LBT, RingT> S;
    const int lane = threadIdx.x;
    const int k = blockIdx.x;
    if (k >= njobs) return;
    // The canonical codes' sorted symbols (for the bit-serial path: long codes, end-of-block) live
    // in global scratch, PPG_SORT_SLOT per wave: their 640 B of LDS now hold a 2 KiB history ring
    // at 8 waves per SIMD (InflateLds<11, 8>: 4,976 B of the 5,120 a wave gets).  A table build
    // sorts into LDS that is free at that moment -- the distance table's for the litlen and
    // code-length codes, the dead code lengths' head for the distance code -- and copies the
    // result out once.  r05, one same-box A/B of the 50 GB step (profiles/r05zzb_ab_gsort.json):
    // 555.2 ms (1 KiB ring, sorted symbols in LDS) -> 533.3; the global sorted symbols alone (1 KiB
    // ring) 565.2, sorting straight into global memory 562.8 / 540.4 (r05zza).
    uint16_t *const lit_sorted = gsort + (size_t)k * PPG_SORT_SLOT;
    // (r06) the distance code's (30 symbols at most) stay in LDS: no global load per long distance code
    uint16_t *const dst_sorted = S.dsort;
    uint16_t *const lit_tmp = (uint16_t *)S.dst, *const cl_tmp = (uint16_t *)S.dst, *const dst_tmp = (uint16_t *)S.lens;
#ifdef PPG_STAMPS
    const uint64_t tk0 = __builtin_amdgcn_s_memtime();
    uint64_t sx_spec = 0, sx_nspec = 0, sx_flush = 0, sx_nflush = 0, sx_hdr = 0, sx_nhdr = 0, sx_hp = 0, sx_nhp = 0;
#endif
    const PpgInflateJob J = jobs[k];
    const uint64_t out_off = J.out_off;
    const uint32_t len = IX ? 0xFFFFFFFFu : (uint32_t)J.out_len;   // < 2^31: ppg_index_validate
    // IX: past this many positions the job is a runaway (a false start); IXF: its output's capacity
    const uint32_t ixcap = IXF ? (uint32_t)J.out_len : 0xF0000000u;
    const uint32_t rb0 = (uint32_t)out_off;         // ring slot of chunk position p: (rb0 + p) & RM
    const uint8_t *dict = dicts + J.dict_off;       // chunk position p < 0 is dict[32768 + p]
    // chunk position p >= 0 is ob[oa + p] (IX: 16-bit symbol ((uint16_t *)ob)[p & IX_RING_MASK])
    const uint8_t *ob = IX ? out + 2 * out_off : out + (out_off & ~3ull);
    const uint32_t oa = IX ? 0u : (uint32_t)(out_off & 3);

    if constexpr (IX) {
        // history symbols: position p in [-RING, 0) is history byte 32768 + p
        for (uint32_t w0 = 0; w0 < RING; w0 += 64) {
            const uint32_t w = w0 + lane;
            S.ring[(rb0 - RING + w) & RM] = (uint16_t)(32768u - RING + w);
        }
    } else {
        // history: the last RING bytes of the Point's window -> ring slots of positions [-RING, 0)
        for (uint32_t w0 = 0; w0 < RING / 4; w0 += 64) {
            const uint32_t w = w0 + lane;
            const uint32_t v = *(const uint32_t *)(dict + 32768 - RING + 4 * w);
            const uint32_t slot = rb0 - RING + 4 * w;
#pragma unroll
            for (int q = 0; q < 4; q++) S.ring[(slot + q) & RM] = (uint8_t)(v >> (8 * q));
        }
    }
    constexpr bool census = CEN && !IX;
    if (census && lane == 0) {
        const uint64_t d = (uint64_t)(uintptr_t)(nls + J.nl_off);
        S.cen[0] = 0;
        S.cen[1] = J.prev_byte == '\n';
        S.cen[2] = 0;
        S.cen[3] = J.nl_cap;
        S.cen[4] = J.raw_shift;
        S.cen[5] = (uint32_t)d;
        S.cen[6] = (uint32_t)(d >> 32);
    }
    __syncthreads();

    // chunk-relative compressed stream
    const uint64_t w0abs = (J.bit_start >> 5) & ~127ull;
    Reader r;
    r.sg = 0x7FFFFFF0u;   // nothing resident: the first seek loads
    r.base = comp + w0abs;
    r.nw = (uint32_t)min(nwords > w0abs ? nwords - w0abs : 1ull, 0xFFFFFFFFull);
    const uint32_t bit_limit = (uint32_t)min(J.bit_limit - w0abs * 32, 0xFFFFFFFFull);   // < 2^32 - 2^12: ppg_index_validate
    rd_seek(r, S.stream, (uint32_t)(J.bit_start - w0abs * 32), lane);

    // lane constants of the round loop
    const uint64_t lanes_le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);   // lanes <= this one

    uint32_t pos = 0;                                        // output bytes produced
    uint32_t fl_done = 0;                                    // flushed up to this position
    uint32_t fl_next = UNIT - (uint32_t)(out_off % UNIT);   // next global UNIT boundary
    int status = ST_OK, flags = 0, last = 0, in_block = 0;
    Canon clit = {0, 0, 0}, cdst = {0, 0, 0};   // per-lane canonical codes of the current block
    // flush of chunk positions [lo, hi) (never across a UNIT boundary except the plain case)
#ifdef PPG_IX_STATS
    uint64_t ix_unk = 0;
    uint32_t ix_last = 0;
#endif
    auto flush = [&](uint32_t lo, uint32_t hi) {
        if constexpr (IX) {
#ifdef PPG_IX_STATS
            for (uint32_t p0 = lo; p0 < hi; p0 += 64) {
                const uint32_t p = p0 + (uint32_t)lane;
                const uint64_t b = __ballot(p < hi && S.ring[(rb0 + p) & RM] < 0x8000u);
                ix_unk += (uint64_t)__popcll(b);
                if (b) ix_last = p0 + 64u - (uint32_t)__clzll(b);
            }
#endif
            const uint64_t g = out_off + (lo & IXM);
            flush_range_sym<RB>(S.ring, (uint16_t *)out, g, g + (hi - lo), lane);
        } else {
            if constexpr (census) {
                flush_census<RB>(S.ring, out, out_off, lo, hi, lane, S.cen);
            } else {
                flush_range<RB>(S.ring, out, out_off + lo, out_off + hi, lane);
            }
        }
    };
    uint32_t nblk = 0;
#ifdef PPG_STAMPS
    uint64_t sa_dec = 0, sa_walk = 0, sa_rd = 0, sa_far = 0, sa_dep = 0, sa_tail = 0, sa_rounds = 0, sa_farr = 0;
    uint64_t hs_dec = 0, hs_walk = 0, hs_look = 0, hs_fin = 0, hs_words = 0, hs_emit = 0, hs_rounds = 0;
#endif
#ifdef PPG_STATS
    // debug build only (EXTRA=-DPPG_STATS): per-chunk round / token / path counts, printed for the
    // first chunks (tools/ab_bench.sh-style runs; DESIGN.md quotes them)
    uint32_t st_rounds = 0, st_tokens = 0, st_spec = 0, st_short = 0, st_far = 0, st_dep = 0, st_dbl = 0,
             st_blit = 0, st_beob = 0, st_bmatch = 0;
#endif
    // IX: record a block end (chunk-relative bit e); false = stop decoding
    auto block_end = [&](uint32_t e) -> bool {
        if (nblk >= J.blk_cap) { flags |= PPG_FLAG_BLK_FULL; return false; }
        if (lane == 0) blk[J.blk_off + nblk] = PpgBlockEnd{w0abs * 32 + e, pos};
        nblk++;
        return w0abs * 32 + e < J.stop_bit;
    };


    while (pos < len && !last) {
        r.sg = uni(r.sg);
        r.wi = uni(r.wi);
        r.bb = uni64(r.bb);
        r.bn = uni(r.bn);
        pos = uni(pos);
        fl_done = uni(fl_done);
        fl_next = uni(fl_next);
        status = (int)uni((uint32_t)status);
#ifdef PPG_STAMPS
        const uint64_t th0 = __builtin_amdgcn_s_memtime();
#endif
        rd_refill(r, S.stream, lane);
        last = (int)br_take(r, 1);
        const uint32_t type = br_take(r, 2);
        if (type == 0) {
            // ---- stored block ----
            br_take(r, r.bn & 7);
            rd_refill(r, S.stream, lane);
            const uint32_t slen = br_take(r, 16), nlen = br_take(r, 16);
            if ((slen ^ 0xFFFFu) != nlen) { status = ST_DATA_ERROR; break; }
            const uint32_t bytepos = rd_pos(r) >> 3;
            const uint8_t *c8 = (const uint8_t *)r.base + bytepos;
            const uint32_t remain = min(slen, len - pos);
            if ((uint64_t)bytepos + remain > (uint64_t)r.nw * 4) { status = ST_DATA_ERROR; break; }
            uint32_t copied = 0;
            while (copied < remain) {
                const uint32_t piece = min(remain - copied, (uint32_t)UNIT);
                for (uint32_t j0 = 0; j0 < piece; j0 += 64) {
                    const uint32_t j = j0 + lane;
                    if (j < piece) S.ring[(rb0 + pos + j) & RM] = (RingT)((IX ? 0x8000u : 0u) | c8[copied + j]);
                }
                pos += piece;
                copied += piece;
                if (pos >= fl_next) {
                    flush(fl_done, fl_next);
                    fl_done = fl_next;
                    fl_next += UNIT;
                }
            }
            rd_seek(r, S.stream, (bytepos + copied) * 8, lane);
            if (copied < slen) break;   // output full mid-block (zlib stops at avail_out == 0)
            in_block = 0;
            if constexpr (IX) {
                if (!block_end((bytepos + copied) * 8)) break;
            }
            continue;
        }
        if (type == 3) { status = ST_DATA_ERROR; break; }
        if (type == 1) {
            // ---- fixed Huffman codes (RFC 1951 3.2.6) ----
            for (int s0 = 0; s0 < 320; s0 += 64) {
                const int s = s0 + lane;
                uint8_t L;
                if (s < 144) L = 8; else if (s < 256) L = 9; else if (s < 280) L = 7; else if (s < 288) L = 8;
                else L = 5;   // 288..319: the 32 distance codes
                S.lens[s] = L;
            }
            __syncthreads();
            build_table<LBT>(S.lens, 288, S.lit, &clit, lit_tmp, TAB_LIT, lane, lit_sorted);
            build_table<DB>(S.lens + 288, 32, S.dst, &cdst, dst_tmp, TAB_DST, lane, dst_sorted);
        } else {
            // ---- dynamic Huffman codes (RFC 1951 3.2.7) ----
            asm volatile("s_setprio 2");
            rd_refill(r, S.stream, lane);
            const uint32_t hlit = br_take(r, 5) + 257, hdist = br_take(r, 5) + 1, hclen = br_take(r, 4) + 4;
            if (hlit > 286 || hdist > 30) { status = ST_DATA_ERROR; break; }
            if (lane < 19) S.lens[lane] = 0;
            __syncthreads();
            for (uint32_t i = 0; i < hclen; i++) {
                rd_refill(r, S.stream, lane);
                const uint32_t v = br_take(r, 3);
                if (lane == 0) S.lens[c_clorder[i]] = (uint8_t)v;
            }
            __syncthreads();
            if (build_table<CB>(S.lens, 19, S.cl, nullptr, cl_tmp, TAB_CL, lane) != 0) { status = ST_DATA_ERROR; break; }
            uint32_t idx = 0;
            const uint32_t total = hlit + hdist;
            bool bad = false;
            while (idx < total) {
                rd_refill(r, S.stream, lane);
                const uint32_t e = uni(S.cl[(uint32_t)r.bb & ((1u << CB) - 1)]);
                const uint32_t L = e & 15;
                if (L == 0) { bad = true; break; }
                br_take(r, L);
                const uint32_t sym = e >> 8;
                uint32_t val = 0, rep = 1;
                if (sym < 16) { val = sym; }
                else if (sym == 16) {
                    if (idx == 0) { bad = true; break; }
                    val = uni(S.lens[idx - 1]);
                    rep = 3 + br_take(r, 2);
                } else if (sym == 17) { rep = 3 + br_take(r, 3); }
                else { rep = 11 + br_take(r, 7); }
                if (idx + rep > total) { bad = true; break; }
                for (uint32_t j0 = 0; j0 < rep; j0 += 64)
                    if (j0 + lane < rep) S.lens[idx + j0 + lane] = (uint8_t)val;
                idx += rep;
            }
            __syncthreads();
            if (bad) { status = ST_DATA_ERROR; break; }
            if (uni(S.lens[256]) == 0) { status = ST_DATA_ERROR; break; }   // no end-of-block code
            if (build_table<LBT>(S.lens, (int)hlit, S.lit, &clit, lit_tmp, TAB_LIT, lane, lit_sorted) != 0) { status = ST_DATA_ERROR; break; }
            if (build_table<DB>(S.lens + hlit, (int)hdist, S.dst, &cdst, dst_tmp, TAB_DST, lane, dst_sorted) != 0) { status = ST_DATA_ERROR; break; }
        }
        in_block = 1;
#ifdef PPG_STAMPS
        sx_hdr += __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(S.lit[lane]) - th0;
        sx_nhdr++;
#endif
        asm volatile("s_setprio 0");
        // once per block: tell the compiler the decoder state is wave-uniform (it cannot prove it
        // through the outer loop), so the token rounds keep it in SGPRs with scalar branches
        r.sg = uni(r.sg);
        r.wi = uni(r.wi);
        r.bb = uni64(r.bb);
        r.bn = uni(r.bn);
        pos = uni(pos);
        fl_done = uni(fl_done);
        fl_next = uni(fl_next);

        // ---- token rounds ----
        // A round emits at most 64 output bytes.  A match crossing that boundary is carried: its
        // remaining bytes open the next round as a token at output offset 0.  (Software pipelining
        // the next round's decode over this round's far loads measured no gain: at 8 waves per
        // SIMD the kernel is issue-bound, chiefly on SALU — see DESIGN.md.)
        uint32_t bp = rd_pos(r);
#ifdef PPG_STAMPS
        uint64_t st_w0 = 0;        // stamp: the round's spec tokens are decoded, the walk starts
#endif
        uint32_t cn = 0, cw = 0;   // carried: bytes left of the last round's last match, its token word

        // decode of the round starting at output position pos, stream bit bp, carry (cn, cw):
        // returns the token words placed at their output offsets (vtin), the output bytes the
        // round's tokens cover (off), the bit advance (adv), the last token word walked (tl: the
        // carry whenever the round's tokens cross 64 bytes) and the walk's final state (xr: bit 7 =
        // it stopped at a special token)
        struct Round { uint32_t vtin, off, adv, tl, xr; };
        // the five stream words a lane decodes from at bit bp (st_enter made their segments
        // resident): (bp >> 5) + (((bp & 31) + lane) >> 5) == (bp + lane) >> 5, in VALU only
        struct Words { uint32_t x0, x1, x2, x3, x4; };
        auto words = [&](uint32_t bp) -> Words {
            const uint32_t *sw = S.stream + __builtin_amdgcn_ubfe(bp + (uint32_t)lane, 5u, 7u);
            return Words{sw[0], sw[1], sw[2], sw[3], sw[4]};
        };
        // HOT: at least 322 output bytes are left (a round's tokens cover at most 63 + 258), so
        // neither the walk's stop nor the emitted bytes need the chunk's end, and pos >= 32768, so
        // no far source lies in the Point's window
        auto decode = [&](auto hot, uint32_t bp, uint32_t cn, uint32_t cw, uint32_t pos, const Words &W) -> Round {
            constexpr bool HOT = decltype(hot)::value;
            uint32_t s = 0, off = cn, t = 0, half = 0;
            uint32_t tl = cw, xr = 0;   // no walk (cn >= 64): the carried word stays
            // lane 0 unconditionally: with no carry (cn == 0) the walk's first token overwrites it
            uint32_t vtin = (uint32_t)llvm_writelane((int)cw, 0, 0);
            // the walk-less round (a carry of >= 64 bytes) is rare: laid out off the hot path, the walk
            // falls through into the emit (r06: -0.7% per 50 GB step, profiles/r06j_ab_layout.json)
            if (__builtin_expect(off < (HOT ? 64u : min(64u, len - pos)), 1)) {
                // the stream bits at bp + lane and bp + 64 + lane (five words per lane from the LDS
                // ring, read during the previous round's emit); v_alignbit reads only bits [4:0]
                const uint32_t o = bp + (uint32_t)lane;
                const uint32_t x0 = W.x0, x1 = W.x1, x2 = W.x2, x3 = W.x3, x4 = W.x4;
                // speculative tokens at every bit offset of the 128-bit span (two per lane)
                const uint32_t vta = spec_token<LBT>(S.lit, S.dst, __builtin_amdgcn_alignbit(x1, x0, o),
                                                     __builtin_amdgcn_alignbit(x2, x1, o), (uint32_t)lane);
                const uint32_t vtb = spec_token<LBT>(S.lit, S.dst, __builtin_amdgcn_alignbit(x3, x2, o),
                                                     __builtin_amdgcn_alignbit(x4, x3, o), (uint32_t)lane);

                // ---- walk the real token chain (wave-uniform): offset s -> s + bits(s) ----
                // Each token goes to the lane of its output offset (vtin).  The walk state is one
                // SGPR, X = s | off << 8 (+ carry-free garbage above bit 16 from the fields): a token
                // word adds its bits to s and its bytes to off in one s_add, and v_readlane /
                // v_writelane use only bits [5:0] of their lane select (checked on gfx950), so
                // X itself selects candidate s and X >> 8 output offset off.  The walk runs through
                // the first 64 offsets (vta), then the next 64 (vtb), and stops at a special token
                // (recorded with 0 bytes, harmlessly; s gains 128), past the span, or once no
                // further token can start inside the round's first min(64, len - pos) output bytes.
                // Per token: 2 VALU, 3 SALU, 1 branch.
                constexpr uint32_t STOP = 0x1C0C0u;   // s >= 64 (bits 7:6) or off >= 64 (bits 16:14)
                uint32_t X;
#ifdef PPG_STAMPS
                st_w0 = __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(vta ^ vtb);
#endif
                if (HOT || len - pos >= 64) {
                    X = off << 8;
                    asm volatile("s_setprio 2");
                    walk2_asm(vta, vtb, vtin, X, tl, half);
                    // the HOT rounds keep priority 2 through the token lookup (hot_pipe), then 0
                    if constexpr (!HOT) asm volatile("s_setprio 1");
                    off = (X >> 8) & 511u;
                } else {
                    const uint32_t cl = 64u - (len - pos);   // off < len - pos  <=>  off + cl < 64
                    X = (off + cl) << 8;
                    do {
                        t = rdlane(vta, X);
                        vtin = (uint32_t)llvm_writelane((int)t, (int)((X >> 8) - cl), (int)vtin);
                        X += t;
                    } while ((X & STOP) == 0u);
                    if ((X & (STOP & ~0x40u)) == 0u) {
                        X -= 64;
                        half = 64;
                        do {
                            t = rdlane(vtb, X);
                            vtin = (uint32_t)llvm_writelane((int)t, (int)((X >> 8) - cl), (int)vtin);
                            X += t;
                        } while ((X & STOP) == 0u);
                    }
                    off = ((X >> 8) & 511u) - cl;
                    tl = t;
                }
                xr = X;
                s = half + (X & 127u);   // bit offset of the next token (of the special one: bit 7 dropped)
            }
            return Round{vtin, off, s, tl, xr};
        };

        st_enter(r, S.stream, bp >> 10, lane);
        Words W = words(bp);
        // One round: decode + walk, then one output byte per lane.  Returns the walk's final state
        // (bit 7: a special token ended the round).
        // The general form of a round (the last 322 bytes of a chunk or piece, short chunks): the
        // round's far load waited for in the round.  The PPG_STAMPS / PPG_STATS diagnostics
        // instrument this form only (r04: every other round runs hot_pipe below).
        auto one_round = [&]() -> uint32_t {
            constexpr bool HOT = false;
            PPG_STAMP(t0);
            const Round R = decode(std::false_type{}, bp, cn, cw, pos, W);
            // the next round's stream words, read now: their LDS latency overlaps this round's
            // emit instead of opening the next round's chain of dependent LDS reads (r03)
            st_enter(r, S.stream, (bp + R.adv) >> 10, lane);
            W = words(bp + R.adv);
#ifdef PPG_STAMPS
            const uint64_t t1 = __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(R.vtin);
            if (st_w0 < t0) st_w0 = t1;   // no walk this round
            sa_dec += st_w0 - t0;
            sa_walk += t1 - st_w0;
            sa_rounds++;
#endif
#ifdef PPG_STATS
            st_rounds++;
            st_tokens += (uint32_t)__popcll(__ballot(R.vtin != 0));
            if (R.xr & 128u) st_spec++;
            if (R.off < 64) st_short++;
#endif
            const uint32_t tot = HOT ? R.off : min(R.off, len - pos);   // output bytes of the round's tokens
            const uint32_t rout = min(tot, 64u);          // ... emitted this round
            const uint64_t mo = __ballot(R.vtin != 0);    // token start offsets (never 0 words)
            // All 64 lanes write: lanes past rout leave garbage in the slots of positions
            // [pos + rout, pos + 64), which later rounds overwrite before use; the slots' previous
            // bytes (positions >= pos + rout - RING) are therefore never read from the ring —
            // references reach back at most RING - 64 bytes (REACH), older bytes come from HBM.
            {
                // 4 * (63 - clz) in one v_mad_i32_i24 (the compiler's form: shift + xor)
                uint32_t sj4;
                asm("v_mad_i32_i24 %0, %1, -4, %2" : "=v"(sj4) : "v"((uint32_t)__builtin_clzll(mo & lanes_le)), "s"(252u));
                const uint32_t inf = bperm(sj4, R.vtin);
                const int32_t jj = lane - 1 - (int32_t)(inf >> 17);   // source, relative to the round
                const uint32_t rv = S.ring[(rb0 + pos + (uint32_t)jj) & RM];
                uint32_t val;   // (IX: a literal is the symbol 0x8000 | byte; written apart, the DecompressAll
                                // instance's code is unchanged -- the folded "| 0" moved its schedule)
                if constexpr (IX) val = ((inf >> 8) & 511u) != 1u ? rv : (0x8000u | ((inf >> 17) & 255u));
                else val = ((inf >> 8) & 511u) != 1u ? rv : ((inf >> 17) & 255u);
                const bool far = jj < -(int32_t)(RING - 64);          // far (literals: jj >= -512)
                const uint64_t fm = __ballot(far);
#ifdef PPG_STATS
                if (fm) st_far++;
#endif
#ifdef PPG_STAMPS
                const uint64_t t2 = __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(val);
                sa_rd += t2 - t1;
#endif
                if (fm) {
                  {
                    // older than the ring: the flushed output (this wave's own earlier stores), as
                    // one saddr load for the whole wave (non-far lanes read out[0]: no exec
                    // juggling); references into the Point's window (first 32 KiB only) separately
                    const int32_t p = (int32_t)pos + jj;
                    const bool fo = far && p >= 0;
                    if constexpr (IX) {
                        const uint32_t q = 2u * ((uint32_t)p & IXM);
                        const uint32_t w = far_load(ob, fo ? (q & ~3u) : 0u);
                        val = fo ? __builtin_amdgcn_ubfe(w, q << 3, 16u) : val;
                    } else {
                        // one byte load at ob + oa + p (pos + oa is wave-uniform)
                        const uint32_t b = far_load_u8(ob, fo ? (uint32_t)jj + (pos + oa) : 0u);
                        val = fo ? b : val;
                    }
                    const bool fd = far && p < 0;
                    const uint64_t dm = fm & __ballot(p < 0);   // (a ballot of fd itself went through two VALU)
                    if (dm) {   // rare: the chunk's first 32 KiB
                        uint32_t db;
                        if constexpr (IX) db = 32768u + (uint32_t)p;          // the history symbol itself
                        else db = dict[fd ? 32768u + (uint32_t)p : 0u];       // p >= -32768
                        val = fd ? db : val;
                    }
                  }
                }
#ifdef PPG_STAMPS
                const uint64_t t3 = __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(val);
                sa_far += t3 - t2;
                sa_farr += fm ? 1 : 0;
#endif
                const bool dep = jj >= 0;                             // produced in this round
                if (__ballot(dep)) {
                    // chains inside the round (short distances): pointer doubling to a resolved byte
                    int32_t ptr = dep ? jj : lane;
#ifdef PPG_STATS
                    st_dep++;
#endif
                    for (;;) {
#ifdef PPG_STATS
                        st_dbl++;
#endif
                        const int32_t p2 = (int32_t)bperm((uint32_t)ptr << 2, (uint32_t)ptr);
                        if (!__ballot(p2 != ptr)) break;
                        ptr = p2;
                    }
                    val = bperm((uint32_t)ptr << 2, val);
                }
                S.ring[(rb0 + pos + lane) & RM] = (RingT)val;
#ifdef PPG_STAMPS
                const uint64_t t4 = __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(val);
                sa_dep += t4 - t3;
                st_w0 = t4;   // reused below: start of the round's tail
#endif
            }
            cn = tot - rout;
            // the walk's last token is the one crossing the round's 64 bytes whenever cn > 0: the
            // carry, as a match (bytes field 0) -- no lane read, no branch; unused when cn == 0
            cw = R.tl & ~(511u << 8);
            pos += rout;
            bp += R.adv;
            asm volatile("s_setprio 0");
            if constexpr (IX) {   // past the member, or runaway output (a false start)
                if (bp > bit_limit || pos > ixcap) { status = ST_DATA_ERROR; return 128u; }
            }
#ifdef PPG_STAMPS
            sa_tail += __builtin_amdgcn_s_memtime() + 0 * (uint64_t)bp - st_w0;
            st_w0 = 0;
#endif
            return R.xr;
        };
        // The HOT rounds software-pipelined (DecompressAll): a round's far load is issued at its
        // emit and consumed at the next round's, after that round's decode and walk (which do not
        // read the ring); the pending round is finished (far bytes merged, in-round chains resolved,
        // ring written) before the next emit reads the ring, and at the loop's exit.  The far load
        // (~1,000 cycles of a ~2,950-cycle round, PPG_STAMPS) now hides behind the next decode +
        // walk: 640.8 -> 575.8 ms per 50 GB step in one same-box A/B
        // (profiles/r04j_ab_pipelined_far.json).  (r02 tried the same on a kernel bound by SALU
        // issue: no gain.)
        // EARLY: the rounds of the chunk's (or piece's) first 32 KiB, where a far source may lie in the
        // Point's window (p < 0): its byte comes from the window (DecompressAll: a per-lane address
        // select) or is the history symbol itself (CreateIndex pass 1)
        auto hot_pipe = [&](auto early, uint32_t limh) -> uint32_t {
            constexpr bool EARLY = decltype(early)::value;
            // no "pending" test: the loop starts with a dummy pending round (no far, no chain
            // sources) whose 64 garbage bytes land in the slots of positions [pos, pos + 64),
            // which the first real round's finish overwrites before anything reads them; and no
            // far-lane ballot: the far load is issued every round (97% of rounds have a far lane)
            // -- together 567.5 -> 559.5 ms (profiles/r04o_ab_lean_unrolled.json)
            uint32_t p_val = 0, p_b = 0, p_pos = pos, lim_r;
            int32_t p_jj = -1;
            auto finish = [&]() {
                uint32_t val = p_val;
                if constexpr (IX) {   // CreateIndex pass 1: the 16-bit symbol in the loaded dword
                    const uint32_t q = 2u * ((p_pos + (uint32_t)p_jj) & IXM);
                    uint32_t fv = __builtin_amdgcn_ubfe(p_b, q << 3, 16u);
                    if constexpr (EARLY) {   // before the piece: the history symbol itself
                        const int32_t p = (int32_t)p_pos + p_jj;
                        fv = p < 0 ? 32768u + (uint32_t)p : fv;
                    }
                    val = p_jj < -(int32_t)(RING - 64) ? fv : val;
                } else {
                    val = p_jj < -(int32_t)(RING - 64) ? p_b : val;   // (no far lane: p_b unused)
                }
                const bool dep = p_jj >= 0;
                if (__ballot(dep)) {
                    int32_t ptr = dep ? p_jj : lane;
                    for (;;) {
                        const int32_t p2 = (int32_t)bperm((uint32_t)ptr << 2, (uint32_t)ptr);
                        if (!__ballot(p2 != ptr)) break;
                        ptr = p2;
                    }
                    val = bperm((uint32_t)ptr << 2, val);
                }
                S.ring[(rb0 + p_pos + lane) & RM] = (RingT)val;
            };
            do {
                PPG_STAMP(h0);
                const Round R = decode(std::true_type{}, bp, cn, cw, pos, W);
#ifdef PPG_STAMPS
                const uint64_t h1 = __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(R.vtin);
                if (st_w0 < h0) st_w0 = h1;   // no walk this round
                hs_dec += st_w0 - h0;
                hs_walk += h1 - st_w0;
                hs_rounds++;
#endif
                // the token lookup does not read the ring: issued before the pending round's finish
                const uint32_t rout = min(R.off, 64u);
                const uint64_t mo = __ballot(R.vtin != 0);
                uint32_t sj4;
                asm("v_mad_i32_i24 %0, %1, -4, %2" : "=v"(sj4) : "v"((uint32_t)__builtin_clzll(mo & lanes_le)), "s"(252u));
                const uint32_t inf = bperm(sj4, R.vtin);
                // r06: the walk's priority 2 held through the token lookup, then 0 for the rest of the
                // round (finish, flush, stream words, emit) -- was 1 from the walk's end to the round's
                // tail: 520.0 -> 518.4 / 515.8 -> 513.8 ms per 50 GB step on two boxes
                // (profiles/r06zj_ab_prio_place2.json, r06zk_ab_prio_place3.json; the tail's own
                // s_setprio 0, now redundant, stays: without it 522.6)
                asm volatile("s_setprio 0");
#ifdef PPG_STAMPS
                const uint64_t h2 = __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(inf);
                hs_look += h2 - h1;
#endif
                finish();
                if constexpr (!EARLY && !IX) {
                    // the flush inside the pipelined loop (r06): every byte before pos is in the ring once
                    // the pending round is finished, and nothing of this round reads the ring yet -- the
                    // loop no longer ends (and waits for its pending round's far load) at every 1 KiB
                    // unit (518.3 vs 520.4 ms per 50 GB step, profiles/r06p_ab_inflush.json)
                    if (pos >= fl_next) {
                        flush(fl_done, fl_next);
                        fl_done = fl_next;
                        fl_next += UNIT;
                    }
                }
#ifdef PPG_STAMPS
                const uint64_t h3 = __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(
                                                                       S.ring[(rb0 + p_pos + lane) & RM]);
                hs_fin += h3 - h2;
#endif
                // the next round's stream words after the finish: the finish's s_waitcnt vmcnt(0)
                // (the compiler's, for the far load) would otherwise also wait for a stream DMA
                // issued here -- an HBM miss every ~9 rounds (574.6 -> 569.2 ms with the lookup
                // above, profiles/r04l_ab_pipeline_variants.json)
                st_enter(r, S.stream, (bp + R.adv) >> 10, lane);
                W = words(bp + R.adv);
#ifdef PPG_STAMPS
                const uint64_t h4 = __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(W.x4);
                hs_words += h4 - h3;
#endif
                const int32_t jj = lane - 1 - (int32_t)(inf >> 17);
                const uint32_t rv = S.ring[(rb0 + pos + (uint32_t)jj) & RM];
                if constexpr (IX) p_val = ((inf >> 8) & 511u) != 1u ? rv : (0x8000u | ((inf >> 17) & 255u));
                else p_val = ((inf >> 8) & 511u) != 1u ? rv : ((inf >> 17) & 255u);
                const bool far = jj < -(int32_t)(RING - 64);
                // pos >= 32768: every far source is the flushed output; a compiler-tracked load (its
                // s_waitcnt lands at the first use, in finish)
                if constexpr (IX) {   // the job's 64 Ki-symbol ring, as the dword holding the symbol
                    const uint32_t q = 2u * ((pos + (uint32_t)jj) & IXM);
                    const bool ld = EARLY ? far && (int32_t)pos + jj >= 0 : far;
                    p_b = *(const uint32_t *)(ob + (uint64_t)(ld ? (q & ~3u) : 0u));
                } else if constexpr (EARLY) {
                    // the flushed output (p >= 0) or the Point's window (p >= -32768)
                    const int32_t p = (int32_t)pos + jj;
                    const uint8_t *src = p >= 0 ? ob + (oa + (uint32_t)p) : dict + (uint32_t)(32768 + p);
                    p_b = *(far ? src : ob);
                } else {
                    p_b = ob[(uint64_t)(far ? (uint32_t)jj + (pos + oa) : 0u)];
                }
                p_jj = jj;
                p_pos = pos;
                cn = R.off - rout;
                cw = R.tl & ~(511u << 8);
                pos += rout;
                bp += R.adv;
                asm volatile("s_setprio 0");
                lim_r = latch_limit(R.xr, limh);
                if constexpr (IX) {   // past the member, or runaway output (a false start)
                    if (bp > bit_limit || pos > ixcap) { status = ST_DATA_ERROR; lim_r = 0; }
                }
#ifdef PPG_STAMPS
                hs_emit += __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(p_b + lim_r) - h4;
                st_w0 = 0;
#endif
            } while (pos < lim_r);
            finish();
            return lim_r;
        };
        for (;;) {
            // The rounds up to the next flush boundary (or the output's end) as inner loops with ONE
            // latch each: pos < lim_r, where lim_r = 0 once a special token ended a round
            // (latch_limit), so one compare leaves the rounds for all three reasons.  The pipelined
            // loop (hot_pipe) runs every round at least 322 bytes before the chunk's end -- its
            // EARLY form those of the first 32 KiB --; the general form (one_round) the others.
            // (r04: 679.2 -> 641.8 ms per 50 GB step for the round control, then 640.8 -> 552.8 ms
            // for the pipelining; profiles/r04_ab_round_control.json, r04j_*, r04l_*, r04o_*, r04r/.)
            bool spec_ = false;
            const uint32_t lim = min(len, fl_next);
            uint32_t lim_r;
            {
                const uint32_t limh = min(fl_next, len > 322u ? len - 322u : 0u);
                // the first 32 KiB of a chunk or piece (far sources may lie in the Point's window):
                // the same pipelined loop with a per-lane source select (r04: the N = 8 / 4 shares
                // 74.17 -> 73.58 / 144.95 -> 143.65 ms, N = 1 unchanged; profiles/r04r/)
                if (pos < 32768u && pos < limh) {
                    const uint32_t lime = min(limh, 32768u);
#ifdef PPG_STAMPS
                    const uint64_t tq0 = __builtin_amdgcn_s_memtime();
#endif
                    lim_r = hot_pipe(std::true_type{}, lime);
#ifdef PPG_STAMPS
                    sx_hp += __builtin_amdgcn_s_memtime() + 0 * (uint64_t)lim_r - tq0;
                    sx_nhp++;
#endif
                    spec_ = lim_r == 0u;   // lime > pos >= 0 otherwise
                }
                const uint32_t limp = IX ? limh : (len > 322u ? len - 322u : 0u);   // flushes inside the loop
                if (!spec_ && pos >= 32768u && pos < limp) {
                    // DecompressAll and CreateIndex pass 1 (r04: pass 1 792 -> 671 ms per 50 GB member,
                    // profiles/r04q/)
#ifdef PPG_STAMPS
                    const uint64_t tq0 = __builtin_amdgcn_s_memtime();
#endif
                    lim_r = hot_pipe(std::false_type{}, limp);
#ifdef PPG_STAMPS
                    sx_hp += __builtin_amdgcn_s_memtime() + 0 * (uint64_t)lim_r - tq0;
                    sx_nhp++;
#endif
                    spec_ = lim_r == 0u;   // limh > pos >= 0 otherwise
                }
                if (!spec_ && pos < lim) {
                    do {
                        lim_r = latch_limit(one_round(), lim);
                    } while (pos < lim_r);
                    spec_ = lim_r == 0u;
                }
            }
            if constexpr (IX) {
                if (status != ST_OK) break;
            }
            if (pos >= fl_next) {
#ifdef PPG_STAMPS
                const uint64_t tf0 = __builtin_amdgcn_s_memtime();
#endif
                flush(fl_done, fl_next);
                fl_done = fl_next;
                fl_next += UNIT;
#ifdef PPG_STAMPS
                sx_flush += __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(S.cen[0]) - tf0;
                sx_nflush++;
#endif
            }
            if (!spec_) {
                if (pos < len) continue;   // a flush boundary: more rounds
                break;
            }
            // ---- one token, bit-serially (long code, end-of-block or invalid) ----
#ifdef PPG_STAMPS
            const uint64_t ts0 = __builtin_amdgcn_s_memtime();
            sx_nspec++;
#endif
            asm volatile("s_setprio 2");
            rd_seek(r, S.stream, bp, lane);
            rd_refill(r, S.stream, lane);
            // The token the hot rounds stopped at: a litlen code longer than the root (or end-of-block),
            // or a length whose DISTANCE code is (~60% of them on bench-shape FASTQ): the root tables
            // first, the sorted symbols (litlen: global scratch; distance: LDS) only for the long code
            int sym;
            uint32_t ml = 0;
            {
                const uint32_t e = uni(S.lit[(uint32_t)r.bb & ((1u << LBT) - 1)]);
                if (!(e & 0x80u)) {
                    const uint32_t L = e & 15u;
                    br_take(r, L);
                    if (e & 0x40u) {
                        ml = ((e >> 16) & 0x1FFu) + br_take(r, ((e >> 8) & 0xFFu) - L);
                        sym = 257;
                    } else {
                        sym = (int)((e >> 17) & 0xFFu);
                    }
                } else {
                    sym = canon_decode(r, clit, lit_sorted, lane);
                    if (sym > 256 && sym < 286) {
                        ml = c_lbase[sym - 257] + br_take(r, c_lext[sym - 257]);
                        sym = 257;
                    }
                }
            }
#ifdef PPG_STATS
            if (sym < 256) st_blit++; else if (sym == 256) st_beob++; else st_bmatch++;
#endif
            if (sym < 0 || sym > 257) { status = ST_DATA_ERROR; break; }
            if (sym < 256) {
                if (lane == 0) S.ring[(rb0 + pos) & RM] = (RingT)((IX ? 0x8000u : 0u) | (uint32_t)sym);
                pos++;
            } else if (sym == 256) {
                in_block = 0;
                bp = rd_pos(r);
                break;
            } else {
                rd_refill(r, S.stream, lane);
                uint32_t ds;
                const uint32_t d = uni(S.dst[(uint32_t)r.bb & ((1u << DB) - 1)]);
                if (d != ~0u) {
                    br_take(r, d & 15u);
                    ds = (d >> 16) + 1u + br_take(r, (d >> 10) & 31u);
                } else {
                    const int dsym = canon_decode(r, cdst, dst_sorted, lane);
                    if (dsym < 0 || dsym >= 30) { status = ST_DATA_ERROR; break; }
                    ds = c_dbase[dsym] + br_take(r, c_dext[dsym]);
                }
                const uint32_t n = min(ml, len - pos);
                copy_match<RB, IX, RingT, IXM>(S.ring, ob, oa, dict, rb0, pos, ds, n, lane);
                pos += n;
            }
            bp = rd_pos(r);
            if (pos >= fl_next) {
                flush(fl_done, fl_next);
                fl_done = fl_next;
                fl_next += UNIT;
            }
            st_enter(r, S.stream, bp >> 10, lane);
            W = words(bp);
            asm volatile("s_setprio 0");
#ifdef PPG_STAMPS
            sx_spec += __builtin_amdgcn_s_memtime() + 0 * (uint64_t)__builtin_amdgcn_readfirstlane(W.x4) - ts0;
#endif
            if (pos >= len) break;
        }
        if (status != ST_OK) break;
        rd_seek(r, S.stream, bp, lane);   // the next block header / the R-E5 check read from bp
        if constexpr (IX) {
            if (in_block) { status = ST_DATA_ERROR; break; }   // output limit inside a block
            if (!block_end(bp)) break;
        }
    }
    flush(fl_done, pos);

    // zlib was handed only the chunk's slice (LazyFileReader.cs:63-69): needing bits past it is
    // the DATA_ERROR of Core.cs:174.  R-E5: the next symbol should be the block's end-of-block.
    uint32_t end_bit = rd_pos(r);
    if (end_bit > bit_limit) {
        flags |= PPG_FLAG_OVERRUN;
        if (status == ST_OK) status = ST_DATA_ERROR;
    }
    if (!IX && status == ST_OK && in_block && pos == len) {
        rd_refill(r, S.stream, lane);
        if (canon_decode(r, clit, lit_sorted, lane) == 256) end_bit = rd_pos(r);
        else flags |= PPG_FLAG_NO_EOB;
    }
#ifdef PPG_STATS
    if (!IX && lane == 0 && k < 4)
        printf("PPG_STATS chunk %d: bytes %u rounds %u tokens %u spec %u short %u far %u dep %u dbl %u "
               "bitserial lit %u eob %u match %u\n", k, pos, st_rounds, st_tokens, st_spec, st_short, st_far, st_dep,
               st_dbl, st_blit, st_beob, st_bmatch);
#endif
#ifdef PPG_IX_STATS
    if (IX && lane == 0) {
        atomicAdd(&ppg_ixstat[0], (unsigned long long)ix_unk);
        atomicAdd(&ppg_ixstat[1], (unsigned long long)ix_last);
        atomicAdd(&ppg_ixstat[2], (unsigned long long)pos);
        atomicAdd(&ppg_ixstat[3], 1ull);
        atomicAdd(&ppg_ixstat[4 + min(9u, (uint32_t)(10ull * ix_last / max(pos, 1u)))], 1ull);
        atomicMax(&ppg_ixstat[14], (unsigned long long)ix_last);
    }
#endif
#ifdef PPG_STAMPS
    if (!IX && lane == 0) {
        atomicAdd(&ppg_stamp_acc[0], (unsigned long long)sa_dec);
        atomicAdd(&ppg_stamp_acc[1], (unsigned long long)sa_walk);
        atomicAdd(&ppg_stamp_acc[2], (unsigned long long)sa_rd);
        atomicAdd(&ppg_stamp_acc[3], (unsigned long long)sa_far);
        atomicAdd(&ppg_stamp_acc[4], (unsigned long long)sa_dep);
        atomicAdd(&ppg_stamp_acc[5], (unsigned long long)sa_tail);
        atomicAdd(&ppg_stamp_acc[6], (unsigned long long)sa_rounds);
        atomicAdd(&ppg_stamp_acc[7], (unsigned long long)sa_farr);
        atomicAdd(&ppg_stamp_acc[8], (unsigned long long)hs_dec);
        atomicAdd(&ppg_stamp_acc[9], (unsigned long long)hs_walk);
        atomicAdd(&ppg_stamp_acc[10], (unsigned long long)hs_look);
        atomicAdd(&ppg_stamp_acc[11], (unsigned long long)hs_fin);
        atomicAdd(&ppg_stamp_acc[12], (unsigned long long)hs_words);
        atomicAdd(&ppg_stamp_acc[13], (unsigned long long)hs_emit);
        atomicAdd(&ppg_stamp_acc[14], (unsigned long long)hs_rounds);
        atomicAdd(&ppg_stamp_acc[15], (unsigned long long)(__builtin_amdgcn_s_memtime() - tk0));
        atomicAdd(&ppg_stamp_acc[16], (unsigned long long)sx_spec);
        atomicAdd(&ppg_stamp_acc[17], (unsigned long long)sx_nspec);
        atomicAdd(&ppg_stamp_acc[18], (unsigned long long)sx_flush);
        atomicAdd(&ppg_stamp_acc[19], (unsigned long long)sx_nflush);
        atomicAdd(&ppg_stamp_acc[20], (unsigned long long)sx_hdr);
        atomicAdd(&ppg_stamp_acc[21], (unsigned long long)sx_nhdr);
        atomicAdd(&ppg_stamp_acc[22], 1ull);
        atomicAdd(&ppg_stamp_acc[23], (unsigned long long)sx_hp);
        atomicAdd(&ppg_stamp_acc[24], (unsigned long long)sx_nhp);
    }
#endif
    if (lane == 0) {
        res[k].produced = pos;
        res[k].end_bit = w0abs * 32 + end_bit;
        res[k].status = status;
        res[k].flags = flags;
        res[k].nblocks = nblk;
        res[k].last = (uint32_t)last;
        res[k].newlines = census ? S.cen[0] : 0;
        res[k].pflags = census ? S.cen[2] : 0;
    }
}

// per-launch scratch of the sorted-symbol tables, stream-ordered: no device-wide sync.  From a private
// memory pool per device whose release threshold keeps the memory between launches (the
// threshold used to be raised on the device's DEFAULT pool -- process-wide state that every other
// hipMallocAsync user of the process then inherited); the default pool, untouched, only if a private
// pool cannot be made.
static hipError_t gsort_alloc(hipStream_t s, int njobs, uint16_t **p) {
    static std::mutex mu;
    static hipMemPool_t pools[64] = {};
    static bool tried[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const size_t bytes = (size_t)njobs * PPG_SORT_SLOT * sizeof(uint16_t);
    hipMemPool_t pool = nullptr;
    if (dev >= 0 && dev < 64) {
        std::lock_guard<std::mutex> lk(mu);
        if (!tried[dev]) {
            tried[dev] = true;
            hipMemPoolProps props = {};
            props.allocType = hipMemAllocationTypePinned;
            props.handleTypes = hipMemHandleTypeNone;
            props.location.type = hipMemLocationTypeDevice;
            props.location.id = dev;
            if (hipMemPoolCreate(&pools[dev], &props) == hipSuccess) {
                uint64_t t = ~0ull;
                (void)hipMemPoolSetAttribute(pools[dev], hipMemPoolAttrReleaseThreshold, &t);
            } else {
                pools[dev] = nullptr;
                (void)hipGetLastError();
            }
        }
        pool = pools[dev];
    }
    if (pool) return hipMallocFromPoolAsync((void **)p, bytes, pool, s);
    return hipMallocAsync((void **)p, bytes, s);
}
#define PPG_GSORT_BEGIN(s, njobs)                          \
    uint16_t *gsort = nullptr;                             \
    {                                                      \
        const hipError_t ge = gsort_alloc(s, njobs, &gsort); \
        if (ge != hipSuccess) return ge;                   \
    }
#define PPG_GSORT_END(s) (void)hipFreeAsync(gsort, s)

// ------------------------------------------------------------------------------------------
// Host-side launcher (called from ppg_api.cpp).  ring_bits selects the history ring.
// ------------------------------------------------------------------------------------------
// (ring bits, litlen root bits) variants; default (11, 8)
#define PPG_VARIANTS(X) X(10, 8) X(10, 9) X(11, 9) X(11, 8) X(12, 9) X(12, 8) X(13, 9) X(15, 9)

#ifdef PPG_STAMPS
struct PpgStampPrinter;
static void ppg_stamp_dump(hipStream_t s);
#define PPG_STAMP_DUMP(s) ppg_stamp_dump(s)
#else
#define PPG_STAMP_DUMP(s)
#endif

size_t ppg_inflate_lds_bytes(int ring_bits, int lit_bits) {
#define X(R, L) if (ring_bits == R && lit_bits == L) return sizeof(InflateLds<R, L>);
    PPG_VARIANTS(X)
#undef X
    return 0;
}

hipError_t ppg_launch_inflate(hipStream_t s, int ring_bits, int lit_bits, const uint32_t *comp, uint64_t nwords,
                              const PpgInflateJob *jobs, const uint8_t *dicts, uint8_t *out, PpgInflateResult *res,
                              int njobs, uint32_t *nls) {
    if (njobs <= 0) return hipSuccess;
    // A/B probe only (PPG_PROBE_NO_CENSUS=1): the kernel without the fused newline census, to time
    // what the census costs; the records of such a run are not valid
    static const bool no_census = getenv("PPG_PROBE_NO_CENSUS") != nullptr;
    if (no_census) nls = nullptr;
#define X(R, L)                                                                                               \
    if (ring_bits == R && lit_bits == L) {                                                                    \
        PPG_GSORT_BEGIN(s, njobs);                                                                            \
        if (nls)                                                                                              \
            hipLaunchKernelGGL((ppg_inflate_kernel<R, L, false, true>), dim3(njobs), dim3(64),                \
                               0, s, comp, nwords, jobs, dicts, out, res, njobs, nullptr, nls, gsort);          \
        else                                                                                                  \
            hipLaunchKernelGGL((ppg_inflate_kernel<R, L, false, false>), dim3(njobs), dim3(64),               \
                               0, s, comp, nwords, jobs, dicts, out, res, njobs, nullptr, nls, gsort);          \
        const hipError_t le = hipGetLastError();                                                              \
        PPG_GSORT_END(s);                                                                                     \
        PPG_STAMP_DUMP(s);                                                                                    \
        return le;                                                                                            \
    }
    PPG_VARIANTS(X)
#undef X
    return hipErrorInvalidValue;
}

#ifdef PPG_STAMPS
// diagnostic build: print and reset the per-phase round totals (after the stream drains)
struct PpgStampPrinter {
    static void dump(hipStream_t s) {
        unsigned long long h[25] = {0};
        if (hipStreamSynchronize(s) != hipSuccess) return;
        if (hipMemcpyFromSymbol(h, HIP_SYMBOL(ppg_stamp_acc), sizeof h) != hipSuccess) return;
        const unsigned long long z[25] = {0};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(ppg_stamp_acc), z, sizeof z);
        const double r = h[6] ? (double)h[6] : 1.0;
        fprintf(stderr, "PPG_STAMPS rounds %llu far-rounds %llu cycles/round: decode %.1f walk %.1f read %.1f far %.1f "
                        "dep+write %.1f tail %.1f total %.1f\n", h[6], h[7], h[0] / r, h[1] / r, h[2] / r, h[3] / r,
                h[4] / r, h[5] / r, (h[0] + h[1] + h[2] + h[3] + h[4] + h[5]) / r);
        const double q = h[14] ? (double)h[14] : 1.0;
        fprintf(stderr, "PPG_STAMPS hot rounds %llu cycles/round: decode %.1f walk %.1f lookup %.1f finish %.1f "
                        "words %.1f emit+tail %.1f total %.1f\n", h[14], h[8] / q, h[9] / q, h[10] / q, h[11] / q,
                h[12] / q, h[13] / q, (h[8] + h[9] + h[10] + h[11] + h[12] + h[13]) / q);
        // where a wave's whole job goes (r06): hot rounds, general rounds, bit-serial tokens, flushes,
        // block headers, the rest (job start, seeks, the last flush, the R-E5 check)
        const double T = h[15] ? (double)h[15] : 1.0;
        const double hot = h[8] + h[9] + h[10] + h[11] + h[12] + h[13], gen = h[0] + h[1] + h[2] + h[3] + h[4] + h[5];
        fprintf(stderr, "PPG_STAMPS jobs %llu wave cycles %.4g: hot rounds %.1f%% general rounds %.1f%% bit-serial tokens "
                        "%.1f%% (%llu, %.0f cycles each) flushes %.1f%% (%llu, %.0f each) block headers %.1f%% (%llu, %.0f "
                        "each) other %.1f%%\n", h[22], T, 100 * hot / T, 100 * gen / T, 100 * h[16] / T, h[17],
                h[16] / (h[17] ? (double)h[17] : 1.0), 100 * h[18] / T, h[19], h[18] / (h[19] ? (double)h[19] : 1.0),
                100 * h[20] / T, h[21], h[20] / (h[21] ? (double)h[21] : 1.0),
                100 * (T - hot - gen - h[16] - h[18] - h[20]) / T);
        fprintf(stderr, "PPG_STAMPS pipelined-loop calls %llu: %.1f%% of wave cycles inside them, %.0f cycles per call "
                        "outside their rounds (entry, the pending round's finish, exit)\n", h[24], 100 * h[23] / T,
                (h[23] - hot) / (h[24] ? (double)h[24] : 1.0));
    }
};
#endif

// CreateIndex pass 1: jobs decode whole blocks into 64 KiB output rings (out + k * 64 KiB)
hipError_t ppg_launch_inflate_ix(hipStream_t s, const uint32_t *comp, uint64_t nwords, const PpgInflateJob *jobs,
                                 const uint8_t *dicts, uint8_t *out, PpgInflateResult *res, PpgBlockEnd *blk,
                                 int njobs) {
    if (njobs <= 0) return hipSuccess;
    PPG_GSORT_BEGIN(s, njobs);
    hipLaunchKernelGGL((ppg_inflate_kernel<10, 8, true, false>), dim3(njobs), dim3(64), 0, s, comp,
                       nwords, jobs, dicts, out, res, njobs, blk, nullptr, gsort);
    const hipError_t le = hipGetLastError();
    PPG_GSORT_END(s);
    if (le != hipSuccess) return le;
#ifdef PPG_IX_STATS
    {
        unsigned long long h[16] = {0};
        if (hipStreamSynchronize(s) == hipSuccess && hipMemcpyFromSymbol(h, HIP_SYMBOL(ppg_ixstat), sizeof h) == hipSuccess) {
            const unsigned long long z[16] = {0};
            (void)hipMemcpyToSymbol(HIP_SYMBOL(ppg_ixstat), z, sizeof z);
            fprintf(stderr, "PPG_IX_STATS jobs %llu bytes %llu unknown %llu (%.4f%%) mean last %.0f max last %llu tenths", h[3],
                    h[2], h[0], 100.0 * h[0] / (h[2] ? h[2] : 1), (double)h[1] / (h[3] ? h[3] : 1), h[14]);
            for (int i = 4; i < 14; i++) fprintf(stderr, " %llu", h[i]);
            fprintf(stderr, "\n");
        }
    }
#endif
    return hipGetLastError();
}

#ifdef PPG_STAMPS
static void ppg_stamp_dump(hipStream_t s) { PpgStampPrinter::dump(s); }
#endif

// the lone-chunk Decompress's pass 1 (ppg_chunk.cpp): symbolic output kept whole per job (IXF)
hipError_t ppg_launch_inflate_ixf(hipStream_t s, const uint32_t *comp, uint64_t nwords, const PpgInflateJob *jobs,
                                  const uint8_t *dicts, uint8_t *out, PpgInflateResult *res, PpgBlockEnd *blk,
                                  int njobs) {
    if (njobs <= 0) return hipSuccess;
    PPG_GSORT_BEGIN(s, njobs);
    hipLaunchKernelGGL((ppg_inflate_kernel<10, 8, true, false, true>), dim3(njobs), dim3(64), 0, s, comp, nwords, jobs,
                       dicts, out, res, njobs, blk, nullptr, gsort);
    const hipError_t le = hipGetLastError();
    PPG_GSORT_END(s);
    return le;
}

// A piece whose pass-1 symbols and exact starting history are known is written out without a second
// decode: symbol 0x8000 | b is the byte b, symbol i < 32768 is byte i of the history.  The bytes go
// through the inflate kernel's own flush path -- an LDS ring by global output address, flushed in
// aligned units with the fused newline census (flush_census) -- so the piece's result and census
// region are exactly what decoding it (ppg_inflate_kernel, CEN) would have produced.  A unit's 32
// symbols per lane are loaded at once, and the next unit's while this one's census runs (r05: one
// load after another, a 4,096-piece launch took 9.9 ms, latency-bound at 4 waves per CU).
// mi[k].prev: the census's "previous byte" (a chunk's first piece: the job's own, from the Point's
// offset), or > 255: the history's last byte.
template <int RB>
__global__ __launch_bounds__(64) void ppg_materialize_kernel(const uint16_t *__restrict__ sym,
                                                             const uint8_t *__restrict__ wins,
                                                             const PpgMatInfo *__restrict__ mi,
                                                             const PpgInflateJob *__restrict__ jobs,
                                                             uint8_t *__restrict__ out, PpgInflateResult *__restrict__ res,
                                                             int njobs, uint32_t *__restrict__ nls) {
    constexpr uint32_t RING = 1u << RB, RM = RING - 1, UNIT = RING / 2, PER = UNIT / 64;
    __shared__ __attribute__((aligned(16))) uint8_t W[32768];
    __shared__ __attribute__((aligned(16))) uint8_t ring[RING];
    __shared__ uint32_t cen[8];
    const int k = blockIdx.x, lane = threadIdx.x;
    if (k >= njobs) return;
    const PpgInflateJob J = jobs[k];
    const PpgMatInfo M = mi[k];
    for (uint32_t i = 16u * (uint32_t)lane; i < 32768u; i += 1024u)
        *(uint4 *)&W[i] = *(const uint4 *)(wins + M.win_off + i);
    if (lane == 0) {
        const uint64_t d = (uint64_t)(uintptr_t)(nls + J.nl_off);
        cen[0] = 0;
        cen[2] = 0;
        cen[3] = J.nl_cap;
        cen[4] = J.raw_shift;
        cen[5] = (uint32_t)d;
        cen[6] = (uint32_t)(d >> 32);
    }
    __syncthreads();
    if (lane == 0) cen[1] = (M.prev > 255u ? W[32767] : M.prev) == '\n';
    const uint32_t len = (uint32_t)J.out_len;
    const uint64_t out_off = J.out_off;
    const uint16_t *sy = sym + M.sym_off;
    // units end at UNIT-aligned output addresses (or the piece's end)
    auto unit_end = [&](uint32_t p) { return min(len, p + (UNIT - (uint32_t)((out_off + p) & (UNIT - 1)))); };
    uint32_t v[PER];
    auto fetch = [&](uint32_t p0, uint32_t p1) {
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            const uint32_t p = p0 + (uint32_t)lane + 64u * i;
            v[i] = p < p1 ? (uint32_t)sy[p] : 0x8000u;
        }
    };
    uint32_t p0 = 0, p1 = unit_end(0);
    fetch(p0, p1);
    while (p0 < len) {
#pragma unroll
        for (uint32_t i = 0; i < PER; i++) {
            const uint32_t p = p0 + (uint32_t)lane + 64u * i;
            if (p < p1) ring[(uint32_t)(out_off + p) & RM] = (uint8_t)((v[i] & 0x8000u) ? v[i] : W[v[i] & 32767u]);
        }
        __syncthreads();
        const uint32_t q1 = unit_end(p1);
        fetch(p1, q1);   // (empty past the end)
        flush_census<RB>(ring, out, out_off, p0, p1, lane, cen);
        __syncthreads();
        p0 = p1;
        p1 = q1;
    }
    if (lane == 0) {
        res[k].produced = len;
        res[k].end_bit = M.end_bit;
        res[k].status = 0;
        res[k].flags = 0;
        res[k].nblocks = M.nblocks;
        res[k].last = M.last;
        res[k].newlines = cen[0];
        res[k].pflags = cen[2];
    }
}

hipError_t ppg_launch_materialize(hipStream_t s, const uint16_t *sym, const uint8_t *wins, const PpgMatInfo *mi,
                                  const PpgInflateJob *jobs, uint8_t *out, PpgInflateResult *res, int njobs,
                                  uint32_t *nls) {
    if (njobs <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_materialize_kernel<12>, dim3(njobs), dim3(64), 0, s, sym, wins, mi, jobs, out, res, njobs, nls);
    return hipGetLastError();
}
