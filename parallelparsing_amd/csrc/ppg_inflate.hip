// ppg_inflate.hip — gfx950 (MI355X / CDNA4) DEFLATE inflate for checkpoint chunks.
//
// Replaces the zlib calls of Core.ExtractDeflateIndex (Decompressor/Core.cs:133-192):
// inflateInit2(-15) + inflatePrime(from.Bits) + inflateSetDictionary(from.Window, 32768) +
// inflate(Z_NO_FLUSH) until to.Output - from.Output bytes exist.  One 64-lane wavefront decodes
// one chunk; chunks are independent because every Point carries its 32 KiB history.
//
// Where the time goes on gfx950 (measured, scratch micro-benchmarks, 2.39 GHz): a dependent
// uniform ds_read + v_readfirstlane costs ~92 cycles, an s_load hit ~52, a dependent SALU op
// ~6-8.  Inflate is a serial chain of such steps per chunk, so the kernel is built to keep the
// chain short and to fit many wavefronts per CU:
//   * decoder state (bit buffer, positions) is wave-uniform in SGPRs; every branch is scalar;
//   * the compressed stream sits in two VGPRs (128 words across the lanes, refilled 256 B at a
//     time by coalesced loads issued a buffer ahead) and is read with v_readlane -> no memory
//     wait on the bit-buffer refill;
//   * 6-bit first-level litlen/distance tables live in one VGPR each (v_readlane, ~90% of
//     symbols); the full 10/8-bit root tables and the bit-serial slow path sit in LDS;
//   * history is an LDS ring of 2^RB bytes (8-16 KiB -> 7-11 waves per CU) indexed by the
//     GLOBAL output address; back-references further than the ring read the already flushed
//     output (or the Point's window) from HBM;
//   * a match's LDS read is left in flight while the next symbol decodes (deferred write);
//   * completed 4 KiB units leave the ring as 16-B-per-lane coalesced stores.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "ppg_device.h"
#include "ppg_huffman.h"

template <int RB>
struct __attribute__((aligned(16))) InflateLds {
    uint8_t ring[1u << RB];
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

// v_writelane_b32 (value, lane, old) — the LLVM intrinsic, not exposed as a clang builtin
extern "C" __device__ int llvm_writelane(int, int, int) __asm("llvm.amdgcn.writelane");

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// Compressed stream of one chunk: word i (chunk-relative) is base[i].  256 words live across the
// lanes (lane l holds word wb+l in A and wb+64+l in B), so fetching stream words is v_readlane.
// A reload is two coalesced dword loads per lane whose results are consumed at once: the wait
// (~one memory latency per ~500 B of input) is paid there and nowhere else.  A load whose result
// stayed in flight across loop iterations would make the compiler wait for every outstanding
// memory operation at each use (including the output flush stores).
struct Reader {
    const uint32_t *base;
    uint32_t nw;            // readable words from base (>= 1)
    uint32_t A, B;          // words wb+lane, wb+64+lane
    uint32_t wb;            // first word of the buffer
    uint32_t wi;            // next word to append to bb
    uint64_t bb;            // bit buffer, LSB = next bit
    uint32_t bn;            // valid bits in bb
};

__device__ __forceinline__ void rd_load(Reader &r, int lane) {
    const uint32_t i = r.wb + lane;
    r.A = i < r.nw ? r.base[i] : 0u;          // past the end: zeros (an overrun is an error anyway)
    r.B = i + 64 < r.nw ? r.base[i + 64] : 0u;
    // consume the loads here, so the compiler waits for them in this (rare) block rather than
    // at every v_readlane of A/B (there the wait would drain every store in flight, too)
    asm volatile("" ::"v"(r.A), "v"(r.B));
}

__device__ __forceinline__ uint32_t rd_word(const Reader &r, uint32_t idx) {
    return idx < 64 ? rdlane(r.A, idx) : rdlane(r.B, idx - 64);
}

// position the bit buffer at chunk-relative bit `bit` (reloads only when outside the buffer)
__device__ __forceinline__ void rd_seek(Reader &r, uint32_t bit, int lane) {
    r.wi = bit >> 5;
    if (r.wi < r.wb || r.wi >= r.wb + 128) {
        r.wb = r.wi;
        rd_load(r, lane);
    }
    const uint32_t w = rd_word(r, r.wi - r.wb);
    r.wi++;
    const uint32_t sh = bit & 31;
    r.bb = (uint64_t)(w >> sh);
    r.bn = 32 - sh;
}

// guarantees bn >= 32
__device__ __forceinline__ void rd_refill(Reader &r, int lane) {
    if (r.bn <= 32) {
        if (r.wi >= r.wb + 128) {
            r.wb = r.wi;
            rd_load(r, lane);
        }
        const uint32_t w = rd_word(r, r.wi - r.wb);
        r.wi++;
        r.bb |= (uint64_t)w << r.bn;
        r.bn += 32;
    }
}

__device__ __forceinline__ uint32_t rd_pos(const Reader &r) { return r.wi * 32 - r.bn; }

// Symbol -> entry: the VGPR first level (6 bits), else the LDS root table, else the slow path.
__device__ __forceinline__ uint32_t lookup(uint32_t vtab, const uint32_t *tab, uint32_t tmask, Reader &r,
                                           const uint16_t *count, const uint16_t *sorted, int kind) {
    uint32_t e = rdlane(vtab, (uint32_t)r.bb & 63);
    if (e == 0) {
        e = uni(tab[(uint32_t)r.bb & tmask]);
        if ((e & 15) == 0) e = slow_entry(r, count, sorted, kind);
    }
    return e;
}

// 6-bit first level: the root entry when its code fits 6 bits, else 0 (= go to LDS).
__device__ __forceinline__ uint32_t first_level(const uint32_t *tab, int lane) {
    const uint32_t e = tab[lane];
    const uint32_t L = e & 15;
    return (L != 0 && L <= 6) ? e : 0u;
}

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

// Byte at chunk position p older than the ring: the flushed output (p >= 0) or the Point's window.
// Read as an aligned dword so the compiler never merges it with an LDS byte load into one flat load.
__device__ __forceinline__ uint32_t far_byte(const uint8_t *out, const uint8_t *dict, uint64_t out_off, int32_t p) {
    const uint8_t *a = p >= 0 ? out + out_off + (uint32_t)p : dict + 32768 + p;   // p >= -32768
    const uint32_t w = *(const uint32_t *)((uintptr_t)a & ~(uintptr_t)3);
    return (w >> (8 * ((uintptr_t)a & 3))) & 255u;
}

// One LZ77 copy of n bytes from dist back, at chunk position pos (all 64 lanes, uniform args).
template <int RB>
__device__ __forceinline__ void copy_match(uint8_t *ring, const uint8_t *out, const uint8_t *dict, uint64_t out_off,
                                           uint32_t rb0, uint32_t pos, uint32_t dist, uint32_t n, int lane) {
    constexpr uint32_t RING = 1u << RB;
    constexpr uint32_t RM = RING - 1;
    const uint32_t dst0 = rb0 + pos;   // ring slot of the first output byte
    if (dist + n <= RING) {
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
        // far reference (dist > RING - n >= n): bytes older than the ring come from the flushed
        // output (this wave's own earlier stores: same-wave accesses to an address are ordered)
        // or the Point's window
        for (uint32_t j0 = 0; j0 < n; j0 += 64) {
            const uint32_t j = j0 + lane;
            if (j < n) {
                const uint32_t back = dist - j;                 // source = pos - back
                const int32_t rel = (int32_t)pos - (int32_t)back;
                uint32_t v;
                if (back + n <= RING) v = ring[(dst0 - back) & RM];
                else v = far_byte(out, dict, out_off, rel);
                ring[(dst0 + j) & RM] = (uint8_t)v;
            }
        }
    }
}

template <int RB>
__global__ __launch_bounds__(64) void ppg_inflate_kernel(const uint32_t *__restrict__ comp, uint64_t nwords,
                                                         const PpgInflateJob *__restrict__ jobs,
                                                         const uint8_t *__restrict__ dicts, uint8_t *__restrict__ out,
                                                         PpgInflateResult *__restrict__ res, int njobs) {
    constexpr uint32_t RING = 1u << RB;
    constexpr uint32_t RM = RING - 1;
    static_assert(RB >= 13 && RB <= 15, "far back-references assume the ring spans >= 2 flush units");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    InflateLds<RB> &S = *reinterpret_cast<InflateLds<RB> *>(smem);
    const int lane = threadIdx.x;
    const int k = blockIdx.x;
    if (k >= njobs) return;
    const PpgInflateJob J = jobs[k];
    const uint64_t out_off = J.out_off;
    const uint32_t len = (uint32_t)J.out_len;       // host guarantees < 2^31
    const uint32_t rb0 = (uint32_t)out_off;         // ring slot of chunk position p: (rb0 + p) & RM
    const uint8_t *dict = dicts + J.dict_off;       // chunk position p < 0 is dict[32768 + p]

    // history: the last RING bytes of the Point's window -> ring slots of positions [-RING, 0)
    for (uint32_t w0 = 0; w0 < RING / 4; w0 += 64) {
        const uint32_t w = w0 + lane;
        const uint32_t v = *(const uint32_t *)(dict + 32768 - RING + 4 * w);
        const uint32_t slot = rb0 - RING + 4 * w;
#pragma unroll
        for (int q = 0; q < 4; q++) S.ring[(slot + q) & RM] = (uint8_t)(v >> (8 * q));
    }
    __syncthreads();

    // chunk-relative compressed stream
    const uint64_t w0abs = (J.bit_start >> 5) & ~127ull;
    Reader r;
    r.wb = 0x80000000u;   // empty buffer: the first seek loads
    r.base = comp + w0abs;
    r.nw = (uint32_t)min(nwords > w0abs ? nwords - w0abs : 1ull, 0xFFFFFFFFull);
    const uint32_t bit_limit = (uint32_t)min(J.bit_limit - w0abs * 32, 0xFFFFFFFFull);
    rd_seek(r, (uint32_t)(J.bit_start - w0abs * 32), lane);

    uint32_t pos = 0;                                        // output bytes produced
    uint32_t fl_done = 0;                                    // flushed up to this position
    uint32_t fl_next = UNIT - (uint32_t)(out_off & (UNIT - 1));   // next global 4 KiB boundary
    int status = ST_OK, flags = 0, last = 0, in_block = 0;
    uint32_t vlit = 0, vdst = 0;    // first-level tables (one entry per lane)

    while (pos < len && !last) {
        r.wb = uni(r.wb);
        r.wi = uni(r.wi);
        r.bb = uni64(r.bb);
        r.bn = uni(r.bn);
        pos = uni(pos);
        fl_done = uni(fl_done);
        fl_next = uni(fl_next);
        status = (int)uni((uint32_t)status);
        rd_refill(r, lane);
        last = (int)br_take(r, 1);
        const uint32_t type = br_take(r, 2);
        if (type == 0) {
            // ---- stored block ----
            br_take(r, r.bn & 7);
            rd_refill(r, lane);
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
                    if (j < piece) S.ring[(rb0 + pos + j) & RM] = c8[copied + j];
                }
                pos += piece;
                copied += piece;
                if (pos >= fl_next) {
                    flush_range<RB>(S.ring, out, out_off + fl_done, out_off + fl_next, lane);
                    fl_done = fl_next;
                    fl_next += UNIT;
                }
            }
            rd_seek(r, (bytepos + copied) * 8, lane);
            if (copied < slen) break;   // output full mid-block (zlib stops at avail_out == 0)
            in_block = 0;
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
            build_table<LB>(S.lens, 288, S.lit, S.lit_count, S.lit_sorted, TAB_LIT, lane);
            build_table<DB>(S.lens + 288, 32, S.dst, S.dst_count, S.dst_sorted, TAB_DST, lane);
        } else {
            // ---- dynamic Huffman codes (RFC 1951 3.2.7) ----
            rd_refill(r, lane);
            const uint32_t hlit = br_take(r, 5) + 257, hdist = br_take(r, 5) + 1, hclen = br_take(r, 4) + 4;
            if (hlit > 286 || hdist > 30) { status = ST_DATA_ERROR; break; }
            if (lane < 19) S.lens[lane] = 0;
            __syncthreads();
            for (uint32_t i = 0; i < hclen; i++) {
                rd_refill(r, lane);
                const uint32_t v = br_take(r, 3);
                if (lane == 0) S.lens[c_clorder[i]] = (uint8_t)v;
            }
            __syncthreads();
            if (build_table<CB>(S.lens, 19, S.cl, nullptr, S.cl_sorted, TAB_CL, lane) != 0) { status = ST_DATA_ERROR; break; }
            uint32_t idx = 0;
            const uint32_t total = hlit + hdist;
            bool bad = false;
            while (idx < total) {
                rd_refill(r, lane);
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
            if (build_table<LB>(S.lens, (int)hlit, S.lit, S.lit_count, S.lit_sorted, TAB_LIT, lane) != 0) { status = ST_DATA_ERROR; break; }
            if (build_table<DB>(S.lens + hlit, (int)hdist, S.dst, S.dst_count, S.dst_sorted, TAB_DST, lane) != 0) { status = ST_DATA_ERROR; break; }
        }
        vlit = first_level(S.lit, lane);
        vdst = first_level(S.dst, lane);
        in_block = 1;
        // once per block: tell the compiler the decoder state is wave-uniform (it cannot prove it
        // through the outer loop), so the token loop keeps it in SGPRs with scalar branches
        r.wb = uni(r.wb);
        r.wi = uni(r.wi);
        r.bb = uni64(r.bb);
        r.bn = uni(r.bn);
        pos = uni(pos);
        fl_done = uni(fl_done);
        fl_next = uni(fl_next);

        // ---- token rounds ----
        // Speculative lane-parallel decode: every lane decodes one whole token (litlen code, length
        // extra bits, distance code, distance extra bits) as if a token started at bit bp + lane.
        // A scalar walk then follows the real chain of tokens (start, start + bits, ...) through
        // the lanes, emitting each one, until the chain leaves the 64-bit span; the next round
        // starts where it left.  Codes longer than the root tables, end-of-block and invalid codes
        // stop the walk and are decoded by the bit-serial path below.
        uint32_t bp = rd_pos(r);
        while (pos < len) {
            const uint32_t wq = bp >> 5;
            if (wq < r.wb || wq + 4 >= r.wb + 128) {
                r.wb = wq;
                rd_load(r, lane);
            }
            const uint32_t wi = wq - r.wb;
            uint32_t w0, w1, w2, w3, w4;
            if (wi + 4 < 64) {
                w0 = rdlane(r.A, wi); w1 = rdlane(r.A, wi + 1); w2 = rdlane(r.A, wi + 2);
                w3 = rdlane(r.A, wi + 3); w4 = rdlane(r.A, wi + 4);
            } else if (wi >= 64) {
                w0 = rdlane(r.B, wi - 64); w1 = rdlane(r.B, wi - 63); w2 = rdlane(r.B, wi - 62);
                w3 = rdlane(r.B, wi - 61); w4 = rdlane(r.B, wi - 60);
            } else {
                w0 = rd_word(r, wi); w1 = rd_word(r, wi + 1); w2 = rd_word(r, wi + 2);
                w3 = rd_word(r, wi + 3); w4 = rd_word(r, wi + 4);
            }
            // 64 stream bits at bp + lane
            const uint32_t o = (bp & 31) + (uint32_t)lane;   // 0..94
            const uint32_t kq = o >> 5, sh = o & 31;
            const uint32_t x0 = kq == 0 ? w0 : (kq == 1 ? w1 : w2);
            const uint32_t x1 = kq == 0 ? w1 : (kq == 1 ? w2 : w3);
            const uint32_t x2 = kq == 0 ? w2 : (kq == 1 ? w3 : w4);
            const uint32_t lo = __builtin_amdgcn_alignbit(x1, x0, sh);
            const uint32_t hi = __builtin_amdgcn_alignbit(x2, x1, sh);
            // litlen symbol + length extra bits
            const uint32_t e = S.lit[lo & ((1u << LB) - 1)];
            const uint32_t L = e & 15, kind = (e >> 4) & 3;
            const bool islen = kind == K_BASE;
            const uint64_t xs = ((((uint64_t)hi) << 32) | lo) >> L;
            const uint32_t xb = islen ? (e >> 8) & 15 : 0u;
            const uint32_t mlen = (e >> 16) + ((uint32_t)xs & ((1u << xb) - 1));
            // distance symbol + extra bits (harmless garbage on literal lanes)
            const uint32_t y = (uint32_t)(xs >> xb);
            const uint32_t d = S.dst[y & ((1u << DB) - 1)];
            const uint32_t L2 = d & 15, xd = (d >> 8) & 15;
            const uint32_t dist = (d >> 16) + ((y >> L2) & ((1u << xd) - 1));
            const bool special = L == 0 || kind >= K_EOB || (islen && (L2 == 0 || ((d >> 4) & 3) != K_BASE));
            const uint32_t tb = islen ? L + xb + L2 + xd : L;
            // token word: [6:0] lane of the next token, [31:23] output bytes; a special token is
            // 0xFF | lane << 8 (next lane 127 ends the walk, 0 bytes)
            const uint32_t vtok = special ? (0xFFu | ((uint32_t)lane << 8))
                                          : (((uint32_t)lane + tb) | ((islen ? mlen : 1u) << 23));
            // token info: [31] match, [15:0] distance (match) or the literal byte
            const uint32_t vinf = islen ? (0x80000000u | dist) : ((e >> 8) & 255);

            // ---- walk the real token chain (wave-uniform): lane s -> lane s + bits(s) ----
            // Records each token's info at the lane of its output offset (vtin) and the offsets in
            // the mask mo; stops when the chain leaves the 64-bit span, at a special token (which
            // is recorded with 0 bytes, harmlessly), or once no further token can start inside
            // the first lim output bytes of the round.
            const uint32_t lim = min(64u, len - pos);
            const uint32_t cl = 64u - lim;   // off < lim  <=>  off + cl < 64
            uint32_t s = 0, off = 0, t;
            uint64_t mo = 0;
            uint32_t vtin = 0;
            do {
                t = rdlane(vtok, s);
                mo |= 1ull << off;
                vtin = (uint32_t)llvm_writelane((int)rdlane(vinf, s), (int)off, (int)vtin);
                off += t >> 23;
                s = t & 127u;
            } while (max(s, off + cl) < 64u);
            const bool spec = (t & 0x80u) != 0;
            if (spec) s = (t >> 8) & 63u;
            const uint32_t rout = min(off, len - pos);   // output bytes of this round

            // ---- emit the round's first 64 output bytes, one per lane ----
            {
                const uint32_t j = (uint32_t)lane;
                const uint64_t mle = j == 63 ? ~0ull : ((2ull << j) - 1ull);   // lanes <= j
                const uint32_t sj = 63u - (uint32_t)__builtin_clzll(mo & mle);   // start of j's token (bit 0 of mo is set)
                const uint32_t inf = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(sj << 2), (int)vtin);
                const bool act = j < rout;
                const bool ism = (inf >> 31) != 0;
                const int32_t jj = (int32_t)j - (int32_t)(inf & 0xFFFFu);   // source, relative to the round
                const bool dep = act && ism && jj >= 0;                      // produced in this round
                uint32_t val = inf & 255u;
                if (act && ism && jj < 0 && jj >= -(int32_t)RING) val = S.ring[(rb0 + pos + (uint32_t)jj) & RM];
                const bool far = act && ism && jj < -(int32_t)RING;
                if (__ballot(far)) {
                    if (far) val = far_byte(out, dict, out_off, (int32_t)pos + jj);
                }
                if (__ballot(dep)) {
                    // chains inside the round (short distances): pointer doubling to a resolved byte
                    int32_t ptr = dep ? jj : (int32_t)j;
                    for (;;) {
                        const int32_t p2 = __builtin_amdgcn_ds_bpermute(ptr << 2, ptr);
                        if (!__ballot(p2 != ptr)) break;
                        ptr = p2;
                    }
                    val = (uint32_t)__builtin_amdgcn_ds_bpermute(ptr << 2, (int)val);
                }
                if (act) S.ring[(rb0 + pos + j) & RM] = (uint8_t)val;
            }
            if (rout > 64) {
                // the rest of the last token (a match): bytes 64.. of the round
                const uint32_t last = 63u - (uint32_t)__builtin_clzll(mo);
                const uint32_t dl = rdlane(vtin, last) & 0xFFFFu;
                copy_match<RB>(S.ring, out, dict, out_off, rb0, pos + 64, dl, rout - 64, lane);
            }
            pos += rout;
            if (pos >= fl_next) {
                flush_range<RB>(S.ring, out, out_off + fl_done, out_off + fl_next, lane);
                fl_done = fl_next;
                fl_next += UNIT;
            }
            bp += s;
            if (!spec) continue;

            // ---- one token by the bit-serial path (long code, end-of-block or error) ----
            rd_seek(r, bp, lane);
            rd_refill(r, lane);
            const uint32_t e1 = lookup(vlit, S.lit, (1u << LB) - 1, r, S.lit_count, S.lit_sorted, TAB_LIT);
            br_take(r, e1 & 15);
            const uint32_t kind1 = (e1 >> 4) & 3;
            if (kind1 == K_LIT) {
                if (lane == 0) S.ring[(rb0 + pos) & RM] = (uint8_t)(e1 >> 8);
                pos++;
            } else if (kind1 == K_BASE) {
                const uint32_t ml = (e1 >> 16) + br_take(r, (e1 >> 8) & 15);
                rd_refill(r, lane);
                const uint32_t d1 = lookup(vdst, S.dst, (1u << DB) - 1, r, S.dst_count, S.dst_sorted, TAB_DST);
                br_take(r, d1 & 15);
                if (((d1 >> 4) & 3) != K_BASE) { status = ST_DATA_ERROR; break; }
                const uint32_t ds = (d1 >> 16) + br_take(r, (d1 >> 8) & 15);
                const uint32_t n = min(ml, len - pos);
                copy_match<RB>(S.ring, out, dict, out_off, rb0, pos, ds, n, lane);
                pos += n;
            } else if (kind1 == K_EOB) {
                in_block = 0;
                bp = rd_pos(r);
                break;
            } else {
                status = ST_DATA_ERROR;
                break;
            }
            bp = rd_pos(r);
            if (pos >= fl_next) {
                flush_range<RB>(S.ring, out, out_off + fl_done, out_off + fl_next, lane);
                fl_done = fl_next;
                fl_next += UNIT;
            }
        }
        if (status == ST_OK) rd_seek(r, bp, lane);   // the next block header / the R-E5 check read from bp
        if (status != ST_OK) break;
    }
    flush_range<RB>(S.ring, out, out_off + fl_done, out_off + pos, lane);

    // zlib was handed only the chunk's slice (LazyFileReader.cs:63-69): needing bits past it is
    // the DATA_ERROR of Core.cs:174.  R-E5: the next symbol should be the block's end-of-block.
    uint32_t end_bit = rd_pos(r);
    if (end_bit > bit_limit) {
        flags |= PPG_FLAG_OVERRUN;
        if (status == ST_OK) status = ST_DATA_ERROR;
    }
    if (status == ST_OK && in_block && pos == len) {
        rd_refill(r, lane);
        const uint32_t e = lookup(vlit, S.lit, (1u << LB) - 1, r, S.lit_count, S.lit_sorted, TAB_LIT);
        if (((e >> 4) & 3) == K_EOB) {
            br_take(r, e & 15);
            end_bit = rd_pos(r);
        } else {
            flags |= PPG_FLAG_NO_EOB;
        }
    }
    if (lane == 0) {
        res[k].produced = pos;
        res[k].end_bit = w0abs * 32 + end_bit;
        res[k].status = status;
        res[k].flags = flags;
    }
}

// ------------------------------------------------------------------------------------------
// Host-side launcher (called from ppg_api.cpp).  ring_bits selects the history ring.
// ------------------------------------------------------------------------------------------
size_t ppg_inflate_lds_bytes(int ring_bits) {
    switch (ring_bits) {
        case 13: return sizeof(InflateLds<13>);
        case 14: return sizeof(InflateLds<14>);
        default: return sizeof(InflateLds<15>);
    }
}

hipError_t ppg_launch_inflate(hipStream_t s, int ring_bits, const uint32_t *comp, uint64_t nwords,
                              const PpgInflateJob *jobs, const uint8_t *dicts, uint8_t *out, PpgInflateResult *res,
                              int njobs) {
    if (njobs <= 0) return hipSuccess;
    switch (ring_bits) {
        case 13:
            hipLaunchKernelGGL(ppg_inflate_kernel<13>, dim3(njobs), dim3(64), sizeof(InflateLds<13>), s, comp, nwords,
                               jobs, dicts, out, res, njobs);
            break;
        case 14:
            hipLaunchKernelGGL(ppg_inflate_kernel<14>, dim3(njobs), dim3(64), sizeof(InflateLds<14>), s, comp, nwords,
                               jobs, dicts, out, res, njobs);
            break;
        default:
            hipLaunchKernelGGL(ppg_inflate_kernel<15>, dim3(njobs), dim3(64), sizeof(InflateLds<15>), s, comp, nwords,
                               jobs, dicts, out, res, njobs);
            break;
    }
    return hipGetLastError();
}
