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

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

// Compressed stream of one chunk: word i (chunk-relative) is base[i].  128 words live across the
// lanes (lane l holds words wb+2l in A and wb+2l+1 in B), so a refill is one v_readlane.  The
// buffer is reloaded with ONE global_load_dwordx2 per lane whose result is used at once: the
// wait (~one memory latency per 512 B of input, ~280 symbols) is paid there and nowhere else.
// A load whose result stayed in flight across loop iterations would make the compiler wait for
// every outstanding memory operation at each use (its per-register tracking is conservative
// around loops), and an untracked asm load can be copied by the register allocator before it
// lands.
struct Reader {
    const uint32_t *base;   // 128-word aligned
    uint32_t nw;            // readable words from base (>= 1)
    uint32_t A, B;          // words wb+2*lane, wb+2*lane+1
    uint32_t wb;            // first word of the buffer
    uint32_t wi;            // next word to append to bb
    uint64_t bb;            // bit buffer, LSB = next bit
    uint32_t bn;            // valid bits in bb
};

__device__ __forceinline__ void rd_load(Reader &r, int lane) {
    const uint32_t i = r.wb + 2 * lane;
    if (i + 1 < r.nw) {
        const uint2 v = *(const uint2 *)(r.base + i);   // 8-B aligned: wb and base are
        r.A = v.x;
        r.B = v.y;
    } else {
        r.A = i < r.nw ? r.base[i] : 0u;   // past the end: zeros (an overrun is an error anyway)
        r.B = 0u;
    }
    // consume the load here, so the compiler waits for it in this (rare) block rather than at
    // every v_readlane of A/B (there the wait would drain every store in flight, too)
    asm volatile("" ::"v"(r.A), "v"(r.B));
}

__device__ __forceinline__ uint32_t rd_word(const Reader &r, uint32_t idx) {
    return (idx & 1) ? rdlane(r.B, idx >> 1) : rdlane(r.A, idx >> 1);
}

__device__ __forceinline__ void rd_seek(Reader &r, uint32_t bit, int lane) {
    r.wi = bit >> 5;
    r.wb = r.wi & ~127u;
    rd_load(r, lane);
    const uint32_t w = rd_word(r, r.wi - r.wb);
    r.wi++;
    const uint32_t sh = bit & 31;
    r.bb = (uint64_t)(w >> sh);
    r.bn = 32 - sh;
}

// guarantees bn >= 32
__device__ __forceinline__ void rd_refill(Reader &r, int lane) {
    if (r.bn <= 32) {
        if (r.wi == r.wb + 128) {
            r.wb += 128;
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
    r.base = comp + w0abs;
    r.nw = (uint32_t)min(nwords > w0abs ? nwords - w0abs : 1ull, 0xFFFFFFFFull);
    const uint32_t bit_limit = (uint32_t)min(J.bit_limit - w0abs * 32, 0xFFFFFFFFull);
    rd_seek(r, (uint32_t)(J.bit_start - w0abs * 32), lane);

    uint32_t pos = 0;                                        // output bytes produced
    uint32_t fl_done = 0;                                    // flushed up to this position
    uint32_t fl_next = UNIT - (uint32_t)(out_off & (UNIT - 1));   // next global 4 KiB boundary
    int status = ST_OK, flags = 0, last = 0, in_block = 0;
    uint32_t vlit = 0, vdst = 0;    // first-level tables (one entry per lane)
    uint32_t pv = 0;                // deferred match bytes (one per lane) ...
    uint32_t ppos = 0, pn = 0;      // ... for ring slots [ppos, ppos + pn)

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
        pn = 0;

        // ---- token loop: everything below is wave-uniform (scalar branches) ----
        while (pos < len) {
            rd_refill(r, lane);
            const uint32_t e = lookup(vlit, S.lit, (1u << LB) - 1, r, S.lit_count, S.lit_sorted, TAB_LIT);
            br_take(r, e & 15);
            const uint32_t kind = (e >> 4) & 3;
            if (kind == K_LIT) {
                if (pn) { if ((uint32_t)lane < pn) S.ring[(ppos + lane) & RM] = (uint8_t)pv; pn = 0; }
                if (lane == 0) S.ring[(rb0 + pos) & RM] = (uint8_t)(e >> 8);
                pos++;
            } else if (kind == K_BASE) {
                const uint32_t mlen = (e >> 16) + br_take(r, (e >> 8) & 15);
                rd_refill(r, lane);
                const uint32_t d = lookup(vdst, S.dst, (1u << DB) - 1, r, S.dst_count, S.dst_sorted, TAB_DST);
                br_take(r, d & 15);
                if (((d >> 4) & 3) != K_BASE) { status = ST_DATA_ERROR; break; }
                const uint32_t dist = (d >> 16) + br_take(r, (d >> 8) & 15);
                const uint32_t n = min(mlen, len - pos);
                if (pn) { if ((uint32_t)lane < pn) S.ring[(ppos + lane) & RM] = (uint8_t)pv; pn = 0; }
                const uint32_t dst0 = rb0 + pos;          // ring slot of the first output byte
                if (dist + n <= RING) {
                    // source entirely in the ring and never overwritten by this copy; every
                    // source byte precedes pos, so no 64-byte group reads another's output.  The
                    // last group's write is deferred: its LDS read overlaps the next decode.
                    const uint32_t src0 = dst0 - dist;
                    uint32_t j0 = 0;
                    if (dist >= n) {
                        for (; j0 + 64 < n; j0 += 64) {
                            const uint8_t v = S.ring[(src0 + j0 + lane) & RM];
                            S.ring[(dst0 + j0 + lane) & RM] = v;
                        }
                        if (j0 + lane < n) pv = S.ring[(src0 + j0 + lane) & RM];
                    } else {
                        // overlapping run: byte j repeats byte j mod dist
                        for (; j0 + 64 < n; j0 += 64) {
                            const uint8_t v = S.ring[(src0 + (j0 + lane) % dist) & RM];
                            S.ring[(dst0 + j0 + lane) & RM] = v;
                        }
                        if (j0 + lane < n) pv = S.ring[(src0 + (j0 + lane) % dist) & RM];
                    }
                    ppos = dst0 + j0;
                    pn = n - j0;
                } else {
                    // far reference (dist > RING - n >= n): bytes older than the ring come from
                    // the flushed output or the Point's window; the flush stores complete first
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    for (uint32_t j0 = 0; j0 < n; j0 += 64) {
                        const uint32_t j = j0 + lane;
                        if (j < n) {
                            const uint32_t back = dist - j;                 // source = pos - back
                            const int32_t rel = (int32_t)pos - (int32_t)back;
                            uint8_t v;
                            if (back + n <= RING) v = S.ring[(dst0 - back) & RM];
                            else if (rel >= 0) v = out[out_off + (uint32_t)rel];
                            else v = dict[32768 + rel];                    // rel >= -32768
                            S.ring[(dst0 + j) & RM] = v;
                        }
                    }
                }
                pos += n;
            } else if (kind == K_EOB) {
                in_block = 0;
                break;
            } else {
                status = ST_DATA_ERROR;
                break;
            }
            if (pos >= fl_next) {
                if (pn) { if ((uint32_t)lane < pn) S.ring[(ppos + lane) & RM] = (uint8_t)pv; pn = 0; }
                flush_range<RB>(S.ring, out, out_off + fl_done, out_off + fl_next, lane);
                fl_done = fl_next;
                fl_next += UNIT;
            }
        }
        if (pn) { if ((uint32_t)lane < pn) S.ring[(ppos + lane) & RM] = (uint8_t)pv; pn = 0; }
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
