// ppg_index.hip — gfx950 kernels of the GPU CreateIndex (host side: ppg_index_gpu.cpp).
//
// Core.BuildDeflateIndex (Decompressor/Core.cs:14-131) is one serial zlib pass over the whole
// member.  On the GPU the member is cut into pieces that are decoded in parallel
// (ppg_inflate_kernel<.., IX = true>); these kernels supply the pieces' starting points, the
// 32 KiB histories that chain them, and the '@' census from which the Points are chosen:
//   ppg_block_find_kernel   first plausible dynamic-block header at or after each piece's nominal
//                           start (one wave per piece; lanes test 64 bit offsets at a time)
//   ppg_gather_kernel       32 KiB histories ending at a given output position (piece tails,
//                           Point windows), optionally compared against a previous copy
//   ppg_at_stats_kernel     per-block '@' count / first / last / largest gap (Core.cs:79-96)
//   ppg_resolve_kernel      exact starting histories of all pieces from their symbolic tails
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include "ppg_device.h"
#include "ppg_huffman.h"

namespace {

// wave-uniform bit reader straight from global memory (the finder's header check)
struct GBits {
    const uint32_t *w;
    uint64_t nw;
    uint64_t pos;
    __device__ uint32_t peek() const {
        const uint64_t i = pos >> 5;
        const uint32_t x0 = i < nw ? w[i] : 0u, x1 = i + 1 < nw ? w[i + 1] : 0u;
        return __builtin_amdgcn_alignbit(x1, x0, (uint32_t)(pos & 31));
    }
    __device__ uint32_t take(uint32_t n) {
        const uint32_t v = peek() & ((1u << n) - 1u);
        pos += n;
        return v;
    }
};

struct FindLds {
    uint8_t lens[320];
    uint32_t cl[1 << CB];
    uint32_t scratch[64];
    uint16_t sorted[288];
};

// Would zlib 1.2.11 accept a dynamic-block header at bit c?  (inflate.c TABLE/LENLENS/CODELENS:
// HLIT/HDIST ranges, complete code-length code, repeat rules, litlen/distance codes per
// inflate_table, end-of-block present.)  Every true block header passes; false positives are
// caught by the pass-1 chain check.
__device__ bool header_ok(const uint32_t *comp, uint64_t nwords, uint64_t c, FindLds &S, int lane) {
    GBits g{comp, nwords, c + 3};
    const uint32_t hlit = g.take(5) + 257, hdist = g.take(5) + 1, hclen = g.take(4) + 4;
    if (hlit > 286 || hdist > 30) return false;
    {
        GBits f{comp, nwords, g.pos + 3ull * (uint32_t)(lane < 19 ? lane : 0)};
        const uint32_t v = f.take(3);
        __syncthreads();
        if (lane < 19) S.lens[c_clorder[lane]] = (uint8_t)((uint32_t)lane < hclen ? v : 0u);
        __syncthreads();
    }
    g.pos += 3ull * hclen;
    if (build_table<CB>(S.lens, 19, S.cl, nullptr, S.sorted, TAB_CL, lane) != 0) return false;
    uint32_t idx = 0;
    const uint32_t total = hlit + hdist;
    // running Kraft sums (units of 2^-15) of the litlen and distance codes: an over-subscribed code
    // is one inflate_table refuses, so a false start -- random bits decode into code lengths that
    // over-subscribe within a few symbols -- is rejected here instead of after all hlit + hdist
    // lengths (r05: this check and the staged scan took a lone chunk's search 4.4 -> ~0.3 ms)
    uint32_t kl = 0, kd = 0;
    while (idx < total) {
        const uint32_t e = uni(S.cl[g.peek() & ((1u << CB) - 1)]);
        const uint32_t L = e & 15;
        if (L == 0) return false;
        g.pos += L;
        const uint32_t sym = e >> 8;
        uint32_t val = 0, rep = 1;
        if (sym < 16) {
            val = sym;
        } else if (sym == 16) {
            if (idx == 0) return false;
            val = uni(S.lens[idx - 1]);
            rep = 3 + g.take(2);
        } else if (sym == 17) {
            rep = 3 + g.take(3);
        } else {
            rep = 11 + g.take(7);
        }
        if (idx + rep > total) return false;
        if (val) {
            const uint32_t nl = idx < hlit ? min(rep, hlit - idx) : 0u, nd = rep - nl;
            kl += nl << (15 - val);
            kd += nd << (15 - val);
            if (kl > (1u << 15) || kd > (1u << 15)) return false;
        }
        for (uint32_t j0 = 0; j0 < rep; j0 += 64)
            if (j0 + lane < rep) S.lens[idx + j0 + lane] = (uint8_t)val;
        idx += rep;
        __syncthreads();
    }
    if (uni(S.lens[256]) == 0) return false;
    // validity only (build_table's checks); the 64-entry table is scratch
    if (build_table<6>(S.lens, (int)hlit, S.scratch, nullptr, S.sorted, TAB_LIT, lane) != 0) return false;
    if (build_table<6>(S.lens + hlit, (int)hdist, S.scratch, nullptr, S.sorted, TAB_DST, lane) != 0) return false;
    return true;
}

}  // namespace

// cand[k] = the first bit b in [lo[k], hi[k]) where a dynamic Huffman block header zlib would
// accept starts, or ~0.  Prefilter per lane: BFINAL = 0, BTYPE = 2, HLIT <= 29, HDIST <= 29 and a complete
// code-length code (Kraft sum exactly 1); survivors get the full header_ok check, lowest first.
// sub > 1: range k is searched by `sub` waves at once (blockIdx.y = part of the range), each from
// the start of its part; the lowest find wins (atomic min; cand[k] = ~0 beforehand) -- a lone
// chunk's few ranges then take a fraction of one wave's scan (ppg_decompress_chunk)
__global__ __launch_bounds__(64) void ppg_block_find_kernel(const uint32_t *__restrict__ comp, uint64_t nwords,
                                                            const uint64_t *__restrict__ lo,
                                                            const uint64_t *__restrict__ hi, uint64_t *cand, int n) {
    __shared__ FindLds S;
    const int k = blockIdx.x;
    const int lane = threadIdx.x;
    if (k >= n) return;
    const uint32_t sub = gridDim.y, part = blockIdx.y;
    uint64_t a = lo[k], b = hi[k];
    if (sub > 1) {
        const uint64_t span = b > a ? b - a : 0;
        const uint64_t a2 = a + span * part / sub, b2 = a + span * (part + 1) / sub;
        a = a2;
        b = b2;
    }
    uint64_t found = ~0ull;
    for (uint64_t base = a; base < b; base += 64) {
        const uint64_t bit = base + (uint64_t)lane;
        const uint64_t w = bit >> 5;
        const uint32_t sh = (uint32_t)(bit & 31);
        const uint32_t x0 = w < nwords ? comp[w] : 0u, x1 = w + 1 < nwords ? comp[w + 1] : 0u;
        const uint32_t x2 = w + 2 < nwords ? comp[w + 2] : 0u, x3 = w + 3 < nwords ? comp[w + 3] : 0u;
        const uint32_t v0 = __builtin_amdgcn_alignbit(x1, x0, sh);
        const uint32_t v1 = __builtin_amdgcn_alignbit(x2, x1, sh);
        const uint32_t v2 = __builtin_amdgcn_alignbit(x3, x2, sh);
        const uint64_t u01 = ((uint64_t)v1 << 32) | v0, u12 = ((uint64_t)v2 << 32) | v1;
        // BFINAL = 0: an inner block start is never the member's last block (missing that one only
        // lengthens the piece before it), and the bit halves the survivors of the prefilter, whose
        // serial header_ok checks are what the scan spends its time on
        bool ok = bit < b && (v0 & 7) == 4 && ((v0 >> 3) & 31) <= 29 && ((v0 >> 8) & 31) <= 29;
        const uint32_t ncl = ((v0 >> 13) & 15) + 4;
        uint32_t kraft = 0;
#pragma unroll
        for (uint32_t i = 0; i < 19; i++) {
            const uint32_t o = 17 + 3 * i;
            const uint32_t L = (uint32_t)((o + 3 <= 64 ? (u01 >> o) : (u12 >> (o - 32))) & 7u);
            kraft += (i < ncl && L) ? (128u >> L) : 0u;
        }
        ok = ok && kraft == 128;
        uint64_t m = __ballot(ok);
        while (m) {
            const uint32_t c = (uint32_t)__builtin_ctzll(m);
            if (header_ok(comp, nwords, base + c, S, lane)) {
                found = base + c;
                break;
            }
            m &= m - 1;
        }
        if (found != ~0ull) break;
        // a lower part has found one already: nothing here can win
        if (sub > 1 && part > 0 && uni64(*(volatile const uint64_t *)&cand[k]) < a) break;
    }
    if (lane == 0) {
        if (sub > 1) {
            if (found != ~0ull) atomicMin((unsigned long long *)&cand[k], (unsigned long long)found);
        } else {
            cand[k] = found;
        }
    }
}

// dst[k] = the 32 KiB of history before output position g[k].end of a piece: position p >= 0 is
// out[out_off + (p & mask)] (mask: 64 KiB rings of pass 1, or ~0), p < 0 is
// dicts[dict_off + 32768 + p] (the piece's own starting history).  With ref, diff[k] = 1 when
// the new history differs from ref[ref_off, +32768).
__global__ __launch_bounds__(256) void ppg_gather_kernel(const uint8_t *__restrict__ out,
                                                         const uint8_t *__restrict__ dicts,
                                                         const PpgGather *__restrict__ g, uint8_t *__restrict__ dst,
                                                         const uint8_t *__restrict__ ref, uint32_t *diff, int n) {
    const int k = blockIdx.x;
    if (k >= n) return;
    const PpgGather G = g[k];
    uint32_t *d32 = (uint32_t *)(dst + (uint64_t)k * 32768);
    const uint32_t *r32 = ref ? (const uint32_t *)(ref + G.ref_off) : nullptr;
    int differs = 0;
    for (uint32_t i = threadIdx.x; i < 8192; i += 256) {
        uint32_t v = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int64_t p = (int64_t)G.end - 32768 + 4 * (int64_t)i + q;
            const uint32_t byte = p >= 0 ? out[G.out_off + ((uint64_t)p & G.mask)] : dicts[G.dict_off + 32768 + p];
            v |= byte << (8 * q);
        }
        d32[i] = v;
        if (r32 && r32[i] != v) differs = 1;
    }
    differs = __syncthreads_or(differs);
    if (diff && threadIdx.x == 0) diff[k] = (uint32_t)differs;
}

// '@' census of out[s.lo, s.hi) per block (Core.cs:79-96): count, first and last '@' (relative to
// lo) and the largest distance between consecutive '@' inside the block (SURVEY Q4 needs the
// gaps).  One wave per block, 16 bytes per lane per 1 KiB step, four steps' loads issued together;
// the "last '@' so far" prefix maximum is a DPP scan (r03: six ds_bpermute-based shuffles per step
// held the kernel at ~2.3 TB/s).
__device__ __forceinline__ uint32_t at_mask16(uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t x = w[j] ^ 0x40404040u;   // '@' bytes -> 0
        const uint32_t t = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
        m |= (((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u)) << (4 * j);
    }
    return m;
}

// inclusive prefix maximum over the wave (DPP row shifts + row broadcasts, GFX9 encodings); lanes
// without a source take -1
__device__ __forceinline__ int32_t wave_incl_max(int32_t x) {
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xF, 0xF, false));   // row_shr:1
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xF, 0xF, false));   // row_shr:2
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xF, 0xF, false));   // row_shr:4
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xF, 0xF, false));   // row_shr:8
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x142, 0xA, 0xF, false));   // row_bcast:15
    x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x143, 0xC, 0xF, false));   // row_bcast:31
    return x;
}

__global__ __launch_bounds__(64) void ppg_at_stats_kernel(const uint8_t *__restrict__ out,
                                                          const PpgSpan *__restrict__ spans, PpgAtStats *st, int n) {
    const int k = blockIdx.x;
    const int lane = threadIdx.x;
    if (k >= n) return;
    const uint64_t a = spans[k].lo, b = spans[k].hi;
    uint32_t cnt = 0, gmax = 0;
    int32_t first = 0x7FFFFFFF, carry = -1;   // carry: last '@' so far (relative), -1 none
    for (uint64_t g0 = a & ~15ull; g0 < b; g0 += 4096) {
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t q = g0 + 1024ull * i + 16ull * (uint64_t)lane;
            v[i] = q < b ? *(const uint4 *)(out + q) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t q = g0 + 1024ull * i + 16ull * (uint64_t)lane;
            uint32_t m = q < b ? at_mask16(v[i]) : 0u;
            if (q < a) m &= 0xFFFFu << (uint32_t)(a - q);   // lane 0 of the first step only
            if (q < b && q + 16 > b) m &= (1u << (uint32_t)(b - q)) - 1u;
            const int32_t rel = (int32_t)(q - a);
            const int32_t f = m ? rel + __builtin_ctz(m) : 0x7FFFFFFF;
            const int32_t l = m ? rel + 31 - __builtin_clz(m) : -1;
            // gaps between consecutive '@' of this lane's 16 bytes
            uint32_t mm = m, lg = 0;
            int32_t prev = -1;
            while (mm) {
                const int32_t j = __builtin_ctz(mm);
                if (prev >= 0) lg = max(lg, (uint32_t)(j - prev));
                prev = j;
                mm &= mm - 1;
            }
            // last '@' before this lane's bytes: prefix max over lower lanes, then the carry
            const int32_t incl = wave_incl_max(l);
            const int32_t excl = max(__builtin_amdgcn_update_dpp(-1, incl, 0x138, 0xF, 0xF, false), carry);   // wave_shr:1
            if (m && excl >= 0) lg = max(lg, (uint32_t)(f - excl));
            gmax = max(gmax, lg);
            carry = max(carry, __builtin_amdgcn_readlane(incl, 63));
            cnt += (uint32_t)__builtin_popcount(m);
            first = min(first, f);
        }
    }
    for (int d = 32; d >= 1; d >>= 1) {
        cnt += __shfl_xor(cnt, d);
        gmax = max(gmax, (uint32_t)__shfl_xor((int)gmax, d));
        first = min(first, __shfl_xor(first, d));
    }
    if (lane == 0) st[k] = PpgAtStats{cnt, first == 0x7FFFFFFF ? -1 : first, carry, gmax};
}

// dense[pre[k] + i] = blk[jobs[k].blk_off + i] for i < min(res[k].nblocks, blk_cap): pass-1 block
// lists packed for one device-to-host copy
__global__ __launch_bounds__(256) void ppg_pack_blocks_kernel(const PpgBlockEnd *__restrict__ blk,
                                                              const PpgInflateJob *__restrict__ jobs,
                                                              const PpgInflateResult *__restrict__ res,
                                                              const uint64_t *__restrict__ pre, PpgBlockEnd *dense, int n) {
    const int k = blockIdx.x;
    if (k >= n) return;
    const uint32_t nb = min(res[k].nblocks, jobs[k].blk_cap);
    for (uint32_t i = threadIdx.x; i < nb; i += 256) dense[pre[k] + i] = blk[jobs[k].blk_off + i];
}

hipError_t ppg_launch_pack_blocks(hipStream_t s, const PpgBlockEnd *blk, const PpgInflateJob *jobs,
                                  const PpgInflateResult *res, const uint64_t *pre, PpgBlockEnd *dense, int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_pack_blocks_kernel, dim3(n), dim3(256), 0, s, blk, jobs, res, pre, dense, n);
    return hipGetLastError();
}

// Symbolic tails: pass 1 decodes every piece twice, with history patterns A[i] = i & 0xFF and
// B[i] = ((i >> 8) + 1 + (i & 0xFF)) & 0xFF.  Decoding only copies bytes, so an output byte is
// either a literal (x == y in both runs) or history byte i (x = A[i], y = B[i], x != y, and
// i = ((((y - x) & 0xFF) - 1) << 8) | x).  Piece j+1 starts with piece j's last 32 KiB, so
//   W[j+1] = T_j(W[j]),  T_j(W)[t] = x == y ? x : W[i(x, y)],   W[0] = zeros (the stream start).
// The chain is serial, but the maps compose: as u16 entries (0x8000 | literal, or a history index)
// T_{j+1} o T_j is again such a map.  So the pieces are cut into G groups of L (G, L ~ sqrt(np)):
//   compose  (G workgroups)  M_g = T_{last} o ... o T_{first} of group g, in LDS;
//   groups   (1 workgroup)   W[first of g+1] = M_g(W[first of g]), g = 0..G-1;
//   fill     (G workgroups)  the W of every piece inside its group, from the group's first.
// ~3 sqrt(np) dependent 32 KiB steps instead of np (r01-v12 form: one workgroup, np steps).
__device__ __forceinline__ uint32_t sym_entry(uint32_t x, uint32_t y) {
    return x == y ? 0x8000u | x : (((((y - x) & 255u) - 1u) << 8) | x) & 0x7FFFu;   // (mask: corrupt data stays in range)
}

// entries 4t..4t+3 of piece j's tail: 16-bit symbols straight from pass 1 (tb == nullptr: ta holds
// 32 Ki u16 per slot, r03), or from two byte tails over two synthetic histories (sym_entry)
__device__ __forceinline__ void tail4(const uint8_t *ta, const uint8_t *tb, uint32_t slot, uint32_t t, uint32_t e[4]) {
    if (!tb) {
        const uint2 v = ((const uint2 *)(ta + (uint64_t)slot * 65536))[t];
        e[0] = v.x & 0xFFFFu; e[1] = v.x >> 16; e[2] = v.y & 0xFFFFu; e[3] = v.y >> 16;
#pragma unroll
        for (int q = 0; q < 4; q++) e[q] &= (e[q] & 0x8000u) ? 0x80FFu : 0x7FFFu;   // corrupt data stays in range
        return;
    }
    const uint32_t xa = ((const uint32_t *)(ta + (uint64_t)slot * 32768))[t];
    const uint32_t xb = ((const uint32_t *)(tb + (uint64_t)slot * 32768))[t];
#pragma unroll
    for (int q = 0; q < 4; q++) e[q] = sym_entry((xa >> (8 * q)) & 255u, (xb >> (8 * q)) & 255u);
}

__global__ __launch_bounds__(1024) void ppg_resolve_compose_kernel(const uint8_t *__restrict__ ta,
                                                                   const uint8_t *__restrict__ tb,
                                                                   const uint32_t *__restrict__ slots, int np,
                                                                   int L, uint16_t *__restrict__ M) {
    __shared__ uint16_t m[32768];
    const int j0 = blockIdx.x * L, j1 = min(np, j0 + L);
    if (j0 >= j1) return;
    for (int j = j0; j < j1; j++) {
        uint32_t nv[16];   // this thread's 32 new entries, two per register
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const uint32_t t = threadIdx.x + 1024u * r;   // 4 entries 4t..4t+3
            uint32_t e[4];
            tail4(ta, tb, slots[j], t, e);
#pragma unroll
            for (int q = 0; q < 4; q++) e[q] = (j == j0 || (e[q] & 0x8000u)) ? e[q] : m[e[q]];
            nv[2 * r] = e[0] | (e[1] << 16);
            nv[2 * r + 1] = e[2] | (e[3] << 16);
        }
        __syncthreads();   // every read of the old map is done
#pragma unroll
        for (int r = 0; r < 8; r++) {
            uint32_t *m32 = (uint32_t *)m;
            const uint32_t t = threadIdx.x + 1024u * r;
            m32[2 * t] = nv[2 * r];
            m32[2 * t + 1] = nv[2 * r + 1];
        }
        __syncthreads();
    }
    uint32_t *dst = (uint32_t *)(M + (uint64_t)blockIdx.x * 32768);
    for (uint32_t t = threadIdx.x; t < 16384; t += 1024) dst[t] = ((const uint32_t *)m)[t];
}

__global__ __launch_bounds__(1024) void ppg_resolve_groups_kernel(const uint16_t *__restrict__ M, int np, int L,
                                                                  int G, uint8_t *W) {
    for (int g = 0; g < G; g++) {
        const int j0 = g * L, j1 = min(np, j0 + L);
        const uint8_t *src = W + (uint64_t)j0 * 32768;
        uint32_t *d = (uint32_t *)(W + (uint64_t)j1 * 32768);
        const uint32_t *mg = (const uint32_t *)(M + (uint64_t)g * 32768);
        for (uint32_t t = threadIdx.x; t < 8192; t += 1024) {
            const uint32_t e01 = mg[2 * t], e23 = mg[2 * t + 1];
            const uint32_t e[4] = {e01 & 0xFFFFu, e01 >> 16, e23 & 0xFFFFu, e23 >> 16};
            uint32_t v = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) v |= (e[q] & 0x8000u ? e[q] & 255u : (uint32_t)src[e[q]]) << (8 * q);
            d[t] = v;
        }
        __threadfence_block();
        __syncthreads();
    }
}

__global__ __launch_bounds__(1024) void ppg_resolve_fill_kernel(const uint8_t *__restrict__ ta,
                                                                const uint8_t *__restrict__ tb,
                                                                const uint32_t *__restrict__ slots, int np, int L,
                                                                uint8_t *W) {
    const int j0 = blockIdx.x * L, j1 = min(np, j0 + L);
    for (int j = j0; j + 1 < j1; j++) {   // W[j1] came from the groups pass
        const uint8_t *src = W + (uint64_t)j * 32768;
        uint32_t *d = (uint32_t *)(W + (uint64_t)(j + 1) * 32768);
        for (uint32_t t = threadIdx.x; t < 8192; t += 1024) {
            uint32_t e[4], v = 0;
            tail4(ta, tb, slots[j], t, e);
#pragma unroll
            for (int q = 0; q < 4; q++) v |= (e[q] & 0x8000u ? e[q] & 255u : (uint32_t)src[e[q]]) << (8 * q);
            d[t] = v;
        }
        __threadfence_block();
        __syncthreads();
    }
}

// Many short chains at once (the per-chunk Decompress path, ppg_chunk.cpp find_mat: one chain per
// chunk of ~16 pieces, up to 256 chunks a launch): one workgroup per chain, its steps serial with the
// current history in LDS -- composing maps only pays for one long chain.  chains[c] = {wb, m, src}:
//   W[wb] = windows[src],  W[wb + j + 1] = T_{slots[wb + j]}(W[wb + j]),  j < m - 1.
__global__ __launch_bounds__(1024) void ppg_resolve_chains_kernel(const uint8_t *__restrict__ ta,
                                                                  const uint32_t *__restrict__ slots,
                                                                  const uint4 *__restrict__ chains,
                                                                  const uint8_t *__restrict__ windows, uint8_t *W) {
    __shared__ uint32_t h[2][8192];
    const uint4 c = chains[blockIdx.x];
    const uint32_t *src = (const uint32_t *)(windows + (uint64_t)c.z * 32768);
    uint32_t *w0 = (uint32_t *)(W + (uint64_t)c.x * 32768);
    for (uint32_t t = threadIdx.x; t < 8192; t += 1024) {
        const uint32_t v = src[t];
        h[0][t] = v;
        w0[t] = v;
    }
    __syncthreads();
    for (uint32_t j = 0; j + 1 < c.y; j++) {
        const uint8_t *cur = (const uint8_t *)h[j & 1];
        uint32_t *nx = h[(j + 1) & 1];
        uint32_t *d = (uint32_t *)(W + (uint64_t)(c.x + j + 1) * 32768);
        const uint32_t slot = slots[c.x + j];
#pragma unroll 2
        for (uint32_t t = threadIdx.x; t < 8192; t += 1024) {
            uint32_t e[4], v = 0;
            tail4(ta, nullptr, slot, t, e);
#pragma unroll
            for (int q = 0; q < 4; q++) v |= (e[q] & 0x8000u ? e[q] & 255u : (uint32_t)cur[e[q]]) << (8 * q);
            nx[t] = v;
            d[t] = v;
        }
        __syncthreads();
    }
}

hipError_t ppg_launch_resolve_chains(hipStream_t s, const uint8_t *ta, const uint32_t *slots, const uint4 *chains,
                                     int nchains, const uint8_t *windows, uint8_t *W) {
    if (nchains <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_resolve_chains_kernel, dim3(nchains), dim3(1024), 0, s, ta, slots, chains, windows, W);
    return hipGetLastError();
}

// dst window i = src window idx[i] (32 KiB each): the kept histories of many chains, packed for one copy
__global__ __launch_bounds__(256) void ppg_pick_windows_kernel(const uint8_t *__restrict__ src,
                                                               const uint32_t *__restrict__ idx, uint8_t *dst) {
    const uint4 *s = (const uint4 *)(src + (uint64_t)idx[blockIdx.x] * 32768);
    uint4 *d = (uint4 *)(dst + (uint64_t)blockIdx.x * 32768);
    for (uint32_t t = threadIdx.x; t < 2048; t += 256) d[t] = s[t];
}

hipError_t ppg_launch_pick_windows(hipStream_t s, const uint8_t *src, const uint32_t *idx, int n, uint8_t *dst) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_pick_windows_kernel, dim3(n), dim3(256), 0, s, src, idx, dst);
    return hipGetLastError();
}

// W[1..np] from W[0] (zeroed by the caller); M: scratch of ppg_resolve_groups(np) x 32768 u16
int ppg_resolve_groups(int np) {
    int g = 1;
    while ((int64_t)g * g < np) g++;
    return g;
}

hipError_t ppg_launch_resolve(hipStream_t s, const uint8_t *ta, const uint8_t *tb, const uint32_t *slots, int np,
                              uint8_t *W, uint16_t *M) {
    if (np <= 0) return hipSuccess;
    const int G0 = ppg_resolve_groups(np), L = (np + G0 - 1) / G0, G = (np + L - 1) / L;
    hipLaunchKernelGGL(ppg_resolve_compose_kernel, dim3(G), dim3(1024), 0, s, ta, tb, slots, np, L, M);
    hipLaunchKernelGGL(ppg_resolve_groups_kernel, dim3(1), dim3(1024), 0, s, M, np, L, G, W);
    hipLaunchKernelGGL(ppg_resolve_fill_kernel, dim3(G), dim3(1024), 0, s, ta, tb, slots, np, L, W);
    return hipGetLastError();
}

hipError_t ppg_launch_block_find(hipStream_t s, const uint32_t *comp, uint64_t nwords, const uint64_t *lo,
                                 const uint64_t *hi, uint64_t *cand, int n, int sub) {
    if (n <= 0) return hipSuccess;
    sub = std::max(1, std::min(sub, 256));
    if (sub > 1) {
        const hipError_t e = hipMemsetAsync(cand, 0xFF, 8 * (size_t)n, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(ppg_block_find_kernel, dim3(n, sub), dim3(64), 0, s, comp, nwords, lo, hi, cand, n);
    return hipGetLastError();
}

hipError_t ppg_launch_gather(hipStream_t s, const uint8_t *out, const uint8_t *dicts, const PpgGather *g, uint8_t *dst,
                             const uint8_t *ref, uint32_t *diff, int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_gather_kernel, dim3(n), dim3(256), 0, s, out, dicts, g, dst, ref, diff, n);
    return hipGetLastError();
}

hipError_t ppg_launch_at_stats(hipStream_t s, const uint8_t *out, const PpgSpan *spans, PpgAtStats *st, int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_at_stats_kernel, dim3(n), dim3(64), 0, s, out, spans, st, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// CRC-32 of the exact output (GPU CreateIndex, RFC 1952 trailer check that zlib's gzip mode makes
// in the reference's CreateIndex, Core.cs:30 inflateInit2(47) -> Z_DATA_ERROR at Core.cs:68-74).
//
// Register algebra (reflected CRC-32, poly 0xEDB88320): R(c, A||B) = R(0, B) ^ Z(c, |B|), where
// Z(c, n) = R(c, n zero bytes) is linear in c.  A batch of n bytes is viewed front-padded with
// zeros to a multiple of kCrcSeg (R(0, zeros||A) = R(0, A)); one wave per kCrcSeg virtual bytes,
// one lane per kCrcSub of them: lane registers start at 0, the wave folds them in order with the
// table of Z(., kCrcSub) (4 x 256 u32), and the host folds the segments with Z(., kCrcSeg) and the
// batches with zlib's crc32_combine (= Z(c1, n2) ^ c2).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void ppg_crc_kernel(const uint8_t *__restrict__ out, uint64_t n, uint64_t pad,
                                                     const uint32_t *__restrict__ tabs, uint32_t *__restrict__ seg_raw,
                                                     uint64_t nseg) {
    __shared__ uint32_t T[4][256];   // slicing-by-4 byte tables
    __shared__ uint32_t Z[4][256];   // Z(., kCrcSub) by byte lane
    __shared__ uint32_t part[64];
    const int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) {
        (&T[0][0])[i] = tabs[i];
        (&Z[0][0])[i] = tabs[1024 + i];
    }
    __syncthreads();
    const uint64_t w = blockIdx.x;
    if (w >= nseg) return;
    // this lane's real byte range [a, b) of the batch (virtual v -> real v - pad)
    const uint64_t v0 = w * (uint64_t)kCrcSeg + (uint64_t)lane * kCrcSub;
    const uint64_t a = v0 + kCrcSub <= pad ? 0 : (v0 < pad ? 0 : v0 - pad);
    const uint64_t b = v0 + kCrcSub <= pad ? 0 : min(n, v0 + kCrcSub - pad);
    uint32_t c = 0;
    uint64_t p = a;
    auto byte = [&](uint32_t x) { c = T[0][(c ^ x) & 255] ^ (c >> 8); };
    for (; p < b && (p & 15); p++) byte(out[p]);
    for (; p + 16 <= b; p += 16) {
        const uint4 q = *(const uint4 *)(out + p);
        const uint32_t ws[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t x = c ^ ws[j];
            c = T[3][x & 255] ^ T[2][(x >> 8) & 255] ^ T[1][(x >> 16) & 255] ^ T[0][x >> 24];
        }
    }
    for (; p < b; p++) byte(out[p]);
    part[lane] = c;
    __syncthreads();
    if (lane == 0) {
        uint32_t r = 0;
        for (int i = 0; i < 64; i++)
            r = (Z[0][r & 255] ^ Z[1][(r >> 8) & 255] ^ Z[2][(r >> 16) & 255] ^ Z[3][r >> 24]) ^ part[i];
        seg_raw[w] = r;
    }
}

hipError_t ppg_launch_crc(hipStream_t s, const uint8_t *out, uint64_t n, uint64_t pad, const uint32_t *tabs,
                          uint32_t *seg_raw, uint64_t nseg) {
    if (!nseg) return hipSuccess;
    hipLaunchKernelGGL(ppg_crc_kernel, dim3((uint32_t)nseg), dim3(64), 0, s, out, n, pad, tabs, seg_raw, nseg);
    return hipGetLastError();
}
