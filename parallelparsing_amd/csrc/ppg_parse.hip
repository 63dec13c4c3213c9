// ppg_parse.hip — gfx950 kernels for the FASTQ record scan of the DecompressAll path
// (Decompressor/Parsing.cs:11-69 over raw_k = offset_k ++ chunk_k).
//
//   ppg_parse_finish  per-chunk record counts from the newline census fused into the inflate
//                     flush, + whether "record j = newlines 4j..4j+3" equals the serial machine (R-P3)
//   ppg_parse_place   per-record descriptors (n1..n4) from the census's stored newline positions
//   ppg_parse_serial  the exact Parsing.Parse state machine for chunks the census declines
//   ppg_scan_counts   exclusive scan of per-chunk record counts -> record bases
//   ppg_parse_emit    descriptors by scanning the body (chunks whose census overflowed nl_cap)
//   ppg_record_keys   per-record spot ("major") number from the identifier line, for pairing
//                     the two files of a read pair
//   ppg_split_merge   chunks decoded as several sub-jobs (ppg_shard_set_split): one chunk result
//                     and one contiguous newline census per chunk, as if one wave had decoded it
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include "ppg_device.h"

// ------------------------------------------------------------------------------------------
// FASTQ record scan.  raw_k = offset_k ++ out[out_off, out_off+produced).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint8_t raw_at(const uint8_t *off, uint32_t off_len, const uint8_t *body, uint64_t blen,
                                          uint64_t i) {
    if (i < off_len) return off[i];
    i -= off_len;
    return i < blen ? body[i] : (uint8_t)0;
}

// Per-chunk record counts from the newline census that ppg_inflate_kernel fused into its output
// flush: raw_k = offset_k ++ body_k has off_nl + body_nl newlines; "record j = newlines 4j..4j+3"
// equals the serial state machine unless raw_k has an empty line or a NUL (R-P3) -- those chunks
// go to ppg_parse_serial.  One thread per chunk.
extern "C" __global__ __launch_bounds__(256) void ppg_parse_finish(const PpgInflateResult *__restrict__ ires,
                                                                   const PpgOffsetRef *__restrict__ oref,
                                                                   PpgParseInfo *__restrict__ info, int nchunks) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= nchunks) return;
    const PpgInflateResult r = ires[k];
    const uint32_t onl = oref[k].nl & PPG_OFF_COUNT;
    const bool ok = r.status == 0;
    const bool serial = (oref[k].nl & PPG_OFF_SERIAL) || (r.pflags & PPG_PF_SERIAL);
    const uint32_t nl = onl + (ok ? r.newlines : 0);
    PpgParseInfo f;
    f.newlines = nl;
    f.serial = serial ? 1 : 0;
    f.emit = ok && !serial && (r.pflags & PPG_PF_OVERFLOW) ? 1 : 0;
    f.records = ok && !serial ? nl / 4 : 0;
    info[k] = f;
}

// A chunk the census declined (R-P3 fails: an empty line) whose newline positions are all known --
// the census kept them (no overflow), no NUL byte anywhere, a short offset -- is parsed by
// ppg_parse_chain from those positions; any other declined chunk byte by byte (ppg_parse_serial).
constexpr uint32_t kChainOffsetNl = 1024;   // offset newlines ppg_parse_chain stages in LDS

__device__ __forceinline__ bool chain_eligible(const PpgInflateResult &r, const PpgOffsetRef &o, int chain) {
    return chain && !(r.pflags & (PPG_PF_NUL | PPG_PF_OVERFLOW)) && !(o.nl & PPG_OFF_NUL) &&
           (o.nl & PPG_OFF_COUNT) <= kChainOffsetNl;
}

// Parsing.Parse (Parsing.cs:11-69) exactly, one lane per chunk that the census declined.
// mode 0: count into info[k].records; mode 1: also write descriptors at base[k].
extern "C" __global__ __launch_bounds__(64) void ppg_parse_serial(
    const uint8_t *__restrict__ out, const PpgInflateJob *__restrict__ jobs, const PpgInflateResult *__restrict__ ires,
    const uint8_t *__restrict__ offs, const PpgOffsetRef *__restrict__ oref, PpgParseInfo *__restrict__ info,
    const uint64_t *__restrict__ base, uint32_t *__restrict__ recs, int nchunks, int mode, uint64_t cap, int chain) {
    const int k = blockIdx.x;
    if (k >= nchunks || threadIdx.x != 0) return;
    if (!info[k].serial || ires[k].status != 0) return;
    if (chain_eligible(ires[k], oref[k], chain)) return;   // ppg_parse_chain's
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
        if (dst && 4 * (base[k] + n) + 4 <= cap) {   // cap: the descriptor buffer's u32 entries
            dst[4 * n + 0] = (uint32_t)nn[0];
            dst[4 * n + 1] = (uint32_t)nn[1];
            dst[4 * n + 2] = (uint32_t)nn[2];
            dst[4 * n + 3] = (uint32_t)nn[3];
        }
        n++;
    }
    if (!mode) info[k].records = n;
}

// Parsing.Parse (Parsing.cs:11-69) for a declined chunk from its newline positions, one wave per
// chunk (replaces the byte-by-byte lane of ppg_parse_serial, which cost a quarter of the inflate
// time on a file where every chunk has blank lines).  With terminators N[0..M) = the '\n'
// positions of raw (no NUL: the only 0 is raw[total]), the state machine becomes a walk over
// terminator indices, O(1) per record: a record starting after the previous record's n4 = N[p]
//   n1 = the first '\n' at or after N[p] + 2   (raw[N[p]+1] was skipped as the '@', Parsing.cs:19)
//      = N[p+1], or N[p+2] if N[p+1] == N[p] + 1 (a blank line there)
//   n2 = the next '\n' = N[j1+1]
//   n3 = the first '\n' at or after n2 + 2     (raw[n2+1] skipped as the '+', Parsing.cs:30)
//   n4 = the next '\n'
// and any terminator index >= M is the 0 at raw[total] (ParseLine's stop: no record).  The walk
// is wave-uniform; the terminators come 64 at a time into a VGPR window read with v_readlane, and
// descriptors leave 16 records (64 dwords) per vector store.
extern "C" __global__ __launch_bounds__(64) void ppg_parse_chain(
    const PpgInflateJob *__restrict__ jobs, const PpgInflateResult *__restrict__ ires, const uint8_t *__restrict__ offs,
    const PpgOffsetRef *__restrict__ oref, PpgParseInfo *__restrict__ info, const uint64_t *__restrict__ base,
    const uint32_t *__restrict__ nls, uint32_t *__restrict__ recs, int nchunks, int mode, uint64_t cap) {
    __shared__ uint32_t onl_pos[kChainOffsetNl];
    const int k = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    if (k >= nchunks) return;
    const PpgInflateResult r = ires[k];
    const PpgOffsetRef o = oref[k];
    if (!info[k].serial || r.status != 0 || !chain_eligible(r, o, 1)) return;
    // the offset's newlines (raw indices [0, olen)), in order
    const uint8_t *off = offs + o.start;
    const uint32_t olen = o.len;
    uint32_t onl = 0;
    for (uint32_t g = 0; g < olen; g += 64) {
        const bool nl = g + lane < olen && off[g + lane] == '\n';
        const uint64_t b = __ballot(nl);
        if (nl) onl_pos[onl + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = g + lane;
        onl += (uint32_t)__popcll(b);
    }
    __syncthreads();
    const int64_t M = (int64_t)onl + r.newlines;
    const uint64_t total = (uint64_t)olen + r.produced;
    const uint32_t *bnl = nls + jobs[k].nl_off;
    auto load = [&](int64_t wb) -> uint32_t {
        const int64_t j = wb + (int64_t)lane;
        return j < (int64_t)onl ? onl_pos[j] : (j < M ? bnl[j - onl] : 0u);
    };
    int64_t wb = 0;
    uint32_t win = load(0);
    auto N = [&](int64_t j) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)win, (int)(j - wb)); };
    uint64_t count = 0;
    const uint64_t b0 = mode ? base[k] : 0;
    uint32_t acc = 0;                                  // lane 4q+f: field f of the q-th pending record
    int64_t p = -1;
    uint64_t np1 = 0;                                  // N[p] + 1: where the next record's state starts
    for (;;) {
        if (np1 >= total) break;                       // raw[i] == 0 (Parsing.cs:16)
        if (p + 7 > wb + 64) {                         // indices up to p + 6 must be in the window
            wb = p + 1;
            win = load(wb);
        }
        int64_t j = p + 1;
        if (j >= M) break;
        uint32_t n1 = N(j);
        if (n1 == np1) {                               // raw[N[p]+1] == '\n': skipped, then a blank line
            if (++j >= M) break;
            n1 = N(j);
        }
        if (++j >= M) break;
        const uint32_t n2 = N(j);
        if (++j >= M) break;
        uint32_t n3 = N(j);
        if (n3 == n2 + 1) {                            // the skipped '+' byte was a '\n'
            if (++j >= M) break;
            n3 = N(j);
        }
        if (++j >= M) break;
        const uint32_t n4 = N(j);
        if (mode) {
            const uint32_t q = (uint32_t)(count & 15) * 4;
            acc = lane == q ? n1 : lane == q + 1 ? n2 : lane == q + 2 ? n3 : lane == q + 3 ? n4 : acc;
            if ((count & 15) == 15) {                  // 16 records: one 256-B store
                const uint64_t at = 4 * (b0 + count - 15) + lane;
                if (4 * (b0 + count + 1) <= cap) recs[at] = acc;
            }
        }
        count++;
        p = j;
        np1 = (uint64_t)n4 + 1;
    }
    if (mode) {
        const uint32_t q = (uint32_t)(count & 15);
        if (q && lane < 4 * q && 4 * (b0 + count) <= cap) recs[4 * (b0 + count - q) + lane] = acc;
    } else if (lane == 0) {
        info[k].records = count;
    }
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

// Descriptors of fast-path chunks whose census overflowed nl_cap: a scan of the body for its
// newlines.  Newline m (m < 4*records) is field m%4 of record m/4.
extern "C" __global__ __launch_bounds__(256) void ppg_parse_emit(
    const uint8_t *__restrict__ out, const PpgInflateJob *__restrict__ jobs, const PpgInflateResult *__restrict__ ires,
    const uint8_t *__restrict__ offs, const PpgOffsetRef *__restrict__ oref, const PpgParseInfo *__restrict__ info,
    const uint64_t *__restrict__ base, uint32_t *__restrict__ recs, int nchunks, uint64_t cap) {
    const int k = blockIdx.x;
    if (k >= nchunks) return;
    if (!info[k].emit || info[k].serial || ires[k].status != 0) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    __shared__ uint32_t wsum[4];
    const uint64_t nrec = info[k].records;
    if (nrec == 0) return;
    if (4 * (base[k] + nrec) > cap) return;   // the host grows the buffer and runs this again
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

// Descriptors of fast-path chunks from the census: the offset's newlines (a few hundred bytes,
// scanned here) then the body's, already stored as raw indices by the inflate kernel; newline m
// (m < 4*records) is field m%4 of record m/4.  One block per chunk; a copy, not a scan.
extern "C" __global__ __launch_bounds__(256) void ppg_parse_place(
    const PpgInflateJob *__restrict__ jobs, const PpgInflateResult *__restrict__ ires, const uint8_t *__restrict__ offs,
    const PpgOffsetRef *__restrict__ oref, const PpgParseInfo *__restrict__ info, const uint64_t *__restrict__ base,
    const uint32_t *__restrict__ nls, uint32_t *__restrict__ recs, int nchunks, uint64_t cap) {
    const int k = blockIdx.x;
    if (k >= nchunks) return;
    const PpgParseInfo f = info[k];
    if (f.serial || f.emit || ires[k].status != 0 || f.records == 0) return;
    if (4 * (base[k] + f.records) > cap) return;   // the host grows the buffer and runs this again
    const uint64_t limit = 4 * f.records;
    uint32_t *dst = recs + 4 * base[k];
    const uint32_t onl = oref[k].nl & PPG_OFF_COUNT;
    if (onl) {
        // the offset's newlines by the whole block, 256 bytes a step (ballot + wave counts): one
        // thread's byte loop over the offset (~400 B) held every block open while the other 255
        // copied (r05: 5.7 ms of the 50 GB step)
        __shared__ uint32_t wcnt[4];
        const uint8_t *off = offs + oref[k].start;
        const uint32_t n = oref[k].len, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
        uint64_t m = 0;   // the offset's newlines before this step
        for (uint32_t g = 0; g < n; g += 256) {
            const uint32_t i = g + threadIdx.x;
            const bool nl = i < n && off[i] == '\n';
            const uint64_t b = __ballot(nl);
            if (lane == 0) wcnt[wv] = (uint32_t)__popcll(b);
            __syncthreads();
            uint64_t idx = m + (uint64_t)__popcll(b & ((1ull << lane) - 1ull));
            for (uint32_t q = 0; q < wv; q++) idx += wcnt[q];
            if (nl && idx < limit) dst[idx] = i;
            m += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
            __syncthreads();
        }
    }
    if (limit <= onl) return;
    const uint64_t cnt = min(limit - onl, (uint64_t)ires[k].newlines);
    const uint32_t *src = nls + jobs[k].nl_off;
    for (uint64_t i = threadIdx.x; i < cnt; i += 256) dst[onl + i] = src[i];
}

// Spot number of every record: Identifier = raw[start+1, n1) ("SRR<id>.<major>.<minor> ..."):
// the digits between its first and second '.'; -1 when the identifier has no such field.  The
// first record of a chunk that lies wholly inside offset_k is the previous chunk's last record
// parsed again (the Point fell on a record start) and gets -2, so a pairing can drop
// it and keep global record numbers aligned.  One block per chunk, a thread per record.
// The spot number of an identifier whose bytes start at p (L of them before the line's end or
// the 96-byte bound): the digits between the first two '.', 1..18 of them, else -1 -- the byte
// loop of ppg_record_keys, over 48 bytes gathered as 13 aligned dwords (one load each instead of
// one dependent byte load per character).  Returns 1 when the window ends before the answer does.
// p + 52 stays inside the output buffer (a 64-byte tail follows it).
__device__ __forceinline__ int spot_key_window(const uint8_t *p, uint64_t L_total, int64_t &key) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t x[13], u[12];
#pragma unroll
    for (int k = 0; k < 13; k++) x[k] = w[k];
#pragma unroll
    for (int k = 0; k < 12; k++) u[k] = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sh);
    const uint32_t L = (uint32_t)min(L_total, (uint64_t)48);
    int state = 0;   // 0: before the first '.', 1: digits, 2: done
    int64_t v = 0;
    int nd = 0;
    key = -1;
#pragma unroll
    for (int i = 0; i < 48; i++) {
        const uint32_t c = (u[i >> 2] >> (8 * (i & 3))) & 255u;
        const bool in = (uint32_t)i < L;
        if (state == 0) {
            if (!in) state = 2;                       // the line ended: -1
            else if (c == '.') state = 1;
        } else if (state == 1) {
            if (!in) state = 2;                       // the line ended inside the digits: -1
            else if (c >= '0' && c <= '9') {
                if (nd == 18) state = 2;              // a 19th digit: -1
                else { v = v * 10 + (int64_t)(c - '0'); nd++; }
            } else {
                if (c == '.' && nd > 0) key = v;
                state = 2;
            }
        }
    }
    return state == 2 || L_total <= 48 ? 0 : 1;
}

extern "C" __global__ __launch_bounds__(256) void ppg_record_keys(
    const uint8_t *__restrict__ out, const PpgInflateJob *__restrict__ jobs, const PpgInflateResult *__restrict__ ires,
    const uint8_t *__restrict__ offs, const PpgOffsetRef *__restrict__ oref, const PpgParseInfo *__restrict__ info,
    const uint64_t *__restrict__ base, const uint32_t *__restrict__ recs, int64_t *__restrict__ keys, int nchunks) {
    const int k = blockIdx.x;
    if (k >= nchunks || ires[k].status != 0) return;
    const uint64_t nrec = info[k].records;
    const uint8_t *off = offs + oref[k].start;
    const uint32_t olen = oref[k].len;
    const uint8_t *body = out + jobs[k].out_off;
    const uint64_t blen = ires[k].produced;
    const uint32_t *r = recs + 4 * base[k];
    int64_t *kk = keys + base[k];
    for (uint64_t j = threadIdx.x; j < nrec; j += 256) {
        const uint64_t start = j ? (uint64_t)r[4 * j - 1] + 1 : 0;
        const uint64_t n1 = r[4 * j];
        if (j == 0 && (uint64_t)r[3] < olen) { kk[j] = -2; continue; }
        int64_t key = -1;
        uint64_t i = start + 1;
        const uint64_t end = min(n1, start + 96);   // identifiers are short; bound the scan
        if (start >= olen) {   // the identifier lies in the body: its first 48 bytes in registers
            const int r2 = spot_key_window(body + (start + 1 - olen), end > start + 1 ? end - start - 1 : 0, key);
            if (r2 == 0) { kk[j] = key; continue; }
            key = -1;           // not settled inside the window: the byte loop below
        }
        while (i < end && raw_at(off, olen, body, blen, i) != '.') i++;
        if (i < end) {
            i++;
            int64_t v = 0;
            int nd = 0;
            uint8_t c = 0;
            while (i < end && (c = raw_at(off, olen, body, blen, i)) >= '0' && c <= '9' && nd < 18) {
                v = v * 10 + (c - '0');
                nd++;
                i++;
            }
            if (nd > 0 && i < end && c == '.') key = v;
        }
        kk[j] = key;
    }
}

// ------------------------------------------------------------------------------------------
// The record cursor's batch layout (ppg_cursor, BatchedFASTQ's enumerator): raw_k = offset_k ++
// chunk_k (Parsing.cs's CombinedMemory) of every chunk of a batch packed contiguously at
// dst + raw_off[k] on the device, so the batch crosses PCIe as one device -> host copy instead of
// one per chunk.  Grid (stripes, chunk slots); a block copies its stripe of chunks
// blockIdx.y, blockIdx.y + gridDim.y, ... (lanes in a row: every wave access is one contiguous run).
// ------------------------------------------------------------------------------------------
// dst may be pinned host memory (the cursor writes each batch straight into it: the kernel's
// stores cross PCIe, which leaves the copy engines to the host -> device direction -- SDMA copies
// of the two directions on two streams ran one after the other on the box, r03).  The body part
// goes as aligned 16-B stores assembled from 5 dwords (v_alignbyte); the offset carry and the
// unaligned ends bytewise.
__device__ __forceinline__ uint32_t raw_byte(const uint8_t *off, uint64_t olen, const uint8_t *body, uint64_t i) {
    return i < olen ? off[i] : body[i - olen];
}

extern "C" __global__ __launch_bounds__(256) void ppg_pack_raw(const uint8_t *__restrict__ out,
                                                               const PpgInflateJob *__restrict__ jobs,
                                                               const PpgInflateResult *__restrict__ ires,
                                                               const uint8_t *__restrict__ offs,
                                                               const PpgOffsetRef *__restrict__ oref,
                                                               const int64_t *__restrict__ raw_off,
                                                               uint8_t *__restrict__ dst, int n) {
    for (int k = blockIdx.y; k < n; k += gridDim.y) {
        const uint64_t olen = oref[k].len, blen = ires[k].produced;
        const uint8_t *off = offs + oref[k].start, *body = out + jobs[k].out_off;
        const uint64_t d0 = (uint64_t)raw_off[k], total = olen + blen;   // raw byte i -> dst[d0 + i]
        // 16-B destination words [w0, w1) lying entirely inside the body part; the rest bytewise
        const uint64_t body_d = d0 + olen;
        const uint64_t w0 = (body_d + 15) / 16, w1 = (d0 + total) / 16;
        const uint64_t nw = w1 > w0 ? w1 - w0 : 0;
        const uint64_t per = (nw + gridDim.x - 1) / gridDim.x;
        const uint64_t a = w0 + min(nw, (uint64_t)blockIdx.x * per), z = w0 + min(nw, (uint64_t)(blockIdx.x + 1) * per);
        for (uint64_t w = a + threadIdx.x; w < z; w += 256) {
            const uint64_t sb = 16 * w - body_d;                     // body byte of the word's first byte
            const uint8_t *src = body + sb;
            const uint32_t *s32 = (const uint32_t *)((uintptr_t)src & ~(uintptr_t)3);
            const uint32_t sh = (uint32_t)((uintptr_t)src & 3);
            const uint32_t x0 = s32[0], x1 = s32[1], x2 = s32[2], x3 = s32[3], x4 = s32[4];   // out has a 64-B tail
            uint4 v;
            v.x = __builtin_amdgcn_alignbyte(x1, x0, sh);
            v.y = __builtin_amdgcn_alignbyte(x2, x1, sh);
            v.z = __builtin_amdgcn_alignbyte(x3, x2, sh);
            v.w = __builtin_amdgcn_alignbyte(x4, x3, sh);
            *(uint4 *)(dst + 16 * w) = v;
        }
        if (blockIdx.x == 0) {   // the head (offset carry + unaligned start) and the unaligned tail
            const uint64_t head = nw ? 16 * w0 - d0 : total;
            for (uint64_t i = threadIdx.x; i < head; i += 256) dst[d0 + i] = (uint8_t)raw_byte(off, olen, body, i);
            if (nw)
                for (uint64_t i = 16 * w1 - d0 + threadIdx.x; i < total; i += 256)
                    dst[d0 + i] = (uint8_t)raw_byte(off, olen, body, i);
        }
    }
}

// n 16-B words src -> dst (dst may be pinned host memory: the cursor's descriptors)
extern "C" __global__ __launch_bounds__(256) void ppg_copy16(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                             uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
}

// ------------------------------------------------------------------------------------------
// Split chunks (ppg_shard_set_split): chunk k was decoded as sub-jobs [sidx[k], sidx[k+1]) that
// start at deflate block boundaries inside it, each with its own 32 KiB history.  Their results
// are folded into the chunk's (in order: the first failing sub-job's status; every sub-job but
// the last must produce exactly its bytes and end exactly where the next one starts), and their
// stored newline positions -- already chunk-relative raw indices, in regions of the same buffer
// past every chunk's own -- are concatenated into the chunk's region, so the parse kernels see the
// chunk as one job.  A chunk decoded whole censused straight into its region.  One block per chunk.
// ------------------------------------------------------------------------------------------
// inv (may be null): sub-job j's result is sres[inv[j]] -- the launch ran the sub-jobs in another
// order (longest first, ppg_shard_set_split)
extern "C" __global__ __launch_bounds__(256) void ppg_split_merge(const PpgInflateJob *__restrict__ sjobs,
                                                                  const PpgInflateResult *__restrict__ sres,
                                                                  const uint32_t *__restrict__ inv,
                                                                  const uint32_t *__restrict__ sidx,
                                                                  const uint32_t *__restrict__ snls,
                                                                  const PpgInflateJob *__restrict__ jobs,
                                                                  PpgInflateResult *__restrict__ res,
                                                                  uint32_t *__restrict__ nls, int n) {
    const int k = blockIdx.x;
    if (k >= n) return;
    const uint32_t s0 = sidx[k], s1 = sidx[k + 1];
    if (s1 == s0 + 1) {   // decoded whole: its census is already in the chunk's region
        if (threadIdx.x == 0) res[k] = sres[inv ? inv[s0] : s0];
        return;
    }
    const PpgInflateJob &C = jobs[k];
    PpgInflateResult m = {};
    uint32_t nl = 0;
    for (uint32_t j = s0; j < s1; j++) {
        const PpgInflateResult r = sres[inv ? inv[j] : j];
        const bool tail = j + 1 == s1;
        if (m.status == 0 && r.status != 0) m.status = r.status;
        if (m.status == 0 && !tail && (r.produced != sjobs[j].out_len || r.end_bit != sjobs[j + 1].bit_start))
            m.status = -3;   // Z_DATA_ERROR: the side point is not where this sub-job's blocks end
        m.produced += r.produced;
        m.flags |= tail ? r.flags : (r.flags & ~PPG_FLAG_NO_EOB);
        m.pflags |= r.pflags;
        m.nblocks += r.nblocks;
        if (tail) { m.end_bit = r.end_bit; m.last = r.last; }
        // positions of this sub-job, stored while its own capacity lasted
        const uint32_t cnt = r.newlines;
        if (!(m.pflags & PPG_PF_OVERFLOW) && nl + cnt <= C.nl_cap) {
            const uint32_t *src = snls + sjobs[j].nl_off;
            uint32_t *dst = nls + C.nl_off + nl;
            for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) dst[i] = src[i];
        } else {
            m.pflags |= PPG_PF_OVERFLOW;
        }
        nl += cnt;
    }
    m.newlines = nl;
    if (threadIdx.x == 0) res[k] = m;
}

// ------------------------------------------------------------------------------------------
// Host-side launchers (called from ppg_api.cpp).
// ------------------------------------------------------------------------------------------
// after the inflate launch: per-chunk counts (census, or the serial machine) and their scan
// PPG_PARSE_CHAIN=0 parses every declined chunk byte by byte (A/B and tests of both paths)
static int chain_enabled() {
    const char *e = getenv("PPG_PARSE_CHAIN");
    return e && e[0] == '0' ? 0 : 1;
}

hipError_t ppg_launch_parse_count(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                  const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                  PpgParseInfo *info, uint64_t *base, uint64_t *total, int n, const uint32_t *nls) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_parse_finish, dim3((n + 255) / 256), dim3(256), 0, s, ires, oref, info, n);
    const int chain = chain_enabled();
    hipLaunchKernelGGL(ppg_parse_serial, dim3(n), dim3(64), 0, s, out, jobs, ires, offs, oref, info,
                       (const uint64_t *)nullptr, (uint32_t *)nullptr, n, 0, (uint64_t)0, chain);
    if (chain)
        hipLaunchKernelGGL(ppg_parse_chain, dim3(n), dim3(64), 0, s, jobs, ires, offs, oref, info,
                           (const uint64_t *)nullptr, nls, (uint32_t *)nullptr, n, 0, (uint64_t)0);
    hipLaunchKernelGGL(ppg_scan_counts, dim3(1), dim3(1024), 0, s, info, base, total, n);
    return hipGetLastError();
}

// A batch's record total into pinned host memory by a one-lane kernel store, not hipMemcpyAsync: a
// device -> host copy queued behind the batch's kernels sits on a DMA engine until they finish, and
// when the runtime puts it on the engine that carries the host ingest's H2D copy stream, every piece
// copy queued after it waits for the whole decode (r06: ~130 ms stalls of one 8 GiB piece's
// read + copy in the 50 GB ingest, the bubble of VERDICT r05 weak #5).
__global__ __launch_bounds__(64) void ppg_total_to_host(const uint64_t *__restrict__ total, uint64_t *host) {
    if (threadIdx.x == 0) *(volatile uint64_t *)host = *total;
}
hipError_t ppg_launch_total_to_host(hipStream_t s, const uint64_t *total, uint64_t *host) {
    hipLaunchKernelGGL(ppg_total_to_host, dim3(1), dim3(64), 0, s, total, host);
    return hipGetLastError();
}

// descriptors: census copy (most chunks), body scan (census overflow), serial machine (R-P3 fails)
hipError_t ppg_launch_parse_emit(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                 const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                 PpgParseInfo *info, const uint64_t *base, const uint32_t *nls, uint32_t *recs,
                                 uint64_t cap, int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_parse_place, dim3(n), dim3(256), 0, s, jobs, ires, offs, oref, info, base, nls, recs, n, cap);
    hipLaunchKernelGGL(ppg_parse_emit, dim3(n), dim3(256), 0, s, out, jobs, ires, offs, oref, info, base, recs, n, cap);
    const int chain = chain_enabled();
    hipLaunchKernelGGL(ppg_parse_serial, dim3(n), dim3(64), 0, s, out, jobs, ires, offs, oref, info, base, recs, n, 1, cap,
                       chain);
    if (chain)
        hipLaunchKernelGGL(ppg_parse_chain, dim3(n), dim3(64), 0, s, jobs, ires, offs, oref, info, base, nls, recs, n, 1,
                           cap);
    return hipGetLastError();
}

hipError_t ppg_launch_record_keys(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                  const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                  const PpgParseInfo *info, const uint64_t *base, const uint32_t *recs, int64_t *keys,
                                  int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_record_keys, dim3(n), dim3(256), 0, s, out, jobs, ires, offs, oref, info, base, recs, keys, n);
    return hipGetLastError();
}

hipError_t ppg_launch_pack_raw(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs, const PpgInflateResult *ires,
                               const uint8_t *offs, const PpgOffsetRef *oref, const int64_t *raw_off, uint8_t *dst,
                               int n, int blocks) {
    if (n <= 0) return hipSuccess;
    // blocks > 0: at most that many workgroups (4 stripes each looping over chunks), so that a pack
    // into pinned host memory -- PCIe-bound for ~170 ms per 8 GiB -- leaves the CUs to the next
    // batch's decode instead of queueing (16 x chunks) workgroups ahead of it
    const dim3 g = blocks > 0 ? dim3(4, (unsigned)std::max(1, std::min(n, blocks / 4))) : dim3(16, (unsigned)n);
    hipLaunchKernelGGL(ppg_pack_raw, g, dim3(256), 0, s, out, jobs, ires, offs, oref, raw_off, dst, n);
    return hipGetLastError();
}

hipError_t ppg_launch_copy16(hipStream_t s, const void *src, void *dst, uint64_t n16, int blocks) {
    if (!n16) return hipSuccess;
    const uint64_t cap = blocks > 0 ? (uint64_t)blocks : 4096;
    hipLaunchKernelGGL(ppg_copy16, dim3((unsigned)std::min<uint64_t>(cap, (n16 + 255) / 256)), dim3(256), 0, s,
                       (const uint4 *)src, (uint4 *)dst, n16);
    return hipGetLastError();
}

hipError_t ppg_launch_split_merge(hipStream_t s, const PpgInflateJob *sjobs, const PpgInflateResult *sres,
                                  const uint32_t *inv, const uint32_t *sidx, const uint32_t *snls,
                                  const PpgInflateJob *jobs, PpgInflateResult *res, uint32_t *nls, int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_split_merge, dim3(n), dim3(256), 0, s, sjobs, sres, inv, sidx, snls, jobs, res, nls, n);
    return hipGetLastError();
}
