// ppg_parse.hip — gfx950 kernels for the FASTQ record scan of the DecompressAll path
// (Decompressor/Parsing.cs:11-69 over raw_k = offset_k ++ chunk_k).
//
//   ppg_parse_count   per-chunk newline census + the conditions under which "record j = newlines
//                     4j..4j+3" equals the serial state machine (R-P3)
//   ppg_parse_serial  the exact Parsing.Parse state machine for chunks the census declines
//   ppg_scan_counts   exclusive scan of per-chunk record counts -> record bases
//   ppg_parse_emit    per-record descriptors (n1..n4 newline positions) for fast chunks
//   ppg_record_keys   per-record spot ("major") number from the identifier line, for pairing
//                     the two files of a read pair
#include <hip/hip_runtime.h>
#include <stdint.h>
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

// Spot number of every record: Identifier = raw[start+1, n1) ("SRR<id>.<major>.<minor> ..."):
// the digits between its first and second '.'; -1 when the identifier has no such field.  The
// first record of a chunk that lies wholly inside offset_k is the previous chunk's last record
// parsed again (the Point fell on a record start) and gets -2, so a pairing can drop
// it and keep global record numbers aligned.  One block per chunk, a thread per record.
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
// Host-side launchers (called from ppg_api.cpp).
// ------------------------------------------------------------------------------------------
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

hipError_t ppg_launch_record_keys(hipStream_t s, const uint8_t *out, const PpgInflateJob *jobs,
                                  const PpgInflateResult *ires, const uint8_t *offs, const PpgOffsetRef *oref,
                                  const PpgParseInfo *info, const uint64_t *base, const uint32_t *recs, int64_t *keys,
                                  int n) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(ppg_record_keys, dim3(n), dim3(256), 0, s, out, jobs, ires, offs, oref, info, base, recs, keys, n);
    return hipGetLastError();
}
