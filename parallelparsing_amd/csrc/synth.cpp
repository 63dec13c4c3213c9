// synth.cpp — synthetic inputs for tests and bench.py (host only; NOT the hot path).
//
// Record shape follows Generator/Generator.cs:9-61 with the read length fixed (150 in
// BASELINE.json):  "@SRR{id}.{major}.{minor} {major} length={L}\n" + L bases from ACGT +
// "+SRR{id2}.{major}.{minor} {major} length={L}\n" + L quality chars ('?' .90, '*' .05,
// '!' .05).  id ~ U[10^7, 2*10^7), major = no/2+1, minor = no%2+1 (Generator.cs:36-43).
// The RNG is counter-based (record number -> stream), so any record range can be generated
// independently and in parallel; it is not .NET's Random(0) (unreproducible without .NET).
//
// Compression produces ONE gzip member (the reference cannot read multi-member files, SURVEY
// Q3).  For large inputs it is pigz-style: pieces compressed in parallel, each primed with the
// previous piece's last 32 KiB and closed by Z_SYNC_FLUSH, CRCs joined with crc32_combine.
//
// The 50 GB bench file is a "tiled" member: a segment S of whole records is deflated with no
// history (its first piece has no dictionary) and ends byte-aligned, so the same compressed
// segment bytes can be repeated T times inside one member; the decompressed stream is S^T.
// ppg_synth_tiled_points() derives that file's CreateIndex points (Core.cs:14-131 semantics)
// from the segment's deflate block list without inflating the 50 GB.
#include <zlib.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>
#include <thread>
#include <vector>
#include <atomic>
#include <algorithm>

namespace {

inline uint64_t splitmix(uint64_t &s) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline int put_u(char *p, uint64_t v) {
    char tmp[24];
    int n = 0;
    do { tmp[n++] = char('0' + v % 10); v /= 10; } while (v);
    for (int i = 0; i < n; i++) p[i] = tmp[n - 1 - i];
    return n;
}

inline int digits(uint64_t v) { int n = 1; while (v >= 10) { v /= 10; n++; } return n; }

// mate 0: the reference Generator's single file (major = no/2+1, minor = no%2+1); mate 1/2: one
// file of a read pair: major = no+1, minor = mate, and the SRR ids are
// drawn from the record number alone, so R1 and R2 records share them.
inline uint64_t rec_major(int64_t no, int mate) { return mate ? (uint64_t)no + 1 : (uint64_t)no / 2 + 1; }

// bytes of record `no` (independent of the random draws: ids always have 8 digits)
inline int64_t rec_size(int64_t no, int L, int mate = 0) {
    uint64_t major = rec_major(no, mate);
    int64_t hdr = 1 + 3 + 8 + 1 + digits(major) + 1 + 1 + 1 + digits(major) + 8 + digits((uint64_t)L) + 1;
    return 2 * hdr + 2 * (int64_t)(L + 1);
}

int64_t write_rec(char *p, uint64_t seed, int64_t no, int L, int mate = 0) {
    uint64_t s = seed * 0xD1B54A32D192ED03ull ^ ((uint64_t)no * 0x9E3779B97F4A7C15ull) ^ 0x5851F42D4C957F2Dull;
    splitmix(s);
    uint64_t sid = ((uint64_t)no * 0x9E3779B97F4A7C15ull) ^ 0x2545F4914F6CDD1Dull;   // pair-shared ids
    char *p0 = p;
    uint64_t major = rec_major(no, mate), minor = mate ? (uint64_t)mate : (uint64_t)no % 2 + 1;
    for (int line = 0; line < 2; line++) {
        // header ('@') then, after the sequence, the '+' line with a fresh id (Generator.cs:11-14)
        if (line == 1) {
            for (int i = 0; i < L; i += 32) {
                uint64_t r = splitmix(s);
                int m = L - i < 32 ? L - i : 32;
                for (int b = 0; b < m; b++) { p[i + b] = "ATCG"[r & 3]; r >>= 2; }
            }
            p += L;
            *p++ = '\n';
        }
        *p++ = line == 0 ? '@' : '+';
        memcpy(p, "SRR", 3); p += 3;
        p += put_u(p, 10000000ull + splitmix(mate ? sid : s) % 10000000ull);
        *p++ = '.'; p += put_u(p, major); *p++ = '.'; p += put_u(p, minor);
        *p++ = ' '; p += put_u(p, major);
        memcpy(p, " length=", 8); p += 8;
        p += put_u(p, (uint64_t)L);
        *p++ = '\n';
    }
    for (int i = 0; i < L; i += 4) {
        uint64_t r = splitmix(s);
        int m = L - i < 4 ? L - i : 4;
        for (int b = 0; b < m; b++) {
            uint32_t u = (uint32_t)(r & 0xFFFF); r >>= 16;
            p[i + b] = u < 58982u ? '?' : (u < 62259u ? '*' : '!');   // .90 / .05 / .05
        }
    }
    p += L;
    *p++ = '\n';
    return p - p0;
}

// ---- "Illumina-like" records: what real SRA FASTQ looks like, unlike the
// Generator shape -- variable read lengths (70% 151 bp, else 35..151), N bases, and Phred+33
// qualities over '!'..'J' that include '@' (Q31): about 1.2% of quality bytes, so CreateIndex's
// '@' count (Core.cs:86-94) sees "records" inside quality lines and Points land mid-record
// (SURVEY Q2).  Header "@SRR6750041.{no+1} {no+1} length={L}", '+' line the same with '+'.
inline int ill_len(uint64_t seed, int64_t no) {
    uint64_t s = seed * 0xA0761D6478BD642Full ^ ((uint64_t)no * 0xE7037ED1A0B428DBull) ^ 0x8EBC6AF09C88C6E3ull;
    const uint64_t r = splitmix(s);
    return (r & 1023) < 717 ? 151 : 35 + (int)((r >> 10) % 117);
}

inline int64_t ill_hdr(int64_t no, int L) {   // "SRR6750041." + no+1 + " " + no+1 + " length=" + L + "\n"
    return 11 + 2 * digits((uint64_t)no + 1) + 1 + 8 + digits((uint64_t)L) + 1;
}

inline int64_t ill_size(uint64_t seed, int64_t no) {
    const int L = ill_len(seed, no);
    return 2 * (1 + ill_hdr(no, L)) + 2 * (int64_t)(L + 1);
}

int64_t write_ill(char *p, uint64_t seed, int64_t no) {
    const int L = ill_len(seed, no);
    uint64_t s = seed * 0x9FB21C651E98DF25ull ^ ((uint64_t)no * 0xC2B2AE3D27D4EB4Full) ^ 0x165667B19E3779F9ull;
    splitmix(s);
    char *p0 = p;
    char *seq = nullptr;
    for (int line = 0; line < 2; line++) {
        *p++ = line == 0 ? '@' : '+';
        memcpy(p, "SRR6750041.", 11); p += 11;
        p += put_u(p, (uint64_t)no + 1);
        *p++ = ' ';
        p += put_u(p, (uint64_t)no + 1);
        memcpy(p, " length=", 8); p += 8;
        p += put_u(p, (uint64_t)L);
        *p++ = '\n';
        if (line == 0) {
            seq = p;
            for (int i = 0; i < L; i++) {
                const uint64_t r = splitmix(s);
                p[i] = (r & 1023) < 4 ? 'N' : "ACGT"[(r >> 10) & 3];
            }
            p += L;
            *p++ = '\n';
        }
    }
    for (int i = 0; i < L; i++) {
        const uint64_t r = splitmix(s);
        const uint32_t u = (uint32_t)(r & 0xFFFF), v = (uint32_t)(r >> 16);
        char q;
        if (seq[i] == 'N') q = (v & 1) ? '!' : '#';
        else if (u < 1311) q = '#';                                   // 2%: Q2, Illumina's low-quality tail
        else if (u < 3277) q = (char)('!' + v % 11);                   // 3%: Q0..Q10
        else if (u < 19661) q = (char)(',' + v % 21);                  // 25%: Q11..Q31 (',' .. '@')
        else q = (char)('A' + v % 10);                                 // Q32..Q41 ('A' .. 'J')
        p[i] = q;
    }
    p += L;
    *p++ = '\n';
    return p - p0;
}

}  // namespace

extern "C" {

int64_t ppg_synth_illumina_size(uint64_t seed, int64_t no0, int64_t n) {
    int64_t t = 0;
    for (int64_t no = no0; no < no0 + n; no++) t += ill_size(seed, no);
    return t;
}

// Illumina-like records [no0, no0+n) into out (cap bytes).  Returns bytes written or -1.
int64_t ppg_synth_illumina(uint64_t seed, int64_t no0, int64_t n, uint8_t *out, int64_t cap, int threads) {
    if (threads < 1) threads = 1;
    const int64_t per = (n + threads - 1) / threads;
    std::vector<int64_t> off(threads + 1, 0);
    for (int t = 0; t < threads; t++) {
        const int64_t a = no0 + std::min(n, t * per), b = no0 + std::min(n, (t + 1) * per);
        off[t + 1] = off[t] + ppg_synth_illumina_size(seed, a, b - a);
    }
    if (off[threads] > cap) return -1;
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        th.emplace_back([=, &off] {
            const int64_t a = no0 + std::min(n, t * per), b = no0 + std::min(n, (t + 1) * per);
            char *p = (char *)out + off[t];
            for (int64_t no = a; no < b; no++) p += write_ill(p, seed, no);
        });
    }
    for (auto &x : th) x.join();
    return off[threads];
}

// exact byte size of records [no0, no0+n) of file `mate` (0: single file, 1/2: pair mates)
int64_t ppg_synth_fastq_size_mate(int64_t no0, int64_t n, int read_len, int mate) {
    int64_t t = 0;
    for (int64_t no = no0; no < no0 + n; no++) t += rec_size(no, read_len, mate);
    return t;
}

int64_t ppg_synth_fastq_size(int64_t no0, int64_t n, int read_len) { return ppg_synth_fastq_size_mate(no0, n, read_len, 0); }

// Writes records [no0, no0+n) of file `mate` into out (cap bytes).  Returns bytes written or -1.
int64_t ppg_synth_fastq_mate(uint64_t seed, int mate, int64_t no0, int64_t n, int read_len, uint8_t *out,
                             int64_t cap, int threads) {
    if (threads < 1) threads = 1;
    int64_t per = (n + threads - 1) / threads;
    std::vector<int64_t> off(threads + 1, 0);
    for (int t = 0; t < threads; t++) {
        int64_t a = no0 + std::min(n, t * per), b = no0 + std::min(n, (t + 1) * per);
        off[t + 1] = off[t] + ppg_synth_fastq_size_mate(a, b - a, read_len, mate);
    }
    if (off[threads] > cap) return -1;
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        th.emplace_back([=, &off] {
            int64_t a = no0 + std::min(n, t * per), b = no0 + std::min(n, (t + 1) * per);
            char *p = (char *)out + off[t];
            for (int64_t no = a; no < b; no++) p += write_rec(p, seed, no, read_len, mate);
        });
    }
    for (auto &x : th) x.join();
    return off[threads];
}

int64_t ppg_synth_fastq(uint64_t seed, int64_t no0, int64_t n, int read_len, uint8_t *out, int64_t cap,
                        int threads) {
    return ppg_synth_fastq_mate(seed, 0, no0, n, read_len, out, cap, threads);
}

// Raw-deflates text[lo,hi) primed with dict (dlen<=32768); `last` -> Z_FINISH, else Z_SYNC_FLUSH.
static int64_t deflate_piece(const uint8_t *text, int64_t lo, int64_t hi, const uint8_t *dict, int dlen,
                             int level, int last, std::vector<uint8_t> &out) {
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -1;
    if (dlen > 0) deflateSetDictionary(&zs, dict, (uInt)dlen);
    out.resize((size_t)deflateBound(&zs, (uLong)(hi - lo)) + 64);
    zs.next_out = out.data();
    zs.avail_out = (uInt)out.size();
    int64_t pos = lo;
    const int64_t STEP = 1 << 30;
    int ret;
    do {
        int64_t n = std::min(STEP, hi - pos);
        zs.next_in = (Bytef *)(text + pos);
        zs.avail_in = (uInt)n;
        pos += n;
        int flush = pos < hi ? Z_NO_FLUSH : (last ? Z_FINISH : Z_SYNC_FLUSH);
        ret = deflate(&zs, flush);
        if (ret == Z_STREAM_ERROR) { deflateEnd(&zs); return -1; }
    } while (pos < hi);
    int64_t got = (int64_t)zs.total_out;
    deflateEnd(&zs);
    out.resize((size_t)got);
    return got;
}

static void put_le32(uint8_t *p, uint32_t v) { for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i)); }

// Single-member gzip of text.  piece<=0 -> one serial deflate (byte-identical to zlib's
// own gzip wrapper output at that level); piece>0 -> pigz-style parallel pieces.
// Returns the .gz length, or -1 if cap is too small.
int64_t ppg_synth_gzip(const uint8_t *text, int64_t len, int level, int64_t piece, int threads, uint8_t *out,
                       int64_t cap) {
    if (piece <= 0) piece = len > 0 ? len : 1;
    int64_t np = (len + piece - 1) / piece;
    if (np == 0) np = 1;
    std::vector<std::vector<uint8_t>> parts((size_t)np);
    std::vector<uint32_t> crcs((size_t)np);
    std::atomic<int64_t> next{0};
    std::atomic<int> bad{0};
    if (threads < 1) threads = 1;
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        th.emplace_back([&] {
            for (;;) {
                int64_t i = next.fetch_add(1);
                if (i >= np) break;
                int64_t lo = i * piece, hi = std::min(len, lo + piece);
                int64_t dl = std::min<int64_t>(lo, 32768);
                if (deflate_piece(text, lo, hi, text + lo - dl, (int)dl, level, i == np - 1, parts[i]) < 0) bad = 1;
                crcs[i] = (uint32_t)crc32(0L, text + lo, (uInt)(hi - lo));
            }
        });
    }
    for (auto &x : th) x.join();
    if (bad) return -1;
    int64_t tot = 10 + 8;
    for (auto &p : parts) tot += (int64_t)p.size();
    if (tot > cap) return -1;
    static const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3};
    memcpy(out, hdr, 10);
    uint8_t *w = out + 10;
    uLong crc = 0;
    for (int64_t i = 0; i < np; i++) {
        memcpy(w, parts[i].data(), parts[i].size());
        w += parts[i].size();
        int64_t lo = i * piece, hi = std::min(len, lo + piece);
        crc = crc32_combine(crc, crcs[i], (z_off_t)(hi - lo));
    }
    put_le32(w, (uint32_t)crc);
    put_le32(w + 4, (uint32_t)len);
    return tot;
}

// ---- tiled member -------------------------------------------------------------------------
// Segment deflate: text deflated as pigz pieces, first piece without dictionary, every piece
// closed by Z_SYNC_FLUSH (so the segment ends byte-aligned and references nothing before it).
// seg_out receives the raw deflate bytes; returns their length.
int64_t ppg_synth_segment(const uint8_t *text, int64_t len, int level, int64_t piece, int threads,
                          uint8_t *seg_out, int64_t cap, uint32_t *crc_out) {
    if (piece <= 0) piece = len;
    int64_t np = (len + piece - 1) / piece;
    std::vector<std::vector<uint8_t>> parts((size_t)np);
    std::atomic<int64_t> next{0};
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < std::max(1, threads); t++) {
        th.emplace_back([&] {
            for (;;) {
                int64_t i = next.fetch_add(1);
                if (i >= np) break;
                int64_t lo = i * piece, hi = std::min(len, lo + piece);
                int64_t dl = std::min<int64_t>(lo, 32768);
                if (deflate_piece(text, lo, hi, text + lo - dl, (int)dl, level, 0, parts[i]) < 0) bad = 1;
            }
        });
    }
    for (auto &x : th) x.join();
    if (bad) return -1;
    int64_t tot = 0;
    for (auto &p : parts) tot += (int64_t)p.size();
    if (tot > cap) return -1;
    uint8_t *w = seg_out;
    for (auto &p : parts) { memcpy(w, p.data(), p.size()); w += p.size(); }
    *crc_out = (uint32_t)crc32(0L, text, (uInt)0);
    {
        uLong c = 0;
        int64_t pos = 0;
        while (pos < len) {
            int64_t n = std::min<int64_t>(len - pos, 1 << 30);
            c = crc32(c, text + pos, (uInt)n);
            pos += n;
        }
        *crc_out = (uint32_t)c;
    }
    return tot;
}

// gzip header (10 B) and the tail that closes a tiled member: an empty final fixed block
// (bits 1,01,0000000 -> 0x03 0x00) + CRC-32 + ISIZE of S^T.
void ppg_synth_tiled_frame(uint32_t seg_crc, int64_t seg_len, int64_t repeats, uint8_t *hdr10, uint8_t *tail10) {
    static const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3};
    memcpy(hdr10, hdr, 10);
    uLong crc = 0;
    for (int64_t r = 0; r < repeats; r++) crc = crc32_combine(crc, seg_crc, (z_off_t)seg_len);
    tail10[0] = 0x03;
    tail10[1] = 0x00;
    put_le32(tail10 + 2, (uint32_t)crc);
    put_le32(tail10 + 6, (uint32_t)((uint64_t)seg_len * (uint64_t)repeats));
}

// Deflate block ends of the segment (raw stream, no dictionary), found exactly as CreateIndex
// sees them: inflate(Z_BLOCK) returns with data_type bit 128 (Core.cs:64,98).  Writes, per block
// end, its bit position within the segment and its output position.  Returns the count.
int64_t ppg_synth_segment_blocks(const uint8_t *seg, int64_t seg_len, int64_t text_len, int64_t *bit_end,
                                 int64_t *out_end, int64_t cap) {
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) return -1;
    std::vector<uint8_t> win(1 << 20);
    int64_t n = 0, totin = 0, totout = 0, pos = 0;
    int ret = Z_OK;
    zs.avail_out = 0;
    (void)text_len;
    for (;;) {
        if (zs.avail_in == 0) {  // every byte of the segment is consumed, so trailing empty blocks count
            int64_t k = std::min<int64_t>(seg_len - pos, 1 << 20);
            if (k <= 0) break;
            zs.next_in = (Bytef *)(seg + pos);
            zs.avail_in = (uInt)k;
            pos += k;
        }
        if (zs.avail_out == 0) { zs.next_out = win.data(); zs.avail_out = (uInt)win.size(); }
        totin += zs.avail_in; totout += zs.avail_out;
        ret = inflate(&zs, Z_BLOCK);
        totin -= zs.avail_in; totout -= zs.avail_out;
        if (ret != Z_OK && ret != Z_BUF_ERROR) { inflateEnd(&zs); return -1; }
        if ((zs.data_type & 128) && !(zs.data_type & 64)) {
            if (n < cap) { bit_end[n] = 8 * totin - (zs.data_type & 7); out_end[n] = totout; }
            n++;
        }
    }
    inflateEnd(&zs);
    return n;
}

// CreateIndex points of the tiled file  hdr(10) + seg^T + tail  (Core.cs:14-131), from the
// segment block list: per point output / input / bits, the offset length and the absolute
// position of the '@' that starts the offset (-1: no offset).  Windows and offset bytes are
// filled separately for any point range (ppg_synth_tiled_fill), so each rank materialises only
// its own.  Returns the point count, -1 if cap is short, -2 on Q4 overflow.
int64_t ppg_synth_tiled_points(const uint8_t *text, int64_t text_len, int64_t seg_gz_len, int64_t repeats,
                               const int64_t *bit_end, const int64_t *out_end, int64_t nblocks, uint32_t chunksize,
                               int64_t *p_output, int64_t *p_input, int32_t *p_bits, int32_t *p_off_len,
                               int64_t *p_at, int64_t cap) {
    // '@' census of one segment at every block end (count and position of the last '@')
    std::vector<int64_t> at_blk((size_t)nblocks), last_at_blk((size_t)nblocks);
    int64_t cnt = 0, last = -1, x = 0;
    for (int64_t b = 0; b < nblocks; b++) {
        for (; x < out_end[b]; x++) if (text[x] == '@') { cnt++; last = x; }
        at_blk[(size_t)b] = cnt;
        last_at_blk[(size_t)b] = last;
    }
    for (; x < text_len; x++) if (text[x] == '@') { cnt++; last = x; }
    const int64_t seg_at = cnt, seg_last_at = last;
    int64_t np = 0;
    auto emit = [&](int64_t output, int64_t input, int bits, int64_t at_abs) -> int {
        if (np >= cap) return -1;
        int32_t ol = 0;
        if (at_abs >= 0) {
            if (output - at_abs > 32768) return -2;   // C# offset buffer overflow
            ol = (int32_t)(output - at_abs);
        }
        p_output[np] = output; p_input[np] = input; p_bits[np] = bits; p_off_len[np] = ol;
        p_at[np] = ol ? at_abs : -1;
        np++;
        return 0;
    };
    if (emit(0, 10, 0, -1) < 0) return -1;   // right after the gzip header (Core.cs:101-102)
    int64_t counter_base = 0;                 // '@' count at the last point
    const int64_t seg_bits = seg_gz_len * 8;
    const int64_t thresh = (int64_t)(uint32_t)(chunksize - 8u);   // int > uint compared as long
    for (int64_t r = 0; r < repeats; r++) {
        for (int64_t b = 0; b < nblocks; b++) {
            const int64_t out_abs = r * text_len + out_end[b];
            const int64_t at_abs = r * seg_at + at_blk[(size_t)b];
            const int64_t bitpos = 80 + r * seg_bits + bit_end[b];
            const int64_t totin = (bitpos + 7) / 8;
            if (out_abs == 0) {
                int rc = emit(0, totin, (int)(totin * 8 - bitpos), -1);
                if (rc < 0) return rc;
                continue;
            }
            if (at_abs - counter_base > thresh) {
                int64_t last_abs;
                if (last_at_blk[(size_t)b] >= 0) last_abs = r * text_len + last_at_blk[(size_t)b];
                else if (r > 0 && seg_last_at >= 0) last_abs = (r - 1) * text_len + seg_last_at;
                else return -2;
                int rc = emit(out_abs, totin, (int)(totin * 8 - bitpos), last_abs);
                if (rc < 0) return rc;
                counter_base = at_abs;
            }
        }
    }
    // the final point at stream end (Core.cs:123): bits 0, input = file length
    if (emit(repeats * text_len, 10 + repeats * seg_gz_len + 10, 0, -1) < 0) return -1;
    return np;
}

// Windows (32 KiB each, Index.cs:42-46: the last 32 KiB of S^T before Output, zeros before the
// start) and offset bytes (concatenated) of points [lo, hi).
void ppg_synth_tiled_fill(const uint8_t *text, int64_t text_len, const int64_t *p_output, const int32_t *p_off_len,
                          const int64_t *p_at, int64_t lo, int64_t hi, uint8_t *windows, uint8_t *offsets) {
    int64_t o = 0;
    for (int64_t p = lo; p < hi; p++) {
        uint8_t *w = windows + (p - lo) * 32768;
        for (int64_t i = 0; i < 32768;) {
            int64_t q = p_output[p] - 32768 + i;
            if (q < 0) { w[i++] = 0; continue; }
            int64_t off = q % text_len, take = std::min<int64_t>(32768 - i, text_len - off);
            memcpy(w + i, text + off, (size_t)take);
            i += take;
        }
        for (int32_t i = 0; i < p_off_len[p]; i++) offsets[o + i] = text[(p_at[p] + i) % text_len];
        o += p_off_len[p];
    }
}

}  // extern "C"
