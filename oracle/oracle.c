/*
 * oracle/oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C restatement of the reference's chunked-gzip path, calling the same
 * third-party engine the reference P/Invokes: system zlib 1.2.11
 * (/usr/lib/x86_64-linux-gnu/libz.so.1.2.11; the reference pins "1.2.11" at
 * Common/Constants.cs:6 and binds it at Interop/PlatformInterop.cs:9-34).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product (libppgpu.so) never links or calls it.
 *
 * Parity status: the reference ships no tests, fixtures or known answers
 * (SURVEY.md §4, §8c), and its C# cannot run here (no .NET).  This
 * restatement is therefore "parity unpinned" against reference-owned vectors.
 * What pins it instead: (1) the gzip trailer (CRC-32 + ISIZE) of every input,
 * (2) Python's zlib module decompressing the same files independently, and
 * (3) a second, independent Python/ctypes restatement of CreateIndex
 * (oracle/oracle_py.py), both checked in tests/test_oracle.py.
 *
 *   orc_build_index      <- Decompressor/Core.cs:14-131   (BuildDeflateIndex)
 *   orc_add_point        <- Common/Index.cs:24-48          (Index.AddPoint)
 *   orc_extract          <- Decompressor/Core.cs:133-192  (ExtractDeflateIndex)
 *   orc_parse            <- Decompressor/Parsing.cs:11-69 (Parse / ParseLine)
 *   orc_serialize        <- Common/IndexIO.cs:7-27
 *   orc_deserialize      <- Common/IndexIO.cs:29-53
 *   orc_decompress_all   <- Decompressor/BatchedFASTQ.cs:54-98 + LazyFileReader.cs:41-97
 *                           (threaded; counts records per chunk — the CPU baseline)
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <zlib.h>

#define WINSIZE 32768   /* Common/Constants.cs:9  */
#define CHUNK   16384   /* Common/Constants.cs:12 */

/* extra return codes beyond zlib's (ZResult, Interop/Conventions.cs:9-20) */
#define ORC_INDEX_OUT_OF_RANGE (-50)  /* C# IndexOutOfRangeException (Q4, Core.cs:93) */
#define ORC_IO_ERROR (-51)
#define ORC_ARG_ERROR (-52)

typedef struct {
    int64_t output;           /* Common/Index.cs:64 */
    int64_t input;            /* Common/Index.cs:67 */
    int32_t bits;             /* Common/Index.cs:70 */
    uint8_t *window;          /* WINSIZE bytes, Common/Index.cs:73 */
    uint8_t *offset;          /* Common/Index.cs:75 */
    int32_t offset_len;
} orc_point;

typedef struct {
    int32_t count, cap;
    int32_t chunk_max_bytes;  /* Common/Index.cs:10 */
    orc_point *pts;
} orc_index;

static orc_index *idx_new(void) {
    orc_index *ix = (orc_index *)calloc(1, sizeof(orc_index));
    ix->cap = 8;
    ix->pts = (orc_point *)calloc((size_t)ix->cap, sizeof(orc_point));
    return ix;
}

void orc_index_free(orc_index *ix) {
    if (!ix) return;
    for (int i = 0; i < ix->count; i++) { free(ix->pts[i].window); free(ix->pts[i].offset); }
    free(ix->pts);
    free(ix);
}

static orc_point *idx_push(orc_index *ix) {
    if (ix->count == ix->cap) {
        ix->cap *= 2;
        ix->pts = (orc_point *)realloc(ix->pts, (size_t)ix->cap * sizeof(orc_point));
    }
    orc_point *p = &ix->pts[ix->count++];
    memset(p, 0, sizeof *p);
    return p;
}

/* Index.AddPoint (Common/Index.cs:24-48): ChunkMaxBytes with C# int casts, window rotated
 * so the oldest byte comes first. */
static void orc_add_point(orc_index *ix, int bits, int64_t input, int64_t output, uint32_t left,
                          const uint8_t *window, const uint8_t *offset, int32_t offset_len) {
    if (ix->count == 0) {
        ix->chunk_max_bytes = (int32_t)output;
    } else {
        int32_t outputSize = (int32_t)((uint32_t)(int32_t)output - (uint32_t)(int32_t)ix->pts[ix->count - 1].output);
        if (outputSize > ix->chunk_max_bytes) ix->chunk_max_bytes = outputSize;
    }
    orc_point *p = idx_push(ix);
    p->output = output;
    p->input = input;
    p->bits = bits;
    p->window = (uint8_t *)calloc(WINSIZE, 1);
    if (left != 0) memcpy(p->window, window + (WINSIZE - left), left);
    if (left < WINSIZE) memcpy(p->window + left, window, WINSIZE - left);
    p->offset_len = offset_len;
    p->offset = (uint8_t *)malloc(offset_len > 0 ? (size_t)offset_len : 1);
    if (offset_len > 0) memcpy(p->offset, offset, (size_t)offset_len);
}

/* Core.BuildDeflateIndex (Decompressor/Core.cs:14-131).  `file` is the whole .gz; reads are
 * emulated as FileStream.Read(input, 0, CHUNK) calls (Core.cs:41). */
int orc_build_index(const uint8_t *file, int64_t flen, uint32_t chunksize, orc_index **out) {
    z_stream strm;
    memset(&strm, 0, sizeof strm);
    orc_index *index = idx_new();
    uint8_t *input = (uint8_t *)malloc(CHUNK);
    uint8_t *window = (uint8_t *)calloc(WINSIZE, 1);
    uint8_t *offsetBeforePoint = (uint8_t *)calloc(WINSIZE, 1);
    int recordCounter = 0, prevAvailOut = 0, offsetArraySize = 0;
    int64_t fpos = 0, totin, totout;
    int ret = inflateInit2(&strm, 47);                           /* Core.cs:30 */
    int err = 0;
    int have_out = 0;                                            /* C#: strm.NextOut != null */
    if (ret != Z_OK) { err = ret; goto done; }
    totin = totout = 0;
    strm.avail_out = 0;
    do {
        int64_t n = flen - fpos < CHUNK ? flen - fpos : CHUNK;   /* Core.cs:41 */
        memcpy(input, file + fpos, (size_t)n);
        fpos += n;
        strm.avail_in = (uInt)n;
        if (strm.avail_in == 0) { err = Z_DATA_ERROR; goto done; }
        strm.next_in = input;
        do {
            if (strm.avail_out == 0) {                           /* Core.cs:52-56 */
                strm.avail_out = WINSIZE;
                strm.next_out = window;
                have_out = 1;
            }
            totin += strm.avail_in;
            totout += strm.avail_out;
            ret = inflate(&strm, Z_BLOCK);                       /* Core.cs:64 */
            totin -= strm.avail_in;
            totout -= strm.avail_out;
            if (ret == Z_NEED_DICT || ret == Z_MEM_ERROR || ret == Z_DATA_ERROR ||
                ret == Z_STREAM_ERROR || ret == Z_BUF_ERROR || ret == Z_VERSION_ERROR) {
                err = ret; goto done;                            /* Core.cs:68-74 */
            }
            if (have_out) {
                int cur = WINSIZE;                               /* Core.cs:79-96 */
                int iStart = prevAvailOut == 0 ? 0 : cur - prevAvailOut;
                int iEnd = cur - (int)strm.avail_out;
                for (int i = iStart; i < iEnd; i++) {
                    uint8_t c = window[i];
                    if (c == 64) { recordCounter++; offsetArraySize = 0; }
                    if (offsetArraySize >= WINSIZE) { err = ORC_INDEX_OUT_OF_RANGE; goto done; } /* Q4 */
                    offsetBeforePoint[offsetArraySize++] = c;
                }
                prevAvailOut = strm.avail_out > 0 ? (int)strm.avail_out : 0;
                if ((strm.data_type & 128) != 0 && (strm.data_type & 64) == 0) {  /* Core.cs:98 */
                    if (totout == 0) {
                        orc_add_point(index, strm.data_type & 7, totin, totout, strm.avail_out, window, NULL, 0);
                    } else if ((int64_t)recordCounter > (int64_t)(uint32_t)(chunksize - 8u)) { /* int vs uint -> long */
                        orc_add_point(index, strm.data_type & 7, totin, totout, strm.avail_out, window,
                                      offsetBeforePoint, offsetArraySize);
                        recordCounter = 0;
                    }
                }
            }
            if (ret == Z_STREAM_END) {                           /* Core.cs:114-125 */
                if (strm.avail_in != 0 || fpos != flen) {
                    ret = inflateReset(&strm);
                    if (ret != Z_OK) { err = ret; goto done; }
                    continue;
                }
                orc_add_point(index, strm.data_type & 7, totin, totout, strm.avail_out, window, NULL, 0);
                break;
            }
        } while (strm.avail_in != 0);
    } while (ret != Z_STREAM_END);
done:
    inflateEnd(&strm);
    free(input); free(window); free(offsetBeforePoint);
    if (err) { orc_index_free(index); *out = NULL; return err; }
    *out = index;
    return 0;
}

/* Core.ExtractDeflateIndex (Decompressor/Core.cs:133-192).
 * fileBuffer[0] is file byte from.Input-1 and its length is to.Input-from.Input+1
 * (LazyFileReader.cs:63-69).  Returns the produced byte count (>= 0) or a negative code. */
int64_t orc_extract(const uint8_t *fileBuffer, int64_t fbLen, const orc_point *from, const orc_point *to,
                    uint8_t *buf, int64_t bufLen) {
    z_stream strm;
    memset(&strm, 0, sizeof strm);
    int len = (int)(to->output - from->output);                 /* Core.cs:140 */
    int64_t posInFile;
    int ret;
    if (len < 0) return 0;
    if ((int64_t)len > bufLen) return ORC_ARG_ERROR;
    ret = inflateInit2(&strm, -15);                              /* Core.cs:148 */
    if (ret != Z_OK) return ret;
    posInFile = from->bits == 0 ? 1 : 0;                         /* Core.cs:151-157 */
    if (from->bits != 0) {
        int value = fileBuffer[0];
        inflatePrime(&strm, from->bits, value >> (8 - from->bits));
        posInFile++;
    }
    inflateSetDictionary(&strm, from->window, WINSIZE);          /* Core.cs:158 */
    strm.avail_in = 0;
    strm.avail_out = (uInt)len;
    strm.next_out = buf;
    do {
        if (strm.avail_in == 0) {                                /* Core.cs:166-176 */
            int64_t value = fbLen - posInFile < CHUNK ? fbLen - posInFile : CHUNK;
            if (value < 0) value = 0;
            strm.next_in = (Bytef *)(fileBuffer + posInFile);
            strm.avail_in = (uInt)value;
            posInFile += value;
            if (value == 0) { inflateEnd(&strm); return Z_DATA_ERROR; }
        }
        ret = inflate(&strm, Z_NO_FLUSH);                        /* Core.cs:177 */
        if (ret == Z_MEM_ERROR || ret == Z_DATA_ERROR || ret == Z_NEED_DICT) { inflateEnd(&strm); return ret; }
        if (ret == Z_STREAM_ERROR) break;                        /* "stream error" printed, Core.cs:180-184 */
        if (ret == Z_STREAM_END) break;
    } while (strm.avail_out != 0);
    inflateEnd(&strm);
    return (int64_t)len - (int64_t)strm.avail_out;              /* Core.cs:191 */
}

/* CombinedMemory indexer (Parsing.cs:80-87) over offset ++ chunk; the rented buffer's zeroed
 * slack (BatchedFASTQ.cs:65-66,73) is modelled as 0 for every index >= off_len+len (Q11). */
static inline int rawat(const uint8_t *off, int64_t off_len, const uint8_t *chunk, int64_t len, int64_t i) {
    if (i < off_len) return off[i];
    i -= off_len;
    return i < len ? chunk[i] : 0;
}

/* Parsing.ParseLine (Parsing.cs:53-69): returns line length incl. '\n', or -1 at '\0'. */
static inline int64_t parse_line(int64_t *pos, const uint8_t *off, int64_t ol, const uint8_t *ch, int64_t cl) {
    int64_t start = *pos;
    for (;;) {
        int b = rawat(off, ol, ch, cl, *pos);
        if (b == '\n' || b == 0) break;
        (*pos)++;
    }
    if (rawat(off, ol, ch, cl, *pos) == 0) return -1;
    (*pos)++;
    return *pos - start;
}

/* Parsing.Parse (Parsing.cs:11-51).  Emits, per record, the four line-terminating newline
 * positions n1..n4 relative to raw = offset ++ chunk (rec[4*j+0..3]); the record's fields are
 * id=[r+1,n1) seq=[n1+1,n2) other=[n2+2,n3) qual=[n3+1,n4) where r is its first byte.  When
 * `rec` is NULL only counts.  Returns the record count (rec_cap bounds what is written). */
int64_t orc_parse(const uint8_t *off, int64_t off_len, const uint8_t *chunk, int64_t len,
                  uint32_t *rec, int64_t rec_cap, int64_t *starts) {
    int64_t n = 0, i = 0;
    int64_t total = off_len + len;
    /* raw.Length is offset + rented length; every index past off_len+len reads 0, so the loop
     * always stops at the first slack byte: bounding it by total+1 is equivalent. */
    while (i <= total) {
        if (rawat(off, off_len, chunk, len, i) == 0) break;      /* Parsing.cs:16 */
        i++;                                                      /* skip '@' (Parsing.cs:19) */
        int64_t start = i;
        if (parse_line(&i, off, off_len, chunk, len) - 1 < 0) break;   /* identifier */
        int64_t n1 = i - 1;
        if (parse_line(&i, off, off_len, chunk, len) - 1 < 0) break;   /* sequence */
        int64_t n2 = i - 1;
        i++;                                                      /* skip '+' (Parsing.cs:30) */
        if (parse_line(&i, off, off_len, chunk, len) - 1 < 0) break;   /* other */
        int64_t n3 = i - 1;
        if (parse_line(&i, off, off_len, chunk, len) - 1 < 0) break;   /* quality */
        int64_t n4 = i - 1;
        if (rec && n < rec_cap) {
            rec[4 * n + 0] = (uint32_t)n1; rec[4 * n + 1] = (uint32_t)n2;
            rec[4 * n + 2] = (uint32_t)n3; rec[4 * n + 3] = (uint32_t)n4;
            if (starts) starts[n] = start - 1;
        }
        n++;
    }
    return n;
}

/* ---- IndexIO (Common/IndexIO.cs), little-endian BinaryWriter layout ---- */
int orc_serialize(const orc_index *ix, const char *path) {
    FILE *f = fopen(path, "wb");
    if (!f) return ORC_IO_ERROR;
    int32_t zero = 0, winlen = WINSIZE;
    fwrite(&zero, 4, 1, f);
    fwrite(&ix->chunk_max_bytes, 4, 1, f);
    fwrite(&ix->count, 4, 1, f);
    for (int i = 0; i < ix->count; i++) {
        const orc_point *p = &ix->pts[i];
        fwrite(&p->output, 8, 1, f);
        fwrite(&p->input, 8, 1, f);
        fwrite(&p->bits, 4, 1, f);
        fwrite(&winlen, 4, 1, f);
        fwrite(p->window, 1, WINSIZE, f);
        fwrite(&p->offset_len, 4, 1, f);
        if (p->offset_len) fwrite(p->offset, 1, (size_t)p->offset_len, f);
    }
    return fclose(f) == 0 ? 0 : ORC_IO_ERROR;
}

int orc_deserialize(const char *path, orc_index **out) {
    FILE *f = fopen(path, "rb");
    if (!f) return ORC_IO_ERROR;
    orc_index *ix = idx_new();
    int32_t hdr[3];
    if (fread(hdr, 4, 3, f) != 3) goto bad;
    ix->chunk_max_bytes = hdr[1];
    for (int i = 0; i < hdr[2]; i++) {
        orc_point *p = idx_push(ix);
        int32_t winlen;
        if (fread(&p->output, 8, 1, f) != 1 || fread(&p->input, 8, 1, f) != 1 ||
            fread(&p->bits, 4, 1, f) != 1 || fread(&winlen, 4, 1, f) != 1) goto bad;
        if (winlen < 0) goto bad;
        p->window = (uint8_t *)calloc(WINSIZE > winlen ? WINSIZE : (size_t)winlen, 1);
        if (fread(p->window, 1, (size_t)winlen, f) != (size_t)winlen) goto bad;
        if (fread(&p->offset_len, 4, 1, f) != 1 || p->offset_len < 0) goto bad;
        p->offset = (uint8_t *)malloc(p->offset_len ? (size_t)p->offset_len : 1);
        if (p->offset_len && fread(p->offset, 1, (size_t)p->offset_len, f) != (size_t)p->offset_len) goto bad;
    }
    fclose(f);
    *out = ix;
    return 0;
bad:
    fclose(f);
    orc_index_free(ix);
    return ORC_IO_ERROR;
}

/* Index from point arrays (windows count*32768 bytes, offsets concatenated) — lets the CPU
 * baseline run on an index produced elsewhere (the bench's tiled file). */
int orc_index_from_points(int count, const int64_t *output, const int64_t *input, const int32_t *bits,
                          const uint8_t *windows, const int32_t *offset_len, const uint8_t *offsets, orc_index **out) {
    orc_index *ix = idx_new();
    int64_t o = 0;
    for (int i = 0; i < count; i++) {
        orc_point *p = idx_push(ix);
        p->output = output[i]; p->input = input[i]; p->bits = bits[i];
        p->window = (uint8_t *)malloc(WINSIZE);
        memcpy(p->window, windows + (size_t)i * WINSIZE, WINSIZE);
        p->offset_len = offset_len[i];
        p->offset = (uint8_t *)malloc(offset_len[i] > 0 ? (size_t)offset_len[i] : 1);
        if (offset_len[i] > 0) memcpy(p->offset, offsets + o, (size_t)offset_len[i]);
        o += offset_len[i];
    }
    *out = ix;
    return 0;
}

/* ---- accessors for ctypes ---- */
int orc_index_count(const orc_index *ix) { return ix->count; }
int32_t orc_index_chunk_max_bytes(const orc_index *ix) { return ix->chunk_max_bytes; }
const orc_point *orc_index_point(const orc_index *ix, int i) { return &ix->pts[i]; }
void orc_point_get(const orc_point *p, int64_t *output, int64_t *input, int32_t *bits, int32_t *offset_len) {
    *output = p->output; *input = p->input; *bits = p->bits; *offset_len = p->offset_len;
}
const uint8_t *orc_point_window(const orc_point *p) { return p->window; }
const uint8_t *orc_point_offset(const orc_point *p) { return p->offset; }

/* Extract + Parse of chunk k of a whole in-memory .gz (the body of BatchedFASTQ's populateCache,
 * BatchedFASTQ.cs:63-74).  out must hold to.Output-from.Output bytes. */
int64_t orc_chunk(const orc_index *ix, int k, const uint8_t *gz, int64_t gzlen, uint8_t *out, int64_t out_cap,
                  int64_t *produced) {
    const orc_point *from = &ix->pts[k], *to = &ix->pts[k + 1];
    int64_t lo = from->input - 1, n = to->input - from->input + 1;
    if (lo < 0 || lo + n > gzlen) return ORC_ARG_ERROR;
    int64_t got = orc_extract(gz + lo, n, from, to, out, out_cap);
    *produced = got;
    if (got < 0) return got;
    return orc_parse(from->offset, from->offset_len, out, got, NULL, 0, NULL);
}

/* ---- threaded DecompressAll (the CPU baseline): BatchedFASTQ.Count() restated as T worker
 * threads pulling chunks, each doing slice-read + ExtractDeflateIndex + Parse.  mode 0 counts
 * records; mode 1 also materialises every record into its own heap buffer as FastqRecord does
 * (Parsing.cs:41-47) and frees it as the consumer would (BatchedFASTQ.cs:56). ---- */
typedef struct {
    const orc_index *ix; const uint8_t *gz; int64_t gzlen; int first, last; int mode;
    volatile int next; int64_t *counts; int err;
    pthread_mutex_t mu;
} all_job;

static void *all_worker(void *arg) {
    all_job *j = (all_job *)arg;
    uint8_t *buf = NULL; int64_t cap = 0;
    uint32_t *rec = NULL; int64_t rcap = 0;
    int64_t *starts = NULL;
    for (;;) {
        int k = __sync_fetch_and_add(&j->next, 1);
        if (k >= j->last) break;
        const orc_point *from = &j->ix->pts[k], *to = &j->ix->pts[k + 1];
        int64_t need = to->output - from->output;
        if (need > cap) { free(buf); cap = need; buf = (uint8_t *)malloc((size_t)cap + 1); }
        int64_t got = 0;
        int64_t lo = from->input - 1, n = to->input - from->input + 1;
        got = orc_extract(j->gz + lo, n, from, to, buf, cap);
        if (got < 0) { j->err = (int)got; j->counts[k] = got; continue; }
        if (j->mode == 0) {
            j->counts[k] = orc_parse(from->offset, from->offset_len, buf, got, NULL, 0, NULL);
        } else {
            int64_t nrec = orc_parse(from->offset, from->offset_len, buf, got, NULL, 0, NULL);
            if (nrec > rcap) { free(rec); free(starts); rcap = nrec; rec = (uint32_t *)malloc((size_t)rcap * 16); starts = (int64_t *)malloc((size_t)rcap * 8); }
            orc_parse(from->offset, from->offset_len, buf, got, rec, rcap, starts);
            for (int64_t r = 0; r < nrec; r++) {
                int64_t s = starts[r] + 1, e = (int64_t)rec[4 * r + 3] + 1;
                uint8_t *own = (uint8_t *)malloc((size_t)(e - s));
                for (int64_t q = s; q < e; q++) own[q - s] = (uint8_t)rawat(from->offset, from->offset_len, buf, got, q);
                __asm__ volatile("" ::"r"(own) : "memory");
                free(own);
            }
            j->counts[k] = nrec;
        }
    }
    free(buf); free(rec); free(starts);
    return NULL;
}

/* Runs chunks [first, last) on `threads` threads; counts[k] receives chunk k's record count.
 * Returns the total, or a negative code if any chunk failed. */
int64_t orc_decompress_all(const orc_index *ix, const uint8_t *gz, int64_t gzlen, int first, int last,
                           int threads, int mode, int64_t *counts) {
    all_job j;
    memset(&j, 0, sizeof j);
    j.ix = ix; j.gz = gz; j.gzlen = gzlen; j.first = first; j.last = last; j.mode = mode;
    j.next = first; j.counts = counts;
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, all_worker, &j);
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    free(th);
    if (j.err) return j.err;
    int64_t tot = 0;
    for (int k = first; k < last; k++) tot += counts[k];
    return tot;
}
