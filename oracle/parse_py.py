"""TEST INFRASTRUCTURE ONLY — a second, independent restatement of Parsing.Parse / ParseLine /
CombinedMemory (Decompressor/Parsing.cs:11-117), written as a literal Python port of the C#.

It exists to pin oracle/oracle.c's orc_parse, the restatement every record-table parity claim
leans on: the two were written separately, in different languages and shapes (orc_parse records
the terminator positions as it scans; this port yields the C# slices -- idnFrom/idnLen, ... --
and the record's owned copy, exactly as Parsing.cs:41-49 builds a FastqRecord), and must agree on
every input (tests/test_parse_py.py).

What the port keeps from the C#, on purpose:
  * CombinedMemory (Parsing.cs:72-117): `prepend ++ rest` behind an indexer and CopyTo, where
    `rest` is the WHOLE rented buffer, not the chunk: MemoryPool<byte>.Shared.Rent(n)
    (BatchedFASTQ.cs:65) hands out an ArrayPool<byte>.Shared array -- n rounded up to a power of
    two, at least 16, for n <= 2^30 (a fresh n-byte array above that) -- which the reference
    clears before returning it (BatchedFASTQ.cs:73), so the bytes past the chunk are zeros;
  * the loop `for (i = 0; i < raw.Length;)` over that length, `raw[i] == '\\0'` (Parsing.cs:16),
    the unchecked `i++` over the '@' (:19) and the '+' (:30), `ParseLine(...) - 1 < 0` on each of
    the four lines (:23-38) and ParseLine's scan to '\\n' or 0 (:54-69);
  * an index past `raw.Length` raises IndexOutOfRange (a Span indexer would): a chunk whose
    length is exactly a power of two has no zero slack and can read past the end.
    orc_parse and the GPU stop at the chunk's end there instead; callers of this port
    see the exception.

ParseLine is a per-byte loop (parse_literal).  parse_fast replaces only that loop by
bytes.find over the two buffers (same result: the first '\\n' or 0 at or after pos); the tests
check the two agree on random byte soups before using parse_fast on the 100k-read files.
"""


class IndexOutOfRange(IndexError):
    """System.IndexOutOfRangeException from a Span indexer."""


def rented_length(n):
    """Length of the array MemoryPool<byte>.Shared.Rent(n) returns (ArrayPool<byte>.Shared:
    power-of-two buckets from 16 up to 2^30; larger requests get an exact new array)."""
    if n > 1 << 30:
        return n
    size = 16
    while size < n:
        size <<= 1
    return size


class CombinedMemory:
    """Parsing.cs:72-117."""

    def __init__(self, prepend, rest):
        self._prepend = bytes(prepend or b"")
        self._rest = rest
        self._length_p = len(self._prepend)
        self.Length = self._length_p + len(self._rest)

    def __getitem__(self, i):                     # Parsing.cs:87-94
        if i < self._length_p:
            return self._prepend[i]
        j = i - self._length_p
        if j >= len(self._rest):
            raise IndexOutOfRange(i)
        return self._rest[j]

    def CopyTo(self, frm, to, buf):               # Parsing.cs:96-116 (buf: a bytearray, len >= to - frm)
        lp = self._length_p
        if frm < lp and to < lp:
            buf[0:to - frm] = self._prepend[frm:to]
        elif frm < lp and to >= lp:
            pre = self._prepend[frm:lp]
            buf[0:len(pre)] = pre
            buf[lp - frm:lp - frm + (to - lp)] = self._rest[0:to - lp]
        else:
            buf[0:to - frm] = self._rest[frm - lp:to - lp]


def _parse_line_literal(pos, raw):
    """ParseLine (Parsing.cs:53-69): (line length incl. the '\\n', or -1 at a 0; new pos)."""
    start = pos
    while True:
        b = raw[pos]
        if b == 10 or b == 0:
            break
        pos += 1
    if raw[pos] == 0:
        return -1, pos
    pos += 1                                      # consume \n
    return pos - start, pos


def _parse_line_fast(pos, raw):
    """The same function: the first '\\n' or 0 at or after pos found with bytes.find over the
    prepend, then the rented buffer."""
    lp = raw._length_p
    hit = -1
    if pos < lp:
        a, b = raw._prepend.find(b"\n", pos), raw._prepend.find(b"\0", pos)
        c = [x for x in (a, b) if x >= 0]
        if c:
            hit = min(c)
    if hit < 0:
        q = max(pos, lp) - lp
        a, b = raw._rest.find(b"\n", q), raw._rest.find(b"\0", q)
        c = [x for x in (a, b) if x >= 0]
        if not c:
            raise IndexOutOfRange(raw.Length)
        hit = lp + min(c)
    if raw[hit] == 0:
        return -1, hit
    return hit + 1 - pos, hit + 1


def _parse(raw, parse_line, materialize):
    """Parsing.Parse (Parsing.cs:11-51).  Yields (start, end, (idnFrom, idnLen), (seqFrom, seqLen),
    (plsFrom, plsLen), (qltFrom, qltLen), record bytes or None) -- offsets into raw, as the C# has
    them before slicing its owned copy."""
    i = 0
    while i < raw.Length:
        if raw[i] == 0:                           # empty space
            break
        i += 1                                    # skip @
        start = i
        idn_from = i
        n, i = parse_line(i, raw)
        idn_len = n - 1
        if idn_len < 0:
            break
        seq_from = i
        n, i = parse_line(i, raw)
        seq_len = n - 1
        if seq_len < 0:
            break
        i += 1                                    # skip +
        pls_from = i
        n, i = parse_line(i, raw)
        pls_len = n - 1
        if pls_len < 0:
            break
        qlt_from = i
        n, i = parse_line(i, raw)
        qlt_len = n - 1
        if qlt_len < 0:
            break
        end = i
        mem = None
        if materialize:                           # Parsing.cs:41-47: Rent(end - start), CopyTo, Slice
            mem = bytearray(end - start)
            raw.CopyTo(start, end, mem)
        yield (start, end, (idn_from, idn_len), (seq_from, seq_len), (pls_from, pls_len), (qlt_from, qlt_len),
               bytes(mem) if mem is not None else None)


def chunk_raw(offset, chunk, rented=None):
    """new CombinedMemory(from.offset, buf) with buf the rented, zero-padded chunk buffer
    (BatchedFASTQ.cs:65-68)."""
    chunk = bytes(chunk)
    size = rented_length(len(chunk)) if rented is None else rented
    return CombinedMemory(offset, chunk + bytes(size - len(chunk)))


def parse_literal(offset, chunk, materialize=False, rented=None):
    return list(_parse(chunk_raw(offset, chunk, rented), _parse_line_literal, materialize))


def parse_fast(offset, chunk, materialize=False, rented=None):
    return list(_parse(chunk_raw(offset, chunk, rented), _parse_line_fast, materialize))


def terminators(records):
    """The records as orc_parse / the GPU descriptors state them: the positions in raw of each
    field's terminating '\\n' (n1..n4 = From + Len of the four slices)."""
    return [(i[0] + i[1], s[0] + s[1], p[0] + p[1], q[0] + q[1]) for _, _, i, s, p, q, _ in records]
