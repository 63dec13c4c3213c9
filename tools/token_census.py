"""Token census of the bench member's deflate stream ("measure first").

Decodes a bench-shape sample (the same generator and zlib level 6 as the 50 GB member) into
tokens with a table-driven pure-Python decoder, then replays the kernel's hot round (two 64-bit
candidate spans, 64 output bytes, a code the 8-bit root tables cannot resolve ends it;
tools/round_sim.py) and counts, per round: tokens walked by kind (literal / match), literal runs,
and how many walk steps a root entry carrying TWO short literals (both codes within the 8-bit
litlen root) would save.

  python tools/token_census.py [records] [--json out.json]
"""
import ctypes as C
import json
import os
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CLORD = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LE = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DE = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


class BR:
    def __init__(s, b):
        s.b = b + bytes(16)
        s.p = 0

    def peek(s, n):
        q = s.p >> 3
        return (int.from_bytes(s.b[q:q + 8], 'little') >> (s.p & 7)) & ((1 << n) - 1)

    def take(s, n):
        r = s.peek(n)
        s.p += n
        return r


def mktab(lens):
    """15-bit lookup: reversed code bits -> (sym, len)"""
    bl = [0] * 16
    for l in lens:
        if l:
            bl[l] += 1
    code = 0
    nxt = [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    tab = [None] * (1 << 15)
    for sym, l in enumerate(lens):
        if l:
            c = nxt[l]
            nxt[l] += 1
            rc = int(bin(c)[2:].zfill(l)[::-1], 2)
            for hi in range(1 << (15 - l)):
                tab[rc | (hi << l)] = (sym, l)
    return tab


def tokens(raw):
    """(bitpos, nbits, nbytes, litlen codelen, dist codelen, kind: 0 literal 1 match 2 eob, literal byte)"""
    br = BR(raw)
    out = []
    while True:
        last = br.take(1)
        t = br.take(2)
        assert t == 2, t
        hlit = br.take(5) + 257
        hd = br.take(5) + 1
        hc = br.take(4) + 4
        cl = [0] * 19
        for i in range(hc):
            cl[CLORD[i]] = br.take(3)
        ct = mktab(cl)
        lens = []
        while len(lens) < hlit + hd:
            sym, l = ct[br.peek(15)]
            br.p += l
            if sym < 16:
                lens.append(sym)
            elif sym == 16:
                lens += [lens[-1]] * (3 + br.take(2))
            elif sym == 17:
                lens += [0] * (3 + br.take(3))
            else:
                lens += [0] * (11 + br.take(7))
        lt = mktab(lens[:hlit])
        dt = mktab(lens[hlit:])
        while True:
            p0 = br.p
            sym, l1 = lt[br.peek(15)]
            br.p += l1
            if sym < 256:
                out.append((p0, l1, 1, l1, 0, 0, sym))
                continue
            if sym == 256:
                out.append((p0, l1, 0, l1, 0, 2, 0))
                break
            i = sym - 257
            ml = LB[i] + br.take(LE[i])
            ds, l2 = dt[br.peek(15)]
            br.p += l2
            br.take(DE[ds])
            out.append((p0, br.p - p0, ml, l1, l2, 1, 0))
        if last:
            return out


def census(T, LBT=8, DBT=8, width=64, nspan=2):
    """replay the hot round; count walk steps by kind and what literal pairs would save"""
    pos_bits, by, l1, l2, kind = T[:, 0], T[:, 2], T[:, 3], T[:, 4], T[:, 5]
    special = (l1 > LBT) | (l2 > DBT) | (kind == 2)
    N = len(T)
    i = cn = rounds = 0
    c = dict(walk_lit=0, walk_match=0, walk_steps=0, walk_steps_pairs=0, lit_runs2=0, rounds_span=0,
             rounds_full=0, rounds_spec=0, bytes=0)
    while i < N:
        rounds += 1
        bp, off = pos_bits[i], cn
        reason = None
        run = 0       # current run of pairable literals in this round's walk
        steps_pair = 0
        while True:
            if off >= width:
                reason = "full"
                break
            if i >= N:
                reason = "end"
                break
            if pos_bits[i] - bp >= 64 * nspan:
                reason = "span"
                break
            if special[i]:
                reason = "spec"
                break
            c["walk_steps"] += 1
            if kind[i] == 0:
                c["walk_lit"] += 1
                # a pair: this literal and the next, both codes in one 8-bit root index, and the
                # pair starting inside the span (greedy from the run's start)
                if run == 0 and i + 1 < N and kind[i + 1] == 0 and l1[i] + l1[i + 1] <= LBT \
                        and pos_bits[i + 1] - bp < 64 * nspan:
                    run = 1
                    steps_pair += 1
                    c["lit_runs2"] += 1
                elif run == 1:
                    run = 0       # second half of a pair: no walk step of its own
                else:
                    steps_pair += 1
            else:
                run = 0
                c["walk_match"] += 1
                steps_pair += 1
            off += by[i]
            i += 1
        c["walk_steps_pairs"] += steps_pair
        out = min(off, width)
        cn = off - out
        c["bytes"] += out
        c["rounds_" + (reason if reason != "end" else "span")] += 1
        if reason == "spec":
            c["bytes"] += by[i]
            i += 1
            cn = 0
    c["rounds"] = rounds
    r = {k: int(v) for k, v in c.items()}
    r["bytes_per_round"] = round(c["bytes"] / rounds, 2)
    r["tokens_per_round"] = round(c["walk_steps"] / rounds, 3)
    r["literal_share_of_walk_steps"] = round(c["walk_lit"] / max(1, c["walk_steps"]), 4)
    r["walk_steps_saved_by_pairs"] = round(1 - c["walk_steps_pairs"] / max(1, c["walk_steps"]), 4)
    return r


if __name__ == "__main__":
    from parallelparsing_amd import _lib
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    nrec = int(args[0]) if args else 20000
    S = _lib.synth()
    sz = S.ppg_synth_fastq_size(0, nrec, 150)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(1, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 4)
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    T = np.array(tokens(co.compress(txt.tobytes()) + co.flush()), np.int64)
    lits = T[T[:, 5] == 0]
    res = dict(records=nrec, text_bytes=int(sz), tokens=len(T),
               literal_tokens=int(len(lits)), match_tokens=int((T[:, 5] == 1).sum()),
               literal_bytes_share=round(len(lits) / sz, 4),
               literal_code_len_hist={int(k): int(v) for k, v in zip(*np.unique(lits[:, 3], return_counts=True))},
               literal_byte_hist={chr(int(k)): int(v) for k, v in zip(*np.unique(lits[:, 6], return_counts=True))},
               match_len_mean=round(float(T[T[:, 5] == 1][:, 2].mean()), 2),
               hot_round=census(T))
    print(json.dumps(res, indent=1))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(res, f, indent=1)
