"""Token-level model of the inflate kernel's round structure ("third span").

Decodes a deflate stream into tokens in pure Python (slow: ~7 min for 3 MB of FASTQ text, so the
sample is small), then replays the kernel's rounds on the token list: a round walks candidate
tokens at bit offsets [0, 64 * spans) and stops at 64 output bytes, at a span's end, or at a code
the 8-bit root tables cannot resolve.  Prints rounds and bytes per round for several layouts.

  python tools/round_sim.py [records]      (bench-shape records, zlib level 6)
"""
import ctypes as C
import os
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CLORD=[16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
LB=[3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
LE=[0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0]
DBASE=[1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577]
DE=[0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]
class BR:
    def __init__(s,b): s.v=int.from_bytes(b,'little'); s.p=0
    def take(s,n):
        r=(s.v>>s.p)&((1<<n)-1); s.p+=n; return r
def mkdec(lens):
    # canonical: map (len,code)->sym
    bl=[0]*16
    for l in lens:
        if l: bl[l]+=1
    code=0; nxt=[0]*16
    for b in range(1,16):
        code=(code+bl[b-1])<<1; nxt[b]=code
    d={}
    for sym,l in enumerate(lens):
        if l:
            c=nxt[l]; nxt[l]+=1
            rc=int(bin(c)[2:].zfill(l)[::-1],2)
            d[(l,rc)]=sym
    return d
def dec(br,d):
    c=0
    for l in range(1,16):
        c|=((br.v>>(br.p+l-1))&1)<<(l-1)
        if (l,c) in d:
            br.p+=l; return d[(l,c)],l
    raise ValueError
def tokens(raw):
    """yields (bitpos, nbits, nbytes, litlen_codelen, dist_codelen, kind) kind 0 lit 1 match 2 eob"""
    br=BR(raw); out=[]
    while True:
        last=br.take(1); t=br.take(2)
        assert t==2, t
        hlit=br.take(5)+257; hd=br.take(5)+1; hc=br.take(4)+4
        cl=[0]*19
        for i in range(hc): cl[CLORD[i]]=br.take(3)
        cd=mkdec(cl); lens=[]
        while len(lens)<hlit+hd:
            sym,_=dec(br,cd)
            if sym<16: lens.append(sym)
            elif sym==16: lens+= [lens[-1]]*(3+br.take(2))
            elif sym==17: lens+=[0]*(3+br.take(3))
            else: lens+=[0]*(11+br.take(7))
        ld=mkdec(lens[:hlit]); dd=mkdec(lens[hlit:])
        while True:
            p0=br.p
            sym,l1=dec(br,ld)
            if sym<256: out.append((p0,l1,1,l1,0,0)); continue
            if sym==256: out.append((p0,l1,0,l1,0,2)); break
            i=sym-257; ml=LB[i]+br.take(LE[i])
            ds,l2=dec(br,dd); dist=DBASE[ds]+br.take(DE[ds])
            out.append((p0,br.p-p0,ml,l1,l2,1))
        if last: return out


def simulate(T, nspan=2, width=64, lazy=False, LBT=8, DBT=8):
    pos_bits, by, l1, l2, kind = T[:, 0], T[:, 2], T[:, 3], T[:, 4], T[:, 5]
    special = (l1 > LBT) | (l2 > DBT) | (kind == 2)
    N = len(T)
    i = cn = rounds = spec_r = span_r = full_r = spans = 0
    total = 0
    while i < N:
        rounds += 1
        bp, off, used, reason = pos_bits[i], cn, 1, None
        while True:
            if off >= width:
                reason = "full"; break
            if i >= N:
                reason = "end"; break
            s = pos_bits[i] - bp
            if s >= 64 * nspan:
                reason = "span"; break
            used = max(used, s // 64 + 1)
            if special[i]:
                reason = "spec"; break
            off += by[i]; i += 1
        spans += used if lazy else nspan
        out = min(off, width); cn = off - out; total += out
        if reason == "spec":
            spec_r += 1; total += by[i]; i += 1; cn = 0
        elif reason == "span":
            span_r += 1
        elif reason == "full":
            full_r += 1
    return dict(rounds=rounds, bytes_per_round=round(total / rounds, 2), special=round(spec_r / rounds, 4),
                span_limited=round(span_r / rounds, 4), full=round(full_r / rounds, 4),
                spans_decoded=round(spans / rounds, 3))


if __name__ == "__main__":
    from parallelparsing_amd import _lib
    S = _lib.synth()
    nrec = int(sys.argv[1]) if len(sys.argv) > 1 else 8000
    sz = S.ppg_synth_fastq_size(0, nrec, 150)
    txt = np.zeros(sz, np.uint8)
    S.ppg_synth_fastq(1, 0, nrec, 150, C.c_void_p(txt.ctypes.data), sz, 4)
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    T = np.array(tokens(co.compress(txt.tobytes()) + co.flush()), np.int64)
    print(f"{sz} bytes of text, {len(T)} tokens")
    for ns in (1, 2, 3):
        print(f"{ns} span(s), 64-byte rounds:", simulate(T, ns))
    print("3 spans, lazily decoded:", simulate(T, 3, lazy=True))
    print("4 spans, 128-byte rounds:", simulate(T, 4, 128))
