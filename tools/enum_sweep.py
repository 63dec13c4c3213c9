"""Sweep of the record cursor's (ppg_cursor) knobs on the GPU box: batches in flight
(PPG_CURSOR_SLOTS), per-chunk copies vs device packing (PPG_CURSOR_PACK), batch size and reader
threads, over the bench's tiled member written to $TMPDIR.  One JSON line per configuration.

  python tools/enum_sweep.py [--repeats 26] [--runs 1] [--configs slots:pack:gib:threads[:pack_blocks[:pack_cus[:h2d[:d2h_piece_mib]]]] ...]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=26)
    ap.add_argument("--runs", type=int, default=1)
    ap.add_argument("--configs", nargs="*", default=["3:0:8:16", "4:0:4:8", "5:0:4:6", "6:0:2:4", "4:1:4:8"])
    a = ap.parse_args()
    import torch
    import parallelparsing_amd as pp
    from parallelparsing_amd.tiled import TiledFile
    import bench
    tf = TiledFile(10_485_760, a.repeats, 10000, threads=16)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"ppg_enum_{os.getpid()}.gz")
    try:
        with open(path, "wb") as f:
            for lo in range(0, tf.file_len, 1 << 30):
                f.write(tf.file_bytes(lo, min(tf.file_len, lo + (1 << 30))))
        ix = tf.index(0, tf.npoints)
        dev = pp.Device(0)
        pcie = bench.pcie_d2h_GBps(torch.device("cuda", 0))
        print(json.dumps({"pcie_d2h_GBps": pcie, "gz_GB": tf.file_len / 1e9}), flush=True)
        for c in a.configs:
            slots, pack, gib, th, *pb = c.split(":")
            os.environ["PPG_CURSOR_SLOTS"], os.environ["PPG_CURSOR_PACK"] = slots, pack
            os.environ["PPG_CURSOR_PACK_BLOCKS"] = pb[0] if pb else "256"
            os.environ["PPG_CURSOR_PACK_CUS"] = pb[1] if len(pb) > 1 else "0"
            os.environ["PPG_CURSOR_H2D"] = pb[2] if len(pb) > 2 else "0"
            os.environ["PPG_CURSOR_D2H_PIECE_MIB"] = pb[3] if len(pb) > 3 else "0"
            for _ in range(a.runs):
                r = bench.enumerate_run(tf, ix, path, dev, int(th), float(gib), pcie)
                r.pop("note")
                print(json.dumps(dict(r, config=c)), flush=True)
    finally:
        if os.path.exists(path):
            os.remove(path)


if __name__ == "__main__":
    main()
