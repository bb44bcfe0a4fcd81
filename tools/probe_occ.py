"""The pattern probe (libkinprobe.so kinprobe_pattern3) over the occupancies bench.py sweeps: the headline's
8-in / 60-out pattern at 2^20 (tiled 8192, plain ld = N + 256, plain ld = N), 2^22 tiled, 2^24 tiled grid-strided."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.Stream(dev)
for name, n, tile, ld, pl in (("2^20 tiled", 1 << 20, 8192, 0, 1), ("2^20 ld=N+256", 1 << 20, 0, (1 << 20) + 256, 1),
                              ("2^20 ld=N", 1 << 20, 0, 1 << 20, 1), ("2^22 tiled", 1 << 22, 8192, 0, 1),
                              ("2^24 tiled strided", 1 << 24, 8192, 0, 2)):
    r = [bench._pattern_at(8, 60, n, tile, st, 10, 2, ld, pl, lds, blk) for lds, blk in bench.PROBE_OCC]
    print(name, " ".join(f"{l}/{b}:{t:.1f}us" for (l, b), t in zip(bench.PROBE_OCC, r)), flush=True)
    if pl == 1:  # the LDS-staged 16-byte row stores (p_pattern_x4)
        occ = ((61440, 256), (65536, 256), (30720, 128), (53248, 128), (65536, 128))
        r = [bench._pattern_at(8, 60, n, tile, st, 10, 2, ld, -1, lds, blk) for lds, blk in occ]
        print(name, "x4", " ".join(f"{l}/{b}:{t:.1f}us" for (l, b), t in zip(occ, r)), flush=True)
