"""Run tools/probe_kernels.hip variants (development only): per-launch time and write/read rates."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libprobe.so"))
L.probe_launch.argtypes = ([ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 6
                          + [ctypes.c_void_p, ctypes.c_void_p])

n = 256
item_out = 3 * 224 * 224 * 4
src_item = 256 * 256 * 3
pool = (400 << 20) // (n * src_item) + 1
src = torch.randint(0, 256, (pool * n * src_item,), dtype=torch.uint8, device="cuda")
out = torch.empty(n * item_out, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
names = {0: "write/wg-per-tile", 1: "write/persistent", 2: "load+write/wg-per-tile", 3: "load+write/persistent",
         4: "desc+load+write", 5: "load+valu+write", 6: "desc+load+valu+write"}
desc = torch.zeros(n * 32, dtype=torch.int64, device="cuda")
desc[::32] = src.data_ptr() + torch.arange(n, device="cuda", dtype=torch.int64) * src_item
cases = [(m, r, g, 0) for m in (0, 2, 3) for r in (9, 18) for g in ((256 * 4,) if m == 3 else (0,))]
cases += [(4, 16, 0, 0)] + [(5, 16, 0, w) for w in (100, 300, 600)] + [(6, 16, 0, w) for w in (300, 600)]
for mode, rows, grid, work in cases:
    if True:
        if True:
            tile_src = rows * 200 * 3  # ~ the staged source footprint of a tile
            def run(k):
                L.probe_launch(mode, ctypes.c_void_p(src.data_ptr() + (k % pool) * n * src_item),
                               ctypes.c_void_p(out.data_ptr()), n, rows, src_item, tile_src, grid, work,
                               ctypes.c_void_p(desc.data_ptr()), ctypes.c_void_p(st.cuda_stream))
            for k in range(3):
                run(k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            it = 20
            for k in range(it):
                run(k)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / it * 1e3
            tiles = n * ((224 + rows - 1) // rows)
            wr = n * item_out
            rd = tiles * tile_src if mode >= 2 else 0
            print(f"{names[mode]:24s} rows={rows:2d} grid={grid:5d} work={work:4d}  {us:6.1f} us  write {wr/us/1e3:6.0f} GB/s"
                  f"  total {(wr+rd)/us/1e3:6.0f} GB/s", flush=True)
