"""The JPEG stage alone (bench.run_jpeg_stage): rate, GPU µs per record (HIP events around the
IDCT + colour launches) and host Huffman µs per file.  AEON_HIP_LIB selects a library variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    r = bench.run_jpeg_stage(A, torch, 256, 10)
    r.pop("what", None)
    print(os.environ.get("AEON_HIP_LIB", "cur"), json.dumps(r), flush=True)
