import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
import aeon_amd as A, bench
from aeon_amd import configs as C
torch.cuda.set_device(0)
for cfg, b in (("C3", 1024), ("C2", 256)):
    e, kt, pus, sub = bench.run_device(A, C, torch, cfg, b, 20, 3, 0, 1, 400, None, 0)
    print(cfg, "step us %.1f host submit us/step %.1f make_params us/rec %.2f" % (e / 20 * 1e6, sub / 20 * 1e6, pus))
