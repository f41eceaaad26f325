"""Probe: torch.distributed.gather on the nccl (RCCL) backend, world size 1 on one GPU (the
multi-rank bench gathers the rank framebuffers with it; RCCL refuses two ranks on one device)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from vulkancomputeraytracing_amd import distributed as D  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29517")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
local = torch.arange(64 * 4 * 3, dtype=torch.float32, device="cuda").view(-1, 4)
out = D.gather_tiles(local, 3)
torch.cuda.synchronize()
assert out is not None and torch.equal(out, local)
print("nccl gather ok", dist.get_backend(), tuple(out.shape))
dist.destroy_process_group()
