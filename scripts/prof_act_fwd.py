"""Diagnostic: run only the ACT forward at rollout batch size (for rocprofv3 kernel traces)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from robomanipbaselines_amd.policy.act.act_model import ActModel  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
part = sys.argv[2] if len(sys.argv) > 2 else "all"
torch.backends.cudnn.benchmark = True
torch.manual_seed(0)
m = ActModel().eval().requires_grad_(False)
m.fuse_backbone()
m = m.to("cuda:0", torch.bfloat16)
m._fused = m._fused.to(memory_format=torch.channels_last)
img = torch.rand(B, 1, 3, 480, 640, device="cuda:0").to(torch.bfloat16)
q = torch.randn(B, 7, device="cuda:0", dtype=torch.bfloat16)
with torch.no_grad():
    for _ in range(3):
        m(q, img)
    torch.cuda.synchronize()
    torch.cuda.nvtx.range_push("timed") if hasattr(torch.cuda, "nvtx") else None
    for _ in range(2):
        m(q, img)
    torch.cuda.synchronize()
print("done", flush=True)
