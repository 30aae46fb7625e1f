"""Control for the rocprofv3 --memory-copy-trace exit crash: torch only, no framework
code — pinned host <-> device copies and one kernel, then a normal interpreter exit."""
import torch

x = torch.ones(1 << 20, device="cuda")
h = torch.empty(1 << 20, pin_memory=True)
h.copy_(x, non_blocking=True)
x.copy_(h, non_blocking=True)
torch.cuda.synchronize()
print("control ok", float(x.sum()))
