"""Control for the rocprofv3 --memory-copy-trace exit crash (profiles/r4/spill/README.md):
torch only, no framework code. `pinned`: pinned host <-> device copies on a side stream;
`pageable`: copies from / to ordinary (pageable) host memory, as the engine's begin() of a
400K-node frontier (beyond its pinned staging) does; then a normal interpreter exit."""
import sys

import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "pinned"
n = 16 << 20  # 64 MB of float32
x = torch.ones(n, device="cuda")
h = torch.empty(n, pin_memory=(mode == "pinned"))
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(4):
        h.copy_(x, non_blocking=(mode == "pinned"))
        x.copy_(h, non_blocking=(mode == "pinned"))
torch.cuda.synchronize()
print("control ok", mode, float(x.sum()))
