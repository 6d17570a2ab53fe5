"""Locates a host-side fault among the torch ops of partition_edges at a given size."""
import sys
import time

import numpy as np
import torch

m = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 29
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 24


def step(name, f):
    t = time.time()
    print(f"{name} ...", flush=True)
    r = f()
    torch.cuda.synchronize()
    print(f"{name} ok {time.time() - t:.2f}s", flush=True)
    return r


src = np.random.randint(0, n, size=m, dtype=np.uint32)
dst = np.random.randint(0, n, size=m, dtype=np.uint32)
s = step("upload s", lambda: torch.from_numpy(src.view(np.int32)).to("cuda").long() & 0xFFFFFFFF)
d = step("upload d", lambda: torch.from_numpy(dst.view(np.int32)).to("cuda").long() & 0xFFFFFFFF)
key = step("key", lambda: s * n + d)
sk = step("sort", lambda: torch.sort(key).values)
rs = step("div", lambda: sk // n)
rd = step("mod", lambda: sk % n)
deg = step("bincount", lambda: torch.bincount(rs, minlength=n).to(torch.int32))
step("cumsum", lambda: np.cumsum(deg.cpu().numpy().astype(np.uint64)))
step("col", lambda: rd.to(torch.int32).cpu().numpy())
print("all ok", flush=True)
