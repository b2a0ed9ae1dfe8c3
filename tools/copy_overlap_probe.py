"""Does a pinned host->device copy on a side stream overlap a long kernel on another stream?
Prints the time of the copy alone, the kernels alone, and both issued together (tools only)."""
import json
import time

import torch

dev = torch.device("cuda:0")
n = 72 * 2**20
h = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device=dev)
a = torch.randn(8192, 8192, device=dev)
cs, ks = torch.cuda.Stream(), torch.cuda.Stream()


def kern():
    with torch.cuda.stream(ks):
        for _ in range(4):
            torch.mm(a, a)


def copy(chunks=1):
    with torch.cuda.stream(cs):
        step = n // chunks
        for i in range(chunks):
            d[i * step:(i + 1) * step].copy_(h[i * step:(i + 1) * step], non_blocking=True)


def timed(f):
    torch.cuda.synchronize()
    t = time.perf_counter()
    f()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t) * 1e3, 3)


for _ in range(3):
    kern(); copy()
res = {"copy_ms": timed(copy), "copy128_ms": timed(lambda: copy(128)), "kern_ms": timed(kern),
       "both_ms": timed(lambda: (kern(), copy())), "both128_ms": timed(lambda: (kern(), copy(128)))}
print(json.dumps(res))
