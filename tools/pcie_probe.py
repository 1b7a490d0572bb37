"""PCIe rates of this box: pinned / pageable host <-> device copies of the FABRIK
host path's sizes (24 MB points in, 36 MB angles + iterations out per 1M points),
one direction at a time and both at once on two streams."""
import json
import time

import torch


def rate(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


out = {}
for label, nb in (("24MB", 24_000_000), ("36MB", 36_000_000)):
    d = torch.empty(nb, dtype=torch.uint8, device="cuda")
    hp = torch.empty(nb, dtype=torch.uint8).pin_memory()
    hq = torch.empty(nb, dtype=torch.uint8)
    out[f"h2d_pinned_{label}"] = rate(lambda: d.copy_(hp, non_blocking=True), nb)
    out[f"d2h_pinned_{label}"] = rate(lambda: hp.copy_(d, non_blocking=True), nb)
    out[f"h2d_pageable_{label}"] = rate(lambda: d.copy_(hq), nb)
    out[f"d2h_pageable_{label}"] = rate(lambda: hq.copy_(d), nb)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
d1 = torch.empty(24_000_000, dtype=torch.uint8, device="cuda")
d2 = torch.empty(36_000_000, dtype=torch.uint8, device="cuda")
h1 = torch.empty(24_000_000, dtype=torch.uint8).pin_memory()
h2 = torch.empty(36_000_000, dtype=torch.uint8).pin_memory()


def both():
    with torch.cuda.stream(s1):
        d1.copy_(h1, non_blocking=True)
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)


out["duplex_60MB_GBps"] = rate(both, 60_000_000)
print(json.dumps({k: round(v, 2) for k, v in out.items()}))
