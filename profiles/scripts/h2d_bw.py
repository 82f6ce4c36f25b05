"""H2D / D2H bandwidth from pinned host memory on MI355X: one copy, chunks on one stream, chunks
spread over 2 / 4 streams (the host-boundary question: is one copy stream the limit?)."""
import time

import torch

N = 30 << 20
REPS = 20
h = torch.empty(N, dtype=torch.uint8).pin_memory()
d = torch.empty(N, dtype=torch.uint8, device="cuda")
streams = [torch.cuda.Stream() for _ in range(4)]


def run(nchunks, nstreams, d2h=False):
    cs = N // nchunks
    for rep in range(REPS + 3):
        if rep == 3:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        for c in range(nchunks):
            s = streams[c % nstreams]
            with torch.cuda.stream(s):
                if d2h:
                    h[c * cs:(c + 1) * cs].copy_(d[c * cs:(c + 1) * cs], non_blocking=True)
                else:
                    d[c * cs:(c + 1) * cs].copy_(h[c * cs:(c + 1) * cs], non_blocking=True)
        for s in streams[:nstreams]:
            s.synchronize()
    dt = (time.perf_counter() - t0) / REPS
    return N / dt / 1e9


for d2h in (False, True):
    for nc, ns in ((1, 1), (4, 1), (4, 2), (4, 4), (8, 4), (16, 4)):
        print(f"{'D2H' if d2h else 'H2D'} chunks={nc:2d} streams={ns}: {run(nc, ns, d2h):6.1f} GB/s", flush=True)
# both directions at once
cs = N
t0 = time.perf_counter()
for _ in range(REPS):
    with torch.cuda.stream(streams[0]):
        d.copy_(h, non_blocking=True)
    with torch.cuda.stream(streams[1]):
        h2 = h  # noqa: F841
    torch.cuda.synchronize()
print("H2D 30 MB single copy + sync:", round(N * REPS / (time.perf_counter() - t0) / 1e9, 1), "GB/s")
