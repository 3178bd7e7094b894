"""PCIe host→device ceiling on the box: one θ batch's worth of bytes (C3: 830 MB)
copied from pinned and from pageable host memory, split over 1, 2, 4 and 8
streams (torch tensors, HIP streams).  Prints one JSON line per variant."""
import json
import time

import torch

BYTES = 65536 * 1584 * 8
dev = torch.device("cuda", 0)
dst = torch.empty(BYTES // 8, dtype=torch.float64, device=dev)
for kind in ("pinned", "pageable"):
    src = torch.empty(BYTES // 8, dtype=torch.float64, pin_memory=(kind == "pinned"))
    src.fill_(1.0)
    for S in (1, 2, 4, 8):
        streams = [torch.cuda.Stream(dev) for _ in range(S)]
        parts = list(zip(src.chunk(S * 4), dst.chunk(S * 4)))
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for i, (s, d) in enumerate(parts):
                with torch.cuda.stream(streams[i % S]):
                    d.copy_(s, non_blocking=True)
            torch.cuda.synchronize(dev)
            best = min(best, time.perf_counter() - t0)
        print(json.dumps({"host": kind, "streams": S, "GB/s": BYTES / best / 1e9, "ms": best * 1e3}), flush=True)
