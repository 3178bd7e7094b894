"""Multi-GPU batched solves: one process per GPU, instances sharded, one all-gather.

The reference solves instances serially on one core (benchmark/path.jl:78-87);
instances are independent, so the batch shards over ranks with no exchange
during the solve.  The only collective is the final solution collection
(north_star: "RCCL all-gather over xGMI only for the final solution
collection"): every rank writes its per-instance results into one packed fp64
record buffer (x | y | s | kkt_error | ϵ) and one int32 buffer
(active_mask words | outer_iters | status | newton_iters | fail_reason bytes),
and two all-gathers (RCCL over xGMI with the "nccl" backend; gloo works the
same way on CPU, which the tests use) deliver the whole batch to every rank —
the integer active-set indices and the per-instance failure reasons included
(north_star: "integer active-set indices bit-exact").

Shards may differ by one instance (``shard_range``: ⌊B/G⌋, +1 for the first
B mod G ranks).  A collective needs equal buffer sizes, so every rank's packed
buffers have room for ``capacity`` = ⌈B/G⌉ instances and the kernel writes
the first ``B_rank`` of them; ``Gatherer.unpack`` drops each rank's padding.
"""

from __future__ import annotations

from dataclasses import dataclass


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard of `total` instances for `rank`: ⌊B/G⌋ (+1 for rank < B mod G),
    the same split as mcpx_solve_batch over devices."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def shard_capacity(total: int, world: int) -> int:
    """Largest shard of `total` over `world` ranks, ⌈B/G⌉ (the common buffer size)."""
    return -(-int(total) // int(world))


_FP_FIELDS = (("x", "n"), ("y", "m"), ("s", "m"), ("kkt_error", 1), ("eps", 1))
_INT_FIELDS = ("outer_iters", "status", "newton_iters")


def mask_words(m: int) -> int:
    """uint64 words of one instance's active-set mask (include/mcpx.h: ⌈m/64⌉, at least 1)."""
    return max(1, (int(m) + 63) // 64)


def irec_len(cap: int, m: int) -> int:
    """int32 entries of the integer record for `cap` instances: the mask words (two int32 each,
    first, so the uint64 view is 8-byte aligned), three counters, ⌈cap/4⌉ words of fail_reason
    bytes; rounded up to even, so that every rank's block of the gathered buffer starts 8-byte
    aligned."""
    L = cap * (2 * mask_words(m) + 3) + (cap + 3) // 4
    return L + (L & 1)


@dataclass
class PackedResults:
    """Per-instance outputs laid out for a single collective each.

    Field blocks are `cap` instances long; the first `B` of each are this
    rank's results (the rest is padding so that every rank's buffer has the
    same size)."""

    rec: "object"   # fp64 [cap * (n + 2m + 2)]: x (cap×n) | y (cap×m) | s (cap×m) | kkt (cap) | ϵ (cap)
    irec: "object"  # int32 [irec_len(cap, m)]: active_mask (cap×words uint64) | outer_iters | status |
    #                 newton_iters | fail_reason (cap bytes)
    B: int
    n: int
    m: int
    cap: int = -1

    def __post_init__(self):
        if self.cap < 0:
            self.cap = self.B
        if self.cap < self.B:
            raise ValueError(f"capacity {self.cap} < batch {self.B}")

    def _width(self, w) -> int:
        return {"n": self.n, "m": self.m}.get(w, w)

    def views(self) -> dict:
        """Output dict (mcp_amd.batch layout) aliasing the packed buffers, so the
        kernel writes its results directly into them."""
        B, cap = self.B, self.cap
        out, o = {}, 0
        for k, w in _FP_FIELDS:
            w = self._width(w)
            out[k] = self.rec[o:o + B * w].view(B, w) if k in ("x", "y", "s") else self.rec[o:o + B]
            o += cap * w
        return dict(out, **_int_views(self.irec, B, cap, self.m), alpha_trace=None)


def alloc_packed(B: int, n: int, m: int, device, capacity: int | None = None) -> PackedResults:
    import torch

    cap = B if capacity is None else int(capacity)
    return PackedResults(torch.empty(max(cap, 1) * (n + 2 * m + 2), dtype=torch.float64, device=device),
                         torch.zeros(irec_len(max(cap, 1), m), dtype=torch.int32, device=device), B, n, m, cap)


def _int_views(irec, B: int, cap: int, m: int) -> dict:
    """The first B instances of each integer field of one rank's int32 record."""
    import torch

    W = mask_words(m)
    o = 2 * W * cap
    out = {"active_mask": irec[:2 * W * B].view(torch.int64).view(B, W)}
    for i, k in enumerate(_INT_FIELDS):
        out[k] = irec[o + i * cap:o + i * cap + B]
    o += 3 * cap
    out["fail_reason"] = irec[o:o + (cap + 3) // 4].view(torch.uint8)[:B]
    return out


class Gatherer:
    """All-gather of PackedResults over a process group (buffers allocated once)."""

    def __init__(self, packed: PackedResults, group=None):
        import torch
        import torch.distributed as dist

        self.p = packed
        self.group = group
        self.world = dist.get_world_size(group)
        self.grec = torch.empty(self.world * packed.rec.numel(), dtype=packed.rec.dtype, device=packed.rec.device)
        self.girec = torch.empty(self.world * packed.irec.numel(), dtype=packed.irec.dtype,
                                 device=packed.irec.device)
        self._into = dist.get_backend(group) != "gloo"  # gloo lacks all_gather_into_tensor
        # gloo gathers host tensors only: device records are staged through host copies
        self._stage = not self._into and packed.rec.is_cuda
        if self._stage:
            self._h = [torch.empty_like(t, device="cpu") for t in (packed.rec, packed.irec, self.grec, self.girec)]

    def __call__(self):
        import torch.distributed as dist

        if self._into:
            dist.all_gather_into_tensor(self.grec, self.p.rec, group=self.group)
            dist.all_gather_into_tensor(self.girec, self.p.irec, group=self.group)
        elif self._stage:
            rec, irec, grec, girec = self._h
            rec.copy_(self.p.rec)
            irec.copy_(self.p.irec)
            dist.all_gather(list(grec.chunk(self.world)), rec, group=self.group)
            dist.all_gather(list(girec.chunk(self.world)), irec, group=self.group)
            self.grec.copy_(grec)
            self.girec.copy_(girec)
        else:
            dist.all_gather(list(self.grec.chunk(self.world)), self.p.rec, group=self.group)
            dist.all_gather(list(self.girec.chunk(self.world)), self.p.irec, group=self.group)

    def unpack(self, counts=None) -> dict:
        """Whole-batch results in global instance order (rank-major = shard order).
        `counts[r]` = instances rank r solved (default: every rank's B, the
        equal-shard case); each rank's padding beyond its count is dropped."""
        import torch

        cap, n, m = self.p.cap, self.p.n, self.p.m
        counts = [self.p.B] * self.world if counts is None else [int(c) for c in counts]
        if len(counts) != self.world or any(c < 0 or c > cap for c in counts):
            raise ValueError(f"bad shard counts {counts} for capacity {cap} x {self.world} ranks")
        recs = self.grec.view(self.world, -1)
        irecs = self.girec.view(self.world, -1)
        out, o = {}, 0
        for k, w in _FP_FIELDS:
            w = self.p._width(w)
            parts = [recs[r, o:o + counts[r] * w].reshape(counts[r], w) for r in range(self.world)]
            cat = torch.cat(parts, 0)
            out[k] = cat if k in ("x", "y", "s") else cat.reshape(-1)
            o += cap * w
        parts = [_int_views(irecs[r], counts[r], cap, m) for r in range(self.world)]
        for k in _INT_FIELDS + ("active_mask", "fail_reason"):
            out[k] = torch.cat([p[k] for p in parts])
        return out
