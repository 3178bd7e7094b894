"""Multi-GPU batched solves: one process per GPU, instances sharded, one all-gather.

The reference solves instances serially on one core (benchmark/path.jl:78-87);
instances are independent, so the batch shards over ranks with no exchange
during the solve.  The only collective is the final solution collection
(north_star: "RCCL all-gather over xGMI only for the final solution
collection"): every rank writes its per-instance results into one packed fp64
record buffer (x | y | s | kkt_error | ϵ) and one int32 buffer
(outer_iters | status | newton_iters), and two all-gathers (RCCL over xGMI with
the "nccl" backend; gloo works the same way on CPU, which the tests use)
deliver the whole batch to every rank.
"""

from __future__ import annotations

from dataclasses import dataclass


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard of `total` instances for `rank`: ⌊B/G⌋ (+1 for rank < B mod G),
    the same split as mcpx_solve_batch over devices."""
    base, extra = divmod(int(total), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


@dataclass
class PackedResults:
    """Per-instance outputs laid out for a single collective each."""

    rec: "object"   # fp64 [B * (n + 2m + 2)]: x (B×n) | y (B×m) | s (B×m) | kkt (B) | ϵ (B)
    irec: "object"  # int32 [3B]: outer_iters | status | newton_iters
    B: int
    n: int
    m: int

    def views(self) -> dict:
        """Output dict (mcp_amd.batch layout) aliasing the packed buffers, so the
        kernel writes its results directly into them."""
        B, n, m = self.B, self.n, self.m
        out, o = {}, 0
        for k, w in (("x", n), ("y", m), ("s", m), ("kkt_error", 1), ("eps", 1)):
            out[k] = self.rec[o:o + B * w].view(B, w) if k in ("x", "y", "s") else self.rec[o:o + B]
            o += B * w
        out["outer_iters"] = self.irec[:B]
        out["status"] = self.irec[B:2 * B]
        out["newton_iters"] = self.irec[2 * B:]
        out["active_mask"] = None
        out["alpha_trace"] = None
        return out


def alloc_packed(B: int, n: int, m: int, device) -> PackedResults:
    import torch

    return PackedResults(torch.empty(B * (n + 2 * m + 2), dtype=torch.float64, device=device),
                         torch.empty(3 * B, dtype=torch.int32, device=device), B, n, m)


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

    def __call__(self):
        import torch.distributed as dist

        if self._into:
            dist.all_gather_into_tensor(self.grec, self.p.rec, group=self.group)
            dist.all_gather_into_tensor(self.girec, self.p.irec, group=self.group)
        else:
            dist.all_gather(list(self.grec.chunk(self.world)), self.p.rec, group=self.group)
            dist.all_gather(list(self.girec.chunk(self.world)), self.p.irec, group=self.group)

    def unpack(self) -> dict:
        """Whole-batch results in global instance order (rank-major = shard order);
        requires equal shard sizes (the weak-scaling benchmark)."""
        import torch

        B, n, m = self.p.B, self.p.n, self.p.m
        recs = self.grec.view(self.world, -1)
        irecs = self.girec.view(self.world, -1)
        out, o = {}, 0
        for k, w in (("x", n), ("y", m), ("s", m), ("kkt_error", 1), ("eps", 1)):
            part = recs[:, o:o + B * w]
            out[k] = part.reshape(self.world * B, w) if k in ("x", "y", "s") else part.reshape(-1)
            o += B * w
        for i, k in enumerate(("outer_iters", "status", "newton_iters")):
            out[k] = irecs[:, i * B:(i + 1) * B].reshape(-1)
        return {k: torch.as_tensor(v) for k, v in out.items()}
