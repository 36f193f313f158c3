"""Multi-GPU layout for the threshold-BLS engine.

Jobs (validator, signing root) are independent: rank r of W takes a contiguous block of
validators, balanced by share count, and runs the whole pipeline on its own GPU with no
collective in the kernel path.  The single exchange per batch is an all-gather (RCCL over xGMI
when the tensors live on the GPU, gloo in the CPU tests) of
  * the verdict bitmap (1 bit per share),
  * the per-job status words,
  * the 96-byte combined signatures.
"""
from typing import List, Tuple

import torch


def shard_jobs(share_off: List[int], world: int, rank: int) -> Tuple[int, int]:
    """Contiguous job range [j0, j1) for `rank`, balanced by share count."""
    n_jobs = len(share_off) - 1
    total = share_off[-1]
    lo = total * rank // world
    hi = total * (rank + 1) // world
    j0 = next((j for j in range(n_jobs + 1) if share_off[j] >= lo), n_jobs)
    j1 = next((j for j in range(n_jobs + 1) if share_off[j] >= hi), n_jobs) if rank < world - 1 else n_jobs
    return j0, j1


def pack_bits(verdicts_u8: torch.Tensor) -> torch.Tensor:
    """uint8 0/1 per share -> little-endian bitmap, ceil(n/8) bytes (on the verdicts' device)."""
    n = verdicts_u8.numel()
    pad = torch.zeros(((n + 7) // 8) * 8, dtype=torch.int32, device=verdicts_u8.device)
    pad[:n] = verdicts_u8.to(torch.int32)
    w = (2 ** torch.arange(8, dtype=torch.int32, device=verdicts_u8.device)).view(1, 8)
    return (pad.view(-1, 8) * w).sum(1).to(torch.uint8)


def unpack_bits(bits: torch.Tensor, n: int) -> torch.Tensor:
    w = (2 ** torch.arange(8, dtype=torch.int32, device=bits.device)).view(1, 8)
    return ((bits.to(torch.int32).view(-1, 1) & w) != 0).view(-1)[:n].to(torch.uint8)


def exchange(verdicts_u8: torch.Tensor, sigs96: torch.Tensor, status: torch.Tensor, group=None):
    """All-gather one batch's results from every rank (equal shapes on every rank).
    Returns (bitmaps[W, ceil(n/8)], sigs[W, J, 96], status[W, J])."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    bits = pack_bits(verdicts_u8)
    out = []
    for x in (bits, sigs96, status):
        # concatenated (world * dim0) output: the form both RCCL and gloo accept
        g = torch.empty((world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(g, x.contiguous(), group=group)
        out.append(g.view((world,) + tuple(x.shape)))
    return tuple(out)
