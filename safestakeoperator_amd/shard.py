"""Multi-GPU layout for the threshold-BLS engine.

Jobs (validator, signing root) are independent: rank r of W takes a contiguous block of
validators, balanced by share count, and runs the whole pipeline on its own GPU with no
collective in the kernel path.  The single exchange per batch is an all-gather (RCCL over xGMI
when the tensors live on the GPU, gloo in the CPU tests) of
  * the verdict bitmap (1 bit per share),
  * the per-job status words (and error fields),
  * the 96-byte combined signatures.

Two ways to use it:
  * weak scaling (bench.py default): every rank has its own batch of the same shape -> `exchange`
    (equal shapes, one all-gather per array);
  * strong scaling (one global batch, e.g. C4's 1,048,576 shares split over 2/4/8 GPUs):
    `shard_jobs` picks each rank's contiguous job range (share-balanced, so ranks may hold
    different job and share counts; every rank knows every shard's size, `shard_sizes`),
    `local_batch` re-bases that slice, and `exchange_var` all-gathers the variable-size results as
    pad-to-max tensors and trims them back into the global job / share order -- byte-identical to
    a single-rank run of the whole batch.
This replaces the reference's per-validator fan-out (src/validation/impls/hotstuff.rs:146-166: one
async task per operator and duty) with one batched pass per GPU.
"""
from typing import Dict, List, Sequence, Tuple

import torch


def shard_jobs(share_off: Sequence[int], world: int, rank: int) -> Tuple[int, int]:
    """Contiguous job range [j0, j1) for `rank`, balanced by share count: rank r starts at the
    first job whose first share is >= r/W of all shares."""
    import bisect
    n_jobs = len(share_off) - 1
    total = share_off[-1]
    lo = total * rank // world
    hi = total * (rank + 1) // world
    j0 = min(bisect.bisect_left(share_off, lo), n_jobs)
    j1 = min(bisect.bisect_left(share_off, hi), n_jobs) if rank < world - 1 else n_jobs
    return j0, j1


def local_batch(share_off: Sequence[int], j0: int, j1: int) -> Dict[str, object]:
    """The slice of a global batch a rank runs: local share offsets (starting at 0) and the global
    share range [s0, s1) its per-share arrays come from."""
    s0, s1 = int(share_off[j0]), int(share_off[j1])
    return {"share_off": [int(x) - s0 for x in share_off[j0:j1 + 1]], "s0": s0, "s1": s1, "j0": j0, "j1": j1}


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


def _all_gather(x: torch.Tensor, world: int, group, async_op: bool):
    # concatenated (world * dim0) output: the form both RCCL and gloo accept
    import torch.distributed as dist
    g = torch.empty((world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    work = dist.all_gather_into_tensor(g, x.contiguous(), group=group, async_op=async_op)
    return g.view((world,) + tuple(x.shape)), work


def exchange(verdicts_u8: torch.Tensor, sigs96: torch.Tensor, status: torch.Tensor, group=None, async_op: bool = False):
    """All-gather one batch's results from every rank (equal shapes on every rank).
    Returns (bitmaps[W, ceil(n/8)], sigs[W, J, 96], status[W, J]), plus the list of collective
    handles when async_op (the caller orders the next use of the input buffers after
    handle.wait(), which makes the CURRENT stream wait -- the host never blocks)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    bits = pack_bits(verdicts_u8)
    out, works = [], []
    for x in (bits, sigs96, status):
        g, w = _all_gather(x, world, group, async_op)
        out.append(g)
        works.append(w)
    return (tuple(out), works) if async_op else tuple(out)


def shard_sizes(share_off: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """(shares, jobs) of every rank's shard -- known to every rank without communication."""
    out = []
    for r in range(world):
        j0, j1 = shard_jobs(share_off, world, r)
        out.append((int(share_off[j1]) - int(share_off[j0]), j1 - j0))
    return out


def exchange_var(verdicts_u8: torch.Tensor, sigs96: torch.Tensor, status: torch.Tensor, err: torch.Tensor,
                 group=None, sizes: Sequence[Tuple[int, int]] = None, async_op: bool = False, batches: int = 1):
    """All-gather results whose sizes differ per rank (a strong-scaling split of one batch): every
    array padded to the largest rank's size, gathered, then trimmed and concatenated in rank order.
    `sizes` = every rank's (shares, jobs) of ONE batch (shard_sizes); gathered first when not given.
    Returns the GLOBAL (verdicts[N], sigs[J, 96], status[J], err[J, 2]) on every rank; with async_op
    the padded gathers are left in flight and a finish() closure (trim + concatenate, call after the
    handles' wait()) is returned with the handles.
    batches > 1: the local arrays are that many same-shape batches of this rank's shard back to back
    (one collective for a group of pipelined batches); the result is then a list of `batches` global
    tuples, batch b reassembled from every rank's b-th slice."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = verdicts_u8.device
    B = max(1, int(batches))
    n_loc, j_loc = int(verdicts_u8.numel()) // B, int(status.numel()) // B
    if sizes is None:
        g, _ = _all_gather(torch.tensor([n_loc, j_loc], dtype=torch.int64, device=dev), world, group, False)
        sizes = [tuple(x) for x in g.cpu().tolist()]
    n_max = max(max(s[0] for s in sizes), 1)
    j_max = max(max(s[1] for s in sizes), 1)
    nb_max = (n_max + 7) // 8

    def padded(x, m):   # (B * rows, ...) -> (B * m, ...), each batch's rows padded to m
        x = x.reshape((B, -1) + tuple(x.shape[1:]))
        p = torch.zeros((B, m) + tuple(x.shape[2:]), dtype=x.dtype, device=dev)
        p[:, :x.shape[1]] = x
        return p.reshape((B * m,) + tuple(x.shape[2:]))

    bits_loc = torch.cat([pack_bits(verdicts_u8[b * n_loc:(b + 1) * n_loc]) for b in range(B)]) if B > 1 else pack_bits(verdicts_u8)
    gathered, works = [], []
    for x, m in ((bits_loc, nb_max), (sigs96, j_max), (status, j_max), (err, j_max)):
        g, w = _all_gather(padded(x, m), world, group, async_op)
        gathered.append(g.view((world, B, m) + tuple(g.shape[2:])))
        works.append(w)
    bits, sg, st, er = gathered

    def one(b):
        ver = torch.cat([unpack_bits(bits[r, b], sizes[r][0]) for r in range(world)])
        return (ver, torch.cat([sg[r, b, :sizes[r][1]] for r in range(world)]),
                torch.cat([st[r, b, :sizes[r][1]] for r in range(world)]),
                torch.cat([er[r, b, :sizes[r][1]] for r in range(world)]))

    def finish():
        return [one(b) for b in range(B)] if B > 1 else one(0)
    return (finish, works) if async_op else finish()


def run_sharded(batch_fn, share_off: Sequence[int], per_share: Dict[str, Sequence], per_job: Dict[str, Sequence],
                group=None):
    """Strong scaling of ONE global batch: this rank runs `batch_fn(share_off_local, shares, jobs)`
    on its job range -- shares / jobs are the per-share and per-job argument lists sliced to the
    range -- which returns (verdicts_u8[n], sigs96[j, 96], status[j], err[j, 2]) tensors; the
    results of all ranks are all-gathered back into the global order."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    j0, j1 = shard_jobs(share_off, world, rank)
    lb = local_batch(share_off, j0, j1)
    shares = {k: v[lb["s0"]:lb["s1"]] for k, v in per_share.items()}
    jobs = {k: v[j0:j1] for k, v in per_job.items()}
    ver, sg, st, er = batch_fn(lb["share_off"], shares, jobs)
    return exchange_var(ver, sg, st, er, group=group, sizes=shard_sizes(share_off, world))


class BatchExchange:
    """The per-group exchange step of a pipelined run (bench.py): the results of the batches
    submitted since the last exchange -- one per pipeline slot -- are all-gathered in ONE
    collective per array (fewer, larger collectives), asynchronously; the caller makes each
    slot's next batch wait for the handles (`works`) before it rewrites that slot's outputs.

      weak:   every rank runs its own batch of the same shape (`exchange`);
      strong: every rank runs its shard of ONE global batch (`exchange_var` with `sizes` = the
              per-batch (shares, jobs) of every rank, `batches` = the group size), reassembled
              into the global order per batch.

    `check_last()` (untimed) verifies the last group's gathered results against this rank's local
    outputs at this rank's position, and returns the gathered / reassembled results for further
    checks.  `outs[k]` holds the slot's tensors "ver", "out", "st", "err"."""

    def __init__(self, strong: bool, sizes: Sequence[Tuple[int, int]] = None, group=None, device=None):
        self.strong, self.sizes, self.group, self.device = strong, sizes, group, device
        self.last = None     # (local output dicts, gathered or finish closure, works)

    def flush(self, outs: Sequence[Dict[str, torch.Tensor]]):
        dev = self.device
        cat = lambda key: torch.cat([o[key] for o in outs]).to(dev) if dev is not None else torch.cat([o[key] for o in outs])
        if self.strong:
            res, works = exchange_var(cat("ver"), cat("out"), cat("st"), cat("err"), group=self.group, sizes=self.sizes,
                                      async_op=True, batches=len(outs))
        else:
            res, works = exchange(cat("ver"), cat("out"), cat("st"), group=self.group, async_op=True)
        works = [w for w in works if w is not None]
        self.last = (list(outs), res, works)
        return works

    def check_last(self):
        """(ok, results): ok iff every batch of the last group came back from the collective equal
        to this rank's local outputs (weak: the gathered row of this rank; strong: the slice of the
        reassembled global batch at this rank's offsets)."""
        import torch.distributed as dist
        if self.last is None:
            return True, None
        outs, res, works = self.last
        for w in works:
            w.wait()
        rank = dist.get_rank(self.group)
        ok = True
        if self.strong:
            glob = res()
            if not isinstance(glob, list):
                glob = [glob]
            s0 = sum(s[0] for s in self.sizes[:rank])
            j0 = sum(s[1] for s in self.sizes[:rank])
            for o, (ver, sg, st, er) in zip(outs, glob):
                n, j = o["ver"].numel(), o["st"].numel()
                ok = ok and torch.equal(ver[s0:s0 + n].cpu(), o["ver"].cpu()) and torch.equal(sg[j0:j0 + j].cpu(), o["out"].cpu())
                ok = ok and torch.equal(st[j0:j0 + j].cpu(), o["st"].cpu()) and torch.equal(er[j0:j0 + j].cpu(), o["err"].cpu())
            return ok, glob
        bits, sg, st = res
        B = len(outs)
        n, j = outs[0]["ver"].numel(), outs[0]["st"].numel()
        world = bits.shape[0]
        per_batch = []
        all_ver = [unpack_bits(bits[r], B * n) for r in range(world)]
        for b, o in enumerate(outs):
            ok = ok and torch.equal(all_ver[rank][b * n:(b + 1) * n].cpu(), o["ver"].cpu())
            ok = ok and torch.equal(sg[rank][b * j:(b + 1) * j].cpu(), o["out"].cpu())
            ok = ok and torch.equal(st[rank][b * j:(b + 1) * j].cpu(), o["st"].cpu())
            per_batch.append([(all_ver[r][b * n:(b + 1) * n], sg[r][b * j:(b + 1) * j], st[r][b * j:(b + 1) * j])
                              for r in range(world)])
        return ok, per_batch
