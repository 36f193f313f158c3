"""CPU: the N>1 layout and exchange step with torch.distributed gloo, world_size 2."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from safestakeoperator_amd.shard import exchange, pack_bits, shard_jobs, unpack_bits


def test_shard_jobs_cover_and_balance():
    off = [0]
    for j in range(1000):
        off.append(off[-1] + (4 if j % 3 else 13))
    for W in (1, 2, 4, 8):
        ranges = [shard_jobs(off, W, r) for r in range(W)]
        assert ranges[0][0] == 0 and ranges[-1][1] == 1000
        for a, b in zip(ranges, ranges[1:]):
            assert a[1] == b[0]
        sizes = [off[j1] - off[j0] for j0, j1 in ranges]
        assert max(sizes) - min(sizes) <= 2 * 13


def test_bits_roundtrip():
    v = (torch.arange(1003) % 7 == 3).to(torch.uint8)
    assert torch.equal(unpack_bits(pack_bits(v), 1003), v)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, J = 37, 9
    g = torch.Generator().manual_seed(100 + rank)
    ver = (torch.rand(n, generator=g) > 0.1).to(torch.uint8)
    sig = torch.randint(0, 256, (J, 96), dtype=torch.uint8, generator=g)
    st = torch.randint(0, 5, (J,), dtype=torch.int32, generator=g)
    bits, sigs, sts = exchange(ver, sig, st)
    q.put((rank, [unpack_bits(bits[r], n) for r in range(world)], sigs.clone(), sts.clone(), ver, sig, st))
    dist.barrier()
    dist.destroy_process_group()


def test_exchange_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        _, vers, sigs, sts, _, _, _ = res[r]
        for src in range(world):
            assert torch.equal(vers[src], res[src][4])
            assert torch.equal(sigs[src], res[src][5])
            assert torch.equal(sts[src], res[src][6])
