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


# ---- strong scaling: one global batch split over ranks (uneven shards), results reassembled ----
def _golden_global_batch():
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "threshold_cases.json")) as f:
        cases = json.load(f)["cases"]
    roots, t, off, sigs, pks, ids, jr = [], [], [0], [], [], [], []
    for c in cases:
        r = bytes.fromhex(c["root"])
        if r not in roots:
            roots.append(r)
        jr.append(roots.index(r))
        t.append(c["t"])
        sigs += [bytes.fromhex(s) for s in c["sigs"]]
        pks += [bytes.fromhex(p) for p in c["pks"]]
        ids += c["ids"]
        off.append(len(sigs))
    return roots, t, off, sigs, pks, ids, jr


def _oracle_batch(roots):
    """the C oracle as the per-rank engine (every share verified, the engine's semantics)"""
    from oracle import bls_c

    def fn(share_off, shares, jobs):
        out, st, err, ver = bls_c.threshold_batch(share_off, jobs["t"], b"".join(shares["sigs"]), b"".join(shares["pks"]),
                                                  shares["ids"], jobs["jr"], roots, 2, verify_all=True)
        n = share_off[-1]
        return (torch.from_numpy(ver[:n].copy()), torch.from_numpy(out.copy()), torch.from_numpy(st.copy()),
                torch.from_numpy(err.astype("int64")))
    return fn


def _strong_worker(rank, world, port, q):
    import torch.distributed as dist
    from safestakeoperator_amd.shard import run_sharded, shard_jobs
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    roots, t, off, sigs, pks, ids, jr = _golden_global_batch()
    ver, sg, st, er = run_sharded(_oracle_batch(roots), off, {"sigs": sigs, "pks": pks, "ids": ids}, {"t": t, "jr": jr})
    j0, j1 = shard_jobs(off, world, rank)
    q.put((rank, j1 - j0, ver.numpy(), sg.numpy(), st.numpy(), er.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_strong_scaling_reassembles_global_batch(world):
    """One global batch (every golden threshold case: mixed t, roots, error paths) split over
    `world` gloo ranks by shard_jobs (world 3: uneven job and share counts), each rank running the
    C oracle on its slice, results all-gathered by exchange_var: every rank holds exactly the
    single-rank run's verdicts, statuses, error fields and combined signatures, byte for byte."""
    from oracle import bls_c
    roots, t, off, sigs, pks, ids, jr = _golden_global_batch()
    out, st, err, ver = bls_c.threshold_batch(off, t, b"".join(sigs), b"".join(pks), ids, jr, roots, 2, verify_all=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == list(range(world))
    if world == 3:
        assert len({r[1] for r in res}) > 1            # the shards really are uneven
    for _, _, v, sg, s, e in res:
        assert (v == ver[:off[-1]]).all()
        assert (s == st).all() and (e.astype("uint64") == err).all()
        assert (sg[s == 0] == out[st == 0]).all()
