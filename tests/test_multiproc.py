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
    # numpy (pickled by value): torch tensors go through fd sharing, which races with this
    # process's exit
    q.put((rank, [unpack_bits(bits[r], n).numpy() for r in range(world)], sigs.numpy().copy(), sts.numpy().copy(),
           ver.numpy(), sig.numpy(), st.numpy()))
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
            assert (vers[src] == res[src][4]).all()
            assert (sigs[src] == res[src][5]).all()
            assert (sts[src] == res[src][6]).all()


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


# ---- bench.py's own exchange step (BatchExchange): groups of pipelined batches, weak and strong ----
def _stub_global(N_jobs, n):
    """a deterministic 'engine' over a global batch: job j -> (status, sig bytes, err); share s -> verdict"""
    j = torch.arange(N_jobs)
    st = (j % 5 == 3).to(torch.int32) * 4
    sig = ((j.view(-1, 1) * 7 + torch.arange(96).view(1, -1)) % 251).to(torch.uint8)
    err = torch.stack([j % 3, j % 7], 1).to(torch.int64)
    s = torch.arange(N_jobs * n)
    ver = (s % 11 != 4).to(torch.uint8)
    return ver, sig, st, err


def _bx_worker(rank, world, port, q, strong):
    import torch.distributed as dist
    from safestakeoperator_amd.shard import BatchExchange, shard_jobs, shard_sizes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, J, G = 3, 41, 3                       # shares per job, global jobs, batches per group
    off = list(range(0, J * n + 1, n))
    gver, gsig, gst, gerr = _stub_global(J, n)
    if strong:
        j0, j1 = shard_jobs(off, world, rank)
        sizes = shard_sizes(off, world)
        loc = dict(ver=gver[j0 * n:j1 * n], out=gsig[j0:j1], st=gst[j0:j1], err=gerr[j0:j1])
    else:
        sizes = None
        loc = dict(ver=gver ^ (rank & 1), out=gsig + rank, st=gst + rank, err=gerr)
    bx = BatchExchange(strong=strong, sizes=sizes)
    outs = [{k: v.clone() for k, v in loc.items()} for _ in range(G)]
    for b in range(G):                       # the batches of one group differ in their statuses
        outs[b]["st"] = outs[b]["st"] + 10 * b
    bx.flush(outs)
    ok, res = bx.check_last()
    if strong:
        full = all(torch.equal(r[0], gver) and torch.equal(r[1], gsig) and torch.equal(r[2], gst + 10 * b)
                   and torch.equal(r[3], gerr) for b, r in enumerate(res))
    else:
        full = all(torch.equal(res[b][r][2], gst + r + 10 * b) and torch.equal(res[b][r][0], gver ^ (r & 1))
                   for b in range(G) for r in range(world))
    q.put((rank, bool(ok), bool(full)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("strong", [False, True], ids=["weak", "strong"])
def test_bench_batch_exchange_gloo_world2(strong):
    """The exchange step bench.py runs after each group of pipelined batches (shard.BatchExchange),
    driven with a stub batch function over gloo at world 2: a group of 3 batches per collective;
    weak -- every rank's gathered rows equal that rank's local outputs; strong (uneven 41-job global
    batch) -- every batch of the group reassembles to the single-rank global result."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bx_worker, args=(r, world, port, q, strong)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == [0, 1]
    assert all(r[1] and r[2] for r in res), res


# ---- bench.py's exchanger: the helper thread that issues each group's all-gather once the group's
# batches are done, in group order on every rank, drained before the main thread's own collectives ----
class _Done:
    """a stand-in for a recorded torch.cuda.Event: ready after `delay` seconds"""
    def __init__(self, delay):
        import time
        self.t = time.monotonic() + delay

    def synchronize(self):
        import time
        time.sleep(max(0.0, self.t - time.monotonic()))


def _exchanger_worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from safestakeoperator_amd.shard import BatchExchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, J, G, rounds = 3, 17, 4, 5
    gver, gsig, gst, gerr = _stub_global(J, n)
    ex = bench.Exchanger(BatchExchange(strong=False), None)
    ok = True
    futs = []
    for r in range(rounds):
        outs = [dict(ver=gver ^ ((rank + b) & 1), out=gsig + rank, st=gst + 100 * r + 10 * b + rank, err=gerr)
                for b in range(G)]
        # rank 1's batches "finish" later than rank 0's: the collectives must still pair up in group order
        futs.append((r, ex.submit([(o, _Done(0.02 * rank * (G - b))) for b, o in enumerate(outs)])))
    ex.drain()
    dist.barrier()                         # the main thread's own collective, after the drain
    for r, f in futs:
        for w in f.result(timeout=60):
            w.wait()
    ok_last, res = ex.xchg.check_last()    # the last group, every rank's rows
    ok = ok and ok_last and all(torch.equal(res[b][x][2], gst + 100 * (rounds - 1) + 10 * b + x)
                                for b in range(G) for x in range(world))
    ex.close()
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_exchanger_gloo_world2():
    """bench.Exchanger over gloo at world 2: five groups of four batches submitted with staggered
    completion times, drained, then a barrier; every group's collective pairs with the same group on the
    other rank (the last group's gathered statuses carry its round number), and nothing deadlocks."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchanger_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == [0, 1] and all(r[1] for r in res), res
