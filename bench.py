"""Benchmark: the threshold-BLS hot path on MI355X (BASELINE.json metric, config C2 per GPU).

One step = one ssb_threshold_aggregate_batch_dev pass over one batch resident in HBM:
  4,096 validators x 4 operator shares (3-of-4), 64 distinct signing roots  (BASELINE.json configs[1])
  = hash_to_G2 per root + verify every partial signature (RLC multi-pairing, exact fallback)
    + reference scan/selection + Lagrange combine + compress,
  and for N > 1 the per-batch RCCL all-gather of verdict bitmaps, statuses and combined signatures.
Scaling is weak: every rank runs its own C2 batch (distinct validators), no data-path collective.

Batches are independent (each is one slot's duties), so the engine keeps --pipeline of them in flight
(ssb_set_pipeline_depth: one set of streams and workspace per slot); every step still processes
one complete batch.  The single-batch latency (pipeline depth 1, synchronised after every batch)
and the per-kernel hipEvent timings are measured in a separate phase and reported beside the value.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pipeline S] [--validators V] [--no-cpu-baseline]
"""
import argparse
import ctypes
import hashlib
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

def set_hw_queues(n):
    """Hardware queues per process for the HIP runtime (read at HIP init, so before torch).  Each
    pipeline slot drives `slot_streams` streams and the engine two context streams; with HIP's
    default of 4 queues (the GPU box exports GPU_MAX_HW_QUEUES=4) independent batches serialise on
    shared queues.  Raised here, never lowered, never above 32."""
    n = max(16, min(32, n))
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < n:
        os.environ["GPU_MAX_HW_QUEUES"] = str(n)

DIST_QUEUES = 0   # hardware queues added for the process group's streams (RCCL) beside the slots (see main)

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
METRIC = "verified partial sigs/sec + combined threshold sigs/sec, 1 and 8 MI355X"
MAD_PEAK_MEASURED = 3.8235e13  # v_mad_u64_u32/s, profiles/r01_madpeak.json (16 chains, 4096 WGs)
MAD_PEAK_ISSUE = 256 * 4 * 16 * 2.4e9  # 16 lanes/clk/SIMD (wave64 mad = 4 cycles) x 1024 SIMDs x 2.4 GHz


# Per-GPU workloads of BASELINE.json's configs.  One step = one batch of the config.
#   C2  configs[1]: 4,096 validators x 4 shares (3-of-4), 64 roots -- the headline
#   C3  configs[2]: 65,536 validators, 3-of-4 and 5-of-7, one batch
#   C4  configs[3]: 1,048,576 attestation shares over 8 GPUs -> 131,072 shares (32,768 x 4) per GPU
#   C5  configs[4]: 1M validators x 13 shares (10-of-13) over 8 GPUs -> 131,072 validators per GPU
CONFIGS = {
    "C2": dict(validators=4096, threshold=3, operators=4, roots=64, pipeline=20),
    # C3 / C5 name a final verify: the step also verifies every combined signature against the
    # validator's master key (batched across validators by RLC, ssb_verify_batch_cached_dev)
    "C3_3of4": dict(validators=65536, threshold=3, operators=4, roots=64, pipeline=3, final_verify=True),
    "C3_5of7": dict(validators=65536, threshold=5, operators=7, roots=64, pipeline=3, final_verify=True),
    "C4_per_gpu": dict(validators=32768, threshold=3, operators=4, roots=64, pipeline=4),
    "C5_per_gpu": dict(validators=131072, threshold=10, operators=13, roots=64, pipeline=2, final_verify=True),
    # ONE global batch of 1,048,576 shares split over the ranks (--scaling strong)
    "C4_global": dict(validators=262144, threshold=3, operators=4, roots=64, pipeline=2),
}


def opcount_mads():
    with open(os.path.join(ROOT, "bench_tools", "opcount.json")) as f:
        oc = json.load(f)
    return {k: 300.0 * (v["fp_mul"] + v["fp_sqr"]) + 136.0 * v["fr_mul"] for k, v in oc.items() if isinstance(v, dict)}


def msm_plan(N, n_roots):
    """The window widths / bucket teams of the RLC bucket MSMs (plan_msm in csrc/ssbls.hip)."""
    def pick_c(n, g, cmin, cmax):
        best = None
        for c in range(cmin, cmax + 1):
            W, B = (64 + c - 1) // c, 2 ** c
            L = min(B, 64)
            reduce = 2 * (B - 1) if c <= 4 else 2 * B + L * (math.log2(L) + 1)
            cost = n * W * (1 - 1 / B) + 1.5 * g * W * reduce
            if best is None or cost < best[0]:
                best = (cost, c)
        return best[1]

    def pick_lj(n, g, c):
        pb, lj = n / (g * 2 ** c), 0
        while lj < 6 and pb / 2 ** (lj + 1) >= 8:
            lj += 1
        return lj
    g1n = max(n_roots, 1)
    c2, c1 = pick_c(N, 1, 3, 8), pick_c(N, g1n, 2, 8)
    keys = lambda c, g: ((64 + c - 1) // c) * g * 2 ** c
    while c1 > 2 and keys(c2, 1) + keys(c1, g1n) > 1024 * 1024:
        c1 -= 1
    return {"c2": c2, "W2": (64 + c2 - 1) // c2, "lj2": pick_lj(N, 1, c2),
            "c1": c1, "W1": (64 + c1 - 1) // c1, "lj1": pick_lj(N, g1n, c1), "groups1": g1n,
            "g1_msm": N >= 128 * g1n}


def msm_mads(mads, N, c, W, lj, groups, g):
    """MADs of one bucket MSM launch sequence (curve g = "g1"/"g2"): entry madds, bucket-team
    trees, window reduce (running sums, suffix scan, lane doublings, tree), to-affine/Horner."""
    B, L = 2 ** c, min(2 ** c, 64)
    m = B // L
    madd, add, dbl = mads["madd_" + g], mads["sum_%s_add" % g], mads["dbl_" + g]
    entries = N * W * (1 - 1 / B)
    trees = groups * W * B * ((1 << lj) - 1) * add
    scan = sum(L - off for off in (2 ** i for i in range(int(math.log2(L))))) if L > 1 else 0
    if g == "g1" and c <= 4:
        window = groups * W * 2 * (B - 1) * add
    else:
        window = groups * W * ((L * (2 * (m - 1) + 1) + scan + (L - 1)) * add + (L - 1) * math.log2(m) * dbl
                               + (L - 1) * add)
    return entries * madd + trees + window


def kernel_mads(mads, V, t, n, n_roots, pk_cached=True):
    """Algorithmic MADs per launch of each kernel (per-unit counts x units per launch).  With the
    public-key cache the per-batch decode is the signatures only."""
    N = V * n
    p = msm_plan(N, n_roots)
    small = mads["combine_small_t3"] if t <= 3 else (mads["combine_small_t5"] if t <= 5 else mads["combine_small_t10"])
    npairs = n_roots + p["W2"]
    if pk_cached and p["g1_msm"]:
        # the merged G1 MSM over the cache's precomputed bases (plan_msm g1_pre): 16 entries per share
        # into the root's 16 buckets, one 15-bucket running sum per root, no Horner
        g1n, lj1 = p["groups1"], 0
        while lj1 < 6 and N / g1n / 2 ** (lj1 + 1) >= 8:
            lj1 += 1
        g1 = (N * 16 * (1 - 1 / 16) * mads["madd_g1"] + g1n * 16 * ((1 << lj1) - 1) * mads["sum_g1_add"]
              + g1n * (2 * 14 * mads["sum_g1_add"] + mads["to_affine_g1"]))
    else:
        g1 = (msm_mads(mads, N, p["c1"], p["W1"], p["lj1"], p["groups1"], "g1")
              + p["groups1"] * ((p["W1"] - 1) * (p["c1"] * mads["dbl_g1"] + mads["sum_g1_add"]) + mads["to_affine_g1"]))
    return {
        "k_hash_to_g2": n_roots * mads["hash_to_g2"],
        "k_decode": N * (mads["decode_sig"] + (0.0 if pk_cached else mads["decode_pk"])),
        "k_subgroup": N * mads["subgroup"],
        "k_msm_g2": msm_mads(mads, N, p["c2"], p["W2"], p["lj2"], 1, "g2") + p["W2"] * mads["to_affine_g2"],
        "k_msm_g1": g1 if p["g1_msm"] else 0.0,
        "k_rlc_pk": 0.0 if p["g1_msm"] else N * mads["rlc_pk"],
        "k_sum_g1": 0.0 if p["g1_msm"] else N * mads["sum_g1_add"] + n_roots * mads["to_affine_g1"],
        "k_miller": npairs * mads["miller_pair"],
        "k_final": (npairs - 1) * mads["fp12_mul"] + mads["final_exp"],
        "k_combine_fast": V * small,   # ids 1..n: integer Lagrange coefficients (ssb_units.h)
    }


def valu_per_mad(sq, mads):
    """SQ_INSTS_VALU of the roofline launch (committed PMC summary: instructions per wave x waves) per
    64 algorithmic MADs (one wave-instruction's worth), or None."""
    try:
        rb = sq["roofline_batch"]
        return round(rb["valu_insts_per_wave"] * rb["SQ_WAVES"] / (mads / 64.0), 3)
    except (KeyError, TypeError, ZeroDivisionError):
        return None


def pmc_traffic(kernel, shares=None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (FETCH_SIZE x 2 on
    gfx950 + WRITE_SIZE, separate passes; bench_tools/pmc_summary.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(kernel, {})
        if shares and e.get("hbm_bytes_per_share"):   # measured on one batch size, scaled per share
            return round(e["hbm_bytes_per_share"] * shares)
        return e.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def make_workload(engine, V, t, n, n_roots, rank, invalid_rate=0.0, invalid_count=0, v0=0, bad_operator=0, ids="seq"):
    """Synthetic committees: deterministic keys (seed 0x5AFE57A4E, rank), Shamir shares, partial
    signatures from the engine's batched signer (H(m)*sk), public keys sk*g1.  invalid_rate: that
    fraction of the shares (deterministic choice) signs the NEXT root instead -- a valid G2 point
    that fails verification (SURVEY.md §8d C2/C4 invalid variants).  v0: index of the first
    validator (a rank's shard of one global batch: validators v0 .. v0+V-1 of seed `rank`).
    bad_operator: every share of the operator with that id is invalid (a faulty / malicious operator,
    the reference skips and logs its shares: generic_threshold.rs:166-168).
    ids: "seq" -- operator ids 1..n in every committee (the reference's tests and DKG helper); "registry"
    -- n distinct pseudo-random ids in [1, 2^16) per committee, as registry operator ids arrive from the
    contract (src/node/node.rs:470-474, validator.releated_operators)."""
    seed = b"ssbls-bench" + (0x5AFE57A4E).to_bytes(8, "little") + rank.to_bytes(4, "little")
    roots = [hashlib.sha256(seed + b"root" + i.to_bytes(4, "little")).digest() for i in range(n_roots)]

    def h(*parts):
        return int.from_bytes(hashlib.sha256(seed + b"".join(parts)).digest(), "little") % R_ORDER

    import numpy as np
    # Shamir shares by Horner over r, vectorised over validators (object arrays of Python ints)
    coef = np.empty((V, t), dtype=object)
    for v in range(V):
        vb = (v0 + v).to_bytes(4, "little")
        coef[v, 0] = h(b"sk", vb)
        for k in range(1, t):
            coef[v, k] = h(b"c", vb, k.to_bytes(4, "little"))
    master = coef[:, 0].tolist()
    if ids == "registry":
        idm = np.empty((V, n), dtype=object)
        for v in range(V):
            vb = (v0 + v).to_bytes(4, "little")
            got, k = [], 0
            while len(got) < n:
                x = 1 + int.from_bytes(hashlib.sha256(seed + b"id" + vb + k.to_bytes(4, "little")).digest()[:4], "little") % 65535
                if x not in got:
                    got.append(x)
                k += 1
            idm[v, :] = got
    else:
        idm = np.asarray([list(range(1, n + 1))] * V, dtype=object)
    shares = np.empty((V, n), dtype=object)
    for i in range(n):
        x = idm[:, i]
        acc = coef[:, t - 1].copy()
        for k in range(t - 2, -1, -1):
            acc = (acc * x + coef[:, k]) % R_ORDER
        shares[:, i] = acc
    share_sk = shares.reshape(-1).tolist()
    ids = [int(x) for x in idm.reshape(-1).tolist()]
    jr = [(v0 + v) % n_roots for v in range(V)]
    share_root = [r for r in jr for _ in range(n)]
    bad = [i for i in range(len(share_sk))
           if invalid_rate > 0 and int.from_bytes(hashlib.sha256(seed + b"bad" + (v0 * n + i).to_bytes(4, "little")).digest()[:8],
                                                   "little") < invalid_rate * 2.0 ** 64]
    if invalid_count:                                  # exactly that many, spread over the batch
        N = len(share_sk)
        bad = sorted(set(bad) | {(k * (N // invalid_count) + 4099 * (k + 1)) % N for k in range(invalid_count)})
    if bad_operator:                                   # every share of that operator id
        bad = sorted(set(bad) | {i for i, x in enumerate(ids) if x == bad_operator})
    sign_root = list(share_root)
    for i in bad:
        sign_root[i] = (share_root[i] + 1) % n_roots
    sigs = engine.sign_batch(share_sk, sign_root, roots)
    pks = engine.sk_to_pk_batch(share_sk)
    valid = [1] * len(share_sk)
    for i in bad:
        valid[i] = 0
    return dict(roots=roots, sigs=b"".join(sigs), pks=b"".join(pks), ids=ids, job_root=jr, master=master,
                share_sigs=sigs, share_pks=pks, valid=valid, n_bad=len(bad), share_sk=share_sk, sign_root=sign_root)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(wl, t, n, gpu_out=None, n_val=4096, n_val_share=1024, threads=None, reps=5):
    """The plain-C oracle (oracle/bls_c.c, multi-threaded, `kind: "port"`) on a bounded sample of
    the same workload, H(root) once per root, two columns ("per-signature verify and
    RLC batch, both reported"), each the MEDIAN of `reps` (>= 5) whole passes:
      * rlc (the `value`): the batch-verify algorithm family the engine and lighthouse's
        verify_signature_sets use -- per share decompress + subgroup check + 64-bit [k]pk, [k]sig,
        one multi-pairing and one final exponentiation, then the integer-Lagrange combine -- over the
        first n_val validators x n shares of rank 0's batch;
      * per_share: every share verified on its own (2 Miller loops + final exponentiation each,
        the reference's loop at generic_threshold.rs:149-169), 255-bit Lagrange combine, over the
        first n_val_share validators.
    Threads: the GPU box's CPU share (16 per GPU), fewer if the host has fewer.  Both columns are
    checked against the GPU's combined signatures for the same validators."""
    from oracle import bls_c
    threads = threads or max(1, min(16, os.cpu_count() or 1))
    bls_c.load()

    def args_for(nv):
        N = nv * n
        return (list(range(0, N + 1, n)), [t] * nv, wl["sigs"][:96 * N], wl["pks"][:48 * N], wl["ids"][:N],
                wl["job_root"][:nv], wl["roots"], threads)

    def median_time(fn, k):
        ts, res = [], None
        for _ in range(k):
            t0 = time.perf_counter()
            res = fn()
            ts.append(time.perf_counter() - t0)
        return res, sorted(ts)[len(ts) // 2], ts

    a_rlc, a_share = args_for(n_val), args_for(n_val_share)
    (out, st, _, ver, batch_ok), dt_rlc, ts_rlc = median_time(lambda: bls_c.threshold_batch_rlc(*a_rlc), reps)
    (out2, st2, _, ver2), dt_share, ts_share = median_time(lambda: bls_c.threshold_batch(*a_share, verify_all=True), reps)
    N, N2 = n_val * n, n_val_share * n
    ok = bool((st == 0).all()) and bool(ver[:N].all()) and batch_ok and bool((st2 == 0).all()) and bool(ver2[:N2].all())
    if gpu_out is not None:
        ok = ok and all(out[v].tobytes() == gpu_out[v].tobytes() for v in range(n_val))
        ok = ok and all(out2[v].tobytes() == gpu_out[v].tobytes() for v in range(n_val_share))
    return dict(value=round(N / dt_rlc, 1), unit="partial_sigs/s", cores=threads, kind="port", cpu_model=cpu_model(),
                per_core=round(N / dt_rlc / threads, 1), combined_per_s=round(n_val / dt_rlc, 1),
                seconds=round(dt_rlc, 3), matches_gpu=bool(ok), repetitions=reps, statistic="median",
                per_share=dict(value=round(N2 / dt_share, 1), per_core=round(N2 / dt_share / threads, 1),
                               combined_per_s=round(n_val_share / dt_share, 1), seconds=round(dt_share, 3)),
                sample="rlc: %d validators x %d shares of the rank-0 C2 batch (batch verify + %d-of-%d combine); "
                       "per_share: the first %d validators (every share verified on its own); median of %d whole "
                       "passes each; H(root) once per root; oracle/bls_c.c (plain C, 64-bit limbs), %d threads"
                       % (n_val, n, t, n, n_val_share, reps, threads),
                seconds_total=round(sum(ts_rlc) + sum(ts_share), 2))


class Exchanger:
    """The helper thread of exchange_group: for each group in submission order, wait (on the host)
    for the group's batch events, then issue its all-gather (BatchExchange.flush) -- the same order
    on every rank, and drain() before any other collective (barrier, all_reduce) of the main
    thread.  submit() returns a Future of the collective's handles."""

    def __init__(self, xchg, dev):
        import queue
        import threading
        self.xchg, self.dev = xchg, dev
        self.q = queue.Queue()
        self.t = threading.Thread(target=self._run, name="bench-exchange", daemon=True)
        self.t.start()

    def submit(self, items):
        from concurrent.futures import Future
        fut = Future()
        self.q.put((items, fut))
        return fut

    def _run(self):
        import torch
        if self.dev is not None and getattr(self.dev, "type", "cpu") == "cuda":
            torch.cuda.set_device(self.dev)
        while True:
            job = self.q.get()
            try:
                if job is None:
                    return
                items, fut = job
                try:
                    for _, ev in items:
                        ev.synchronize()
                    fut.set_result(self.xchg.flush([o for o, _ in items]))
                except BaseException as e:  # noqa: BLE001 (re-raised by the main thread's job.result())
                    fut.set_exception(e)
            finally:
                self.q.task_done()

    def drain(self):
        self.q.join()

    def close(self):
        self.q.put(None)
        self.t.join()


def launch_command(n, argv, port):
    """The torch.distributed.run command bench.py --gpus N runs itself when no launcher set WORLD_SIZE."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    # the ranks' stdout through a pipe: rank 0's JSON line stays on stdout, anything else the launcher
    # or a backend prints there (gloo's "[Gloo] Rank ... connected" lines) goes to stderr
    p = subprocess.Popen(launch_command(n, argv, port), stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return p.wait()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (200 steps by default: with 20 batches in flight a short run is dominated by the pipeline's
    # drain -- the last batch's whole latency inside the timed region; 48 steps measured 12.0-12.8 M
    # where 200 measured 14.2-14.6 M on the same build, round 4)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="BASELINE.json workload per GPU (the headline is C2; the others are reported under profiles/); "
                         "default C2, or C4_global with --scaling strong")
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="weak: every rank runs its own batch (the headline); strong: ONE global batch (C4_global: "
                         "1,048,576 shares) split over the ranks by shard_jobs, results all-gathered back in order")
    ap.add_argument("--validators", type=int, default=None)
    ap.add_argument("--threshold", type=int, default=None)
    ap.add_argument("--operators", type=int, default=None)
    ap.add_argument("--roots", type=int, default=None)
    ap.add_argument("--pipeline", type=int, default=None, help="independent batches in flight (engine pipeline slots)")
    ap.add_argument("--slot-streams", type=int, default=1, choices=(1, 3),
                    help="streams per slot (1: batch in order on one queue; 3: hash / G1 side overlapped)")
    ap.add_argument("--final-verify", dest="final_verify", action="store_true", default=None,
                    help="each step also verifies the combined signatures against the master keys (a-8); "
                         "default on for the C3 / C5 configs, which name it")
    ap.add_argument("--no-final-verify", dest="final_verify", action="store_false")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-buffers", action="store_true", help="skip the PCIe-inclusive host-buffer run")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (RCCL, the measured path) or gloo (rehearsal: ranks may share a GPU)")
    ap.add_argument("--compressed-pk", action="store_true",
                    help="headline on the compressed-public-key entry point (default: keys decompressed once, "
                         "ssb_pk_cache_set, as lighthouse's PublicKey holds them; the other variant is reported beside)")
    ap.add_argument("--invalid-count", type=int, default=0,
                    help="exactly this many invalid shares per batch (e.g. 2 ~ C4's 1e-4 rate at C2 size)")
    ap.add_argument("--invalid-rate", type=float, default=0.0,
                    help="fraction of shares signed over the wrong root (the RLC batch fails; exact verdicts "
                         "come from the per-share fallback).  The headline is the all-valid C2 batch.")
    ap.add_argument("--bad-operator", type=int, default=0,
                    help="every share of the operator with this id is invalid (a faulty operator in every committee)")
    ap.add_argument("--ids", default="seq", choices=("seq", "registry"),
                    help="operator ids: 1..n per committee (seq), or distinct pseudo-random registry ids in [1, 2^16) "
                         "per committee (registry, src/node/node.rs:470-474)")
    ap.add_argument("--no-registry", dest="registry_leg", action="store_false",
                    help="skip the registry-operator-id leg (value_registry: the same path and --steps, ids from "
                         "the registry contract instead of 1..n)")
    ap.add_argument("--no-adversarial", dest="adversarial_legs", action="store_false",
                    help="skip the adversarial legs (value_invalid_1e2, value_bad_operator: the same path and --steps "
                         "with 1%% of the shares invalid / one faulty operator in every committee)")
    ap.add_argument("--sustained-steps", type=int, default=1000,
                    help="length of the sustained-rate run reported as value_sustained (0: skip)")
    ap.add_argument("--collector-windows", type=int, default=200,
                    help="4,096-job windows pushed through the native per-slot collector for value_collector (0: skip)")
    ap.add_argument("--collector-threads", type=int, default=8, help="native submitter threads of value_collector")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="GPU_MAX_HW_QUEUES for this process (default: pipeline x slot streams + 3, + %d with "
                         "torch.distributed; at most 32)" % DIST_QUEUES)
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the process group even at one rank (rehearses RCCL's stream beside the slot "
                         "queues on one GPU: torchrun --nproc-per-node 1 ... --force-dist)")
    args = ap.parse_args()
    # --gpus N without an external launcher: start the N ranks here, BEFORE anything touches the GPU
    # (this process only waits for them), one process per GPU over RCCL, and exit with their status
    if os.environ.get("WORLD_SIZE") is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if os.environ.get("WORLD_SIZE") is not None and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d" % (os.environ["WORLD_SIZE"], args.gpus), file=sys.stderr)
        sys.exit(2)
    if args.config is None:
        args.config = "C4_global" if args.scaling == "strong" else "C2"
    strong = args.scaling == "strong"
    preset = CONFIGS[args.config]
    for k in ("validators", "threshold", "operators", "roots", "pipeline"):
        if getattr(args, k) is None:
            setattr(args, k, preset[k])
    if args.final_verify is None:
        args.final_verify = bool(preset.get("final_verify", False))
    # Hardware queues: every ACTIVE engine stream needs its own, and past 20 the firmware
    # time-slices them.  Measured C2 at the driver's 20 steps, one-stream slots, each batch wholly on
    # its slot's stream (hash_to_G2, verdicts and combine too): 19 slots 7.18 M sigs/s (the 20th
    # batch waits for a slot), 20 slots 9.33 M (every batch in flight at once), 21 slots 6.51 M,
    # 20 slots + 2 hash streams 4.05 M.  With N > 1 the all-gather runs on RCCL's stream: it is
    # issued once per pipeline round (exchange_group), after the round's batches, so that stream is
    # not active beside the 20 slot queues.
    # slot streams + the context's speculative-combine and tail streams (idle with one-stream slots,
    # which run every stage on the slot's stream) + one for torch; with torch.distributed, room for
    # the process group's streams too (RCCL at N = 1 with no room: two slots shared a queue, 9.36 M
    # against 12.27 M without the process group, round 5)
    dist_run = int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.force_dist
    set_hw_queues(args.hw_queues or (args.pipeline * args.slot_streams + 3 + (DIST_QUEUES if dist_run else 0)))

    import numpy as np
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # --dist-backend gloo: rehearsal of the N > 1 path on fewer GPUs than ranks (ranks share
    # devices round robin, the collectives run on host copies); the measured path is RCCL.
    gpu = local % max(1, torch.cuda.device_count()) if args.dist_backend == "gloo" else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")   # where collectives run
    local = gpu

    # the library (a no-op when the in-tree build is current); ranks of one node take turns
    import fcntl
    from safestakeoperator_amd.build import build
    with open(os.path.join(ROOT, ".bench_build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        build(verbose=False)
    from safestakeoperator_amd import Engine, DST
    from safestakeoperator_amd import _lib

    V, t, n, n_roots = args.validators, args.threshold, args.operators, args.roots
    V_glob = V * (1 if strong else world)             # validators of the whole job (all ranks)
    S = max(1, args.pipeline)
    if args.dist_backend == "gloo" and world > 1:
        # rehearsal with ranks sharing GPUs: the GPU's slot queues are split between its ranks (each
        # slot is a hardware queue with its own scratch reservation; 24 on one GPU exhausted it)
        per_gpu = -(-world // max(1, torch.cuda.device_count()))
        S = max(1, S // per_gpu)
    eng = Engine(local)
    from safestakeoperator_amd.shard import BatchExchange, shard_jobs, shard_sizes
    sizes = None
    if strong:
        # this rank's contiguous, share-balanced slice of the ONE global batch (seed of rank 0, so the
        # data of validator v does not depend on the number of ranks)
        goff = list(range(0, V * n + 1, n))
        j0, j1 = shard_jobs(goff, world, rank)
        sizes = shard_sizes(goff, world)
        V = j1 - j0
        wl = make_workload(eng, V, t, n, n_roots, 0, args.invalid_rate, args.invalid_count, v0=j0,
                           bad_operator=args.bad_operator, ids=args.ids)
    else:
        wl = make_workload(eng, V, t, n, n_roots, rank, args.invalid_rate, args.invalid_count,
                           bad_operator=args.bad_operator, ids=args.ids)
    N = V * n
    valid = np.asarray(wl["valid"], dtype=np.uint8)
    job_ok = valid.reshape(V, n).sum(axis=1) >= t

    # inputs resident in HBM before the timed region
    def dt8(b):
        return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    d_sig = dt8(wl["sigs"])
    d_pk = dt8(wl["pks"])
    d_ids = torch.tensor(wl["ids"], dtype=torch.int64, device=dev)
    d_off = torch.arange(0, N + 1, n, dtype=torch.int32, device=dev)
    d_t = torch.full((V,), t, dtype=torch.int32, device=dev)
    d_jr = torch.tensor(wl["job_root"], dtype=torch.int32, device=dev)
    d_roots = dt8(b"".join(wl["roots"]))
    def out_set():
        return dict(out=torch.empty((V, 96), dtype=torch.uint8, device=dev), st=torch.empty((V,), dtype=torch.int32, device=dev),
                    err=torch.empty((V, 2), dtype=torch.int64, device=dev), ver=torch.empty((N,), dtype=torch.uint8, device=dev),
                    fv=torch.empty((V,), dtype=torch.uint8, device=dev))
    # with a process group every slot alternates between TWO output sets: a batch's results are all-
    # gathered while the slot's next batch writes the other set (exchange_group)
    out_sets = [[out_set(), out_set()] if dist_run else [out_set()] for _ in range(S)]
    sel = [0] * S                                   # the set slot k's last batch wrote
    outs = [o[0] for o in out_sets]                 # slot k's last batch's outputs
    dst_arr = (ctypes.c_uint8 * len(DST)).from_buffer_copy(DST)
    lib = eng._lib
    seed_base = 0x5AFE57A4E ^ (rank << 40)

    streams = {}
    pending = {}    # id(output set) -> the exchange job (all-gather handles) reading that set

    # validator registration (outside the timed region): every operator key decompressed once, and
    # with the final verify the validators' master keys after them (table rows N .. N+V-1)
    mpks = b"".join(eng.sk_to_pk_batch(wl["master"])) if args.final_verify else b""
    pk_host = np.frombuffer(wl["pks"] + mpks, dtype=np.uint8)
    if lib.ssb_pk_cache_set(eng.handle, N + (V if args.final_verify else 0), pk_host.ctypes.data_as(_lib._u8p)) != 0:
        raise RuntimeError("ssb_pk_cache_set: %s" % lib.ssb_last_error(eng.handle))
    d_pkidx = torch.arange(0, N, dtype=torch.int32, device=dev)
    d_midx = torch.arange(N, N + V, dtype=torch.int32, device=dev)
    d_mpk = dt8(mpks) if args.final_verify else None
    use_cache = [not args.compressed_pk]

    # host-buffer variant (reported beside the headline, never the value): every batch's inputs
    # start in ordinary host memory and its results end there, PCIe inclusive -- through the
    # library's asynchronous host entry point (ssb_threshold_aggregate_batch[_cached]_submit /
    # ssb_batch_wait): one host memcpy into the slot's pinned, device-mapped staging buffer, the
    # kernels read it and write their outputs in place over PCIe, the outputs are delivered when the
    # batch is waited for; up to S batches in flight
    use_host = [False]
    host_io = {}                                   # slot -> the PendingBatch last submitted on it
    h_in = dict(off=np.arange(0, N + 1, n, dtype=np.uint32), t=np.full(V, t, dtype=np.uint32),
                sig=np.frombuffer(wl["sigs"], dtype=np.uint8), pk=np.frombuffer(wl["pks"], dtype=np.uint8),
                pkidx=np.arange(0, N, dtype=np.uint32), ids=np.asarray(wl["ids"], dtype=np.uint64),
                jr=np.asarray(wl["job_root"], dtype=np.uint32), roots=np.frombuffer(b"".join(wl["roots"]), dtype=np.uint8))

    def step(i, k):
        """batch i on pipeline slot k (engine slot k, output buffers k); the caller's stream is the
        slot's own main stream (ssb_slot_stream), so the bench adds no hardware queue"""
        sel[k] = (sel[k] + 1) % len(out_sets[k])
        o = outs[k] = out_sets[k][sel[k]]
        if k not in streams:
            streams[k] = torch.cuda.ExternalStream(lib.ssb_slot_stream(eng.handle, k), device=dev)
        s = streams[k]
        fn = lib.ssb_threshold_aggregate_batch_cached_dev if use_cache[0] else lib.ssb_threshold_aggregate_batch_dev
        pk_arg = d_pkidx if use_cache[0] else d_pk
        src = inputs
        if use_host[0]:   # (world == 1 only; the library picks slot k round robin like the _dev calls)
            host_io[k] = eng.submit_batch_raw(h_in["t"], h_in["off"], h_in["sig"], h_in["pk"], h_in["ids"], h_in["jr"],
                                              h_in["roots"], seed=(seed_base + i) & (2 ** 64 - 1),
                                              pk_index=h_in["pkidx"] if use_cache[0] else None)
            return
        # this output set is rewritten by this batch: order it after the all-gather that read it (two
        # batches of this slot ago: issued long since, so neither the host nor the stream waits in
        # practice -- a stream wait on RCCL's event)
        job = pending.pop(id(o), None)
        if job is not None:
            for w in job.result():
                with torch.cuda.stream(s):
                    w.wait()
        # (the argument tuple of slot k is built once: the timed loop's host time per submit is the
        # library's, not Python's -- the last batch of a round starts that much later)
        key = (k, sel[k], use_cache[0], s.cuda_stream, inputs["gen"])
        a = call_args.get(key)
        if a is None:
            a = call_args[key] = (
                (eng.handle, V, N, d_off.data_ptr(), d_t.data_ptr(), src["d_sig"].data_ptr(), pk_arg.data_ptr(),
                 src["d_ids"].data_ptr(), src["d_jr"].data_ptr(), n_roots, src["d_roots"].data_ptr(),
                 ctypes.cast(dst_arr, _lib._u8p), len(DST)),
                (o["out"].data_ptr(), o["st"].data_ptr(), o["err"].data_ptr(), o["ver"].data_ptr(), ctypes.c_void_p(s.cuda_stream)))
        rc = fn(*a[0], (seed_base + i) & (2 ** 64 - 1), *a[1])
        if rc != 0:
            raise RuntimeError("ssb_threshold_aggregate_batch_dev: %s" % lib.ssb_last_error(eng.handle))
        if True:
            if args.final_verify:
                # a-8: every combined signature against its validator's master key, same slot and
                # stream, after the combine (a job that did not combine holds zero bytes: verdict 0)
                vfn = lib.ssb_verify_batch_cached_dev if use_cache[0] else lib.ssb_verify_batch_dev
                mk = d_midx if use_cache[0] else d_mpk
                rc = vfn(eng.handle, V, mk.data_ptr(), o["out"].data_ptr(), src["d_jr"].data_ptr(), n_roots,
                         src["d_roots"].data_ptr(), ctypes.cast(dst_arr, _lib._u8p), len(DST),
                         (seed_base + i + (1 << 32)) & (2 ** 64 - 1), o["fv"].data_ptr(), ctypes.c_void_p(s.cuda_stream))
                if rc != 0:
                    raise RuntimeError("ssb_verify_batch_cached_dev: %s" % lib.ssb_last_error(eng.handle))
        group.append(k)
        if len(group) >= S:
            exchange_group()

    call_args = {}  # per (slot, key variant, input generation): the submit call's fixed arguments
    inputs = dict(d_sig=d_sig, d_ids=d_ids, d_jr=d_jr, d_roots=d_roots, gen=0)   # the batch step() submits
    group = []      # slots whose results are not exchanged yet
    xchg = None     # the process group's exchange (phase 2; phases 1 / 1b run before the group exists)
    exchanger = None   # its helper thread

    def exchange_group():
        """RCCL all-gather over xGMI of the results of the batches since the last exchange, ONE
        collective per array for the group (fewer, larger collectives).  Issued by a helper thread
        (exchanger) once the group's batches have FINISHED -- an event per slot, waited on the host
        -- so no GPU queue sits blocked on them: round 5 issued it at once, with RCCL's stream and
        one slot stream waiting on the whole group, and the 1,000-step sustained rate at N = 1 fell to
        0.76x of the run without the process group (profiles/r05_rccl_n1.json): a stream blocked on a
        barrier still holds its hardware queue, and past ~20 active queues the firmware time-slices
        them.  The slot's next batch writes its OTHER output set, so the main thread never waits for
        the exchange; the batch after it, which rewrites this set, waits (a stream wait) for the
        all-gather that read it.  Weak scaling: every rank's own batch (shard.exchange); strong: this
        rank's shard of the one global batch, reassembled per batch in the global order
        (shard.exchange_var)."""
        if dist is None or not group:
            group.clear()
            return
        items = []
        for k in group:
            ev = torch.cuda.Event()
            ev.record(streams[k])
            items.append((outs[k], ev))
        job = exchanger.submit(items)
        for o, _ in items:
            pending[id(o)] = job
        group.clear()

    # phase 1: single-batch latency and per-kernel times (depth 1, no overlap between batches)
    # (latency configuration: 3 streams per slot, hash_to_G2 and the G1 side beside the main chain)
    # (the single-batch latency is timed without the per-stage hipEvents, in both slot forms -- three
    # streams, and the one-stream fused path the throughput run uses -- and batch_latency_ms is the
    # faster; the per-stage times come from three more batches with the events on)
    def one_batch_latency(n_streams):
        if lib.ssb_set_pipeline_depth(eng.handle, 1) != 0 or lib.ssb_set_slot_streams(eng.handle, n_streams) != 0:
            raise RuntimeError("ssb_set_pipeline_depth / ssb_set_slot_streams")
        # (reconfiguring the slots destroys their streams: no cached handle of an old one may be
        # passed as the caller's stream -- a use after free that crashed a run under rocprofv3, round 5)
        streams.clear()
        call_args.clear()
        step(0, 0)
        exchange_group()
        torch.cuda.synchronize(dev)
        lat = []
        for i in range(3):
            t0 = time.perf_counter()
            step(1 + i, 0)
            exchange_group()
            torch.cuda.synchronize(dev)
            lat.append(time.perf_counter() - t0)
        return sorted(lat)[1] * 1e3
    latency_by_config = {"one_stream_slot": round(one_batch_latency(1), 3),
                         "three_stream_slot": round(one_batch_latency(3), 3)}
    eng.kernel_timing(True)
    for i in range(3):
        step(1 + i, 0)
        exchange_group()
        torch.cuda.synchronize(dev)
    kt = {k: eng.kernel_time(k) for k in ["k_hash_to_g2", "k_decode", "k_subgroup", "k_msm_sort", "k_msm_g2",
                                         "k_msm_g1", "k_rlc_pk", "k_sum_g1", "k_miller", "k_final",
                                         "k_fallback_verify", "k_select", "k_combine_fast", "k_lagrange",
                                         "k_combine_terms", "k_combine_sum"]}
    eng.kernel_timing(False)
    latency_ms = min(latency_by_config.values())

    # phase 1b: the roofline of the headline path's dominant kernel, k_subgroup_map (the fused
    # one-stream path's subgroup checks, + the SWU map of the roots and the MSM sort's scatter
    # riding along), and of k_decode_count, measured where the kernel fills the chip: a one-stream
    # slot at depth 1 running ONE batch of R x the C2 batch (R = 8: 131,072 shares = 2,048 waves, two
    # per SIMD -- the occupancy the kernel is built for).  The C2 batch alone is 256 waves on 1,024
    # SIMDs; the pipelined run fills the chip with 20 of them, where per-launch times are shared.
    rf = None
    if not strong and not args.compressed_pk:
        R = 8
        rf_in = dict(sig=d_sig.repeat(R), pk=d_pkidx.repeat(R), ids=d_ids.repeat(R),
                     off=torch.arange(0, R * N + 1, n, dtype=torch.int32, device=dev),
                     t=torch.full((R * V,), t, dtype=torch.int32, device=dev), jr=d_jr.repeat(R))
        rf_out = dict(out=torch.empty((R * V, 96), dtype=torch.uint8, device=dev),
                      st=torch.empty((R * V,), dtype=torch.int32, device=dev),
                      err=torch.empty((R * V, 2), dtype=torch.int64, device=dev),
                      ver=torch.empty((R * N,), dtype=torch.uint8, device=dev))
        if lib.ssb_set_slot_streams(eng.handle, 1) != 0 or lib.ssb_set_pipeline_depth(eng.handle, 1) != 0:
            raise RuntimeError("ssb_set_slot_streams / ssb_set_pipeline_depth")
        rs = torch.cuda.ExternalStream(lib.ssb_slot_stream(eng.handle, 0), device=dev)

        def rf_step(i):
            rc = lib.ssb_threshold_aggregate_batch_cached_dev(
                eng.handle, R * V, R * N, rf_in["off"].data_ptr(), rf_in["t"].data_ptr(), rf_in["sig"].data_ptr(),
                rf_in["pk"].data_ptr(), rf_in["ids"].data_ptr(), rf_in["jr"].data_ptr(), n_roots, d_roots.data_ptr(),
                ctypes.cast(dst_arr, _lib._u8p), len(DST), (seed_base + 7777 + i) & (2 ** 64 - 1),
                rf_out["out"].data_ptr(), rf_out["st"].data_ptr(), rf_out["err"].data_ptr(), rf_out["ver"].data_ptr(),
                ctypes.c_void_p(rs.cuda_stream))
            if rc != 0:
                raise RuntimeError("roofline batch: %s" % lib.ssb_last_error(eng.handle))
        rf_step(0)
        torch.cuda.synchronize(dev)
        eng.kernel_timing(True)
        for i in range(3):
            rf_step(1 + i)
        torch.cuda.synchronize(dev)
        rf = {k: eng.kernel_time(k) for k in ("k_subgroup", "k_decode")}
        eng.kernel_timing(False)
        rf_ok = (bool(((rf_out["st"].cpu().numpy() == 0) == np.tile(job_ok, R)).all())
                 and bool((rf_out["ver"].cpu().numpy() == np.tile(valid, R)).all()))
        rf = dict(R=R, shares=R * N, ok=rf_ok, ms={k: (v[0] / v[1] if v[1] else 0.0) for k, v in rf.items()})
        del rf_in, rf_out

    # phase 2: the timed run, S batches in flight
    # (throughput configuration: S slots of args.slot_streams streams)
    if lib.ssb_set_slot_streams(eng.handle, args.slot_streams) != 0 or lib.ssb_set_pipeline_depth(eng.handle, S) != 0:
        raise RuntimeError("ssb_set_pipeline_depth / ssb_set_slot_streams")
    streams.clear()
    # The process group starts only now: the S slots' streams exist and hold a hardware queue each,
    # and the group's streams, created after, take the queues left -- the slot configuration stays
    # as it is from here on.  (Process group first, slots re-created after the latency phases: two
    # slots shared a queue and RCCL at N = 1 measured 9.15 M against 12.4 M without it, round 5.)
    # Phases 1 / 1b above are therefore per-rank and exchange nothing.
    if world > 1 or args.force_dist:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
        xchg = BatchExchange(strong, sizes=sizes, device=cdev)
        exchanger = Exchanger(xchg, dev)
    # the master key's signature of every validator: every combined signature must equal it
    # (tests/test_generic_threshold.rs:35), checked for every slot's batch, untimed
    msig = eng.sign_batch(wl["master"], wl["job_root"], wl["roots"])
    msig_arr = np.frombuffer(b"".join(msig), dtype=np.uint8).reshape(V, 96)
    truth = dict(job_ok=job_ok, valid=valid, msig=msig_arr)
    primed = []

    def check_slots(host=False):
        """every slot's last batch: statuses, every share verdict and every combined signature (all
        V validators) == the workload's truth; with host=True the copies in the pinned host buffers"""
        ok = True
        for k, o in enumerate(outs):
            if host:
                out_host, st_host, _, ver_host = host_io[k].wait()
            else:
                st_host, ver_host, out_host = o["st"].cpu().numpy(), o["ver"].cpu().numpy(), o["out"].cpu().numpy()
            jo = truth["job_ok"]
            ok = ok and bool(((st_host == 0) == jo).all()) and bool((ver_host == truth["valid"]).all())
            ok = ok and bool((out_host[jo] == truth["msig"][jo]).all())
            if args.final_verify and not host:
                fv = o["fv"].cpu().numpy()
                ok = ok and bool(((fv == 1) == jo).all())
        return ok

    def warm_and_check():
        """warmup, then correctness of every slot's last batch"""
        if os.environ.get("SSB_PRIME", "1") != "0" and not primed:
            # first use of each slot's queue one at a time (untimed): 20 queues acquiring their
            # scratch at once intermittently failed with HSA_STATUS_ERROR_OUT_OF_RESOURCES
            for k in range(S):
                step(k, k)
                exchange_group()
                if exchanger is not None:
                    exchanger.drain()
                torch.cuda.synchronize(dev)
            primed.append(1)
        for i in range(max(args.warmup, S)):
            step(i, i % S)
        exchange_group()
        if exchanger is not None:
            exchanger.drain()
        torch.cuda.synchronize(dev)
        return check_slots(host=use_host[0])

    def timed_run(steps=None):
        steps = args.steps if steps is None else steps
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)
        dbg = bool(os.environ.get("SSB_DEBUG_HOST"))
        # SSB_DEBUG_GATE: hold every slot's stream until all steps are enqueued (profiling aid: a
        # kernel trace then shows the device timeline, not the tracer's per-launch host overhead)
        gate = torch.zeros((1,), dtype=torch.int32, device=dev) if os.environ.get("SSB_DEBUG_GATE") else None
        if gate is not None:
            torch.cuda.synchronize(dev)
            for k in range(S):
                lib.ssb_debug_hold(ctypes.c_void_p(lib.ssb_slot_stream(eng.handle, k)), ctypes.c_void_p(gate.data_ptr()), 3000000)
        ev = []
        t0 = time.perf_counter()
        host_ms = []
        for i in range(steps):
            th = time.perf_counter()
            if dbg:   # when the slot's stream reaches / finishes this batch
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(streams.get(i % S) or torch.cuda.ExternalStream(lib.ssb_slot_stream(eng.handle, i % S), device=dev))
            step(args.warmup + i, i % S)
            if dbg:
                e1.record(streams[i % S])
                ev.append((e0, e1))
            host_ms.append((time.perf_counter() - th) * 1e3)
        exchange_group()
        if gate is not None:
            gate.fill_(1)
        if use_host[0]:
            for pb in host_io.values():   # every batch's outputs delivered to host memory
                pb.wait()
        if exchanger is not None:
            exchanger.drain()             # every group's collective issued before the barrier below
        torch.cuda.synchronize(dev)
        if dbg:
            print("host ms per submit:", " ".join("%.2f" % x for x in host_ms), file=sys.stderr)
            print("batch start/end ms:", " ".join("%.1f/%.1f" % (ev[0][0].elapsed_time(a), ev[0][0].elapsed_time(b))
                                                   for a, b in ev), file=sys.stderr)
        if dist is not None:
            dist.barrier()
        return time.perf_counter() - t0

    # the other public-key variant first (reported beside the headline), then the headline
    # (after each timed run, untimed: the batches the timed steps produced -- the last one on every
    # slot -- are checked like the warm-up ones, and for N > 1 the last exchange's gathered results)
    use_cache[0] = args.compressed_pk
    ok_other = warm_and_check()
    elapsed_other = timed_run()
    ok_other = ok_other and check_slots()
    use_cache[0] = not args.compressed_pk
    ok_head = warm_and_check()
    elapsed = timed_run()
    ok_timed = check_slots()
    ok_x = True
    if xchg is not None:
        ok_x, _ = xchg.check_last()
    elapsed_host = None
    ok_host = True
    if world == 1 and not args.no_host_buffers and not args.final_verify:
        use_host[0] = True
        ok_host = warm_and_check()
        elapsed_host = timed_run()
        ok_host = ok_host and check_slots(host=True)
        use_host[0] = False
    # sustained rate: the same path for --sustained-steps batches (a continuous per-slot service
    # rather than the driver's burst of `steps` batches, every one in flight at once)
    elapsed_sus, ok_sus = None, True
    if args.sustained_steps > 0:
        ok_sus = warm_and_check()
        elapsed_sus = timed_run(args.sustained_steps)
        ok_sus = ok_sus and check_slots()
    # the reference-side caller's path: jobs pushed one by one through the library's native per-slot
    # collector (ssb_collector_submit, what HotstuffOperatorCommittee::sign calls under --features hip)
    # by native submitter threads, 4,096-job windows, `S` windows in flight, keys as rows of the
    # decoded-key table (ssb_pk_cache_add), timed from the first submit to the last result
    coll = None
    if args.collector_windows > 0 and not strong:
        from safestakeoperator_amd.collector import NativeCollector, collbench_run, wire_records

        def collector_leg(wire):
            """(seconds, results, windows, profile) of n_jobs jobs through a collector; wire: the jobs'
            shares as the records operators send (bincode(bls::Signature), encoded before the run),
            through ssb_collector_submit_wire and the device's record decode"""
            torch.cuda.synchronize(dev)
            streams.clear()
            col = NativeCollector(eng, max_jobs=V, max_shares=V * n, window_s=0.005, in_flight=S, wire=wire)
            rec = wire_records(wl["sigs"]) if wire else None
            try:
                rows = col.rows(wl["share_pks"])
                collbench_run(col, wl, V, n, t, rows, S * V, threads=args.collector_threads, wire=rec)  # warm-up
                n_jobs = args.collector_windows * V
                if dist is not None:
                    dist.barrier()
                c_sec, c_res = collbench_run(col, wl, V, n, t, rows, n_jobs, threads=args.collector_threads, wire=rec)
                return c_sec, c_res, n_jobs, col.stats(), col.profile()
            finally:
                col.close()

        def collector_ok(c_res, n_jobs):
            vv = np.arange(n_jobs) % V
            vbits = (valid.reshape(V, n).astype(np.uint64) << np.arange(n, dtype=np.uint64)).sum(axis=1)
            return (bool((c_res["done"] == 1).all()) and bool((c_res["rc"] == 0).all())
                    and bool(((c_res["status"] == 0) == job_ok[vv]).all()) and bool((c_res["verdicts"] == vbits[vv]).all())
                    and bool((c_res["absent"] == 0).all())
                    and bool((c_res["sig96"][job_ok[vv]] == msig_arr[vv[job_ok[vv]]]).all()))

        c_sec, c_res, n_jobs, cw, cprof = collector_leg(False)
        coll = dict(seconds=c_sec, jobs=n_jobs, windows=cw[0], ok=collector_ok(c_res, n_jobs), profile=cprof)
        w_sec, w_res, _, ww, _ = collector_leg(True)
        coll.update(wire_seconds=w_sec, wire_windows=ww[0], wire_ok=collector_ok(w_res, n_jobs))
    # adversarial legs: the same path, slots, key table and --steps with invalid shares -- 1% of the shares
    # signed over the wrong root (invalid_1e2), and every share of operator 1 invalid, a faulty operator in
    # every committee (bad_operator) -- the inputs the reference's per-share scan exists for
    # (generic_threshold.rs:149-169).  Every batch fails its RLC check and takes the exact fallback;
    # statuses, every share verdict and every combined signature are checked like the headline's.
    adv = {}
    if args.adversarial_legs and args.ids == "seq" and not strong and not args.final_verify and not wl["n_bad"]:
        for gi, (name, kw) in enumerate((("invalid_1e2", dict(invalid_rate=0.01)), ("bad_operator", dict(bad_operator=1)))):
            torch.cuda.synchronize(dev)
            wl_a = make_workload(eng, V, t, n, n_roots, rank, **kw)
            assert wl_a["pks"] == wl["pks"]   # (the same keys: the key table stands)
            va = np.asarray(wl_a["valid"], dtype=np.uint8)
            inputs.update(d_sig=dt8(wl_a["sigs"]), gen=10 + gi)
            truth.update(valid=va, job_ok=va.reshape(V, n).sum(axis=1) >= t, msig=msig_arr)
            use_cache[0] = True
            streams.clear()
            ok_a = warm_and_check()
            el_a = timed_run()
            ok_a = ok_a and check_slots()
            adv[name] = dict(seconds=el_a, ok=ok_a, n_bad=wl_a["n_bad"])
        inputs.update(d_sig=d_sig, gen=0)
        truth.update(valid=valid, job_ok=job_ok, msig=msig_arr)
    # the same path and the same --steps on committees with REGISTRY operator ids (distinct pseudo-random
    # ids in [1, 2^16) per committee, src/node/node.rs:470-474): the Lagrange coefficients are ratios of
    # small integers, so the combine is [M^-1](sum c_i sig_i) per job (k_combine_ratio) where ids 1..n
    # combine with small integers.  New keys, so the key table is replaced (after every other leg).
    reg = None
    if args.registry_leg and args.ids == "seq" and not strong and not args.final_verify and not wl["n_bad"]:
        torch.cuda.synchronize(dev)
        wl_r = make_workload(eng, V, t, n, n_roots, rank, ids="registry")
        if lib.ssb_pk_cache_set(eng.handle, N, np.frombuffer(wl_r["pks"], dtype=np.uint8).ctypes.data_as(_lib._u8p)) != 0:
            raise RuntimeError("ssb_pk_cache_set: %s" % lib.ssb_last_error(eng.handle))
        inputs.update(d_sig=dt8(wl_r["sigs"]), d_ids=torch.tensor(wl_r["ids"], dtype=torch.int64, device=dev), gen=1)
        msig_r = eng.sign_batch(wl_r["master"], wl_r["job_root"], wl_r["roots"])
        truth.update(msig=np.frombuffer(b"".join(msig_r), dtype=np.uint8).reshape(V, 96),
                     job_ok=np.ones(V, dtype=bool), valid=np.ones(N, dtype=np.uint8))
        use_cache[0] = True
        streams.clear()
        ok_r = warm_and_check()
        elapsed_reg = timed_run()
        ok_r = ok_r and check_slots()
        reg = dict(seconds=elapsed_reg, ok=ok_r)
    ok_st = ok_comb = ok_head and ok_other and ok_timed and ok_x and ok_host and ok_sus and (
        coll is None or (coll["ok"] and coll["wire_ok"]))
    ok_st = ok_st and (reg is None or reg["ok"]) and all(a["ok"] for a in adv.values())
    if dist is not None:
        tt = torch.tensor([elapsed, elapsed_other, elapsed_sus or 0.0, coll["seconds"] if coll else 0.0,
                           reg["seconds"] if reg else 0.0, coll["wire_seconds"] if coll else 0.0,
                           adv["invalid_1e2"]["seconds"] if adv else 0.0, adv["bad_operator"]["seconds"] if adv else 0.0],
                          dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, elapsed_other = float(tt[0].item()), float(tt[1].item())
        if elapsed_sus:
            elapsed_sus = float(tt[2].item())
        if coll:
            coll["seconds"] = float(tt[3].item())
        if reg:
            reg["seconds"] = float(tt[4].item())
        if coll:
            coll["wire_seconds"] = float(tt[5].item())
        if adv:
            adv["invalid_1e2"]["seconds"], adv["bad_operator"]["seconds"] = float(tt[6].item()), float(tt[7].item())
        okt = torch.tensor([1 if (ok_st and ok_comb) else 0], dtype=torch.int32, device=cdev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok_all = bool(okt.item())
    else:
        ok_all = ok_st and ok_comb

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        total_shares = V_glob * n * args.steps
        value = total_shares / elapsed
        combined = V_glob * args.steps / elapsed
        mads = opcount_mads()
        km = kernel_mads(mads, V, t, n, n_roots, pk_cached=not args.compressed_pk)
        avg = {k: (v[0] / v[1] if v[1] else 0.0) for k, v in kt.items()}
        # the dominant kernel = the one doing most of the step's algorithmic work
        dom = max(km, key=lambda k: km[k] if avg.get(k, 0.0) > 0 else -1.0)
        achieved = km[dom] / (avg[dom] * 1e-3) / 1e12 if avg[dom] > 0 else 0.0
        peak = MAD_PEAK_MEASURED / 1e12
        step_mads = sum(km.values())
        if args.final_verify:   # + the combined-signature verify: V shares, no combine
            step_mads += sum(v for k, v in kernel_mads(mads, V, 1, 1, n_roots).items() if k != "k_combine_fast")
        # roofline: k_subgroup_map at full occupancy (phase 1b); the depth-1 C2 figure beside it
        roof = None
        if rf is not None and rf["ms"]["k_subgroup"] > 0:
            mp = msm_plan(rf["shares"], n_roots)
            sg_mads = rf["shares"] * mads["subgroup"]
            dec_mads = rf["shares"] * mads["decode_sig"]
            # algorithmic bytes per share of k_subgroup_map: the affine signature (g2_aff, 4 x 48 B +
            # flag word) and three flag / root words read, two flag words written, and the sort's
            # scatter (the share's root word read, one 4-byte entry written per MSM window)
            sg_bytes_share = 196 + 3 * 4 + 2 * 4 + 4 + 4 * (mp["W2"] + mp["W1"])
            pmc = pmc_traffic("k_subgroup_map", rf["shares"])
            try:
                with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
                    sq = json.load(f).get("k_subgroup_map", {}).get("sq")
            except (OSError, ValueError):
                sq = None
            roof = {"bound": "valu-int32-mad", "kernel": "k_subgroup_map",
                    "achieved": round(sg_mads / (rf["ms"]["k_subgroup"] * 1e-3) / 1e12, 4),
                    "peak": round(MAD_PEAK_MEASURED / 1e12, 2), "unit": "TMAD/s",
                    "frac": round(sg_mads / (rf["ms"]["k_subgroup"] * 1e-3) / MAD_PEAK_MEASURED, 5),
                    "traffic": pmc, "algorithmic_bytes": sg_bytes_share * rf["shares"],
                    "traffic_over_algorithmic": round(pmc / (sg_bytes_share * rf["shares"]), 2) if pmc else None,
                    "mads_per_launch": sg_mads, "avg_launch_ms": round(rf["ms"]["k_subgroup"], 4),
                    "timing": "hipEvents on the slot's stream, one-stream slot at depth 1, one batch of %d x the C2 "
                              "batch (%d shares = %d waves: the chip full at the kernel's two waves per SIMD); MADs = "
                              "the subgroup checks only (the roots' SWU map riding along is < 1%%)" % (
                                  rf["R"], rf["shares"], rf["shares"] // 64),
                    "results_ok": rf["ok"],
                    "pmc_sq": sq,   # SQ_INSTS_VALU / wave and VALU-active / busy cycle: roofline batch and pipelined C2
                    # VALU wave-instructions issued per algorithmic MAD wave-instruction (SQ_INSTS_VALU of the
                    # roofline launch / (MADs / 64)): 2 is the engine product's floor (a v_addc per MAD)
                    "valu_insts_per_mad": valu_per_mad(sq, sg_mads),
                    "k_decode_count": {"achieved": round(dec_mads / (rf["ms"]["k_decode"] * 1e-3) / 1e12, 4),
                                       "frac": round(dec_mads / (rf["ms"]["k_decode"] * 1e-3) / MAD_PEAK_MEASURED, 5),
                                       "avg_launch_ms": round(rf["ms"]["k_decode"], 4), "mads_per_launch": dec_mads,
                                       "traffic": pmc_traffic("k_decode_count", rf["shares"])},
                    "depth1_c2": {"kernel": dom, "achieved": round(achieved, 4), "frac": round(achieved / peak, 5),
                                  "avg_launch_ms": round(avg[dom], 4),
                                  "timing": "one C2 batch alone, three-stream slot (256 waves on 1,024 SIMDs)"}}
        rec = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "partial_sigs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u32-limb modular integer (BLS12-381 Fp/Fr)",
            "data": "synthetic (deterministic keys, GPU-signed shares)",
            "config": {"workload": ("%s: %d validators x %d shares (%d-of-%d), %d roots, ONE batch split over %d GPU(s); "
                                    "verify + combine" % (args.config, V_glob, n, t, n, n_roots, world)) if strong else
                                   ("%s: %d validators x %d shares (%d-of-%d), %d roots per GPU; verify + combine"
                                    % (args.config, V, n, t, n, n_roots)) + (" + final verify" if args.final_verify else ""),
                       "validators_per_gpu": V, "threshold": t, "operators": n, "roots": n_roots,
                       "parallelism": "dp%d (validator shards, RCCL all-gather of verdicts+signatures)" % world,
                       "batches_in_flight": S, "streams_per_slot": args.slot_streams},
            "batch_latency_ms": round(latency_ms, 3),
            "batch_latency_ms_by_config": latency_by_config,
            "public_keys": ("compressed per batch (ssb_threshold_aggregate_batch_dev)" if args.compressed_pk else
                            "decompressed once at registration (ssb_pk_cache_set + _cached_dev), as lighthouse's "
                            "PublicKey holds the point"),
            ("value_pk_cached" if args.compressed_pk else "value_compressed_pk"):
                round(V_glob * n * args.steps / elapsed_other, 1),
            "combined_sigs_per_s": round(combined, 1),
            "final_verify": ("every step verifies its %d combined signatures against the master keys "
                             "(ssb_verify_batch_cached_dev, RLC batch); combined_sigs_per_s counts verified ones" % V
                             if args.final_verify else None),
            "value_host_buffers": (round(V_glob * n * args.steps / elapsed_host, 1) if elapsed_host else None),
            "value_sustained": (round(V_glob * n * args.sustained_steps / elapsed_sus, 1) if elapsed_sus else None),
            "sustained": ("the headline path for %d batches (%d in flight), results of every slot's last batch checked"
                          % (args.sustained_steps, S)) if elapsed_sus else None,
            "value_collector": (round(coll["jobs"] * n * world / coll["seconds"], 1) if coll else None),
            "value_collector_wire": (round(coll["jobs"] * n * world / coll["wire_seconds"], 1) if coll else None),
            "collector": (dict(jobs_per_gpu=coll["jobs"], windows=coll["windows"], window_jobs=V, in_flight=S,
                               submitter_threads=args.collector_threads, seconds=round(coll["seconds"], 4),
                               combined_sigs_per_s=round(coll["jobs"] * world / coll["seconds"], 1),
                               frac_of_value=round(coll["jobs"] * n * world / coll["seconds"] / value, 3),
                               frac_of_sustained=(round(coll["jobs"] * n * world / coll["seconds"] /
                                                        (V_glob * n * args.sustained_steps / elapsed_sus), 3)
                                                  if elapsed_sus else None),
                               worker_profile_incl_warmup=coll["profile"],
                               wire=dict(seconds=round(coll["wire_seconds"], 4), windows=coll["wire_windows"],
                                         frac_of_value=round(coll["jobs"] * n * world / coll["wire_seconds"] / value, 3),
                                         path="the same jobs with every share as the record an operator sends "
                                              "(bincode(bls::Signature), 202 B) through ssb_collector_submit_wire: "
                                              "a SSB_COLLECTOR_WIRE collector, records decoded and decompressed on "
                                              "the device (ssb_threshold_aggregate_batch_wire_cached_dev) -- the "
                                              "receive path of RemoteOperator::sign without the CPU deserialize"),
                               path="ssb_collector_submit per job from native threads (bench_tools/collbench.cpp) -> "
                                    "4,096-job windows -> ssb_threshold_aggregate_batch_cached_dev on %d one-stream "
                                    "slots; timed first submit -> last result; every job's status, verdicts and "
                                    "combined signature checked" % S) if coll else None),
            "value_registry": (round(V_glob * n * args.steps / reg["seconds"], 1) if reg else None),
            "registry": (dict(ms_per_step=round(reg["seconds"] / args.steps * 1e3, 3), steps=args.steps,
                              combined_sigs_per_s=round(V_glob * args.steps / reg["seconds"], 1),
                              frac_of_value=round(elapsed / reg["seconds"], 3), results_ok=reg["ok"],
                              path="the headline path (same slots, steps, key cache) on committees with registry "
                                   "operator ids: distinct pseudo-random ids in [1, 2^16) per committee "
                                   "(src/node/node.rs:470-474); lambda_i = c_i / M, combined as [M^-1](sum c_i sig_i), "
                                   "one lane per job (k_combine_ratio)") if reg else None),
            "value_invalid_1e2": (round(V_glob * n * args.steps / adv["invalid_1e2"]["seconds"], 1) if adv else None),
            "value_bad_operator": (round(V_glob * n * args.steps / adv["bad_operator"]["seconds"], 1) if adv else None),
            "adversarial": ({k: dict(ms_per_step=round(a["seconds"] / args.steps * 1e3, 3), steps=args.steps,
                                     invalid_shares_per_batch=a["n_bad"], frac_of_value=round(elapsed / a["seconds"], 3),
                                     results_ok=a["ok"]) for k, a in adv.items()} | {
                                "path": "the headline path (same slots, steps, key cache) with invalid shares: "
                                        "invalid_1e2 -- 1% of the shares signed over the next root; bad_operator -- every "
                                        "share of operator 1 invalid (a faulty operator in every committee).  Every batch "
                                        "fails its RLC check and takes the exact fallback (committee stage, exclusion "
                                        "check / group tests); statuses, share verdicts and combined signatures checked"}
                            if adv else None),
            "host_buffers": "every batch's inputs start in, and its results end in, ordinary host memory: "
                            "ssb_threshold_aggregate_batch%s_submit copies them into the slot's pinned device-mapped "
                            "staging buffer, the kernels read / write it in place over PCIe, ssb_batch_wait delivers "
                            "the outputs; timed from the first submit to the last delivery (the headline's inputs are "
                            "resident in HBM)" % ("_cached" if not args.compressed_pk else ""),
            "results_ok": ok_all,
            "results_checked": "every slot's last warm-up AND last timed batch: all %d statuses, %d share verdicts and "
                               "combined signatures (== the master key's signature)%s" % (
                                   V, N, "; the last exchange's gathered results == local" if world > 1 else ""),
            "invalid_shares_per_batch": wl["n_bad"],
            "operator_ids": ("registry: distinct pseudo-random ids in [1, 2^16) per committee" if args.ids == "registry"
                             else "1..%d in every committee" % n),
            "bad_operator": args.bad_operator or None,
            "roofline": roof or {"bound": "valu-int32-mad", "kernel": dom, "achieved": round(achieved, 4),
                                 "peak": round(peak, 2), "unit": "TMAD/s", "frac": round(achieved / peak, 5),
                                 "traffic": pmc_traffic(dom), "mads_per_launch": km[dom], "avg_launch_ms": round(avg[dom], 4),
                                 "timing": "hipEvents on the kernel's stream, pipeline depth 1"},
            "step_roofline": {"mads_per_step_per_gpu": step_mads,
                              "achieved_TMAD_s": round(step_mads * world * args.steps / elapsed / 1e12, 4),
                              "frac": round(step_mads * args.steps / elapsed / MAD_PEAK_MEASURED, 5)},
            "kernel_ms": {k: round(v, 4) for k, v in avg.items()},
        }
        if world == 1 and not args.no_cpu_baseline and not wl["n_bad"]:
            # about 10 s of host CPU work: whole passes over the C2 batch, >= 4 s per column
            rec["cpu_baseline"] = cpu_baseline(wl, t, n, gpu_out=outs[0]["out"].cpu().numpy(), n_val=min(4096, V),
                                               n_val_share=min(1024, V))
        print(json.dumps(rec), flush=True)
    if exchanger is not None:
        exchanger.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    torch.cuda.synchronize(dev)
    host_io.clear()
    streams.clear()
    eng.close()


if __name__ == "__main__":
    main()
