"""GPU: exact verdicts of a FAILED batch on bench.py's timed path (one-stream slots, keys from the
cache, the fused launches), through each stage of the fallback (csrc/ssb_k_bisect.hip):

  committee stage  a job whose shares break their committee relation (sum_i c_i sig_i != O over t + 1
                   shares) has its shares checked one by one, and the rest of the batch is decided by
                   ONE exclusion check (the batch check without the suspects, from its own Miller
                   product) -- one invalid share, 1% invalid shares, registry operator ids;
  tree             what the committee stage cannot decide: a faulty operator in every committee (too
                   many suspects), shares that are invalid but consistent (every share of a job signed
                   over the wrong root: the exclusion check fails), jobs without redundancy (t = n).

Every verdict, status, error field and combined signature == the plain-C oracle (oracle/bls_c.c) on
the same bytes, and == the construction truth."""
import numpy as np
import pytest

import bench
from test_gpu_configs import _c_oracle, _cached_one_stream, _check_against_truth

pytestmark = pytest.mark.gpu


def _check(engine, wl, V, t, n):
    runs = _cached_one_stream(engine, wl, V, t, n)
    o_out, o_st, o_err, o_ver = _c_oracle(wl, list(range(V)), t, n)
    for out, st, err, ver in runs:
        assert (ver == o_ver[:V * n]).all(), np.nonzero(ver != o_ver[:V * n])[0][:20]
        assert (st == o_st).all() and (err.astype(np.uint64) == o_err.astype(np.uint64)).all()
        ok = st == 0
        assert (out[ok] == o_out[ok]).all()
        _check_against_truth(wl, V, t, n, out, st, err, ver)
    return o_ver


@pytest.mark.parametrize("ids", ["seq", "registry"])
@pytest.mark.parametrize("case", ["one", "pct1"])
def test_committee_stage_matches_c_oracle(engine, case, ids):
    V, t, n, R = 4096, 3, 4, 64
    wl = bench.make_workload(engine, V, t, n, R, rank=21, ids=ids, invalid_count=1 if case == "one" else 0,
                             invalid_rate=0.01 if case == "pct1" else 0.0)
    o_ver = _check(engine, wl, V, t, n)
    assert int((o_ver[:V * n] == 0).sum()) == wl["n_bad"] and wl["n_bad"] >= 1


@pytest.mark.parametrize("op", [1, 4])
def test_bad_operator_matches_c_oracle(engine, op):
    """Every share of operator `op` invalid in every committee (4,096 suspect jobs: the tree decides)."""
    V, t, n, R = 4096, 3, 4, 64
    wl = bench.make_workload(engine, V, t, n, R, rank=22, bad_operator=op)
    o_ver = _check(engine, wl, V, t, n)
    assert int((o_ver[:V * n] == 0).sum()) == V


def test_consistent_invalid_jobs_fall_to_the_tree(engine):
    """Jobs whose four shares are ALL signed over the wrong root are consistent (the relation holds)
    yet invalid: the exclusion check fails and the tree decides them exactly; a job with one wrong share
    beside them is a suspect."""
    V, t, n, R = 1024, 3, 4, 16
    wl = bench.make_workload(engine, V, t, n, R, rank=23)
    # re-sign every share of jobs 5, 77, 900 over the next root, and share 2 of job 300
    bad_jobs, N = [5, 77, 900], V * n
    sigs = bytearray(wl["sigs"])
    shares = []
    for v in bad_jobs:
        shares += [(v * n + i, (wl["job_root"][v] + 1) % R) for i in range(n)]
    shares.append((300 * n + 2, (wl["job_root"][300] + 1) % R))
    # the shares' secret keys are not kept by make_workload: derive the wrong-root signatures from a
    # second workload with the same seed whose every share signs the next root
    wl2 = bench.make_workload(engine, V, t, n, R, rank=23, invalid_rate=1.0)
    for i, _ in shares:
        sigs[96 * i:96 * (i + 1)] = wl2["sigs"][96 * i:96 * (i + 1)]
    wl["sigs"] = bytes(sigs)
    valid = np.ones(N, dtype=np.uint8)
    for i, _ in shares:
        valid[i] = 0
    wl["valid"] = valid.tolist()
    o_ver = _check(engine, wl, V, t, n)
    assert int((o_ver[:N] == 0).sum()) == len(shares)


def test_no_redundancy_jobs_fall_to_the_tree(engine):
    """3-of-3 jobs (an operator offline: no relation to test) with invalid shares: every job is left to
    the exclusion check, which fails; the tree decides."""
    V, t, n, R = 2048, 3, 3, 32
    wl = bench.make_workload(engine, V, t, n, R, rank=24, invalid_count=5)
    o_ver = _check(engine, wl, V, t, n)
    assert int((o_ver[:V * n] == 0).sum()) == 5


@pytest.mark.parametrize("t,n,V", [(3, 4, 4096), (5, 7, 1024)], ids=["3of4_full_c2", "5of7"])
def test_registry_ids_match_c_oracle(engine, t, n, V):
    """Registry operator ids (distinct pseudo-random ids in [1, 2^16) per committee, src/node/node.rs:470-474):
    the Lagrange coefficients are ratios of small integers.  3-of-4: [M^-1](sum c_i sig_i) on one lane
    per job, lane-uniform windows (k_combine_ratio, unit_combine_ratio_w4); 5-of-7: coefficients past 62
    bits, the general GLS combine with the Fr-exponentiation lambda_i.  Every status, verdict and
    combined signature == the C oracle."""
    wl = bench.make_workload(engine, V, t, n, 64, rank=25, ids="registry")
    assert len(set(wl["ids"][:n])) == n and max(wl["ids"]) > n
    _check(engine, wl, V, t, n)


def test_knobs_tree_only_and_no_ratio(engine, monkeypatch):
    """SSB_NO_COMMITTEE (a failed batch goes straight to the tree) and SSB_NO_RATIO (registry-id jobs
    through the general combine -- lambda_i, four GLS lanes per share -- instead of k_combine_ratio):
    the same exact results."""
    monkeypatch.setenv("SSB_NO_COMMITTEE", "1")
    monkeypatch.setenv("SSB_NO_RATIO", "1")
    V, t, n, R = 1024, 3, 4, 16
    wl = bench.make_workload(engine, V, t, n, R, rank=26, ids="registry", invalid_rate=0.01)
    _check(engine, wl, V, t, n)


@pytest.mark.parametrize("exact", [False, True], ids=["lane_groups", "exact_knob"])
@pytest.mark.parametrize("t,n,V", [(3, 4, 1024), (9, 13, 512)], ids=["3of4", "9of13"])
def test_few_ratio_jobs_per_wave(engine, monkeypatch, t, n, V, exact):
    """Operator ids 1..n with a share skipped (an invalid share among the first t): the Lagrange
    coefficients are ratios c_i / M, a few such jobs per 64-job wave -- each combined on one
    workgroup's eight lane groups (k_combine_sum's extra blocks, ratio_lane_job: [c_i] sig_i per group,
    9-of-13 in two passes over the groups, then [M^-1] T by the four base-u digits); with
    SSB_RATIO_LANE_EXACT=1 every such job takes the exact single-lane fallback instead.  Every status,
    verdict and combined signature == the C oracle."""
    if exact:
        monkeypatch.setenv("SSB_RATIO_LANE_EXACT", "1")
    wl = bench.make_workload(engine, V, t, n, 16, rank=27, invalid_rate=0.02)
    bad = [i for i, v in enumerate(wl["valid"]) if not v]
    assert any(i % n < t for i in bad)                   # some job skips one of its first t shares
    _check(engine, wl, V, t, n)
