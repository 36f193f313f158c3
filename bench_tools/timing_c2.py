import sys, time, hashlib
sys.path.insert(0, '.')
import numpy as np
from safestakeoperator_amd import Engine
sys.path.insert(0, 'tests')
from test_gpu_parity import _gen_committees
e = Engine(0)
t0 = time.time()
V, t, n = 4096, 3, 4
roots, master, sigs, pks, ids, jr, msig = _gen_committees(e, V, t, n, 64)
print("gen s", time.time() - t0, flush=True)
offs = list(range(0, V * n + 1, n))
S, P = b"".join(sigs), b"".join(pks)
e.kernel_timing(True, last_only=True)
for it in range(3):
    t0 = time.time()
    out, st, err, ver = e.threshold_aggregate_batch_raw([t] * V, offs, S, P, ids, jr, roots)
    dt = time.time() - t0
    ks = {k: e.last_kernel_ms(k) for k in ["k_hash_to_g2", "k_decode", "k_subgroup", "k_msm_sort", "k_msm_g2", "k_msm_g1", "k_miller", "k_final", "k_fallback_verify", "k_select", "k_combine_fast"]}
    print("iter", it, "wall s %.4f" % dt, {k: round(v, 3) for k, v in ks.items()}, "ok", bool((st == 0).all() and ver.all()), flush=True)
